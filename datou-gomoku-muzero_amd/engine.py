"""BatchedSelfPlayEngine — G concurrent games searched and played on one MI355X.

Host orchestration of the HIP kernels in csrc/gmz_tree.hip (C ABI: include/gmz.h).  One call of
:meth:`search` performs, for every game at once, exactly what one ``MuZeroMCTS.search(game)``
(/root/reference/mcts.py:288-362) or ``AlphaZeroMCTS.search(game)`` (mcts.py:197-280) does for
one game; :meth:`play` is ``game.do_move`` + ``get_game_ended`` (workers.py:178-181).

The network is a pluggable *device backend* (``initial`` / ``recurrent`` writing straight into
the engine's slot-indexed buffers) — the in-process replacement of the reference's
InferenceServer queue round trip (workers.py:331-369).  Backends: ``HashNetBackend`` (tree
parity) and ``network.GomokuNetHip`` (GomokuNetEZ on MFMA kernels).

Everything stays resident in HBM; the only host<->device traffic per move is the game status
(G bytes) used to size the next move's wave loop, plus whatever the caller copies out.
"""
import contextlib
import ctypes

import numpy as np
import torch

from . import _lib
from .config import from_any
from ._lib import GmzError, check, ptr


class HashNetBackend:
    """HashNet test network on the device (oracle/hashnet.py definition, csrc/gmz_hashnet.hip)."""

    def __init__(self, num_slots, action_space, device="cuda"):
        self.A = action_space
        self.pool = torch.zeros(num_slots, dtype=torch.int32, device=device)  # uint32 ids

    def ensure_slots(self, n, stream=None):
        """At least ``n`` hidden-state slots (a larger pool, contents not kept: called between moves); the old
        pool is recorded on ``stream`` (default: the current one), the stream that used it."""
        if n > self.pool.numel():
            self.pool.record_stream(stream if stream is not None else torch.cuda.current_stream(self.pool.device))
            self.pool = torch.zeros(int(n * 1.25) + 1, dtype=torch.int32, device=self.pool.device)

    def split(self, parts, max_grid=0):
        """Backends over disjoint equal slices of the pool (SplitSelfPlayEngine)."""
        n = self.pool.numel() // parts
        out = []
        for i in range(parts):
            q = HashNetBackend.__new__(HashNetBackend)
            q.A, q.pool = self.A, self.pool[i * n:(i + 1) * n]
            out.append(q)
        return out

    def initial(self, obs, out_slot, logits, value, stream):
        check(_lib.load().gmz_hashnet_initial(ptr(obs), obs.shape[0], self.A, ptr(out_slot), ptr(self.pool),
                                              ptr(logits), ptr(value), stream))

    def recurrent(self, in_slot, action, out_slot, logits, value, reward, stream):
        check(_lib.load().gmz_hashnet_recurrent(ptr(self.pool), ptr(in_slot), ptr(action), ptr(out_slot),
                                                in_slot.shape[0], self.A, ptr(logits), ptr(value), ptr(reward),
                                                stream))


class BatchedSelfPlayEngine:
    """G games per GPU.  ``cfg``: any object with the reference config attribute names."""

    def __init__(self, cfg=None, num_games=1, net=None, device="cuda", seed=0, descent_hint=None, game_offset=0,
                 wpb=None, layout=None, pair=None, **overrides):
        self.cfg = from_any(cfg, **overrides)
        c = self.cfg
        if c.MCTS_IMPLEMENTATION not in ("AlphaZero", "MuZero"):
            raise ValueError("Unknown MCTS implementation in config: '%s'" % c.MCTS_IMPLEMENTATION)  # workers.py:140-142
        self.lib = _lib.load()
        self.device = torch.device(device)
        self.G, self.A, self.size = int(num_games), c.ACTION_SPACE_SIZE, c.BOARD_SIZE
        if layout is None:
            layout = default_layout(self.G)
        if layout not in ("dense", "lists"):
            raise ValueError("layout: 'dense' (every node's full child row) or 'lists' (compact child lists)")
        if descent_hint is None:
            # dense rows: the hint kernels (cached exp rows + next-visit prefetch) at every G measured; the
            # no-hint dense kernels keep the reference's exp(logit + t - max) form (A/B and tests).
            # Compact lists always use the cached exp rows; there the hint only switches the prefetch,
            # which measured slower (8,192 games: 110 vs 125 us; profiles/r03_tree_layout_ab.txt)
            descent_hint = layout == "dense"
        self.mode = 1 if c.MCTS_IMPLEMENTATION == "MuZero" else 0
        self.slots_per_game = c.NUM_SIMULATIONS + 2
        if wpb not in (None, 1, 4):
            raise ValueError("wpb: games per workgroup of the fused expand/select kernel must be None, 1 or 4")
        self.descent_hint = bool(descent_hint)
        self.layout = layout
        # two waves per game in the fused expand/select kernel (MuZero, dense rows with the hint, 129..256
        # actions; k_expand_select_pair): None = default_pair(G)
        pair_ok = self.mode == 1 and layout == "dense" and self.descent_hint and 128 < self.A <= 256
        self.pair = bool(pair_ok and (default_pair(self.G) if pair is None else pair))
        # flags (include/gmz.h): bit 0 no hint; bits 1 / 2 force 4-wave / 1-wave workgroups (None: by occupancy);
        # bit 3 compact child lists for non-root nodes; bit 4 two waves per game
        flags = ((0 if descent_hint else 1) | {None: 0, 4: 2, 1: 4}[wpb] | (8 if layout == "lists" else 0)
                 | (16 if self.pair else 0))
        self.ecfg = _lib.EngineCfg(self.G, c.BOARD_SIZE, c.N_IN_ROW, c.NUM_SIMULATIONS, c.NUM_TOP_ACTIONS, self.mode,
                                   int(c.C_VISIT), flags, float(c.C_SCALE),
                                   float(c.VALUE_MINMAX_DELTA), float(c.DISCOUNT), int(game_offset))
        h = ctypes.c_void_p()
        check(self.lib.gmz_engine_create(ctypes.byref(self.ecfg), ctypes.byref(h)))
        self.handle = h
        self.seed = int(seed)
        self.fuse_waves = True  # expand/backup + next select in one launch (False: the two entry points)
        G, A, dev = self.G, self.A, self.device
        # hidden-state slots per game by legal-move count (gmz_engine_set_hidden_bases): MuZero creates one
        # node per wave (mcts.py:320-350), so a game needs waves(L) + 2 slots, not num_simulations + 2
        self._slot_need = slot_need_table(self.ecfg, A, self.mode, self.lib)
        self.net = net if net is not None else HashNetBackend(G * int(self._slot_need[A]), A, device)
        f32, i32 = torch.float32, torch.int32
        self.obs = torch.zeros(G, 3, c.BOARD_SIZE, c.BOARD_SIZE, dtype=f32, device=dev)
        self.logits = torch.zeros(G, A, dtype=f32, device=dev)
        self.value = torch.zeros(G, dtype=f32, device=dev)
        self.reward = torch.zeros(G, dtype=f32, device=dev)
        self.in_slot = torch.zeros(G, dtype=i32, device=dev)
        self.out_slot = torch.zeros(G, dtype=i32, device=dev)
        self.act_req = torch.zeros(G, dtype=i32, device=dev)
        # hidden-state slot of each game's root (= its node 0): hbase[g], rewritten when the bases move, and
        # beside it each game's slot budget (gmz_engine_set_hidden_budget): one device buffer [2G]
        self._hb_dev = torch.empty(2 * G, dtype=i32, device=dev)
        self.root_slot = self._hb_dev[:G]
        self.hidden_budget = self._hb_dev[G:]
        self.root_slot.copy_(torch.arange(G, dtype=i32, device=dev) * self.slots_per_game)
        self.hidden_budget.fill_(self.slots_per_game)
        self._hb_host = [torch.zeros(2 * G, dtype=i32).pin_memory() for _ in range(2)]
        self._hb_events = [None, None]
        self._hb_flip = 0
        self._hb_last = None  # the bases last handed to the engine (host copy)
        self.hidden_slots_used = 0
        self.policy = torch.zeros(G, A, dtype=torch.float64, device=dev)
        self.root_value = torch.zeros(G, dtype=f32, device=dev)
        self.action = torch.zeros(G, dtype=i32, device=dev)
        self.status = torch.zeros(G, dtype=torch.int8, device=dev)
        self._status_host = torch.zeros(G, dtype=torch.int8).pin_memory()
        self._err_host = torch.zeros(1, dtype=i32).pin_memory()  # the engine's error word, copied with each status
        self._status_event = None
        self._n_legal = np.full(G, A, dtype=np.int32)
        self._last_reset = True
        self.waves_last = 0
        self.tree_timer = None  # optional network.KernelTimer around the fused expand/backup+select launches
        # the packed per-game hidden-state bases and budgets from the start, so a direct ABI caller
        # (begin_move / select without search_steps) already uses slots inside the network's pool
        self._place_hidden(self._stream())

    # ------------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "handle", None):
            self.lib.gmz_engine_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self, stream=None):
        return _lib.stream_ptr(stream)

    # ------------------------------------------------------------------ game state
    def game_state(self):
        """Copies of the engine-owned game state: boards int8[G,S,S], players int8[G],
        last_moves int32[G], move_counts int32[G] (device tensors)."""
        G, A, dev = self.G, self.A, self.device
        b = torch.empty(G, A, dtype=torch.int8, device=dev)
        p = torch.empty(G, dtype=torch.int8, device=dev)
        lm = torch.empty(G, dtype=torch.int32, device=dev)
        mc = torch.empty(G, dtype=torch.int32, device=dev)
        check(self.lib.gmz_engine_copy_state(self.handle, 0, ptr(b), ptr(p), ptr(lm), ptr(mc), self._stream()))
        return b.view(G, self.size, self.size), p, lm, mc

    def set_positions(self, boards, players, last_moves, move_counts=None):
        """Load G positions: boards int8[G,S,S], players ±1, last_moves (-1 = none)."""
        G, A, dev = self.G, self.A, self.device
        b = torch.as_tensor(np.ascontiguousarray(boards, dtype=np.int8).reshape(G, A))
        nz = (b != 0).sum(dim=1).to(torch.int32)
        p = torch.as_tensor(np.ascontiguousarray(players, dtype=np.int8).reshape(G))
        lm = torch.as_tensor(np.ascontiguousarray(last_moves, dtype=np.int32).reshape(G))
        mc = nz if move_counts is None else torch.as_tensor(np.asarray(move_counts, dtype=np.int32).reshape(G))
        b, p, lm, mc = (t.to(dev).contiguous() for t in (b, p, lm, mc))
        check(self.lib.gmz_engine_copy_state(self.handle, 1, ptr(b), ptr(p), ptr(lm), ptr(mc), self._stream()))
        torch.cuda.current_stream().synchronize()
        self._n_legal = (A - nz.numpy()).astype(np.int32)
        self._status_event = None

    def reset_games(self, mask=None):
        m = None
        if mask is not None:
            m = torch.as_tensor(np.asarray(mask, dtype=np.uint8)).to(self.device)
            self._n_legal[np.asarray(mask, dtype=bool)] = self.A
        else:
            self._n_legal[:] = self.A
        check(self.lib.gmz_engine_reset_games(self.handle, ptr(m), self._stream()))

    # ------------------------------------------------------------------ search
    def _sync_status(self):
        if self._status_event is not None:
            self._status_event.synchronize()
            err = int(self._err_host[0])
            if err:  # a void search must not reach self-play records or the replay buffer
                raise GmzError("engine error bits 0x%x after the last move: a search passed its game's hidden-state "
                               "slot budget, so that game's search result is void (gmz_engine_errors)" % err)
            st = self._status_host.numpy()
            ended = st != 2
            played = st != 3
            self._n_legal[played & ~ended] -= 1
            if self._last_reset:
                self._n_legal[played & ended] = self.A
            else:
                self._n_legal[played & ended] = np.maximum(self._n_legal[played & ended] - 1, 0)
            self._status_event = None

    def _place_hidden(self, s, stream=None):
        """Give every game the hidden-state slots its coming search can use: waves(L) + 2 for MuZero at
        its legal count L (num_simulations + 2 for AlphaZero), packed game after game into the network's
        pool.  L is known exactly after set_positions / reset_games; after a play() whose status has not
        been read yet it is the last search's L - 1, or A for a game that ended and restarted: the larger
        need of the two is taken.  The bases change only when a game's need does (late-game positions with
        fewer than NUM_TOP_ACTIONS legal moves); then they are copied to the device on the search's stream."""
        nl = self._n_legal
        need = self._slot_need[np.clip(nl, 0, self.A)]
        if self._status_event is not None:  # a move was played since nl was read
            need = np.maximum(self._slot_need[np.clip(nl - 1, 0, self.A)], self._slot_need[self.A])
        base = np.zeros(self.G, np.int64)
        np.cumsum(need[:-1], out=base[1:])
        total = int(base[-1] + need[-1])
        key = np.concatenate([base, need])
        if self._hb_last is not None and np.array_equal(key, self._hb_last):
            return
        if total >= 2 ** 31:
            raise ValueError("hidden-state pool: %d slots exceed the int32 slot index" % total)
        if hasattr(self.net, "ensure_slots"):
            self.net.ensure_slots(total, stream)
        i = self._hb_flip
        self._hb_flip ^= 1
        if self._hb_events[i] is not None:
            self._hb_events[i].synchronize()  # (a copy two placements ago: long done)
        hb = self._hb_host[i].numpy()
        hb[:self.G] = base
        hb[self.G:] = need
        with torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext():
            self._hb_dev.copy_(self._hb_host[i], non_blocking=True)  # on the search's stream
            ev = torch.cuda.Event()
            ev.record()
        self._hb_events[i] = ev
        check(self.lib.gmz_engine_set_hidden_bases(self.handle, ptr(self.root_slot), s))
        check(self.lib.gmz_engine_set_hidden_budget(self.handle, ptr(self.hidden_budget), s))
        self._hb_last = key
        self.hidden_slots_used = total

    def errors(self, reset=False):
        """Sticky error bits of the engine's kernels (synchronises the device; gmz_engine_errors): bit 0 = a
        search created more nodes than its game's hidden-state budget (its result is void; no other game's
        states were touched)."""
        out = ctypes.c_int32()
        check(self.lib.gmz_engine_errors(self.handle, ctypes.byref(out), 1 if reset else 0))
        return out.value

    def waves_needed(self):
        out = ctypes.c_int32()
        nl = np.ascontiguousarray(self._n_legal, dtype=np.int32)
        check(self.lib.gmz_engine_waves_for_legal(ctypes.byref(self.ecfg), nl.ctypes.data_as(ctypes.c_void_p),
                                                  self.G, ctypes.byref(out)))
        return out.value

    def search(self, gumbel=None, stream=None):
        """One search for every game (mcts.py:288-362 / 197-280).  ``gumbel``: optional f64[G,A]
        noise (host or device); default = device noise from (seed, move counter).
        Returns device tensors (policy f64[G,A], value f32[G], action int32[G])."""
        for _ in self.search_steps(gumbel, stream):
            pass
        return self.policy, self.root_value, self.action

    def search_steps(self, gumbel=None, stream=None):
        """:meth:`search` as a generator that yields after each simulation wave has been enqueued
        (SplitSelfPlayEngine interleaves the waves of engines on different streams)."""
        s = self._stream(stream)
        L = self.lib
        g = None
        if gumbel is not None:
            g = torch.as_tensor(gumbel, dtype=torch.float64).to(self.device).contiguous()
        self._place_hidden(s, stream)
        check(L.gmz_engine_begin_move(self.handle, ptr(g), self.seed, ptr(self.obs), s))
        self.net.initial(self.obs, self.root_slot, self.logits, self.value, s)
        check(L.gmz_engine_set_root(self.handle, ptr(self.logits), ptr(self.value), s))
        self._sync_status()  # previous move's status → legal counts (overlaps the root inference)
        waves = self.waves_needed()
        self.waves_last = waves
        rw = ptr(self.reward) if self.mode == 1 else None
        if waves > 0:
            check(L.gmz_engine_select(self.handle, ptr(self.in_slot), ptr(self.act_req), ptr(self.out_slot),
                                      ptr(self.obs), s))
        for w in range(waves):
            if self.mode == 1:
                self.net.recurrent(self.in_slot, self.act_req, self.out_slot, self.logits, self.value, self.reward, s)
            else:
                self.net.initial(self.obs, self.out_slot, self.logits, self.value, s)
            if w + 1 < waves and self.fuse_waves:  # backup of this wave + selection of the next in one launch
                if self.tree_timer is not None:
                    self.tree_timer.start()
                check(L.gmz_engine_expand_backup_select(self.handle, ptr(self.logits), ptr(self.value), rw,
                                                        ptr(self.in_slot), ptr(self.act_req), ptr(self.out_slot),
                                                        ptr(self.obs), s))
                if self.tree_timer is not None:
                    self.tree_timer.stop(0)
            else:
                check(L.gmz_engine_expand_backup(self.handle, ptr(self.logits), ptr(self.value), rw, s))
                if w + 1 < waves:
                    check(L.gmz_engine_select(self.handle, ptr(self.in_slot), ptr(self.act_req), ptr(self.out_slot),
                                              ptr(self.obs), s))
            yield w
        check(L.gmz_engine_finish_move(self.handle, ptr(self.policy), ptr(self.root_value), ptr(self.action), s))

    def play(self, action=None, reset_finished=True, stream=None):
        """do_move + get_game_ended for all games.  Returns the device status tensor
        (+1/-1 winner, 0 draw, 2 ongoing, 3 untouched)."""
        s = self._stream(stream)
        a = self.action if action is None else torch.as_tensor(action, dtype=torch.int32).to(self.device)
        check(self.lib.gmz_engine_play(self.handle, ptr(a), ptr(self.status), 1 if reset_finished else 0, s))
        self._status_host.copy_(self.status, non_blocking=True)
        check(self.lib.gmz_engine_errors_async(self.handle, ptr(self._err_host), s))
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream() if stream is None else stream)
        self._status_event = ev
        self._last_reset = bool(reset_finished)
        return self.status

    def winning_scan(self, boards, players, action=None, counters=None, stream=None):
        """workers.py:49-123 find_winning_moves_rebuilt on the device for G positions (see
        ``winning_scan``); ``counters`` = (missed_fives, missed_totals) int32[G] accumulated in place."""
        return winning_scan(boards, players, action, self.cfg.N_IN_ROW, counters, stream, self.lib)

    def tree_counters(self, reset=False):
        """Work done by the fused expand/backup + select launches since the last reset, summed over
        games: dict(backups, backup_levels, selects, select_levels) (gmz_engine_tree_counters)."""
        c = torch.zeros(self.G, 4, dtype=torch.int32, device=self.device)
        check(self.lib.gmz_engine_tree_counters(self.handle, ptr(c), 1 if reset else 0, self._stream()))
        t = c.to(torch.int64).sum(0).tolist()
        return dict(backups=t[0], backup_levels=t[1], selects=t[2], select_levels=t[3])

    def max_visited_children(self):
        """Largest visited-children count of any non-root node in the current trees (diagnostics, synchronous)."""
        out = ctypes.c_int32()
        check(self.lib.gmz_engine_max_visited_children(self.handle, ctypes.byref(out)))
        return out.value

    def root_stats(self):
        G, A, dev = self.G, self.A, self.device
        visits = torch.zeros(G, A, dtype=torch.int32, device=dev)
        rn = torch.zeros(G, dtype=torch.int32, device=dev)
        rw = torch.zeros(G, dtype=torch.float32, device=dev)
        mx = torch.zeros(G, dtype=torch.float32, device=dev)
        mn = torch.zeros(G, dtype=torch.float32, device=dev)
        check(self.lib.gmz_engine_root_stats(self.handle, ptr(visits), ptr(rn), ptr(rw), ptr(mx), ptr(mn),
                                             self._stream()))
        return visits, rn, rw, mx, mn


# the CUs a two-stream engine's tower leaves to the other part's latency-bound tree and head kernels: a 512-game tree
# launch is 512 waves at 4 waves per SIMD (the 15x15 hint kernel's 105 VGPRs), which 32 free CUs hold in one round
# and 24 in two — the cliff below.  Sweep with the round-6 tower
# (tools/cap_sweep.sh, profiles/r06_tower_cap_sweep.txt, 1,024 games, two rounds): cap 192 12,270-12,347 moves/s, 208
# 12,279-12,285, 216 12,321-12,342, 224 = 256 - 32: 12,465-12,515, 232 10,364-10,381, 240 10,257-10,340, no cap 11,357
TOWER_FREE_CUS = 32


class SplitSelfPlayEngine:
    """G games as ``parts`` BatchedSelfPlayEngines of G/parts games, each on its own HIP stream, with
    their simulation waves interleaved on the host (same public interface as BatchedSelfPlayEngine).

    Why: one tower launch fills every CU (a persistent workgroup per CU), and the tree / head kernels
    between two towers are short and latency-bound.  With two halves on two streams and each half's
    tower grid capped at all CUs but TOWER_FREE_CUS (``max_grid``), one half's tree and head kernels run on the
    CUs the other half's tower leaves free, and each tower's ramp-up and tail overlap the other
    half's work (measured with tools/dual_stream_probe.py).  Every game's search is
    exactly the unsplit engine's: part i plays games [i*G/parts, (i+1)*G/parts) with ``game_offset``
    so the device Gumbel noise per game is unchanged, its outputs are row views of the full
    tensors.  Layout and descent hint default per part (from G/parts games: ``default_layout(g)``);
    every default uses the cached-exp softmax, so the results equal one engine's with
    all G games whatever layout each side picks.  Calls fork from the caller's stream and join back."""

    def __init__(self, cfg=None, num_games=2, net=None, device="cuda", seed=0, parts=2, max_grid=None,
                 descent_hint=None, layout=None, pair=None, **overrides):
        self.cfg = from_any(cfg, **overrides)
        c = self.cfg
        G = int(num_games)
        if parts < 1 or G % parts:
            raise ValueError("SplitSelfPlayEngine: num_games must be a multiple of parts")
        self.lib = _lib.load()
        self.device = torch.device(device)
        self.G, self.A, self.size, self.parts = G, c.ACTION_SPACE_SIZE, c.BOARD_SIZE, int(parts)
        self.mode = 1 if c.MCTS_IMPLEMENTATION == "MuZero" else 0
        self.slots_per_game = c.NUM_SIMULATIONS + 2
        g = self.g = G // parts
        # descent_hint / layout None: each part's defaults — the cached-exp softmax in every part, as one
        # engine with every game (the layout may differ per part: results are identical)
        if max_grid is None:  # every CU but TOWER_FREE_CUS for the other part's tree and head kernels
            cus = torch.cuda.get_device_properties(self.device).multi_processor_count
            max_grid = max(cus // 2, cus - TOWER_FREE_CUS) if parts > 1 else 0
        if net is None:
            net = HashNetBackend(hidden_slots(c, G), self.A, device)
        self.net = net
        nets = net.split(parts, max_grid) if parts > 1 else [net]
        if layout is None:
            layout = default_layout(g)
        self.engines = [BatchedSelfPlayEngine(c, g, nets[i], device, seed, descent_hint, game_offset=i * g,
                                              layout=layout, pair=pair) for i in range(parts)]
        self.streams = engine_streams(self.device, parts)
        dev = self.device
        self.policy = torch.zeros(G, self.A, dtype=torch.float64, device=dev)
        self.root_value = torch.zeros(G, dtype=torch.float32, device=dev)
        self.action = torch.zeros(G, dtype=torch.int32, device=dev)
        self.status = torch.zeros(G, dtype=torch.int8, device=dev)
        for i, e in enumerate(self.engines):  # the parts write straight into row slices
            sl = slice(i * g, (i + 1) * g)
            e.policy, e.root_value, e.action, e.status = self.policy[sl], self.root_value[sl], self.action[sl], self.status[sl]
        self.waves_last = 0

    # ------------------------------------------------------------------ streams
    def _fork(self, stream=None):
        main = stream if stream is not None else torch.cuda.current_stream(self.device)
        ev = torch.cuda.Event()
        ev.record(main)
        for st in self.streams:
            st.wait_event(ev)
        return main

    def _join(self, main):
        for st in self.streams:
            ev = torch.cuda.Event()
            ev.record(st)
            main.wait_event(ev)

    def _rows(self, x, i):
        return None if x is None else x[i * self.g:(i + 1) * self.g]

    # ------------------------------------------------------------------ interface of BatchedSelfPlayEngine
    def close(self):
        for e in self.engines:
            e.close()

    def search(self, gumbel=None, stream=None):
        g = None
        if gumbel is not None:  # to the device on the caller's stream, before the fork
            g = torch.as_tensor(gumbel, dtype=torch.float64).to(self.device).contiguous()
        main = self._fork(stream)
        gens = [e.search_steps(self._rows(g, i), st) for i, (e, st) in enumerate(zip(self.engines, self.streams))]
        live = list(zip(gens, self.streams))
        while live:  # one wave of each part in turn
            for item in list(live):
                gen, st = item
                with torch.cuda.stream(st):
                    try:
                        next(gen)
                    except StopIteration:
                        live.remove(item)
        self._join(main)
        self.waves_last = max(e.waves_last for e in self.engines)
        return self.policy, self.root_value, self.action

    def play(self, action=None, reset_finished=True, stream=None):
        a = None if action is None else torch.as_tensor(action, dtype=torch.int32).to(self.device)
        main = self._fork(stream)
        for i, (e, st) in enumerate(zip(self.engines, self.streams)):
            with torch.cuda.stream(st):
                e.play(self._rows(a, i), reset_finished)
        self._join(main)
        return self.status

    def reset_games(self, mask=None):
        for i, e in enumerate(self.engines):
            e.reset_games(None if mask is None else np.asarray(mask)[i * self.g:(i + 1) * self.g])

    def game_state(self):
        parts = [e.game_state() for e in self.engines]
        return tuple(torch.cat([p[k] for p in parts]) for k in range(4))

    def set_positions(self, boards, players, last_moves, move_counts=None):
        b = np.asarray(boards).reshape(self.G, -1)
        p, lm = np.asarray(players).reshape(self.G), np.asarray(last_moves).reshape(self.G)
        mc = None if move_counts is None else np.asarray(move_counts).reshape(self.G)
        for i, e in enumerate(self.engines):
            e.set_positions(self._rows(b, i), self._rows(p, i), self._rows(lm, i), self._rows(mc, i))

    def winning_scan(self, boards, players, action=None, counters=None, stream=None):
        return winning_scan(boards, players, action, self.cfg.N_IN_ROW, counters, stream, self.lib)

    def tree_counters(self, reset=False):
        out = dict(backups=0, backup_levels=0, selects=0, select_levels=0)
        for e in self.engines:
            for k, v in e.tree_counters(reset).items():
                out[k] += v
        return out

    def root_stats(self):
        parts = [e.root_stats() for e in self.engines]
        return tuple(torch.cat([p[k] for p in parts]) for k in range(5))


def slot_need_table(ecfg, A, mode, lib=None):
    """Hidden-state slots one game's search can use, by legal-move count L = 0..A: MuZero creates the
    root and one node per wave (mcts.py:320-350), i.e. gmz_engine_waves_for_legal(L) + 1, plus one
    spare; AlphaZero one node per simulation (mcts.py:233-268): num_simulations + 2."""
    L = lib if lib is not None else _lib.load()
    tab = np.full(A + 1, ecfg.num_simulations + 2, np.int64)
    if mode == 1:
        out = ctypes.c_int32()
        for n in range(A + 1):
            one = np.array([n], np.int32)
            check(L.gmz_engine_waves_for_legal(ctypes.byref(ecfg), one.ctypes.data_as(ctypes.c_void_p), 1,
                                               ctypes.byref(out)))
            tab[n] = out.value + 2
    return tab


def hidden_slots(cfg, num_games):
    """Initial size of the network's hidden-state pool for ``num_games`` games: every game at a legal
    count >= NUM_TOP_ACTIONS (MuZero C2: 102 slots per game instead of NUM_SIMULATIONS + 2 = 402; the
    pool grows if late-game positions need more, BatchedSelfPlayEngine._place_hidden)."""
    c = from_any(cfg)
    A = c.ACTION_SPACE_SIZE
    mode = 1 if c.MCTS_IMPLEMENTATION == "MuZero" else 0
    ecfg = _lib.EngineCfg(1, c.BOARD_SIZE, c.N_IN_ROW, c.NUM_SIMULATIONS, c.NUM_TOP_ACTIONS, mode, int(c.C_VISIT), 0,
                          float(c.C_SCALE), float(c.VALUE_MINMAX_DELTA), float(c.DISCOUNT), 0)
    if mode == 0:
        return int(num_games) * (c.NUM_SIMULATIONS + 2)
    out = ctypes.c_int32()
    one = np.array([A], np.int32)
    check(_lib.load().gmz_engine_waves_for_legal(ctypes.byref(ecfg), one.ctypes.data_as(ctypes.c_void_p), 1,
                                                 ctypes.byref(out)))
    return int(num_games) * (out.value + 2)


_ENGINE_STREAMS = {}


def engine_streams(device, parts):
    """The HIP streams of the split engines: created once per device and process and shared by every
    SplitSelfPlayEngine (one at a time).  HIP maps each new stream onto the device's hardware queues
    round-robin (GPU_MAX_HW_QUEUES, 4 on MI355X), so streams created later — a second engine's, after a
    trainer's side streams — can land on the queue of the default stream or of each other and serialise
    the two halves: measured 123 vs 90 ms per move for the same worker (profiles/r03_worker_streams.txt)."""
    key = (str(torch.device(device)), parts)
    if key not in _ENGINE_STREAMS:
        _ENGINE_STREAMS[key] = [torch.cuda.Stream(device) for _ in range(parts)]
    return _ENGINE_STREAMS[key]


def default_layout(num_games):
    """Tree layout of the non-root nodes of one engine: 'dense' (a 16-B edge per action) or 'lists'
    (compact lists of the visited children, gmz_engine_cfg.flags bit 3), as measured on k_expand_select
    (profiles/r03_tree_layout_ab.txt): the dense rows in the latency-bound regime (one wave per SIMD
    or less, below 4,096 games), the lists from 4,096 (fewer bytes and instructions per tree level).
    Results are identical either way (tests/test_tree_lists_gpu.py)."""
    return "lists" if num_games >= 4096 else "dense"


def default_pair(num_games):
    """Two waves per game in the fused expand/select kernel (k_expand_select_pair) when one wave per game
    would leave the SIMDs at one wave or fewer: as measured."""
    return PAIR_DEFAULT and num_games <= PAIR_MAX_GAMES


PAIR_DEFAULT = False
PAIR_MAX_GAMES = 2048


def default_streams(cfg, num_games):
    """HIP streams for G games, as measured (profiles/r02_dual_stream_sweep.txt, r02_configs_two_streams.txt):
    two half-size engines for 15x15 MuZero from 256 games up (+5-7 % moves/s: the 0.8 ms tower leaves
    room beside it for the other half's ~0.1 ms of tree and head kernels); one engine otherwise (19x19:
    the 2.6 ms tower dwarfs the rest and loses more to the capped grid, -2 %; 9x9 AlphaZero: -4 %)."""
    c = from_any(cfg)
    if c.BOARD_SIZE == 15 and c.MCTS_IMPLEMENTATION == "MuZero" and num_games >= 256 and num_games % 2 == 0:
        return 2
    return 1


def make_engine(cfg=None, num_games=1, net=None, device="cuda", seed=0, streams=None, **kw):
    """BatchedSelfPlayEngine, or SplitSelfPlayEngine over ``streams`` HIP streams when streams > 1
    (None: default_streams(cfg, num_games))."""
    if streams is None:
        streams = default_streams(cfg, num_games)
    if streams > 1:
        return SplitSelfPlayEngine(cfg, num_games, net, device, seed, parts=streams, **kw)
    return BatchedSelfPlayEngine(cfg, num_games, net, device, seed, **kw)


def winning_scan(boards, players, actions=None, n_in_row=5, counters=None, stream=None, lib=None):
    """Batched workers.py:49-123 ``find_winning_moves_rebuilt`` (``gmz_game_winning_scan``).

    boards int8[G,S,S] and players int8[G] (the player to move) on the device.  Without
    ``actions``: returns uint8[G,S*S] cell classes (0 none, 1 five, 2 open_four, 3 combo).  With
    ``actions`` int32[G] and ``counters`` = (missed_fives, missed_totals) int32[G] device tensors:
    adds the workers.py:191-203 missed-win counts of this position (action < 0: game skipped)."""
    L = lib if lib is not None else _lib.load()
    b = torch.as_tensor(boards).contiguous()
    G, S = b.shape[0], b.shape[-1]
    p = torch.as_tensor(players, dtype=torch.int8).to(b.device).contiguous()
    cls, mf, mt, a = None, None, None, None
    if actions is None:
        cls = torch.zeros(G, S * S, dtype=torch.uint8, device=b.device)
    else:
        a = torch.as_tensor(actions, dtype=torch.int32).to(b.device).contiguous()
        mf, mt = counters
    check(L.gmz_game_winning_scan(ptr(b), ptr(p), ptr(a), G, S, int(n_in_row), ptr(cls), ptr(mf), ptr(mt),
                                  _lib.stream_ptr(stream)))
    return cls


def _has_five(board, n_in_row=5):
    """Any run of n_in_row equal non-zero stones on an int8 [S,S] board (rows, columns, diagonals)."""
    S = board.shape[0]
    for b in (board, board.T):
        for k in range(S - n_in_row + 1):
            w = b[:, k:k + n_in_row]
            if ((w == w[:, :1]).all(axis=1) & (w[:, 0] != 0)).any():
                return True
    for b in (board, board[:, ::-1]):
        for off in range(-(S - n_in_row), S - n_in_row + 1):
            d = np.diagonal(b, off)
            for k in range(len(d) - n_in_row + 1):
                w = d[k:k + n_in_row]
                if w[0] != 0 and (w == w[0]).all():
                    return True
    return False


def _place_stones(rs, A, size, n, n_in_row):
    """n stones of alternating colour (black first) on random cells of an empty board with no n_in_row
    line, drawn from ``rs`` (redrawn until the board holds no line).  Returns (board int8[A], cells)."""
    while True:
        cells = rs.permutation(A)[:n]
        b = np.zeros(A, np.int8)
        b[cells[0::2]] = 1
        b[cells[1::2]] = -1
        if not _has_five(b.reshape(size, size), n_in_row):
            return b, cells


def seeded_openings(game_ids, size, seed, ks=(0, 4, 8), stagger=0, n_in_row=5):
    """SURVEY §8(d)'s synthetic starts: game ``gid`` draws from ``RandomState(seed + gid)`` an opening of
    k in ``ks`` stones (empty boards plus k in {0, 4, 8}) and, with ``stagger`` > 0, uniform(0, stagger)
    further stones (at most 2A/5 in all), so that the G games are spread over their lifetimes and some finish (and restart
    from the empty board) in any window of a few moves: the steady state a long self-play run is in.
    Returns (boards int8 [G,S,S], players int8 [G], last_moves int32 [G], move_counts int32 [G])."""
    A = size * size
    G = len(game_ids)
    boards = np.zeros((G, size, size), np.int8)
    players = np.ones(G, np.int8)
    last = np.full(G, -1, np.int32)
    counts = np.zeros(G, np.int32)
    for i, gid in enumerate(game_ids):
        rs = np.random.RandomState((int(seed) + int(gid)) % (2 ** 32))
        n = int(ks[rs.randint(len(ks))]) + (int(rs.randint(0, stagger + 1)) if stagger > 0 else 0)
        n = min(n, 2 * A // 5)  # small boards: room left to play, and a line-free draw stays likely
        b, cells = _place_stones(rs, A, size, n, n_in_row)
        boards[i] = b.reshape(size, size)
        players[i] = 1 if n % 2 == 0 else -1
        last[i] = cells[-1] if n else -1
        counts[i] = n
    return boards, players, last, counts


def random_openings(G, size, rs, max_stones, n_in_row=5):
    """Staggered game starts for measurements: game g gets an opening of uniform(0, max_stones) stones of
    alternating colour (black first) on random cells, with no n_in_row line on the board, the player to
    move after it and its last stone.  Returns (boards int8 [G,S,S], players int8 [G], last_moves int32 [G],
    move_counts int32 [G]) for BatchedSelfPlayEngine.set_positions / GameHistory.set_start."""
    A = size * size
    boards = np.zeros((G, size, size), np.int8)
    players = np.ones(G, np.int8)
    last = np.full(G, -1, np.int32)
    counts = rs.randint(0, max_stones + 1, G).astype(np.int32)
    for g in range(G):
        while True:
            n = int(counts[g])
            cells = rs.permutation(A)[:n]
            b = np.zeros(A, np.int8)
            b[cells[0::2]] = 1
            b[cells[1::2]] = -1
            if not _has_five(b.reshape(size, size), n_in_row):
                break
        boards[g] = b.reshape(size, size)
        players[g] = 1 if n % 2 == 0 else -1
        last[g] = cells[-1] if n else -1
    return boards, players, last, counts
