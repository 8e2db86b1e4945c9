"""Drop-in single-game MCTS engines with the reference's interface (/root/reference/mcts.py:50-64).

    engine = HipMuZeroMCTS(worker_id, request_queue, result_queue)
    policy, value, action = engine.search(game)
    policies, values, actions = engine.search_batch(games)      # G games in one batched search

The tree search (select / expand / backup / sequential halving / decision) runs in the HIP kernels
of csrc/gmz_tree.hip on a one-game ``BatchedSelfPlayEngine``; the network is reached through the
reference's inference-queue protocol, request for request:
  * ``(worker_id, 'initial', obs f32[3,H,W])`` -> ``(p f32[A], v, h)``           (mcts.py:73-75)
  * ``(worker_id, 'recurrent_batch', (h[k,...], a int32[k]))`` -> ``(p, v, h, r)`` (mcts.py:77-85),
    with the reference's k duplicate rows per wave (k = len(selected_children_actions));
so MuZero issues 1 'initial' + one 'recurrent_batch' per wave and AlphaZero NUM_SIMULATIONS
'initial' requests, exactly as the reference (tests/test_mcts_logic.py:116-136 count them).
Gumbel noise is drawn from the global numpy RandomState (``np.random.gumbel(0, 1, A)``,
mcts.py:312) so a seeded run reproduces the reference's search.

Returns (policy float64[A], value np.float32, action int); on an inference timeout at the root:
(zeros(A), 0.0, -1) as the reference (mcts.py:298-302); a timed-out 'recurrent_batch' is logged and
the same wave is requested again, as the reference's ``continue`` does (mcts.py:82-85, 337).
"""
import logging
from queue import Empty

import numpy as np
import torch

from . import _lib
from .config import from_any
from .engine import BatchedSelfPlayEngine
from ._lib import check, ptr

_TIMEOUT = 20


class _QueueNet:
    """Engine network backend that forwards every request through the reference queue protocol."""

    def __init__(self, owner):
        self.o = owner
        self.hidden = {}  # slot -> hidden state object returned by the inference server

    def initial(self, obs, out_slot, logits, value, stream):
        o = self.o
        slots = out_slot.cpu().numpy()
        ob = obs.cpu().numpy()
        for r in range(obs.shape[0]):
            if slots[r] < 0:
                continue
            o.request_queue.put((o.worker_id, "initial", np.ascontiguousarray(ob[r], dtype=np.float32)))
            p, v, h = o.result_queue.get(timeout=_TIMEOUT)
            self.hidden[int(slots[r])] = h
            logits[r].copy_(torch.as_tensor(np.asarray(p, dtype=np.float32).reshape(-1)))
            value[r] = float(np.float32(v))

    def recurrent(self, in_slot, action, out_slot, logits, value, reward, stream):
        o = self.o
        eng = o._engine
        kk = torch.zeros(eng.G, dtype=torch.int32, device=eng.device)
        check(eng.lib.gmz_engine_wave_k(eng.handle, ptr(kk), stream))
        ks = kk.cpu().numpy()
        ins, acts, outs = in_slot.cpu().numpy(), action.cpu().numpy(), out_slot.cpu().numpy()
        for r in range(in_slot.shape[0]):
            k = int(ks[r])
            if outs[r] < 0 or k <= 0:
                continue
            h = self.hidden[int(ins[r])]
            hb = np.concatenate([h] * k, axis=0)
            while True:
                o.request_queue.put((o.worker_id, "recurrent_batch", (hb, np.array([acts[r]] * k, dtype=np.int32))))
                try:
                    p, v, hn, rw = o.result_queue.get(timeout=_TIMEOUT)
                    break
                except Empty:  # mcts.py:82-85 + 337: warn, then the same wave (same leaves) is re-requested
                    o.logger.warning("Worker %s timed out waiting for recurrent inference." % o.worker_id)
            self.hidden[int(outs[r])] = hn[0:1]
            logits[r].copy_(torch.as_tensor(np.asarray(p, dtype=np.float32)[0].reshape(-1)))
            value[r] = float(np.asarray(v, dtype=np.float32).reshape(-1)[0])
            reward[r] = float(np.asarray(rw, dtype=np.float32).reshape(-1)[0])


class _HipGumbelMCTS:
    MODE = None

    def __init__(self, worker_id, request_queue, result_queue, cfg=None, device="cuda"):
        self.worker_id = worker_id
        self.request_queue = request_queue
        self.result_queue = result_queue
        self.logger = logging.getLogger("MCTS-%s-%s" % (self.__class__.__name__, worker_id))
        self._cfg_src = cfg
        self._device = device
        self._engine = None
        self._key = None

    def _get_engine(self, G=1):
        if self._cfg_src is None:
            try:  # the reference's global config singleton, read at call time like mcts.py does
                from config import config as ref_config  # noqa: WPS433
                src = ref_config
            except Exception:
                src = None
        else:
            src = self._cfg_src
        cfg = from_any(src, MCTS_IMPLEMENTATION=self.MODE)
        key = (G,) + tuple(sorted(cfg.as_dict().items()))
        if self._engine is None or key != self._key:
            net = _QueueNet(self)
            self._engine = BatchedSelfPlayEngine(cfg, num_games=G, net=net, device=self._device)
            self._net = net
            self._key = key
        return self._engine

    def search(self, game):
        try:  # mcts.py:289-292 drain stale results
            while True:
                self.result_queue.get_nowait()
        except Empty:
            pass
        eng = self._get_engine()
        self._net.hidden.clear()
        A = eng.A
        board = np.asarray(game.board, dtype=np.int8).reshape(1, -1)
        lm = -1 if game.last_move is None else int(game.last_move[0]) * eng.size + int(game.last_move[1])
        eng.set_positions(board, [game.current_player], [lm], [getattr(game, "move_count", int((board != 0).sum()))])
        gumbel = np.random.gumbel(0, 1, A)  # mcts.py:312 / 221 — global RandomState
        try:
            pol, val, act = eng.search(gumbel=gumbel.reshape(1, A))
        except Empty:
            self.logger.warning("Worker %s timed out on inference." % self.worker_id)
            return np.zeros(A), 0.0, -1
        torch.cuda.synchronize()
        a = int(act[0].item())
        if a < 0:
            return np.zeros(A), 0.0, -1
        return pol[0].cpu().numpy().astype(np.float64), np.float32(val[0].item()), a


    def search_batch(self, games):
        """G games in one batched search -> (policy f64[G,A], value f32[G], action int32[G]).

        Same results as ``[self.search(g) for g in games]`` from the same global RandomState (the
        Gumbel noise is drawn game after game, mcts.py:312); the network requests still go through
        the queue protocol, row by row.  An inference timeout returns zeros/0/-1 for every game."""
        try:
            while True:
                self.result_queue.get_nowait()
        except Empty:
            pass
        G = len(games)
        eng = self._get_engine(G)
        self._net.hidden.clear()
        A, S = eng.A, eng.size
        boards = np.stack([np.asarray(g.board, dtype=np.int8).reshape(-1) for g in games])
        lms = [-1 if g.last_move is None else int(g.last_move[0]) * S + int(g.last_move[1]) for g in games]
        mcs = [getattr(g, "move_count", int((b != 0).sum())) for g, b in zip(games, boards)]
        eng.set_positions(boards, [g.current_player for g in games], lms, mcs)
        gumbel = np.random.gumbel(0, 1, (G, A))
        try:
            pol, val, act = eng.search(gumbel=gumbel)
        except Empty:
            self.logger.warning("Worker %s timed out on inference." % self.worker_id)
            return np.zeros((G, A)), np.zeros(G, np.float32), np.full(G, -1, np.int32)
        torch.cuda.synchronize()
        pol, val, act = pol.cpu().numpy().astype(np.float64), val.cpu().numpy().astype(np.float32), act.cpu().numpy()
        bad = act < 0
        pol[bad], val[bad] = 0.0, 0.0
        return pol, val, act.astype(np.int32)


class HipMuZeroMCTS(_HipGumbelMCTS):
    """MuZeroMCTS (mcts.py:283-362) on the MI355X tree kernels."""
    MODE = "MuZero"


class HipAlphaZeroMCTS(_HipGumbelMCTS):
    """AlphaZeroMCTS (mcts.py:191-280) on the MI355X tree kernels."""
    MODE = "AlphaZero"


def make_engine(worker_id, request_queue, result_queue, cfg=None):
    """workers.py:134-142: pick the implementation from config.MCTS_IMPLEMENTATION."""
    c = from_any(cfg)
    if c.MCTS_IMPLEMENTATION == "AlphaZero":
        return HipAlphaZeroMCTS(worker_id, request_queue, result_queue, cfg)
    if c.MCTS_IMPLEMENTATION == "MuZero":
        return HipMuZeroMCTS(worker_id, request_queue, result_queue, cfg)
    raise ValueError("Unknown MCTS implementation in config: '%s'" % c.MCTS_IMPLEMENTATION)


__all__ = ["HipMuZeroMCTS", "HipAlphaZeroMCTS", "make_engine", "_lib"]
