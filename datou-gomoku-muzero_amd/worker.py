"""``gpu_selfplay_worker`` — drop-in process target for the reference's self-play worker.

Replaces N ``universal_worker`` processes + the ``inference_server_worker`` (workers.py:129-241,
314-373) by ONE process per GPU that plays ``num_games`` games at once on the HIP engine, and emits
the same messages on the same queues:
  * per move of each game: ``ui_queue.put(SelfPlayMove())`` (workers.py:179);
  * per finished game: ``data_queue.put((GameRecord, [TrainingSlice], latest_model_step.value))``
    (workers.py:228-230), ``SelfPlayStatus(move_count, missed_fives, missed_totals)`` on the log and
    ui queues, ``GameCompletedNotice`` on the ui and trainer-event queues (workers.py:235-237).
Weights: the inference server's handshake (``InitialModelRequest`` -> ``ModelWeightsUpdate``,
workers.py:319-322) when ``initial_model_requests_queue``/``model_update_queue`` are given, and
hot-swap between moves (workers.py:332-335); otherwise ``state_dict`` (or seeded synthetic weights).
``openings`` (bench only): (boards, players, last_moves, move_counts) the first game of every slot
starts from, e.g. engine.random_openings — so a short measurement sees games at every stage; their
records hold the moves searched from there on.  ``worker_mode`` 1 (re-analysis, workers.py:243-305; off by default, config.py:85): the worker locks up to
``reanalysis_games`` stored games of the reference's SQLite database at a time (``db_path``), searches all
their positions in batches of ``num_games`` on a second engine that shares the network, rewrites their
slices and posts ``ReAnalysisStatus`` (reanalysis.py).  The current trainer step is the stored
checkpoint's ``train_step_count``, as the reference reads it (workers.py:247-249; decoded by
formats.RecordStore.load_trainer_state's restricted loader); no checkpoint yet -> wait 5 s.  Self-play
games in progress are kept and resume in mode 0.

Launch from main.py's ``process_definitions`` in place of the workers + server, e.g.
    mp.Process(target=gpu_selfplay_worker, args=(0, worker_mode, data_queue, log_status_queue,
               ui_queue, shutdown_event, None, None, replay_data_queue, trainer_event_queue,
               latest_model_step, log_queue, pause_event),
               kwargs=dict(device=0, num_games=1024, model_update_queue=model_update_queues[0],
                           initial_model_requests_queue=initial_model_requests_queue))
"""
import logging
import time
from concurrent.futures import ThreadPoolExecutor
from queue import Empty

import numpy as np
import torch

from . import records as R
from .config import from_any


def board_states_to_obs(boards, players, last_moves, H):
    """game.py:12-17 for a whole game at once: boards int8[n, A], players int8[n], last_moves int32[n]
    (-1 = none) -> float32 [n, 3, H, H] (the observation the search saw at each move)."""
    n = boards.shape[0]
    b = boards.reshape(n, H, H)
    p = players.reshape(n, 1, 1)
    obs = np.zeros((n, 3, H, H), dtype=np.float32)
    obs[:, 0] = b == p
    obs[:, 1] = b == -p
    has = last_moves >= 0
    obs[np.nonzero(has)[0], 2, last_moves[has] // H, last_moves[has] % H] = 1
    return obs


class GameHistory:
    """Per-game move history kept on the device, harvested one move behind (no per-move host sync).

    Every move appends, for each game, the position the search saw (board, player to move, last
    move), the search's improved policy (f64), root value and action at index move_count of the game's
    row in one of two banks.  ``after_play`` snapshots the move's status / move counts / missed-win
    counters / banks into pinned host buffers (async copies + an event) and flips the bank of every
    game that just ended, so the next game of that slot writes the other bank.  ``harvest`` (called
    after the NEXT move has been queued) waits for that event — already passed by then — and copies
    each finished game's rows to the host with DMA copies on a side stream.  A bank is rewritten only
    when its slot's next game ends too, at least 2*N_IN_ROW-1 moves later, long after the harvest."""

    def __init__(self, G, A, device, min_game_len=9):
        assert min_game_len >= 2, "a bank must survive one move after its game ended"
        L = A  # a game has at most A moves
        self.G, self.A, self.L, self.dev = G, A, L, device
        z = lambda *sh, dt: torch.zeros(*sh, dtype=dt, device=device)  # noqa: E731
        self.board = z(2, G, L, A, dt=torch.int8)
        self.pol = z(2, G, L, A, dt=torch.float64)
        self.val = z(2, G, L, dt=torch.float32)
        self.act = z(2, G, L, dt=torch.int32)
        self.player = z(2, G, L, dt=torch.int8)
        self.last = z(2, G, L, dt=torch.int32)
        self.bank = z(G, dt=torch.int64)
        # first recorded move index per (bank, game slot): 0 for games from the empty board; a game
        # started from a given position (set_start) records from its move count on
        self.start = np.zeros((2, G), dtype=np.int64)
        self.gidx = torch.arange(G, device=device)
        self.side = torch.cuda.Stream(device)
        self.k = 0
        pin = lambda dt: torch.zeros(G, dtype=dt).pin_memory()  # noqa: E731
        self.snaps = [dict(status=pin(torch.int8), mc=pin(torch.int32), bank=pin(torch.int64), mf=pin(torch.int32),
                           mt=pin(torch.int32), act=pin(torch.int32), ev=None) for _ in range(2)]

    def set_start(self, move_counts):
        """The current games start from positions with ``move_counts`` stones (before their first
        move; every slot is still on bank 0): their records hold the searched moves from there on."""
        assert self.k == 0, "set_start before the first move"
        self.start[0] = np.asarray(move_counts, dtype=np.int64)
        self.start[1] = 0

    def record(self, boards, players, last_moves, move_counts, policy, value, action):
        """Append this move's search inputs/outputs (all device tensors, before the move is played)."""
        i = (self.bank, self.gidx, move_counts.long().clamp(0, self.L - 1))
        self.board[i] = boards.reshape(self.G, self.A)
        self.player[i] = players
        self.last[i] = last_moves
        self.pol[i] = policy
        self.val[i] = value
        self.act[i] = action

    def after_play(self, status, move_counts, action, missed_f, missed_t):
        """Snapshot the move's results (async) and start the next game of every finished slot in the
        other bank; the missed-win counters of finished games restart from zero."""
        sn = self.snaps[self.k & 1]
        self.k += 1
        for key, t in (("status", status), ("mc", move_counts), ("bank", self.bank), ("mf", missed_f),
                       ("mt", missed_t), ("act", action)):
            sn[key].copy_(t, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        sn["ev"] = ev
        ended = (status != 2) & (status != 3)
        missed_f.masked_fill_(ended, 0)
        missed_t.masked_fill_(ended, 0)
        self.bank ^= ended.long()
        return sn

    def harvest(self, sn):
        """Finished games of snapshot ``sn`` -> list of (game index, winner, n_moves, missed_fives,
        missed_totals, boards int8[n,A], players int8[n], last_moves int32[n], policies f64[n,A],
        values f32[n], actions int32[n]) on the host.  Games whose search found no legal move
        (action -1, workers.py:169-170) are abandoned without a record, as the reference does."""
        if sn is None or sn["ev"] is None:
            return []
        sn["ev"].synchronize()
        st = sn["status"].numpy()
        fin = np.nonzero((st != 2) & (st != 3))[0]
        out = []
        if len(fin) == 0:
            return out
        mc, bank, act = sn["mc"].numpy(), sn["bank"].numpy(), sn["act"].numpy()
        jobs = []
        with torch.cuda.stream(self.side):
            self.side.wait_event(sn["ev"])
            for g in fin:
                bk = int(bank[g])
                s0 = int(self.start[bk, g])
                self.start[bk, g] = 0  # this bank's next game starts from the empty board
                if act[g] < 0:
                    continue
                n = int(mc[g]) + 1 - s0
                host = [torch.empty((n,) + tuple(t.shape[3:]), dtype=t.dtype, pin_memory=True)
                        for t in (self.board, self.player, self.last, self.pol, self.val, self.act)]
                for h, t in zip(host, (self.board, self.player, self.last, self.pol, self.val, self.act)):
                    h.copy_(t[bk, g, s0:s0 + n], non_blocking=True)
                jobs.append((int(g), int(st[g]), n, int(sn["mf"][g]), int(sn["mt"][g]), host))
        self.side.synchronize()
        for g, winner, n, mf, mt, host in jobs:
            out.append((g, winner, n, mf, mt) + tuple(h.numpy() for h in host))
        return out


def gpu_selfplay_worker(worker_id, worker_mode, data_queue, log_status_queue, ui_queue, shutdown_event,
                        request_queue=None, result_queue=None, replay_data_queue=None, trainer_event_queue=None,
                        latest_model_step=None, log_queue=None, pause_event=None, *, device=0, num_games=1024,
                        model_update_queue=None, initial_model_requests_queue=None, state_dict=None, cfg=None,
                        seed=0, max_moves=None, emit_move_notices=True, db_path="outputs/training_state.db",
                        reanalysis_games=64, precision="fp16", move_times=None, streams=None, openings=None):
    logger = logging.getLogger("GpuSelfPlay-%s" % worker_id)
    if log_queue is not None:
        try:
            from logger_config import setup_worker_logging  # reference logging (logger_config.py:21)
            setup_worker_logging(log_queue)
        except Exception:
            pass
    if cfg is None:
        try:
            from config import config as cfg  # the reference's global config, when launched from main.py
        except Exception:
            cfg = None
    c = from_any(cfg)
    torch.cuda.set_device(device)
    from . import engine as E, network as N, weights as W

    if state_dict is None and model_update_queue is not None:
        if initial_model_requests_queue is not None:
            try:
                from ipc_messages import InitialModelRequest
                initial_model_requests_queue.put(InitialModelRequest())
            except Exception:
                initial_model_requests_queue.put(None)
        state_dict = model_update_queue.get(timeout=120).weights
    if state_dict is None:
        state_dict = W.synthetic_state_dict(c, seed=seed, with_projection=False)
    G = int(num_games)
    net = N.GomokuNetHip(state_dict, c, num_slots=E.hidden_slots(c, G), max_rows=G, precision=precision)
    eng = E.make_engine(c, num_games=G, net=net, seed=seed + 7919 * int(worker_id), streams=streams)
    eng.reset_games()
    H, A = c.BOARD_SIZE, c.ACTION_SPACE_SIZE
    hist = GameHistory(G, A, eng.device, min_game_len=2 * c.N_IN_ROW - 1)
    if openings is not None:  # bench: the first games start from given positions (E.random_openings)
        eng.set_positions(*openings)
        hist.set_start(openings[3])
    pool = ThreadPoolExecutor(max_workers=4)
    moves_done = 0
    # missed-win counters of workers.py:191-203, accumulated on the device move by move by the batched
    # find_winning_moves scan (gmz_game_winning_scan) instead of a Python scan per finished game
    missed_f = torch.zeros(G, dtype=torch.int32, device=eng.device)
    missed_t = torch.zeros(G, dtype=torch.int32, device=eng.device)

    def finish_game(winner, n, mf, mt, boards, players, lasts, pols, vals, acts):
        obs = board_states_to_obs(boards, players, lasts, H)
        record, slices = R.build_game_record(list(obs), [int(x) for x in acts], list(pols), list(vals),
                                             list(boards.reshape(n, H, H)), winner, c.DISCOUNT, c.N_STEPS,
                                             c.NUM_UNROLL_STEPS)
        version = latest_model_step.value if latest_model_step is not None else 0
        if slices:
            data_queue.put((record, slices, version))
        status = R.SelfPlayStatus(n, mf, mt)
        if log_status_queue is not None:
            log_status_queue.put(status)
        if ui_queue is not None:
            ui_queue.put(status)
            ui_queue.put(R.GameCompletedNotice())
        if trainer_event_queue is not None:
            trainer_event_queue.put(R.GameCompletedNotice())

    def move_notices(n):
        for _ in range(n):
            if ui_queue.full():
                break
            ui_queue.put(R.SelfPlayMove())

    def drain(sn):
        """Host side of a played move (one move behind the device): per-move UI notices, finished games."""
        if sn is None:
            return
        for item in hist.harvest(sn):
            pool.submit(finish_game, *item[1:])
        if emit_move_notices and ui_queue is not None:
            pool.submit(move_notices, int((sn["act"].numpy() >= 0).sum()))

    reanalyser, store = None, None
    pending = None  # snapshot of the last played move, harvested after the next move is queued

    logger.info("GPU self-play worker %s: %d games on cuda:%d" % (worker_id, G, device))
    while not shutdown_event.is_set():
        mode = getattr(worker_mode, "value", 0) if worker_mode is not None else 0
        if mode == 0 and pause_event is not None and pause_event.is_set():  # workers.py:158-160
            time.sleep(5)
            continue
        if model_update_queue is not None:  # the inference server's hot swap (workers.py:332-335)
            try:
                net.load_state_dict(model_update_queue.get_nowait().weights)
                logger.info("Inference model updated.")
            except Empty:
                pass
        if mode == 1:  # re-analysis (workers.py:243-305)
            from . import formats as F, reanalysis as RA
            if reanalyser is None:
                reanalyser = RA.Reanalyser(E.BatchedSelfPlayEngine(c, num_games=G, net=net,
                                                                   seed=seed + 104729 * (int(worker_id) + 1)))
                store = F.RecordStore(db_path)
            try:  # workers.py:247-249: the trainer step comes from the stored checkpoint
                ts = store.load_trainer_state()
            except Exception as e:
                logger.error("Worker %s: unreadable trainer_state: %s" % (worker_id, e))
                ts = None
            if not ts:
                time.sleep(5)
                continue
            step = int(ts.get("train_step_count", 0))
            try:
                n = RA.reanalysis_step(reanalyser, store, step, c, reanalysis_games, ui_queue)
            except Exception as e:  # workers.py:297-299
                logger.error("Error in re-analysis for worker %s: %s" % (worker_id, e))
                n = 0
            if n == 0:
                time.sleep(5)
            continue
        if mode != 0:  # workers.py:301-303
            logger.warning("Worker %s: Unknown worker mode '%s'. Sleeping." % (worker_id, mode))
            time.sleep(10)
            continue
        b, p, lm, mc = eng.game_state()
        pol, val, act = eng.search()
        eng.winning_scan(b, p, act, counters=(missed_f, missed_t))  # position before the move
        hist.record(b, p, lm, mc, pol, val, act)
        status = eng.play(reset_finished=True)
        sn = hist.after_play(status, mc, act, missed_f, missed_t)
        drain(pending)  # the previous move's host work runs while this move is on the device
        pending = sn
        moves_done += 1
        if move_times is not None:  # tools/worker_bench.py: host clock after each move was queued
            move_times.append(time.perf_counter())
        if max_moves is not None and moves_done >= max_moves:
            break
    drain(pending)
    pool.shutdown(wait=True)
    if move_times is not None:
        torch.cuda.synchronize()
        move_times.append(time.perf_counter())  # every move played and every record posted
    eng.close()
    if reanalyser is not None:
        reanalyser.eng.close()
        store.close(checkpoint=False)
