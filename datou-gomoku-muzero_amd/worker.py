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
``worker_mode`` 1 (re-analysis, workers.py:243-305; off by default, config.py:85): the worker locks up to
``reanalysis_games`` stored games of the reference's SQLite database at a time (``db_path``), searches all
their positions in batches of ``num_games`` on a second engine that shares the network, rewrites their
slices and posts ``ReAnalysisStatus`` (reanalysis.py).  The current trainer step is
``latest_model_step.value`` (the reference reads it from the pickled trainer_state blob, which is not
decoded here; formats.py).  Self-play games in progress are kept and resume in mode 0.

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


def _board_state(board, player, last_move):
    """game.py:12-17 on the host (records keep the observation the search saw)."""
    obs = np.zeros((3,) + board.shape, dtype=np.float32)
    obs[0] = board == player
    obs[1] = board == -player
    if last_move is not None:
        obs[2, last_move[0], last_move[1]] = 1
    return obs


class _Game:
    __slots__ = ("obs", "actions", "policies", "values", "boards")

    def __init__(self):
        self.obs, self.actions, self.policies, self.values, self.boards = [], [], [], [], []


def gpu_selfplay_worker(worker_id, worker_mode, data_queue, log_status_queue, ui_queue, shutdown_event,
                        request_queue=None, result_queue=None, replay_data_queue=None, trainer_event_queue=None,
                        latest_model_step=None, log_queue=None, pause_event=None, *, device=0, num_games=1024,
                        model_update_queue=None, initial_model_requests_queue=None, state_dict=None, cfg=None,
                        seed=0, max_moves=None, emit_move_notices=True, db_path="outputs/training_state.db",
                        reanalysis_games=64):
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
    net = N.GomokuNetHip(state_dict, c, num_slots=G * (c.NUM_SIMULATIONS + 2), max_rows=G)
    eng = E.BatchedSelfPlayEngine(c, num_games=G, net=net, seed=seed + 7919 * int(worker_id))
    eng.reset_games()
    H, A = c.BOARD_SIZE, c.ACTION_SPACE_SIZE
    games = [_Game() for _ in range(G)]
    pool = ThreadPoolExecutor(max_workers=4)
    moves_done = 0
    # missed-win counters of workers.py:191-203, accumulated on the device move by move by the batched
    # find_winning_moves scan (gmz_game_winning_scan) instead of a Python scan per finished game
    missed_f = torch.zeros(G, dtype=torch.int32, device=eng.device)
    missed_t = torch.zeros(G, dtype=torch.int32, device=eng.device)

    def finish_game(g, winner, move_count, mf, mt):
        record, slices = R.build_game_record(g.obs, g.actions, g.policies, g.values, g.boards, winner,
                                             c.DISCOUNT, c.N_STEPS, c.NUM_UNROLL_STEPS)
        version = latest_model_step.value if latest_model_step is not None else 0
        if slices:
            data_queue.put((record, slices, version))
        status = R.SelfPlayStatus(move_count, mf, mt)
        if log_status_queue is not None:
            log_status_queue.put(status)
        if ui_queue is not None:
            ui_queue.put(status)
            ui_queue.put(R.GameCompletedNotice())
        if trainer_event_queue is not None:
            trainer_event_queue.put(R.GameCompletedNotice())

    reanalyser, store = None, None

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
            step = latest_model_step.value if latest_model_step is not None else 0
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
        status = eng.play(reset_finished=True)
        torch.cuda.synchronize()
        mf_all, mt_all = missed_f.cpu().numpy(), missed_t.cpu().numpy()
        b, p, lm, mc = b.cpu().numpy(), p.cpu().numpy(), lm.cpu().numpy(), mc.cpu().numpy()
        pol, val, act, status = pol.cpu().numpy(), val.cpu().numpy(), act.cpu().numpy(), status.cpu().numpy()
        ended = torch.from_numpy((status != 2) & (status != 3)).to(eng.device)
        missed_f.masked_fill_(ended, 0)
        missed_t.masked_fill_(ended, 0)
        for i in range(G):
            a = int(act[i])
            if a < 0:  # workers.py:169-170 (no legal move)
                games[i] = _Game()
                continue
            gm = games[i]
            last = None if lm[i] < 0 else (int(lm[i]) // H, int(lm[i]) % H)
            gm.obs.append(_board_state(b[i], int(p[i]), last))
            gm.policies.append(pol[i].copy())
            gm.values.append(np.float32(val[i]))
            gm.actions.append(a)
            gm.boards.append(b[i].copy())
            if emit_move_notices and ui_queue is not None and not ui_queue.full():
                ui_queue.put(R.SelfPlayMove())
            st = int(status[i])
            if st != 2:
                pool.submit(finish_game, gm, st, int(mc[i]) + 1, int(mf_all[i]), int(mt_all[i]))
                games[i] = _Game()
        moves_done += 1
        if max_moves is not None and moves_done >= max_moves:
            break
    pool.shutdown(wait=True)
    eng.close()
    if reanalyser is not None:
        reanalyser.eng.close()
        store.close(checkpoint=False)
