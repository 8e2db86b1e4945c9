"""End-to-end throughput of the drop-in self-play worker (worker.py:gpu_selfplay_worker) with the
reference's process graph: real torch.multiprocessing queues (main.py:60-78 sizes) and a consumer
process that drains them like the reference's DataLoader / DisplayManager / log readers do
(unpickling every GameRecord + TrainingSlice payload).  G games on one GPU.

Prints one JSON line: worker moves/s over the steady-state moves (after --warmup moves) until every
record of those moves has been posted, the engine-only bench figure for comparison is bench.py's."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def consumer(qs, counts):
    """One reader thread per queue (blocking get, unpickling every payload) until its None sentinel."""
    import threading
    n, slices = {}, {}

    def read(k, q):
        c = s = 0
        while True:
            item = q.get()
            if item is None:
                break
            c += 1
            if k == "data":
                s += len(item[1])
        n[k], slices[k] = c, s

    th = [threading.Thread(target=read, args=kq) for kq in qs.items()]
    for t in th:
        t.start()
    for t in th:
        t.join()
    counts.update(n)
    counts["slices"] = slices.get("data", 0)


class Ev:
    def __init__(self):
        self.f = False

    def is_set(self):
        return self.f


def main():
    import faulthandler
    import threading
    faulthandler.dump_traceback_later(90, repeat=True)  # a stuck run names where it waits
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=1024)
    ap.add_argument("--moves", type=int, default=24)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--size", type=int, default=15)
    ap.add_argument("--sims", type=int, default=400)
    ap.add_argument("--no-move-notices", action="store_true")
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    qs = {"data": ctx.Queue(maxsize=50000), "ui": ctx.Queue(), "log": ctx.Queue(), "trainer": ctx.Queue()}
    stop = ctx.Event()
    mgr = ctx.Manager()
    counts = mgr.dict()
    cons = ctx.Process(target=consumer, args=(qs, counts))
    cons.start()
    from datou_gomoku_muzero_amd.worker import gpu_selfplay_worker
    from datou_gomoku_muzero_amd.config import GmzConfig
    cfg = GmzConfig(BOARD_SIZE=a.size, NUM_SIMULATIONS=a.sims)
    times = []
    t0 = time.perf_counter()

    def progress():
        while not stop.is_set():
            time.sleep(10)
            print("worker_bench: %d moves after %.0f s" % (len(times), time.perf_counter() - t0), file=sys.stderr, flush=True)
    threading.Thread(target=progress, daemon=True).start()
    gpu_selfplay_worker(0, None, qs["data"], qs["log"], qs["ui"], Ev(), trainer_event_queue=qs["trainer"],
                        num_games=a.games, cfg=cfg, max_moves=a.warmup + a.moves,
                        emit_move_notices=not a.no_move_notices, move_times=times)
    print("worker_bench: worker done after %.1f s, waiting for the consumer" % (time.perf_counter() - t0), file=sys.stderr,
          flush=True)
    stop.set()
    for q in qs.values():
        q.put(None)
    cons.join(timeout=300)
    t_cons = time.perf_counter() - t0
    steady = times[-1] - times[a.warmup - 1]
    # the bare engine on the same box and workload (bench.py's step: search + play), for the ratio
    from datou_gomoku_muzero_amd import engine as E, network as N, weights as W
    sd = W.synthetic_state_dict(cfg, seed=0, with_projection=False)
    net = N.GomokuNetHip(sd, cfg, num_slots=E.hidden_slots(cfg, a.games), max_rows=a.games)
    eng = E.make_engine(cfg, num_games=a.games, net=net, seed=0)  # the worker's own choice of streams
    eng.reset_games()
    for i in range(a.warmup + a.moves):
        if i == a.warmup:
            torch.cuda.synchronize()
            te = time.perf_counter()
        eng.search()
        eng.play(reset_finished=True)
    torch.cuda.synchronize()
    engine_rate = a.games * a.moves / (time.perf_counter() - te)
    print(json.dumps({"metric": "drop-in worker self-play moves/sec (%dx%d, %d sims)" % (a.size, a.size, a.sims),
                      "value": a.games * a.moves / steady, "unit": "moves/s", "games": a.games, "moves": a.moves,
                      "warmup_moves": a.warmup, "steady_s": steady, "setup_and_warmup_s": times[a.warmup - 1] - t0,
                      "queues": "torch.multiprocessing (spawn) Queues, main.py sizes; consumer process unpickles",
                      "move_notices": not a.no_move_notices, "messages": dict(counts),
                      "consumer_done_s": t_cons, "engine_only_moves_per_s": engine_rate,
                      "worker_over_engine": a.games * a.moves / steady / engine_rate,
                      "streams": E.default_streams(cfg, a.games)}))


if __name__ == "__main__":
    main()
