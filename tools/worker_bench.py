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


def consumer(qs, stop, counts):
    """Drain every queue (unpickling the payloads) until told to stop and the queues are empty."""
    import queue as Q
    n = {k: 0 for k in qs}
    slices = 0
    while True:
        busy = False
        for k, q in qs.items():
            try:
                item = q.get(timeout=0.01)
            except Q.Empty:
                continue
            busy = True
            n[k] += 1
            if k == "data":
                slices += len(item[1])
        if not busy and stop.is_set():
            break
    counts.update(n)
    counts["slices"] = slices


class Ev:
    def __init__(self):
        self.f = False

    def is_set(self):
        return self.f


def main():
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
    cons = ctx.Process(target=consumer, args=(qs, stop, counts))
    cons.start()
    from datou_gomoku_muzero_amd.worker import gpu_selfplay_worker
    from datou_gomoku_muzero_amd.config import GmzConfig
    cfg = GmzConfig(BOARD_SIZE=a.size, NUM_SIMULATIONS=a.sims)
    times = []
    t0 = time.perf_counter()
    gpu_selfplay_worker(0, None, qs["data"], qs["log"], qs["ui"], Ev(), trainer_event_queue=qs["trainer"],
                        num_games=a.games, cfg=cfg, max_moves=a.warmup + a.moves,
                        emit_move_notices=not a.no_move_notices, move_times=times)
    stop.set()
    cons.join(timeout=300)
    steady = times[-1] - times[a.warmup - 1]
    print(json.dumps({"metric": "drop-in worker self-play moves/sec (%dx%d, %d sims)" % (a.size, a.size, a.sims),
                      "value": a.games * a.moves / steady, "unit": "moves/s", "games": a.games, "moves": a.moves,
                      "warmup_moves": a.warmup, "steady_s": steady, "setup_and_warmup_s": times[a.warmup - 1] - t0,
                      "queues": "torch.multiprocessing (spawn) Queues, main.py sizes; consumer process unpickles",
                      "move_notices": not a.no_move_notices, "messages": dict(counts)}))


if __name__ == "__main__":
    main()
