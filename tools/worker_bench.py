"""End-to-end throughput of the drop-in self-play worker (worker.py:gpu_selfplay_worker) with the
reference's queue protocol: G games on one GPU, records/slices/status messages built on the host.
Prints moves/s of the worker loop (compare with bench.py, which times the engine alone)."""
import argparse
import os
import queue
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--games", type=int, default=1024)
ap.add_argument("--moves", type=int, default=12)
ap.add_argument("--size", type=int, default=15)
ap.add_argument("--sims", type=int, default=400)
a = ap.parse_args()

from datou_gomoku_muzero_amd.worker import gpu_selfplay_worker  # noqa: E402
from datou_gomoku_muzero_amd.config import GmzConfig  # noqa: E402


class Ev:
    def __init__(self):
        self.f = False

    def is_set(self):
        return self.f


class Sink(queue.Queue):
    """unbounded queue that drops payloads (counts them) so memory stays flat"""

    def __init__(self):
        super().__init__()
        self.n = 0

    def put(self, item, block=True, timeout=None):
        self.n += 1

    def full(self):
        return False


cfg = GmzConfig(BOARD_SIZE=a.size, NUM_SIMULATIONS=a.sims)
dq, lq, uq, tq = Sink(), Sink(), Sink(), Sink()
t0 = time.time()
gpu_selfplay_worker(0, None, dq, lq, uq, Ev(), trainer_event_queue=tq, num_games=a.games, cfg=cfg, max_moves=2)
torch.cuda.synchronize()
t1 = time.time()
gpu_selfplay_worker(0, None, dq, lq, uq, Ev(), trainer_event_queue=tq, num_games=a.games, cfg=cfg, max_moves=a.moves)
torch.cuda.synchronize()
t2 = time.time()
print("worker: %d games x %d moves in %.2f s -> %.1f moves/s (includes engine + net construction ~%.1f s); "
      "records %d, ui messages %d" % (a.games, a.moves, t2 - t1, a.games * a.moves / (t2 - t1), t1 - t0, dq.n, uq.n))
