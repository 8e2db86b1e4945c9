"""Tree-kernel microbenchmark: G games × M moves of 15×15 MuZero/400 with the HashNet device
backend (network cost ≈ 0), so the time is the search kernels alone."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import datou_gomoku_muzero_amd.engine as E  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--games", type=int, default=1024)
ap.add_argument("--moves", type=int, default=4)
ap.add_argument("--size", type=int, default=15)
ap.add_argument("--sims", type=int, default=400)
ap.add_argument("--mode", default="MuZero")
a = ap.parse_args()
eng = E.BatchedSelfPlayEngine(None, num_games=a.games, BOARD_SIZE=a.size, NUM_SIMULATIONS=a.sims,
                              MCTS_IMPLEMENTATION=a.mode, seed=1)
eng.reset_games()
eng.search(); eng.play(); torch.cuda.synchronize()
t0 = time.time()
for m in range(a.moves):
    eng.search()
    eng.play()
torch.cuda.synchronize()
dt = time.time() - t0
print("games %d moves %d waves/move %d: %.3f s  -> %.1f moves/s, %.1f us/wave" % (
    a.games, a.moves, eng.waves_last, dt, a.games * a.moves / dt, dt / a.moves / max(1, eng.waves_last) * 1e6))
