"""Self-play moves/s of one engine with all G games vs engine.SplitSelfPlayEngine (G/parts games per
HIP stream, waves interleaved, tower grid capped at --max-grid CUs), same box, same process layout as
bench.py's step.  The sweep that chose 2 streams and 3/4 of the CUs: tools/dual_probe.sh,
profiles/r02_dual_stream_sweep.txt.
  python tools/dual_stream_probe.py --parts 1|2|4 [--max-grid 192 --games 1024 --moves 6 --warmup 2]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--parts", type=int, default=2)
ap.add_argument("--max-grid", type=int, default=None)
ap.add_argument("--games", type=int, default=1024)
ap.add_argument("--moves", type=int, default=6)
ap.add_argument("--warmup", type=int, default=2)
ap.add_argument("--size", type=int, default=15)
ap.add_argument("--sims", type=int, default=400)
ap.add_argument("--mode", default="MuZero")
ap.add_argument("--blocks", type=int, default=8)
a = ap.parse_args()
from datou_gomoku_muzero_amd import engine as E, network as N, weights as W  # noqa: E402
from datou_gomoku_muzero_amd.config import GmzConfig  # noqa: E402

cfg = GmzConfig(BOARD_SIZE=a.size, NUM_SIMULATIONS=a.sims, MCTS_IMPLEMENTATION=a.mode, NUM_RES_BLOCKS=a.blocks)
sd = W.synthetic_state_dict(cfg, seed=1234, with_projection=False)
net = N.GomokuNetHip(sd, cfg, num_slots=E.hidden_slots(cfg, a.games), max_rows=a.games)
if a.parts == 1:
    eng = E.BatchedSelfPlayEngine(cfg, num_games=a.games, net=net, seed=7)
else:
    eng = E.SplitSelfPlayEngine(cfg, num_games=a.games, net=net, seed=7, parts=a.parts, max_grid=a.max_grid)
eng.reset_games()
for _ in range(a.warmup):
    eng.search()
    eng.play(reset_finished=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.moves):
    eng.search()
    eng.play(reset_finished=True)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(json.dumps({"size": a.size, "mode": a.mode, "parts": a.parts, "max_grid": a.max_grid, "games": a.games, "moves_per_s": a.games * a.moves / dt,
                  "ms_per_move": dt / a.moves * 1e3}))
