"""Phase breakdown of the fused tree kernel k_expand_select in the real self-play step: s_memtime
cycle stamps around each phase, summed over waves by lane 0 (library built with -DGMZ_TREE_PROF:
  make -C datou-gomoku-muzero_amd/csrc OBJDIR=../_alt/build_prof OUT=../_alt/libgmz_prof.so EXTRA=-DGMZ_TREE_PROF).
  python tools/tree_prof.py [--games 1024 --moves 3]
Cycles are per wave (one game); a non-root level = fetch + q/hint issue + improved policy + argmax + hint."""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("GMZ_LIB", os.path.join(REPO, "datou-gomoku-muzero_amd", "_alt", "libgmz_prof.so"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--games", type=int, default=1024)
ap.add_argument("--moves", type=int, default=3)
ap.add_argument("--warmup", type=int, default=1)
ap.add_argument("--no-hint", action="store_true")
a = ap.parse_args()
from datou_gomoku_muzero_amd import engine as E, network as N, weights as W, _lib  # noqa: E402
from datou_gomoku_muzero_amd.config import GmzConfig  # noqa: E402

lib = _lib.load()
rd = lib.gmz_tree_prof_read
rd.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * 16)()
cfg = GmzConfig(BOARD_SIZE=15, NUM_SIMULATIONS=400)
sd = W.synthetic_state_dict(cfg, seed=1234, with_projection=False)
net = N.GomokuNetHip(sd, cfg, num_slots=a.games * 402, max_rows=a.games)
eng = E.BatchedSelfPlayEngine(cfg, num_games=a.games, net=net, seed=7, descent_hint=not a.no_hint)
eng.reset_games()
for m in range(a.warmup + a.moves):
    if m == a.warmup:
        torch.cuda.synchronize()
        rd(buf, 1)
    eng.search()
    eng.play(reset_finished=True)
torch.cuda.synchronize()
rd(buf, 0)
v = list(buf)
names = ["fetch_wait", "q_and_hint_issue", "improved_policy", "scores_argmax", "hint_calc", "root_select",
         "expand_backup", "nonroot_levels", "waves", "kernel_total", "select_total", "hint_hits"]
out = {n: v[i] for i, n in enumerate(names)}
lv = max(1, out["nonroot_levels"])
wv = max(1, out["waves"])
per_level = {n: out[n] / lv for n in names[:5]}
per_wave = {n: out[n] / wv for n in ("root_select", "expand_backup", "kernel_total", "select_total")}
print(json.dumps({"cycles_per_nonroot_level": per_level, "cycles_per_game_wave": per_wave,
                  "nonroot_levels_per_game_wave": lv / wv, "hint_hit_rate": out["hint_hits"] / lv,
                  "raw": out, "games": a.games, "moves": a.moves, "hint": not a.no_hint}, indent=1))
