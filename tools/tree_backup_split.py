"""The north-star backup kernel inside the fused tree launch: k_expand_select runs the backup of
wave i (expand_backup_game: the leaf's expansion + the k-fold duplicate-leaf backup, mcts.py:119-138) and the
selection of wave i+1 in one launch.  With a -DGMZ_TREE_PROF library (s_memtime stamps; GMZ_LIB, default
datou-gomoku-muzero_amd/_alt/libgmz_prof.so) this measures, per game-wave, the cycles of the backup phase and of the
whole launch, at the engine's default layout for G games on one stream, and the counted algorithmic bytes of each
phase (bench.tree_bytes' model split: expand + backup vs select).  Writes a JSON the bench reads for
roofline_tree.backup_frac: backup bytes / (backup share x the live launch time) / 8 TB/s.
  python tools/tree_backup_split.py OUT.json [--games 1024 8192] [--moves 3]"""
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
ap.add_argument("out")
ap.add_argument("--games", type=int, nargs="+", default=[1024, 8192])
ap.add_argument("--moves", type=int, default=3)
ap.add_argument("--warmup", type=int, default=1)
a = ap.parse_args()
from datou_gomoku_muzero_amd import engine as E, network as N, weights as W, _lib  # noqa: E402
from datou_gomoku_muzero_amd.config import GmzConfig  # noqa: E402

lib = _lib.load()
rd = lib.gmz_tree_prof_read
rd.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * 16)()
cfg = GmzConfig(BOARD_SIZE=15, NUM_SIMULATIONS=400)
sd = W.synthetic_state_dict(cfg, seed=1234, with_projection=False)
A = 225
res = {"note": __doc__.split("\n\n")[0], "library": os.path.basename(os.environ["GMZ_LIB"]), "moves": a.moves}
for G in a.games:
    net = N.GomokuNetHip(sd, cfg, num_slots=G * 402, max_rows=G)
    eng = E.BatchedSelfPlayEngine(cfg, num_games=G, net=net, seed=7)
    eng.reset_games()
    for m in range(a.warmup + a.moves):
        if m == a.warmup:
            torch.cuda.synchronize()
            rd(buf, 1)
            eng.tree_counters(reset=True)
        eng.search()
        eng.play(reset_finished=True)
    torch.cuda.synchronize()
    rd(buf, 0)
    v = list(buf)
    ctr = eng.tree_counters()
    backup_cycles, waves, total_cycles = v[6], v[8], v[9]
    b_bytes = ctr["backups"] * (24 * A + 16) + 24 * ctr["backup_levels"]
    s_bytes = 20 * A * (ctr["select_levels"] - ctr["selects"]) + 8 * ctr["select_levels"]
    launches = a.moves * eng.waves_last if eng.waves_last else None
    res["G%d" % G] = {"layout": eng.layout if hasattr(eng, "layout") else None, "game_waves": waves,
                      "backup_cycles_per_game_wave": backup_cycles / max(1, waves),
                      "launch_cycles_per_game_wave": total_cycles / max(1, waves),
                      "backup_share": backup_cycles / max(1, total_cycles),
                      "backup_bytes": b_bytes, "select_bytes": s_bytes,
                      "backup_bytes_share": b_bytes / max(1, b_bytes + s_bytes), "counters": ctr}
    print(G, json.dumps(res["G%d" % G]))
    eng.close()
    del eng, net
    torch.cuda.empty_cache()
json.dump(res, open(a.out, "w"), indent=1)
