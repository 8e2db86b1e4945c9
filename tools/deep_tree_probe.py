"""Deep trees: engine (dense hint / dense no-hint / lists) vs the C oracle at growing simulation counts on
empty boards (HashNet), with the oracle's deepest leaf per search.  Diagnostic for paths deeper than a wave.
  python tools/deep_tree_probe.py [--size 9] [--sims 800,2000,4000,8000,16000] [--games 2]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import oracle  # noqa: E402  (checker)
import datou_gomoku_muzero_amd.engine as E  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=9)
ap.add_argument("--sims", default="800,2000,4000,8000,16000")
ap.add_argument("--games", type=int, default=2)
ap.add_argument("--mode", default="MuZero")
a = ap.parse_args()
A, G = a.size * a.size, a.games
for sims in [int(x) for x in a.sims.split(",")]:
    rs = np.random.RandomState(sims)
    gum = rs.gumbel(0, 1, (G, A))
    boards = np.zeros((G, A), np.int8)
    res = {}
    for name, kw in (("dense_hint", dict(descent_hint=True, layout="dense")),
                     ("dense_nohint", dict(descent_hint=False, layout="dense")),
                     ("lists", dict(descent_hint=False, layout="lists"))):
        eng = E.BatchedSelfPlayEngine(None, num_games=G, BOARD_SIZE=a.size, NUM_SIMULATIONS=sims,
                                      MCTS_IMPLEMENTATION=a.mode, **kw)
        eng.set_positions(boards, np.ones(G, np.int8), np.full(G, -1, np.int32))
        pol, val, act = eng.search(gumbel=gum)
        _, rn, rw, _, _ = eng.root_stats()
        torch.cuda.synchronize()
        res[name] = (act.cpu().numpy().copy(), val.cpu().numpy().copy(), rn.cpu().numpy().copy(), eng.max_visited_children())
        eng.close()
    cfg = oracle.make_cfg(a.size, sims, a.mode)
    for g in range(G):
        opol, oval, oact, orv, st = oracle.search(cfg, boards[g], 1, None, 0, gum[g])
        line = "sims %6d game %d oracle act %3d val %.6f root_n %6d max_depth %3d |" % (sims, g, oact, oval, st["root_n"], st["max_depth"])
        for name, (ac, va, rn, nv) in res.items():
            ok = ac[g] == oact and va[g] == oval and rn[g] == st["root_n"]
            line += " %s %s (act %d val %.6f n %d nvis %d)" % (name, "ok" if ok else "DIFF", ac[g], va[g], rn[g], nv)
        print(line, flush=True)
