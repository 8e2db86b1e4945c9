"""A/B of the descent prefetch hint (gmz_tree.hip node_last; gmz_engine_cfg.flags bit 0) in the real
self-play step: two engines (hint on / off) on the same network, same seeds and so the same trees
(the hint never changes a result: checked here move by move), moves alternated in one process so both
see the same box and clock; k_expand_select timed with HIP events on its stream.
  python tools/tree_hint_ab.py [--games 1024 --moves 8]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--games", type=int, default=1024)
ap.add_argument("--moves", type=int, default=8)
ap.add_argument("--warmup", type=int, default=2)
a = ap.parse_args()
from datou_gomoku_muzero_amd import engine as E, network as N, weights as W  # noqa: E402
from datou_gomoku_muzero_amd.config import GmzConfig  # noqa: E402

cfg = GmzConfig(BOARD_SIZE=15, NUM_SIMULATIONS=400)
sd = W.synthetic_state_dict(cfg, seed=1234, with_projection=False)
net = N.GomokuNetHip(sd, cfg, num_slots=a.games * 402, max_rows=a.games)
engs = {h: E.BatchedSelfPlayEngine(cfg, num_games=a.games, net=net, seed=7, descent_hint=h) for h in (True, False)}
for e in engs.values():
    e.reset_games()
res = {True: [], False: []}
for m in range(a.warmup + a.moves):
    acts = {}
    for h, e in engs.items():
        e.tree_timer = N.KernelTimer() if m >= a.warmup else None
        pol, val, act = e.search()
        e.play(reset_finished=True)
        torch.cuda.synchronize()
        acts[h] = (act.cpu().clone(), val.cpu().clone(), pol.cpu().clone())
        if e.tree_timer is not None:
            n, ms, _ = e.tree_timer.summary()
            res[h].append(ms)
    assert all(torch.equal(x, y) for x, y in zip(acts[True], acts[False])), "hint changed a result at move %d" % m
mean = {h: sum(v) / len(v) for h, v in res.items()}
print(json.dumps({"k_expand_select_mean_us": {"hint": mean[True] * 1e3, "no_hint": mean[False] * 1e3},
                  "speedup": mean[False] / mean[True], "per_move_us": {"hint": [x * 1e3 for x in res[True]],
                                                                        "no_hint": [x * 1e3 for x in res[False]]},
                  "games": a.games, "moves": a.moves, "results_identical": True}))
