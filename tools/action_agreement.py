"""How often does the 16-bit HIP network change a search's decision?  

The same batched Gumbel-MuZero search (engine.BatchedSelfPlayEngine, the HIP tree kernels) runs on
the same positions with the same Gumbel noise three times: with the HIP network in f16 (product
default), in bf16, and with a float32 PyTorch restatement of the reference network
(tests/torch_refnet.py, the checker; pinned to oracle/netref.py).  The tree given identical network
outputs is bit-exact with the reference (tests/test_engine_gpu.py), so every difference below comes
from network precision.  Reports per 16-bit type: top-1 action agreement with the float32 search,
mean |Δ root value|, mean total-variation distance of the improved policy.

  python tools/action_agreement.py [--games 256 --size 15 --sims 400 --blocks 8 --out FILE]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def positions(G, size, rs, max_stones=60):
    """Random legal-looking midgame positions: k alternating stones (k < max_stones), no finished games."""
    A = size * size
    boards = np.zeros((G, A), np.int8)
    players = np.ones(G, np.int8)
    last = np.full(G, -1, np.int32)
    for g in range(G):
        k = rs.randint(0, max_stones)
        cells = rs.permutation(A)[:k]
        p = 1
        for c in cells:
            boards[g, c] = p
            p = -p
        players[g], last[g] = p, (cells[-1] if k else -1)
    return boards, players, last


def run(cfg, G, net, boards, players, last, gumbel):
    from datou_gomoku_muzero_amd import engine as E
    eng = E.BatchedSelfPlayEngine(cfg, num_games=G, net=net)
    eng.set_positions(boards, players, last)
    pol, val, act = eng.search(gumbel=gumbel)
    torch.cuda.synchronize()
    out = pol.cpu().numpy(), val.cpu().numpy(), act.cpu().numpy()
    eng.close()
    return out


def agreement(G=256, size=15, sims=400, blocks=8, seed=0):
    from datou_gomoku_muzero_amd import network as N, weights as W
    from datou_gomoku_muzero_amd.config import GmzConfig
    from torch_refnet import TorchRefNet
    cfg = GmzConfig(BOARD_SIZE=size, NUM_SIMULATIONS=sims, NUM_RES_BLOCKS=blocks)
    sd = W.synthetic_state_dict(cfg, seed=seed + 1, with_projection=False)
    rs = np.random.RandomState(seed)
    boards, players, last = positions(G, size, rs)
    gumbel = rs.gumbel(0, 1, (G, size * size))
    slots = G * (sims + 2)
    t0 = time.time()
    ref = run(cfg, G, TorchRefNet(sd, size, blocks, slots), boards, players, last, gumbel)
    torch.cuda.empty_cache()
    t_ref = time.time() - t0
    res = {"games": G, "board": size, "sims": sims, "blocks": blocks, "seed": seed, "fp32_search_s": t_ref}
    for prec in ("fp16", "bf16"):
        net = N.GomokuNetHip(sd, cfg, num_slots=slots, max_rows=G, precision=prec)
        pol, val, act = run(cfg, G, net, boards, players, last, gumbel)
        del net
        torch.cuda.empty_cache()
        res[prec] = {"top1_agreement": float((act == ref[2]).mean()),
                     "mean_abs_dvalue": float(np.abs(val - ref[1]).mean()),
                     "max_abs_dvalue": float(np.abs(val - ref[1]).max()),
                     "mean_policy_tv": float(0.5 * np.abs(pol - ref[0]).sum(1).mean())}
    return res


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=256)
    ap.add_argument("--size", type=int, default=15)
    ap.add_argument("--sims", type=int, default=400)
    ap.add_argument("--blocks", type=int, default=8)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    r = agreement(a.games, a.size, a.sims, a.blocks, a.seed)
    print(json.dumps(r))
    if a.out:
        json.dump(r, open(a.out, "w"), indent=1)
