"""CPU baseline worker for bench.py's ``cpu_baseline`` leg — TEST / MEASUREMENT INFRASTRUCTURE.

ORACLE ONLY: run by bench.py as a child process (one per host core it uses), never by the product.
It plays self-play moves of ONE 15x15 game (or the configured board) with the C oracle's search
(oracle/gmz_oracle.c: the reference's MuZeroMCTS / AlphaZeroMCTS, mcts.py:197-362) and the float32
numpy GomokuNetEZ (oracle/netref.py, network.py:137-152), keeping the reference's duplicate-leaf
batches (k identical rows per wave, as its inference server evaluates them), single-threaded BLAS.
The game starts from a random opening of ``--opening`` stones (so the sample covers mid-game
positions), continues move after move (a finished game restarts from a new opening) and stops at the
first move that ends past ``--seconds``.  Prints one JSON line: moves, NN rows, elapsed seconds.

  python oracle/cpu_baseline.py --size 15 --sims 400 --mode MuZero --blocks 8 --seed 1234 \
      --opening 40 --seconds 20
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=15)
    ap.add_argument("--sims", type=int, default=400)
    ap.add_argument("--mode", default="MuZero")
    ap.add_argument("--blocks", type=int, default=8)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--weights-seed", type=int, default=1234)
    ap.add_argument("--opening", type=int, default=0)
    ap.add_argument("--seconds", type=float, default=20.0)
    a = ap.parse_args()
    try:  # one BLAS thread per worker process: the parallelism is the processes
        from threadpoolctl import threadpool_limits
        threadpool_limits(1)
    except Exception:
        pass
    import oracle
    import netref
    from datou_gomoku_muzero_amd import weights as W
    from datou_gomoku_muzero_amd.config import GmzConfig
    cfg = GmzConfig(BOARD_SIZE=a.size, NUM_SIMULATIONS=a.sims, MCTS_IMPLEMENTATION=a.mode, NUM_RES_BLOCKS=a.blocks)
    sd = W.synthetic_state_dict(cfg, seed=a.weights_seed, with_projection=False)
    H, A = a.size, a.size * a.size

    def init(obs):
        p, v, h = netref.initial_inference(sd, obs)
        return p, v[:, 0], list(h)

    def rec(hs, acts):
        p, v, h, r = netref.recurrent_inference(sd, np.stack(hs), acts)
        return p, v[:, 0], r[:, 0], list(h)

    net = oracle.CallbackNet(A, H, init, rec)
    ocfg = oracle.make_cfg(H, a.sims, a.mode, hashnet=False)
    rs = np.random.RandomState(a.seed)

    def opening():
        b = np.zeros(A, np.int8)
        n = min(a.opening, A - 1)
        cells = rs.permutation(A)[:n]
        b[cells[0::2]] = 1
        b[cells[1::2]] = -1
        return b, (1 if n % 2 == 0 else -1), (int(cells[-1]) if n else None)

    board, player, last = opening()
    moves = rows = 0
    stones = []
    t0 = time.perf_counter()
    while True:
        net.reset()
        mc = int(np.count_nonzero(board))
        stones.append(mc)
        pol, val, act, _, st = oracle.search(ocfg, board, player, last, mc, rs.gumbel(0, 1, A), net=net)
        rows += st["n_initial"] + st["recurrent_rows"]
        moves += 1
        board[act] = player
        last, player = act, -player
        dt = time.perf_counter() - t0
        if dt >= a.seconds:
            break
        if oracle.game_ended(board, H, act, int(np.count_nonzero(board))) is not None:
            board, player, last = opening()
    print(json.dumps({"moves": moves, "rows": rows, "seconds": dt, "stones": stones}), flush=True)


if __name__ == "__main__":
    main()
