"""Self-play throughput benchmark (BASELINE.json metric: self-play moves/sec, 15x15, 400 sims).

One *step* = one move of every game on this GPU: the full Gumbel-MuZero search (1 initial +
~100 waves of select -> GomokuNetEZ recurrent inference -> expand/backup, mcts.py:288-362) and the
move itself (do_move + get_game_ended, workers.py:178-181), G games at once (config 2: G = 1024).
Finished games restart immediately.  Data: synthetic — empty boards, random-init GomokuNetEZ
(8 blocks x 128 channels, numpy-seeded), Gumbel noise from the device RNG.

  python bench.py [--gpus N --steps K --warmup W]              (N > 1: launched by torch.distributed.run)

Prints ONE JSON line on rank 0 (schema: the driver contract) including
  roofline     : the dominant kernel (dynamics tower k_tower3<15,true>) timed with HIP events on its
                 launch stream inside the timed region; achieved = algorithmic FLOP per launch /
                 mean launch duration vs the 2.5 PFLOP/s dense bf16 MFMA peak;
  cpu_baseline : the C oracle's search (oracle/gmz_oracle.c) with the float32 numpy network
                 (oracle/netref.py) on the same weights, rank 0 / N=1 only, bounded sample.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402



def repr_flop_per_row(size, blocks):
    """Algorithmic FLOP of one representation-tower row (network.py:30-56 + the 1x1 head convs):
    stem conv 3->128 (2*A*128*3*9) + 2*blocks ResBlock convs + 2*A*128*3."""
    A = size * size
    return 2 * A * 128 * 3 * 9 + 2 * blocks * 2 * A * 128 * 128 * 9 + 2 * A * 128 * 3


def tower_flop_per_row(size, blocks):
    """Algorithmic FLOP of one dynamics-tower row (network.py:81-83 + the 1x1 head convs):
    conv 144->128 (2*A*128*144*9) + 2*blocks ResBlock convs (2*A*128*128*9 each) + 2*A*128*3.
    15x15, 8 blocks: 1,136,505,600."""
    A = size * size
    return 2 * A * 128 * 144 * 9 + 2 * blocks * 2 * A * 128 * 128 * 9 + 2 * A * 128 * 3
PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, no sparsity)
PEAK_HBM_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--games", type=int, default=1024, help="concurrent games per GPU (config 2: 1024)")
    ap.add_argument("--size", type=int, default=15)
    ap.add_argument("--sims", type=int, default=400)
    ap.add_argument("--blocks", type=int, default=8)
    ap.add_argument("--mode", default="MuZero")
    ap.add_argument("--net", default="hip", choices=["hip", "hash"])
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--cpu-baseline-sec", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pmc-file", default=os.path.join(REPO, "profiles", "pmc_tower_latest.json"))
    return ap.parse_args()


def collective_max(x, dist, backend="nccl"):
    """Max of a per-rank float over all ranks (the driver contract's max-over-ranks timing)."""
    if dist is None:
        return x
    dev = "cuda" if backend == "nccl" else "cpu"
    t = torch.tensor([x], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def result_line(args, world, dt, waves, G):
    """The JSON object rank 0 prints (without roofline / cpu_baseline)."""
    total_moves = G * args.steps * world
    return {
        "metric": "self-play moves/sec (15x15, 400 sims)" if (args.size, args.sims) == (15, 400)
        else "self-play moves/sec (%dx%d, %d sims)" % (args.size, args.size, args.sims),
        "value": total_moves / dt, "unit": "moves/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
        "config": {"workload": "%dx%d Gumbel %s, %d sims/move, %d concurrent games per GPU, GomokuNetEZ %d blocks x "
                               "128 ch (numpy-seeded random init), empty-board starts, device Gumbel RNG"
                               % (args.size, args.size, args.mode, args.sims, G, args.blocks),
                   "games_per_gpu": G, "global_games": G * world, "board_size": args.size,
                   "num_simulations": args.sims, "mcts": args.mode, "waves_per_move": waves / max(1, args.steps),
                   "parallelism": "dp%d (independent games per GPU, no collective)" % world},
    }


def cpu_baseline(args, sd, cfg):
    """C oracle search + float32 numpy GomokuNetEZ on the host cores (reported baseline)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    import netref
    try:
        from threadpoolctl import threadpool_info
        cores = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:
        cores = os.cpu_count() or 1
    H = args.size
    A = H * H

    def init(obs):
        p, v, h = netref.initial_inference(sd, obs)
        return p, v[:, 0], list(h)

    def rec(hs, acts):
        p, v, h, r = netref.recurrent_inference(sd, np.stack(hs), acts)
        return p, v[:, 0], r[:, 0], list(h)

    net = oracle.CallbackNet(A, H, init, rec)
    ocfg = oracle.make_cfg(H, args.sims, args.mode, hashnet=False)
    rs = np.random.RandomState(args.seed)
    board = np.zeros(A, np.int8)
    player, last, moves, rows = 1, None, 0, 0
    t0 = time.perf_counter()
    while True:
        net.reset()
        pol, val, act, _, st = oracle.search(ocfg, board, player, last, int(np.count_nonzero(board)),
                                             rs.gumbel(0, 1, A), net=net)
        rows += st["n_initial"] + st["recurrent_rows"]
        moves += 1
        board[act] = player
        last, player = act, -player
        if oracle.game_ended(board, H, act, int(np.count_nonzero(board))) is not None:
            board[:] = 0
            player, last = 1, None
        dt = time.perf_counter() - t0
        if dt >= args.cpu_baseline_sec or moves >= 64:
            break
    return {"value": moves / dt, "unit": "moves/s", "cores": int(cores), "kind": "port",
            "sample": "%d move(s) of one 15x15 game from the empty board, %d sims, %d NN rows (the reference's "
                      "duplicate-leaf batches kept), %.1f s; C oracle search + numpy fp32 GomokuNetEZ"
                      % (moves, args.sims, rows, dt)}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        # GMZ_DIST_BACKEND=gloo rehearses the N>1 path with several ranks sharing one GPU
        backend = os.environ.get("GMZ_DIST_BACKEND", "nccl")
        torch.cuda.set_device(local % torch.cuda.device_count())
        dist.init_process_group(backend, init_method="env://")
    else:
        torch.cuda.set_device(0)
    import datou_gomoku_muzero_amd.engine as E
    from datou_gomoku_muzero_amd import network as N, weights as W
    from datou_gomoku_muzero_amd.config import GmzConfig

    cfg = GmzConfig(BOARD_SIZE=args.size, NUM_SIMULATIONS=args.sims, MCTS_IMPLEMENTATION=args.mode,
                    NUM_RES_BLOCKS=args.blocks)
    G = args.games
    sd = W.synthetic_state_dict(cfg, seed=args.seed, with_projection=False)
    if dist is not None:  # the self-play tier's one exchange: rank 0's weights -> all ranks (RCCL)
        from datou_gomoku_muzero_amd.weight_sync import broadcast_state_dict
        dev = "cuda" if os.environ.get("GMZ_DIST_BACKEND", "nccl") == "nccl" else "cpu"
        sd = {k: v.cpu().numpy() for k, v in broadcast_state_dict(sd, src=0, device=dev).items()}
    slots = G * (cfg.NUM_SIMULATIONS + 2)
    if args.net == "hip":
        net = N.GomokuNetHip(sd, cfg, num_slots=slots, max_rows=G)
    else:
        net = E.HashNetBackend(slots, cfg.ACTION_SPACE_SIZE)
    eng = E.BatchedSelfPlayEngine(cfg, num_games=G, net=net, seed=args.seed + 7919 * rank)
    eng.reset_games()
    log("rank %d: engine G=%d %dx%d %s/%d, net=%s" % (rank, G, args.size, args.size, args.mode, args.sims, args.net))

    def step():
        eng.search()
        eng.play(reset_finished=True)

    for i in range(args.warmup):
        step()
        torch.cuda.synchronize()
        log("warmup %d/%d done" % (i + 1, args.warmup))
    timer = None
    az = args.mode == "AlphaZero"  # AlphaZero searches run the representation tower per wave
    if args.net == "hip":
        timer = N.KernelTimer()
        if az:
            net.repr_timer = timer
        else:
            net.tower_timer = timer
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    waves = 0
    for i in range(args.steps):
        step()
        waves += eng.waves_last
        if (i + 1) % max(1, args.steps // 5) == 0:
            log("step %d/%d" % (i + 1, args.steps))
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    dt = collective_max(dt, dist, os.environ.get("GMZ_DIST_BACKEND", "nccl"))
    out = result_line(args, world, dt, waves, G)
    if timer is not None:
        n_launch, ms, rows = timer.summary()
        fpr = (repr_flop_per_row if az else tower_flop_per_row)(args.size, args.blocks)
        flop = fpr * rows
        achieved = flop / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
        traffic = None
        if os.path.exists(args.pmc_file) and (args.size, args.blocks) == (15, 8) and not az:  # the PMC pass's config
            try:
                traffic = json.load(open(args.pmc_file)).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        kname = ("k_tower3<%d,REPR> (representation tower, stem + %d fused convs + head 1x1 convs)" % (args.size, 2 * args.blocks)
                 if az else "k_tower3<%d,DYN> (dynamics tower, %d fused convs + head 1x1 convs)" % (args.size, 1 + 2 * args.blocks))
        out["roofline"] = {"bound": "mfma", "kernel": kname,
                           "achieved": achieved, "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                           "frac": achieved / PEAK_BF16_TFLOPS, "traffic": traffic,
                           "launches": n_launch, "mean_launch_ms": ms, "rows_per_launch": rows,
                           "flop_per_row": fpr}
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.net == "hip":
        log("cpu baseline (bounded sample ~%.0f s)..." % args.cpu_baseline_sec)
        out["cpu_baseline"] = cpu_baseline(args, sd, cfg)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
