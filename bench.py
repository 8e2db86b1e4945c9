"""Self-play throughput benchmark (BASELINE.json metric: self-play moves/sec, 15x15, 400 sims;
trainer steps/sec).

One *step* = one move of every game on this GPU: the full Gumbel-MuZero search (1 initial +
~100 waves of select -> GomokuNetEZ recurrent inference -> expand/backup, mcts.py:288-362) and the
move itself (do_move + get_game_ended, workers.py:178-181), G games at once (config 2: G = 1024).
Finished games restart immediately.  Data: synthetic — empty boards, random-init GomokuNetEZ
(8 blocks x 128 channels, numpy-seeded), Gumbel noise from the device RNG.  The G games run as two
half-size engines on two HIP streams (15x15 MuZero default; engine.SplitSelfPlayEngine: the same games
as one engine, bit for bit; one half's tree/head kernels overlap the other half's tower).

  python bench.py [--gpus N --steps K --warmup W]

N > 1: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set) the ranks are the
launcher's; with WORLD_SIZE unset, ``--gpus N`` starts the N rank processes itself (before anything
touches the GPU) with RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR=127.0.0.1 set.  Games shard by rank
with no data-path collective (main.py:100-101: independent workers), rank 0's weights are broadcast
once (RCCL), timing is the max over ranks.  GMZ_DIST_BACKEND=gloo rehearses the N > 1 path with
several ranks sharing one GPU.

Prints ONE JSON line on rank 0 (schema: the driver contract) including
  roofline      : the dominant kernel (dynamics tower k_tower3<15,DYN>) timed with HIP events on its
                  launch stream(s) inside the timed region; achieved = algorithmic FLOP of the rows the
                  searches actually requested / the kernel's busy time (union of its launch intervals
                  over both streams; = launches x mean duration with one stream) vs the 2.5 PFLOP/s
                  dense f16/bf16 MFMA peak; per-launch figures beside it;
  roofline_tree : the fused expand/backup + select kernel (k_expand_select), same timing; achieved =
                  algorithmic bytes counted from the per-game work counters (gmz_engine_tree_counters,
                  byte model in DESIGN.md §5) / its busy time vs 8 TB/s HBM;
  trainer       : config C4's trainer (B = 360 per GPU, 5 unroll steps, PER, fp16 autocast, HIP convs),
                  steps/s after the self-play region, on every rank (DDP: one RCCL gradient all-reduce +
                  the sharded-PER syncs per step), plus the MFMA fraction of its dominant HIP conv;
  loop_c4       : config C4 composed on every rank (datou-gomoku-muzero_amd/loop.py): self-play moves of
                  G games -> finished games' slices into the rank's PER shard -> DDP trainer steps ->
                  periodic weight push (RCCL broadcast) into the self-play network; moves/s and trainer
                  steps/s of the whole job over the timed iterations (time-sliced: moves, then steps);
  loop_c4_concurrent : the same loop with each iteration's trainer steps on their own HIP stream,
                  running beside that iteration's self-play moves;
  sublines      : BASELINE configs 5 and 1 on the GPU, a few steps each after the headline engine is freed:
                  C5 = 19x19, 800 sims, 16 blocks (G games); C1 = 9x9 AlphaZero, 50 sims (G games), each with
                  moves/s and the tower's and tree kernel's roofline fractions (one stream: every launch alone);
                  g8192 = config 2's search on 8,192 trees as one engine (the tree kernel alone at SURVEY §8(d)'s
                  measurement point; skipped, and said so, on a GPU without ~100 GiB free);
  worker        : the drop-in worker (worker.gpu_selfplay_worker) over torch.multiprocessing queues with a
                  consumer process unpickling every payload (the reference's process graph): moves/s over
                  the steady-state moves including every per-move and per-game record, and its ratio to
                  the headline engine rate;
  cpu_baseline  : the C oracle's search (oracle/gmz_oracle.c) with the float32 numpy network
                  (oracle/netref.py) on the same weights, one single-threaded process per host core used
                  (oracle/cpu_baseline.py), mid-game openings, rank 0 / N=1 only, bounded sample.
"""
import argparse
import json
import os
import socket
import subprocess
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


def tree_bytes(ctr, A):
    """Algorithmic HBM bytes of the fused expand/backup + select launches (SURVEY §8d model):
      expand, per game-wave : read the leaf's logits (4A) + store them (4A) + its empty child row (16A)
      backup, per game-wave : 24 B per level (parent index, R, N r+w, W r+w) + 16 B (min/max, value, k)
      select, per level     : 20A B per non-root level (child N, W, R, child index, logits) + 8 B (path)
    ``ctr``: engine.tree_counters().  (The root level's <= 16 selected edges are not counted.)"""
    return (ctr["backups"] * (24 * A + 16) + 24 * ctr["backup_levels"]
            + 20 * A * (ctr["select_levels"] - ctr["selects"]) + 8 * ctr["select_levels"])


def backup_bytes(ctr, A):
    """The backup phase's share of tree_bytes: the leaf's expansion (24A + 16 per game-wave) and 24 B per level backed
    up (mcts.py:119-138, the north-star 'backup kernel')."""
    return ctr["backups"] * (24 * A + 16) + 24 * ctr["backup_levels"]


BACKUP_SPLIT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r06_tree_backup_split.json")


def backup_roofline(ctr, A, n_launch, busy_ms, G):
    """roofline_tree.backup: the north-star backup kernel inside the fused launch.  k_expand_select runs the backup
    of wave i and the selection of wave i+1 in one launch, so the backup's time is its measured share of the launch's
    cycles (s_memtime phase stamps per game-wave, tools/tree_backup_split.py with a -DGMZ_TREE_PROF build, committed
    as profiles/r06_tree_backup_split.json; builder-measured) times this run's busy time."""
    try:
        sp = json.load(open(BACKUP_SPLIT)).get("G%d" % G)
    except Exception:
        sp = None
    if not sp or n_launch <= 0 or busy_ms <= 0 or A != 225:
        return None
    b = backup_bytes(ctr, A)
    t = sp["backup_share"] * busy_ms * 1e-3
    gbs = b / t / 1e9
    return {"bound": "hbm", "achieved": gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": gbs / PEAK_HBM_GBS,
            "bytes_per_launch": b / n_launch, "share_of_launch": sp["backup_share"],
            "share_source": "builder-measured phase cycles, %s (G=%d, layout %s)" % (
                os.path.relpath(BACKUP_SPLIT, os.path.dirname(os.path.abspath(__file__))), G, sp.get("layout"))}


PEAK_MFMA_TFLOPS = 2500.0   # MI355X dense f16 / bf16 MFMA (MI355X_MICROARCH.md, no sparsity)
PEAK_HBM_GBS = 8000.0


def pmc_traffic(path, args, G, az, streams, size=None, blocks=None):
    """HBM bytes per launch from a committed PMC summary (tools/gpu.sh pmc -> tools/pmc_summary.py) when it
    was measured on this configuration (15x15, 8 blocks, MuZero, the same games per GPU — 1,024 unless the
    summary says otherwise —, precision and number of streams as this run resolved to)."""
    size = args.size if size is None else size
    blocks = args.blocks if blocks is None else blocks
    if not os.path.exists(path) or (size, blocks) != (15, 8) or az:
        return None
    try:
        pm = json.load(open(path))
    except Exception:
        return None
    if pm.get("precision", "bf16") != args.precision or int(pm.get("streams", 1)) != int(streams or 1):
        return None
    if int(pm.get("games", 1024)) != int(G):
        return None
    return pm.get("hbm_bytes_per_launch")


PMC_TREE_G8192 = os.path.join(REPO, "profiles", "pmc_tree_g8192.json")  # the g8192 sub-line's PMC pass


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse(argv=None):
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
    ap.add_argument("--streams", type=int, default=None,
                    help="HIP streams per GPU: the G games as this many engines whose waves interleave "
                         "(engine.SplitSelfPlayEngine; 1 = one BatchedSelfPlayEngine; default: "
                         "engine.default_streams, i.e. 2 for 15x15 MuZero, else 1)")
    ap.add_argument("--single-stream-moves", type=int, default=2,
                    help="with --streams > 1: moves of ONE engine on one stream after the timed region, for the two "
                         "kernels' single-stream launch times (0: skip)")
    ap.add_argument("--layout", default=None, choices=["dense", "lists"],
                    help="tree layout of the non-root nodes (engine.default_layout when omitted): dense child rows "
                         "or compact lists of the visited children (identical results)")
    ap.add_argument("--hint", default=None, choices=["on", "off"],
                    help="descent prefetch hint / cached exp rows of the tree kernels (default: by game count)")
    ap.add_argument("--kernel-timers", default="on", choices=["on", "off"],
                    help="HIP events around every tower / tree launch in the timed moves (off: A/B of their cost; the "
                         "line then has no roofline)")
    ap.add_argument("--pair", default=None, choices=["on", "off"],
                    help="two waves per game in the fused tree kernel (engine.default_pair when omitted)")
    ap.add_argument("--precision", default="fp16", choices=["fp16", "bf16"],
                    help="MFMA operand type of the network towers (f32 accumulation either way)")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--cpu-baseline-sec", type=float, default=20.0)
    ap.add_argument("--cpu-baseline-procs", type=int, default=16,
                    help="single-threaded oracle processes (capped by the cores this process may use); 16 = the "
                         "reference's process graph size: NUM_WORKERS = 15 self-play workers (config.py:13) + its "
                         "inference server, each a CPU process")
    ap.add_argument("--sublines", default="empty_board,c5,c1,g8192",
                    help="measured besides the headline: c5 (BASELINE config 5: 19x19/800/16 blocks), c1 (config 1: 9x9 "
                         "AlphaZero/50), g8192 (config 2's search on 8,192 trees, one engine: the tree kernel's "
                         "SURVEY 8(d) measurement point)")
    ap.add_argument("--subline-games", type=int, default=1024)
    ap.add_argument("--c5-steps", type=int, default=3)
    ap.add_argument("--c1-steps", type=int, default=10)
    ap.add_argument("--worker-moves", type=int, default=40,
                    help="timed moves of the drop-in worker leg (0: skip); 40 so the one-move drain at the end of the "
                         "timed region (the last move's records) weighs ~2.5 %, not 5 %")
    ap.add_argument("--worker-warmup", type=int, default=4, help="untimed worker moves first")
    ap.add_argument("--worker-openings", type=int, default=80,
                    help="staggered starts: each slot's first game from a random opening of 0..N stones "
                         "(engine.random_openings), so games finish in the short timed window (0: empty boards)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--trainer-steps", type=int, default=20, help="timed trainer steps (0: no trainer leg)")
    ap.add_argument("--trainer-warmup", type=int, default=6)
    ap.add_argument("--trainer-f32-steps", type=int, default=10,
                    help="timed steps of the same trainer with the reference's float32 target network (value_target_f32; "
                         "0: skip)")
    ap.add_argument("--trainer-batch", type=int, default=360)
    ap.add_argument("--trainer-buffer", type=int, default=4096, help="synthetic slices per rank's PER shard")
    ap.add_argument("--loop-iters", type=int, default=20, help="timed iterations of the C4 loop (0: no loop leg)")
    ap.add_argument("--loop-warmup", type=int, default=6)
    ap.add_argument("--loop-openings", type=int, default=80,
                    help="staggered starts of the C4 loop's games (random openings of 0..N stones; 0: empty boards)")
    ap.add_argument("--loop-modes", default="sliced",
                    help="C4 loop legs: 'sliced' (moves then steps), 'concurrent' (steps on their own HIP stream "
                         "beside the moves); comma-separated")
    ap.add_argument("--loop-games", type=int, default=1024, help="self-play games per GPU inside the C4 loop")
    ap.add_argument("--loop-moves-per-iter", type=int, default=1)
    ap.add_argument("--loop-train-per-iter", type=int, default=1)
    ap.add_argument("--loop-update-interval", type=int, default=1000,
                    help="trainer steps between weight pushes (reference MODEL_UPDATE_INTERVAL = 1000); the cost of "
                         "one push is measured separately (weight_push_ms)")
    ap.add_argument("--loop-buffer", type=int, default=65536, help="replay shard capacity per rank")
    ap.add_argument("--loop-prefill", type=int, default=4096, help="synthetic slices in each shard before the loop")
    ap.add_argument("--stagger", type=int, default=80,
                    help="headline starts (SURVEY 8(d)): k in {0,4,8} opening stones plus uniform(0, N) staggered "
                         "stones per game from RandomState(seed + game id), so games finish and restart inside the "
                         "timed moves; -1: empty boards (rounds 1-3's headline)")
    ap.add_argument("--isolate", default="auto", choices=["auto", "on", "off"],
                    help="run each phase (headline, extras, trainer, loop) as fresh rank processes under a wall-time "
                         "cap (auto: when N > 1)")
    ap.add_argument("--dist-timeout", type=float, default=150.0,
                    help="seconds: bound on every collective of a rank process (init_process_group timeout)")
    ap.add_argument("--phase-timeout-selfplay", type=float, default=240.0)
    ap.add_argument("--phase-timeout-extras", type=float, default=200.0)
    ap.add_argument("--phase-timeout-trainer", type=float, default=150.0)
    ap.add_argument("--phase-timeout-loop", type=float, default=180.0)
    ap.add_argument("--deadline", type=float, default=540.0,
                    help="isolated phases (N > 1): wall-time budget of the whole run in s; each phase's cap shrinks to "
                         "what is left of it (a later phase with < 15 s left is skipped), so the sum of the caps never "
                         "exceeds it (0: the per-phase caps only)")
    ap.add_argument("--pmc-file", default=os.path.join(REPO, "profiles", "pmc_tower_latest.json"))
    ap.add_argument("--pmc-tree-file", default=os.path.join(REPO, "profiles", "pmc_tree_latest.json"))
    return ap.parse_args(argv)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n, argv, script=None):
    """Start ``n`` rank processes of ``script`` (default: this file) with the torch.distributed env
    contract (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT) and
    wait for them.  Called before anything initialises the GPU.  If one rank fails, the others are
    terminated (their exact PIDs).  Returns the first non-zero exit code, else 0."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", script or os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    for p in procs:
        p.wait()
    return rc


def collective_max(x, dist, backend="nccl"):
    """Max of a per-rank float over all ranks (the driver contract's max-over-ranks timing)."""
    if dist is None:
        return x
    dev = "cuda" if backend == "nccl" else "cpu"
    t = torch.tensor([x], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def collective_sum(x, dist, backend="nccl"):
    if dist is None:
        return x
    dev = "cuda" if backend == "nccl" else "cpu"
    t = torch.tensor([x], device=dev, dtype=torch.float64)
    dist.all_reduce(t)
    return float(t.item())


def collective_gather(x, dist, backend="nccl"):
    """Every rank's float, in rank order (a one-hot all-reduce SUM)."""
    if dist is None:
        return [x]
    dev = "cuda" if backend == "nccl" else "cpu"
    t = torch.zeros(dist.get_world_size(), device=dev, dtype=torch.float64)
    t[dist.get_rank()] = x
    dist.all_reduce(t)
    return [float(v) for v in t.tolist()]


def result_line(args, world, dt, waves, G, backend=None):
    """The JSON object rank 0 prints (without roofline / cpu_baseline / trainer)."""
    total_moves = G * args.steps * world
    return {
        "metric": "self-play moves/sec (15x15, 400 sims)" if (args.size, args.sims) == (15, 400)
        else "self-play moves/sec (%dx%d, %d sims)" % (args.size, args.size, args.sims),
        "value": total_moves / dt, "unit": "moves/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": getattr(args, "precision", "fp16"), "data": "synthetic",
        "config": {"workload": "%dx%d Gumbel %s, %d sims/move, %d concurrent games per GPU, GomokuNetEZ %d blocks x "
                               "128 ch (numpy-seeded random init), %s, device Gumbel RNG"
                               % (args.size, args.size, args.mode, args.sims, G, args.blocks, starts_text(args)),
                   "games_per_gpu": G, "global_games": G * world, "board_size": args.size,
                   "num_simulations": args.sims, "mcts": args.mode, "waves_per_move": waves / max(1, args.steps),
                   "ranks": world, "dist_backend": backend, "streams_per_gpu": getattr(args, "streams", None) or 1,
                   "parallelism": "dp%d (independent games per GPU, no collective)" % world},
    }


def starts_text(args):
    if getattr(args, "stagger", -1) < 0:
        return "empty-board starts"
    return ("steady-state starts: game g from RandomState(seed + g) with k in {0,4,8} opening stones plus "
            "uniform(0, %d) staggered stones (engine.seeded_openings; finished games restart from the empty "
            "board inside the timed moves)" % args.stagger)


def headline_openings(args, rank, G, size, n_in_row=5):
    """The headline's start positions: global game ids rank*G .. rank*G + G - 1."""
    if getattr(args, "stagger", 0) < 0:
        return None
    import datou_gomoku_muzero_amd.engine as E
    return E.seeded_openings(range(rank * G, (rank + 1) * G), size, args.seed, stagger=args.stagger,
                             n_in_row=n_in_row)


_PEAKS = {}


def achievable_peaks():
    """SURVEY §8(d) 'Peak references', measured live on this GPU after the timed region (once per process):
    the dense f16 GEMM rate hipBLASLt delivers (torch.matmul, 16384^3, f32 accumulation — the tower's operand
    type) and device-to-device copy bandwidth (2 GiB, read + write bytes), so that each roofline ``frac``
    (against the vendor peaks, 2.5 PF and 8 TB/s) can also be read against what this chip delivers."""
    if _PEAKS:
        return _PEAKS

    def timed(fn, reps):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e-3 / reps

    m = 16384
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(m, m, dtype=torch.float16, device="cuda", generator=g)  # random data: the clock it holds
    y = torch.randn(m, m, dtype=torch.float16, device="cuda", generator=g)
    t = timed(lambda: torch.matmul(x, y), 4)
    _PEAKS["gemm_f16_tflops"] = 2.0 * m ** 3 / t / 1e12
    del x, y
    n = 2 << 30
    a = torch.empty(n, dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    t = timed(lambda: b.copy_(a), 8)
    _PEAKS["copy_gbs"] = 2.0 * n / t / 1e9
    del a, b
    torch.cuda.empty_cache()
    _PEAKS["how"] = ("measured after the timed region: torch.matmul f16 16384^3 on random data (hipBLASLt), "
                     "device copy of 2 GiB (read + write bytes)")
    return _PEAKS


def with_achievable(roof, key):
    """``roof`` (a roofline dict) plus the live achievable peak of its unit and the fraction of it."""
    pk = achievable_peaks()
    v = pk[key]
    roof["achievable"] = {"peak": v, "unit": roof.get("unit"), "frac": roof["achieved"] / v if v else None,
                          "how": pk["how"]}
    return roof


def timer_stats(timers, base):
    """Launch statistics of KernelTimers (one per stream): (launches, mean launch ms, busy ms) where
    busy = the union of the launch intervals over all streams (ms, from HIP events against ``base``)."""
    iv = []
    for t in timers:
        for a, b, _ in t.pairs:
            iv.append((base.elapsed_time(a), base.elapsed_time(b)))
    if not iv:
        return 0, 0.0, 0.0
    n = len(iv)
    mean = sum(b - a for a, b in iv) / n
    iv.sort()
    busy, cur0, cur1 = 0.0, iv[0][0], iv[0][1]
    for a, b in iv[1:]:
        if a > cur1:
            busy += cur1 - cur0
            cur0, cur1 = a, b
        else:
            cur1 = max(cur1, b)
    busy += cur1 - cur0
    return n, mean, busy


def cpu_baseline(args):
    """The C oracle's search + float32 numpy GomokuNetEZ on the host cores (reported baseline, kind
    "port"): one single-threaded process per core used (oracle/cpu_baseline.py, started as child
    processes), each playing its own game from a random opening of 0..~120 stones for about
    ``--cpu-baseline-sec`` seconds; value = all processes' moves / the wall time of the slowest."""
    try:
        avail = len(os.sched_getaffinity(0))
    except Exception:
        avail = os.cpu_count() or 1
    P = max(1, min(args.cpu_baseline_procs, avail))
    script = os.path.join(REPO, "oracle", "cpu_baseline.py")
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    procs = []
    t0 = time.perf_counter()
    for i in range(P):
        opening = (i * 8) % 128
        cmd = [sys.executable, script, "--size", str(args.size), "--sims", str(args.sims), "--mode", args.mode,
               "--blocks", str(args.blocks), "--seed", str(args.seed + 101 * i), "--weights-seed", str(args.seed),
               "--opening", str(opening), "--seconds", str(args.cpu_baseline_sec)]
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env))
    res = []
    for p in procs:
        out, err = p.communicate(timeout=args.cpu_baseline_sec * 6 + 120)
        if p.returncode != 0:
            raise RuntimeError("cpu_baseline worker failed: %s" % err[-2000:])
        res.append(json.loads(out.strip().splitlines()[-1]))
    wall = time.perf_counter() - t0
    moves = sum(r["moves"] for r in res)
    rows = sum(r["rows"] for r in res)
    slowest = max(r["seconds"] for r in res)
    stones = sorted(x for r in res for x in r["stones"])
    return {"value": moves / slowest, "unit": "moves/s", "cores": P, "kind": "port",
            "sample": "%d moves over %d single-threaded processes (one per core used, as many as the reference's "
                      "process graph runs: NUM_WORKERS = 15 self-play workers + 1 inference server, config.py:13; "
                      "%d cores available to the process), each one %dx%d game from a random opening (%d..%d stones at the searched positions), "
                      "%d sims (%s), %d NN rows (the reference's duplicate-leaf batches kept); slowest process %.1f s, "
                      "wall %.1f s; C oracle search + numpy fp32 GomokuNetEZ (oracle/cpu_baseline.py)"
                      % (moves, P, avail, args.size, args.size, stones[0], stones[-1], args.sims, args.mode, rows,
                         slowest, wall)}


def trainer_flop_per_step(H, blocks, B, U, C=128, hd=64, proj=512):
    """Algorithmic FLOP of one training step (loss.py:30-158 at B boards, U unroll steps): the
    convolutions and Linears of every forward, x3 for the parts with gradients (forward, input and weight
    gradients), x1 for the no-grad parts (the target network's representation and the U consistency
    representations).  Elementwise work (BatchNorm, activations, losses) is not counted."""
    A = H * H
    conv = 2.0 * A * C * C * 9                      # one 128 -> 128 3x3 conv, one board
    repr_ = 2 * blocks * conv + 2.0 * A * C * 3 * 9  # representation: stem 3 -> 128 + residual blocks
    dyn = 2 * blocks * conv + 2.0 * A * C * (C + 16) * 9 + 2.0 * A * 16  # dynamics: embed + 144 -> 128 + blocks
    pred = 2.0 * A * C * 3 + 2.0 * (2 * A) * A + 2.0 * A * hd + 2.0 * hd * 3   # 1x1 convs, policy_fc, value MLP
    projection = 2.0 * (A * C) * proj + 2.0 * proj * proj
    reward = 2.0 * (A * C) * hd + 2.0 * hd * 3
    grad = repr_ + U * dyn + (U + 1) * pred + U * projection + U * reward
    nograd = repr_ + U * repr_ + U * projection + pred  # target value, consistency trunks + their projections
    return B * (3.0 * grad + nograd)


def trainer_leg(args, world, rank, dist, backend):
    """Config C4's training step on every rank (DDP when world > 1), timed like the self-play region."""
    from datou_gomoku_muzero_amd import trainer as T, weights as W
    torch.backends.cudnn.benchmark = True  # MIOpen Find for the convolutions left on MIOpen
    cfg = T.TrainConfig(BOARD_SIZE=args.size, NUM_RES_BLOCKS=args.blocks, PHYSICAL_BATCH_SIZE=args.trainer_batch,
                        TRAIN_BUFFER_SIZE=args.trainer_buffer, ENABLE_PER=True)
    rb = T.ReplayBuffer(cfg, device="cuda")
    rs = np.random.RandomState(args.seed + 31 * rank)
    rb.add_arrays(*W.synthetic_slices(args.trainer_buffer, args.size, cfg.NUM_UNROLL_STEPS, rs))
    group = dist if dist is not None else None

    def timed_run(steps, target_f16):
        """A fresh trainer with trainer.TARGET_F16 = target_f16: warm-up, then `steps` timed steps -> (seconds, last
        loss, allreduce_ms)."""
        saved = T.TARGET_F16
        T.TARGET_F16 = target_f16
        try:
            tr = T.Trainer(cfg, device="cuda")
            pending = [None]

            def step():
                batch, idx, w = rb.sample(args.trainer_batch, rs, dist=group)
                logs, td = tr.step(batch, w, sync=False)
                rb.update_priorities(idx, td, dist=group)
                pending[0] = logs

            t_w = time.perf_counter()
            for _ in range(args.trainer_warmup):
                step()
            torch.cuda.synchronize()
            log("rank %d: trainer warm-up %.1f s (MIOpen Find, graph capture; target trunk %s)"
                % (rank, time.perf_counter() - t_w, "f16" if target_f16 else "f32"))
            tr.reset_allreduce_times()
            if dist:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            torch.cuda.synchronize()
            if dist:
                dist.barrier()
            dt = collective_max(time.perf_counter() - t0, dist, backend)
            return dt, float(pending[0][0]) if pending[0] is not None else None, tr.allreduce_times()
        finally:
            T.TARGET_F16 = saved

    dt, loss, ar = timed_run(args.trainer_steps, True)
    ar_ms = None if ar is None else ar["wait_ms"]
    # the reference's precision for the target network's value (loss.py:54-55: a float32 forward outside autocast):
    # the same step with trainer.TARGET_F16 = False, beside the line's f16-trunk rate
    f32_steps = args.trainer_f32_steps
    dt32 = timed_run(f32_steps, False)[0] if f32_steps > 0 else None
    torch.cuda.empty_cache()
    step_flop = trainer_flop_per_step(args.size, args.blocks, args.trainer_batch, cfg.NUM_UNROLL_STEPS)
    step_ach = step_flop * args.trainer_steps / dt / 1e12
    # the dominant HIP kernel of the step: the 128->128 residual-block conv (forward and input gradient),
    # timed standalone at the step's shape (B boards, f16 NHWC) with HIP events
    B, H = args.trainer_batch, args.size
    x = torch.randn(B, 128, H, H, device="cuda").half().contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(128, 128, 3, 3, device="cuda") / 34).contiguous(memory_format=torch.channels_last)
    pk = T._packed_conv_weight(wt, torch.float16, 0)
    for _ in range(3):
        T._conv3x3_hip(x, pk)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    n = 20
    for _ in range(n):
        T._conv3x3_hip(x, pk)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / n
    flop = 2.0 * B * H * H * 128 * 128 * 9
    ach = flop / (ms * 1e-3) / 1e12
    return {"metric": "trainer steps/sec (C4: B=%d per GPU, %d unroll steps, %dx%d, %d blocks, PER)"
                      % (B, cfg.NUM_UNROLL_STEPS, H, H, args.blocks),
            "value": args.trainer_steps / dt, "unit": "steps/s", "n_gpus": world, "steps": args.trainer_steps,
            "warmup": args.trainer_warmup, "ms_per_step": dt / args.trainer_steps * 1e3,
            "samples_per_s": args.trainer_steps * B * world / dt, "higher_is_better": True, "scaling": "weak",
            "dtype": ("fp16 autocast (f32 master weights); the target network's value on an f16 trunk (f16 operands, f32 "
                      "accumulation, f16 activations: trainer.TARGET_F16, a stated parity exception, DESIGN.md 8) — "
                      "value_target_f32 is the same step with the reference's float32 target"),
            "value_target_f32": f32_steps / dt32 if dt32 else None,
            "steps_target_f32": f32_steps,
            "data": "synthetic slices in a device PER shard per rank (%d each)" % args.trainer_buffer,
            "parallelism": "ddp%d: one flat-bucket gradient all-reduce + sharded-PER syncs per step" % world
            if world > 1 else "single GPU",
            "last_loss": loss,
            "allreduce_ms": ar_ms,
            "wgrad_flush_ms": None if ar is None else ar["flush_ms"],
            "allreduce_window_ms": None if ar is None else ar["window_ms"],
            "allreduce_note": ("per step on the compute stream: allreduce_ms = the exposed communication, from bucket B's "
                               "weight gradients enqueued to both buckets averaged (B's all-reduce + what of A's did not "
                               "hide); wgrad_flush_ms = bucket B's weight gradients, which A's all-reduce overlaps "
                               "(trainer.allreduce_times)" if ar_ms is not None else "single GPU: no all-reduce"),
            "roofline_step": {"bound": "mfma", "achieved": step_ach, "peak": PEAK_MFMA_TFLOPS, "unit": "TFLOP/s",
                              "frac": step_ach / PEAK_MFMA_TFLOPS, "flop_per_step": step_flop,
                              "count": "bench.trainer_flop_per_step (DESIGN.md 8): convs + Linears, x3 with gradients"},
            "roofline": {"bound": "mfma", "kernel": "gmz_conv3x3 (128->128 3x3 conv, f16 NHWC, B=%d)" % B,
                         "achieved": ach, "peak": PEAK_MFMA_TFLOPS, "unit": "TFLOP/s", "frac": ach / PEAK_MFMA_TFLOPS,
                         "mean_launch_ms": ms, "timed": "standalone at the step's shape, %d launches" % n,
                         "traffic": None},
            "roofline_in_step": trainer_trace_summary(args)}


def trainer_trace_summary(args):
    """The dominant convolution inside the graph-replayed trainer step and the step's launch count, from the
    committed rocprofv3 trace summary (tools/trainer_profile.sh -> tools/trainer_trace_summary.py; a HIP
    graph's kernels cannot be timed from inside the process): builder-measured, not this run."""
    import glob
    paths = sorted(glob.glob(os.path.join(REPO, "profiles", "r[0-9][0-9]_trainer_trace.json")))
    path = paths[-1] if paths else ""
    if not path or (args.size, args.blocks, args.trainer_batch) != (15, 8, 360):
        return None
    try:
        d = json.load(open(path))
    except Exception:
        return None
    out = dict(d.get("dominant", {}))  # launches_per_step / ms_per_step here: the dominant kernel's, per step
    out.update(bound="mfma", step_launches=d.get("launches_per_step"), weight_gradient=d.get("weight_gradient"),
               source="builder-measured: %s (%s)" % (os.path.relpath(path, REPO), d.get("source", "")))
    return out


def selfplay_leg(args, rank, world, dist, backend, size, sims, mode, blocks, G, steps, warmup, streams=None,
                 single_stream_moves=0, log_prefix="", openings=None):
    """G games of (size, sims, mode, blocks) self-play on this rank's GPU: ``warmup`` untimed moves, then
    ``steps`` timed moves (barrier + synchronize on both sides, max over ranks).  ``openings``: the games'
    start positions (engine.seeded_openings; None = empty boards).  Returns a dict with dt (s, max over
    ranks), rank_dt (every rank's own time), finished_games (games that ended in the timed moves, all
    ranks), waves, streams, roofline (dominant tower), roofline_tree and, with single_stream_moves > 0
    and two streams, single_stream_kernels."""
    import datou_gomoku_muzero_amd.engine as E
    from datou_gomoku_muzero_amd import network as N, weights as W
    from datou_gomoku_muzero_amd.config import GmzConfig
    cfg = GmzConfig(BOARD_SIZE=size, NUM_SIMULATIONS=sims, MCTS_IMPLEMENTATION=mode, NUM_RES_BLOCKS=blocks)
    sd = W.synthetic_state_dict(cfg, seed=args.seed, with_projection=False)
    if dist is not None:  # the self-play tier's one exchange: rank 0's weights -> all ranks (RCCL)
        from datou_gomoku_muzero_amd.weight_sync import broadcast_state_dict
        dev = "cuda" if backend == "nccl" else "cpu"
        sd = {k: v.cpu().numpy() for k, v in broadcast_state_dict(sd, src=0, device=dev).items()}
    slots = E.hidden_slots(cfg, G)  # the steady-state pool (grows if late-game searches need more)
    if args.net == "hip":
        net = N.GomokuNetHip(sd, cfg, num_slots=slots, max_rows=G, precision=args.precision)
    else:
        net = E.HashNetBackend(slots, cfg.ACTION_SPACE_SIZE)
    if streams is None:
        streams = E.default_streams(cfg, G)
    tkw = dict(layout=args.layout, descent_hint=None if args.hint is None else args.hint == "on",
               pair=None if getattr(args, "pair", None) is None else args.pair == "on")
    eng = E.make_engine(cfg, num_games=G, net=net, seed=args.seed + 7919 * rank, streams=streams, **tkw)
    eng.reset_games()
    if openings is not None:
        eng.set_positions(*openings)
    parts = eng.engines if streams > 1 else [eng]
    pstreams = eng.streams if streams > 1 else [torch.cuda.current_stream()]
    log("%srank %d: engine G=%d %dx%d %s/%d, %d blocks, net=%s, %d stream(s), %s tree, hint %s"
        % (log_prefix, rank, G, size, size, mode, sims, blocks, args.net, streams, parts[0].layout,
           parts[0].descent_hint))

    finished = torch.zeros((), dtype=torch.int64, device="cuda")

    def step():
        eng.search()
        st = eng.play(reset_finished=True)
        # +1 / -1 winner or 0 draw: the game ended on this move (and restarts from the empty board).  Counted
        # in the warm-up moves too, so the first use of these kernels (a lazy code-object load, ~0.1 s on a
        # fresh box) is not inside the timed moves; zeroed before them
        finished.add_(((st == 1) | (st == -1) | (st == 0)).sum())

    for i in range(warmup):
        step()
        torch.cuda.synchronize()
        log("%swarmup %d/%d done" % (log_prefix, i + 1, warmup))
    az = mode == "AlphaZero"  # AlphaZero searches run the representation tower per wave
    timers, tree_timers = [], []
    for e, st in zip(parts, pstreams):  # HIP events on each part's launch stream
        if getattr(args, "kernel_timers", "on") == "off":  # (A/B of the events' own cost; no roofline then)
            break
        if args.net == "hip":
            t = N.KernelTimer(st)
            timers.append(t)
            if az:
                e.net.repr_timer = t
            else:
                e.net.tower_timer = t
        e.tree_timer = N.KernelTimer(st)
        tree_timers.append(e.tree_timer)
    eng.tree_counters(reset=True)
    finished.zero_()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    base = torch.cuda.Event(enable_timing=True)
    base.record()
    t0 = time.perf_counter()
    waves = 0
    marks = [t0]
    for i in range(steps):
        step()
        waves += eng.waves_last
        marks.append(time.perf_counter())  # host clock per move (the host reads each move's status)
        if (i + 1) % max(1, steps // 5) == 0:
            log("%sstep %d/%d" % (log_prefix, i + 1, steps))
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    own = time.perf_counter() - t0
    dt = collective_max(own, dist, backend)
    res = {"dt": dt, "waves": waves, "streams": streams, "rank_dt": collective_gather(own, dist, backend),
           "finished_games": int(collective_sum(float(finished.item()), dist, backend)),
           "step_ms": [round((b - a) * 1e3, 2) for a, b in zip(marks, marks[1:])]}
    ctr = eng.tree_counters()
    traffic_note = "from the committed builder PMC pass %s (not measured in this run)"
    fpr = (repr_flop_per_row if az else tower_flop_per_row)(size, blocks)
    if timers:
        n_launch, ms, busy = timer_stats(timers, base)
        # rows the searches requested (finished games' rows are skipped by the tower): every selected
        # game-wave is one row; AlphaZero's representation tower also runs each move's G root rows
        rows = (ctr["selects"] + (G * steps if az else 0)) / max(1, n_launch)
        flop = fpr * rows
        per_launch = flop / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
        # delivered rate while the kernel runs: all launches' FLOP over the union of their intervals
        # (with one stream = the per-launch figure; with two, launches of the two streams overlap)
        achieved = flop * n_launch / (busy * 1e-3) / 1e12 if busy > 0 else 0.0
        is_c2 = (size, blocks, G, mode) == (15, 8, 1024, "MuZero")
        traffic = pmc_traffic(args.pmc_file, args, G, az, streams) if is_c2 else None
        kname = ("k_tower3<%d,REPR> (representation tower, stem + %d fused convs + head 1x1 convs)" % (size, 2 * blocks)
                 if az else "k_tower3<%d,DYN> (dynamics tower, %d fused convs + head 1x1 convs)" % (size, 1 + 2 * blocks))
        res["roofline"] = {"bound": "mfma", "kernel": kname + ", " + args.precision,
                           "achieved": achieved, "peak": PEAK_MFMA_TFLOPS, "unit": "TFLOP/s",
                           "frac": achieved / PEAK_MFMA_TFLOPS, "traffic": traffic,
                           "traffic_source": (traffic_note % os.path.relpath(args.pmc_file, REPO)) if traffic else None,
                           "launches": n_launch, "mean_launch_ms": ms, "rows_per_launch": rows,
                           "flop_per_row": fpr, "streams": streams, "busy_ms": busy,
                           "achieved_per_launch": per_launch,
                           "timing": "HIP events around every launch on its stream; achieved = algorithmic FLOP of all "
                                     "launches / busy_ms (union of the launch intervals of all streams)"}
    n_tree, ms_tree, busy_tree = timer_stats(tree_timers, base)
    if n_tree:
        A = size * size
        bpl = tree_bytes(ctr, A) / n_tree
        gbs = bpl * n_tree / (busy_tree * 1e-3) / 1e9 if busy_tree > 0 else 0.0
        tfile = {1024: args.pmc_tree_file, 8192: PMC_TREE_G8192}.get(G)
        tr = (pmc_traffic(tfile, args, G, az, streams, size, blocks)
              if (tfile and (size, blocks, mode) == (15, 8, "MuZero")) else None)
        # the same rate on the kernel's MEASURED bytes (PMC FETCH_SIZE x2 + WRITE_SIZE per launch, committed
        # pass of this configuration) in place of the SURVEY 8(d) model's: the lists move fewer bytes than the
        # model counts, the dense hint kernel more (its cached exp rows)
        gbs_m = tr * n_tree / (busy_tree * 1e-3) / 1e9 if (tr and busy_tree > 0) else None
        res["roofline_tree"] = {
            "bound": "hbm", "kernel": "k_expand_select<%d> (backup of wave i + selection of wave i+1)" % ((A + 63) // 64),
            "achieved": gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": gbs / PEAK_HBM_GBS,
            "achieved_measured": gbs_m, "frac_measured": gbs_m / PEAK_HBM_GBS if gbs_m else None,
            "traffic": tr, "traffic_source": (traffic_note % os.path.relpath(tfile, REPO)) if tr else None,
            "launches": n_tree, "mean_launch_ms": ms_tree, "bytes_per_launch": bpl,
            "mean_backup_levels": ctr["backup_levels"] / max(1, ctr["backups"]),
            "mean_select_levels": ctr["select_levels"] / max(1, ctr["selects"]),
            "games_per_launch": ctr["backups"] / n_tree, "streams": streams, "busy_ms": busy_tree,
            "layout": parts[0].layout, "descent_hint": parts[0].descent_hint, "waves_per_game": 2 if parts[0].pair else 1,
            "achieved_per_launch": bpl / (ms_tree * 1e-3) / 1e9,
            "backup": backup_roofline(ctr, A, n_tree, busy_tree, G),
            "note": ("two streams: each launch runs on the CUs the other stream's capped tower leaves free (about "
                     "a quarter of them), so this is the kernel inside the step, not its own rate; "
                     "single_stream_kernels.tree has the kernel alone on every CU" if streams > 1 else
                     "one stream: the kernel alone on every CU")}
    if streams > 1 and single_stream_moves > 0:
        # the same G games as ONE engine on one stream (every CU per launch): the kernels' launch times
        # without the other stream beside them (not the headline: the two-stream step above is)
        for e in parts:
            e.net.tower_timer = e.net.repr_timer = None
        eng.close()
        e1 = E.BatchedSelfPlayEngine(cfg, num_games=G, net=net, seed=args.seed + 7919 * rank + 1, **tkw)
        e1.reset_games()
        e1.search()
        e1.play(reset_finished=True)
        t1, tt1 = (N.KernelTimer() if args.net == "hip" else None), N.KernelTimer()
        if t1 is not None:
            if az:
                net.repr_timer = t1
            else:
                net.tower_timer = t1
        e1.tree_timer = tt1
        e1.tree_counters(reset=True)
        torch.cuda.synchronize()
        b1 = torch.cuda.Event(enable_timing=True)
        b1.record()
        for _ in range(single_stream_moves):
            e1.search()
            e1.play(reset_finished=True)
        torch.cuda.synchronize()
        c1 = e1.tree_counters()
        ss = {"moves": single_stream_moves, "games": G}
        if t1 is not None:
            n1, m1, _ = timer_stats([t1], b1)
            r1 = (c1["selects"] + (G * single_stream_moves if az else 0)) / max(1, n1)
            a1 = fpr * r1 / (m1 * 1e-3) / 1e12
            ss["tower"] = {"mean_launch_ms": m1, "rows_per_launch": r1, "achieved": a1, "frac": a1 / PEAK_MFMA_TFLOPS}
        n2, m2, _ = timer_stats([tt1], b1)
        if n2:
            g2 = tree_bytes(c1, size * size) / n2 / (m2 * 1e-3) / 1e9
            ss["tree"] = {"mean_launch_ms": m2, "achieved_gbs": g2, "frac": g2 / PEAK_HBM_GBS,
                          "backup": backup_roofline(c1, size * size, n2, m2 * n2, G)}
        res["single_stream_kernels"] = ss
        net.tower_timer = net.repr_timer = None
        e1.close()
        del e1
    eng.close()
    del eng, net
    torch.cuda.empty_cache()
    return res


SUBLINES = {  # BASELINE.json configs run on the GPU besides the headline (C2)
    # the headline's configuration from empty boards (the round 1-3 headline, kept for continuity): the first
    # warmup + steps moves of every game, so no game ends and the tree shapes are those of openings
    "empty_board": dict(size=15, sims=400, mode="MuZero", blocks=8, headline_games=True, headline_steps=True,
                        name="C2 from empty boards (no game ends in the window; rounds 1-3's headline workload)"),
    "c5": dict(size=19, sims=800, mode="MuZero", blocks=16,
               name="C5: 19x19, 800 sims/move, GomokuNetEZ 16 blocks (BASELINE config 5)"),
    "c1": dict(size=9, sims=50, mode="AlphaZero", blocks=8,
               name="C1 on the GPU: 9x9 AlphaZero, 50 sims/move, 8 blocks (BASELINE config 1's search; the "
                    "reference runs it with one CPU worker)"),
    # SURVEY §8(d)'s tree-kernel measurement point (>= 8,192 trees): config C2's search with 8,192 games as ONE
    # engine on one stream (compact child lists, engine.default_layout), so roofline_tree is the kernel alone
    "g8192": dict(size=15, sims=400, mode="MuZero", blocks=8, games=8192, streams=1, steps=2, warmup=1,
                  min_free_gb=100,
                  name="C2's search at 8,192 trees on one GPU (one engine, one stream): the tree kernel at SURVEY "
                       "8(d)'s >= 8,192-tree measurement point"),
}


def subline(args, key, rank, world, dist, backend):
    c = SUBLINES[key]
    G = args.games if c.get("headline_games") else c.get("games", args.subline_games)
    steps, warmup = {"c5": (args.c5_steps, 1), "c1": (args.c1_steps, 2)}.get(key, (c.get("steps", 2), c.get("warmup", 1)))
    if c.get("headline_steps"):
        steps, warmup = args.steps, args.warmup
    if "min_free_gb" in c:  # a bounded leg: skipped (and said so) when this GPU lacks the memory
        torch.cuda.empty_cache()
        free = torch.cuda.mem_get_info()[0] / 2 ** 30
        # ranks sharing a GPU (the gloo rehearsal of N > 1 on one card) each need the leg's memory
        share = ranks_per_gpu(dist)
        need = c["min_free_gb"] * share
        if collective_max(-free, dist, backend) > -need:
            return {"config": c["name"], "skipped": "needs %d GiB free per GPU (%d rank(s) per GPU), %.0f GiB free"
                    % (need, share, free)}
    r = selfplay_leg(args, rank, world, dist, backend, c["size"], c["sims"], c["mode"], c["blocks"], G, steps, warmup,
                     streams=c.get("streams"), log_prefix="[%s] " % key)
    out = {"config": c["name"], "value": G * steps * world / r["dt"], "unit": "moves/s", "n_gpus": world,
           "games_per_gpu": G, "steps": steps, "warmup": warmup, "ms_per_step": r["dt"] / steps * 1e3,
           "waves_per_move": r["waves"] / max(1, steps), "streams": r["streams"], "dtype": args.precision,
           "finished_games": r["finished_games"]}
    for k in ("roofline", "roofline_tree"):
        if k in r:
            q = r[k]
            out[k] = {x: q[x] for x in ("kernel", "achieved", "unit", "frac", "mean_launch_ms", "bytes_per_launch",
                                        "layout", "games_per_launch", "mean_select_levels", "traffic",
                                        "achieved_measured", "frac_measured", "traffic_source", "backup") if x in q}
    return out


def ranks_per_gpu(dist):
    """How many ranks use this rank's GPU (1 on a node with one rank per GPU): ranks are matched by
    host name and the device's PCI location, gathered over the process group."""
    if dist is None:
        return 1
    import socket
    p = torch.cuda.get_device_properties(torch.cuda.current_device())
    me = (socket.gethostname(), p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
    everyone = [None] * dist.get_world_size()
    dist.all_gather_object(everyone, me)
    return sum(1 for x in everyone if x == me)


def consumer_proc(qs, ctl, report):
    """The reference's queue readers (DataLoader, DisplayManager, log reader; main.py:60-78): one thread
    per queue, blocking gets that unpickle every payload, until a None sentinel; then the counts go to
    ``report``.  Started by bench.py before anything touches the GPU; ``ctl`` starts a round (None: exit)."""
    import threading
    while True:
        go = ctl.get()  # one round per worker leg; None ends the process
        if go is None:
            return
        n, slices = {}, {}

        def read(k, q):
            c = sl = 0
            while True:
                item = q.get()
                if item is None:
                    break
                c += 1
                if k == "data":
                    sl += len(item[1])
            n[k], slices[k] = c, sl

        th = [threading.Thread(target=read, args=(k, q)) for k, q in qs.items()]
        for t in th:
            t.start()
        for t in th:
            t.join()
        report.put(dict(n, slices=slices.get("data", 0)))


class _Flag:
    def __init__(self):
        self.f = False

    def is_set(self):
        return self.f


def start_consumer():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    qs = {"data": ctx.Queue(maxsize=50000), "ui": ctx.Queue(), "log": ctx.Queue(), "trainer": ctx.Queue()}
    ctl, report = ctx.Queue(), ctx.Queue()
    p = ctx.Process(target=consumer_proc, args=(qs, ctl, report), daemon=True)
    p.start()
    return p, qs, ctl, report


def worker_leg(args, rank, world, dist, backend, consumer, engine_rate):
    """worker.gpu_selfplay_worker (the drop-in for N universal_workers + the inference server,
    workers.py:129-241 / 314-373) on this rank's GPU with real torch.multiprocessing queues and a
    consumer process: moves/s over the steady-state moves, until every record of them is posted."""
    from datou_gomoku_muzero_amd.worker import gpu_selfplay_worker
    from datou_gomoku_muzero_amd.config import GmzConfig
    proc, qs, ctl, report = consumer
    cfg = GmzConfig(BOARD_SIZE=args.size, NUM_SIMULATIONS=args.sims, MCTS_IMPLEMENTATION=args.mode,
                    NUM_RES_BLOCKS=args.blocks)
    ctl.put(True)  # the consumer starts its readers
    times = []
    warm, moves = args.worker_warmup, args.worker_moves
    if dist:
        dist.barrier()
    import datou_gomoku_muzero_amd.engine as E
    op = (E.random_openings(args.games, args.size, np.random.RandomState(args.seed + 29 * rank), args.worker_openings,
                            n_in_row=cfg.N_IN_ROW)
          if args.worker_openings > 0 else None)
    gpu_selfplay_worker(rank, None, qs["data"], qs["log"], qs["ui"], _Flag(), trainer_event_queue=qs["trainer"],
                        num_games=args.games, cfg=cfg, max_moves=warm + moves, emit_move_notices=True,
                        move_times=times, seed=args.seed + 7919 * rank, precision=args.precision,
                        device=torch.cuda.current_device(), openings=op)
    for q in qs.values():
        q.put(None)
    counts = report.get(timeout=300)
    steady = collective_max(times[-1] - times[warm - 1], dist, backend)
    tot = {k: collective_sum(float(v), dist, backend) for k, v in counts.items()}
    value = args.games * moves * world / steady
    return {"metric": "drop-in worker self-play moves/sec (worker.gpu_selfplay_worker, %dx%d, %d sims)"
                      % (args.size, args.size, args.sims),
            "value": value, "unit": "moves/s", "n_gpus": world, "games_per_gpu": args.games, "moves": moves,
            "warmup_moves": warm, "steady_s": steady, "worker_over_engine": value / engine_rate if engine_rate else None,
            "move_ms": [round((b - a) * 1e3, 2) for a, b in zip(times[warm - 1:-1], times[warm:])],
            "finished_games": int(tot.get("data", 0)), "slices": int(tot.get("slices", 0)),
            "messages": {k: int(v) for k, v in tot.items() if k != "slices"},
            "queues": "torch.multiprocessing (spawn) Queues of main.py's sizes; a consumer process unpickles every "
                      "payload (GameRecord + TrainingSlices, SelfPlayMove / SelfPlayStatus / GameCompletedNotice)",
            "data": ("each slot's first game from a random opening of 0..%d stones (staggered starts; its record "
                     "holds the moves searched from there), later games from the empty board" % args.worker_openings
                     if args.worker_openings > 0 else "games from the empty board"),
            "timed": "from the host clock after warm-up move %d was queued to after the last move's records were "
                     "posted (per-move history, winning-move scan, record building all inside)" % warm}


PHASE_ENV = "GMZ_BENCH_PHASE"
PHASE_MARK = "GMZ_PHASE_RESULT "


def phase_keys(name, args):
    """The keys of the line a phase fills (a phase that fails puts {"error": ...} in each)."""
    modes = [m.strip() for m in args.loop_modes.split(",") if m.strip()]
    return {"selfplay": [],
            "extras": (["sublines"] if [k for k in args.sublines.split(",") if k.strip()] else [])
            + (["worker"] if args.worker_moves > 0 else []),
            "trainer": ["trainer"],
            "loop": ["loop_c4" if m == "sliced" else "loop_c4_concurrent" for m in modes]}[name]


def phase_plan(args):
    """The phases this run needs, in order, with their wall-time caps (s).  ``selfplay`` = the headline
    (+ its single-stream kernel times); ``extras`` = the sublines and the drop-in worker leg (self-play only:
    no collective but barriers and timing reductions); ``trainer`` and ``loop`` carry the heavy RCCL traffic
    (gradient all-reduce, PER syncs, weight broadcast)."""
    plan = [("selfplay", args.phase_timeout_selfplay)]
    if args.net == "hip":
        if [k for k in args.sublines.split(",") if k.strip()] or args.worker_moves > 0:
            plan.append(("extras", args.phase_timeout_extras))
        if args.trainer_steps > 0:
            plan.append(("trainer", args.phase_timeout_trainer))
        if args.loop_iters > 0 and [m for m in args.loop_modes.split(",") if m.strip()]:
            plan.append(("loop", args.phase_timeout_loop))
    return plan


def inject_failure(phase, rank):
    """GMZ_BENCH_INJECT_FAIL=<phase>:<rank> makes that rank's leg of that phase raise after the process
    group is up, so its peers are left waiting in a collective (the failure an untested RCCL path would
    cause) - the rehearsal that the headline survives it."""
    spec = os.environ.get("GMZ_BENCH_INJECT_FAIL", "")
    if spec and spec == "%s:%d" % (phase, rank):
        raise RuntimeError("injected failure (GMZ_BENCH_INJECT_FAIL=%s)" % spec)


def run_phase(phase, args, rank, world, dist, backend, consumer=None, out=None):
    """The legs of one phase on this rank; returns the line's fragment (rank 0's is the one printed).
    In-process mode passes ``out`` (the line so far) so the worker leg can quote the headline rate."""
    frag = {}
    if phase == "selfplay":
        G = args.games
        r = selfplay_leg(args, rank, world, dist, backend, args.size, args.sims, args.mode, args.blocks, G,
                         args.steps, args.warmup, streams=args.streams, single_stream_moves=args.single_stream_moves,
                         openings=headline_openings(args, rank, G, args.size))
        args.streams = r["streams"]
        frag = result_line(args, world, r["dt"], r["waves"], G, backend)
        frag["finished_games"] = r["finished_games"]
        frag["rank_values"] = [G * args.steps / t if t > 0 else None for t in r["rank_dt"]]
        frag["step_ms"] = r["step_ms"]  # rank 0's host time per timed move
        for k in ("roofline", "roofline_tree", "single_stream_kernels"):
            if k in r:
                frag[k] = r[k]
        if rank == 0 and args.net == "hip" and "roofline" in frag:  # after every timed region of this phase
            with_achievable(frag["roofline"], "gemm_f16_tflops")
            if "roofline_tree" in frag:
                with_achievable(frag["roofline_tree"], "copy_gbs")
        return frag
    inject_failure(phase, rank)
    if phase == "extras":
        subs = {}
        for key in [k.strip() for k in args.sublines.split(",") if k.strip()]:
            if key not in SUBLINES:
                raise SystemExit("bench.py: unknown --sublines entry %r" % key)
            subs[key] = subline(args, key, rank, world, dist, backend)
        if subs:
            frag["sublines"] = subs
        if consumer is not None:
            rate = (out or {}).get("value") or args.headline_value
            frag["worker"] = worker_leg(args, rank, world, dist, backend, consumer, rate)
            consumer[2].put(None)  # the consumer process exits
            torch.cuda.empty_cache()
    elif phase == "trainer":
        torch.cuda.empty_cache()
        frag["trainer"] = trainer_leg(args, world, rank, dist, backend)
    elif phase == "loop":
        frag.update(loop_legs(args, rank, world, dist, backend))
    return frag


def loop_legs(args, rank, world, dist, backend):
    from datou_gomoku_muzero_amd.loop import run_c4
    out = {}
    for mode in [m.strip() for m in args.loop_modes.split(",") if m.strip()]:
        if mode not in ("sliced", "concurrent"):
            raise SystemExit("bench.py: unknown --loop-modes entry %r" % mode)
        args.loop_concurrent = mode == "concurrent"
        torch.cuda.empty_cache()
        d, dt_loop = run_c4(args, rank, world, dist, backend, log=log)
        dt_loop = collective_max(dt_loop, dist, backend)
        push_ms = collective_max(d.pop("push_ms"), dist, backend)
        tot = {k: collective_sum(float(v), dist, backend) for k, v in d.items()}
        step_ms = dt_loop / max(1, d["train_steps"]) * 1e3
        out["loop_c4" if mode == "sliced" else "loop_c4_concurrent"] = {
            "metric": "C4 loop: self-play moves/sec and trainer steps/sec with both running on every GPU",
            "mode": mode + (": each iteration's trainer steps run on their own HIP stream beside its self-play "
                            "moves" if mode == "concurrent" else ": each iteration = moves, then trainer steps"),
            "moves_per_s": tot["moves"] * args.loop_games / dt_loop, "trainer_steps_per_s": d["train_steps"] / dt_loop,
            "unit": "moves/s, steps/s", "n_gpus": world, "iterations": args.loop_iters, "seconds": dt_loop,
            "games_per_gpu": args.loop_games, "moves_per_iter": args.loop_moves_per_iter,
            "train_steps_per_iter": args.loop_train_per_iter, "batch_per_gpu": args.trainer_batch,
            "warmup_iterations": args.loop_warmup,
            "finished_games": int(tot["games"]), "slices_added": int(tot["slices"]),
            "weight_pushes": d["weight_pushes"], "model_update_interval": args.loop_update_interval,
            "weight_push_ms": push_ms,
            "push_share_at_interval": {"interval": 1000, "ms_per_trainer_step": push_ms / 1000.0,
                                       "share_of_iteration": push_ms / 1000.0 / step_ms if step_ms else None},
            "data": "self-play with the trainer's weights, each slot's first game from a random opening of "
                    "0..%d stones (staggered starts, so games finish in the timed window; later games from the "
                    "empty board); each PER shard also pre-filled with %d synthetic slices so training starts "
                    "at once" % (args.loop_openings, args.loop_prefill),
            "parallelism": "dp%d: self-play + replay shard per GPU; one gradient all-reduce + sharded-PER syncs "
                           "per step; rank 0 weight broadcast per push" % world}
    return out


def init_dist(args, rank, local, world):
    """This process's GPU and (world > 1) its process group, every collective bounded by --dist-timeout."""
    import datetime
    dist = backend = None
    if world > 1:
        import torch.distributed as dist
        # GMZ_DIST_BACKEND=gloo rehearses the N>1 path with several ranks sharing one GPU
        backend = os.environ.get("GMZ_DIST_BACKEND", "nccl")
        torch.cuda.set_device(local % torch.cuda.device_count())
        dist.init_process_group(backend, init_method="env://",
                                timeout=datetime.timedelta(seconds=args.dist_timeout))
        if rank == 0:
            log("torch.distributed: world_size=%d backend=%s (%s)" % (dist.get_world_size(), dist.get_backend(),
                                                                      "RCCL" if backend == "nccl" else backend))
    else:
        torch.cuda.set_device(0)
    return dist, backend


def phase_child(args, phase, rank, local, world):
    """A phase's rank process (started by ``orchestrate``): its legs, then rank 0 prints the fragment."""
    consumer = start_consumer() if (phase == "extras" and args.worker_moves > 0 and args.net == "hip") else None
    dist, backend = init_dist(args, rank, local, world)
    frag = run_phase(phase, args, rank, world, dist, backend, consumer)
    if rank == 0:
        print(PHASE_MARK + json.dumps(frag), flush=True)
    if dist:
        dist.destroy_process_group()


def _parse_fragment(text):
    for line in reversed((text or "").splitlines()):
        if line.startswith(PHASE_MARK):
            return json.loads(line[len(PHASE_MARK):])
    return None


MIN_PHASE_S = 15.0  # a later phase with less of the deadline left is skipped, not started


def orchestrate(args, argv, rank, world, script=None):
    """N > 1: this rank process never touches the GPU.  Every phase runs as a FRESH set of rank processes
    (one per rank, a process group of their own on a new port) under a wall-time cap, so a failure or hang
    in one phase - the trainer's first multi-rank RCCL all-reduce, say - cannot take the headline with it.
    The rank processes talk over a CPU (gloo) group: the phase ports, and each phase's exit status (a rank
    whose phase process failed raises a flag in the group's store, and its peers stop theirs at once instead
    of waiting for their collectives to time out).  Rank 0 assembles the ONE line: the selfplay phase's
    fragment, then each later phase's, or {"error": ...} in the keys of a phase that failed or timed out."""
    import datetime
    import torch.distributed as dist
    t_start = time.time()
    caps = phase_plan(args)
    store = None
    if world > 1:
        dist.init_process_group("gloo", init_method="env://",
                                timeout=datetime.timedelta(seconds=max(c for _, c in caps) + 300))
        try:
            from torch.distributed import distributed_c10d as c10d
            store = c10d._get_default_store()
        except Exception:
            store = None
        box = [[_free_port() for _ in caps] if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        ports = box[0]
    else:  # --isolate on with one GPU: the phases run one after the other as single processes
        ports = [None for _ in caps]
    out, phases = None, {}
    # what the deadline leaves after the phases: the per-phase status exchange and the line (+ the CPU baseline
    # sample with one rank)
    reserve = 10.0 + ((args.cpu_baseline_sec + 15.0) if (world == 1 and not args.no_cpu_baseline) else 0.0)
    for (name, cap), port in zip(caps, ports):
        left = None
        if args.deadline > 0:  # rank 0's clock decides every rank's cap (the ranks' phase processes must agree)
            left = args.deadline - (time.time() - t_start) - reserve
            if name == "selfplay":
                left = max(left, 60.0)
            if world > 1:
                box = [left]
                dist.broadcast_object_list(box, src=0)
                left = box[0]
            cap = min(cap, left)
        if left is not None and left < MIN_PHASE_S:  # too little of the deadline left: skipped, its keys say so
            every = [{"status": "skipped: %.0f s of the %.0f s deadline left" % (max(left, 0.0), args.deadline),
                      "seconds": 0.0}] * world
            if rank == 0:
                phases[name] = {"ranks": every, "cap_s": 0.0}
                log("phase %s: skipped (deadline)" % name)
                err = {"error": "phase %s skipped: %s" % (name, every[0]["status"]), "n_gpus": world}
                for k in phase_keys(name, args):
                    out[k] = err
            continue
        env = dict(os.environ, **{PHASE_ENV: name})
        if port is not None:
            env["MASTER_PORT"] = str(port)
        env.pop("TORCHELASTIC_USE_AGENT_STORE", None)  # the phase group hosts its own store
        if out is not None and out.get("value"):
            env["GMZ_BENCH_HEADLINE_VALUE"] = repr(out["value"])
        t0 = time.time()
        # its own session: a kill takes the phase's helper processes (the worker leg's queue consumer) with it
        p = subprocess.Popen([sys.executable, "-u", script or os.path.abspath(__file__)] + list(argv), env=env,
                             stdout=subprocess.PIPE, text=True, start_new_session=True)
        flag = "gmz_phase_failed/%s" % name
        status, text = None, ""
        import threading
        buf = []
        reader = threading.Thread(target=lambda: buf.append(p.stdout.read()), daemon=True)
        reader.start()
        while True:
            code = p.poll()
            if code is not None:
                status = "ok" if code == 0 else "exit %d" % code
                break
            if time.time() - t0 > cap:
                status = "timeout after %d s" % cap
                break
            if store is not None:
                try:
                    if store.check([flag]):
                        status = "stopped: another rank's %s phase failed" % name
                        break
                except Exception:
                    pass
            time.sleep(0.25)
        if p.poll() is None:
            import signal
            try:
                os.killpg(p.pid, signal.SIGKILL)  # the process group this phase started (its own session)
            except ProcessLookupError:
                pass
            p.wait()
        reader.join(timeout=30)
        text = buf[0] if buf else ""
        if status != "ok" and store is not None and not status.startswith("stopped"):
            try:
                store.set(flag, "1")
            except Exception:
                pass
        every = [None] * world
        mine = {"status": status, "seconds": round(time.time() - t0, 1)}
        if world > 1:
            dist.all_gather_object(every, mine)
        else:
            every = [mine]
        if rank == 0:
            frag = _parse_fragment(text)
            failed = [i for i, e in enumerate(every) if e["status"] != "ok"]
            phases[name] = {"ranks": every, "cap_s": round(cap, 1)}
            log("phase %s: %s" % (name, ", ".join("rank %d %s (%.1f s)" % (i, e["status"], e["seconds"])
                                                  for i, e in enumerate(every))))
            if name == "selfplay":
                if frag is None or failed:
                    out = {"metric": "self-play moves/sec (15x15, 400 sims)", "value": None, "unit": "moves/s",
                           "n_gpus": world, "higher_is_better": True,
                           "error": "headline phase failed: %s" % "; ".join(
                               "rank %d %s" % (i, every[i]["status"]) for i in failed) if failed else
                           "headline phase printed no result"}
                else:
                    out = frag
            else:
                if frag is not None and not failed:
                    out.update(frag)
                else:
                    err = {"error": "phase %s failed: %s" % (name, "; ".join(
                        "rank %d %s" % (i, every[i]["status"]) for i in failed) or "no result"), "n_gpus": world}
                    for k in phase_keys(name, args):  # rank 0's numbers, if any, kept but flagged
                        out[k] = dict((frag or {}).get(k) or {}, **err)
    if rank == 0:
        out["phases"] = {"isolated": True, "detail": phases, "deadline_s": args.deadline,
                         "seconds": round(time.time() - t_start, 1),
                         "note": "each phase ran as fresh rank processes with a wall-time cap (bench.orchestrate), "
                                 "the caps shrunk to what the deadline left"}
        if world == 1 and not args.no_cpu_baseline and args.net == "hip":
            log("cpu baseline (bounded sample ~%.0f s)..." % args.cpu_baseline_sec)
            out["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0 if (rank != 0 or out.get("value")) else 1


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # no external launcher: one process per GPU, started here before any GPU call
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(env_world or "1")
    if world != args.gpus:
        log("bench.py: --gpus %d disagrees with WORLD_SIZE=%d" % (args.gpus, world))
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    args.headline_value = float(os.environ.get("GMZ_BENCH_HEADLINE_VALUE", "0")) or None
    phase = os.environ.get(PHASE_ENV)
    if phase:  # a phase's rank process
        phase_child(args, phase, rank, local, world)
        return
    isolate = args.isolate == "on" or (args.isolate == "auto" and world > 1)
    if isolate:
        rc = orchestrate(args, sys.argv[1:], rank, world)
        sys.exit(rc)
    # one process (the N = 1 default): every phase in this process, in order; a later phase's failure is
    # recorded in its keys and does not lose the headline
    consumer = start_consumer() if (args.worker_moves > 0 and args.net == "hip") else None
    dist, backend = init_dist(args, rank, local, world)
    out = None
    for name, _ in phase_plan(args):
        if name == "selfplay":
            out = run_phase(name, args, rank, world, dist, backend)
            continue
        try:
            out.update(run_phase(name, args, rank, world, dist, backend, consumer, out))
        except Exception as ex:  # noqa: BLE001 - recorded in the line; the headline is already measured
            import traceback
            traceback.print_exc()
            for k in phase_keys(name, args):
                out.setdefault(k, {"error": "phase %s failed: %r" % (name, ex), "n_gpus": world})
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.net == "hip":
        log("cpu baseline (bounded sample ~%.0f s)..." % args.cpu_baseline_sec)
        out["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
