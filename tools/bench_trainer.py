"""Trainer throughput (B = 360 per GPU, 5 unroll steps, 15x15, 8 blocks):
training steps/s of datou-gomoku-muzero_amd/trainer.py on synthetic slices resident in a device
ReplayBuffer (uniform sampling, the reference default; --per for PER).  N>1: launch with
torch.distributed.run; each rank samples its own batch, gradients are averaged by one RCCL
all-reduce per step; the line reports steps/s of the job (all ranks step together) and samples/s.

  python tools/bench_trainer.py [--steps 20 --warmup 3 --batch 360 --per]"""
import argparse
import json
import os
import sys
import time
from collections import namedtuple

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--batch", type=int, default=360)
ap.add_argument("--size", type=int, default=15)
ap.add_argument("--blocks", type=int, default=8)
ap.add_argument("--buffer", type=int, default=20000)
ap.add_argument("--per", action="store_true")
ap.add_argument("--no-amp", action="store_true")
ap.add_argument("--bf16", action="store_true", help="autocast to bfloat16 instead of the reference's float16")
ap.add_argument("--nchw", action="store_true", help="NCHW activations (default: channels-last, MIOpen's NHWC kernels)")
ap.add_argument("--sync-logs", action="store_true", help="read each step's losses on the host before the next step")
ap.add_argument("--eager", action="store_true", help="no HIP-graph capture of the step")
ap.add_argument("--miopen-wgrad", action="store_true", help="3x3 weight gradients on MIOpen (trainer.HIP_WGRAD off)")
ap.add_argument("--sequential-forward", action="store_true", help="no side streams in the forward (trainer.CONCURRENT_FORWARD off)")
ap.add_argument("--nchw-flatten", action="store_true", help="K = 28,800 Linears on an NCHW copy of the hidden state (trainer.FLAT_NHWC off)")
ap.add_argument("--no-res-fold", action="store_true", help="autograd sums the residual blocks' input gradients (trainer.FUSED_RES_GRAD off)")
ap.add_argument("--no-defer-wgrad", action="store_true", help="3x3 weight gradients at each use (trainer.DEFER_WGRAD off)")
ap.add_argument("--target-f32", action="store_true", help="the target network's value in float32 on MIOpen (trainer.TARGET_F16 off)")
ap.add_argument("--per-step-loss", action="store_true", help="loss terms per unroll step (trainer.BATCHED_LOSS off)")
ap.add_argument("--relu-mask", action="store_true", help="BatchNorm backward reads 1-bit ReLU masks (trainer.RELU_MASK on)")
ap.add_argument("--hip-stem", action="store_true",
                help="the dynamics trunk's 144-channel first conv on the HIP conv + action stamp (trainer.DYN_STEM_HIP on)")
ap.add_argument("--per-step-consistency", action="store_true",
                help="five consistency representations, one per unroll step (trainer.BATCHED_CONSISTENCY off)")
ap.add_argument("--per-step-heads", action="store_true",
                help="prediction / reward / projection heads once per unroll step (trainer.BATCHED_HEADS off)")
ap.add_argument("--torch-head-convs", action="store_true",
                help="the prediction heads' 1x1 convs on PyTorch GEMMs (trainer.FUSED_HEADS off)")
ap.add_argument("--torch-seg-bn", action="store_true",
                help="the batched heads' segmented BatchNorms in PyTorch ops (trainer.SEG_BN_HIP off)")
ap.add_argument("--op-sources", type=int, default=0, metavar="N",
                help="with --eager: profile one more step and print the N trainer.py lines launching the most PyTorch kernels")
ap.add_argument("--bn-bwd-stats", action="store_true",
                help="BatchNorm backward sums in the input-gradient conv's epilogue (trainer.FUSED_BN_BWD_STATS on)")
ap.add_argument("--torch-small-bn", action="store_true",
                help="the 1- and 2-channel heads' segmented BatchNorms on PyTorch (trainer.SEG_BN_SMALL off)")
ap.add_argument("--no-batch-repack", action="store_true",
                help="each packed conv weight re-packed at its first use, one launch each (trainer.BATCH_REPACK off)")
ap.add_argument("--torch-opt", action="store_true",
                help="PyTorch's unscale_ / clip_grad_norm_ / fused Adam / foreach soft update (trainer.FUSED_OPT off)")
ap.add_argument("--no-defer-bn", action="store_true",
                help="BatchNorm outputs written by their own pass, not the consuming conv's prologue (trainer.DEFER_BN_APPLY off)")
ap.add_argument("--no-benchmark", action="store_true", help="no torch.backends.cudnn.benchmark (MIOpen Find per shape)")
a = ap.parse_args()
a.channels_last, a.benchmark = not a.nchw, not a.no_benchmark
torch.backends.cudnn.benchmark = a.benchmark

world = int(os.environ.get("WORLD_SIZE", "1"))
rank = int(os.environ.get("RANK", "0"))
local = int(os.environ.get("LOCAL_RANK", "0"))
torch.cuda.set_device(local % torch.cuda.device_count())
dist = None
if world > 1:
    import torch.distributed as dist
    dist.init_process_group(os.environ.get("GMZ_DIST_BACKEND", "nccl"), init_method="env://")
from datou_gomoku_muzero_amd import trainer as T  # noqa: E402

T.HIP_WGRAD = T.HIP_WGRAD and not a.miopen_wgrad
T.CONCURRENT_FORWARD = T.CONCURRENT_FORWARD and not a.sequential_forward
T.FLAT_NHWC = T.FLAT_NHWC and not a.nchw_flatten
T.FUSED_RES_GRAD = T.FUSED_RES_GRAD and not a.no_res_fold
T.BATCHED_LOSS = T.BATCHED_LOSS and not a.per_step_loss
T.BATCHED_CONSISTENCY = T.BATCHED_CONSISTENCY and not a.per_step_consistency
T.BATCHED_HEADS = T.BATCHED_HEADS and not a.per_step_heads
T.FUSED_HEADS = T.FUSED_HEADS and not a.torch_head_convs
T.SEG_BN_HIP = T.SEG_BN_HIP and not a.torch_seg_bn
T.DYN_STEM_HIP = T.DYN_STEM_HIP or a.hip_stem
T.RELU_MASK = T.RELU_MASK or a.relu_mask
T.TARGET_F16 = T.TARGET_F16 and not a.target_f32
T.DEFER_WGRAD = T.DEFER_WGRAD and not a.no_defer_wgrad
T.DEFER_BN_APPLY = T.DEFER_BN_APPLY and not a.no_defer_bn
T.FUSED_OPT = T.FUSED_OPT and not a.torch_opt
T.SEG_BN_SMALL = T.SEG_BN_SMALL and not a.torch_small_bn
T.BATCH_REPACK = T.BATCH_REPACK and not a.no_batch_repack
T.FUSED_BN_BWD_STATS = T.FUSED_BN_BWD_STATS or a.bn_bwd_stats

cfg = T.TrainConfig(BOARD_SIZE=a.size, NUM_RES_BLOCKS=a.blocks, PHYSICAL_BATCH_SIZE=a.batch,
                    TRAIN_BUFFER_SIZE=a.buffer, ENABLE_PER=a.per)
tr = T.Trainer(cfg, device="cuda", amp=not a.no_amp, amp_dtype=torch.bfloat16 if a.bf16 else None,
               channels_last=a.channels_last, graph=not a.eager)
rb = T.ReplayBuffer(cfg, device="cuda")
S = namedtuple("S", "observation action_history reward_history policy_history value_history")
rs = np.random.RandomState(rank)
U, A = cfg.NUM_UNROLL_STEPS, a.size * a.size
chunk = []
for i in range(a.buffer):
    ends = rs.randint(1, U + 1)
    act = rs.randint(0, A, U).astype(np.int32)
    act[ends:] = -1
    chunk.append(S((rs.rand(U + 1, 3, a.size, a.size) < 0.2).astype(np.uint8), act,
                   rs.choice([-1.0, 0.0, 1.0], U).astype(np.float32),
                   rs.dirichlet(np.ones(A), U + 1).astype(np.float32), rs.uniform(-1, 1, U + 1).astype(np.float32)))
    if len(chunk) == 2000:
        rb.add(chunk)
        chunk = []
rb.add(chunk)


pending = [None]


def step():
    """One step; its five losses reach the host one step later (read after the next step is queued,
    so the GPU never waits for the host's sampling and launch work).  --sync-logs: read every
    step's losses before the next step, like the reference's calculate_loss .item() calls."""
    batch, idx, w = rb.sample(a.batch, rs)
    logs, td = tr.step(batch, w, sync=a.sync_logs)
    rb.update_priorities(idx, td)
    if a.sync_logs:
        return logs
    prev, pending[0] = pending[0], logs
    return tuple(prev.tolist()) if prev is not None else None


def drain():
    return tuple(pending[0].tolist()) if pending[0] is not None else None


for _ in range(a.warmup):
    step()
if dist:
    dist.barrier()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.steps):
    logs = step()
logs = drain() or logs
torch.cuda.synchronize()
if dist:
    dist.barrier()
dt = time.perf_counter() - t0
if dist:
    t = torch.tensor([dt], device="cuda" if os.environ.get("GMZ_DIST_BACKEND", "nccl") == "nccl" else "cpu",
                     dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
if rank == 0:
    print(json.dumps({"metric": "trainer steps/sec (config C4)", "value": a.steps / dt, "unit": "steps/s",
                      "n_gpus": world, "samples_per_s": a.steps * a.batch * world / dt, "ms_per_step": dt / a.steps * 1e3,
                      "batch_per_gpu": a.batch, "unroll": U, "board": a.size, "blocks": a.blocks, "amp": ("bf16" if a.bf16 else "fp16") if not a.no_amp else None, "channels_last": a.channels_last, "benchmark": a.benchmark, "graph": tr.graph,
                      "per": a.per, "sync_logs": a.sync_logs, "last_loss": logs[0], "data": "synthetic slices in a device ReplayBuffer",
                      "max_memory_allocated_gb": torch.cuda.max_memory_allocated() / 2 ** 30,
                      "defer_wgrad": T.DEFER_WGRAD, "batched_heads": T.BATCHED_HEADS, "fused_heads": T.FUSED_HEADS,
                      "dyn_stem_hip": T.DYN_STEM_HIP, "relu_mask": T.RELU_MASK,
                      "seg_bn_hip": T.SEG_BN_HIP}))
if a.op_sources and rank == 0:
    # which trainer.py lines launch PyTorch's kernels (the libgmz launches have no aten op and are not counted)
    from collections import Counter
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    per_line, per_kernel = Counter(), Counter()
    for ev in prof.events():
        ks = getattr(ev, "kernels", None) or []
        if not ks:
            continue
        # the kernels hang on the innermost aten op; the Python stack is on its outermost ancestor, and the
        # backward's ops sit under the autograd node that ran them
        fr, up = None, ev
        while up is not None:
            if up.name.startswith("autograd::engine::evaluate_function"):
                fr = up.name.split(": ", 1)[-1]
                break
            if up.stack:
                fr = next((f for f in up.stack if "trainer.py" in f), up.stack[0])
                break
            up = up.cpu_parent
        per_line[(fr or "?", ev.name)] += len(ks)
        for k in ks:
            per_kernel[k.name[:60]] += 1
    print("op-sources: %d PyTorch kernels in one eager step" % sum(per_line.values()))
    # the same step under a dispatch mode: every aten op by the trainer.py line that issued it (forward, and the
    # custom Functions' backward bodies; built-in backward nodes show as "<autograd>")
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode

    class _Lines(TorchDispatchMode):
        def __init__(self):
            super().__init__()
            self.n = Counter()

        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            out = func(*args, **(kwargs or {}))
            dev = any(isinstance(t, torch.Tensor) and t.is_cuda for t in torch.utils._pytree.tree_leaves((args, kwargs, out)))
            if dev and func.__name__ not in ("view.default", "_unsafe_view.default", "t.default", "detach.default",
                                             "as_strided.default", "permute.default", "expand.default",
                                             "slice.Tensor", "select.int", "unsqueeze.default", "squeeze.dim",
                                             "transpose.int", "reshape.default", "empty.memory_format",
                                             "empty_strided.default", "alias.default", "unbind.int", "split.Tensor",
                                             "split_with_sizes.default", "chunk.default", "narrow.default",
                                             "_reshape_alias.default", "view_as.default", "empty_like.default",
                                             "new_empty.default", "new_empty_strided.default", "is_same_size.default",
                                             "set_.source_Storage_storage_offset", "_local_scalar_dense.default",
                                             "squeeze.default", "diagonal.default", "view.dtype", "unflatten.int", "flatten.using_ints"):
                fr = [f for f in traceback.extract_stack() if os.path.basename(f.filename) == "trainer.py"]
                key = "%s:%d %s" % ("trainer.py", fr[-1].lineno, fr[-1].name) if fr else "<autograd>"
                self.n[(key, func.__name__)] += 1
            return out

    m = _Lines()
    with m:
        step()
        torch.cuda.synchronize()
    print("dispatch: %d device aten ops (not view-like) in one eager step" % sum(m.n.values()))
    for (fr, name), n in m.n.most_common(a.op_sources):
        print("%5d  %-40s %s" % (n, name, fr))
    for (fr, name), n in per_line.most_common(a.op_sources):
        print("%5d  %-28s %s" % (n, name, fr))
    for k, n in per_kernel.most_common(20):
        print("%5d  %s" % (n, k))
if dist:
    dist.destroy_process_group()
