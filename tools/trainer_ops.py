"""Op census of one eager trainer step (config C4 shapes): aten ops and GPU kernels by count, with
input shapes, from torch.profiler — to find which small kernels the HIP-graph step is made of.

  python tools/trainer_ops.py [--batch 360] > gpurun_out/trainer_ops.txt"""
import argparse
import os
import sys
from collections import Counter, namedtuple

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=360)
ap.add_argument("--top", type=int, default=60)
a = ap.parse_args()
torch.backends.cudnn.benchmark = True
from datou_gomoku_muzero_amd import trainer as T  # noqa: E402

cfg = T.TrainConfig(BOARD_SIZE=15, NUM_RES_BLOCKS=8, PHYSICAL_BATCH_SIZE=a.batch, TRAIN_BUFFER_SIZE=2000)
tr = T.Trainer(cfg, device="cuda", graph=False)
rb = T.ReplayBuffer(cfg, device="cuda")
S = namedtuple("S", "observation action_history reward_history policy_history value_history")
rs = np.random.RandomState(0)
U, A = cfg.NUM_UNROLL_STEPS, 225
chunk = []
for i in range(2000):
    act = rs.randint(0, A, U).astype(np.int32)
    chunk.append(S((rs.rand(U + 1, 3, 15, 15) < 0.2).astype(np.uint8), act,
                   rs.choice([-1.0, 0.0, 1.0], U).astype(np.float32),
                   rs.dirichlet(np.ones(A), U + 1).astype(np.float32), rs.uniform(-1, 1, U + 1).astype(np.float32)))
rb.add(chunk)
for _ in range(3):
    batch, idx, w = rb.sample(a.batch, rs)
    tr.step(batch, w)
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402

with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    batch, idx, w = rb.sample(a.batch, rs)
    tr.step(batch, w)
    torch.cuda.synchronize()
ops = Counter()
for e in prof.events():
    if e.device_type.name == "CPU" and e.name.startswith("aten::") and not e.cpu_parent:
        ops[(e.name, str(e.input_shapes)[:110])] += 1
kern = Counter()
ktime = Counter()
for e in prof.events():
    if e.device_type.name == "CUDA":
        kern[e.name[:100]] += 1
        ktime[e.name[:100]] += e.device_time
print("kernels per step:", sum(kern.values()), " GPU time (us):", round(sum(ktime.values())))
for k, n in sorted(kern.items(), key=lambda kv: -ktime[kv[0]])[:a.top]:
    print(f"{n:5d} {ktime[k]:9.0f} us  {k}")
print("\ntop-level aten ops by count:")
for (name, shp), n in ops.most_common(a.top):
    print(f"{n:5d}  {name}  {shp}")
print("\nGPU kernels by launching aten op (top-level):")
print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=a.top, max_name_column_width=40,
                                                          max_shapes_column_width=70))

# which ops launch the small elementwise kernels (copies, casts, adds): innermost aten op with its input
# shapes and its outermost ancestor (an autograd node name in the backward, a module op forward)
pat = ("copy", "CUDAFunctor_add", "direct_copy", "float16", "FillFunctor", "type_sp", "reduce_kernel")
who = Counter()
wtime = Counter()
for e in prof.events():
    if e.device_type.name != "CPU":
        continue
    for k in getattr(e, "kernels", []) or []:
        if not any(p in k.name for p in pat):
            continue
        top = e
        while top.cpu_parent is not None:
            top = top.cpu_parent
        key = (k.name[:60], e.name, str(e.input_shapes)[:70], top.name[:60])
        who[key] += 1
        wtime[key] += k.duration
print("\nsmall elementwise kernels by launching op (innermost op, shapes, outermost ancestor):")
for key, n in sorted(who.items(), key=lambda kv: -wtime[kv[0]])[:a.top]:
    print(f"{n:4d} {wtime[key]:8.0f} us  {key[0]:<60} | {key[1]} {key[2]} | {key[3]}")

