"""Achievable peaks on this GPU (SURVEY §8d 'Peak references'): HBM copy bandwidth (device-to-device
copy of a 4 GiB buffer, read + write bytes) and dense bf16 GEMM throughput (torch.matmul ->
hipBLASLt, 8192^3 and 16384^3), so the tower's roofline fraction can be read against both the vendor
peaks (8 TB/s, 2.5 PF) and what the chip delivers here."""
import json
import sys
import time

import torch


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


out = {}
n = 4 << 30
a = torch.empty(n, dtype=torch.uint8, device="cuda")
b = torch.empty_like(a)
t = timed(lambda: b.copy_(a), 10)
out["hbm_copy_GBs"] = 2 * n / t / 1e9
del a, b
for m in (8192, 16384):
    x = torch.randn(m, m, dtype=torch.bfloat16, device="cuda")
    y = torch.randn(m, m, dtype=torch.bfloat16, device="cuda")
    t = timed(lambda: torch.matmul(x, y), 10 if m == 8192 else 4)
    out["bf16_gemm_%d_TFLOPs" % m] = 2 * m ** 3 / t / 1e12
    del x, y
print(json.dumps(out))
if len(sys.argv) > 1:
    json.dump(out, open(sys.argv[1], "w"), indent=1)
