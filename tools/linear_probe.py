"""Times the trainer's large-K linear layers (projection fc1 28800->512, reward fc 28800->64 at
B = 360, float16 under autocast) in a few formulations, to pick the fastest hipBLASLt path."""
import time

import torch
import torch.nn.functional as F

torch.manual_seed(0)
dev = "cuda"
B, K = 360, 28800


def bench(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6


for N in (512, 64):
    x = torch.randn(B, K, device=dev, dtype=torch.float16)
    w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.01
    b = torch.randn(N, device=dev, dtype=torch.float16)
    wt = w.t().contiguous()
    dy = torch.randn(B, N, device=dev, dtype=torch.float16)
    fl = 2 * B * N * K
    res = {
        "linear+bias": bench(lambda: F.linear(x, w, b)),
        "linear": bench(lambda: F.linear(x, w)),
        "x@wt (K-major w)": bench(lambda: x @ wt),
        "addmm(b, x, w.t())": bench(lambda: torch.addmm(b, x, w.t())),
        "dgrad dy@w": bench(lambda: dy @ w),
        "wgrad dy.t()@x": bench(lambda: dy.t() @ x),
        "wgrad (x.t()@dy).t()": bench(lambda: (x.t() @ dy)),
    }
    for k, v in res.items():
        print("N=%4d %-24s %8.1f us  %6.1f TFLOP/s" % (N, k, v, fl / v / 1e6))
