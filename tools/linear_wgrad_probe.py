"""Probe formulations of the big-K-small-batch Linear weight gradients of the trainer
(projection fc1 28800->512 and reward fc 28800->64 at B = 360, fp16): hipBLASLt picks 16x16
tiles for dW = dY^T X (K = 360) and runs at ~14 TFLOP/s."""
import torch, time
torch.manual_seed(0)
dev = "cuda"
def t(fn, n=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n): fn()
    e.record(); torch.cuda.synchronize(); return s.elapsed_time(e) / n * 1e3
for B, K, N in ((360, 28800, 512), (360, 28800, 64), (360, 450, 225), (360, 225, 64)):
    for dt in (torch.float16, torch.bfloat16):
        x = torch.randn(B, K, device=dev, dtype=dt); dy = torch.randn(B, N, device=dev, dtype=dt)
        w = torch.randn(N, K, device=dev, dtype=dt)
        fl = 2 * B * K * N
        r = {}
        r["fwd x@wT"] = t(lambda: x @ w.t())
        r["dgrad dy@w"] = t(lambda: dy @ w)
        r["wgrad dyT@x"] = t(lambda: dy.t() @ x)
        r["wgrad (xT@dy).T"] = t(lambda: (x.t() @ dy).t())
        xt = x.t().contiguous(); dyt = dy.t().contiguous()
        r["wgrad dyTc@x"] = t(lambda: dyt @ x)
        r["wgrad contig(x.T) "] = t(lambda: dy.t() @ x.t().contiguous().t())
        r["wgrad f32 dyT@x"] = t(lambda: dy.float().t() @ x.float())
        print(B, K, N, dt, "  ".join("%s %.1fus(%.0fTF)" % (k, v, fl / v / 1e6) for k, v in r.items()), flush=True)
