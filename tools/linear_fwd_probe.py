"""Probe formulations of the trainer's big-K Linear forwards (projection fc1 28800->512, reward
fc 28800->64 at B = 360, fp16): hipBLASLt's pick for x @ W^T uses 24 workgroups."""
import torch
dev = "cuda"


def t(fn, n=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


for B, K, N in ((360, 28800, 512), (360, 28800, 64)):
    x = torch.randn(B, K, device=dev, dtype=torch.float16)
    w = torch.randn(N, K, device=dev, dtype=torch.float16) / 170
    ref = (x.float() @ w.float().t())
    fl = 2 * B * K * N
    r = {}
    r["x@wT"] = (t(lambda: x @ w.t()), x @ w.t())
    r["(w@xT).T"] = (t(lambda: (w @ x.t()).t()), (w @ x.t()).t())
    wt = w.t().contiguous()
    r["x@wTc"] = (t(lambda: x @ wt), x @ wt)
    for S in (8, 16, 32):
        xs = x.view(B, S, K // S).transpose(0, 1)
        ws = w.view(N, S, K // S).permute(1, 2, 0)
        r["splitK%d f16" % S] = (t(lambda: torch.bmm(xs, ws).sum(0, dtype=torch.float32)), torch.bmm(xs, ws).sum(0, dtype=torch.float32))
        try:
            r["splitK%d f32out" % S] = (t(lambda: torch.bmm(xs, ws, out_dtype=torch.float32).sum(0)), torch.bmm(xs, ws, out_dtype=torch.float32).sum(0))
        except Exception as ex:
            print("out_dtype unsupported:", str(ex)[:80])
    for k, (us, y) in r.items():
        err = float((y.float() - ref).abs().max() / ref.abs().max())
        print("%d %d %d %-16s %7.1f us %5.0f TF  err %.2e" % (B, K, N, k, us, fl / us / 1e6, err), flush=True)
