"""Diagnostics for gmz_conv3x3: per-position error maps of forward and input gradient vs float32."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from datou_gomoku_muzero_amd import trainer as T
for H, N in ((9, 24), (15, 37)):
    g = torch.Generator().manual_seed(H)
    x = torch.randn(N, 128, H, H, generator=g).cuda().half().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(128, 128, 3, 3, generator=g) / 34.0).cuda().contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, 128, H, H, generator=g).cuda().half().contiguous(memory_format=torch.channels_last)
    y = T._conv3x3_hip(x, T._packed_conv_weight(w, torch.float16, 0)).float()
    gx = T._conv3x3_hip(dy, T._packed_conv_weight(w, torch.float16, 1)).float()
    wr = w.half().float()
    yr = torch.nn.functional.conv2d(x.float(), wr, padding=1)
    gxr = torch.nn.grad.conv2d_input(x.shape, wr, dy.float(), padding=1)
    for name, a, b in (("fwd", y, yr), ("dgrad", gx, gxr)):
        e = (a - b).abs()
        rel = e / (b.abs() + 1e-3)
        print(H, name, "max err %.3e  mean err %.3e  max|ref| %.3f  mean rel %.3e" % (e.max(), e.mean(), b.abs().max(), rel.mean()))
        em = e.mean(dim=(0, 1))
        print("  per-position mean err (x1e4):")
        for r in range(H):
            print("   ", " ".join("%4.1f" % (1e4 * float(v)) for v in em[r]))
        ec = e.mean(dim=(0, 2, 3))
        print("  per-channel mean err (x1e4) min %.2f max %.2f argmax %d" % (1e4 * ec.min(), 1e4 * ec.max(), int(ec.argmax())))
        bias = (a - b).mean()
        print("  mean signed err %.3e" % bias)
