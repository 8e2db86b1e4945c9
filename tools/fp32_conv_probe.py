"""The target network's float32 3x3 convs (loss.py:54-55, no autocast): MIOpen per layout at the
trainer's shape (360 boards, 15x15, 128 -> 128), with and without Find (benchmark).
  python tools/fp32_conv_probe.py"""
import torch

N, H = 360, 15
for bench in (True, False):
    torch.backends.cudnn.benchmark = bench
    for fmt in ("nchw", "nhwc"):
        mf = torch.channels_last if fmt == "nhwc" else torch.contiguous_format
        x = torch.randn(N, 128, H, H, device="cuda").contiguous(memory_format=mf)
        w = (torch.randn(128, 128, 3, 3, device="cuda") / 34).contiguous(memory_format=mf)
        with torch.no_grad():
            for _ in range(5):
                torch.nn.functional.conv2d(x, w, padding=1)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(30):
                torch.nn.functional.conv2d(x, w, padding=1)
            e.record()
            torch.cuda.synchronize()
        us = s.elapsed_time(e) / 30 * 1e3
        print("benchmark=%-5s %s  %7.1f us  %6.1f TFLOP/s" % (bench, fmt, us, 2 * N * H * H * 128 * 128 * 9 / us / 1e6))
