"""The trainer's HIP conv (k_conv3) alone, for PMC passes and A/B builds: forward (no statistics), forward with
the masked BatchNorm statistics epilogue, and the input gradient, at N boards of HxH.
  python tools/conv_probe.py [N] [H] [launches]   (GMZ_LIB selects an A/B build)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from datou_gomoku_muzero_amd import trainer as T  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 360
H = int(sys.argv[2]) if len(sys.argv) > 2 else 15
K = int(sys.argv[3]) if len(sys.argv) > 3 else 40
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(N, 128, H, H, device="cuda", generator=g).half().contiguous(memory_format=torch.channels_last)
w = (torch.randn(128, 128, 3, 3, device="cuda", generator=g) / 34).contiguous(memory_format=torch.channels_last)
pk, pkt = T._packed_conv_weight(w, torch.float16, 0), T._packed_conv_weight(w, torch.float16, 1)
mask = torch.ones(N, dtype=torch.uint8, device="cuda")
st, _ = T._conv_stats_buffer(N, x.device)
fl = 2.0 * N * H * H * 128 * 128 * 9


def tm(fn):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(K):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / K * 1e3


res = {"fwd": tm(lambda: T._conv3x3_hip(x, pk)),
       "fwd+stats": tm(lambda: T._conv3x3_hip(x, pk, mask=mask, stats=st)),
       "dgrad": tm(lambda: T._conv3x3_hip(x, pkt))}
y = T._conv3x3_hip(x, pk).float()
yr = torch.nn.functional.conv2d(x.float(), w.half().float(), padding=1)
err = float((y - yr).abs().max() / yr.abs().max())
print("lib=%s N=%d H=%d rel err %.2e" % (os.path.basename(os.environ.get("GMZ_LIB", "libgmz.so")), N, H, err))
for k, v in res.items():
    print("%-10s %8.2f us  %6.0f TFLOP/s" % (k, v, fl / v / 1e6))
