"""gmz_conv3x3 vs MIOpen on the trainer's shape (N = 360 boards, 15x15, 128 -> 128, f16 NHWC):
per-launch time (HIP events, 50 launches after warm-up) and TFLOP/s.
  python tools/conv_bench.py [N] [H]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from datou_gomoku_muzero_amd import trainer as T  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 360
H = int(sys.argv[2]) if len(sys.argv) > 2 else 15
torch.backends.cudnn.benchmark = True
x = torch.randn(N, 128, H, H, device="cuda").half().contiguous(memory_format=torch.channels_last)
w = (torch.randn(128, 128, 3, 3, device="cuda") / 34).contiguous(memory_format=torch.channels_last)
wh = w.half()
pk, pkt = T._packed_conv_weight(w, torch.float16, 0), T._packed_conv_weight(w, torch.float16, 1)
fl = 2.0 * N * H * H * 128 * 128 * 9
gacc = torch.zeros_like(w)
# a BatchNorm (+ReLU) whose output fed this conv: dgrad with its backward dz sums in the epilogue
bnb = T._BnBwdLink(x, (torch.rand(N, device="cuda") < 0.7).to(torch.uint8),
                   torch.stack([torch.zeros(128), torch.ones(128)]).cuda(), 1)


def tm(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


res = {
    "hip fwd": tm(lambda: T._conv3x3_hip(x, pk)),
    "hip dgrad": tm(lambda: T._conv3x3_hip(x, pkt)),
    "hip dgrad+bnsums": tm(lambda: T._conv3x3_hip(x, pkt, bnb=bnb, bn_y=x)),
    "miopen fwd": tm(lambda: torch.nn.functional.conv2d(x, wh, padding=1)),
    "miopen dgrad": tm(lambda: torch.ops.aten.convolution_backward(x, x, wh, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False])),
    "miopen wgrad": tm(lambda: torch.ops.aten.convolution_backward(x, x, wh, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False])),
    "pack": tm(lambda: T._packed_conv_weight(w.add_(0), torch.float16, 0)),
    "hip wgrad": tm(lambda: T._conv3x3_wgrad_hip(x, x, gacc)),
}
y = T._conv3x3_hip(x, pk).float()
yr = torch.nn.functional.conv2d(x.float(), wh.float(), padding=1)
err = float((y - yr).abs().max() / yr.abs().max())
gw = torch.zeros_like(w)
T._conv3x3_wgrad_hip(x, x, gw)
gwr = torch.ops.aten.convolution_backward(x.float(), x.float(), wh.float(), None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False])[1]
werr = float((gw - gwr).abs().max() / gwr.abs().max())
print("N=%d H=%d  rel err %.2e  wgrad rel err %.2e" % (N, H, err, werr))
for k, v in res.items():
    print("%-17s %8.1f us  %6.0f TFLOP/s" % (k, v, fl / v / 1e6))
