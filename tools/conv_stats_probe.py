"""Where the trainer conv's epilogue statistics cost goes: k_conv3 at N boards, HxH, f16, per launch (HIP events):
no statistics, statistics without a row mask, statistics with a row mask.  python tools/conv_stats_probe.py [N] [H]"""
import sys

import torch

sys.path.insert(0, ".")
from datou_gomoku_muzero_amd import _lib, trainer as T  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 360
H = int(sys.argv[2]) if len(sys.argv) > 2 else 15
L = _lib.load()
x = torch.randn(N, 128, H, H, device="cuda").half().contiguous(memory_format=torch.channels_last)
pk = T._packed_conv_weight(torch.randn(128, 128, 3, 3, device="cuda") / 34, torch.float16, 0)
y = torch.empty_like(x)
mask = torch.ones(N, dtype=torch.uint8, device="cuda")
st, ns = T._conv_stats_buffer(N, x.device)


def run(m, s):
    _lib.check(L.gmz_conv3x3_forward_stats(1, H, _lib.ptr(x), _lib.ptr(pk), _lib.ptr(y), N, _lib.ptr(m), _lib.ptr(s),
                                           ns if s is not None else 0, _lib.stream_ptr()))


def tm(fn, n=50):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


for r in range(2):
    print("N=%d H=%d  no stats %.2f us | stats, no mask %.2f us | stats + mask %.2f us | mask, no stats %.2f us" % (
        N, H, tm(lambda: run(None, None)), tm(lambda: run(None, st)), tm(lambda: run(mask, st)), tm(lambda: run(mask, None))))
