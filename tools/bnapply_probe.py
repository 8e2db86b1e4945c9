"""Deferred BatchNorm apply (gmz_conv3x3_forward_bnapply) vs BatchNorm pass + conv, at the trainer's shape:
per-launch times with HIP events.  python tools/bnapply_probe.py [N] [H]"""
import sys

import torch

sys.path.insert(0, ".")
from datou_gomoku_muzero_amd import _lib, trainer as T  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 360
H = int(sys.argv[2]) if len(sys.argv) > 2 else 15
L = _lib.load()
cl = dict(memory_format=torch.channels_last)
z = torch.randn(N, 128, H, H, device="cuda").half().contiguous(**cl)
r = torch.randn(N, 128, H, H, device="cuda").half().contiguous(**cl)
gamma, beta = torch.rand(128, device="cuda") + 0.5, torch.randn(128, device="cuda") * 0.1
packed = T._packed_conv_weight(torch.randn(128, 128, 3, 3, device="cuda") / 34, torch.float16, 0)
st, ns = T._conv_stats_buffer(N, z.device)
st2, _ = T._conv_stats_buffer(N, z.device)
_lib.check(L.gmz_conv3x3_forward_stats(1, H, _lib.ptr(r), _lib.ptr(packed), _lib.ptr(z), N, None, _lib.ptr(st), ns,
                                       _lib.stream_ptr()))
rm, rv = torch.zeros(128, device="cuda"), torch.ones(128, device="cuda")
nb = torch.zeros(1, dtype=torch.int64, device="cuda")
save = torch.empty(2, 128, device="cuda")
y, out = torch.empty_like(z), torch.empty_like(z)
S = _lib.stream_ptr


def bn_pass(res):
    _lib.check(L.gmz_bn_forward_stats(1, _lib.ptr(z), _lib.ptr(res), N, 128, H * H, _lib.ptr(gamma), _lib.ptr(beta), 1e-4,
                                      0.1, _lib.ptr(rm), _lib.ptr(rv), _lib.ptr(nb), 1, _lib.ptr(y), _lib.ptr(save),
                                      _lib.ptr(st), ns, _lib.nbytes(st), S()))


def conv():
    _lib.check(L.gmz_conv3x3_forward_stats(1, H, _lib.ptr(y), _lib.ptr(packed), _lib.ptr(out), N, None, _lib.ptr(st2), ns,
                                           S()))


def deferred():
    _lib.check(L.gmz_bn_forward_deferred(1, _lib.ptr(z), None, N, 128, H * H, 1e-4, 0.1, _lib.ptr(rm), _lib.ptr(rv),
                                         _lib.ptr(nb), _lib.ptr(save), _lib.ptr(st), ns, _lib.nbytes(st), None, 0, S()))


def bnapply(res):
    _lib.check(L.gmz_conv3x3_forward_bnapply(1, H, _lib.ptr(z), _lib.ptr(res), _lib.ptr(gamma), _lib.ptr(beta),
                                             _lib.ptr(save), 1, _lib.ptr(y), _lib.ptr(packed), _lib.ptr(out), N, None,
                                             _lib.ptr(st2), ns, S()))


def timed(f, n=50):
    for _ in range(5):
        f()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


for res in (None, r):
    tag = "res" if res is not None else "nores"
    t_bn, t_conv = timed(lambda: bn_pass(res)), timed(conv)
    t_pair = timed(lambda: (bn_pass(res), conv()))
    t_def, t_bna = timed(deferred), timed(lambda: bnapply(res))
    t_new = timed(lambda: (deferred(), bnapply(res)))
    print("N=%d H=%d %-5s  bn pass %.1f us + conv %.1f us = pair %.1f us  |  finalize %.1f us + bnapply conv %.1f us = "
          "%.1f us" % (N, H, tag, t_bn, t_conv, t_pair, t_def, t_bna, t_new))
