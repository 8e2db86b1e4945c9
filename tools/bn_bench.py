"""Masked BatchNorm kernels alone at the trainer's shape (B = 360, C = 128, 15x15, f16 channels-last, 70 % of
the rows live, residual + ReLU): forward (reduce + finalise + apply) and backward (reduce + finalise + apply)
per call, HIP-event timed over many calls on one stream.  Run from a tree's root to time that tree's
libgmz.so (tools/ab_trainer.sh-style A/Bs).
  python tools/bn_bench.py [reps]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from datou_gomoku_muzero_amd import _lib  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
B, C, H = 360, 128, 15
S = H * H
L = _lib.load()
g = torch.Generator(device="cuda").manual_seed(3)
cl = torch.channels_last
x = torch.randn(B, C, H, H, device="cuda", generator=g).half().contiguous(memory_format=cl)
res = torch.randn(B, C, H, H, device="cuda", generator=g).half().contiguous(memory_format=cl)
dy = torch.randn(B, C, H, H, device="cuda", generator=g).half().contiguous(memory_format=cl)
y, dx, dres = torch.empty_like(x), torch.empty_like(x), torch.empty_like(x)
mask = (torch.rand(B, device="cuda", generator=g) < 0.7).to(torch.uint8)
gamma = torch.rand(C, device="cuda", generator=g) + 0.5
beta = torch.randn(C, device="cuda", generator=g)
rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
nb = torch.zeros(1, dtype=torch.int64, device="cuda")
save = torch.empty(2, C, device="cuda")
dg, db = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
nbytes = __import__("ctypes").c_size_t()
_lib.check(L.gmz_bn_workspace_bytes(1, B, C, S, __import__("ctypes").byref(nbytes)))
ws = torch.empty(nbytes.value, dtype=torch.uint8, device="cuda")
P = _lib.ptr


def fwd():
    _lib.check(L.gmz_bn_forward(1, 1, P(x), P(res), P(mask), B, C, S, P(gamma), P(beta), 1e-4, 0.1, P(rm), P(rv), P(nb),
                                1, P(y), P(save), P(ws), _lib.nbytes(ws), _lib.stream_ptr()))


def bwd():
    _lib.check(L.gmz_bn_backward_acc(1, 1, P(x), P(y), P(dy), P(mask), B, C, S, P(gamma), P(save), 1, P(dx), P(dres),
                                     P(dg), P(db), P(ws), _lib.nbytes(ws), _lib.stream_ptr(), 1))


def timed(fn):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


out = {"forward_us": timed(fwd), "backward_us": timed(bwd), "reps": reps}
if hasattr(L, "gmz_bn_backward_stats"):  # ABI 7: the dz sums already reduced (by the conv epilogue)
    ns = 360  # gmz_conv3x3_stats_slots(360)
    stats = torch.rand(C * ns * 3, dtype=torch.float64, device="cuda")

    def bwd_stats():
        _lib.check(L.gmz_bn_backward_stats(1, P(x), P(y), P(dy), P(mask), B, C, S, P(gamma), P(save), 1, P(dx), P(dres),
                                           P(dg), P(db), P(stats), ns, _lib.nbytes(stats), P(ws),
                                           _lib.nbytes(ws), _lib.stream_ptr(), 1))
    out["backward_given_sums_us"] = timed(bwd_stats)
print(json.dumps(out))
