"""Weight-gradient variants of the channels-last K = 28,800 Linear (trainer._BigKLinear perm path):
time per call of each way to land dW in the f32 .grad in W's (c, p) column order.
  python tools/bigk_wgrad_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

n, O, C, HW = 360, 512, 128, 225
K = C * HW
xs = torch.randn(n, K, device="cuda").half()
gy = torch.randn(n, O, device="cuda").half()
g = torch.zeros(O, K, device="cuda")


def v_xtdy_strided():
    gwt = xs.t() @ gy
    g.view(O, C, HW).add_(gwt.view(HW, C, O).permute(2, 1, 0))


def v_dytx_rowtranspose():
    gwp = gy.t() @ xs
    g.view(O, C, HW).add_(gwp.view(O, HW, C).transpose(1, 2))


def v_xtdy_then_rowtranspose():
    gwt = xs.t() @ gy
    gwp = gwt.t().contiguous()
    g.view(O, C, HW).add_(gwp.view(O, HW, C).transpose(1, 2))


def v_hip_grad_add_t():  # the product path: x^T dy, then gmz_grad_add_t (LDS-tiled transpose-add)
    from datou_gomoku_muzero_amd import _lib
    gwt = xs.t() @ gy
    _lib.check(_lib.load().gmz_grad_add_t(1, _lib.ptr(gwt), HW, C, O, _lib.ptr(g), _lib.stream_ptr()))


def v_nchw_reference_path():  # the unpermuted path: (x^T dy)^T -> f32, then the accumulate
    gw = (xs.t() @ gy).t().float()
    g.add_(gw)


def tm(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for f in (v_xtdy_strided, v_dytx_rowtranspose, v_xtdy_then_rowtranspose, v_hip_grad_add_t, v_nchw_reference_path):
    print("%-28s %8.1f us" % (f.__name__, tm(f)))
