"""Weight-gradient variants of the channels-last K = 28,800 Linear (trainer._BigKLinear perm path):
time per call of each way to land dW in the f32 .grad in W's (c, p) column order.
  python tools/bigk_wgrad_probe.py"""
import torch

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


for f in (v_xtdy_strided, v_dytx_rowtranspose, v_xtdy_then_rowtranspose, v_nchw_reference_path):
    print("%-28s %8.1f us" % (f.__name__, tm(f)))
