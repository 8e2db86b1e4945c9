"""Diagnostics for trainer.FUSED_BN_BWD_STATS: gradients of small HIP-conv stacks with the BatchNorm backward
sums from the conv epilogue vs the separate reduction, per parameter, in several configurations."""
import sys

import torch

sys.path.insert(0, ".")
from datou_gomoku_muzero_amd import trainer as T  # noqa: E402


def run(mod, x0, gy, mask, fused, res_fold=True):
    T.FUSED_BN_BWD_STATS = fused
    T.FUSED_RES_GRAD = res_fold
    mod.zero_grad(set_to_none=True)
    x = x0.clone().requires_grad_()
    with torch.autocast("cuda", dtype=torch.float16):
        h = mod(x, mask)
    (h.float() * gy).sum().backward()
    torch.cuda.synchronize()
    return [("x", x.grad.double())] + [(n, p.grad.double()) for n, p in mod.named_parameters()]


def compare(name, mod, N=37, nvalid=21, H=15, res_fold=True):
    torch.manual_seed(1)
    mod = mod.cuda().train().to(memory_format=torch.channels_last)
    state = {k: v.clone() for k, v in mod.state_dict().items()}
    g = torch.Generator().manual_seed(N)
    x0 = torch.randn(N, 128, H, H, generator=g).cuda().half().contiguous(memory_format=torch.channels_last)
    gy = torch.randn(N, 128, H, H, generator=g).cuda()
    mask = torch.zeros(N, dtype=torch.bool)
    mask[torch.randperm(N, generator=g)[:nvalid]] = True
    mask = mask.cuda()
    out = []
    for fused in (False, False, True, True):
        mod.load_state_dict(state)
        out.append(run(mod, x0, gy, mask, fused, res_fold))
    print("==", name, "res_fold", res_fold, "(runs: unfused, unfused, fused, fused; errors vs run 2)")
    for i, (n, a) in enumerate(out[1]):
        print("   %-28s %s" % (n, "  ".join("%.3e" % float((o[i][1] - a).norm() / (a.norm() + 1e-30)) for o in out)))


class _BlockOnly(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.b = T._Block(128)

    def forward(self, x, mask):
        return self.b(x, mask)


class _Two(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.b0, self.b1 = T._Block(128), T._Block(128)

    def forward(self, x, mask):
        return self.b1(self.b0(x, mask), mask)


compare("two blocks", _Two())
compare("trunk", T._Trunk(128, 128, 2))
compare("trunk, all rows", T._Trunk(128, 128, 2), nvalid=37)
