"""Diagnostics: muzero_loss gradients with the HIP residual-block convs vs MIOpen fp16 vs float32."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from datou_gomoku_muzero_amd import trainer as T
cfg = T.TrainConfig(BOARD_SIZE=9, NUM_RES_BLOCKS=2, NUM_FILTERS=128)
torch.manual_seed(0)
base = T.TrainNet(cfg, reference_init=False)
rs = np.random.RandomState(0)
B, U, A = 24, cfg.NUM_UNROLL_STEPS, 81
act = rs.randint(0, A, (B, U)).astype(np.int64)
act[:5, 3:] = -1
batch = [torch.from_numpy((rs.rand(B, U + 1, 3, 9, 9) < 0.2).astype(np.float32)).cuda(),
         torch.from_numpy(act).cuda(), torch.from_numpy(rs.choice([-1.0, 0.0, 1.0], (B, U)).astype(np.float32)).cuda(),
         torch.from_numpy(rs.dirichlet(np.ones(A), (B, U + 1)).astype(np.float32)).cuda(),
         torch.from_numpy(rs.uniform(-1, 1, (B, U + 1)).astype(np.float32)).cuda()]
mode = sys.argv[1] if len(sys.argv) > 1 else "all"
orig_bwd = T._Conv3x3NHWC.backward


def bwd_miopen_dgrad(ctx, gy):
    x, w = ctx.saved_tensors
    gy = gy.to(x.dtype).contiguous(memory_format=torch.channels_last)
    wd = w.to(x.dtype).contiguous(memory_format=torch.channels_last)
    gx, gw, _ = torch.ops.aten.convolution_backward(gy, x, wd, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                                    [True, True, False])
    return gx, gw.to(w.dtype)


res = {}
for name, fused, amp, bw in (("hip", True, True, None), ("hip_fwd_only", True, True, bwd_miopen_dgrad),
                             ("miopen16", False, True, None), ("f32", False, False, None)):
    T.FUSED_CONV = fused
    T._Conv3x3NHWC.backward = staticmethod(bw) if bw else orig_bwd
    m = T.TrainNet(cfg, reference_init=False).cuda()
    m.load_state_dict(base.state_dict())
    m = m.to(memory_format=torch.channels_last)
    m.channels_last = True
    tgt = T.TrainNet(cfg, reference_init=False).cuda()
    tgt.load_state_dict(base.state_dict())
    with torch.autocast("cuda", enabled=amp, dtype=torch.float16):
        h = m.representation(batch[0][:, 0])
    loss, logs, _ = T.muzero_loss(m, tgt, batch, torch.ones(B, device="cuda"), cfg, k=1, flip=True, amp=amp)
    loss.backward()
    res[name] = (logs, h.float(), {n: float(p.grad.norm()) for n, p in m.named_parameters() if p.grad is not None})
T._Conv3x3NHWC.backward = orig_bwd
for k, v in res.items():
    print(k, ["%.6f" % x for x in v[0]], "h err vs f32 %.3e" % float((v[1] - res["f32"][1]).abs().max()))
names = list(res["f32"][2])
print("%-55s %10s %10s %10s %10s" % ("param", "hip", "hipfwd", "miopen16", "f32"))
for n in names:
    f = res["f32"][2][n]
    print("%-55s %10.5f %10.5f %10.5f %10.5f" % (n, res["hip"][2][n] / f - 1, res["hip_fwd_only"][2][n] / f - 1, res["miopen16"][2][n] / f - 1, f))
