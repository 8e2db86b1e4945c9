"""Which production switch moves the fp16 step's loss away from the reference's float32 fixture?  On a trainer
fixture (default: config C4's shape, tests/golden/train_loss_c15full.npz), the loss and its four components of the
production step with every switch on, then with one switch at a time off, plus the reference's own AMP path
("native") — the loss-parity diagnosis behind tests/test_trainer.py's C4-shape bounds.
  python tools/trainer_loss_diag.py [fixture]"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from datou_gomoku_muzero_amd import trainer as T  # noqa: E402
from test_trainer import GOLDEN, _gpu_grads, _nets, _shape  # noqa: E402

fx = sys.argv[1] if len(sys.argv) > 1 else "train_loss_c15full.npz"
d = np.load(os.path.join(GOLDEN, fx))
p = "c0/"
torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic = False, True
ref = np.concatenate([[float(d[p + "loss"])], np.asarray(d[p + "comps"], np.float64)])


def show(tag, logs):
    v = np.asarray(logs, np.float64)
    print("%-26s loss %.6g (%+.3e)  comps %s  rel %s" % (tag, v[0], (v[0] - ref[0]) / ref[0], np.round(v[1:], 5),
                                                         np.array2string((v[1:] - ref[1:]) / np.abs(ref[1:]), precision=2)))


print("reference f32             loss %.6g  comps %s" % (ref[0], np.round(ref[1:], 5)))
show("native AMP", _gpu_grads(T, d, p, "native")[0])
show("f32 GPU", _gpu_grads(T, d, p, "f32")[0])
show("production", _gpu_grads(T, d, p, "prod")[0])


def step_logs(conv, bn, split, subbatch=False, pert=None, amp=True):
    """The production step's logs with the HIP convs / HIP masked BatchNorm / split-K Linears chosen one by one."""
    saved = (T.FUSED_CONV, T.FUSED_BN, T._BigKLinear.SPLIT, T.SUBBATCH_BN)
    try:
        T.FUSED_CONV, T.FUSED_BN, T.SUBBATCH_BN = conv, bn, subbatch
        if not split:
            T._BigKLinear.SPLIT = 10 ** 9
        cfg, model, target = _nets(T, *_shape(d))
        if pert is not None:  # every weight moved by ~1 f16 ulp: w * (1 + 2^-11 N(0, 1))
            rs = np.random.RandomState(pert)
            with torch.no_grad():
                for q in list(model.parameters()) + list(target.parameters()):
                    q.mul_(1 + 2.0 ** -11 * torch.from_numpy(rs.randn(*q.shape).astype(np.float32)))
        model, target = model.cuda().to(memory_format=torch.channels_last), target.cuda()
        model.channels_last = True
        batch = [torch.from_numpy(d[k]).cuda() for k in ("obs", "act", "rew", "pol", "val")]
        with torch.no_grad():
            _, logs, _ = T.muzero_loss(model, target, batch, torch.from_numpy(d["isw"]).cuda(), cfg,
                                       k=int(d[p + "k"]), flip=bool(d[p + "flip"]), amp=amp)
        return [float(x) for x in logs]
    finally:
        T.FUSED_CONV, T.FUSED_BN, T._BigKLinear.SPLIT, T.SUBBATCH_BN = saved


for conv in (True, False):
    for bn in (True, False):
        show("conv %d bn %d" % (conv, bn), step_logs(conv, bn, True))
show("MIOpen + sub-batch f16 BN", step_logs(False, False, False, True))
for pert in range(4):
    show("f16-ulp weights %d: native" % pert, step_logs(False, False, False, True, pert=pert))
    show("f16-ulp weights %d: prod" % pert, step_logs(True, True, True, pert=pert))
    show("f16-ulp weights %d: f32" % pert, step_logs(False, False, False, pert=pert, amp=False))

for sw in ("TARGET_F16", "BATCHED_CONSISTENCY", "BATCHED_HEADS", "SEG_BN_HIP", "FUSED_HEADS", "BATCHED_LOSS",
           "CONCURRENT_FORWARD", "FLAT_NHWC", "FUSED_CONV", "AUTOCAST_CACHE"):
    saved = getattr(T, sw)
    setattr(T, sw, not saved)
    try:
        show("prod, %s=%s" % (sw, not saved), _gpu_grads(T, d, p, "prod")[0])
    except Exception as e:  # noqa: BLE001
        print("prod, %s=%s failed: %r" % (sw, not saved, e))
    finally:
        setattr(T, sw, saved)
