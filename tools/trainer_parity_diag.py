"""Which part of the GPU training path moves the gradients away from the reference's float32
calculate_loss at 128 filters (tests/golden/train_loss_c128.npz)?  Runs the loss + backward in
variants (fp32 / fp16 autocast, NCHW / channels-last, HIP convs on/off, big-K split-K Linear on/off)
and prints each variant's loss error and worst gradient-norm errors by parameter group."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from datou_gomoku_muzero_amd import trainer as T  # noqa: E402
from test_trainer import _nets  # noqa: E402

torch.backends.cudnn.benchmark = True
d = np.load(os.path.join(REPO, "tests", "golden", sys.argv[1] if len(sys.argv) > 1 else "train_loss_c128.npz"))
p = "c0/"


def run(amp, cl, fused_conv=True, bigk=True, fused_bn=True, scale=16.0):
    T.FUSED_CONV, T.FUSED_BN = fused_conv, fused_bn
    saved = T._BigKLinear.SPLIT
    if not bigk:
        T._BigKLinear.SPLIT = 10 ** 9  # K % SPLIT != 0 -> plain nn.Linear
    cfg, model, target = _nets(T, 9, 2, 128)
    model, target = model.cuda(), target.cuda()
    if cl:
        model = model.to(memory_format=torch.channels_last)
        model.channels_last = True
    batch = [torch.from_numpy(d[k]).cuda() for k in ("obs", "act", "rew", "pol", "val")]
    loss, logs, td = T.muzero_loss(model, target, batch, torch.from_numpy(d["isw"]).cuda(), cfg,
                                   k=int(d[p + "k"]), flip=bool(d[p + "flip"]), amp=amp)
    (loss * scale).backward()
    T._BigKLinear.SPLIT = saved
    groups = {}
    for name, prm in model.named_parameters():
        g = prm.grad.float().cpu().numpy() / scale if prm.grad is not None else np.zeros(prm.shape, np.float32)
        gn = float(d[p + "gn/" + name])
        if gn < 1e-3:
            continue
        rel = abs(np.linalg.norm(g.astype(np.float64)) - gn) / gn
        key = name.split(".")[0] + ("" if "projection" in name else "." + name.split(".")[1])
        groups[key] = max(groups.get(key, 0.0), rel)
    print("amp=%d cl=%d hipconv=%d bigk=%d fusedbn=%d  loss rel %.2e  worst:" % (
        amp, cl, fused_conv, bigk, fused_bn, abs(logs[0] - float(d[p + "loss"])) / float(d[p + "loss"])),
        " ".join("%s %.3g" % kv for kv in sorted(groups.items())), flush=True)


run(False, False)
run(False, True)
run(True, False)
run(True, True, fused_conv=False)
run(True, True, bigk=False)
run(True, True, fused_conv=False, bigk=False, fused_bn=False)
run(True, True)
