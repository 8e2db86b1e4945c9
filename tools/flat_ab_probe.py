"""A/B of trainer.FLAT_NHWC on the production step's gradient-norm errors vs the reference fixture
(deterministic MIOpen): python tools/flat_ab_probe.py"""
import sys, os, numpy as np, torch
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic = False, True
import test_trainer as TT
from datou_gomoku_muzero_amd import trainer as T
d = np.load("tests/golden/train_loss_c128full.npz")
for flat in (True, False):
    T.FLAT_NHWC = flat
    logs, td, err = TT._fp16_grad_errors(T, d, "c0/", fused=True)
    gmax = max(float(d[k]) for k in d.files if k.startswith("c0/gn/"))
    e = {k: v for k, v in err.items() if float(d["c0/gn/" + k]) >= 1e-6 * gmax}
    worst = sorted(e.items(), key=lambda kv: -kv[1])[:4]
    print("FLAT_NHWC", flat, "loss", logs[0], "mean", np.mean(list(e.values())), [(k, round(v, 4)) for k, v in worst])
