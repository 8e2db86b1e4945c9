"""Where the production fp16 trainer step departs from float32 on the reference's ragged batch
(fixture tests/golden/train_loss_c128.npz: 9x9, 128 filters, 2 blocks, 7/6/5/4/3 live
games in the 5 unroll steps) and on the full batch (train_loss_c128full.npz).

Four paths on the same weights, batch and augmentation (GPU, channels-last, as tests/test_trainer.py
_gpu_grads):
  f32      no autocast (MIOpen convs, float32 masked-BN kernels): the truth for the large weights
  prod     fp16 autocast on the production kernels (HIP convs, masked-BN kernels: BN output and the
           residual stream in f16)
  torch16  fp16 autocast, PyTorch kernels, the row-masked BatchNorm of trainer._bn in FLOAT32: its
           output, hence the residual stream of every unroll step, stays f32 (the comparator the round-3
           test called "PyTorch's own fp16")
  native   fp16 autocast, PyTorch kernels, the reference's own sub-batch BatchNorm (trainer.SUBBATCH_BN:
           the live rows gathered through nn.BatchNorm2d in f16, loss.py:89-107 as it runs under AMP)
Prints, per path: the forward hidden state of every unroll step vs f32 (relative L2 over the live rows),
and per parameter e = |g - g_true| / |g_true| (the reference's whole tensor where the fixture stores it,
else the f32 path), grouped by layer in forward order; then the means.  JSON summary on stdout's last line.

  python tools/trainer_ragged_diag.py [--fixture train_loss_c128.npz]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from test_trainer import _nets  # noqa: E402  (the fixture's weight generator)
from datou_gomoku_muzero_amd import trainer as T  # noqa: E402

GOLDEN = os.path.join(REPO, "tests", "golden")


def run(d, p, mode):
    saved = (T.FUSED_CONV, T.FUSED_BN, T._BigKLinear.SPLIT, T.SUBBATCH_BN)
    fused = mode in ("prod", "f32")
    T.FUSED_CONV, T.FUSED_BN = fused, fused
    T.SUBBATCH_BN = mode == "native"
    if not fused:
        T._BigKLinear.SPLIT = 10 ** 9
    hs = []
    try:
        cfg, model, target = _nets(T, 9, 2, 128)
        model, target = model.cuda().to(memory_format=torch.channels_last), target.cuda()
        model.channels_last = True
        dyn = model.dynamics

        def rec(h, a, mask=None):
            out = dyn(h, a, mask)
            hs.append(out[0].detach().float().cpu().numpy())
            return out
        model.dynamics = rec
        rep = model.representation

        def rec0(obs, mask=None):
            out = rep(obs, mask)
            if mask is None and not hs:
                hs.append(out.detach().float().cpu().numpy())
            return out
        model.representation = rec0
        batch = [torch.from_numpy(d[k]).cuda() for k in ("obs", "act", "rew", "pol", "val")]
        for scale in ((2.0 ** 12, 2.0 ** 8, 2.0 ** 4, 1.0) if mode != "f32" else (1.0,)):
            model.zero_grad(set_to_none=True)
            hs.clear()
            loss, logs, td = T.muzero_loss(model, target, batch, torch.from_numpy(d["isw"]).cuda(), cfg,
                                           k=int(d[p + "k"]), flip=bool(d[p + "flip"]), amp=mode != "f32")
            (loss * scale).backward()
            if all(torch.isfinite(q.grad).all() for q in model.parameters() if q.grad is not None):
                break
        grads = {n: (q.grad.float().cpu().numpy() / scale).astype(np.float64) for n, q in model.named_parameters()
                 if q.grad is not None}
        return hs[:6], grads
    finally:
        T.FUSED_CONV, T.FUSED_BN, T._BigKLinear.SPLIT, T.SUBBATCH_BN = saved


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fixture", default="train_loss_c128.npz")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic = False, True
    d = np.load(os.path.join(GOLDEN, a.fixture))
    p = "c0/"
    act = d["act"]
    live = [np.ones(act.shape[0], bool)] + [act[:, s] != -1 for s in range(act.shape[1])]
    out = {m: run(d, p, m) for m in ("f32", "prod", "torch16", "native")}
    gmax = max(float(d[k]) for k in d.files if k.startswith(p + "gn/"))
    stored = {k[len(p) + 2:] for k in d.files if k.startswith(p + "g/")}
    summary = {"fixture": a.fixture, "live_rows_per_step": [int(m.sum()) for m in live], "forward": {}, "grads": {}}
    print("forward hidden states vs f32 (relative L2 over live rows), steps 0..5:")
    for m in ("prod", "torch16", "native"):
        errs = []
        for s, (x, y) in enumerate(zip(out[m][0], out["f32"][0])):
            lv = live[s]
            errs.append(float(np.linalg.norm(x[lv] - y[lv]) / max(np.linalg.norm(y[lv]), 1e-30)))
        summary["forward"][m] = errs
        print("  %-8s %s" % (m, " ".join("%.2e" % e for e in errs)))
    names = [n for n in out["f32"][1]]
    print("\nper-parameter e = |g - g_true| / |g_true| (truth: %s)" % "reference tensor where stored, else f32 GPU")
    print("%-52s %9s %9s %9s" % ("parameter", "prod", "torch16", "native"))
    rows = {}
    for n in names:
        true = d[p + "g/" + n].astype(np.float64) if n in stored else out["f32"][1][n]
        if np.linalg.norm(true) <= 1e-6 * gmax:
            continue
        e = {m: float(np.linalg.norm(out[m][1][n] - true) / np.linalg.norm(true)) for m in ("prod", "torch16", "native")}
        rows[n] = e
        print("%-52s %9.3g %9.3g %9.3g" % (n, e["prod"], e["torch16"], e["native"]))
    for m in ("prod", "torch16", "native"):
        summary["grads"][m] = float(np.mean([e[m] for e in rows.values()]))
    summary["per_param"] = rows
    print("\nmean e: prod %.4g  torch16 (f32 masked BN) %.4g  native (sub-batch f16 BN) %.4g over %d tensors"
          % (summary["grads"]["prod"], summary["grads"]["torch16"], summary["grads"]["native"], len(rows)))
    print(json.dumps({k: v for k, v in summary.items() if k != "per_param"}))
    with open(os.path.join(REPO, "gpurun_out", "ragged_diag_%s.json" % a.fixture.split(".")[0]), "w") as f:
        json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
