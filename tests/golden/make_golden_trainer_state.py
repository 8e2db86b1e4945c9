"""Golden fixture for the trainer checkpoint blob (db_manager.py:231-243, workers.py:469-475,
594-597), made with the REFERENCE's own training setup and DatabaseManager.save_trainer_state (this
container only; /root/reference is never read at test time).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_trainer_state.py

Writes to tests/golden/:
  ref_trainer_state.db   SQLite written by the reference: one trainer_state row = pickle of
                         {model_state_dict, optimizer_state_dict, scheduler_state_dict,
                          train_step_count, games_completed_count} after 3 Adam steps of a small
                         GomokuNetEZ (6x6, 8 filters, 1 block) built and scheduled exactly as
                         workers.py:452-462 does
  ref_trainer_state.npz  what was saved, in plain arrays: every model tensor (m/<name>; tensors over
                         4096 elements as [sum, sum of squares, first 16 values] in ms/<name>), the
                         Adam moments of every parameter that has them, by parameter index
                         (exp_avg/<i>, exp_avg_sq/<i>, step/<i>), the parameter names in order, lr
                         after the steps, the counters
"""
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
for name in ("seaborn",):
    sys.modules.setdefault(name, types.ModuleType(name))
_tb = types.ModuleType("torch.utils.tensorboard")
_tb.SummaryWriter = object
sys.modules.setdefault("torch.utils.tensorboard", _tb)
os.chdir(tempfile.mkdtemp(prefix="gmz_golden_ts_"))

import torch  # noqa: E402
from torch.optim.lr_scheduler import CosineAnnealingLR, LinearLR, SequentialLR  # noqa: E402

import config as ref_config_mod  # noqa: E402
cfg = ref_config_mod.config
cfg.BOARD_SIZE, cfg.ACTION_SPACE_SIZE, cfg.NUM_RES_BLOCKS, cfg.NUM_FILTERS = 6, 36, 1, 8
import network as ref_net  # noqa: E402
import db_manager as ref_db  # noqa: E402


def main():
    torch.manual_seed(7)
    model = ref_net.GomokuNetEZ(cfg)
    # workers.py:452-462: Adam + weight decay, LinearLR warm-up then cosine (per optimiser update)
    optimizer = torch.optim.Adam(model.parameters(), lr=cfg.LEARNING_RATE, weight_decay=cfg.WEIGHT_DECAY)
    acc = cfg.GRADIENT_ACCUMULATION_STEPS
    warm, total = 1000 // acc, 200000 // acc
    scheduler = SequentialLR(optimizer, schedulers=[LinearLR(optimizer, start_factor=0.01, total_iters=warm),
                                                    CosineAnnealingLR(optimizer, T_max=total - warm, eta_min=1e-7)],
                             milestones=[warm])
    x = torch.randn(4, 3, 6, 6)
    for _ in range(3):
        optimizer.zero_grad()
        model.train()
        loss = model.prediction(model.representation(x))[0].square().mean()
        # every parameter except the 512-wide projection head gets Adam state (that head alone would
        # triple the fixture; parameters without gradients have no Adam state, as in torch)
        loss = loss + 1e-3 * sum(p.square().sum() for n, p in model.named_parameters() if "projection" not in n)
        loss.backward()
        optimizer.step()
        scheduler.step()
    state = {"model_state_dict": model.state_dict(), "optimizer_state_dict": optimizer.state_dict(),
             "scheduler_state_dict": scheduler.state_dict(), "train_step_count": 1234, "games_completed_count": 56}
    path = os.path.join(HERE, "ref_trainer_state.db")
    for suffix in ("", "-wal", "-shm"):
        if os.path.exists(path + suffix):
            os.remove(path + suffix)
    mgr = ref_db.DatabaseManager(db_path=path)
    mgr.save_trainer_state(state)
    conn = ref_db.get_db_connection(path)
    conn.execute("PRAGMA wal_checkpoint(TRUNCATE);")
    conn.close()
    for suffix in ("-wal", "-shm"):
        if os.path.exists(path + suffix):
            os.remove(path + suffix)
    out = {}
    for k, v in model.state_dict().items():  # small tensors in full, large ones as checksums
        a = v.detach().numpy()
        if a.size <= 4096:
            out["m/" + k] = a
        else:
            f = a.astype(np.float64).ravel()
            out["ms/" + k] = np.concatenate([[f.sum(), np.square(f).sum()], f[:16]])
    names = [n for n, _ in model.named_parameters()]
    st = optimizer.state_dict()["state"]
    for i in st:
        out["exp_avg/%d" % i] = st[i]["exp_avg"].numpy()
        out["exp_avg_sq/%d" % i] = st[i]["exp_avg_sq"].numpy()
        out["step/%d" % i] = np.float64(st[i]["step"])
    out["param_names"] = np.array(names)
    out["lr"] = np.float64(optimizer.param_groups[0]["lr"])
    out["train_step_count"], out["games_completed_count"] = 1234, 56
    np.savez_compressed(os.path.join(HERE, "ref_trainer_state.npz"), **out)
    print("saved", path, os.path.getsize(path), "bytes; lr", optimizer.param_groups[0]["lr"])


if __name__ == "__main__":
    main()
