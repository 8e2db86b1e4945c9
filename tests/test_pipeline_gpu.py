"""The whole loop on one GPU, through the reference's message types (main.py's process graph in one
process): gpu_selfplay_worker -> (GameRecord, [TrainingSlice]) on data_queue -> RecordStore (the
reference's SQLite format) -> trainer ReplayBuffer -> Trainer steps -> ModelWeightsUpdate on the
model-update queue -> the worker hot-swaps the new weights between moves."""
import os
import queue

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


class _Ev:
    def __init__(self):
        self.flag = False

    def is_set(self):
        return self.flag


class _Upd:  # ipc_messages.ModelWeightsUpdate shape (ipc_messages.py:74-82)
    def __init__(self, weights):
        self.weights = weights


def _drain(q):
    out = []
    while not q.empty():
        out.append(q.get())
    return out


def test_selfplay_records_train_and_hot_swap(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from datou_gomoku_muzero_amd import formats as F
    from datou_gomoku_muzero_amd import trainer as T
    from datou_gomoku_muzero_amd import weights as W
    from datou_gomoku_muzero_amd.config import GmzConfig
    from datou_gomoku_muzero_amd.worker import gpu_selfplay_worker

    cfg = GmzConfig(BOARD_SIZE=6, NUM_SIMULATIONS=16, NUM_RES_BLOCKS=1)
    sd0 = W.synthetic_state_dict(cfg, seed=5)
    dq, lq, uq, tq = queue.Queue(), queue.Queue(), queue.Queue(), queue.Queue()
    gpu_selfplay_worker(0, 0, dq, lq, uq, _Ev(), trainer_event_queue=tq, num_games=16, cfg=cfg, max_moves=40,
                        state_dict=sd0, emit_move_notices=False)
    items = _drain(dq)
    assert items, "no finished game"
    # records -> the reference's on-disk format -> replay warm-up
    st = F.RecordStore(str(tmp_path / "training_state.db"))
    for rec, slices, version in items:
        assert st.add_game_and_slices(rec, slices, version) is not None
    n = sum(len(s) for _, s, _ in items)
    assert st.get_buffer_size() == n
    tc = T.TrainConfig(BOARD_SIZE=6, NUM_RES_BLOCKS=1, PHYSICAL_BATCH_SIZE=8, TRAIN_BUFFER_SIZE=4096)
    rb = T.ReplayBuffer(tc, device="cuda")
    rb.add(st.load_latest_samples(n))
    st.close()
    assert len(rb) == n
    tr = T.Trainer(tc, device="cuda", state_dict=sd0)
    for _ in range(3):
        batch, idx, w = rb.sample(tc.PHYSICAL_BATCH_SIZE, np.random.RandomState(0))
        logs, td = tr.step(batch, w)
        rb.update_priorities(idx, td)
        assert np.isfinite(logs[0])
    sd1 = tr.state_dict_cpu()
    changed = [k for k in sd0 if k in sd1 and not np.allclose(np.asarray(sd0[k]), sd1[k].numpy())]
    assert changed, "the optimiser step left every weight unchanged"
    # hot swap: the worker starts on sd0 and picks sd1 up from the model-update queue between moves
    mq = queue.Queue()
    mq.put(_Upd(sd1))
    dq2 = queue.Queue()
    gpu_selfplay_worker(0, 0, dq2, queue.Queue(), queue.Queue(), _Ev(), num_games=16, cfg=cfg, max_moves=12,
                        state_dict=sd0, model_update_queue=mq, emit_move_notices=False)
    assert mq.empty(), "the worker did not consume the ModelWeightsUpdate"


def test_bench_spawns_its_own_ranks_gloo_rehearsal():
    """`python bench.py --gpus 2` with no external launcher starts 2 rank processes (here sharing the
    one GPU over gloo) and rank 0 prints ONE line with n_gpus 2 and the global game count."""
    import json
    import subprocess
    import sys
    from conftest import REPO
    env = dict(os.environ, GMZ_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--net", "hash", "--games", "64",
                        "--size", "9", "--sims", "50", "--steps", "2", "--warmup", "1", "--trainer-steps", "0"],
                       env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]  # (gloo itself prints connection notes)
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_games"] == 128 and d["config"]["ranks"] == 2
    assert "world_size=2" in p.stderr
