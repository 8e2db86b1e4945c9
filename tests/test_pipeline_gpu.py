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
    one GPU over gloo); each phase (headline, extras, trainer, loop) runs as fresh rank processes under a
    wall-time cap, and rank 0 prints ONE line with n_gpus 2 and the global game count.  The trainer phase
    of rank 1 is made to fail (GMZ_BENCH_INJECT_FAIL) while rank 0 waits in its collectives: the line
    still carries the headline, the extras and the loop (whose DDP trainer steps over the same group
    type), and {"error": ...} in "trainer" only."""
    import json
    import subprocess
    import sys
    from conftest import REPO
    env = dict(os.environ, GMZ_DIST_BACKEND="gloo", GMZ_BENCH_INJECT_FAIL="trainer:1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--games", "64",
                        "--size", "9", "--sims", "50", "--blocks", "1", "--steps", "2", "--warmup", "1",
                        "--trainer-steps", "2", "--trainer-warmup", "4", "--trainer-batch", "16", "--trainer-buffer", "64",
                        "--loop-iters", "4", "--loop-warmup", "4", "--loop-games", "64", "--loop-update-interval", "2",
                        "--loop-prefill", "64", "--loop-buffer", "4096", "--sublines", "c1", "--subline-games", "32",
                        "--c1-steps", "2", "--worker-moves", "3", "--worker-warmup", "2", "--dist-timeout", "60",
                        "--phase-timeout-trainer", "90"],
                       env=env, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]  # (gloo itself prints connection notes)
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_games"] == 128 and d["config"]["ranks"] == 2
    assert d["value"] > 0 and len(d["rank_values"]) == 2 and all(v > 0 for v in d["rank_values"])
    assert "world_size=2" in p.stderr
    assert "error" in d["trainer"] and "rank 1" in d["trainer"]["error"], d["trainer"]
    assert d["phases"]["isolated"] and set(d["phases"]["detail"]) == {"selfplay", "extras", "trainer", "loop"}
    lc = d["loop_c4"]
    assert "error" not in lc
    assert lc["n_gpus"] == 2 and lc["trainer_steps_per_s"] > 0 and lc["moves_per_s"] > 0 and lc["weight_pushes"] == 2
    assert lc["weight_push_ms"] > 0
    wk = d["worker"]
    assert wk["n_gpus"] == 2 and wk["value"] > 0 and wk["messages"]["ui"] > 0
    c1 = d["sublines"]["c1"]
    assert c1["n_gpus"] == 2 and c1["value"] > 0 and 0 < c1["roofline"]["frac"] < 1


def test_c4_loop_on_the_gpu_pushes_trained_weights_into_self_play():
    """loop.C4Loop with the real HIP self-play (single rank): finished games fill the replay shard,
    the trainer steps, and every push hot-swaps exactly the trainer's weights into the engine's
    network (its packed tensors equal a fresh packing of the trainer's state_dict)."""
    from datou_gomoku_muzero_amd import loop as LP, network as N, trainer as T
    from datou_gomoku_muzero_amd.config import GmzConfig
    cfg = GmzConfig(BOARD_SIZE=6, NUM_SIMULATIONS=16, NUM_RES_BLOCKS=1)
    tcfg = T.TrainConfig(BOARD_SIZE=6, NUM_RES_BLOCKS=1, PHYSICAL_BATCH_SIZE=16, TRAIN_BUFFER_SIZE=4096, ENABLE_PER=True)
    tr = T.Trainer(tcfg, device="cuda", graph=False)
    sp = LP.SelfPlay(cfg, 32, tr.state_dict_cpu(), seed=3)
    rb = T.ReplayBuffer(tcfg, device="cuda")
    lp = LP.C4Loop(sp, tr, rb, tcfg, 16, moves_per_iter=2, train_steps_per_iter=1, model_update_interval=2)
    st = lp.run(40)
    torch.cuda.synchronize()
    assert st["games"] > 0 and st["slices"] == len(rb) and st["train_steps"] > 0
    assert st["weight_pushes"] == st["train_steps"] // 2 >= 1
    if st["train_steps"] % 2 == 0:  # the last push is the current trainer state
        want = N.pack_weights(tr.state_dict_cpu(), cfg, "fp16")
        for k, v in want.items():
            assert np.array_equal(sp.net._tensors[k].cpu().numpy(), v), k
    sp.close()


def test_c4_loop_concurrent_stream_trains_and_pushes():
    """loop.C4Loop(concurrent=True): the trainer steps and shard updates run on their own HIP stream
    beside the self-play moves; the counts, the shard contents and the pushed weights are those of a
    consistent loop (every finished game's slices in the shard, pushes = steps / interval, the last
    push = the trainer's current weights)."""
    from datou_gomoku_muzero_amd import loop as LP, network as N, trainer as T
    from datou_gomoku_muzero_amd.config import GmzConfig
    cfg = GmzConfig(BOARD_SIZE=6, NUM_SIMULATIONS=16, NUM_RES_BLOCKS=1)
    tcfg = T.TrainConfig(BOARD_SIZE=6, NUM_RES_BLOCKS=1, PHYSICAL_BATCH_SIZE=16, TRAIN_BUFFER_SIZE=4096, ENABLE_PER=True)
    tr = T.Trainer(tcfg, device="cuda")
    sp = LP.SelfPlay(cfg, 32, tr.state_dict_cpu(), seed=3)
    rb = T.ReplayBuffer(tcfg, device="cuda")
    lp = LP.C4Loop(sp, tr, rb, tcfg, 16, moves_per_iter=2, train_steps_per_iter=1, model_update_interval=2,
                   concurrent=True)
    assert lp.concurrent and lp.train_stream is not None
    st = lp.run(40)
    torch.cuda.synchronize()
    assert st["games"] > 0 and st["slices"] == len(rb) and st["train_steps"] > 0
    assert st["weight_pushes"] == st["train_steps"] // 2 >= 1
    assert torch.isfinite(lp.last_logs).all()
    assert float(rb.prio[: len(rb)].min()) > 0  # every admitted slice carries a priority
    if st["train_steps"] % 2 == 0:
        want = N.pack_weights(tr.state_dict_cpu(), cfg, "fp16")
        for k, v in want.items():
            assert np.array_equal(sp.net._tensors[k].cpu().numpy(), v), k
    sp.close()


@pytest.mark.parametrize("concurrent", [False, True])
def test_c4_loop_at_its_own_workload(concurrent):
    """Config C4 at its own network and batch (BASELINE config 4): 15x15, GomokuNetEZ 128
    filters x 8 blocks, B = 360, 5 unroll steps, PER; self-play of 128 games from the empty board at 32
    simulations per move (the config's 400 cut so the test plays ~120 moves in seconds; the search code
    is the same).  One engine stream, so the tower schedules boards by ticket (the workspace counters a
    weight push must not disturb).  Checks, as main.py:91-109 / workers.py:379-439,587-593
    run them: every finished game's slices reach the replay shard; the trainer samples those slices;
    every push hot-swaps exactly the trainer's weights into the self-play network; and (concurrent:
    trainer on its own HIP stream beside the moves) the same holds with the push on the trainer's stream."""
    from datou_gomoku_muzero_amd import loop as LP, network as N, trainer as T, weights as W
    from datou_gomoku_muzero_amd.config import GmzConfig
    cfg = GmzConfig(BOARD_SIZE=15, NUM_SIMULATIONS=32, NUM_RES_BLOCKS=8)
    tcfg = T.TrainConfig(BOARD_SIZE=15, NUM_RES_BLOCKS=8, PHYSICAL_BATCH_SIZE=360, TRAIN_BUFFER_SIZE=65536,
                         ENABLE_PER=True)
    tr = T.Trainer(tcfg, device="cuda")
    sp = LP.SelfPlay(cfg, 128, tr.state_dict_cpu(), seed=3, streams=1)
    rb = T.ReplayBuffer(tcfg, device="cuda")
    prefill = 512
    rb.add_arrays(*W.synthetic_slices(prefill, 15, tcfg.NUM_UNROLL_STEPS, np.random.RandomState(0)))
    sampled = []
    sample = rb.sample

    def spy(B, rng=np.random, dist=None):
        out = sample(B, rng, dist)
        sampled.append(out[1].clone())
        return out
    rb.sample = spy
    interval = 10
    lp = LP.C4Loop(sp, tr, rb, tcfg, 360, moves_per_iter=2, train_steps_per_iter=1, model_update_interval=interval,
                   concurrent=concurrent)
    st = lp.run(60)
    torch.cuda.synchronize()
    assert st["games"] > 0, "no game finished in 120 moves"
    assert st["slices"] == len(rb) - prefill, (st, len(rb))
    assert st["train_steps"] == 60 and st["weight_pushes"] == 60 // interval
    idx = torch.cat(sampled).cpu().numpy()
    assert (idx >= prefill).sum() > 0, "the trainer never sampled a self-play slice"
    assert np.isfinite(lp.last_logs.cpu().numpy()).all()
    want = N.pack_weights(tr.state_dict_cpu(), cfg, "fp16")  # 60 steps: the last push is the current state
    for k, v in want.items():
        assert np.array_equal(sp.net._tensors[k].cpu().numpy(), v), k
    # after the pushes the self-play network still searches: one more move plays every game
    done = sp.step()
    torch.cuda.synchronize()
    assert isinstance(done, list)
    sp.close()


def test_c2_at_8192_games_and_the_c4_trainer_share_one_card():
    """Config C2's search at 8,192 concurrent games (its two-stream engine, hidden-state pool sized by the
    waves a search can use: engine.hidden_slots) and config C4's trainer (B = 360, 15x15, 8 blocks, PER
    shard) resident on one MI355X together: one self-play move of every game and trainer steps run, and
    the card's used memory stays well inside its 288 GB (the hidden pool alone was 190 GB at 402 slots
    per game before round 4)."""
    from datou_gomoku_muzero_amd import engine as E, loop as LP, trainer as T, weights as W
    from datou_gomoku_muzero_amd.config import GmzConfig
    free0, total = torch.cuda.mem_get_info()
    G = 8192
    cfg = GmzConfig(BOARD_SIZE=15, NUM_SIMULATIONS=400, NUM_RES_BLOCKS=8)
    tcfg = T.TrainConfig(BOARD_SIZE=15, NUM_RES_BLOCKS=8, PHYSICAL_BATCH_SIZE=360, TRAIN_BUFFER_SIZE=65536,
                         ENABLE_PER=True)
    tr = T.Trainer(tcfg, device="cuda")
    sp = LP.SelfPlay(cfg, G, tr.state_dict_cpu(), seed=3)
    pool_gb = sp.net.pool.numel() * 2 / 2 ** 30
    assert sp.net.pool.numel() == E.hidden_slots(cfg, G) * 225 * 128 and pool_gb < 50
    rb = T.ReplayBuffer(tcfg, device="cuda")
    rb.add_arrays(*W.synthetic_slices(2048, 15, tcfg.NUM_UNROLL_STEPS, np.random.RandomState(0)))
    rs = np.random.RandomState(1)
    for _ in range(2):
        sp.step()
        batch, idx, w = rb.sample(360, rs)
        logs, td = tr.step(batch, w)
        rb.update_priorities(idx, td)
        assert np.isfinite(logs[0])
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info()
    used_gb = (free0 - free1) / 2 ** 30
    print("C2 x 8192 games + C4 trainer: %.1f GiB used on the card (hidden pool %.1f GiB) of %.0f GiB"
          % (used_gb, pool_gb, total / 2 ** 30))
    assert used_gb < 0.5 * total / 2 ** 30
    sp.close()
