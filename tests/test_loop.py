"""Config C4's composed loop (datou-gomoku-muzero_amd/loop.py) on CPU: slice building equals the
reference record semantics, and two gloo ranks run self-play -> replay shards -> DDP training with
sharded PER -> weight pushes, staying replica-identical (the self-play source is scripted here: the
HIP engine needs the GPU; tests/test_pipeline_gpu.py runs the GPU version)."""
import os
import socket

import numpy as np
import pytest
import torch

from datou_gomoku_muzero_amd import loop as LP
from datou_gomoku_muzero_amd import records as R


def _random_game(rs, H=6, n_in_row=5):
    """A random legal game on an HxH board (moves until a random length or a full board), as the
    arrays worker.GameHistory.harvest returns."""
    A = H * H
    n = rs.randint(1, A + 1)
    cells = rs.permutation(A)[:n]
    board = np.zeros(A, np.int8)
    boards, players, lasts = [], [], []
    p, last = 1, -1
    for c in cells:
        boards.append(board.copy())
        players.append(p)
        lasts.append(last)
        board[c] = p
        p, last = -p, c
    pols = rs.dirichlet(np.ones(A), n)
    vals = rs.uniform(-1, 1, n).astype(np.float32)
    winner = int(rs.choice([-1, 0, 1]))
    return (0, winner, n, 0, 0, np.array(boards), np.array(players, np.int8), np.array(lasts, np.int32), pols, vals,
            cells.astype(np.int32))


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_slices_from_game_equal_build_game_record(seed):
    rs = np.random.RandomState(seed)
    _, winner, n, _, _, boards, players, lasts, pols, vals, acts = _random_game(rs)
    H = 6
    got = LP.slices_from_game(boards, players, lasts, pols, vals, acts, winner, H, 0.997, 10, 5)
    obs = LP.board_states_to_obs(boards, players, lasts, H)
    _, slices = R.build_game_record(list(obs), [int(a) for a in acts], list(pols), list(vals),
                                    list(boards.reshape(n, H, H)), winner, 0.997, 10, 5)
    want = [np.stack([getattr(s, f) for s in slices]) for f in
            ("observation", "action_history", "reward_history", "policy_history", "value_history")]
    for g, w in zip(got, want):  # compared in the replay buffer's storage types (ReplayBuffer.add casts)
        assert g.shape == w.shape
        assert np.array_equal(g, np.asarray(w).astype(g.dtype)), (g.dtype, w.dtype)


class _ScriptedSelfPlay:
    """CPU stand-in for loop.SelfPlay: finished random games each move, records pushed weights."""

    def __init__(self, seed):
        self.rs = np.random.RandomState(seed)
        self.moves, self.loaded = 0, []

    def step(self):
        self.moves += 1
        return [_random_game(self.rs) for _ in range(self.rs.randint(0, 3))]

    def load_weights(self, sd):
        self.loaded.append({k: torch.as_tensor(v).detach().cpu().clone() for k, v in sd.items()})


def _loop_rank(rank, port, q):
    import torch.distributed as dist
    from datou_gomoku_muzero_amd import trainer as T
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    torch.manual_seed(rank)  # different local inits: the Trainer must broadcast rank 0's
    cfg = T.TrainConfig(BOARD_SIZE=6, NUM_RES_BLOCKS=1, NUM_FILTERS=16, PHYSICAL_BATCH_SIZE=8,
                        TRAIN_BUFFER_SIZE=4096, ENABLE_PER=True)
    tr = T.Trainer(cfg, device="cpu")
    rb = T.ReplayBuffer(cfg, device="cpu")
    sp = _ScriptedSelfPlay(100 + rank)  # different games per rank
    lp = LP.C4Loop(sp, tr, rb, cfg, 8, dist=dist, moves_per_iter=2, train_steps_per_iter=2, model_update_interval=3,
                   seed=7, device="cpu")
    st = lp.run(8)
    params = torch.cat([p.detach().flatten() for p in tr.model.parameters()]).numpy()
    last_push = sp.loaded[-1] if sp.loaded else None
    trained = {k: v.detach().cpu() for k, v in tr.model.state_dict().items()}
    pushed_eq = last_push is not None and all(torch.equal(last_push[k].float(), trained[k].float())
                                              for k in last_push if not k.endswith("num_batches_tracked"))
    q.put((rank, dict(stats=st, params=params, pushed=len(sp.loaded), pushed_eq=pushed_eq,
                      maxp=float(torch.as_tensor(rb.max_priority)), count=len(rb))))
    dist.destroy_process_group()


def test_c4_loop_gloo_world2_replicas_and_weight_pushes():
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_loop_rank, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=600) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    a, b = res[0], res[1]
    assert a["stats"]["train_steps"] == b["stats"]["train_steps"] > 0  # every rank steps together
    assert np.array_equal(a["params"], b["params"])  # DDP replicas identical
    assert a["pushed"] == b["pushed"] == a["stats"]["train_steps"] // 3  # one push per 3 trainer steps
    # the push is the trainer's weights at that step; after the last push at most 2 more steps ran
    if a["stats"]["train_steps"] % 3 == 0:
        assert a["pushed_eq"] and b["pushed_eq"]
    assert a["maxp"] == b["maxp"]  # admission priority kept global (all-reduce MAX)
    assert a["count"] > 0 and b["count"] > 0  # each rank filled its own shard from its own games


def _per_rank(rank, port, q):
    import torch.distributed as dist
    from datou_gomoku_muzero_amd import trainer as T
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    cfg = T.TrainConfig(BOARD_SIZE=6, NUM_RES_BLOCKS=1, NUM_FILTERS=16, TRAIN_BUFFER_SIZE=64, ENABLE_PER=True,
                        PER_BETA=0.4)
    rb = T.ReplayBuffer(cfg, device="cpu")
    n = 20 + 12 * rank  # shards of different sizes and priorities
    from datou_gomoku_muzero_amd.weights import synthetic_slices
    rb.add_arrays(*synthetic_slices(n, 6, 5, np.random.RandomState(rank)))
    rb.prio[:n] = torch.linspace(0.5, 2.0 + rank, n)
    rs = np.random.RandomState(3 + rank)
    _, idx, w = rb.sample(8, rs, dist=dist)
    p = rb.prio[:n].double()
    prob = p[idx] / p.sum() / 2  # rank chosen uniformly, then proportional within the shard
    raw = (52 * prob) ** -0.4  # global count 20 + 32
    q.put((rank, dict(w=w.numpy(), raw=raw.numpy())))
    dist.destroy_process_group()


def test_sharded_per_weights_use_global_count_and_batch_max():
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_per_rank, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    gmax = max(res[0]["raw"].max(), res[1]["raw"].max())
    for r in (0, 1):
        assert np.allclose(res[r]["w"], res[r]["raw"] / gmax, rtol=1e-6)
    assert max(res[0]["w"].max(), res[1]["w"].max()) == pytest.approx(1.0)
