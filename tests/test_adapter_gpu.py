"""Drop-in adapters (datou-gomoku-muzero_amd/mcts.py) and the worker (worker.py) on the GPU:
the reference's own test contracts (tests/test_mcts_logic.py:116-165) and bit-exact parity with
the reference fixtures through the queue protocol."""
import glob
import os
import queue

import numpy as np
import pytest

from conftest import GOLDEN
from queue_helpers import Game, MockQueue, ServerQueue

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def M():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from datou_gomoku_muzero_amd import mcts
    from datou_gomoku_muzero_amd.config import GmzConfig
    return mcts, GmzConfig


def test_request_counts_like_reference(M):
    """test_mcts_logic.py:116-136: AZ -> NUM_SIMULATIONS 'initial', 0 recurrent; MZ -> 1 initial, >0 recurrent."""
    mcts, GmzConfig = M
    cfg = GmzConfig(BOARD_SIZE=6, NUM_SIMULATIONS=15)
    q = MockQueue(36)
    az = mcts.HipAlphaZeroMCTS(0, q, q, cfg=cfg)
    az.search(Game(np.zeros((6, 6)), 1, None))
    kinds = [r[1] for r in q.put_log]
    assert kinds.count("initial") == 15 and kinds.count("recurrent_batch") == 0
    q2 = MockQueue(36)
    mz = mcts.HipMuZeroMCTS(0, q2, q2, cfg=cfg)
    mz.search(Game(np.zeros((6, 6)), 1, None))
    kinds = [r[1] for r in q2.put_log]
    assert kinds.count("initial") == 1 and kinds.count("recurrent_batch") > 0


def test_output_contract_like_reference(M):
    """test_mcts_logic.py:138-165."""
    mcts, GmzConfig = M
    cfg = GmzConfig(BOARD_SIZE=6, NUM_SIMULATIONS=15)
    rs = np.random.RandomState(3)
    b = np.zeros(36, np.int8)
    cells = rs.permutation(36)[:8]
    p = 1
    for c in cells:
        b[c] = p
        p = -p
    game = Game(b.reshape(6, 6), p, (cells[-1] // 6, cells[-1] % 6))
    for cls in (mcts.HipAlphaZeroMCTS, mcts.HipMuZeroMCTS):
        q = MockQueue(36)
        policy, value, action = cls(0, q, q, cfg=cfg).search(game)
        assert isinstance(policy, np.ndarray) and abs(policy.sum() - 1.0) < 1e-5
        assert isinstance(action, int) and b[action] == 0
        assert isinstance(value, (float, np.floating)) and -1.0 <= value <= 1.0


MCTS_FILES = sorted(os.path.basename(f) for f in glob.glob(os.path.join(GOLDEN, "mcts_*.npz")))


@pytest.mark.parametrize("fname", [f for f in MCTS_FILES if "19" not in f])
def test_adapter_reproduces_reference_fixture(M, golden, fname):
    """Seeded global RandomState + HashNet server queue -> the reference's exact search results."""
    mcts, GmzConfig = M
    d = golden(fname)
    size, mode, sims = int(d["size"]), str(d["mode"]), int(d["sims"])
    cfg = GmzConfig(BOARD_SIZE=size, NUM_SIMULATIONS=sims, MCTS_IMPLEMENTATION=mode)
    q = ServerQueue(size * size)
    eng = mcts.make_engine(0, q, q, cfg=cfg)
    np.random.seed(int(d["seed"]))
    for i in range(len(d["action"])):
        lm = int(d["lastmove"][i])
        game = Game(d["board"][i].reshape(size, size), d["player"][i], None if lm < 0 else (lm // size, lm % size))
        q.log.clear()
        policy, value, action = eng.search(game)
        assert action == d["action"][i] and value == d["value"][i]
        assert np.abs(policy - d["policy"][i]).max() <= (1e-6 if size <= 6 else 1e-12)
        assert sum(1 for k, _ in q.log if k == "initial") == d["n_initial"][i]
        assert sum(n for k, n in q.log if k == "recurrent_batch") == d["recurrent_rows"][i]


def test_worker_emits_reference_messages(M):
    """gpu_selfplay_worker: records, slices and status messages for finished games."""
    from datou_gomoku_muzero_amd.worker import gpu_selfplay_worker
    mcts, GmzConfig = M
    cfg = GmzConfig(BOARD_SIZE=6, NUM_SIMULATIONS=16, NUM_RES_BLOCKS=1)

    class Ev:
        def __init__(self):
            self.f = False

        def is_set(self):
            return self.f

    dq, lq, uq, tq = queue.Queue(), queue.Queue(), queue.Queue(), queue.Queue()
    gpu_selfplay_worker(0, None, dq, lq, uq, Ev(), trainer_event_queue=tq, num_games=8, cfg=cfg, max_moves=40)
    items = []
    while not dq.empty():
        items.append(dq.get())
    assert items, "no finished game in 40 moves of 6x6"
    for record, slices, version in items:
        n = len(record.actions)
        assert len(slices) == n and len(record.rewards) == n and len(record.values) == n
        assert record.observations[0].shape == (3, 6, 6) and record.policies[0].shape == (36,)
        assert slices[0].observation.shape == (6, 3, 6, 6) and slices[0].action_history.dtype == np.int32
        assert abs(record.rewards[-1]) in (0.0, 1.0)
    kinds = []
    while not uq.empty():
        kinds.append(type(uq.get()).__name__)
    assert kinds.count("SelfPlayMove") >= 8 * 5 and kinds.count("GameCompletedNotice") == len(items)
    assert tq.qsize() == len(items) and lq.qsize() == len(items)
    # SelfPlayStatus (move count, missed fives, missed totals) from the device scan == the host
    # restatement of workers.py:191-203 (pinned to the reference by tests/test_records.py)
    from datou_gomoku_muzero_amd import records as R
    got = sorted((s.avg_len, s.miss_five, s.miss_total) for s in (lq.get() for _ in range(lq.qsize())))
    want = sorted((len(r.actions),) + R.missed_wins(r.board_states, r.actions, 6) for r, _, _ in items)
    assert got == want


@pytest.mark.parametrize("fname", ["mcts_mz15_400.npz", "mcts_az9_50.npz", "mcts_mz9_50.npz"])
def test_search_batch_equals_per_game_search(M, golden, fname):
    """search_batch(games) == [search(g) for g in games] from the same RandomState."""
    mcts, GmzConfig = M
    d = golden(fname)
    size, mode, sims = int(d["size"]), str(d["mode"]), int(d["sims"])
    cfg = GmzConfig(BOARD_SIZE=size, NUM_SIMULATIONS=sims, MCTS_IMPLEMENTATION=mode)
    games = []
    for i in range(len(d["action"])):
        lm = int(d["lastmove"][i])
        games.append(Game(d["board"][i].reshape(size, size), d["player"][i], None if lm < 0 else (lm // size, lm % size)))
    q1 = ServerQueue(size * size)
    e1 = mcts.make_engine(0, q1, q1, cfg=cfg)
    np.random.seed(int(d["seed"]))
    seq = [e1.search(g) for g in games]
    q2 = ServerQueue(size * size)
    e2 = mcts.make_engine(0, q2, q2, cfg=cfg)
    np.random.seed(int(d["seed"]))
    pol, val, act = e2.search_batch(games)
    assert pol.shape == (len(games), size * size) and pol.dtype == np.float64
    for i, (p, v, a) in enumerate(seq):
        assert act[i] == a and val[i] == v
        assert np.abs(pol[i] - p).max() <= 1e-12
    # and the reference's own outputs
    assert act.tolist() == d["action"].tolist()


class _DropOnce(ServerQueue):
    """ServerQueue whose reply to the n-th 'recurrent_batch' request is lost (a timeout)."""

    def __init__(self, A, drop_at):
        super().__init__(A)
        self.n_rec, self.drop_at = 0, drop_at

    def put(self, item):
        super().put(item)
        if item[1] == "recurrent_batch":
            self.n_rec += 1
            if self.n_rec == self.drop_at:
                self.results.pop()  # the server never answers this one


def test_recurrent_timeout_retries_the_wave(M):
    """mcts.py:82-85 + 337: a timed-out recurrent request returns [] and the loop `continue`s, so
    the same wave is requested again and the search result is unchanged."""
    mcts, GmzConfig = M
    cfg = GmzConfig(BOARD_SIZE=6, NUM_SIMULATIONS=40)
    rs_state = np.random.get_state()
    outs, logs = [], []
    for q in (ServerQueue(36), _DropOnce(36, drop_at=3)):
        np.random.set_state(rs_state)
        eng = mcts.HipMuZeroMCTS(0, q, q, cfg=cfg)
        pol, val, act = eng.search(Game(np.zeros((6, 6)), 1, None))
        outs.append((pol, val, act))
        logs.append(q.log)
    assert outs[0][2] == outs[1][2] >= 0 and outs[0][1] == outs[1][1]
    assert np.array_equal(outs[0][0], outs[1][0])
    assert len(logs[1]) == len(logs[0]) + 1 and logs[1][4] == logs[1][3]  # the dropped request, re-sent


@pytest.mark.parametrize("streams,openings", [(1, False), (2, False), (2, True)])
def test_worker_records_equal_a_synchronous_loop(M, streams, openings):
    """The worker's device-side history harvested one move behind (worker.GameHistory) yields exactly
    the records of a plain synchronous loop over the same engine (same seed, same weights) that copies
    every move's position / policy / value / action to the host before the next move — also with the
    worker's games split over two HIP streams (engine.SplitSelfPlayEngine), and with the first game of
    every slot started from a random opening (bench's staggered starts: its record holds the moves
    searched from the opening on, the slot's later games start from the empty board)."""
    from datou_gomoku_muzero_amd import engine as E, network as N, records as R, weights as W
    from datou_gomoku_muzero_amd.worker import gpu_selfplay_worker
    mcts, GmzConfig = M
    cfg = GmzConfig(BOARD_SIZE=6, NUM_SIMULATIONS=16, NUM_RES_BLOCKS=1)
    G, moves, seed = 8, 45, 5

    class Ev:
        def is_set(self):
            return False

    op = E.random_openings(G, 6, np.random.RandomState(11), 12) if openings else None
    dq = queue.Queue()
    gpu_selfplay_worker(0, None, dq, None, None, Ev(), num_games=G, cfg=cfg, max_moves=moves, seed=seed,
                        streams=streams, openings=op)
    got = []
    while not dq.empty():
        got.append(dq.get())
    # the synchronous reference loop
    sd = W.synthetic_state_dict(cfg, seed=seed, with_projection=False)
    net = N.GomokuNetHip(sd, cfg, num_slots=G * 18, max_rows=G)
    eng = E.BatchedSelfPlayEngine(cfg, num_games=G, net=net, seed=seed)
    eng.reset_games()
    if op is not None:
        eng.set_positions(*op)
    hist = [dict(obs=[], act=[], pol=[], val=[], brd=[]) for _ in range(G)]
    want = []
    for _ in range(moves):
        b, p, lm, mc = eng.game_state()
        pol, val, act = eng.search()
        st = eng.play(reset_finished=True)
        torch.cuda.synchronize()
        b, p, lm = b.cpu().numpy(), p.cpu().numpy(), lm.cpu().numpy()
        pol, val, act, st = pol.cpu().numpy(), val.cpu().numpy(), act.cpu().numpy(), st.cpu().numpy()
        for g in range(G):
            h = hist[g]
            o = np.zeros((3, 6, 6), np.float32)
            o[0], o[1] = b[g] == p[g], b[g] == -p[g]
            if lm[g] >= 0:
                o[2, lm[g] // 6, lm[g] % 6] = 1
            h["obs"].append(o), h["act"].append(int(act[g])), h["pol"].append(pol[g].copy())
            h["val"].append(np.float32(val[g])), h["brd"].append(b[g].copy())
            if st[g] != 2:
                want.append(R.build_game_record(h["obs"], h["act"], h["pol"], h["val"], h["brd"], int(st[g]),
                                                cfg.DISCOUNT, cfg.N_STEPS, cfg.NUM_UNROLL_STEPS))
                hist[g] = dict(obs=[], act=[], pol=[], val=[], brd=[])
    eng.close()
    assert len(got) == len(want) > 0

    def key(rec):
        return (len(rec.actions), tuple(rec.actions))
    got = sorted(((r, s) for r, s, _ in got), key=lambda x: key(x[0]))
    want = sorted(want, key=lambda x: key(x[0]))
    for (r1, s1), (r2, s2) in zip(got, want):
        assert r1.actions == r2.actions and r1.rewards == r2.rewards and r1.values == r2.values
        for f in ("observations", "policies", "board_states"):
            assert all(np.array_equal(x, y) for x, y in zip(getattr(r1, f), getattr(r2, f))), f
        for a, b in zip(s1, s2):
            for x, y in zip(a, b):
                assert np.array_equal(np.asarray(x), np.asarray(y))
