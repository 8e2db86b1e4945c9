"""Pin the C oracle (oracle/gmz_oracle.c) against fixtures produced by running the REFERENCE
(tests/golden/make_golden.py).  CPU only."""
import glob
import os

import numpy as np
import pytest

import oracle
import hashnet
from conftest import GOLDEN

SIZES = (6, 9, 15, 19)


@pytest.mark.parametrize("size", SIZES)
def test_game_steps_match_reference(golden, size):
    """game.py:12-23,25-63 — obs planes, legal set, do_move, check_win, get_game_ended."""
    d = golden("game_cases.npz")
    p = "s%d_" % size
    boards, moves = d[p + "boards"], d[p + "moves"]
    for i in range(len(moves)):
        b = boards[i].copy()
        lm = int(d[p + "lastmove"][i])
        obs = oracle.board_state(b, size, int(d[p + "players"][i]), None if lm < 0 else lm)
        assert (obs.reshape(3, -1).astype(np.uint8) == d[p + "obs"][i]).all()
        assert ((b == 0).astype(np.uint8) == d[p + "valid"][i]).all()
        mv = int(moves[i])
        b[mv] = d[p + "players"][i]
        assert oracle.check_win(b, size, mv // size, mv % size) == bool(d[p + "wins"][i])
        mc = int(np.count_nonzero(b))
        e = oracle.game_ended(b, size, mv, mc)
        assert (2 if e is None else e) == int(d[p + "ended"][i])


@pytest.mark.parametrize("size", SIZES)
def test_check_win_every_cell(golden, size):
    d = golden("game_cases.npz")
    p = "s%d_" % size
    for b, w in zip(d[p + "rand_boards"], d[p + "rand_wins"]):
        got = np.array([oracle.check_win(b, size, a // size, a % size) for a in range(size * size)], np.uint8)
        assert (got == w).all()


def test_set_order_matches_cpython():
    rs = np.random.RandomState(1)
    for t in range(3000):
        A = (36, 81, 225, 361)[t % 4]
        keys = sorted(rs.choice(A, rs.randint(1, A + 1), replace=False).tolist())
        assert oracle.set_order(keys).tolist() == list({k for k in keys})


def test_hashnet_c_matches_numpy():
    rs = np.random.RandomState(2)
    for t in range(50):
        obs = (rs.rand(3, 15, 15) < 0.2).astype(np.float32)
        hid = hashnet.initial_id(obs)
        assert oracle.hash_initial_id(obs) == hid
        a = int(rs.randint(225))
        assert oracle.hash_recurrent_id(hid, a) == hashnet.recurrent_id(hid, a)
        lg, v, r = oracle.hash_outputs(hid, 225)
        assert (lg == hashnet.logits_of(hid, 225)).all()
        assert v == hashnet.value_of(hid) and r == hashnet.reward_of(hid)


MCTS_FILES = sorted(os.path.basename(f) for f in glob.glob(os.path.join(GOLDEN, "mcts_*.npz")))


@pytest.mark.parametrize("fname", MCTS_FILES)
def test_search_matches_reference(golden, fname):
    """mcts.py:197-362 driven by HashNet: bit-exact action/value/visits/W/min-max; policy ≤1e-12."""
    d = golden(fname)
    size, mode, sims = int(d["size"]), str(d["mode"]), int(d["sims"])
    if size == 19 and sims == 800 and os.environ.get("GMZ_FAST"):
        pytest.skip("fast mode")
    cfg = oracle.make_cfg(size, sims, mode)
    for i in range(len(d["action"])):
        lm = int(d["lastmove"][i])
        pol, val, act, rv, st = oracle.search(cfg, d["board"][i], d["player"][i], None if lm < 0 else lm,
                                              d["movecount"][i], d["gumbel"][i])
        assert act == d["action"][i]
        assert val == d["value"][i]
        assert (rv == d["root_visits"][i]).all()
        assert st["root_n"] == d["root_n"][i] and st["root_w"] == d["root_w"][i]
        assert st["mm_max"] == d["mm_max"][i] and st["mm_min"] == d["mm_min"][i]
        assert st["n_initial"] == d["n_initial"][i] and st["recurrent_rows"] == d["recurrent_rows"][i]
        assert np.abs(pol - d["policy"][i]).max() <= 1e-12
        assert abs(pol.sum() - 1.0) < 1e-9


def test_callback_net_equals_builtin_hashnet(golden):
    """The callback path (used with real nets) reproduces the built-in HashNet path."""
    d = golden("mcts_mz9_50.npz")
    hn = hashnet.HashNet(81)

    def init(obs):
        p, v, h = hn.initial(obs)
        return p, v[:, 0], list(h[:, 0])

    def rec(hs, acts):
        p, v, h, r = hn.recurrent(np.array(hs, np.uint32), acts)
        return p, v[:, 0], r[:, 0], list(h[:, 0])
    net = oracle.CallbackNet(81, 9, init, rec)
    cfg = oracle.make_cfg(9, 50, "MuZero", hashnet=False)
    for i in range(2):
        lm = int(d["lastmove"][i])
        pol, val, act, rv, st = oracle.search(cfg, d["board"][i], d["player"][i], None if lm < 0 else lm,
                                              d["movecount"][i], d["gumbel"][i], net=net)
        assert act == d["action"][i] and val == d["value"][i] and (rv == d["root_visits"][i]).all()
