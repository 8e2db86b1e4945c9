"""Two waves per game in the fused expand/select kernel (k_expand_select_pair, gmz_engine_cfg.flags bit 4;
MuZero, dense rows with the descent hint, 15x15) against the reference's MCTS fixtures, the C oracle
(HashNet: tree parity isolated from network drift) and the one-wave kernel.

Exact: action, root value, root visit counts, root N/W, MinMaxStats.  Improved policy |Δ| <= 1e-12 (the
softmax denominator is the sum of the two half-row partial sums: a few ulp)."""
import glob
import os

import numpy as np
import pytest

import oracle
from conftest import GOLDEN

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def E():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import datou_gomoku_muzero_amd.engine as E
    return E


def _engine(E, size, sims, G, pair=True, **kw):
    eng = E.BatchedSelfPlayEngine(None, num_games=G, BOARD_SIZE=size, NUM_SIMULATIONS=sims,
                                  MCTS_IMPLEMENTATION="MuZero", pair=pair, **kw)
    assert eng.pair == pair
    return eng


def _run(eng, boards, players, lastm, gumbel):
    eng.set_positions(boards, players, lastm)
    pol, val, act = eng.search(gumbel=gumbel)
    visits, rn, rw, mx, mn = eng.root_stats()
    torch.cuda.synchronize()
    return [x.cpu().numpy() for x in (pol, val, act, visits, rn, rw, mx, mn)]


def _positions(size, G, rs, max_stones):
    A = size * size
    boards = np.zeros((G, A), np.int8)
    players = np.ones(G, np.int8)
    lastm = np.full(G, -1, np.int32)
    for g in range(G):
        n = int(rs.randint(0, max_stones + 1))
        cells = rs.permutation(A)[:n]
        p = 1
        for c in cells:
            boards[g, c] = p
            p = -p
        players[g] = p
        lastm[g] = cells[-1] if n else -1
    return boards, players, lastm


def _vs_oracle(size, sims, boards, players, lastm, gumbel, out):
    pol, val, act, visits, rn, rw, mx, mn = out
    cfg = oracle.make_cfg(size, sims, "MuZero")
    bad = []
    for g in range(len(act)):
        opol, oval, oact, orv, st = oracle.search(cfg, boards[g], players[g], None if lastm[g] < 0 else lastm[g],
                                                  int(np.count_nonzero(boards[g])), gumbel[g])
        ok = (act[g] == oact and val[g] == oval and (visits[g] == orv).all() and rn[g] == st["root_n"]
              and rw[g] == st["root_w"] and mx[g] == st["mm_max"] and mn[g] == st["mm_min"]
              and np.abs(pol[g] - opol).max() <= 1e-12)
        if not ok:
            bad.append(g)
    return bad


@pytest.mark.parametrize("fname", sorted(os.path.basename(f) for f in glob.glob(os.path.join(GOLDEN, "mcts_*.npz"))))
def test_pair_matches_reference_fixtures(E, golden, fname):
    d = golden(fname)
    size, mode, sims = int(d["size"]), str(d["mode"]), int(d["sims"])
    if mode != "MuZero" or not 128 < size * size <= 256:
        pytest.skip("the two-wave kernel covers MuZero at 129..256 actions")
    eng = _engine(E, size, sims, len(d["action"]))
    pol, val, act, visits, rn, rw, mx, mn = _run(eng, d["board"], d["player"], d["lastmove"], d["gumbel"])
    assert (act == d["action"]).all() and (val == d["value"]).all() and (visits == d["root_visits"]).all()
    assert (rn == d["root_n"]).all() and (rw == d["root_w"]).all()
    assert (mx == d["mm_max"]).all() and (mn == d["mm_min"]).all()
    assert np.abs(pol - d["policy"]).max() <= 1e-12


@pytest.mark.parametrize("sims,G,max_stones", [(400, 96, 224), (15, 64, 224), (400, 5, 224), (64, 130, 120)])
def test_pair_matches_oracle_random_positions(E, sims, G, max_stones):
    size = 15
    rs = np.random.RandomState(4242 + sims + G)
    boards, players, lastm = _positions(size, G, rs, max_stones)
    gumbel = rs.gumbel(0, 1, (G, size * size))
    out = _run(_engine(E, size, sims, G), boards, players, lastm, gumbel)
    bad = _vs_oracle(size, sims, boards, players, lastm, gumbel, out)
    assert not bad, "games diverging from the oracle: %s" % bad


def test_pair_deep_high_visit_trees_match_oracle(E):
    """Thousands of simulations from near-empty boards: deep trees whose visit counts push levels onto the
    rare paths (the logits form past GMZ_EX_MAX_EXP, children all visited), which both waves run on the
    whole row as the one-wave kernel does."""
    size, sims, G = 15, 3000, 4
    rs = np.random.RandomState(9)
    boards, players, lastm = _positions(size, G, rs, 6)
    gumbel = rs.gumbel(0, 1, (G, size * size))
    out = _run(_engine(E, size, sims, G), boards, players, lastm, gumbel)
    bad = _vs_oracle(size, sims, boards, players, lastm, gumbel, out)
    assert not bad, "games diverging from the oracle: %s" % bad


def test_pair_plays_the_one_wave_kernels_games(E):
    """Self-play move after move (device Gumbel noise, play() with restarts) with the two-wave and the
    one-wave kernel: the same actions, values, visit counts and game states; policies within 1e-12."""
    size, sims, G = 15, 100, 256
    outs = []
    for pair in (True, False):
        eng = _engine(E, size, sims, G, pair=pair, seed=5)
        eng.set_positions(*E.seeded_openings(range(G), size, 5, stagger=80)[:3])
        moves = []
        for _ in range(6):
            pol, val, act = eng.search()
            visits = eng.root_stats()[0]
            st = eng.play(reset_finished=True)
            torch.cuda.synchronize()
            moves.append([x.cpu().numpy().copy() for x in (pol, val, act, visits, st)])
        outs.append(moves)
        eng.close()
    for m, (a, b) in enumerate(zip(*outs)):
        assert np.abs(a[0] - b[0]).max() <= 1e-12, m
        for k in range(1, 5):
            assert np.array_equal(a[k], b[k]), (m, k)
