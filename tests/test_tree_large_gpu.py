"""Large-G parity of the fused expand/backup + select kernel (gmz_tree.hip ``k_expand_select``).

The kernel variant depends on the game count (engine.py, gmz_tree.hip launch_expand_select):
  * the engine's default: cached exp rows + descent prefetch, dense rows below 4,096 games per engine and
    compact child lists from 4,096 (tests/test_tree_lists_gpu.py); the no-hint dense kernel (the
    reference's exp(logit + t - max) softmax) on request;
  * 4-wave workgroups while every game has a resident wave, 1-wave workgroups once the games
    outnumber them.
The smaller-G tests (test_engine_gpu.py) never reach the 1-wave variants, so this file runs both at
sizes where the engine selects them on its own, 15x15 / 400 sims MuZero (config C2's search,
mcts.py:288-362) with HashNet (tree parity independent of network floating point):
  * every game bit-identical to the 4-wave launch of the same kernel (forced by gmz_engine_cfg.flags);
  * a sample of games bit-identical to the C oracle (oracle/gmz_oracle.c, pinned to the reference's
    fixtures by tests/test_oracle.py);
  * hint vs no-hint kernels at 4,096 games: the cached-exp softmax vs the logits path,
    the number of games whose search differs in any action / visit count (near-tie argmax flips).
"""
import numpy as np
import pytest

import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

POLICY_ATOL = 1e-12
SIZE, SIMS = 15, 400


@pytest.fixture(scope="module")
def E():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import datou_gomoku_muzero_amd.engine as E
    return E


def _positions(G, rs):
    """Random positions of every density (0..120 stones, alternating colours), host Gumbel noise."""
    A = SIZE * SIZE
    boards = np.zeros((G, A), np.int8)
    players = np.ones(G, np.int8)
    lastm = np.full(G, -1, np.int32)
    nst = rs.randint(0, 121, G)
    for g in range(G):
        cells = rs.permutation(A)[:nst[g]]
        boards[g, cells[0::2]] = 1
        boards[g, cells[1::2]] = -1
        players[g] = 1 if nst[g] % 2 == 0 else -1
        lastm[g] = cells[-1] if nst[g] else -1
    return boards, players, lastm, rs.gumbel(0, 1, (G, A))


def _search(E, G, pos, **kw):
    boards, players, lastm, gumbel = pos
    eng = E.BatchedSelfPlayEngine(None, num_games=G, BOARD_SIZE=SIZE, NUM_SIMULATIONS=SIMS,
                                  MCTS_IMPLEMENTATION="MuZero", **kw)
    eng.set_positions(boards, players, lastm)
    pol, val, act = eng.search(gumbel=gumbel)
    visits, rn, rw, mx, mn = eng.root_stats()
    torch.cuda.synchronize()
    out = dict(pol=pol.cpu().numpy(), val=val.cpu().numpy(), act=act.cpu().numpy(), visits=visits.cpu().numpy(),
               rn=rn.cpu().numpy(), rw=rw.cpu().numpy(), mx=mx.cpu().numpy(), mn=mn.cpu().numpy())
    eng.close()
    del eng
    torch.cuda.empty_cache()
    return out


def _differing_games(a, b):
    bad = np.zeros(len(a["act"]), bool)
    for k in ("act", "val", "rn", "rw", "mx", "mn"):
        bad |= a[k] != b[k]
    bad |= (a["visits"] != b["visits"]).any(axis=1)
    return np.flatnonzero(bad)


def _check_oracle(out, pos, games):
    boards, players, lastm, gumbel = pos
    cfg = oracle.make_cfg(SIZE, SIMS, "MuZero")
    bad = []
    for g in games:
        opol, oval, oact, orv, st = oracle.search(cfg, boards[g], players[g], None if lastm[g] < 0 else lastm[g],
                                                  int(np.count_nonzero(boards[g])), gumbel[g])
        ok = (out["act"][g] == oact and out["val"][g] == oval and (out["visits"][g] == orv).all()
              and out["rn"][g] == st["root_n"] and out["rw"][g] == st["root_w"] and out["mx"][g] == st["mm_max"]
              and out["mn"][g] == st["mm_min"] and np.abs(out["pol"][g] - opol).max() <= POLICY_ATOL)
        if not ok:
            bad.append(int(g))
    return bad


@pytest.mark.parametrize("G,hint", [(4160, False),   # the no-hint dense kernel past 4,096 resident waves
                                    (4160, True),    # the hint dense kernel there
                                    (2112, True)])   # the hint dense kernel past 2,048
def test_one_wave_workgroups_match_four_wave_and_oracle(E, G, hint):
    rs = np.random.RandomState(G)
    pos = _positions(G, rs)
    one = _search(E, G, pos, descent_hint=hint, wpb=1, layout="dense")
    four = _search(E, G, pos, descent_hint=hint, wpb=4, layout="dense")
    diff = _differing_games(one, four)
    assert len(diff) == 0, "games differing between 1-wave and 4-wave workgroups: %s" % diff[:20]
    assert np.array_equal(one["pol"], four["pol"])
    if hint:  # the engine's own choice at this G (lists from 4,096, cached-exp softmax): the same games
        dflt = _search(E, G, pos)
        assert len(_differing_games(dflt, one)) == 0 and np.array_equal(dflt["pol"], one["pol"])
    sample = rs.choice(G, 64, replace=False)
    bad = _check_oracle(one, pos, sample)
    assert not bad, "games diverging from the oracle: %s" % bad


def test_hint_and_no_hint_kernels_agree_at_4096_games(E):
    """The cached-exp softmax of the hint kernels (p ~ E * exp(t - t0)) and the no-hint kernel's
    exp(logit + t - max) differ by a few ulp; the first-index argmax over the scores could flip only on
    a near tie.  Count the games whose search differs anywhere (4,096 searches of 100 waves each)."""
    G = 4096
    rs = np.random.RandomState(4096)
    pos = _positions(G, rs)
    h = _search(E, G, pos, descent_hint=True, layout="dense")
    n = _search(E, G, pos, descent_hint=False, layout="dense")
    diff = _differing_games(h, n)
    print("hint vs no-hint at %d games: %d differing searches" % (G, len(diff)))
    assert len(diff) == 0, "near-tie flips between the two softmax forms in games %s" % diff[:20]
    assert np.abs(h["pol"] - n["pol"]).max() <= POLICY_ATOL
    bad = _check_oracle(h, pos, rs.choice(G, 32, replace=False))
    assert not bad, "hint kernel games diverging from the oracle: %s" % bad
