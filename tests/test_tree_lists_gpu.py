"""Compact child lists (gmz_engine_cfg.flags bit 3, engine ``layout="lists"``) vs the dense layout.

A non-root node's edge row holds only its visited children ({action << 16 | child, N, W, R} entries in
first-visit order); a selection level works on its cached exp row and entries in a per-wave LDS buffer,
with the dense hint kernels' arithmetic on the same values in the same order (gmz_tree.hip
select_nonroot_cl; the lists always use the cached exp rows, the hint setting only switches the descent
prefetch).  So every search must equal the dense layout's with cached exp rows BIT FOR BIT — policy,
value, action, root visit counts, root N/W, MinMaxStats — with and without the prefetch, fused and split
entry points, 1- and 4-wave workgroups, every board size the kernels take (NJ = 1, 2, 4, 6, 8), including
the all-children-visited float32 path at non-root nodes (6x6 empty boards, near-uniform priors) and lists longer
than one wave (> 64 visited children: 9x9 / 2,000 sims with a flat network; both checked with
gmz_engine_max_visited_children).  The lists path is also checked directly against the reference's own MCTS fixtures
(tests/golden/mcts_*.npz) and the C oracle.
Reference: mcts.py:88-138 (select / backup), HashNet for tree parity independent of network floats.
"""
import glob
import os

import numpy as np
import pytest

import oracle
from conftest import GOLDEN

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

POLICY_ATOL = 1e-12
POLICY_ATOL_F32 = 1e-6


@pytest.fixture(scope="module")
def E():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import datou_gomoku_muzero_amd.engine as E
    return E


def _positions(size, G, rs, max_stones):
    A = size * size
    boards = np.zeros((G, A), np.int8)
    players = np.ones(G, np.int8)
    lastm = np.full(G, -1, np.int32)
    nst = rs.randint(0, max_stones + 1, G)
    for g in range(G):
        cells = rs.permutation(A)[:nst[g]]
        boards[g, cells[0::2]] = 1
        boards[g, cells[1::2]] = -1
        players[g] = 1 if nst[g] % 2 == 0 else -1
        lastm[g] = cells[-1] if nst[g] else -1
    return boards, players, lastm


MAX_NVIS = {}  # (size, sims, mode, G, layout) -> longest child list seen after any move


def _play(E, size, sims, mode, G, pos, gumbels, fuse=True, **kw):
    """len(gumbels) moves (search + play) from the positions; per move the search outputs + root stats."""
    eng = E.BatchedSelfPlayEngine(None, num_games=G, BOARD_SIZE=size, NUM_SIMULATIONS=sims, MCTS_IMPLEMENTATION=mode,
                                  **kw)
    eng.fuse_waves = fuse
    eng.set_positions(*pos)
    outs = []
    key = (size, sims, mode, G, eng.layout)
    for gm in gumbels:
        pol, val, act = eng.search(gumbel=gm)
        visits, rn, rw, mx, mn = eng.root_stats()
        torch.cuda.synchronize()
        outs.append([x.cpu().numpy().copy() for x in (pol, val, act, visits, rn, rw, mx, mn)])
        MAX_NVIS[key] = max(MAX_NVIS.get(key, 0), eng.max_visited_children())
        eng.play(reset_finished=True)
    eng.close()
    del eng
    torch.cuda.empty_cache()
    return outs


def _assert_same(a, b, what):
    for mv, (x, y) in enumerate(zip(a, b)):
        for k, (u, v) in enumerate(zip(x, y)):
            if not np.array_equal(u, v):
                rows = np.flatnonzero((u != v).reshape(len(u), -1).any(axis=1)) if u.ndim else []
                raise AssertionError("%s: move %d output %d differs in games %s" % (what, mv, k, list(rows[:20])))


@pytest.mark.parametrize("size,sims,mode,G,max_stones,moves", [
    (15, 400, "MuZero", 256, 224, 2),   # config C2's search, late games included
    (19, 800, "MuZero", 24, 300, 2),    # config C5's search (NJ = 6)
    (9, 50, "AlphaZero", 96, 80, 3),    # config C1 (NJ = 2)
    (6, 400, "MuZero", 64, 35, 2),      # NJ = 1
    (6, 400, "AlphaZero", 32, 35, 2),
    (22, 50, "MuZero", 9, 400, 2),      # NJ = 8, ragged G
    (15, 15, "MuZero", 128, 224, 3),    # tie-heavy tiny searches
    (9, 800, "MuZero", 16, 4, 1),       # deeper trees
])
@pytest.mark.parametrize("hint", [True, False])
def test_lists_equal_dense(E, size, sims, mode, G, max_stones, moves, hint):
    rs = np.random.RandomState(size * 100 + sims + G)
    pos = _positions(size, G, rs, max_stones)
    gumbels = [rs.gumbel(0, 1, (G, size * size)) for _ in range(moves)]
    dense = _play(E, size, sims, mode, G, pos, gumbels, descent_hint=True, layout="dense")
    lists = _play(E, size, sims, mode, G, pos, gumbels, descent_hint=hint, layout="lists")
    _assert_same(dense, lists, "lists (prefetch=%s) vs dense" % hint)
    nv = MAX_NVIS[(size, sims, mode, G, "lists")]
    assert nv == MAX_NVIS[(size, sims, mode, G, "dense")]  # the same trees



class _FlatNet:
    """A network with equal logits and zero values / rewards everywhere: the improved policy is uniform, so
    a node's visits go round-robin over its children and its list grows by one entry per visit."""

    def split(self, parts, max_grid=0):
        return [self] * parts

    def initial(self, obs, out_slot, logits, value, stream):
        logits.zero_()
        value.zero_()

    def recurrent(self, in_slot, action, out_slot, logits, value, reward, stream):
        logits.zero_()
        value.zero_()
        reward.zero_()


def test_lists_longer_than_one_wave(E):
    """A node with more than 64 visited children keeps entries past the wave's first 64 in HBM (read in each
    pass of select_nonroot_cl, appended by the backup at entry nvis >= 64): 9x9 empty boards, 2,000
    simulations with a flat network (every child tied: first-index tie breaks everywhere).  Lists == dense
    (cached exp rows) bit for bit, == the no-hint dense kernel (the reference's arithmetic) on every action,
    value and visit count, and the longest list exceeds 64 entries."""
    size, sims, G, mode = 9, 2000, 4, "MuZero"
    rs = np.random.RandomState(81)
    pos = _positions(size, G, rs, 0)
    gumbels = [rs.gumbel(0, 1, (G, size * size))]
    dense = _play(E, size, sims, mode, G, pos, gumbels, net=_FlatNet(), descent_hint=True, layout="dense")
    lists = _play(E, size, sims, mode, G, pos, gumbels, net=_FlatNet(), descent_hint=False, layout="lists")
    exact = _play(E, size, sims, mode, G, pos, gumbels, net=_FlatNet(), descent_hint=False, layout="dense")
    _assert_same(dense, lists, "lists vs dense, long lists")
    for k in (1, 2, 3, 4, 5, 6, 7):  # value, action, visits, root N/W, min/max (policy: within 1e-12)
        assert np.array_equal(lists[0][k], exact[0][k]), k
    assert np.abs(lists[0][0] - exact[0][0]).max() <= POLICY_ATOL
    assert MAX_NVIS[(size, sims, mode, G, "lists")] > 64, MAX_NVIS[(size, sims, mode, G, "lists")]


class _FlatLogitsNet(_FlatNet):
    """Equal logits, values hashed from the node slot in [-0.5, 0.5), zero rewards: with a small C_SCALE the
    improved policy stays nearly uniform, so nodes visit every child, while the values give MinMaxStats a
    range (the float32 array of _get_transformed_completed_Qs needs one, mcts.py:141-149)."""

    @staticmethod
    def _v(slot, value):
        h = (slot.to(torch.int64) * 2654435761) % 4093
        value.copy_(h.to(torch.float32) / 4093.0 - 0.5)

    def initial(self, obs, out_slot, logits, value, stream):
        logits.zero_()
        self._v(out_slot, value)

    def recurrent(self, in_slot, action, out_slot, logits, value, reward, stream):
        logits.zero_()
        self._v(out_slot, value)
        reward.zero_()


@pytest.mark.parametrize("mode", ["MuZero", "AlphaZero"])
def test_lists_all_children_visited_float32_rule(E, mode):
    """Non-root nodes whose every child is visited take the reference's float32 array path (mcts.py:141-156
    with no unvisited child; select_nonroot_cl's all-visited branch).  It needs an empty board (an occupied
    cell is a child never visited) and a node with more visits than children: 6x6 boards, 1,000 simulations,
    equal logits and C_SCALE = 1e-3 (_FlatLogitsNet).  Lists == dense (cached exp rows) bit for bit, == the
    no-hint dense kernel on every action, value and visit count, and the longest list holds all 36 children."""
    size, sims, G = 6, 1000, 8
    rs = np.random.RandomState(36)
    pos = _positions(size, G, rs, 0)  # empty boards
    gumbels = [rs.gumbel(0, 1, (G, size * size))]
    kw = dict(net=_FlatLogitsNet(), C_SCALE=1e-3)
    dense = _play(E, size, sims, mode, G, pos, gumbels, descent_hint=True, layout="dense", **kw)
    lists = _play(E, size, sims, mode, G, pos, gumbels, descent_hint=False, layout="lists", **kw)
    exact = _play(E, size, sims, mode, G, pos, gumbels, descent_hint=False, layout="dense", **kw)
    _assert_same(dense, lists, "lists vs dense, all children visited")
    for k in (1, 2, 3, 4, 5, 6, 7):
        assert np.array_equal(lists[0][k], exact[0][k]), k
    assert np.abs(lists[0][0] - exact[0][0]).max() <= POLICY_ATOL_F32
    assert MAX_NVIS[(size, sims, mode, G, "lists")] == size * size, MAX_NVIS[(size, sims, mode, G, "lists")]


@pytest.mark.parametrize("size,sims,mode,G", [(15, 400, "MuZero", 40), (9, 50, "AlphaZero", 24), (6, 400, "MuZero", 16)])
@pytest.mark.parametrize("hint", [True, False])
def test_lists_split_entry_points_equal_fused(E, size, sims, mode, G, hint):
    """gmz_engine_expand_backup + gmz_engine_select (k_expand_backup, k_select) on lists == the fused
    k_expand_select on lists == dense."""
    rs = np.random.RandomState(size + sims + 1)
    pos = _positions(size, G, rs, size * size - 1)
    gumbels = [rs.gumbel(0, 1, (G, size * size))]
    fused = _play(E, size, sims, mode, G, pos, gumbels, fuse=True, descent_hint=hint, layout="lists")
    split = _play(E, size, sims, mode, G, pos, gumbels, fuse=False, descent_hint=hint, layout="lists")
    dense = _play(E, size, sims, mode, G, pos, gumbels, fuse=False, descent_hint=True, layout="dense")
    _assert_same(fused, split, "fused vs split (lists)")
    _assert_same(split, dense, "lists vs dense (split entry points)")


MCTS_FILES = sorted(os.path.basename(f) for f in glob.glob(os.path.join(GOLDEN, "mcts_*.npz")))


@pytest.mark.parametrize("fname", MCTS_FILES)
@pytest.mark.parametrize("hint", [True, False])
def test_lists_match_reference_fixture(E, golden, fname, hint):
    d = golden(fname)
    size, mode, sims = int(d["size"]), str(d["mode"]), int(d["sims"])
    G = len(d["action"])
    out = _play(E, size, sims, mode, G, (d["board"], d["player"], d["lastmove"]), [d["gumbel"]],
                descent_hint=hint, layout="lists")[0]
    pol, val, act, visits, rn, rw, mx, mn = out
    assert (act == d["action"]).all(), (act, d["action"])
    assert (val == d["value"]).all()
    assert (visits == d["root_visits"]).all()
    assert (rn == d["root_n"]).all() and (rw == d["root_w"]).all()
    assert (mx == d["mm_max"]).all() and (mn == d["mm_min"]).all()
    assert np.abs(pol - d["policy"]).max() <= (POLICY_ATOL_F32 if size <= 6 else POLICY_ATOL)


@pytest.mark.parametrize("G,hint,wpb", [(4160, False, None),  # past 4,096 resident waves: 1-wave workgroups
                                        (4160, True, None),
                                        (1024, True, 1),      # forced 1-wave workgroups at C2's G
                                        (1024, False, 4)])
def test_lists_large_g_equal_dense_and_oracle(E, G, hint, wpb):
    size, sims = 15, 400
    rs = np.random.RandomState(G + 7)
    pos = _positions(size, G, rs, 120)
    gumbels = [rs.gumbel(0, 1, (G, size * size))]
    kw = dict(descent_hint=hint) if wpb is None else dict(descent_hint=hint, wpb=wpb)
    lists = _play(E, size, sims, "MuZero", G, pos, gumbels, layout="lists", **kw)
    dense = _play(E, size, sims, "MuZero", G, pos, gumbels, layout="dense", descent_hint=True)
    _assert_same(lists, dense, "lists vs dense at G=%d" % G)
    pol, val, act, visits, rn, rw, mx, mn = lists[0]
    boards, players, lastm = pos
    cfg = oracle.make_cfg(size, sims, "MuZero")
    bad = []
    for g in rs.choice(G, 32, replace=False):
        opol, oval, oact, orv, st = oracle.search(cfg, boards[g], players[g], None if lastm[g] < 0 else lastm[g],
                                                  int(np.count_nonzero(boards[g])), gumbels[0][g])
        if not (act[g] == oact and val[g] == oval and (visits[g] == orv).all() and rn[g] == st["root_n"]
                and rw[g] == st["root_w"] and mx[g] == st["mm_max"] and mn[g] == st["mm_min"]
                and np.abs(pol[g] - opol).max() <= POLICY_ATOL):
            bad.append(int(g))
    assert not bad, "games diverging from the oracle: %s" % bad


@pytest.mark.parametrize("layout,hint", [("dense", True), ("lists", False), ("dense", False)])
def test_deep_high_visit_trees_match_oracle(E, layout, hint):
    """Thousands of visits per node: the cached-exp softmax's factor exp(scale * (nq - nq0)), scale = c_visit +
    max N, would overflow float64 (it did: round 3's tools/deep_tree_probe.py showed the hint kernels off the
    oracle from 8,000 simulations, trees 74-156 deep); such levels now take the logits form (GMZ_EX_MAX_EXP).
    9x9 empty boards, 8,000 simulations (trees deeper than one wave), every kernel vs the C oracle."""
    size, sims, G = 9, 8000, 2
    rs = np.random.RandomState(8000)
    pos = _positions(size, G, rs, 0)
    gumbels = [rs.gumbel(0, 1, (G, size * size))]
    out = _play(E, size, sims, "MuZero", G, pos, gumbels, descent_hint=hint, layout=layout)[0]
    pol, val, act, visits, rn, rw, mx, mn = out
    boards, players, lastm = pos
    cfg = oracle.make_cfg(size, sims, "MuZero")
    for g in range(G):
        opol, oval, oact, orv, st = oracle.search(cfg, boards[g], players[g], None, 0, gumbels[0][g])
        assert st["max_depth"] > 64
        assert act[g] == oact and val[g] == oval and (visits[g] == orv).all(), (g, act[g], oact, val[g], oval)
        assert rn[g] == st["root_n"] and rw[g] == st["root_w"] and mx[g] == st["mm_max"] and mn[g] == st["mm_min"]
        assert np.abs(pol[g] - opol).max() <= POLICY_ATOL
