"""engine.SplitSelfPlayEngine — G games as two half-size engines on two HIP streams with a capped
tower grid — must play exactly the games one BatchedSelfPlayEngine plays: same device Gumbel noise
per game (game_offset), same trees, same network rows.  Checked bit-for-bit move after move with
HashNet (tree path) and with the HIP GomokuNetEZ (tower grid capped, workspaces per stream), in
both search modes, including hot-swapped weights and the state-copy entry points."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mods():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import datou_gomoku_muzero_amd.engine as E
    import datou_gomoku_muzero_amd.network as N
    import datou_gomoku_muzero_amd.weights as W
    from datou_gomoku_muzero_amd.config import GmzConfig
    return E, N, W, GmzConfig


def _moves(eng, n, gumbel_rs=None):
    out = []
    for _ in range(n):
        g = None if gumbel_rs is None else gumbel_rs.gumbel(0, 1, (eng.G, eng.A))
        pol, val, act = eng.search(gumbel=g)
        st = eng.play(reset_finished=True)
        torch.cuda.synchronize()
        out.append((pol.cpu().numpy().copy(), val.cpu().numpy().copy(), act.cpu().numpy().copy(),
                    st.cpu().numpy().copy()))
    return out


def _same(a, b):
    for m, (x, y) in enumerate(zip(a, b)):
        for k, (u, v) in enumerate(zip(x, y)):
            assert np.array_equal(u, v), ("move", m, "field", k)


@pytest.mark.parametrize("mode,size,sims", [("MuZero", 9, 50), ("AlphaZero", 9, 30), ("MuZero", 15, 64)])
def test_split_equals_single_hashnet(mods, mode, size, sims):
    E, N, W, GmzConfig = mods
    cfg = GmzConfig(BOARD_SIZE=size, NUM_SIMULATIONS=sims, MCTS_IMPLEMENTATION=mode)
    G = 12
    one = E.BatchedSelfPlayEngine(cfg, num_games=G, seed=5)
    two = E.SplitSelfPlayEngine(cfg, num_games=G, seed=5, parts=2)
    one.reset_games()
    two.reset_games()
    _same(_moves(one, 12), _moves(two, 12))
    ct1, ct2 = one.tree_counters(), two.tree_counters()
    assert ct1 == ct2
    for x, y in zip(one.game_state(), two.game_state()):
        assert torch.equal(x, y)
    for x, y in zip(one.root_stats(), two.root_stats()):
        assert torch.equal(x, y)


@pytest.mark.parametrize("mode", ["MuZero", "AlphaZero"])
def test_split_equals_single_hip_net(mods, mode):
    E, N, W, GmzConfig = mods
    cfg = GmzConfig(BOARD_SIZE=9, NUM_SIMULATIONS=24, MCTS_IMPLEMENTATION=mode, NUM_RES_BLOCKS=2)
    G = 10
    sd = W.synthetic_state_dict(cfg, seed=3, with_projection=False)
    slots = G * (cfg.NUM_SIMULATIONS + 2)
    net1 = N.GomokuNetHip(sd, cfg, num_slots=slots, max_rows=G)
    net2 = N.GomokuNetHip(sd, cfg, num_slots=slots, max_rows=G)
    one = E.BatchedSelfPlayEngine(cfg, num_games=G, net=net1, seed=11)
    two = E.SplitSelfPlayEngine(cfg, num_games=G, net=net2, seed=11, parts=2, max_grid=3)
    one.reset_games()
    two.reset_games()
    rs1, rs2 = np.random.RandomState(4), np.random.RandomState(4)
    _same(_moves(one, 5, rs1), _moves(two, 5, rs2))
    # ModelWeightsUpdate on the parent net reaches both streams' views
    sd2 = W.synthetic_state_dict(cfg, seed=8, with_projection=False)
    net1.load_state_dict(sd2)
    net2.load_state_dict(sd2)
    _same(_moves(one, 4), _moves(two, 4))


def test_split_positions_and_masks(mods):
    E, N, W, GmzConfig = mods
    cfg = GmzConfig(BOARD_SIZE=9, NUM_SIMULATIONS=40, MCTS_IMPLEMENTATION="MuZero")
    G = 8
    rs = np.random.RandomState(0)
    boards = np.zeros((G, 9, 9), np.int8)
    players = np.ones(G, np.int8)
    for g in range(G):  # a few random stones, alternating colours
        cells = rs.choice(81, 2 * (g % 4), replace=False)
        boards[g].flat[cells[0::2]] = 1
        boards[g].flat[cells[1::2]] = -1
    last = np.full(G, -1, np.int32)
    one = E.BatchedSelfPlayEngine(cfg, num_games=G, seed=2)
    two = E.SplitSelfPlayEngine(cfg, num_games=G, seed=2, parts=2)
    for e in (one, two):
        e.set_positions(boards, players, last)
    _same(_moves(one, 3), _moves(two, 3))
    mask = (np.arange(G) % 3 == 0).astype(np.uint8)
    one.reset_games(mask)
    two.reset_games(mask)
    acts = np.array([(g * 7) % 81 for g in range(G)], np.int32)
    for e in (one, two):
        e.search()
        e.play(action=acts, reset_finished=False)
    torch.cuda.synchronize()
    for x, y in zip(one.game_state(), two.game_state()):
        assert torch.equal(x, y)
    _same(_moves(one, 2), _moves(two, 2))


def test_split_with_another_layout_plays_the_same_games(mods):
    """At 4,096 games one engine runs the compact child lists (engine.default_layout: G >= 4096; without
    the prefetch) and two halves of 2,048 the dense rows with the hint kernels: the cached-exp softmax in
    both, so the split engine plays the one engine's games bit for bit (15x15 / 64 sims MuZero, HashNet,
    device Gumbel noise)."""
    E, N, W, GmzConfig = mods
    cfg = GmzConfig(BOARD_SIZE=15, NUM_SIMULATIONS=64, MCTS_IMPLEMENTATION="MuZero")
    G = 4096
    one = E.BatchedSelfPlayEngine(cfg, num_games=G, seed=9)
    two = E.SplitSelfPlayEngine(cfg, num_games=G, seed=9, parts=2)
    assert one.layout == "lists" and all(e.layout == "dense" for e in two.engines)
    assert not one.descent_hint and all(e.descent_hint for e in two.engines)
    one.reset_games()
    two.reset_games()
    _same(_moves(one, 3), _moves(two, 3))
    one.close()
    two.close()
