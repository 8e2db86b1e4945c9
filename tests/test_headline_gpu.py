"""The headline's composed path at its own size (BASELINE config 2 as bench.py runs it).

bench.py times ``engine.make_engine`` with its defaults at 15x15 / 400 simulations / 1,024 games: a
SplitSelfPlayEngine of two 512-game halves on two HIP streams, each half's 8-block f16 dynamics tower on
a grid capped at all CUs but engine.TOWER_FREE_CUS with ticket-scheduled boards, the dense tree rows with the descent hint,
the halves' waves interleaved.  Its pieces are pinned separately at full size elsewhere (the network in
test_net_gpu.py, the tree kernels with HashNet in test_tree_*_gpu.py); here the composition itself is
checked, from the headline's own start positions (engine.seeded_openings, as bench.py --stagger 80):
  (i)  two full moves, play() included, bit-identical to ONE BatchedSelfPlayEngine with the uncapped tower
       on the same weights and host Gumbel noise: every game's action, value, root visit counts, improved
       policy and status;
  (ii) 16 of those searches (8 per move, spread over the games and both halves) equal the C oracle's
       search (oracle/gmz_oracle.c, mcts.py:288-362) driving the SAME HIP network row by row.
"""
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


def _play(eng, noise):
    """Moves of ``eng`` with the given host Gumbel noise; per move the position searched and the outputs."""
    out = []
    for g in noise:
        pos = [t.cpu().numpy().copy() for t in eng.game_state()]
        pol, val, act = eng.search(gumbel=g)
        visits = eng.root_stats()[0]
        st = eng.play(reset_finished=True)
        torch.cuda.synchronize()
        out.append(dict(pos=pos, pol=pol.cpu().numpy().copy(), val=val.cpu().numpy().copy(),
                        act=act.cpu().numpy().copy(), visits=visits.cpu().numpy().copy(), st=st.cpu().numpy().copy()))
    return out


def test_headline_composed_path_at_its_own_size(mods):
    import oracle
    E, N, W, GmzConfig = mods
    size, sims, G = 15, 400, 1024
    A = size * size
    cfg = GmzConfig(BOARD_SIZE=size, NUM_SIMULATIONS=sims, MCTS_IMPLEMENTATION="MuZero", NUM_RES_BLOCKS=8)
    sd = W.synthetic_state_dict(cfg, seed=1234, with_projection=False)
    slots = G * (sims + 2)
    openings = E.seeded_openings(range(G), size, 1234, stagger=80)
    rs = np.random.RandomState(2024)
    noise = [rs.gumbel(0, 1, (G, A)) for _ in range(2)]

    # the bench's engine: make_engine's defaults for C2
    net2 = N.GomokuNetHip(sd, cfg, num_slots=slots, max_rows=G)
    two = E.make_engine(cfg, num_games=G, net=net2, seed=7)
    assert isinstance(two, E.SplitSelfPlayEngine) and two.parts == 2 and two.g == 512
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    assert all(e.net.w.max_grid == max(cus // 2, cus - E.TOWER_FREE_CUS) for e in two.engines)
    assert all(e.layout == "dense" and e.descent_hint for e in two.engines)
    two.reset_games()
    two.set_positions(*openings)
    got = _play(two, noise)
    two.close()
    del two, net2
    torch.cuda.empty_cache()

    # one engine, one stream, every CU
    net1 = N.GomokuNetHip(sd, cfg, num_slots=slots, max_rows=G)
    one = E.BatchedSelfPlayEngine(cfg, num_games=G, net=net1, seed=7)
    assert net1.w.max_grid == 0 and one.layout == "dense" and one.descent_hint
    one.reset_games()
    one.set_positions(*openings)
    want = _play(one, noise)
    one.close()
    del one, net1
    torch.cuda.empty_cache()

    for m, (a, b) in enumerate(zip(got, want)):
        for k in ("pos", "pol", "val", "act", "visits", "st"):
            if k == "pos":
                for x, y in zip(a[k], b[k]):
                    assert np.array_equal(x, y), ("move", m, k)
            else:
                assert np.array_equal(a[k], b[k]), ("move", m, k, np.flatnonzero(
                    (a[k] != b[k]).reshape(G, -1).any(1))[:8])
    assert (got[0]["visits"].sum(1) > 0).all()

    # (ii) the C oracle driving the same HIP network row by row
    onet = N.GomokuNetHip(sd, cfg, num_slots=4096, max_rows=16)
    nxt = [0]

    def alloc(n):
        s = list(range(nxt[0], nxt[0] + n))
        nxt[0] += n
        assert nxt[0] <= 4096
        return s

    def init(obs):
        s = alloc(obs.shape[0])
        lg, v, _ = onet.initial_inference(obs, slots=s)
        torch.cuda.synchronize()
        return lg.cpu().numpy(), v.cpu().numpy(), s

    def rec(hs, acts):
        s = alloc(len(hs))
        lg, v, r = onet.recurrent_inference(hs, acts, s)
        torch.cuda.synchronize()
        return lg.cpu().numpy(), v.cpu().numpy(), r.cpu().numpy(), s

    cb = oracle.CallbackNet(A, size, init, rec)
    ocfg = oracle.make_cfg(size, sims, "MuZero", hashnet=False)
    checked = 0
    for m, mv in enumerate(got):
        boards, players, lastm, counts = mv["pos"]
        for g in np.linspace(m * 61, G - 1 - m * 37, 8).astype(int):  # both halves, varied stone counts
            nxt[0] = 0
            cb.reset()
            lm = int(lastm[g])
            opol, oval, oact, orv, _ = oracle.search(ocfg, boards[g].reshape(-1), int(players[g]),
                                                     None if lm < 0 else lm, int(counts[g]), noise[m][g], net=cb)
            assert mv["act"][g] == oact and mv["val"][g] == oval and (mv["visits"][g] == orv).all(), (m, g)
            assert np.abs(mv["pol"][g] - opol).max() <= 1e-12, (m, g)
            checked += 1
    assert checked == 16


def test_c5_composed_path_at_its_own_size(mods):
    """BASELINE config 5 as bench.py's c5 sub-line runs it: 19x19, 800 simulations, GomokuNetEZ 16 blocks,
    1,024 games, engine.make_engine's default (one engine, one stream at 19x19: the single-image tower with
    its global residual scratch), from the headline's kind of start positions; 8 of its searches equal the
    C oracle driving the SAME HIP network row by row (mcts.py:288-362, network.py:137-152)."""
    import oracle
    E, N, W, GmzConfig = mods
    size, sims, G = 19, 800, 1024
    A = size * size
    cfg = GmzConfig(BOARD_SIZE=size, NUM_SIMULATIONS=sims, MCTS_IMPLEMENTATION="MuZero", NUM_RES_BLOCKS=16)
    sd = W.synthetic_state_dict(cfg, seed=77, with_projection=False)
    net = N.GomokuNetHip(sd, cfg, num_slots=E.hidden_slots(cfg, G), max_rows=G)
    eng = E.make_engine(cfg, num_games=G, net=net, seed=7)
    assert isinstance(eng, E.BatchedSelfPlayEngine)
    eng.reset_games()
    eng.set_positions(*E.seeded_openings(range(G), size, 77, stagger=80))
    noise = np.random.RandomState(5).gumbel(0, 1, (G, A))
    mv = _play(eng, [noise])[0]
    eng.close()
    del eng, net
    torch.cuda.empty_cache()
    onet = N.GomokuNetHip(sd, cfg, num_slots=4096, max_rows=16)
    nxt = [0]

    def alloc(n):
        s = list(range(nxt[0], nxt[0] + n))
        nxt[0] += n
        assert nxt[0] <= 4096
        return s

    def init(obs):
        s = alloc(obs.shape[0])
        lg, v, _ = onet.initial_inference(obs, slots=s)
        torch.cuda.synchronize()
        return lg.cpu().numpy(), v.cpu().numpy(), s

    def rec(hs, acts):
        s = alloc(len(hs))
        lg, v, r = onet.recurrent_inference(hs, acts, s)
        torch.cuda.synchronize()
        return lg.cpu().numpy(), v.cpu().numpy(), r.cpu().numpy(), s

    cb = oracle.CallbackNet(A, size, init, rec)
    ocfg = oracle.make_cfg(size, sims, "MuZero", hashnet=False)
    boards, players, lastm, counts = mv["pos"]
    for g in np.linspace(3, G - 5, 8).astype(int):
        nxt[0] = 0
        cb.reset()
        lm = int(lastm[g])
        opol, oval, oact, orv, _ = oracle.search(ocfg, boards[g].reshape(-1), int(players[g]), None if lm < 0 else lm,
                                                 int(counts[g]), noise[g], net=cb)
        assert mv["act"][g] == oact and mv["val"][g] == oval and (mv["visits"][g] == orv).all(), g
        assert np.abs(mv["pol"][g] - opol).max() <= 1e-12, g
