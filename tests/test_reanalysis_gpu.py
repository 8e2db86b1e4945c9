"""Re-analysis mode on the GPU: every position of stored games searched in
batched HIP searches equals the reference's sequential per-position search (the C oracle, pinned to
the reference's fixtures) with the same Gumbel noise; the win classes of the device scan equal
workers.py:49-123 on the host."""
import numpy as np
import pytest

import oracle
from test_reanalysis import _census, _playout

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mods():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from datou_gomoku_muzero_amd import engine as E, reanalysis as RA, records as R
    return E, RA, R


@pytest.mark.parametrize("mode,size,sims", [("MuZero", 9, 50), ("AlphaZero", 9, 50), ("MuZero", 15, 64)])
def test_batched_reanalysis_equals_sequential_oracle_searches(mods, mode, size, sims):
    E, RA, R = mods
    recs = [_playout(s, size, n) for s, n in ((4, 21), (5, 26), (6, 5))]
    P = sum(len(r.actions) for r in recs)
    rs = np.random.RandomState(17)
    gumbel = rs.gumbel(0, 1, (P, size * size))  # one draw of A per search, game then move (mcts.py:312)
    eng = E.BatchedSelfPlayEngine(None, num_games=16, BOARD_SIZE=size, NUM_SIMULATIONS=sims,
                                  MCTS_IMPLEMENTATION=mode)
    res = RA.Reanalyser(eng).reanalyse(recs, gumbel=gumbel)
    cfg = oracle.make_cfg(size, sims, mode)
    k = 0
    for rec, r in zip(recs, res):
        b, p, lm, mc = RA.positions_of(rec, size)
        for i in range(len(rec.actions)):
            opol, oval, oact, _, _ = oracle.search(cfg, b[i].reshape(-1), int(p[i]), None if lm[i] < 0 else int(lm[i]),
                                                   int(mc[i]), gumbel[k])
            assert float(r.values[i]) == float(oval), (k, r.values[i], oval)
            assert int(np.argmax(r.policies[i])) == int(np.argmax(opol))
            assert np.abs(r.policies[i] - opol).max() < 1e-12, k
            k += 1
        assert (r.corrected_fives, r.original_fives, r.corrected_totals, r.original_totals) == \
            _census(rec, r.policies, size)
        assert r.value_targets == R.compute_n_step_returns(np.array(rec.rewards, np.float32), list(r.values), 0.997, 10)
    eng.close()
