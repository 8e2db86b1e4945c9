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


def test_worker_mode1_reads_the_checkpoint_step(mods, tmp_path):
    """gpu_selfplay_worker in worker mode 1 (workers.py:243-305): the trainer step comes from the
    database's trainer_state checkpoint (workers.py:247-249; here the reference-format blob of a
    Trainer); both stored games are older than REANALYSIS_AGE_THRESHOLD steps, so both are re-analysed
    and stamped with that step."""
    import queue
    import shutil
    import os
    from conftest import GOLDEN
    from datou_gomoku_muzero_amd import formats as F, trainer as T
    from datou_gomoku_muzero_amd.config import GmzConfig
    from datou_gomoku_muzero_amd.worker import gpu_selfplay_worker
    db = str(tmp_path / "training_state.db")
    shutil.copy(os.path.join(GOLDEN, "ref_records.db"), db)
    tr = T.Trainer(T.TrainConfig(BOARD_SIZE=6, NUM_RES_BLOCKS=1), device="cpu")
    tr.step_count = 5000
    st = F.RecordStore(db)
    st.save_trainer_state(tr.trainer_state())
    st.close()

    class Mode:
        value = 1

    class Stop:  # shut down after a few loop checks
        def __init__(self):
            self.n = 0

        def is_set(self):
            self.n += 1
            return self.n > 2
    uq = queue.Queue()
    cfg = GmzConfig(BOARD_SIZE=6, NUM_SIMULATIONS=16, NUM_RES_BLOCKS=1)
    gpu_selfplay_worker(0, Mode(), queue.Queue(), None, uq, Stop(), num_games=8, cfg=cfg, db_path=db,
                        emit_move_notices=False)
    st = F.RecordStore(db)
    versions = sorted(v for _, v in st.conn.execute("SELECT game_id, analysis_version FROM games").fetchall())
    st.close()
    assert versions == [5000, 5000]
    assert sum(type(m).__name__ == "ReAnalysisStatus" for m in list(uq.queue)) == 2
