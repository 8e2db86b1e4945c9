"""Re-analysis mode, host side: RecordStore's re-analysis bookkeeping against the
reference's own db_manager.py (tests/golden/ref_reanalysed.db, made by
tests/golden/make_golden_reanalysis.py), and the Reanalyser's position mapping / missed-win census
(workers.py:256-288) with a stand-in engine.  The batched searches are checked on the GPU in
tests/test_reanalysis_gpu.py."""
import os
import shutil
import sqlite3
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from record_helpers import GAMES

from datou_gomoku_muzero_amd import formats as F
from datou_gomoku_muzero_amd import reanalysis as RA
from datou_gomoku_muzero_amd import records as R


def _rows(path):
    db = sqlite3.connect(path)
    out = (list(db.execute("SELECT game_id, game_record, analysis_version, move_count, status FROM games "
                           "ORDER BY game_id")),
           list(db.execute("SELECT id, game_id, move_index, slice_data FROM replay_buffer ORDER BY id")))
    db.close()
    return out


def test_reanalysis_bookkeeping_matches_reference(tmp_path, golden):
    inp = golden("reanalysis_inputs.npz")
    p = str(tmp_path / "db.db")
    shutil.copy(os.path.join(GOLDEN, "ref_records.db"), p)  # the reference's database before re-analysis
    st = F.RecordStore(p)
    sizes = [st.get_reanalysis_queue_size(s) for s in (903, 904, 908)]
    gid, rec = st.sample_and_lock_game_for_reanalysis(910)
    assert gid == 1
    targets = R.compute_n_step_returns(np.array(rec.rewards, dtype=np.float32), list(inp["new_values"]), 0.997, 10)
    assert np.array_equal(np.array(targets, np.float64), inp["value_targets"])
    assert st.finish_reanalysis_for_game(gid, list(inp["new_policies"]), targets, 910)
    gid2, _ = st.sample_and_lock_game_for_reanalysis(910)
    assert gid2 == 2
    st.unlock_game_on_error(gid2)
    sizes.append(st.get_reanalysis_queue_size(910))
    assert sizes == list(inp["queue_sizes"])
    st.close()
    got, want = _rows(p), _rows(os.path.join(GOLDEN, "ref_reanalysed.db"))
    assert got[0] == want[0]  # games: blobs, versions, DONE / PENDING
    assert got[1] == want[1]  # every slice blob byte-identical (rewritten windows included)


def test_batched_lock_equals_sequential_locks(tmp_path):
    a, b = str(tmp_path / "a.db"), str(tmp_path / "b.db")
    for q in (a, b):
        shutil.copy(os.path.join(GOLDEN, "ref_records.db"), q)
    sa, sb = F.RecordStore(a), F.RecordStore(b)
    seq = [sa.sample_and_lock_game_for_reanalysis(2000)[0] for _ in range(3)]
    bat = [g for g, _ in sb.sample_and_lock_games_for_reanalysis(2000, limit=3)]
    assert seq == [1, 2, None] and bat == [1, 2]
    assert sa.games() == sb.games()
    sa.close(), sb.close()


def test_finish_failure_unlocks(tmp_path):
    p = str(tmp_path / "db.db")
    shutil.copy(os.path.join(GOLDEN, "ref_records.db"), p)
    st = F.RecordStore(p)
    gid, rec = st.sample_and_lock_game_for_reanalysis(2000)
    # too few policies: the window for the last move_index does not exist -> rollback, PENDING again
    assert not st.finish_reanalysis_for_game(gid, [np.zeros(36)], [0.0], 2000, unroll_steps=0)
    assert [s for g, _, _, s in st.games() if g == gid] == ["PENDING"]
    st.close()


class _FakeEngine:
    """Stand-in for BatchedSelfPlayEngine on the CPU: the 'search' policy puts all mass on a
    scripted cell per position; winning_scan is the host restatement of workers.py:49-123."""

    def __init__(self, G, S, choose):
        self.G, self.size, self.A, self.device = G, S, S * S, torch.device("cpu")
        self.choose, self.loaded, self.calls = choose, None, 0

    def set_positions(self, b, p, lm, mc):
        self.loaded = (b.copy(), p.copy(), lm.copy(), mc.copy())

    def search(self, gumbel=None):
        b, p, lm, mc = self.loaded
        pol = torch.zeros(self.G, self.A, dtype=torch.float64)
        act = torch.zeros(self.G, dtype=torch.int32)
        for i in range(self.G):
            a = self.choose(b[i], int(p[i]), int(lm[i]), int(mc[i]))
            pol[i, a], act[i] = 1.0, a
        self.calls += 1
        return pol, torch.from_numpy(mc.astype(np.float32) / 100), act

    def winning_scan(self, boards, players):
        cls = np.zeros((self.G, self.A), np.uint8)
        for i in range(self.G):
            w = R.find_winning_moves(boards[i].numpy(), int(players[i]))
            for k, name in ((1, "five"), (2, "open_four"), (3, "combo")):
                for r, c in w[name]:
                    cls[i, r * self.size + c] = k
        return torch.from_numpy(cls)


def _census(rec, new_pol, S):
    """workers.py:270-288 verbatim semantics on the host."""
    of = cf = ot = ct = 0
    for i in range(len(rec.actions)):
        p = 1 if i % 2 == 0 else -1
        w = R.find_winning_moves(np.asarray(rec.board_states[i]).copy(), p)
        allw = w["five"] + w["open_four"] + w["combo"]
        if not allw:
            continue
        orig = (rec.actions[i] // S, rec.actions[i] % S)
        if orig not in allw:
            ot += 1
            five = bool(w["five"])
            of += five
            nm = int(np.argmax(new_pol[i]))
            if (nm // S, nm % S) in allw:
                ct += 1
                cf += five
    return cf, of, ct, ot


def _playout(seed, S, n):
    """A game whose moves build lines (so wins appear and are missed)."""
    rs = np.random.RandomState(seed)
    obs, acts, pols, vals, boards = [], [], [], [], []
    b = np.zeros(S * S, np.int8)
    p = 1
    for m in range(n):
        empty = np.flatnonzero(b == 0)
        own = np.flatnonzero(b == p)
        if len(own) and rs.rand() < 0.7:
            near = [c + d for c in own for d in (1, S, S + 1) if 0 <= c + d < S * S and b[c + d] == 0]
            a = int(rs.choice(near)) if near else int(rs.choice(empty))
        else:
            a = int(rs.choice(empty))
        obs.append(np.zeros((3, S, S), np.float32))
        pols.append(np.full(S * S, 1.0 / (S * S)))
        vals.append(np.float32(0))
        acts.append(a)
        boards.append(b.reshape(S, S).copy())
        b[a] = p
        p = -p
    return R.build_game_record(obs, acts, pols, vals, boards, 0)[0]


def test_reanalyser_positions_and_census():
    S = 9
    recs = [_playout(s, S, n) for s, n in ((1, 23), (2, 30), (3, 7))]

    def choose(b, p, lm, mc):  # a deterministic 'search': first winning cell if any, else first empty cell
        w = R.find_winning_moves(b, p)
        allw = w["five"] + w["open_four"] + w["combo"]
        if allw:
            return allw[0][0] * S + allw[0][1]
        return int(np.flatnonzero(b.reshape(-1) == 0)[0])
    eng = _FakeEngine(8, S, choose)
    res = RA.Reanalyser(eng).reanalyse(recs, discount=0.997, n_steps=10)
    assert eng.calls == -(-60 // 8)  # 60 positions in batches of G = 8
    tot = 0
    for rec, r in zip(recs, res):
        n = len(rec.actions)
        assert r.policies.shape == (n, S * S) and r.values.dtype == np.float32
        assert np.allclose(r.values, np.arange(n) / 100)  # move_count = i (workers.py:259)
        b, p, lm, mc = RA.positions_of(rec, S)
        assert list(p) == [1 if i % 2 == 0 else -1 for i in range(n)]
        assert list(lm) == [-1] + list(rec.actions[:-1])
        assert r.value_targets == R.compute_n_step_returns(np.array(rec.rewards, np.float32), list(r.values), 0.997, 10)
        assert (r.corrected_fives, r.original_fives, r.corrected_totals, r.original_totals) == _census(rec, r.policies, S)
        tot += r.original_totals
    assert tot > 0  # the scripted games do miss wins


def test_reanalysis_step_end_to_end_cpu(tmp_path):
    """Lock -> batched re-analysis -> slices rewritten -> DONE, one ReAnalysisStatus per game."""
    S = 6
    p = str(tmp_path / "db.db")
    shutil.copy(os.path.join(GOLDEN, "ref_records.db"), p)
    st = F.RecordStore(p)
    eng = _FakeEngine(4, S, lambda b, pl, lm, mc: int(np.flatnonzero(b.reshape(-1) == 0)[-1]))
    cfg = SimpleNamespace(REANALYSIS_AGE_THRESHOLD=900, DISCOUNT=0.997, N_STEPS=10, NUM_UNROLL_STEPS=5)

    class Q(list):
        put = list.append
    q = Q()
    assert RA.reanalysis_step(RA.Reanalyser(eng), st, 2000, cfg, max_games=8, ui_queue=q) == 2
    assert [s for *_, s in st.games()] == ["DONE", "DONE"] and [v for _, v, _, _ in st.games()] == [2000, 2000]
    assert len(q) == 2 and all(m.total_reanalyzed == 1 for m in q)
    sl = st.load_latest_samples(100)
    assert len(sl) == sum(g[1] for g in GAMES)
    rec0 = st.get_game_record_by_id(1)
    first = sl[0]  # game 1, move 0: window of the new policies of moves 0..5
    want = np.zeros((6, S * S))
    for i in range(6):
        b = np.asarray(rec0.board_states[i]).reshape(-1)
        want[i, np.flatnonzero(b == 0)[-1]] = 1.0
    assert np.array_equal(first.policy_history, want) and first.policy_history.dtype == np.float64
    assert RA.reanalysis_step(RA.Reanalyser(eng), st, 2000, cfg) == 0  # nothing PENDING any more
    st.close()
