"""On-disk record format: datou_gomoku_muzero_amd.formats against a database
written by the reference's db_manager.py (tests/golden/ref_records.db, made by
tests/golden/make_golden_db.py) — both directions, byte for byte."""
import os
import pickle
import shutil
import sqlite3

import numpy as np
import pytest

from conftest import GOLDEN
from record_helpers import GAMES, VERSIONS, flat, scripted_game

from datou_gomoku_muzero_amd import formats as F
from datou_gomoku_muzero_amd import records as R

REF_DB = os.path.join(GOLDEN, "ref_records.db")


@pytest.fixture()
def ref_copy(tmp_path):
    p = str(tmp_path / "ref.db")
    shutil.copy(REF_DB, p)
    return p


def _games():
    return [scripted_game(R, *g) for g in GAMES]


def test_reads_reference_database(ref_copy, golden):
    want = golden("ref_records.npz")
    st = F.RecordStore(ref_copy)
    assert st.get_buffer_size() == sum(g[1] for g in GAMES)
    assert [(v, n, s) for _, v, n, s in st.games()] == [(VERSIONS[k], GAMES[k][1], "PENDING") for k in range(2)]
    slices = st.load_latest_samples(100)
    assert len(slices) == st.get_buffer_size()
    off = 0
    for k in range(2):
        rec = st.get_game_record_by_id(k + 1)
        n = len(rec.actions)
        got = flat(rec, slices[off:off + n], k)
        off += n
        for key, val in got.items():
            assert val.dtype == want[key].dtype and np.array_equal(val, want[key]), key
    st.close(checkpoint=False)


def test_blobs_byte_identical_to_reference(ref_copy, tmp_path):
    """Same games -> the same pickle bytes the reference stored; decode -> re-encode is the identity."""
    ref = sqlite3.connect(ref_copy)
    ref_games = [r[0] for r in ref.execute("SELECT game_record FROM games ORDER BY game_id")]
    ref_slices = [r[0] for r in ref.execute("SELECT slice_data FROM replay_buffer ORDER BY id")]
    for blob in ref_games + ref_slices:
        assert F.dumps(F.loads(blob)) == blob
    ours = str(tmp_path / "ours.db")
    st = F.RecordStore(ours)
    for (rec, sl), v in zip(_games(), VERSIONS):
        assert st.add_game_and_slices(rec, sl, v) is not None
    st.close()
    db = sqlite3.connect(ours)
    assert [r[0] for r in db.execute("SELECT game_record FROM games ORDER BY game_id")] == ref_games
    assert [r[0] for r in db.execute("SELECT slice_data FROM replay_buffer ORDER BY id")] == ref_slices
    meta = "SELECT game_id, analysis_version, move_count, status FROM games ORDER BY game_id"
    assert list(db.execute(meta)) == list(ref.execute(meta))
    meta = "SELECT id, game_id, move_index FROM replay_buffer ORDER BY id"
    assert list(db.execute(meta)) == list(ref.execute(meta))
    # same schema (table and index definitions)
    sch = "SELECT type, name, tbl_name, sql FROM sqlite_master WHERE name NOT LIKE 'sqlite_%' ORDER BY name"
    assert list(db.execute(sch)) == list(ref.execute(sch))


def test_reference_reads_our_database(golden):
    """tests/golden/ours_read_by_ref.npz = what the reference's DatabaseManager decoded from a
    RecordStore-written database (at generation time); it must equal the games we wrote."""
    got, want = golden("ours_read_by_ref.npz"), golden("ref_records.npz")
    assert int(got["buffer_size"]) == sum(g[1] for g in GAMES)
    for k in range(2):
        for key, val in flat(*_games()[k], k).items():
            assert np.array_equal(got[key], val) and np.array_equal(want[key], val), key


class _Evil:
    def __reduce__(self):
        return (os.system, ("echo pwned",))


@pytest.mark.parametrize("payload", [_Evil(), {"x": np.zeros(2)}, [eval]])
def test_restricted_unpickler_rejects_foreign_globals(payload):
    blob = pickle.dumps(payload, protocol=pickle.HIGHEST_PROTOCOL)
    with pytest.raises(F.UnsafeBlobError):
        F.loads(blob)


def test_trim_and_warmup_order(tmp_path):
    st = F.RecordStore(str(tmp_path / "t.db"))
    (rec, sl), _ = _games()
    for v in range(3):
        st.add_game_and_slices(rec, sl, v)
    assert st.get_buffer_size() == 3 * len(sl)
    last = st.load_latest_samples(len(sl) + 2)  # oldest first (db_manager.py:124-125)
    assert np.array_equal(last[-1].action_history, sl[-1].action_history)
    assert np.array_equal(last[2].action_history, sl[0].action_history)
    st.trim_buffer(1)  # reference semantics: games deleted, slices kept (no PRAGMA foreign_keys)
    assert st.games() == [] and st.get_buffer_size() == 3 * len(sl)
    st.close()


def test_replay_warmup_from_reference_database(ref_copy):
    """workers.py:388 warm-up: load_latest_samples -> the trainer's device replay buffer."""
    from datou_gomoku_muzero_amd import trainer as T
    st = F.RecordStore(ref_copy)
    slices = st.load_latest_samples(1000)
    cfg = T.TrainConfig(BOARD_SIZE=6, TRAIN_BUFFER_SIZE=64)
    rb = T.ReplayBuffer(cfg, device="cpu")
    rb.add(slices)
    assert len(rb) == len(slices)
    assert np.array_equal(rb.act[:len(slices)].numpy(), np.stack([s.action_history for s in slices]))
    assert np.array_equal(rb.pol[:len(slices)].numpy(), np.stack([s.policy_history for s in slices]).astype(np.float32))
    st.close(checkpoint=False)


def test_reference_trainer_state_resumes(golden, tmp_path):
    """The reference's trainer checkpoint (tests/golden/ref_trainer_state.db, written by its own
    DatabaseManager.save_trainer_state after 3 Adam steps; make_golden_trainer_state.py) decodes with
    the restricted loader and resumes a Trainer exactly: weights, Adam moments and steps, scheduler
    position (lr), train_step_count; our checkpoint round-trips through the same blob format."""
    import torch
    from datou_gomoku_muzero_amd import trainer as T
    d = golden("ref_trainer_state.npz")
    st = F.RecordStore(os.path.join(GOLDEN, "ref_trainer_state.db"))
    state = st.load_trainer_state()
    st.close(checkpoint=False)
    assert state["train_step_count"] == 1234 and state["games_completed_count"] == 56
    cfg = T.TrainConfig(BOARD_SIZE=6, NUM_RES_BLOCKS=1, NUM_FILTERS=8)
    tr = T.Trainer(cfg, device="cpu")
    assert [n for n, _ in tr.model.named_parameters()] == d["param_names"].tolist()  # optimiser index order
    tr.load_trainer_state(state)
    sd = tr.model.state_dict()
    for k in sd:
        a = sd[k].numpy()
        if "m/" + k in d.files:
            assert np.array_equal(a, d["m/" + k]), k
        else:
            f = a.astype(np.float64).ravel()
            want = d["ms/" + k]
            assert np.array_equal(f[:16], want[2:]) and np.isclose(f.sum(), want[0]) and np.isclose(np.square(f).sum(), want[1])
    ost = tr.opt.state_dict()["state"]
    for i in range(len(tr.params)):
        if "exp_avg/%d" % i in d.files:
            assert np.array_equal(ost[i]["exp_avg"].numpy(), d["exp_avg/%d" % i])
            assert np.array_equal(ost[i]["exp_avg_sq"].numpy(), d["exp_avg_sq/%d" % i])
            assert float(ost[i]["step"]) == float(d["step/%d" % i])
    assert tr.step_count == 1234 and abs(tr.opt.param_groups[0]["lr"] - float(d["lr"])) < 1e-15
    # our checkpoint in the reference's blob format round-trips
    st2 = F.RecordStore(str(tmp_path / "ours.db"))
    st2.save_trainer_state(tr.trainer_state())
    back = st2.load_trainer_state()
    st2.close()
    assert back["train_step_count"] == 1234
    for k, v in tr.model.state_dict().items():
        assert torch.equal(back["model_state_dict"][k], v)
    tr2 = T.Trainer(cfg, device="cpu")
    tr2.load_trainer_state(back)
    assert tr2.opt.param_groups[0]["lr"] == tr.opt.param_groups[0]["lr"]


def test_trainer_state_loader_rejects_other_globals():
    import pickle

    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))
    blob = pickle.dumps({"model_state_dict": {}, "x": Evil()})
    with pytest.raises(F.UnsafeBlobError):
        F.loads_trainer_state(blob)
