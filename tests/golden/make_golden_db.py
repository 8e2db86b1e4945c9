"""Golden fixtures for the on-disk record format, made with the REFERENCE's own
db_manager.py (this container only; /root/reference is never read at test time).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_db.py

Writes to tests/golden/:
  ref_records.db      a WAL-checkpointed SQLite file written by the reference's
                      DatabaseManager.add_game_and_slices for two scripted 6x6 games
  ref_records.npz     the games' payloads (the inputs handed to the reference), for comparison
  ours_read_by_ref.npz  what the reference's DatabaseManager decodes from a database written by
                      datou_gomoku_muzero_amd.formats.RecordStore for the same two games
"""
import os
import shutil
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)
sys.path.insert(0, REF)
for name in ("seaborn",):
    sys.modules.setdefault(name, types.ModuleType(name))
os.chdir(tempfile.mkdtemp(prefix="gmz_golden_db_"))

import db_manager as ref_db  # noqa: E402
from datou_gomoku_muzero_amd import formats as F  # noqa: E402
from datou_gomoku_muzero_amd import records as R  # noqa: E402

sys.path.insert(0, os.path.dirname(HERE))
from record_helpers import GAMES, VERSIONS, flat, scripted_game  # noqa: E402


def main():
    games = [scripted_game(R, *g) for g in GAMES]
    versions = list(VERSIONS)
    tmp = tempfile.mkdtemp()
    # 1. the reference writes
    path = os.path.join(tmp, "ref.db")
    mgr = ref_db.DatabaseManager(db_path=path)
    for (rec, sl), v in zip(games, versions):
        assert mgr.add_game_and_slices(rec, sl, v) is not None
    conn = ref_db.get_db_connection(path)
    conn.execute("PRAGMA wal_checkpoint(TRUNCATE);")
    conn.close()
    del ref_db.thread_local.connection
    shutil.copy(path, os.path.join(HERE, "ref_records.db"))
    payload = {"versions": np.array(versions)}
    for k, (rec, sl) in enumerate(games):
        payload.update(flat(rec, sl, k))
    np.savez_compressed(os.path.join(HERE, "ref_records.npz"), **payload)
    # 2. we write, the reference reads
    path2 = os.path.join(tmp, "ours.db")
    st = F.RecordStore(path2)
    for (rec, sl), v in zip(games, versions):
        assert st.add_game_and_slices(rec, sl, v) is not None
    st.close()
    mgr2 = ref_db.DatabaseManager(db_path=path2)
    got = {"buffer_size": np.array(mgr2.get_buffer_size())}
    for k in range(2):
        rec = mgr2.get_game_record_by_id(k + 1)
        n = len(rec.actions)
        sl = mgr2.load_latest_samples(100)
        sl = sl[:n] if k == 0 else sl[len(sl) - n:]
        got.update(flat(rec, sl, k))
    for key, val in got.items():
        if key in payload:
            assert np.array_equal(val, payload[key]), key
    np.savez_compressed(os.path.join(HERE, "ours_read_by_ref.npz"), **got)
    print("wrote ref_records.db (%d B), ref_records.npz, ours_read_by_ref.npz" %
          os.path.getsize(os.path.join(HERE, "ref_records.db")))


if __name__ == "__main__":
    main()
