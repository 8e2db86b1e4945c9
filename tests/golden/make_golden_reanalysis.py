"""Golden fixture for the re-analysis bookkeeping, made with the REFERENCE's own
db_manager.py (this container only; /root/reference is never read at test time).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_reanalysis.py

Starting from the two scripted games of tests/record_helpers.py stored by the reference's
DatabaseManager (the state of tests/golden/ref_records.db), the reference performs:
  queue sizes at steps 903 / 904 / 908; lock at step 910 (-> game 1); finish_reanalysis_for_game(1,
  new policies, new value targets, 910); lock at step 910 again (-> game 2); unlock_game_on_error(2);
  queue size at 910.
Writes tests/golden/ref_reanalysed.db (the database afterwards, WAL checkpointed) and
tests/golden/reanalysis_inputs.npz (the new policies / value targets handed in, the answers).
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
os.chdir(tempfile.mkdtemp(prefix="gmz_golden_rean_"))

import db_manager as ref_db  # noqa: E402
from datou_gomoku_muzero_amd import records as R  # noqa: E402

sys.path.insert(0, os.path.dirname(HERE))
from record_helpers import A, GAMES, VERSIONS, scripted_game  # noqa: E402


def main():
    games = [scripted_game(R, *g) for g in GAMES]
    path = os.path.join(tempfile.mkdtemp(), "ref.db")
    mgr = ref_db.DatabaseManager(db_path=path)
    for (rec, sl), v in zip(games, VERSIONS):
        assert mgr.add_game_and_slices(rec, sl, v) is not None
    sizes = [mgr.get_reanalysis_queue_size(s) for s in (903, 904, 908)]
    gid, rec = mgr.sample_and_lock_game_for_reanalysis(910)
    assert gid == 1 and list(rec.actions) == list(games[0][0].actions)
    rs = np.random.RandomState(11)
    n = len(rec.actions)
    new_pol = [rs.dirichlet(np.ones(A)).astype(np.float64) for _ in range(n)]
    new_val = [np.float32(x) for x in rs.uniform(-1, 1, n)]
    targets = R.compute_n_step_returns(np.array(rec.rewards, dtype=np.float32), new_val, 0.997, 10)
    mgr.finish_reanalysis_for_game(gid, new_pol, targets, 910)
    gid2, _ = mgr.sample_and_lock_game_for_reanalysis(910)
    assert gid2 == 2
    mgr.unlock_game_on_error(gid2)
    sizes.append(mgr.get_reanalysis_queue_size(910))
    conn = ref_db.get_db_connection(path)
    conn.execute("PRAGMA wal_checkpoint(TRUNCATE);")
    conn.close()
    del ref_db.thread_local.connection
    shutil.copy(path, os.path.join(HERE, "ref_reanalysed.db"))
    np.savez_compressed(os.path.join(HERE, "reanalysis_inputs.npz"), new_policies=np.stack(new_pol),
                        new_values=np.array(new_val, np.float32), value_targets=np.array(targets, np.float64),
                        queue_sizes=np.array(sizes))
    print("queue sizes", sizes, "wrote ref_reanalysed.db (%d B)" % os.path.getsize(os.path.join(HERE, "ref_reanalysed.db")))


if __name__ == "__main__":
    main()
