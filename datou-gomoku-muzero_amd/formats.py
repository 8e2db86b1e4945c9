"""On-disk format of the self-play records: the reference's SQLite store.

``RecordStore`` reads and writes the schema of db_manager.py:37-73 — tables ``games`` (pickled
``GameRecord`` blob, analysis_version, move_count, status, timestamp), ``replay_buffer`` (one pickled
``TrainingSlice`` blob per move) and ``trainer_state`` — in WAL mode (db_manager.py:19-26), so a
database written by ``gpu_selfplay_worker``'s records can be resumed by the reference and vice versa.

Blobs are written exactly as the reference writes them (``pickle.dumps(obj, HIGHEST_PROTOCOL)`` of
``data_structures.GameRecord`` / ``TrainingSlice`` namedtuples holding numpy arrays), and read with a
RESTRICTED unpickler that resolves only those two classes and numpy's array / dtype / scalar
constructors: a blob naming anything else is rejected, never executed.  The ``trainer_state`` blob
(a pickled dict of torch state_dicts and optimiser / scheduler state, db_manager.py:231-243) is read
by ``load_trainer_state`` with a second restricted unpickler: only ``collections.OrderedDict``,
torch's tensor rebuild function and its storage constructor resolve, and the storage bytes are
decoded by ``torch.load(weights_only=True)`` (the reference's pickled storages otherwise go through
``torch.storage._load_from_bytes``, an unrestricted ``torch.load``); the result must be the
reference's dict of tensors, numbers, strings and containers.  ``save_trainer_state`` writes the
reference's own blob (``pickle.dumps`` of that dict).

Re-analysis bookkeeping (db_manager.py:151-227): eligible-game count, lock of the oldest eligible
game(s), the sliding-window rewrite of a re-analysed game's slices (same blobs as the reference's
``finish_reanalysis_for_game``), unlock on error.  The search itself is ``reanalysis.py``.
"""
import io
import os
from collections import deque
import pickle
import sqlite3
import sys
import types

import numpy as np

from . import records as R

_SCHEMA = (
    # db_manager.py:40-48
    """CREATE TABLE IF NOT EXISTS games (
                    game_id INTEGER PRIMARY KEY AUTOINCREMENT,
                    game_record BLOB NOT NULL,
                    analysis_version INTEGER NOT NULL,
                    move_count INTEGER NOT NULL,
                    status TEXT DEFAULT 'PENDING' NOT NULL,
                    timestamp DATETIME DEFAULT CURRENT_TIMESTAMP
                )""",
    "CREATE INDEX IF NOT EXISTS status_version_idx ON games (status, analysis_version);",
    # db_manager.py:52-60
    """CREATE TABLE IF NOT EXISTS replay_buffer (
                    id INTEGER PRIMARY KEY AUTOINCREMENT,
                    game_id INTEGER NOT NULL,
                    move_index INTEGER NOT NULL,
                    slice_data BLOB NOT NULL,
                    FOREIGN KEY (game_id) REFERENCES games (game_id) ON DELETE CASCADE
                )""",
    "CREATE INDEX IF NOT EXISTS game_id_idx ON replay_buffer (game_id);",
    # db_manager.py:64-69
    """CREATE TABLE IF NOT EXISTS trainer_state (
                    key TEXT PRIMARY KEY,
                    state_blob BLOB
                )""",
)


def _record_classes():
    """(GameRecord, TrainingSlice) pickled under the module name ``data_structures``, as the
    reference's own classes are (data_structures.py:9-26).  Inside the reference project those ARE
    the classes (records.py imports them); standalone, records.py's field-identical namedtuples are
    published under that module name so that blobs name the same class path."""
    G, T = R.GameRecord, R.TrainingSlice
    if G.__module__ != "data_structures":
        mod = sys.modules.get("data_structures")
        if mod is None:
            mod = types.ModuleType("data_structures")
            mod.__doc__ = "stand-in published by datou_gomoku_muzero_amd.formats (reference not importable)"
            sys.modules["data_structures"] = mod
        if getattr(mod, "GameRecord", None) is None:
            G.__module__ = T.__module__ = "data_structures"
            mod.GameRecord, mod.TrainingSlice = G, T
        G, T = mod.GameRecord, mod.TrainingSlice
    return G, T


_NUMPY_GLOBALS = {
    # ndarray (protocol 5: _frombuffer; older protocols: _reconstruct + ndarray), dtype, scalars
    ("numpy._core.numeric", "_frombuffer"), ("numpy.core.numeric", "_frombuffer"),
    ("numpy._core.multiarray", "_reconstruct"), ("numpy.core.multiarray", "_reconstruct"),
    ("numpy._core.multiarray", "scalar"), ("numpy.core.multiarray", "scalar"),
    ("numpy", "ndarray"), ("numpy", "dtype"),
}


class UnsafeBlobError(pickle.UnpicklingError):
    pass


class _RecordUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if module == "data_structures" and name in ("GameRecord", "TrainingSlice"):
            G, T = _record_classes()
            return G if name == "GameRecord" else T
        if (module, name) in _NUMPY_GLOBALS:
            return super().find_class(module, name)
        raise UnsafeBlobError("blob references %s.%s: only GameRecord / TrainingSlice and numpy arrays are "
                              "decoded" % (module, name))


def loads(blob):
    """Decode a games / replay_buffer blob (restricted: nothing outside the record classes and
    numpy's array constructors is resolved)."""
    obj = _RecordUnpickler(io.BytesIO(bytes(blob))).load()
    if not isinstance(obj, _record_classes()):
        raise UnsafeBlobError("blob holds a %s, not a GameRecord / TrainingSlice" % type(obj).__name__)
    return obj


def dumps(obj):
    """Encode a GameRecord / TrainingSlice exactly as db_manager.py:82,90 does."""
    G, T = _record_classes()
    if type(obj).__name__ == "GameRecord" and not isinstance(obj, G):
        obj = G(*obj)
    elif type(obj).__name__ == "TrainingSlice" and not isinstance(obj, T):
        obj = T(*obj)
    return pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)


def _storage_from_bytes(b):
    """torch.storage._load_from_bytes restated with the weights-only loader."""
    import torch
    return torch.load(io.BytesIO(b), weights_only=True)


class _TrainerStateUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        import collections
        import torch
        if (module, name) == ("collections", "OrderedDict"):
            return collections.OrderedDict
        if (module, name) == ("torch._utils", "_rebuild_tensor_v2"):
            return torch._utils._rebuild_tensor_v2
        if (module, name) == ("torch.storage", "_load_from_bytes"):
            return _storage_from_bytes
        raise UnsafeBlobError("trainer_state blob references %s.%s: only tensors, OrderedDict and plain "
                              "containers are decoded" % (module, name))

    def persistent_load(self, pid):
        raise UnsafeBlobError("trainer_state blob uses persistent ids (not a plain pickle of a dict)")


def _check_plain(obj, depth=0):
    import torch
    if depth > 16:
        raise UnsafeBlobError("trainer_state nests too deep")
    if isinstance(obj, dict):
        for k, v in obj.items():
            _check_plain(k, depth + 1)
            _check_plain(v, depth + 1)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            _check_plain(v, depth + 1)
    elif not (obj is None or isinstance(obj, (bool, int, float, str, bytes, torch.Tensor))):
        raise UnsafeBlobError("trainer_state holds a %s" % type(obj).__name__)


def loads_trainer_state(blob):
    """Decode a trainer_state blob (db_manager.py:238-243) without executing anything it names."""
    obj = _TrainerStateUnpickler(io.BytesIO(bytes(blob))).load()
    if not isinstance(obj, dict) or "model_state_dict" not in obj:
        raise UnsafeBlobError("trainer_state blob is not the reference's state dict")
    _check_plain(obj)
    return obj


def dumps_trainer_state(state):
    """Encode as db_manager.py:233 does: pickle.dumps(state_dict, HIGHEST_PROTOCOL)."""
    return pickle.dumps(state, protocol=pickle.HIGHEST_PROTOCOL)


class RecordStore:
    """db_manager.DatabaseManager's persistence API for game records and training slices."""

    def __init__(self, db_path="outputs/training_state.db"):
        self.db_path = db_path
        d = os.path.dirname(db_path)
        if d:
            os.makedirs(d, exist_ok=True)
        self.conn = sqlite3.connect(db_path, check_same_thread=False, timeout=10)
        self.conn.execute("PRAGMA journal_mode=WAL;")
        self.conn.execute("PRAGMA synchronous=NORMAL;")
        with self.conn:
            for stmt in _SCHEMA:
                self.conn.execute(stmt)

    def close(self, checkpoint=True):
        if checkpoint:  # fold the WAL into the main file (a single self-contained .db)
            self.conn.execute("PRAGMA wal_checkpoint(TRUNCATE);")
        self.conn.close()

    def add_game_and_slices(self, game_record, prepared_slices, model_version):
        """db_manager.py:75-104: one transaction; returns the new game_id (None on failure)."""
        try:
            with self.conn:
                cur = self.conn.cursor()
                cur.execute("INSERT INTO games (game_record, analysis_version, move_count) VALUES (?, ?, ?)",
                            (dumps(game_record), model_version, len(game_record.actions)))
                gid = cur.lastrowid
                cur.executemany("INSERT INTO replay_buffer (game_id, move_index, slice_data) VALUES (?, ?, ?)",
                                [(gid, i, dumps(s)) for i, s in enumerate(prepared_slices)])
            return gid
        except sqlite3.Error:
            return None

    def get_game_record_by_id(self, game_id):
        """db_manager.py:106-112."""
        row = self.conn.execute("SELECT game_record FROM games WHERE game_id = ?", (game_id,)).fetchone()
        return loads(row[0]) if row else None

    def load_latest_samples(self, num_samples):
        """db_manager.py:114-127: the newest slices, returned oldest first (replay warm-up)."""
        rows = self.conn.execute("SELECT slice_data FROM replay_buffer ORDER BY id DESC LIMIT ?",
                                 (num_samples,)).fetchall()
        return [loads(r[0]) for r in reversed(rows)]

    def get_buffer_size(self):
        """db_manager.py:129-132."""
        return self.conn.execute("SELECT COUNT(*) FROM replay_buffer").fetchone()[0]

    def trim_buffer(self, capacity):
        """db_manager.py:134-147: past `capacity` slices, delete (up to) the 100 oldest games.  As in
        the reference the slices stay (no PRAGMA foreign_keys, so ON DELETE CASCADE is inert)."""
        if self.get_buffer_size() > capacity:
            ids = self.conn.execute("SELECT game_id FROM games ORDER BY timestamp ASC LIMIT ?", (100,)).fetchall()
            if ids:
                with self.conn:
                    self.conn.execute("DELETE FROM games WHERE game_id IN (%s)" % ",".join("?" * len(ids)),
                                      [g[0] for g in ids])

    def games(self):
        """(game_id, analysis_version, move_count, status) of every stored game, oldest first."""
        return self.conn.execute("SELECT game_id, analysis_version, move_count, status FROM games "
                                 "ORDER BY game_id").fetchall()

    # ---------------------------------------------------------------- re-analysis (db_manager.py:151-227)
    def get_reanalysis_queue_size(self, current_trainer_step, age_threshold=900):
        """db_manager.py:151-161: PENDING games whose analysis is more than ``age_threshold``
        trainer steps old (config.py:89 REANALYSIS_AGE_THRESHOLD)."""
        return self.conn.execute("SELECT COUNT(*) FROM games WHERE status = 'PENDING' AND ? - analysis_version > ?",
                                 (current_trainer_step, age_threshold)).fetchone()[0]

    def sample_and_lock_games_for_reanalysis(self, current_trainer_step, age_threshold=900, limit=1):
        """db_manager.py:163-181 for up to ``limit`` games in one transaction: the oldest-analysed
        eligible games, marked RUNNING -> [(game_id, GameRecord)].  Same games, in the same order,
        as ``limit`` successive single-game calls."""
        with self.conn:
            rows = self.conn.execute(
                "SELECT game_id, game_record FROM games WHERE status = 'PENDING' AND ? - analysis_version > ? "
                "ORDER BY analysis_version ASC LIMIT ?", (current_trainer_step, age_threshold, int(limit))).fetchall()
            self.conn.executemany("UPDATE games SET status = 'RUNNING' WHERE game_id = ?", [(r[0],) for r in rows])
        return [(gid, loads(blob)) for gid, blob in rows]

    def sample_and_lock_game_for_reanalysis(self, current_trainer_step, age_threshold=900):
        """db_manager.py:163-181 -> (game_id, GameRecord) or (None, None)."""
        got = self.sample_and_lock_games_for_reanalysis(current_trainer_step, age_threshold, 1)
        return got[0] if got else (None, None)

    def finish_reanalysis_for_game(self, game_id, new_policies, new_value_targets, new_analysis_version,
                                   unroll_steps=5):
        """db_manager.py:183-221: windows of ``unroll_steps + 1`` new policies / value targets
        (zero-padded past the end) replace each stored slice's policy_history / value_history; the
        game becomes DONE at ``new_analysis_version``.  On failure the game goes back to PENDING
        and False is returned."""
        k = unroll_steps + 1
        num_moves = len(new_policies)
        pol_q, val_q = deque(maxlen=k), deque(maxlen=k)
        pi_hists, val_hists = [], []
        for i in range(num_moves + k - 1):
            if i < num_moves:
                pol_q.append(new_policies[i])
                val_q.append(new_value_targets[i])
            else:
                pol_q.append(np.zeros_like(new_policies[0]))
                val_q.append(0.0)
            if i >= k - 1:
                pi_hists.append(np.array(pol_q))
                val_hists.append(np.array(val_q, dtype=np.float32))
        try:
            with self.conn:
                rows = self.conn.execute("SELECT id, move_index, slice_data FROM replay_buffer WHERE game_id = ? "
                                         "ORDER BY move_index ASC", (game_id,)).fetchall()
                upd = [(dumps(loads(blob)._replace(policy_history=pi_hists[mi], value_history=val_hists[mi])), sid)
                       for sid, mi, blob in rows]
                self.conn.executemany("UPDATE replay_buffer SET slice_data = ? WHERE id = ?", upd)
                self.conn.execute("UPDATE games SET analysis_version = ?, status = 'DONE' WHERE game_id = ?",
                                  (new_analysis_version, game_id))
            return True
        except Exception:
            with self.conn:
                self.conn.execute("UPDATE games SET status = 'PENDING' WHERE game_id = ?", (game_id,))
            return False

    def save_trainer_state(self, state):
        """db_manager.py:231-236: the whole trainer state as one blob (INSERT OR REPLACE)."""
        self.conn.execute("INSERT OR REPLACE INTO trainer_state (key, state_blob) VALUES (?, ?)",
                          ("singleton_state", dumps_trainer_state(state)))
        self.conn.commit()

    def load_trainer_state(self):
        """db_manager.py:238-243 (restricted decoding: ``loads_trainer_state``); None when absent."""
        row = self.conn.execute("SELECT state_blob FROM trainer_state WHERE key = ?", ("singleton_state",)).fetchone()
        return loads_trainer_state(row[0]) if row else None

    def unlock_game_on_error(self, game_id):
        """db_manager.py:223-227."""
        if game_id is None:
            return
        with self.conn:
            self.conn.execute("UPDATE games SET status = 'PENDING' WHERE game_id = ?", (game_id,))
