"""Scripted self-play games with the worker's per-move payload types (worker.py:142-146), shared by
tests/test_formats.py and tests/golden/make_golden_db.py (which feeds the same games to the
reference's db_manager.py)."""
import numpy as np

H, A = 6, 36
GAMES = ((1, 9, 1), (2, 12, 0))  # (seed, moves, winner)
VERSIONS = (3, 7)


def scripted_game(R, seed, n_moves, winner):
    """-> records.build_game_record(...) of a random 6x6 game (R = the records module)."""
    rs = np.random.RandomState(seed)
    cells = rs.permutation(A)[:n_moves]
    b = np.zeros(A, np.int8)
    obs, acts, pols, vals, boards = [], [], [], [], []
    p, last = 1, -1
    for c in cells:
        o = np.zeros((3, H, H), np.float32)
        o[0] = (b == p).reshape(H, H)
        o[1] = (b == -p).reshape(H, H)
        if last >= 0:
            o[2].reshape(-1)[last] = 1
        obs.append(o)
        pols.append(rs.dirichlet(np.ones(A)).astype(np.float64))
        vals.append(np.float32(rs.uniform(-1, 1)))
        acts.append(int(c))
        boards.append(b.reshape(H, H).copy())
        b[c] = p
        p, last = -p, int(c)
    return R.build_game_record(obs, acts, pols, vals, boards, winner)


def flat(record, slices, k):
    """Game k's record + slices as named arrays."""
    out = {"g%d_actions" % k: np.array(record.actions), "g%d_rewards" % k: np.array(record.rewards, np.float32),
           "g%d_values" % k: np.array(record.values, np.float32), "g%d_obs" % k: np.stack(record.observations),
           "g%d_policies" % k: np.stack(record.policies), "g%d_boards" % k: np.stack(record.board_states)}
    for f in slices[0]._fields:
        out["g%d_slice_%s" % (k, f)] = np.stack([getattr(s, f) for s in slices])
    return out
