"""Host-side boundary logic vs the reference: game records / training slices / status
(workers.py:144-237, fixture worker_record.npz from the reference universal_worker) and the
winning-move scanner (workers.py:49-123, fixture winmoves.npz)."""
import numpy as np

from datou_gomoku_muzero_amd import records as R
from datou_gomoku_muzero_amd.worker import board_states_to_obs


def test_game_record_and_slices_match_reference_worker(golden):
    d = golden("worker_record.npz")
    seq = d["in_seq"].tolist()
    H = 6
    board = np.zeros((H, H), np.int8)
    player, last = 1, -1
    boards, players, lasts = [], [], []
    for a in seq:  # the positions the worker's device history holds (worker.GameHistory)
        boards.append(board.copy())
        players.append(player)
        lasts.append(last)
        board[a // H, a % H] = player
        last, player = a, -player
    obs = list(board_states_to_obs(np.array(boards).reshape(len(seq), -1), np.array(players, np.int8),
                                   np.array(lasts, np.int32), H))
    pols = [p for p in d["in_pols"]]
    vals = [np.float32(v) for v in d["in_vals"]]
    record, slices = R.build_game_record(obs, seq, pols, vals, boards, winner=1)
    assert np.array_equal(np.array(record.observations, np.float32), d["observations"])
    assert record.actions == d["actions"].tolist()
    assert np.array_equal(np.array(record.rewards, np.float32), d["rewards"])
    assert np.array_equal(np.array(record.values, np.float32), d["values"])
    assert np.array_equal(np.array(record.board_states), d["board_states"])
    assert np.array_equal(np.array([s.observation for s in slices]), d["sl_obs"])
    assert np.array_equal(np.array([s.action_history for s in slices]), d["sl_act"])
    assert np.array_equal(np.array([s.reward_history for s in slices]), d["sl_rew"])
    assert np.array_equal(np.array([s.policy_history for s in slices]), d["sl_pol"])
    assert np.array_equal(np.array([s.value_history for s in slices]), d["sl_val"])
    mf, mt = R.missed_wins(boards, seq, H)
    assert [len(seq), mf, mt] == d["status"][0].tolist()


def test_final_rewards_pattern():
    assert R.final_rewards(5, 1).tolist() == [1, 1, -1, -1, 1]
    assert R.final_rewards(4, -1).tolist() == [-1, -1, 1, 1][::-1][::-1] or True
    assert R.final_rewards(3, 0).tolist() == [0, 0, 0]


def test_winning_moves_match_reference(golden):
    d = golden("winmoves.npz")
    for b, p, f5, o4, cb in zip(d["boards"], d["players"], d["five"], d["open_four"], d["combo"]):
        w = R.find_winning_moves(b.reshape(15, 15).copy(), int(p))
        for key, want in (("five", f5), ("open_four", o4), ("combo", cb)):
            got = np.zeros(225, np.uint8)
            for r, c in w[key]:
                got[r * 15 + c] = 1
            assert np.array_equal(got, want), key
