"""Re-analysis mode: stored games searched again with the current network.

The reference's ``universal_worker`` in worker mode 1 (workers.py:243-305) takes ONE game at a time
from the database (db_manager.py:163-181), runs ``mcts_engine.search`` position after position
(move ``i`` = ``board_states[i]``, player ``+1`` on even moves, last move ``actions[i-1]``,
move_count ``i``; workers.py:256-265), recomputes the n-step value targets from the new search values
(workers.py:290-291), rewrites the game's slices (db_manager.py:183-221) and reports how many
missed wins the new policies correct (workers.py:270-288, ``ReAnalysisStatus``).

Here the positions of MANY games are searched in one batch on the HIP engine: every position is an
independent search, so P positions fill ceil(P / G) batched searches of G games (the tail batch is
padded with empty boards whose results are dropped).  The missed-win census runs on the device with
the batched winning-move scan (``gmz_game_winning_scan``), one launch per batch.  The per-position
results are those of the reference's sequential searches with the same Gumbel noise (tested against
the oracle in tests/test_reanalysis_gpu.py).
"""
from dataclasses import dataclass

import numpy as np
import torch

from . import records as R


@dataclass
class ReanalysedGame:
    """One game's re-analysis: new search policies f64[n, A] and values f32[n], the n-step value
    targets written to the slices, and the workers.py:270-288 correction counters."""
    policies: np.ndarray
    values: np.ndarray
    value_targets: list
    corrected_fives: int
    original_fives: int
    corrected_totals: int
    original_totals: int


def positions_of(record, board_size):
    """workers.py:256-262 -> boards int8[n,S,S], players int8[n], last_moves int32[n] (-1 none),
    move_counts int32[n] for every move of a stored game."""
    n = len(record.actions)
    S = board_size
    boards = np.stack([np.asarray(b, dtype=np.int8).reshape(S, S) for b in record.board_states[:n]]) if n else \
        np.zeros((0, S, S), np.int8)
    players = np.array([1 if i % 2 == 0 else -1 for i in range(n)], dtype=np.int8)
    last = np.array([-1] + [int(a) for a in record.actions[:n - 1]], dtype=np.int32)[:n]
    return boards, players, last, np.arange(n, dtype=np.int32)


class Reanalyser:
    """Batched re-analysis on a ``BatchedSelfPlayEngine`` (its G games are the batch)."""

    def __init__(self, engine):
        self.eng = engine
        self.G, self.S, self.A = engine.G, engine.size, engine.A

    def search_positions(self, boards, players, last_moves, move_counts, gumbel=None):
        """Independent searches of P positions -> (policy f64[P,A], value f32[P], action int32[P],
        win classes uint8[P,A] of the position for the player to move: 0 none, 1 five,
        2 open_four, 3 combo).  ``gumbel``: optional f64[P,A] root noise (default: the engine's
        device noise)."""
        eng, G, S, A = self.eng, self.G, self.S, self.A
        P = len(boards)
        pol = np.zeros((P, A), np.float64)
        val = np.zeros(P, np.float32)
        act = np.full(P, -1, np.int32)
        cls = np.zeros((P, A), np.uint8)
        for lo in range(0, P, G):
            n = min(G, P - lo)
            b = np.zeros((G, S, S), np.int8)
            p = np.ones(G, np.int8)
            lm = np.full(G, -1, np.int32)
            mc = np.zeros(G, np.int32)
            b[:n], p[:n], lm[:n], mc[:n] = boards[lo:lo + n], players[lo:lo + n], last_moves[lo:lo + n], \
                move_counts[lo:lo + n]
            eng.set_positions(b, p, lm, mc)
            g = None
            if gumbel is not None:
                g = np.zeros((G, A), np.float64)
                g[:n] = gumbel[lo:lo + n]
            pt, vt, at = eng.search(gumbel=g)
            bd = torch.from_numpy(b).to(eng.device)
            ct = eng.winning_scan(bd, torch.from_numpy(p).to(eng.device))
            if eng.device.type == "cuda":
                torch.cuda.synchronize()
            pol[lo:lo + n] = pt[:n].cpu().numpy()
            val[lo:lo + n] = vt[:n].cpu().numpy()
            act[lo:lo + n] = at[:n].cpu().numpy()
            cls[lo:lo + n] = ct[:n].cpu().numpy()
        bad = act < 0  # no legal move: mcts.py returns (zeros, 0.0, -1)
        pol[bad], val[bad] = 0.0, 0.0
        return pol, val, act, cls

    def reanalyse(self, records, gumbel=None, discount=0.997, n_steps=10):
        """Re-analyse whole games -> [ReanalysedGame].  ``gumbel``: optional f64[total positions, A]
        in game-then-move order (the order of the reference's sequential searches)."""
        per = [positions_of(r, self.S) for r in records]
        counts = [len(x[0]) for x in per]
        if sum(counts) == 0:
            return [ReanalysedGame(np.zeros((0, self.A)), np.zeros(0, np.float32), [], 0, 0, 0, 0) for _ in records]
        cat = [np.concatenate([x[k] for x in per]) for k in range(4)]
        pol, val, act, cls = self.search_positions(*cat, gumbel=gumbel)
        out, off = [], 0
        for rec, n in zip(records, counts):
            p, v, c = pol[off:off + n], val[off:off + n], cls[off:off + n]
            of = ot = cf = ct = 0
            for i in range(n):  # workers.py:270-288
                wins = c[i] != 0
                if not wins.any():
                    continue
                if not wins[int(rec.actions[i])]:
                    ot += 1
                    five = bool((c[i] == 1).any())
                    of += five
                    if wins[int(np.argmax(p[i]))]:
                        ct += 1
                        cf += five
            rewards = np.array(rec.rewards, dtype=np.float32)
            targets = R.compute_n_step_returns(rewards, list(v), discount, n_steps) if n else []
            out.append(ReanalysedGame(p, v, targets, cf, of, ct, ot))
            off += n
        return out


def reanalysis_step(reanalyser, store, current_trainer_step, cfg, max_games=64, ui_queue=None, gumbel=None):
    """One pass of worker mode 1 (workers.py:248-305) over up to ``max_games`` games at once:
    lock the oldest eligible games, re-analyse them in batched searches, rewrite their slices
    (RecordStore.finish_reanalysis_for_game) and post one ``ReAnalysisStatus`` per game.  Returns
    the number of games re-analysed (0: nothing eligible).  Locked games are unlocked on error."""
    locked = store.sample_and_lock_games_for_reanalysis(current_trainer_step, cfg.REANALYSIS_AGE_THRESHOLD,
                                                        max_games)
    if not locked:
        return 0
    try:
        res = reanalyser.reanalyse([rec for _, rec in locked], gumbel=gumbel, discount=cfg.DISCOUNT,
                                   n_steps=cfg.N_STEPS)
    except Exception:
        for gid, _ in locked:
            store.unlock_game_on_error(gid)
        raise
    done = 0
    for (gid, rec), r in zip(locked, res):
        if len(r.policies) != len(rec.actions) or not len(rec.actions):
            store.unlock_game_on_error(gid)
            continue
        if store.finish_reanalysis_for_game(gid, list(r.policies), r.value_targets, current_trainer_step,
                                            cfg.NUM_UNROLL_STEPS):
            done += 1
            if ui_queue is not None:
                ui_queue.put(R.ReAnalysisStatus(1, r.corrected_fives, r.original_fives, r.corrected_totals,
                                                r.original_totals))
    return done
