"""Tree-kernel HBM roofline: G games of 15x15 MuZero/400 with the HashNet device
backend (network cost ~0), timing k_select and k_expand_backup separately with HIP events on the
launch stream, and counting their algorithmic bytes from the per-game path lengths of every wave:
  select : 20*A B per non-root level (child N, W, R, child index = 16 B/edge + 4 B logit) + the
           root level's selected edges (n_sel x 16 B)
  backup : 24 B per path level (parent idx, R, N r+w, W r+w) + 16 B (min/max r+w, leaf value, k)
Prints one line per G: us/launch, GB/s, fraction of 8 TB/s.  Usage:
  python tools/tree_microbench.py [--games 1024,4096,8192,16384] [--moves 2]"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import datou_gomoku_muzero_amd.engine as E  # noqa: E402
from datou_gomoku_muzero_amd._lib import check, ptr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--games", default="1024,2048,4096,8192,16384")
ap.add_argument("--moves", type=int, default=2)
ap.add_argument("--size", type=int, default=15)
ap.add_argument("--sims", type=int, default=400)
ap.add_argument("--out", default=None)
a = ap.parse_args()
PEAK = 8000.0  # GB/s, MI355X HBM3E
out = []
for G in [int(x) for x in a.games.split(",")]:
    eng = E.BatchedSelfPlayEngine(None, num_games=G, BOARD_SIZE=a.size, NUM_SIMULATIONS=a.sims, seed=1)
    eng.reset_games()
    L, A, s = eng.lib, eng.A, eng._stream()
    depth = torch.zeros(G, dtype=torch.int32, device="cuda")
    t_sel = t_bk = 0.0
    n_launch = 0
    b_sel = b_bk = 0
    for m in range(a.moves + 1):
        timed = m > 0  # first move = warm-up
        check(L.gmz_engine_begin_move(eng.handle, None, eng.seed, ptr(eng.obs), s))
        eng.net.initial(eng.obs, eng.root_slot, eng.logits, eng.value, s)
        check(L.gmz_engine_set_root(eng.handle, ptr(eng.logits), ptr(eng.value), s))
        eng._sync_status()
        waves = eng.waves_needed()
        for _ in range(waves):
            e0, e1, e2, e3 = (torch.cuda.Event(enable_timing=True) for _ in range(4))
            e0.record()
            check(L.gmz_engine_select(eng.handle, ptr(eng.in_slot), ptr(eng.act_req), ptr(eng.out_slot), ptr(eng.obs), s))
            e1.record()
            check(L.gmz_engine_wave_depth(eng.handle, ptr(depth), s))
            eng.net.recurrent(eng.in_slot, eng.act_req, eng.out_slot, eng.logits, eng.value, eng.reward, s)
            e2.record()
            check(L.gmz_engine_expand_backup(eng.handle, ptr(eng.logits), ptr(eng.value), ptr(eng.reward), s))
            e3.record()
            if timed:
                torch.cuda.synchronize()
                d = depth.cpu().numpy()
                act = d > 0
                b_sel += int(((d[act] - 1) * 20 * A).sum() + act.sum() * 16 * 16)
                b_bk += int((d[act] * 24 + 16).sum())
                t_sel += e0.elapsed_time(e1)
                t_bk += e2.elapsed_time(e3)
                n_launch += 1
        check(L.gmz_engine_finish_move(eng.handle, ptr(eng.policy), ptr(eng.root_value), ptr(eng.action), s))
        eng.play(reset_finished=True)
    torch.cuda.synchronize()
    r = {"games": G, "waves": n_launch,
         "select_us": t_sel / n_launch * 1e3, "select_GBs": b_sel / (t_sel * 1e-3) / 1e9,
         "backup_us": t_bk / n_launch * 1e3, "backup_GBs": b_bk / (t_bk * 1e-3) / 1e9,
         "select_bytes_per_wave": b_sel / n_launch, "backup_bytes_per_wave": b_bk / n_launch}
    r["select_frac"], r["backup_frac"] = r["select_GBs"] / PEAK, r["backup_GBs"] / PEAK
    print("G %6d  select %7.1f us %7.1f GB/s (%.3f of 8 TB/s)   backup %6.1f us %6.1f GB/s (%.4f)" % (
        G, r["select_us"], r["select_GBs"], r["select_frac"], r["backup_us"], r["backup_GBs"], r["backup_frac"]), flush=True)
    out.append(r)
    eng.close()
    del eng
    torch.cuda.empty_cache()
if a.out:
    json.dump(out, open(a.out, "w"), indent=1)
