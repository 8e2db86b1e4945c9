#!/bin/bash
# Round-2 sweeps on the two-stream engine: games per GPU (tree kernel vs G, SURVEY §8d asks for >= 8192
# trees), C5 (19x19 / 800 sims / 16 blocks) and C9-style AlphaZero 9x9 / 50 sims lines.
OUT=gpurun_out/r2_f
mkdir -p $OUT
SP="--no-cpu-baseline --trainer-steps 0 --loop-iters 0"
for G in 2048 4096 8192; do
  timeout -k 10 500 python3 bench.py --games $G --steps 3 --warmup 1 $SP > $OUT/bench_G$G.json 2> $OUT/bench_G$G.err || { echo "G=$G failed"; tail -5 $OUT/bench_G$G.err; exit 1; }
  echo "G=$G done"
done
timeout -k 10 500 python3 bench.py --size 19 --sims 800 --blocks 16 --steps 3 --warmup 1 $SP > $OUT/c5.json 2> $OUT/c5.err || { echo "c5 failed"; tail -3 $OUT/c5.err; exit 1; }
timeout -k 10 300 python3 bench.py --size 9 --sims 50 --mode AlphaZero --steps 10 --warmup 2 $SP > $OUT/c9.json 2> $OUT/c9.err || { echo "c9 failed"; tail -3 $OUT/c9.err; exit 1; }
timeout -k 10 300 python3 bench.py --size 9 --sims 50 --mode AlphaZero --steps 10 --warmup 2 $SP --streams 1 > $OUT/c9_s1.json 2> $OUT/c9_s1.err || { echo "c9 s1 failed"; tail -3 $OUT/c9_s1.err; exit 1; }
timeout -k 10 500 python3 bench.py --size 19 --sims 800 --blocks 16 --steps 3 --warmup 1 $SP --streams 1 > $OUT/c5_s1.json 2> $OUT/c5_s1.err || { echo "c5 s1 failed"; tail -3 $OUT/c5_s1.err; exit 1; }
python3 - <<'PY'
import json
for f in ("bench_G2048", "bench_G4096", "bench_G8192", "c5", "c5_s1", "c9", "c9_s1"):
    d = json.load(open("gpurun_out/r2_f/%s.json" % f)); r = d["roofline"]; t = d.get("roofline_tree", {}); s = d.get("single_stream_kernels", {})
    print("%-12s %9.1f moves/s  tower %.3f ms frac %.3f | tree %.1f us %.0f GB/s | single-stream tower %s tree %s" % (
        f, d["value"], r["mean_launch_ms"], r["frac"], t.get("mean_launch_ms", 0) * 1e3, t.get("achieved", 0),
        "%.3f ms %.3f" % (s["tower"]["mean_launch_ms"], s["tower"]["frac"]) if "tower" in s else "-",
        "%.1f us %.0f GB/s %.3f" % (s["tree"]["mean_launch_ms"] * 1e3, s["tree"]["achieved_gbs"], s["tree"]["frac"]) if "tree" in s else "-"))
PY
