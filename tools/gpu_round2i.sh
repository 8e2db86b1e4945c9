#!/bin/bash
# Final round-2 evidence: rocprofv3 kernel stats of the default bench command, C5 and C9 bench lines,
# PMC passes (tools/pmc_round2.sh) -> gpurun_out/r2_i
OUT=gpurun_out/r2_i
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
SP="--no-cpu-baseline --trainer-steps 0 --loop-iters 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --steps 3 --warmup 1 $SP > $OUT/bench_under_trace.json 2> $OUT/trace.err || { echo "trace failed"; tail -5 $OUT/trace.err; exit 1; }
find $OUT/trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
echo "trace done"
timeout -k 10 500 python3 bench.py --size 19 --sims 800 --blocks 16 --steps 3 --warmup 1 $SP > $OUT/c5.json 2> $OUT/c5.err || { echo "c5 failed"; tail -5 $OUT/c5.err; exit 1; }
timeout -k 10 500 python3 bench.py --size 9 --sims 50 --mode AlphaZero --steps 10 --warmup 2 $SP > $OUT/c9.json 2> $OUT/c9.err || { echo "c9 failed"; tail -5 $OUT/c9.err; exit 1; }
echo "configs done"
bash tools/pmc_round2.sh > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/pmc.log; exit 1; }
python3 - <<'PY'
import json, csv
for n in ("c5", "c9"):
    d = json.load(open("gpurun_out/r2_i/%s.json" % n))
    print(n, "%.0f moves/s tower %.3f ms frac %.3f tree %.1f us" % (d["value"], d["roofline"]["mean_launch_ms"], d["roofline"]["frac"], d["roofline_tree"]["mean_launch_ms"] * 1e3))
rows = list(csv.DictReader(open("gpurun_out/r2_i/kernel_stats.csv")))
for r in rows[:6]:
    print("%-50s %6s calls avg %9.1f us %5.1f%%" % (r["Name"][:50], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
PY
tail -6 gpurun_out/pmc_r02/summary.txt
