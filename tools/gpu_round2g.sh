#!/bin/bash
# Round-2 evidence refresh: GPU suite, default bench line, rocprofv3 kernel stats, G sweep, PMC passes
OUT=gpurun_out/r2_g
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"
[ $rc -ne 0 ] && { grep -E "FAILED|^E " $OUT/pytest.log | head -30; exit 1; }
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
echo "bench done"
SP="--no-cpu-baseline --trainer-steps 0 --loop-iters 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --steps 3 --warmup 1 $SP --single-stream-moves 0 > $OUT/bench_under_trace.json 2> $OUT/trace.err || { echo "trace failed"; tail -5 $OUT/trace.err; exit 1; }
find $OUT/trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
echo "trace done"
for G in 2048 4096 8192; do
  timeout -k 10 500 python3 bench.py --games $G --steps 3 --warmup 1 $SP > $OUT/bench_G$G.json 2> $OUT/bench_G$G.err || { echo "G=$G failed"; tail -5 $OUT/bench_G$G.err; exit 1; }
done
echo "sweep done"
bash tools/pmc_round2.sh > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/pmc.log; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r2_g/bench.json"))
print("default: %.0f moves/s tower frac %.3f tree %.1f us single-stream %s" % (d["value"], d["roofline"]["frac"], d["roofline_tree"]["mean_launch_ms"] * 1e3, d["single_stream_kernels"]))
print("trainer %.2f steps/s; loop %.0f moves/s %.2f steps/s; cpu %.3f" % (d["trainer"]["value"], d["loop_c4"]["moves_per_s"], d["loop_c4"]["trainer_steps_per_s"], d["cpu_baseline"]["value"]))
for G in (1024, 2048, 4096, 8192):
    f = "gpurun_out/r2_g/bench.json" if G == 1024 else "gpurun_out/r2_g/bench_G%d.json" % G
    d = json.load(open(f)); s = d["single_stream_kernels"]
    print(G, "%.0f moves/s" % d["value"], "tree alone %.1f us %.0f GB/s %.3f" % (s["tree"]["mean_launch_ms"] * 1e3, s["tree"]["achieved_gbs"], s["tree"]["frac"]), "tower alone %.3f ms %.3f" % (s["tower"]["mean_launch_ms"], s["tower"]["frac"]))
PY
tail -12 gpurun_out/pmc_r02/summary.txt
