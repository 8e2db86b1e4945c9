#!/bin/bash
# Round-2 evidence on the final tree kernel: rocprofv3 kernel stats of the default bench command, G sweep,
# PMC passes (tower + tree kernel, two streams) -> gpurun_out/r2_h, gpurun_out/pmc_r02
OUT=gpurun_out/r2_h
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
SP="--no-cpu-baseline --trainer-steps 0 --loop-iters 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --steps 3 --warmup 1 $SP > $OUT/bench_under_trace.json 2> $OUT/trace.err || { echo "trace failed"; tail -5 $OUT/trace.err; exit 1; }
find $OUT/trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
echo "trace done"
for G in 2048 4096 8192; do
  timeout -k 10 500 python3 bench.py --games $G --steps 3 --warmup 1 $SP > $OUT/bench_G$G.json 2> $OUT/bench_G$G.err || { echo "G=$G failed"; tail -5 $OUT/bench_G$G.err; exit 1; }
done
echo "sweep done"
bash tools/pmc_round2.sh > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/pmc.log; exit 1; }
python3 - <<'PY'
import json
for G in (2048, 4096, 8192):
    d = json.load(open("gpurun_out/r2_h/bench_G%d.json" % G)); s = d["single_stream_kernels"]
    print(G, "%.0f moves/s" % d["value"], "tree alone %.1f us %.0f GB/s %.3f" % (s["tree"]["mean_launch_ms"] * 1e3, s["tree"]["achieved_gbs"], s["tree"]["frac"]), "tower alone %.3f ms %.3f" % (s["tower"]["mean_launch_ms"], s["tower"]["frac"]))
PY
tail -14 gpurun_out/pmc_r02/summary.txt
