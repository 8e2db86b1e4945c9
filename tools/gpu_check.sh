#!/bin/bash
# One GPU round trip: full GPU test suite, short bench, kernel-trace stats of the bench.
# Usage: bash tools/gpu_check.sh TAG   (outputs under gpurun_out/check_TAG/)
TAG=${1:-x}
OUT=gpurun_out/check_$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest rc=$? $(tail -1 $OUT/pytest.log)"
timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']; print('moves/s %.1f  ms/step %.1f  tower %.3f ms  frac %.3f' % (d['value'], d['ms_per_step'], r['mean_launch_ms'], r['frac']))"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_trace.json 2> $OUT/trace.err || { echo "trace failed"; exit 1; }
python - <<PY
import csv
rows = list(csv.DictReader(open("$OUT/trace/run_kernel_stats.csv")))
for r in rows[:9]:
    print("%-60s %6s calls  avg %9.1f us  %5.1f%%" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
PY
