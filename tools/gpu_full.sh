#!/bin/bash
# Full round check: GPU suite, smoke(), default bench line.  Usage: bash tools/gpu_full.sh TAG
TAG=${1:-x}
OUT=gpurun_out/full_$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"
[ $rc -ne 0 ] && { grep -E "FAILED|^E " $OUT/pytest.log | head -30; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
s = d["single_stream_kernels"]
print("moves/s %.0f ms/step %.1f tower frac %.3f (%.3f ms) | tree 2-stream %.1f us | single: tower %.3f ms %.3f, tree %.1f us %.0f GB/s %.3f"
      % (d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["mean_launch_ms"], d["roofline_tree"]["mean_launch_ms"] * 1e3,
         s["tower"]["mean_launch_ms"], s["tower"]["frac"], s["tree"]["mean_launch_ms"] * 1e3, s["tree"]["achieved_gbs"], s["tree"]["frac"]))
print("trainer %.2f steps/s; loop %.0f moves/s %.2f steps/s; cpu %.3f %s" % (d["trainer"]["value"], d["loop_c4"]["moves_per_s"], d["loop_c4"]["trainer_steps_per_s"], d["cpu_baseline"]["value"], d["cpu_baseline"]["unit"]))
PY
