#!/bin/bash
# split-engine parity (GPU) + same-box bench with one and two streams + worker record test
OUT=gpurun_out/sp2
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_split_gpu.py tests/test_adapter_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; grep -E "^E |FAILED|Error" $OUT/pytest.log | head -20
[ $rc -ne 0 ] && exit 1
SP="--no-cpu-baseline --trainer-steps 0 --loop-iters 0"
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 6 --warmup 1 $SP --streams 1 > $OUT/b1_$i.json 2> $OUT/b1.err || { tail -5 $OUT/b1.err; exit 1; }
timeout -k 10 300 python bench.py --steps 6 --warmup 1 $SP > $OUT/b2_$i.json 2> $OUT/b2.err || { tail -5 $OUT/b2.err; exit 1; }
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/sp2/b*_*.json")):
    d = json.load(open(f)); r = d["roofline"]; t = d["roofline_tree"]
    print(f.split("/")[-1], "%.0f moves/s" % d["value"], "tower mean %.3f ms frac %.3f (per launch %.3f)" % (r["mean_launch_ms"], r["frac"], r["achieved_per_launch"] / 2500),
          "| tree %.1f us %.0f GB/s (per launch %.0f)" % (t["mean_launch_ms"] * 1e3, t["achieved"], t["achieved_per_launch"]))
PY
