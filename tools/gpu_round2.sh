#!/bin/bash
# GPU round trip used during round 2: GPU test suite, default bench (f16, trainer leg), bf16 bench.
TAG=${1:-x}
OUT=gpurun_out/r2_$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit 1; }
timeout -k 10 400 python bench.py --steps 6 --warmup 1 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu-baseline --precision bf16 --trainer-steps 0 > $OUT/bench_bf16.json 2> $OUT/bench_bf16.err || { echo "bench bf16 failed"; tail -20 $OUT/bench_bf16.err; exit 1; }
cat $OUT/bench_bf16.json
