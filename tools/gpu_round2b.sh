#!/bin/bash
# round 2: GPU suite, drop-in worker throughput (mp queues), action agreement at C2
OUT=gpurun_out/r2_b
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -30; exit 1; }
grep -E "top1_agreement" $OUT/pytest.log | head -3
timeout -k 10 400 python tools/worker_bench.py --moves 24 --warmup 4 > $OUT/worker.json 2> $OUT/worker.err || { echo "worker bench failed"; tail -20 $OUT/worker.err; exit 1; }
cat $OUT/worker.json
timeout -k 10 600 python tools/action_agreement.py --games 256 --out $OUT/agreement.json > $OUT/agreement.log 2>&1 || { echo "agreement failed"; tail -20 $OUT/agreement.log; exit 1; }
cat $OUT/agreement.json
