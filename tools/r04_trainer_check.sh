#!/bin/bash
# trainer GPU tests with the round-4 defaults (DEFER_WGRAD, TARGET_F16), the conv tests under
# GMZ_CONV_HALVES=2, and one defaults-vs-float32-target trainer pair -> gpurun_out/tchk/
set -o pipefail
OUT=gpurun_out/tchk
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_trainer.py -m gpu \
  > $OUT/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|max \|dv|Error" $OUT/tests.log | tail -40
[ $rc = 0 ] || exit $rc
GMZ_CONV_HALVES=2 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_trainer.py -m gpu \
  -k "conv or epilogue or residual or production_training" > $OUT/tests_halves2.log 2>&1; rc=$?
tail -2 $OUT/tests_halves2.log
[ $rc = 0 ] || exit $rc
for v in base tgt32; do
  flag=""; [ $v = tgt32 ] && flag="--target-f32"
  timeout -k 10 200 python3 tools/bench_trainer.py --steps 30 --per $flag > $OUT/$v.json 2> $OUT/$v.err \
    || { echo "$v failed"; tail -5 $OUT/$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$v.json')); print('%-8s %.2f steps/s' % ('$v', d['value']))" | tee -a $OUT/summary.txt
done
