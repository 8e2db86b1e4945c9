#!/bin/bash
# trainer A/Bs, same box, alternating: defaults | per-use weight gradients | target value in float32 |
# one workgroup per board in the 3x3 conv (GMZ_CONV_HALVES=2); conv kernel alone both ways; then the new
# trainer GPU tests (and the conv tests under GMZ_CONV_HALVES=2) -> gpurun_out/tgt/
set -o pipefail
OUT=gpurun_out/tgt
mkdir -p $OUT
for hv in 1 2; do
  GMZ_CONV_HALVES=$hv timeout -k 10 120 python3 tools/conv_bench.py 360 15 > $OUT/conv_h$hv.txt 2>&1 || { echo "conv bench $hv failed"; tail -5 $OUT/conv_h$hv.txt; exit 1; }
  echo "== GMZ_CONV_HALVES=$hv"; grep -v Warning $OUT/conv_h$hv.txt | tail -4
done
for round in 1 2; do
  for v in base nodefer tgt32 halves2; do
    flag=""; [ $v = nodefer ] && flag="--no-defer-wgrad"; [ $v = tgt32 ] && flag="--target-f32"
    hv=1; [ $v = halves2 ] && hv=2
    GMZ_CONV_HALVES=$hv timeout -k 10 200 python3 tools/bench_trainer.py --steps 30 --per $flag > $OUT/${v}_$round.json 2> $OUT/${v}_$round.err \
      || { echo "$v failed"; tail -5 $OUT/${v}_$round.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${v}_$round.json')); print('%-8s %.2f steps/s' % ('$v', d['value']))" | tee -a $OUT/summary.txt
  done
done
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_trainer.py -m gpu \
  -k "deferred or target_value or production" > $OUT/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|max \|dv|mean" $OUT/tests.log | tail -20
[ $rc = 0 ] || exit $rc
GMZ_CONV_HALVES=2 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_trainer.py -m gpu \
  -k "conv or epilogue or residual or production_training" > $OUT/tests_halves2.log 2>&1; rc=$?
tail -2 $OUT/tests_halves2.log
exit $rc
