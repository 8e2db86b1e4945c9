#!/bin/bash
# trainer A/Bs, same box, alternating: defaults | per-use weight gradients | target value with an f16 trunk
# then the new trainer GPU tests -> gpurun_out/tgt/
set -o pipefail
OUT=gpurun_out/tgt
mkdir -p $OUT
for round in 1 2; do
  for v in base nodefer tgt16; do
    flag=""; [ $v = nodefer ] && flag="--no-defer-wgrad"; [ $v = tgt16 ] && flag="--target-f16"
    timeout -k 10 240 python3 tools/bench_trainer.py --steps 40 --per $flag > $OUT/${v}_$round.json 2> $OUT/${v}_$round.err \
      || { echo "$v failed"; tail -5 $OUT/${v}_$round.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${v}_$round.json')); print('%-8s %.2f steps/s' % ('$v', d['value']))" | tee -a $OUT/summary.txt
  done
done
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_trainer.py -m gpu \
  -k "deferred or target_value or production or graph" > $OUT/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|max \|dv|mean" $OUT/tests.log | tail -20
exit $rc
