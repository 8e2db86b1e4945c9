#!/bin/bash
# same-box A/B of the C4 trainer step (tools/bench_trainer.py --per): _ab_old/ (git archive of the base
# commit with its own libgmz.so) vs this tree, alternating ROUNDS times; then this tree's trainer GPU tests
# selected by TESTS (pytest -k; empty: skip).  -> gpurun_out/abt/
#   usage: tools/ab_trainer.sh [ROUNDS] [TESTS]
set -o pipefail
ROUNDS=${1:-3}
TESTS=${2:-}
OUT=gpurun_out/abt
mkdir -p $OUT
for i in $(seq 1 $ROUNDS); do
  (cd _ab_old && timeout -k 10 200 python3 tools/bench_trainer.py --steps 30 --per > ../$OUT/old_$i.json 2> ../$OUT/old_$i.err) \
    || { echo "old failed"; tail -5 $OUT/old_$i.err; exit 1; }
  timeout -k 10 200 python3 tools/bench_trainer.py --steps 30 --per > $OUT/new_$i.json 2> $OUT/new_$i.err \
    || { echo "new failed"; tail -5 $OUT/new_$i.err; exit 1; }
  for v in old new; do
    python3 -c "import json; d=json.load(open('$OUT/${v}_$i.json')); print('%s %d %.2f steps/s' % ('$v', $i, d['value']))" | tee -a $OUT/summary.txt
  done
done
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_trainer.py -m gpu -k "$TESTS" \
    > $OUT/tests.log 2>&1; rc=$?
  grep -E "PASS|FAIL|Error" $OUT/tests.log | tail -30
  exit $rc
fi
