#!/bin/bash
# round 5 GPU batch 4: the default bench line (the driver's N = 1 command), then the DEFER_WGRAD memory A/B.
set -o pipefail
OUT=gpurun_out/r05_b4
mkdir -p $OUT
( while sleep 60; do date >> $OUT/heartbeat; done ) &
HB=$!
timeout -k 10 700 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?
kill $HB
tail -3 $OUT/bench.err
[ $rc -eq 0 ] || exit $rc
python3 tools/summarize_bench.py $OUT/bench.json || true
for V in defer nodefer; do
  ARGS="--steps 20 --per"
  [ $V = nodefer ] && ARGS="$ARGS --no-defer-wgrad"
  timeout -k 10 200 python3 tools/bench_trainer.py $ARGS > $OUT/tr_$V.json 2> $OUT/tr_$V.err || { echo "trainer $V failed"; tail -5 $OUT/tr_$V.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/tr_$V.json')); print('%-8s %.2f steps/s peak %.2f GiB' % ('$V', d['value'], d['max_memory_allocated_gb']))" | tee -a $OUT/summary.txt
done
