#!/bin/bash
# round 5 GPU batch 11: the staged weight gradient (k_conv3_wgrad2, GMZ_WGRAD_STAGED=1): its tests, then the conv
# bench's weight-gradient line and the trainer A/B against k_conv3_wgrad on the same box.
set -o pipefail
OUT=gpurun_out/r05_b11
mkdir -p $OUT
( while sleep 60; do date >> $OUT/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
GMZ_WGRAD_STAGED=1 timeout -k 10 600 python -u -m pytest tests/test_trainer.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "hip_conv3x3 or deferred_multi_segment or production_training_step or batched_consistency_kernels" > $OUT/tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|^E  " $OUT/tests.log | tail -30
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for V in base staged; do
    ENV=""; [ $V = staged ] && ENV="GMZ_WGRAD_STAGED=1"
    for N in 360 1800; do
      env $ENV timeout -k 10 120 python3 tools/conv_bench.py $N > $OUT/conv_${V}_${N}_$i.txt 2>&1 || { echo "conv $V failed"; tail -3 $OUT/conv_${V}_${N}_$i.txt; exit 1; }
      echo "conv $V N=$N $i: $(grep -E '^hip wgrad ' $OUT/conv_${V}_${N}_$i.txt | tr -s ' ') $(grep 'rel err' $OUT/conv_${V}_${N}_$i.txt)" | tee -a $OUT/summary.txt
    done
    env $ENV timeout -k 10 200 python3 tools/bench_trainer.py --steps 30 --per > $OUT/tr_${V}_$i.json 2> $OUT/tr_${V}_$i.err \
      || { echo "trainer $V failed"; tail -5 $OUT/tr_${V}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/tr_${V}_$i.json')); print('trainer %-6s %d %.2f steps/s' % ('$V', $i, d['value']))" | tee -a $OUT/summary.txt
  done
done
