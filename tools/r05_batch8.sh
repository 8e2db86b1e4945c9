#!/bin/bash
# round 5 GPU batch 8: the conv's early next-board DMA (GMZ_CONV_EARLY build): its conv tests on that library,
# then conv and trainer A/B against the product library on the same box.
set -o pipefail
OUT=gpurun_out/r05_b8
mkdir -p $OUT
( while sleep 60; do date >> $OUT/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
EL=$PWD/datou-gomoku-muzero_amd/_alt/libgmz_early.so
GMZ_LIB=$EL timeout -k 10 600 python -u -m pytest tests/test_trainer.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "hip_conv3x3 or conv_epilogue or conv3x3_forward_add or batched_consistency_kernels or residual_gradient_fold or dynamics_stem or bn_backward_sums" > $OUT/tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|^E  " $OUT/tests.log | tail -30
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for V in base early; do
    ENV=""; [ $V != base ] && ENV="GMZ_LIB=$EL"
    for N in 360 1800; do
      env $ENV timeout -k 10 120 python3 tools/conv_bench.py $N > $OUT/conv_${V}_${N}_$i.txt 2>&1 || { echo "conv $V failed"; tail -3 $OUT/conv_${V}_${N}_$i.txt; exit 1; }
      echo "conv $V N=$N $i: $(grep -E '^(hip fwd|hip dgrad) ' $OUT/conv_${V}_${N}_$i.txt | tr -s ' ' | tr '\n' ';') $(head -1 $OUT/conv_${V}_${N}_$i.txt)" | tee -a $OUT/summary.txt
    done
    env $ENV timeout -k 10 200 python3 tools/bench_trainer.py --steps 30 --per > $OUT/tr_${V}_$i.json 2> $OUT/tr_${V}_$i.err \
      || { echo "trainer $V failed"; tail -5 $OUT/tr_${V}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/tr_${V}_$i.json')); print('trainer %-6s %d %.2f steps/s' % ('$V', $i, d['value']))" | tee -a $OUT/summary.txt
  done
done
for V in abl8 abl16 abl28; do
  for N in 360 1800; do
    GMZ_LIB=$PWD/datou-gomoku-muzero_amd/_alt/libgmz_$V.so timeout -k 10 120 python3 tools/conv_bench.py $N > $OUT/conv_${V}_${N}.txt 2>&1 || { echo "conv $V failed"; tail -3 $OUT/conv_${V}_${N}.txt; exit 1; }
    echo "conv $V N=$N: $(grep -E '^(hip fwd|hip dgrad) ' $OUT/conv_${V}_${N}.txt | tr -s ' ' | tr '\n' ';')" | tee -a $OUT/summary.txt
  done
done
bash tools/r05_pmc_tree.sh r05_b8/pmc_tree
