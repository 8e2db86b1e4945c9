#!/bin/bash
# round 5 GPU batch 5: the trainer step's kernel trace (launches per step, k_conv3 inside the replayed step), then the
# trainer conv's PMC passes at the step's shape (N = 360).
set -o pipefail
OUT=gpurun_out/r05_b5
mkdir -p $OUT
timeout -k 10 500 bash tools/trainer_profile.sh --per > $OUT/profile.txt 2>&1 || { echo "trace failed"; tail -5 $OUT/profile.txt; exit 1; }
tail -45 $OUT/profile.txt
python3 tools/trainer_trace_summary.py gpurun_out/tprof/trace/run_kernel_trace.csv gpurun_out/tprof/bench.json $OUT/r05_trainer_trace.json \
  && cat $OUT/r05_trainer_trace.json
timeout -k 10 400 bash tools/pmc_conv.sh 360 > $OUT/pmc_conv.txt 2>&1; rc=$?
cat $OUT/pmc_conv.txt; exit $rc
[ $rc -eq 0 ] || exit $rc
# the conv's weight-ring depth (k-steps of weight fragments in flight from L2): 3 (product) vs 4 / 6 (A/B builds)
for i in 1 2; do
  for V in base rd4 rd6; do
    ENV=""; [ $V != base ] && ENV="GMZ_LIB=$PWD/datou-gomoku-muzero_amd/_alt/libgmz_$V.so"
    for N in 360 1800; do
      env $ENV timeout -k 10 120 python3 tools/conv_bench.py $N > $OUT/conv_${V}_${N}_$i.txt 2>&1 || { echo "conv $V failed"; tail -3 $OUT/conv_${V}_${N}_$i.txt; exit 1; }
      echo "$V N=$N $i: $(grep -E '^(hip fwd|hip dgrad ) ' $OUT/conv_${V}_${N}_$i.txt | tr -s ' ' | tr '\n' ';') $(head -1 $OUT/conv_${V}_${N}_$i.txt)" | tee -a $OUT/conv_ab.txt
    done
  done
done
for i in 1 2; do
  for V in base rd6; do
    ENV=""; [ $V != base ] && ENV="GMZ_LIB=$PWD/datou-gomoku-muzero_amd/_alt/libgmz_$V.so"
    env $ENV timeout -k 10 200 python3 tools/bench_trainer.py --steps 30 --per > $OUT/tr_${V}_$i.json 2> $OUT/tr_${V}_$i.err \
      || { echo "trainer $V failed"; tail -5 $OUT/tr_${V}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/tr_${V}_$i.json')); print('trainer %-6s %d %.2f steps/s' % ('$V', $i, d['value']))" | tee -a $OUT/conv_ab.txt
  done
done
