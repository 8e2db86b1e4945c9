#!/bin/bash
# round 5 GPU batch 6: the batched-heads GPU tests (fused heads-input node), the trainer A/B (heads, conv weight-ring
# depth 3 / 4 / 6 builds), the conv ring-depth A/B standalone, and the tower after the wave-index register fix
# (headline + C5 + C1 sub-lines).
set -o pipefail
OUT=gpurun_out/r05_b6
mkdir -p $OUT
( while sleep 60; do date >> $OUT/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_trainer.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "batched_heads_on_gpu or production_training_step or gpu_loss_and_gradients or elementwise" > $OUT/tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|^E  " $OUT/tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for V in base perheads rd4 rd6; do
    ARGS="--steps 30 --per"; ENV=""
    [ $V = perheads ] && ARGS="$ARGS --per-step-heads"
    [ $V = rd4 -o $V = rd6 ] && ENV="GMZ_LIB=$PWD/datou-gomoku-muzero_amd/_alt/libgmz_$V.so"
    env $ENV timeout -k 10 200 python3 tools/bench_trainer.py $ARGS > $OUT/tr_${V}_$i.json 2> $OUT/tr_${V}_$i.err \
      || { echo "trainer $V failed"; tail -5 $OUT/tr_${V}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/tr_${V}_$i.json')); print('trainer %-8s %d %.2f steps/s' % ('$V', $i, d['value']))" | tee -a $OUT/summary.txt
  done
done
for i in 1; do
  for V in base rd4 rd6; do
    ENV=""; [ $V != base ] && ENV="GMZ_LIB=$PWD/datou-gomoku-muzero_amd/_alt/libgmz_$V.so"
    for N in 360 1800; do
      env $ENV timeout -k 10 120 python3 tools/conv_bench.py $N > $OUT/conv_${V}_${N}_$i.txt 2>&1 || { echo "conv $V failed"; tail -3 $OUT/conv_${V}_${N}_$i.txt; exit 1; }
      echo "conv $V N=$N $i: $(grep -E '^(hip fwd|hip dgrad) ' $OUT/conv_${V}_${N}_$i.txt | tr -s ' ' | tr '\n' ';')" | tee -a $OUT/summary.txt
    done
  done
done
SP="--no-cpu-baseline --trainer-steps 0 --loop-iters 0 --sublines=c5,c1 --worker-moves 0 --single-stream-moves 0 --steps 10 --warmup 2"
timeout -k 10 400 python3 bench.py $SP > $OUT/hl.json 2> $OUT/hl.err || { echo "headline failed"; tail -5 $OUT/hl.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/hl.json'))
print('headline %.1f moves/s tower %.4f ms frac %.3f' % (d['value'], d['roofline']['mean_launch_ms'], d['roofline']['frac']))
for k, v in d['sublines'].items(): print('  %s %.1f moves/s tower %.4f ms frac %.3f' % (k, v['value'], v['roofline']['mean_launch_ms'], v['roofline']['frac']))
" | tee -a $OUT/summary.txt
bash tools/r05_pmc_tree.sh r05_b6/pmc_tree
