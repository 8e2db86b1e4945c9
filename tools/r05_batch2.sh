#!/bin/bash
# round 5 GPU batch 2: trainer — the batched heads and the fused head convs (tests, then a same-box A/B against the
# per-step heads / PyTorch head convs), the HIP dynamics stem, the 1-bit ReLU masks, and the NET_FPC library A/B
# (fp contraction in the net / conv / train kernels) on the trainer and the headline.
set -o pipefail
OUT=gpurun_out/r05_b2
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_trainer.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "relu_mask or head_conv1x1 or prediction_heads or bigk_linear_pair" > $OUT/tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|^E  " $OUT/tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for V in base perheads torchheads hipstem relumask fpc; do
    ARGS="--steps 30 --per"; ENV=""
    [ $V = perheads ] && ARGS="$ARGS --per-step-heads"
    [ $V = torchheads ] && ARGS="$ARGS --torch-head-convs"
    [ $V = hipstem ] && ARGS="$ARGS --hip-stem"
    [ $V = relumask ] && ARGS="$ARGS --relu-mask"
    [ $V = fpc ] && ENV="GMZ_LIB=$PWD/datou-gomoku-muzero_amd/_alt/libgmz_fpc.so"
    env $ENV timeout -k 10 200 python3 tools/bench_trainer.py $ARGS > $OUT/tr_${V}_$i.json 2> $OUT/tr_${V}_$i.err \
      || { echo "trainer $V failed"; tail -5 $OUT/tr_${V}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/tr_${V}_$i.json')); print('trainer %-8s %d %.2f steps/s' % ('$V', $i, d['value']))" | tee -a $OUT/summary.txt
  done
done
SP="--no-cpu-baseline --trainer-steps 0 --loop-iters 0 --sublines= --worker-moves 0 --single-stream-moves 0 --steps 20 --warmup 3"
for i in 1 2; do
  for V in base fpc; do
    ENV=""
    [ $V = fpc ] && ENV="GMZ_LIB=$PWD/datou-gomoku-muzero_amd/_alt/libgmz_fpc.so"
    env $ENV timeout -k 10 300 python3 bench.py $SP > $OUT/hl_${V}_$i.json 2> $OUT/hl_${V}_$i.err \
      || { echo "headline $V failed"; tail -5 $OUT/hl_${V}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/hl_${V}_$i.json')); print('headline %-5s %d %.1f moves/s tower frac %.3f' % ('$V', $i, d['value'], d['roofline']['frac']))" | tee -a $OUT/summary.txt
  done
done
