#!/bin/bash
# round 5 GPU batch 12: the HIP segmented BatchNorm of the batched heads — its kernel test, the batched-heads and
# production GPU tests on it, then the trainer A/B against the PyTorch segmented BatchNorm, and the trainer trace.
set -o pipefail
OUT=gpurun_out/r05_b12
mkdir -p $OUT
( while sleep 60; do date >> $OUT/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_trainer.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "segmented_batchnorm or batched_heads_on_gpu or production_training_step or elementwise or gpu_loss_and_gradients or concurrent_forward" > $OUT/tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|^E  " $OUT/tests.log | tail -30
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for V in base torchsegbn; do
    ARGS="--steps 30 --per"
    [ $V = torchsegbn ] && ARGS="$ARGS --torch-seg-bn"
    timeout -k 10 200 python3 tools/bench_trainer.py $ARGS > $OUT/tr_${V}_$i.json 2> $OUT/tr_${V}_$i.err \
      || { echo "trainer $V failed"; tail -5 $OUT/tr_${V}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/tr_${V}_$i.json')); print('trainer %-10s %d %.2f steps/s' % ('$V', $i, d['value']))" | tee -a $OUT/summary.txt
  done
done
timeout -k 10 500 bash tools/trainer_profile.sh --per > $OUT/trainer_profile.txt 2>&1 && \
  python3 tools/trainer_trace_summary.py gpurun_out/tprof/trace/run_kernel_trace.csv gpurun_out/tprof/bench.json $OUT/r05_trainer_trace.json && \
  python3 -c "import json; d=json.load(open('$OUT/r05_trainer_trace.json')); print('launches per step', d['launches_per_step'])" | tee -a $OUT/summary.txt
