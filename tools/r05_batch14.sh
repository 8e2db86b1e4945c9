#!/bin/bash
# round 5 GPU batch 14: the projection's BatchNorm on the HIP segmented kernel (C >= 64 only): trainer GPU tests,
# the trainer A/B against all-PyTorch segmented BatchNorms, and the trace.
set -o pipefail
OUT=gpurun_out/r05_b14
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
