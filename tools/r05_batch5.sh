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
