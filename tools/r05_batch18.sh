#!/bin/bash
# round 5: the trainer trace on the final BatchNorm grids
set -o pipefail
OUT=gpurun_out/r05_b18
mkdir -p $OUT
timeout -k 10 500 bash tools/trainer_profile.sh --per > $OUT/trainer_profile.txt 2>&1 && \
  python3 tools/trainer_trace_summary.py gpurun_out/tprof/trace/run_kernel_trace.csv gpurun_out/tprof/bench.json $OUT/r05_trainer_trace.json && \
  python3 -c "import json; d=json.load(open('$OUT/r05_trainer_trace.json')); print('launches per step', d['launches_per_step'])" | tee -a $OUT/summary.txt
