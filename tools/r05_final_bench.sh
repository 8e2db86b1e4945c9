#!/bin/bash
# round 5 final: the driver's default bench line, the self-play step's rocprofv3 kernel stats, the tower PMC passes,
# the trainer step's kernel trace.
set -o pipefail
bash tools/gpu.sh bench r05_final && bash tools/gpu.sh trace r05_final && bash tools/gpu.sh pmc r05_final && \
  timeout -k 10 500 bash tools/trainer_profile.sh --per > gpurun_out/r05_final/trainer_profile.txt 2>&1 && \
  python3 tools/trainer_trace_summary.py gpurun_out/tprof/trace/run_kernel_trace.csv gpurun_out/tprof/bench.json gpurun_out/r05_final/r05_trainer_trace.json
