#!/bin/bash
# round 5: the whole GPU test suite + smoke() on the final code, then the trainer line and its trace.
set -o pipefail
bash tools/gpu.sh tests r05_final2 && bash tools/gpu.sh smoke r05_final2 && \
  timeout -k 10 200 python3 tools/bench_trainer.py --steps 30 --per > gpurun_out/r05_final2/trainer.json 2> gpurun_out/r05_final2/trainer.err && \
  cat gpurun_out/r05_final2/trainer.json && \
  timeout -k 10 500 bash tools/trainer_profile.sh --per > gpurun_out/r05_final2/trainer_profile.txt 2>&1 && \
  python3 tools/trainer_trace_summary.py gpurun_out/tprof/trace/run_kernel_trace.csv gpurun_out/tprof/bench.json gpurun_out/r05_final2/r05_trainer_trace.json
