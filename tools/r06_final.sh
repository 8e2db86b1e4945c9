# Round-6 validation on one box: GPU suite, smoke, the default bench line, rocprofv3 kernel stats, PMC passes.
# Each step under its own timeout; the chain stops at the first failure.  -> gpurun_out/r06_final/
set -o pipefail
T=${1:-r06_final}
bash tools/gpu.sh tests $T && \
bash tools/gpu.sh smoke $T && \
bash tools/gpu.sh bench $T && \
bash tools/gpu.sh trace $T --single-stream-moves 0 && \
bash tools/gpu.sh pmc $T
