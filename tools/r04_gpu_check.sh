#!/bin/bash
# round-4 GPU check: the new/changed parity tests, then the default bench (one line) -> gpurun_out/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_engine_gpu.py tests/test_split_gpu.py tests/test_headline_gpu.py \
  "tests/test_pipeline_gpu.py::test_bench_spawns_its_own_ranks_gloo_rehearsal" \
  > gpurun_out/r04_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r04_tests.log; exit 1; }
tail -3 gpurun_out/r04_tests.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 2 > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.log \
  || { echo "bench failed"; tail -30 gpurun_out/r04_bench.log; exit 1; }
tail -c 600 gpurun_out/r04_bench.json
