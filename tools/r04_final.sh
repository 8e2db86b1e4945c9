#!/bin/bash
# round-4 final validation on one box: GPU suite, smoke, the default bench line, its rocprofv3 kernel stats
# and the PMC passes (tower + tree) -> gpurun_out/r04f/
set -o pipefail
OUT=gpurun_out/r04f
mkdir -p $OUT
( while sleep 60; do date >> $OUT/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 720 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 \
  || { echo "GPU tests failed"; grep -E "FAILED|^E  " $OUT/pytest.log | head -30; tail -3 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 500 python -u bench.py --steps 20 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -10 $OUT/bench.err; exit 1; }
python3 tools/summarize_bench.py $OUT/bench.json
bash tools/gpu.sh trace r04f_trace || exit 1
bash tools/gpu.sh pmc r04f_pmc || exit 1
bash tools/r04_tprof.sh || exit 1
