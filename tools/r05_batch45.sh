#!/bin/bash
# round 5 GPU batches 4 + 5 in one call: the default bench line, the DEFER_WGRAD memory A/B, the trainer step's
# kernel trace and the trainer conv's PMC passes.
set -o pipefail
mkdir -p gpurun_out/r05_b45
( while sleep 60; do date >> gpurun_out/r05_b45/heartbeat; done ) &
HB=$!
timeout -k 10 1000 bash tools/r05_batch4.sh && bash tools/r05_batch5.sh
rc=$?
kill $HB
exit $rc
