#!/bin/bash
# round 5 GPU batch 1: the whole GPU test suite, then the tree kernel's PMC bytes (headline + g8192).
set -o pipefail
OUT=gpurun_out/r05_b1
mkdir -p $OUT
( while sleep 60; do date >> $OUT/heartbeat; done ) &
HB=$!
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
kill $HB
tail -3 $OUT/pytest.log
grep -E "FAILED|^E  " $OUT/pytest.log | head -20
[ $rc -eq 0 ] || exit $rc
bash tools/r05_pmc_tree.sh r05_b1/pmc_tree
