#!/bin/bash
# the HIP dynamics stem after the f32-table fix: its equivalence test, then one short trainer run with it on
set -o pipefail
OUT=gpurun_out/r05_dbg3
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_trainer.py -m gpu -x -v --timeout 150 --timeout-method thread \
  -k "dynamics_stem" > $OUT/tests.log 2>&1; rc=$?; grep -E "PASS|FAIL|^E  " $OUT/tests.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/dbg_stem2.py > $OUT/stem2.txt 2>&1; rc=$?; grep -v amdgpu.ids $OUT/stem2.txt | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/bench_trainer.py --steps 20 --per --hip-stem > $OUT/tr_hipstem.json 2> $OUT/tr_hipstem.err; rc=$?
tail -3 $OUT/tr_hipstem.err; cat $OUT/tr_hipstem.json; exit $rc
