#!/bin/bash
OUT=gpurun_out/qedge
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_adapter_gpu.py tests/test_split_gpu.py tests/test_reanalysis_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -1 $OUT/pytest.log; grep -E "^E |FAILED" $OUT/pytest.log | head; [ $rc -ne 0 ] && exit 1
bash tools/ab_tree.sh q1024 $PWD/datou-gomoku-muzero_amd/_alt/libgmz_base.so --steps 4 --warmup 1 && \
bash tools/ab_tree.sh q8192 $PWD/datou-gomoku-muzero_amd/_alt/libgmz_base.so --games 8192 --steps 2 --warmup 1
