#!/bin/bash
OUT=gpurun_out/ldshint
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_split_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -1 $OUT/pytest.log; grep -E "^E |FAILED" $OUT/pytest.log | head; [ $rc -ne 0 ] && exit 1
bash tools/ab_tree.sh lds1024 $PWD/datou-gomoku-muzero_amd/_alt/libgmz_base.so --steps 4 --warmup 1 --streams 1 --single-stream-moves 0 || exit 1
bash tools/ab_tree.sh lds2s $PWD/datou-gomoku-muzero_amd/_alt/libgmz_base.so --steps 4 --warmup 1
