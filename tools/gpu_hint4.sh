#!/bin/bash
OUT=gpurun_out/hint4
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_split_gpu.py tests/test_adapter_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -1 $OUT/pytest.log; grep -E "^E |FAILED" $OUT/pytest.log | head; [ $rc -ne 0 ] && exit 1
for G in 1024 2048 4096 8192; do timeout -k 10 400 python tools/tree_hint_ab.py --games $G --moves 3 --warmup 1 > $OUT/ab$G.json 2> $OUT/ab$G.err || exit 1; python -c "import json; d=json.load(open('$OUT/ab$G.json')); print($G, d['k_expand_select_mean_us'], d['speedup'])"; done
