#!/bin/bash
# tree kernel after the AZ/hint templating: engine/adapter GPU tests, hint A/B at 4096 and 8192 games,
# G = 8192 bench line (its single-stream segment = the tree kernel alone at 8192 trees)
OUT=gpurun_out/tocc
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_adapter_gpu.py tests/test_split_gpu.py tests/test_reanalysis_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -1 $OUT/pytest.log; grep -E "^E |FAILED" $OUT/pytest.log | head; [ $rc -ne 0 ] && exit 1
for G in 4096 8192; do
timeout -k 10 400 python tools/tree_hint_ab.py --games $G --moves 3 --warmup 1 > $OUT/ab$G.json 2> $OUT/ab$G.err || { tail -3 $OUT/ab$G.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/ab$G.json')); print($G, d['k_expand_select_mean_us'], d['speedup'])"
done
timeout -k 10 500 python3 bench.py --games 8192 --steps 3 --warmup 1 --no-cpu-baseline --trainer-steps 0 --loop-iters 0 > $OUT/bench_G8192.json 2> $OUT/bench_G8192.err || { tail -3 $OUT/bench_G8192.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_G8192.json')); print(d['value'], d['single_stream_kernels'])"
