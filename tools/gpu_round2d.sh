#!/bin/bash
# Round-2 re-entry check: GPU test suite, default bench line, descent-hint A/B.
OUT=gpurun_out/r2_d
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -30; exit 1; }
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 python tools/tree_hint_ab.py --moves 10 > $OUT/hint_ab.json 2> $OUT/hint_ab.err || { echo "hint ab failed"; tail -20 $OUT/hint_ab.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/hint_ab.json')); print(d['k_expand_select_mean_us'], d['speedup'])"
