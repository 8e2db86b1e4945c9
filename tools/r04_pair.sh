#!/bin/bash
# round 4: two-waves-per-game tree kernel — parity, then same-box timing A/B (one engine, one stream; and the
# two-stream headline) -> gpurun_out/pair/
set -o pipefail
OUT=gpurun_out/pair
mkdir -p $OUT
SP="--no-cpu-baseline --trainer-steps 0 --loop-iters 0 --sublines= --worker-moves 0"
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_tree_pair_gpu.py \
  > $OUT/tests.log 2>&1 || { echo "pair tests failed"; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; exit 1; }
tail -1 $OUT/tests.log
for round in 1 2; do
  for G in 1024 2048; do
    for P in off on; do
      N=G${G}_s1_${P}_$round
      timeout -k 10 300 python -u bench.py --games $G --streams 1 --steps 4 --warmup 1 --pair $P --single-stream-moves 0 $SP \
        > $OUT/$N.json 2> $OUT/$N.err || { echo "$N failed"; tail -5 $OUT/$N.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); t=d['roofline_tree']; print('%-18s moves/s %8.0f  tree %6.1f us  frac %.3f  wpg %d' % (sys.argv[2], d['value'], t['mean_launch_ms']*1e3, t['frac'], t['waves_per_game']))" $OUT/$N.json $N | tee -a $OUT/summary.txt
    done
  done
  for P in off on; do
    N=headline_${P}_$round
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --pair $P $SP > $OUT/$N.json 2> $OUT/$N.err || { echo "$N failed"; tail -5 $OUT/$N.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); t=d['roofline_tree']; s=d['single_stream_kernels']; print('%-18s moves/s %8.0f  tree in step %6.1f us  alone %6.1f us frac %.3f' % (sys.argv[2], d['value'], t['mean_launch_ms']*1e3, s['tree']['mean_launch_ms']*1e3, s['tree']['frac']))" $OUT/$N.json $N | tee -a $OUT/summary.txt
  done
done
