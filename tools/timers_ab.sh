#!/bin/bash
# the headline with and without the HIP events around every tower / tree launch (their own cost), alternating
# on one box -> gpurun_out/tab/
set -o pipefail
OUT=gpurun_out/tab
mkdir -p $OUT
COMMON="--steps 20 --warmup 2 --sublines= --worker-moves 0 --trainer-steps 0 --loop-iters 0 --no-cpu-baseline --single-stream-moves 0"
for i in 1 2 3; do
  for v in on off; do
    timeout -k 10 200 python3 bench.py $COMMON --kernel-timers $v > $OUT/${v}_$i.json 2> $OUT/${v}_$i.err || { echo "$v failed"; tail -3 $OUT/${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/${v}_$i.json').read().strip().splitlines()[-1]); print('$v $i %.0f moves/s %.2f ms/step' % (d['value'], d['ms_per_step']))" | tee -a $OUT/summary.txt
  done
done
