#!/bin/bash
# Same-box A/B of a runtime environment variable on the self-play bench.  Usage: bash tools/env_ab.sh TAG "VAR=a" "VAR=b"
TAG=$1; A=$2; B=$3
OUT=gpurun_out/env_$TAG
mkdir -p $OUT
SP="--steps 4 --warmup 1 --no-cpu-baseline --trainer-steps 0 --loop-iters 0 --single-stream-moves 0"
for i in 1 2 3; do
  for V in "$A" "$B"; do
    N=$(echo $V | tr '=' '_')
    env $V timeout -k 10 300 python3 bench.py $SP > $OUT/${N}_$i.json 2> $OUT/${N}_$i.err || { echo "$V failed"; tail -3 $OUT/${N}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${N}_$i.json')); print('$V', '%.0f moves/s tower %.3f ms tree %.1f us' % (d['value'], d['roofline']['mean_launch_ms'], d['roofline_tree']['mean_launch_ms']*1e3))"
  done
done
