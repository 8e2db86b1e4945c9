#!/bin/bash
# Same-box trainer A/B: tools/bench_trainer.py with and without extra flags, alternated 3x.
# Usage: bash tools/gpu_trainer_ab.sh TAG "FLAGS_A" "FLAGS_B"
TAG=$1; FA=$2; FB=$3
OUT=gpurun_out/tab_$TAG
mkdir -p $OUT
for i in 1 2 3; do
  for k in a b; do
    F=$FA; [ $k = b ] && F=$FB
    timeout -k 10 300 python3 tools/bench_trainer.py --steps 30 --warmup 5 $F > $OUT/${k}_$i.json 2> $OUT/${k}_$i.err || { echo "$k failed"; tail -5 $OUT/${k}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${k}_$i.json')); print('$k [$F]', '%.2f steps/s' % d['value'])"
  done
done
