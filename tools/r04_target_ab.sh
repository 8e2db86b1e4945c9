#!/bin/bash
# trainer: the target network's value in f16 operands vs float32 (same box, alternating) -> gpurun_out/tgt/
set -o pipefail
OUT=gpurun_out/tgt
mkdir -p $OUT
for round in 1 2; do
  for v in f32 f16; do
    flag=""; [ $v = f16 ] && flag="--target-f16"
    timeout -k 10 240 python3 tools/bench_trainer.py --steps 40 --per $flag > $OUT/${v}_$round.json 2> $OUT/${v}_$round.err \
      || { echo "$v failed"; tail -5 $OUT/${v}_$round.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${v}_$round.json')); print('target %-4s %.2f steps/s' % ('$v', d['value']))" | tee -a $OUT/summary.txt
  done
done
