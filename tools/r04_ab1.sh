#!/bin/bash
# round 4 A/Bs: Winograd core vs the direct tower (same box, same process); trainer batched vs per-step loss terms
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/winograd_core_ab.bin 1024 > gpurun_out/r04_winograd_core_ab.json || { echo "probe failed"; exit 1; }
cat gpurun_out/r04_winograd_core_ab.json
for round in 1 2; do
  for v in batched per_step; do
    flag=""; [ $v = per_step ] && flag="--per-step-loss"
    timeout -k 10 240 python3 tools/bench_trainer.py --steps 40 --per $flag > gpurun_out/r04_trainer_${v}_$round.json 2> gpurun_out/r04_trainer_${v}_$round.err \
      || { echo "$v failed"; tail -5 gpurun_out/r04_trainer_${v}_$round.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r04_trainer_${v}_$round.json')); print('%-10s %.2f steps/s' % ('$v', d['value']))"
  done
done
