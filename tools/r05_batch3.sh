#!/bin/bash
# round 5 GPU batch 3: tower wave decompositions (tools/tower_clock.bin variants 0, 7, 8) and the trainer's eager
# op census after the batched consistency pass.
set -o pipefail
OUT=gpurun_out/r05_b3
mkdir -p $OUT
timeout -k 10 200 tools/tower_clock.bin 1024 3 078 > $OUT/clock.txt 2>&1 || { echo "clock failed"; tail -5 $OUT/clock.txt; exit 1; }
cat $OUT/clock.txt
timeout -k 10 300 python3 tools/trainer_ops.py > $OUT/ops.txt 2> $OUT/ops.err || { echo "census failed"; tail -5 $OUT/ops.err; exit 1; }
head -40 $OUT/ops.txt
