#!/bin/bash
# Tower grid cap sweep of the two-stream engine (tools/dual_stream_probe.py), alternated.  Usage: bash tools/cap_sweep.sh TAG "192 224 256"
TAG=$1; CAPS=$2
OUT=gpurun_out/cap_$TAG
mkdir -p $OUT
for r in 1 2; do
  for c in $CAPS; do
    timeout -k 10 300 python3 tools/dual_stream_probe.py --parts 2 --max-grid $c --moves 6 --warmup 2 > $OUT/c${c}_$r.json 2> $OUT/c${c}_$r.err || { echo "cap $c failed"; tail -3 $OUT/c${c}_$r.err; exit 1; }
    echo "cap $c $(tail -c 300 $OUT/c${c}_$r.json)"
  done
done
