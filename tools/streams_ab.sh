#!/bin/bash
# One vs two HIP streams on the C5 (19x19/800/16 blocks) and 9x9 AlphaZero configs, alternated.
OUT=gpurun_out/streams_ab
mkdir -p $OUT
SP="--no-cpu-baseline --trainer-steps 0 --loop-iters 0 --single-stream-moves 0"
for r in 1 2; do
  for st in 1 2; do
    timeout -k 10 400 python3 bench.py --size 19 --sims 800 --blocks 16 --steps 3 --warmup 1 --streams $st $SP > $OUT/c5_s${st}_$r.json 2> $OUT/c5_s${st}_$r.err || { echo "c5 failed"; tail -3 $OUT/c5_s${st}_$r.err; exit 1; }
    timeout -k 10 300 python3 bench.py --size 9 --sims 50 --mode AlphaZero --steps 8 --warmup 2 --streams $st $SP > $OUT/c9_s${st}_$r.json 2> $OUT/c9_s${st}_$r.err || { echo "c9 failed"; tail -3 $OUT/c9_s${st}_$r.err; exit 1; }
    python3 -c "import json; a=json.load(open('$OUT/c5_s${st}_$r.json')); b=json.load(open('$OUT/c9_s${st}_$r.json')); print('streams $st: C5 %.0f moves/s, C9 %.0f moves/s' % (a['value'], b['value']))"
  done
done
