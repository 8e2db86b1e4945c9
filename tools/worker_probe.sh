#!/bin/bash
# Worker leg vs the engine: staggered openings on/off, one stream vs two (bench.py's worker leg only)
SP="--no-cpu-baseline --trainer-steps 0 --loop-iters 0 --sublines= --steps 4 --warmup 1 --single-stream-moves 0 --worker-moves 20"
OUT=gpurun_out/wprobe
mkdir -p $OUT
for OP in 0 80; do
  for ST in 2 1; do
    N=op${OP}_st$ST
    timeout -k 10 300 python -u bench.py $SP --worker-openings $OP --streams $ST > $OUT/$N.json 2> $OUT/$N.err || { tail -5 $OUT/$N.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); w=d['worker']; print(sys.argv[2], 'engine %.0f (waves/move %.1f) worker %.0f ratio %.3f games %d move_ms %s' % (d['value'], d['config']['waves_per_move'], w['value'], w['worker_over_engine'], w['finished_games'], w['move_ms'][:6]))" $OUT/$N.json $N
  done
done
