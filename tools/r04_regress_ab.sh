#!/bin/bash
# same-box A/B of the headline self-play step (15x15 / 400 sims / 1,024 games, empty boards, two streams):
# round 3's tree (_r03/, git archive of the round-3 driver commit with its own libgmz.so) vs this tree,
# alternating, three rounds -> gpurun_out/reg/
set -o pipefail
OUT=gpurun_out/reg
mkdir -p $OUT
COMMON="--steps 20 --warmup 2 --sublines= --worker-moves 0 --trainer-steps 0 --loop-iters 0 --no-cpu-baseline --single-stream-moves 0"
for round in 1 2 3 4; do
  (cd _r03 && timeout -k 10 200 python3 bench.py $COMMON > ../$OUT/r03_$round.json 2> ../$OUT/r03_$round.err) \
    || { echo "r03 failed"; tail -5 $OUT/r03_$round.err; exit 1; }
  timeout -k 10 200 python3 bench.py $COMMON --stagger -1 --isolate off > $OUT/r04_$round.json 2> $OUT/r04_$round.err \
    || { echo "r04 failed"; tail -5 $OUT/r04_$round.err; exit 1; }
  for v in r03 r04; do
    python3 -c "
import json; d=json.loads(open('$OUT/${v}_$round.json').read().strip().splitlines()[-1]); r=d['roofline']; t=d.get('roofline_tree', {})
print('%s %d  %.0f moves/s  %.2f ms/step  tower %.4f ms x %d busy %.1f ms  tree %.4f ms' % ('$v', $round, d['value'], d['ms_per_step'],
      r['mean_launch_ms'], r['launches'], r['busy_ms'], t.get('mean_launch_ms', 0)), d.get('step_ms', ''))" | tee -a $OUT/summary.txt
  done
done
