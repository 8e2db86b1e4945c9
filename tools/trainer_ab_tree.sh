#!/bin/bash
# Same-box A/B of the trainer step (tools/bench_trainer.py) between the current tree and a git worktree of an older
# commit in _ab_old/ (git worktree add _ab_old <rev>; copy or build its libgmz.so), alternated ROUNDS times.
#   bash tools/trainer_ab_tree.sh TAG ROUNDS [bench_trainer.py args]
TAG=$1; ROUNDS=${2:-3}; shift 2
ARGS=${@:---per --steps 40 --warmup 6}
OUT=$PWD/gpurun_out/tab_$TAG
mkdir -p $OUT
for i in $(seq 1 $ROUNDS); do
  (cd _ab_old && timeout -k 10 300 python tools/bench_trainer.py $ARGS > $OUT/old_$i.json 2> $OUT/old_$i.err) || { echo "old failed"; tail -3 $OUT/old_$i.err; exit 1; }
  timeout -k 10 300 python tools/bench_trainer.py $ARGS > $OUT/new_$i.json 2> $OUT/new_$i.err || { echo "new failed"; tail -3 $OUT/new_$i.err; exit 1; }
  python3 -c "import json;a=json.load(open('$OUT/old_$i.json'));b=json.load(open('$OUT/new_$i.json'));print('round $i: old %.2f new %.2f steps/s'%(a['value'],b['value']))"
done
