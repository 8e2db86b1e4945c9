#!/bin/bash
# with the paired apply pass: elementwise position steps per thread 2 (default) vs 4, trainer
set -o pipefail
OUT=gpurun_out/ewpair
mkdir -p $OUT
for i in 1 2 3; do
  for n in 2 4; do
    GMZ_BN_EW_STEPS=$n timeout -k 10 240 python3 -u tools/bench_trainer.py --steps 40 --warmup 8 --per > $OUT/tr_${n}_$i.json 2> $OUT/tr_${n}_$i.err || { echo "trainer $n failed"; tail -3 $OUT/tr_${n}_$i.err; exit 1; }
    echo "trainer steps $n: $(python3 -c "import json; print(json.loads(open('$OUT/tr_${n}_$i.json').read().strip().splitlines()[-1])['value'])")" | tee -a $OUT/summary.txt
  done
done
