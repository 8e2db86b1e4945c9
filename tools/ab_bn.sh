#!/bin/bash
# masked-BatchNorm kernels alone (tools/bn_bench.py), one box, alternating over trees (each with its own
# libgmz.so): this tree and the directories given (default _ab_old) -> gpurun_out/abbn/
set -o pipefail
OUT=gpurun_out/abbn
mkdir -p $OUT
DIRS=("." "${@:-_ab_old}")
for i in 1 2 3; do
  line=""
  for d in "${DIRS[@]}"; do
    n=$(basename $(cd $d && pwd))
    (cd $d && timeout -k 10 120 python3 $OLDPWD/tools/bn_bench.py 300) > $OUT/${n}_$i.json 2> $OUT/${n}_$i.err || { echo "$d failed"; tail -3 $OUT/${n}_$i.err; exit 1; }
    line="$line | $n $(python3 -c "import json; d=json.load(open('$OUT/${n}_$i.json')); print('fwd %.2f bwd %.2f us' % (d['forward_us'], d['backward_us']))")"
  done
  echo "$line" | tee -a $OUT/summary.txt
done
