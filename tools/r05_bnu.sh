#!/bin/bash
# A/B of the backward reduction's positions per trip (GMZ_BNL_BWD_U build variants in _ab/; this build: 2)
set -o pipefail
OUT=gpurun_out/bnu
mkdir -p $OUT
for i in 1 2 3; do
  for n in u2 u3 u4 u1; do
    L=datou-gomoku-muzero_amd/libgmz.so; [ $n != u2 ] && L=_ab/libgmz_$n.so
    GMZ_LIB=$PWD/$L timeout -k 10 120 python3 tools/bn_bench.py 300 > $OUT/bn_${n}_$i.json 2> $OUT/bn_${n}_$i.err || { echo "bn $n failed"; tail -3 $OUT/bn_${n}_$i.err; exit 1; }
    echo "$n: $(cat $OUT/bn_${n}_$i.json)" | tee -a $OUT/summary.txt
  done
done
