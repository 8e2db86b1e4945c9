#!/bin/bash
# A/B of the NHWC BatchNorm reduction split cap (GMZ_BNL_SPLITS): the BN kernels alone, then the trainer step
set -o pipefail
OUT=gpurun_out/bnsplits
mkdir -p $OUT
for i in 1 2; do
  for n in 512 1024 2048 256; do
    GMZ_BNL_SPLITS=$n timeout -k 10 120 python3 tools/bn_bench.py 300 > $OUT/bn_${n}_$i.json 2> $OUT/bn_${n}_$i.err || { echo "bn $n failed"; tail -3 $OUT/bn_${n}_$i.err; exit 1; }
    echo "splits $n: $(cat $OUT/bn_${n}_$i.json)" | tee -a $OUT/summary.txt
  done
done
for i in 1 2; do
  for n in 512 1024 2048; do
    GMZ_BNL_SPLITS=$n timeout -k 10 240 python3 -u tools/bench_trainer.py --steps 40 --warmup 8 --per > $OUT/tr_${n}_$i.json 2> $OUT/tr_${n}_$i.err || { echo "trainer $n failed"; tail -3 $OUT/tr_${n}_$i.err; exit 1; }
    echo "trainer splits $n: $(python3 -c "import json; print(json.loads(open('$OUT/tr_${n}_$i.json').read().strip().splitlines()[-1])['value'])")" | tee -a $OUT/summary.txt
  done
done
