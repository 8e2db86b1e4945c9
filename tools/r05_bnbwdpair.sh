#!/bin/bash
# A/B of the BatchNorm backward apply pass with two positions per trip (this build) against one (_ab/libgmz_nobwdpair.so)
set -o pipefail
OUT=gpurun_out/bnbwdpair
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_trainer.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "fused_masked_bn or fused_bn_finalisation or bn_backward_sums or trainer_step_on_gpu or gpu_loss_and_gradients or production" > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  for n in pair nobwdpair; do
    L=datou-gomoku-muzero_amd/libgmz.so; [ $n = nobwdpair ] && L=_ab/libgmz_nobwdpair.so
    GMZ_LIB=$PWD/$L timeout -k 10 120 python3 tools/bn_bench.py 300 > $OUT/bn_${n}_$i.json 2> $OUT/bn_${n}_$i.err || { echo "bn $n failed"; tail -3 $OUT/bn_${n}_$i.err; exit 1; }
    echo "$n: $(cat $OUT/bn_${n}_$i.json)" | tee -a $OUT/summary.txt
  done
done
for i in 1 2 3; do
  for n in pair nobwdpair; do
    L=datou-gomoku-muzero_amd/libgmz.so; [ $n = nobwdpair ] && L=_ab/libgmz_nobwdpair.so
    GMZ_LIB=$PWD/$L timeout -k 10 240 python3 -u tools/bench_trainer.py --steps 40 --warmup 8 --per > $OUT/tr_${n}_$i.json 2> $OUT/tr_${n}_$i.err || { echo "trainer $n failed"; tail -3 $OUT/tr_${n}_$i.err; exit 1; }
    echo "trainer $n: $(python3 -c "import json; print(json.loads(open('$OUT/tr_${n}_$i.json').read().strip().splitlines()[-1])['value'])")" | tee -a $OUT/summary.txt
  done
done
