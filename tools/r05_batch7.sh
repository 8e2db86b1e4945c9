#!/bin/bash
# round 5 GPU batch 7: where the trainer conv's time goes — timing ablations of k_conv3 (A/B builds, results wrong):
# abl1 = one board DMA per workgroup (and the weight gradient without its DMA), abl2 = no epilogue stores,
# abl4 = no MFMAs (operand loads kept), abl3 = 1 + 2; then the tree kernel's PMC bytes (headline + g8192).
set -o pipefail
OUT=gpurun_out/r05_b7
mkdir -p $OUT
( while sleep 60; do date >> $OUT/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
for i in 1 2; do
  for V in base abl1 abl2 abl3 abl4; do
    ENV=""; [ $V != base ] && ENV="GMZ_LIB=$PWD/datou-gomoku-muzero_amd/_alt/libgmz_$V.so"
    for N in 360 1800; do
      env $ENV timeout -k 10 120 python3 tools/conv_bench.py $N > $OUT/conv_${V}_${N}_$i.txt 2>&1 || { echo "conv $V failed"; tail -3 $OUT/conv_${V}_${N}_$i.txt; exit 1; }
      echo "conv $V N=$N $i: $(grep -E '^(hip fwd|hip dgrad|hip wgrad) ' $OUT/conv_${V}_${N}_$i.txt | tr -s ' ' | tr '\n' ';')" | tee -a $OUT/summary.txt
    done
  done
done
bash tools/r05_pmc_tree.sh r05_b7/pmc_tree
