#!/bin/bash
# Tree-kernel iteration: engine parity subset, same-box A/B vs the base library at 1,024 and 8,192 games,
# hint on/off A/B per G.  Usage: bash tools/gpu_tree_ab.sh TAG
TAG=${1:-x}
bash tools/gpu_tests.sh $TAG "engine or split or adapter or reanalysis" || exit 1
bash tools/ab_tree.sh $TAG $PWD/datou-gomoku-muzero_amd/_alt/libgmz_base.so --steps 4 --warmup 1 || exit 1
bash tools/ab_tree.sh ${TAG}g8 $PWD/datou-gomoku-muzero_amd/_alt/libgmz_base.so --games 8192 --steps 2 --warmup 1 || exit 1
mkdir -p gpurun_out/hint_$TAG
for G in 2048 4096 8192; do
  timeout -k 10 400 python tools/tree_hint_ab.py --games $G --moves 3 --warmup 1 > gpurun_out/hint_$TAG/ab$G.json 2> gpurun_out/hint_$TAG/ab$G.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/hint_$TAG/ab$G.json')); print($G, d['k_expand_select_mean_us'], d['speedup'])"
done
