#!/bin/bash
# Tree-kernel variant sweep: tools/tree_hint_ab.py (hint on/off, k_expand_select mean us) per library.
# Usage: bash tools/gpu_tree_var.sh TAG G "lib1 lib2 ..." (names under datou-gomoku-muzero_amd/_alt/libgmz_NAME.so; cur = in-tree)
TAG=$1; G=$2; LIBS=$3
OUT=gpurun_out/var_$TAG
mkdir -p $OUT
for r in 1 2; do
  for n in $LIBS; do
    L=$PWD/datou-gomoku-muzero_amd/_alt/libgmz_$n.so
    [ "$n" = cur ] && L=$PWD/datou-gomoku-muzero_amd/libgmz.so
    GMZ_LIB=$L timeout -k 10 300 python tools/tree_hint_ab.py --games $G --moves 3 --warmup 1 > $OUT/${n}_$r.json 2> $OUT/${n}_$r.err || { echo "$n failed"; tail -3 $OUT/${n}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/${n}_$r.json')); m=d['k_expand_select_mean_us']; print('$n', $G, 'hint %.1f  no_hint %.1f' % (m['hint'], m['no_hint']))"
  done
done
