# k_conv3's row-mask bytes: read per board (old lib) vs once per workgroup (in-tree), conv alone at 360 / 1,800 boards
for r in 1 2; do
  for N in 360 1800; do
    echo "old: $(GMZ_LIB=$PWD/datou-gomoku-muzero_amd/_alt/libgmz_prevstats.so timeout -k 10 120 python tools/conv_stats_probe.py $N 15 | tail -1)"
    echo "new: $(timeout -k 10 120 python tools/conv_stats_probe.py $N 15 | tail -1)"
  done
done
