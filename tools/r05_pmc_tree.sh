#!/bin/bash
# PMC HBM bytes of the tree kernel k_expand_select at the headline (1,024 games, two streams) and at the g8192
# sub-line (8,192 games, one engine, one stream): FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes
# (MI355X_MICROARCH.md), summarised by tools/pmc_summary.py into pmc_tree.json (games / streams recorded), which
# bench.py's roofline_tree.frac_measured reads once copied to profiles/pmc_tree_latest.json / pmc_tree_g8192.json.
# Run on the box:  gpurun --timeout 900 -- bash tools/r05_pmc_tree.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-r05_pmc_tree}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
SP="--no-cpu-baseline --trainer-steps 0 --loop-iters 0 --sublines= --worker-moves 0 --single-stream-moves 0"
for CFG in "1024 2" "8192 1"; do
  set -- $CFG
  G=$1; S=$2
  mkdir -p $OUT/G${G}
  for CTR in FETCH_SIZE WRITE_SIZE; do
    D=$OUT/G${G}/$CTR
    timeout -s KILL 240 rocprofv3 --pmc $CTR --kernel-include-regex "k_expand_select" --output-format csv -d $D -o pmc -- \
      python3 bench.py --games $G --streams $S --steps 1 --warmup 0 $SP > $D.json 2> $D.err || { echo "pmc G=$G $CTR failed"; tail -3 $D.err; exit 1; }
  done
  echo "== G=$G streams=$S" | tee -a $OUT/summary.txt
  python3 tools/pmc_summary.py $OUT/G${G} "k_expand_select" fp16 $S $G | tee -a $OUT/summary.txt
done
