#!/bin/bash
# does keeping the tower's weight stream in the XCD L2 raise the clock?
# tools/tower_clock.bin variants (0 product, 1 weights aliased onto <= 3.5 MB = ablation, 2 tail past 3.5 MB
# non-temporal): in-kernel clock + ms per 1,024 rows, then one PMC pass per counter group and variant.
# Run on the box:  gpurun --timeout 900 -- bash tools/r05_tower_l2.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-r05_l2}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 tools/tower_clock.bin 1024 3 > $OUT/clock.txt 2>&1 || { echo "clock failed"; tail -5 $OUT/clock.txt; exit 1; }
cat $OUT/clock.txt
for V in 0 1 2; do
  for CTR in FETCH_SIZE "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"; do
    NAME=v${V}_$(echo $CTR | tr ' ' '_')
    timeout -s KILL 90 rocprofv3 --pmc $CTR --kernel-include-regex "k_tower3" --output-format csv -d $OUT/$NAME -o pmc -- \
      tools/tower_clock.bin 1024 0 $V > $OUT/$NAME.log 2>&1 || { echo "pmc $NAME failed"; tail -3 $OUT/$NAME.log; exit 1; }
  done
  K=("k_tower3<15, true, 0," "k_tower3<15, true, 2048," "k_tower3<15, true, 4096,")
  echo "== variant $V (${K[$V]})" >> $OUT/pmc_summary.txt
  for CTR in FETCH_SIZE "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"; do
    NAME=v${V}_$(echo $CTR | tr ' ' '_')
    python3 tools/pmc_summary.py $OUT/$NAME "${K[$V]}" fp16 1 >> $OUT/pmc_summary.txt
  done
done
cat $OUT/pmc_summary.txt
