#!/bin/bash
# k_conv3 A/B builds on one box: timing (alternated, 3 rounds) and one LDS + one MFMA PMC pass per build.
#   bash tools/conv_lds_ab.sh TAG N lib1 lib2 ...   (lib = a name under datou-gomoku-muzero_amd/_alt/libgmz_NAME.so,
#   or "cur" for the in-tree libgmz.so)  -> gpurun_out/TAG/
set -o pipefail
TAG=$1; N=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
libpath() { [ "$1" = cur ] && echo $PWD/datou-gomoku-muzero_amd/libgmz.so || echo $PWD/datou-gomoku-muzero_amd/_alt/libgmz_$1.so; }
for r in 1 2 3; do
  for L in "$@"; do
    GMZ_LIB=$(libpath $L) timeout -k 10 120 python3 tools/conv_probe.py $N 15 40 >> $OUT/time_$L.txt 2>&1 || { echo "time $L failed"; tail -3 $OUT/time_$L.txt; exit 1; }
  done
done
for L in "$@"; do
  mkdir -p $OUT/pmc_$L
  for CTR in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"; do
    NAME=$(echo $CTR | cut -d' ' -f1)
    GMZ_LIB=$(libpath $L) timeout -s KILL 90 rocprofv3 --pmc $CTR --kernel-include-regex "k_conv3<" --output-format csv \
      -d $OUT/pmc_$L/$NAME -o pmc -- python3 tools/conv_probe.py $N 15 20 > $OUT/pmc_$L/$NAME.txt 2>&1 || { echo "pmc $L $NAME failed"; exit 1; }
  done
  echo "== $L" >> $OUT/summary.txt
  python3 tools/pmc_summary.py $OUT/pmc_$L "k_conv3<15, __half, 2, 1, false, false>" >> $OUT/summary.txt
done
for L in "$@"; do echo "== $L"; grep -h "fwd \|dgrad" $OUT/time_$L.txt | awk '{print $1, $2}' | tr '\n' ' '; echo; done | tee $OUT/time_summary.txt
grep -E "^==|BANK|IDX_ACTIVE|INSTS_LDS|MFMA busy|clock|duration" $OUT/summary.txt
