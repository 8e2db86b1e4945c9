#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) on the self-play step's dominant kernels: the
# dynamics tower (k_tower3) and the backup+select kernel (k_expand_select).  -> gpurun_out/pmc_$TAG
TAG=${1:-r01}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for CTR in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" FETCH_SIZE WRITE_SIZE; do
  NAME=$(echo $CTR | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 240 rocprofv3 --pmc $CTR --kernel-include-regex "k_tower3|k_expand_select" --output-format csv -d $OUT/$NAME -o pmc -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/$NAME.json 2> $OUT/$NAME.err || { echo "pmc $CTR failed"; tail -3 $OUT/$NAME.err; exit 1; }
  echo "pass $NAME done"
done
for K in "k_tower3<15, true" "k_expand_select"; do
  echo "== $K"; python3 tools/pmc_summary.py $OUT "$K"
done > $OUT/summary.txt
cat $OUT/summary.txt
