#!/bin/bash
# PMC passes on the dynamics tower only (one counter group per pass). Usage: tools/pmc_tower.sh TAG
TAG=${1:-x}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for CTR in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES" FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  NAME=$(echo $CTR | tr ' ' '_' | cut -c1-40)
  timeout -k 10 300 rocprofv3 --pmc $CTR --kernel-include-regex "k_tower" --output-format csv -d $OUT/$NAME -o pmc -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/$NAME.json 2> $OUT/$NAME.err || { echo "pmc $CTR failed"; exit 1; }
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt
cat $OUT/summary.txt
