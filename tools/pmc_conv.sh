#!/bin/bash
# PMC passes on the trainer's HIP conv (k_conv3) in tools/conv_bench.py.  -> gpurun_out/pmc_conv
N=${1:-360}
OUT=gpurun_out/pmc_conv_$N
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for CTR in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_WAIT_INST_ANY"; do
  NAME=$(echo $CTR | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-include-regex "k_conv3<" --output-format csv -d $OUT/$NAME -o pmc -- \
    python3 tools/conv_bench.py $N > $OUT/$NAME.txt 2> $OUT/$NAME.err || { echo "pmc $CTR failed"; tail -3 $OUT/$NAME.err; exit 1; }
done
python3 tools/pmc_summary.py $OUT "k_conv3<15, __half, 2, 1, false, false" | tee $OUT/summary.txt
