#!/bin/bash
# PMC passes on the trainer's HIP conv (k_conv3) in tools/conv_bench.py.  -> gpurun_out/pmc_wgrad
OUT=gpurun_out/pmc_wgrad
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for CTR in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM"; do
  NAME=$(echo $CTR | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-include-regex "k_conv3_wgrad" --output-format csv -d $OUT/$NAME -o pmc -- \
    python3 tools/conv_bench.py 360 > $OUT/$NAME.txt 2> $OUT/$NAME.err || { echo "pmc $CTR failed"; tail -3 $OUT/$NAME.err; exit 1; }
done
python3 tools/pmc_summary.py $OUT "k_conv3_wgrad" | tee $OUT/summary.txt
