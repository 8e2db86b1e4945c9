#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root): kernel-trace stats of the bench, then
# separate PMC passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950) restricted to the
# dynamics tower kernel.  Outputs under gpurun_out/prof_<tag>/.
set -e
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_under_trace.json 2> $OUT/trace.err
for CTR in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum"; do
  NAME=$(echo $CTR | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $CTR --kernel-include-regex "k_tower" --output-format csv -d $OUT/pmc_$NAME -o pmc -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc_$NAME.json 2> $OUT/pmc_$NAME.err || echo "pmc $CTR failed rc=$?"
done
echo done
