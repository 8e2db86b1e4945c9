#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) on the default self-play step (two streams: 512 rows /
# games per launch) for the dynamics tower and the tree kernel -> gpurun_out/pmc_r02; the FETCH/WRITE
# summaries become profiles/pmc_tower_latest.json / pmc_tree_latest.json (bench.py 'traffic').
OUT=gpurun_out/pmc_r02
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
SP="--steps 1 --warmup 0 --no-cpu-baseline --trainer-steps 0 --loop-iters 0 --single-stream-moves 0"
for CTR in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES"; do
  NAME=$(echo $CTR | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 240 rocprofv3 --pmc $CTR --kernel-include-regex "k_tower3|k_expand_select" --output-format csv -d $OUT/$NAME -o pmc -- \
    python3 bench.py $SP > $OUT/$NAME.json 2> $OUT/$NAME.err || { echo "pmc $CTR failed"; tail -3 $OUT/$NAME.err; exit 1; }
  echo "pass $NAME done"
done
for K in "k_tower3<15, true" "k_expand_select"; do
  echo "== $K"; python3 tools/pmc_summary.py $OUT "$K" fp16 2
done > $OUT/summary.txt
cat $OUT/summary.txt
