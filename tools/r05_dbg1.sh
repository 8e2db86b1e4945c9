#!/bin/bash
# debug batch: the dynamics stem conv pieces, then the N = 1 C4 loop test, then the 2-rank gloo trainer (serialised
# kernels, stderr kept) - each step bounded; a failure stops the chain
set -o pipefail
OUT=gpurun_out/r05_dbg1
mkdir -p $OUT
timeout -k 10 120 python3 tools/dbg_stem.py > $OUT/stem.txt 2>&1; rc=$?; cat $OUT/stem.txt | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "c4_loop_at_its_own" > $OUT/loop1.log 2>&1; rc=$?; tail -3 $OUT/loop1.log; [ $rc -eq 0 ] || exit $rc
GMZ_DIST_BACKEND=gloo AMD_SERIALIZE_KERNEL=3 timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29731 tools/bench_trainer.py --size 9 --blocks 1 --batch 16 --steps 4 --warmup 4 \
  --buffer 256 > $OUT/gloo_trainer.json 2> $OUT/gloo_trainer.err; rc=$?
tail -20 $OUT/gloo_trainer.err; cat $OUT/gloo_trainer.json; exit $rc
