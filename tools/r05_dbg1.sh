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
tail -20 $OUT/gloo_trainer.err; cat $OUT/gloo_trainer.json; [ $rc -eq 0 ] || exit $rc
# the gloo rehearsal's loop phase alone (the phase that aborted in r05_batch1), kernels serialised
GMZ_DIST_BACKEND=gloo AMD_SERIALIZE_KERNEL=3 timeout -k 10 400 python3 bench.py --gpus 2 --games 64 --size 9 --sims 50 \
  --blocks 1 --steps 2 --warmup 1 --trainer-steps 0 --trainer-batch 16 --trainer-buffer 64 --loop-iters 4 --loop-warmup 4 \
  --loop-games 64 --loop-update-interval 2 --loop-prefill 64 --loop-buffer 4096 --sublines= --worker-moves 0 \
  --dist-timeout 60 --no-cpu-baseline > $OUT/loop2.json 2> $OUT/loop2.err; rc=$?
grep -iE "fault|error|abort|Traceback" $OUT/loop2.err | head -20; tail -c 1500 $OUT/loop2.json; exit $rc
