# the batched conv-weight re-pack (trainer.BATCH_REPACK: one gmz_conv3x3_pack_many per step) vs one pack per weight:
# its tests, then the trainer A/B alternated on one box
set -o pipefail
O=gpurun_out/r06_repack
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_repack_gpu.py tests/test_fused_opt_gpu.py tests/test_bn_apply_gpu.py > $O/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|^E " $O/pytest.log | head -30; tail -3 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  timeout -k 10 300 python tools/bench_trainer.py --per --steps 40 --warmup 6 --no-batch-repack > $O/off_$r.json 2> $O/off_$r.err || exit 1
  timeout -k 10 300 python tools/bench_trainer.py --per --steps 40 --warmup 6 > $O/on_$r.json 2> $O/on_$r.err || exit 1
  python3 -c "import json;a=json.load(open('$O/off_$r.json'));b=json.load(open('$O/on_$r.json'));print('round $r: per-use packs %.2f  batched re-pack %.2f steps/s'%(a['value'],b['value']))"
done
