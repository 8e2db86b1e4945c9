# the unroll's step masks and live-step count from one [U, B] mask (fewer small launches per step) — trainer GPU
# tests, then the default trainer line three times (compare with the same box's earlier lines)
set -o pipefail
O=gpurun_out/r06_loss
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_trainer.py tests/test_repack_gpu.py tests/test_bn_apply_gpu.py tests/test_fused_opt_gpu.py tests/test_rccl_gpu.py > $O/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|^E " $O/pytest.log | head -30; tail -3 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  timeout -k 10 300 python tools/bench_trainer.py --per --steps 40 --warmup 6 > $O/on_$r.json 2> $O/on_$r.err || exit 1
  python3 -c "import json;b=json.load(open('$O/on_$r.json'));print('round $r: %.2f steps/s'%b['value'])"
done
