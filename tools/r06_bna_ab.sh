# DEFER_BN_APPLY A/B (trainer steps/s, alternated on one box) + the bit-identity tests.  -> gpurun_out/r06_bna/
set -o pipefail
O=gpurun_out/r06_bna
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_bn_apply_gpu.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  timeout -k 10 300 python tools/bench_trainer.py --per --steps 40 --warmup 6 > $O/on_$r.json 2> $O/on_$r.err || exit 1
  timeout -k 10 300 python tools/bench_trainer.py --per --steps 40 --warmup 6 --no-defer-bn > $O/off_$r.json 2> $O/off_$r.err || exit 1
  python -c "import json;a=json.load(open('$O/on_$r.json'));b=json.load(open('$O/off_$r.json'));print('defer on %.2f off %.2f steps/s'%(a['value'],b['value']))"
done
