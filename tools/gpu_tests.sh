#!/bin/bash
# GPU test suite only (round 2 iterations).  Usage: bash tools/gpu_tests.sh TAG [pytest -k expr]
OUT=gpurun_out/tests_${1:-x}
mkdir -p $OUT
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"
grep -E "FAILED|^E  " $OUT/pytest.log | head -30
grep -E "^loss |worst relative|top1_agreement" $OUT/pytest.log | head
exit $rc
