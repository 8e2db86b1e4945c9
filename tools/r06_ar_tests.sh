O=gpurun_out/r06_ar2
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_rccl_gpu.py tests/test_graph_allreduce_gpu.py tests/test_capture_race_gpu.py > $O/pytest.log 2>&1; rc=$?; tail -12 $O/pytest.log; exit $rc
