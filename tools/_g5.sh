set -o pipefail
O=gpurun_out/r06_g5; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_net_gpu.py tests/test_headline_gpu.py tests/test_split_gpu.py tests/test_engine_gpu.py tests/test_trainer.py -m gpu -v --timeout 300 --timeout-method thread -k "net or headline or split or engine or conv3x3 or production_training or consistency_kernels" > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; grep -E "FAILED|Error" $O/pytest.log | head; [ $rc = 0 ] || exit $rc
bash tools/ab_lib.sh r06_g5_ab $PWD/datou-gomoku-muzero_amd/_alt/libgmz_prev.so 2 && \
for L in prev cur; do P=$PWD/datou-gomoku-muzero_amd/_alt/libgmz_prev.so; [ $L = cur ] && P=$PWD/datou-gomoku-muzero_amd/libgmz.so; GMZ_LIB=$P timeout -k 10 120 python3 tools/conv_probe.py 360 15 40 >> $O/conv_$L.txt 2>&1 || exit 1; done && tail -4 $O/conv_prev.txt $O/conv_cur.txt && \
timeout -k 10 300 python3 tools/tree_backup_split.py gpurun_out/r06_g5/tree_backup_split.json --games 1024 8192 > gpurun_out/r06_g5/tree_split.log 2>&1 || { tail -5 gpurun_out/r06_g5/tree_split.log; exit 1; }
tail -2 gpurun_out/r06_g5/tree_split.log
