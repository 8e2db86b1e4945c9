# bench.py's N > 1 path rehearsed with 2 gloo ranks sharing the box's one GPU (the driver's launcher form).
O=gpurun_out/r06_n2
mkdir -p $O
GMZ_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --trainer-steps 4 --trainer-warmup 3 --trainer-f32-steps 0 --loop-iters 3 --loop-warmup 2 --sublines , --worker-moves 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
rc=$?
echo "rc=$rc"
tail -c 1500 $O/bench.json
exit $rc
