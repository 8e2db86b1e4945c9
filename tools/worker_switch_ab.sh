SP="--no-cpu-baseline --trainer-steps 0 --loop-iters 0 --sublines= --steps 4 --warmup 1 --single-stream-moves 0 --worker-moves 20"
mkdir -p gpurun_out/wab
for i in 1 2; do
for SI in 0.005 2e-4 5e-5; do
  GMZ_WORKER_SWITCH_INTERVAL=$SI timeout -k 10 300 python -u bench.py $SP > gpurun_out/wab/si_${SI}_$i.json 2> gpurun_out/wab/si_${SI}_$i.err || { tail -5 gpurun_out/wab/si_${SI}_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); w=d['worker']; print('si', sys.argv[2], 'engine %.0f worker %.0f ratio %.3f games %d' % (d['value'], w['value'], w['worker_over_engine'], w['finished_games']))" gpurun_out/wab/si_${SI}_$i.json $SI
done
done
