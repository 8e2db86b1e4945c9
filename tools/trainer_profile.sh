# Trainer step kernel trace on one box: bench line + steady-state per-kernel window.  -> gpurun_out/tprof/
OUT=gpurun_out/tprof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/bench_trainer.py --steps 10 --warmup 5 $@ > $OUT/bench.json 2> $OUT/err.txt || { echo "trace failed"; tail $OUT/err.txt; exit 1; }
cat $OUT/bench.json
python3 tools/trace_window.py $OUT/trace/run_kernel_trace.csv 400 40
