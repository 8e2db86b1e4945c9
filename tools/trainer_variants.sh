# Trainer throughput variants on one box (same process image, sequential).  -> gpurun_out/tvar/
OUT=gpurun_out/tvar
mkdir -p $OUT
run() {  # name, args
  timeout -k 10 240 python3 tools/bench_trainer.py --steps 20 $2 > $OUT/$1.json 2> $OUT/$1.err || { echo "variant $1 failed"; tail -5 $OUT/$1.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/$1.json')); print('%-30s %.2f steps/s %.1f ms' % ('$1', d['value'], d['ms_per_step']))"
}
run default "" && run sync "--sync-logs" && run per "--per" && run per_sync "--per --sync-logs" && run nchw "--nchw"
