set -o pipefail
for v in "" "--benchmark" "--bf16" "--bf16 --benchmark" "--bf16 --channels-last --benchmark" "--channels-last --benchmark"; do
  timeout -k 10 300 python tools/bench_trainer.py --steps 10 --warmup 4 $v > gpurun_out/trv.json 2>gpurun_out/trv.err || { echo "fail $v"; tail -3 gpurun_out/trv.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/trv.json')); print('$v', round(d['value'],2), 'steps/s', round(d['ms_per_step'],1), 'ms')"
done
