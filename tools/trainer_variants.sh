# Trainer throughput variants on one box (same process image, sequential).  -> gpurun_out/tvar/
OUT=gpurun_out/tvar
mkdir -p $OUT
for V in "" "--channels-last" "--bf16" "--bf16 --channels-last" "--channels-last --benchmark"; do
  N=$(echo "x$V" | tr -d ' -')
  timeout -k 10 240 python3 tools/bench_trainer.py --steps 15 $V > $OUT/$N.json 2> $OUT/$N.err || { echo "variant $V failed"; tail -5 $OUT/$N.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/$N.json')); print('%-30s %.2f steps/s %.1f ms' % ('$V', d['value'], d['ms_per_step']))"
done
