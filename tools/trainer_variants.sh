# Trainer throughput variants on one box (same process image, sequential).  -> gpurun_out/tvar/
#   bash tools/trainer_variants.sh                       (default set)
#   bash tools/trainer_variants.sh "name:--flags" ...    (named variants; "base:" = no flags)
OUT=gpurun_out/tvar
mkdir -p $OUT
run() {  # name, args
  timeout -k 10 240 python3 tools/bench_trainer.py --steps 30 $2 > $OUT/$1.json 2> $OUT/$1.err || { echo "variant $1 failed"; tail -5 $OUT/$1.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/$1.json')); print('%-30s %.2f steps/s %.1f ms' % ('$1', d['value'], d['ms_per_step']))"
}
if [ $# -eq 0 ]; then
  set -- "default:" "sync:--sync-logs" "per:--per" "per_sync:--per --sync-logs" "nchw:--nchw"
fi
for v in "$@"; do
  run "${v%%:*}" "${v#*:}" || exit 1
done
