# Trainer step under HIP-runtime environment variants (same box, alternating).  -> gpurun_out/tenv/
#   bash tools/trainer_env_ab.sh "name:VAR=value ..." ...     ("base:" = no variables)
OUT=gpurun_out/tenv
mkdir -p $OUT
for round in 1 2; do
  for v in "$@"; do
    name=${v%%:*}
    vars=${v#*:}
    env_args=()
    for kv in $vars; do env_args+=("$kv"); done
    ( [ ${#env_args[@]} -gt 0 ] && export "${env_args[@]}"; timeout -k 10 240 python3 tools/bench_trainer.py --steps 30 > $OUT/${name}_$round.json 2> $OUT/${name}_$round.err ) || { echo "$name failed"; tail -3 $OUT/${name}_$round.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${name}_$round.json')); print('%-24s %.2f steps/s' % ('$name', d['value']))"
  done
done
