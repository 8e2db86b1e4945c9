# C5 (19x19, 800 sims, 16 blocks) tower time per library build (GMZ_LIB), alternating, 2 rounds.  -> gpurun_out/c5ab/
OUT=gpurun_out/c5ab
mkdir -p $OUT
SP="--size 19 --sims 800 --blocks 16 --steps 2 --warmup 1 --no-cpu-baseline --trainer-steps 0 --loop-iters 0 --sublines= --worker-moves 0 --single-stream-moves 0"
for round in 1 2; do
  for lib in "$@"; do
    n=$(basename $lib .so)
    GMZ_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py $SP > $OUT/${n}_$round.json 2> $OUT/${n}_$round.err || { echo "$n failed"; tail -3 $OUT/${n}_$round.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${n}_$round.json')); r=d['roofline']; print('%-22s moves/s %7.1f  tower %.3f ms frac %.3f' % ('$n', d['value'], r['mean_launch_ms'], r['frac']))"
  done
done
