#!/bin/bash
# trainer A/B of the remaining runtime switches: conv halves per workgroup, finaliser threads
set -o pipefail
OUT=gpurun_out/knobs
mkdir -p $OUT
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python3 -u tools/bench_trainer.py --steps 40 --warmup 8 --per > $OUT/tr_${n}_$i.json 2> $OUT/tr_${n}_$i.err || { echo "trainer $n failed"; tail -3 $OUT/tr_${n}_$i.err; exit 1; }
  echo "trainer $n: $(python3 -c "import json; print(json.loads(open('$OUT/tr_${n}_$i.json').read().strip().splitlines()[-1])['value'])")" | tee -a $OUT/summary.txt
}
for i in 1 2; do
  run base GMZ_NONE=1
  run halves2 GMZ_CONV_HALVES=2
  run fin128 GMZ_BN_FIN_THREADS=128
  run fin64 GMZ_BN_FIN_THREADS=64
done
