# trainer BatchNorm A/B switches re-measured on the round-6 kernels: FUSED_BN_BWD_STATS, RELU_MASK (alternated)
O=gpurun_out/r06_bnknobs
mkdir -p $O
for r in 1 2; do
  for v in "base:" "bwdstats:--bn-bwd-stats" "relumask:--relu-mask"; do
    n=${v%%:*}; f=${v#*:}
    timeout -k 10 300 python tools/bench_trainer.py --per --steps 40 --warmup 6 $f > $O/${n}_$r.json 2> $O/${n}_$r.err || { echo "$n failed"; tail -3 $O/${n}_$r.err; exit 1; }
    python3 -c "import json;a=json.load(open('$O/${n}_$r.json'));print('round $r %-9s %.2f steps/s'%('$n',a['value']))"
  done
done
