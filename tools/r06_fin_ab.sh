# k_bn_finalize's partial-record unroll (GMZ_FIN_UNROLL 2 = product, 4, 8; same summation order): its mean duration
# under rocprofv3 inside the graph-replayed trainer step, and the trainer line, alternated on one box
set -o pipefail
O=gpurun_out/r06_fin
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for r in 1 2; do
  for v in base fin4 fin8; do
    L=""; [ $v != base ] && L=$PWD/datou-gomoku-muzero_amd/_alt/libgmz_$v.so
    GMZ_LIB=$L timeout -k 10 300 python tools/bench_trainer.py --per --steps 40 --warmup 6 > $O/${v}_$r.json 2> $O/${v}_$r.err || exit 1
    GMZ_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_${v}_$r -o run -- python3 tools/bench_trainer.py --per --steps 20 --warmup 6 > /dev/null 2> $O/tr_${v}_$r.err || exit 1
    python3 - $O $v $r <<'PY'
import csv, glob, json, sys
O, v, r = sys.argv[1:]
f = glob.glob("%s/tr_%s_%s/**/run_kernel_stats.csv" % (O, v, r), recursive=True)[0]
fin = [row for row in csv.DictReader(open(f)) if row["Name"].startswith("gmz::(anonymous namespace)::k_bn_finalize(")]
b = json.load(open("%s/%s_%s.json" % (O, v, r)))
print("%s round %s: trainer %.2f steps/s, k_bn_finalize %s calls avg %.2f us" % (v, r, b["value"], fin[0]["Calls"], float(fin[0]["AverageNs"]) / 1e3))
PY
  done
done
