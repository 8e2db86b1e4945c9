# Same-box A/B of the trainer step (tools/bench_trainer.py) between the in-tree libgmz.so and an
# alternative build ($1, e.g. datou-gomoku-muzero_amd/_alt/libgmz_base.so), alternating, 3 runs each.
#   bash tools/trainer_ab_lib.sh ALT_LIB [extra bench_trainer args]   -> gpurun_out/tab/
ALT=$1
shift
OUT=gpurun_out/tab
mkdir -p $OUT
for i in 1 2 3; do
  GMZ_LIB=$PWD/$ALT timeout -k 10 240 python3 tools/bench_trainer.py --steps 30 "$@" > $OUT/alt_$i.json 2> $OUT/alt_$i.err || { echo "alt failed"; tail -5 $OUT/alt_$i.err; exit 1; }
  timeout -k 10 240 python3 tools/bench_trainer.py --steps 30 "$@" > $OUT/new_$i.json 2> $OUT/new_$i.err || { echo "new failed"; tail -5 $OUT/new_$i.err; exit 1; }
done
python3 - "$OUT" <<'PY'
import glob, json, sys
for kind in ("alt", "new"):
    v = [json.load(open(f))["value"] for f in sorted(glob.glob(sys.argv[1] + "/%s_*.json" % kind))]
    print("%-4s steps/s %s" % (kind, " ".join("%.2f" % x for x in v)))
PY
