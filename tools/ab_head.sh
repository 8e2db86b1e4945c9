# Same-box A/B of the self-play step between the in-tree libgmz.so and an alternative build ($1):
# rocprofv3 kernel stats of a short bench each, then 3 alternating headline runs.  -> gpurun_out/abh/
ALT=$1
OUT=gpurun_out/abh
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
SP="--steps 6 --warmup 1 --no-cpu-baseline --trainer-steps 0 --loop-iters 0 --sublines= --worker-moves 0"
GMZ_LIB=$PWD/$ALT timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_alt -o k -- python3 bench.py $SP > $OUT/prof_alt.json 2> $OUT/prof_alt.err || { echo "alt prof failed"; tail -3 $OUT/prof_alt.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_new -o k -- python3 bench.py $SP > $OUT/prof_new.json 2> $OUT/prof_new.err || { echo "new prof failed"; tail -3 $OUT/prof_new.err; exit 1; }
for i in 1 2 3; do
  GMZ_LIB=$PWD/$ALT timeout -k 10 300 python3 bench.py $SP > $OUT/alt_$i.json 2> $OUT/alt_$i.err || { echo "alt failed"; tail -3 $OUT/alt_$i.err; exit 1; }
  timeout -k 10 300 python3 bench.py $SP > $OUT/new_$i.json 2> $OUT/new_$i.err || { echo "new failed"; tail -3 $OUT/new_$i.err; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, json, sys
root = sys.argv[1]
for kind in ("alt", "new"):
    v = [json.load(open(f)) for f in sorted(glob.glob(root + "/%s_*.json" % kind))]
    print("%-4s moves/s %s" % (kind, " ".join("%.0f" % d["value"] for d in v)))
    for f in glob.glob(root + "/prof_%s/**/*kernel_stats.csv" % kind, recursive=True):
        for r in csv.DictReader(open(f)):
            if any(k in r["Name"] for k in ("k_head_gemm", "k_tower3", "k_expand_select", "k_head_finish")):
                print("   %-60s calls %6s avg %8.1f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
