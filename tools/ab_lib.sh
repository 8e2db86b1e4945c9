OUT=gpurun_out/ab_lib
mkdir -p $OUT
for i in 1 2 3; do
  GMZ_LIB=$PWD/datou-gomoku-muzero_amd/_alt/libgmz_oldnet.so timeout -k 10 300 python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline > $OUT/old_$i.json 2> $OUT/old_$i.err || { echo old failed; tail -3 $OUT/old_$i.err; exit 1; }
  timeout -k 10 300 python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline > $OUT/new_$i.json 2> $OUT/new_$i.err || { echo new failed; tail -3 $OUT/new_$i.err; exit 1; }
done
python3 - "$OUT" <<'PY'
import json, sys, glob
for kind in ("old", "new"):
    v = [json.load(open(f)) for f in sorted(glob.glob(sys.argv[1] + "/%s_*.json" % kind))]
    print(kind, " ".join("%.0f" % d["value"] for d in v), v[0]["unit"], "; tower ms", " ".join("%.4f" % d["roofline"]["mean_launch_ms"] for d in v))
PY
