#!/bin/bash
# Same-box A/B of the self-play step against another build of libgmz.so (GMZ_LIB), alternated 3x:
# moves/s, tower ms, k_expand_select us.  Usage: bash tools/ab_tree.sh TAG OLD_LIB [bench.py args]
TAG=${1:-ab}
OLD=${2:-$PWD/datou-gomoku-muzero_amd/_alt/libgmz_base.so}
shift; shift
ARGS=${@:---steps 4 --warmup 1}
OUT=$PWD/gpurun_out/abt_$TAG
mkdir -p $OUT
SP="--no-cpu-baseline --trainer-steps 0 --loop-iters 0"
for i in 1 2 3; do
  GMZ_LIB=$OLD timeout -k 10 300 python3 bench.py $ARGS $SP > $OUT/old_$i.json 2> $OUT/old_$i.err || { echo "old failed"; tail -3 $OUT/old_$i.err; exit 1; }
  timeout -k 10 300 python3 bench.py $ARGS $SP > $OUT/new_$i.json 2> $OUT/new_$i.err || { echo "new failed"; tail -3 $OUT/new_$i.err; exit 1; }
done
python3 - "$OUT" <<'PY'
import json, sys, glob
for kind in ("old", "new"):
    v = [json.load(open(f)) for f in sorted(glob.glob(sys.argv[1] + "/%s_*.json" % kind))]
    print(kind, "moves/s", " ".join("%.0f" % d["value"] for d in v), "| tower ms", " ".join("%.4f" % d["roofline"]["mean_launch_ms"] for d in v),
          "| tree us", " ".join("%.1f" % (d["roofline_tree"]["mean_launch_ms"] * 1e3) for d in v),
          "| tree GB/s", " ".join("%.0f" % d["roofline_tree"]["achieved"] for d in v),
          "| single-stream tree us", " ".join("%.1f" % (d.get("single_stream_kernels", {}).get("tree", {}).get("mean_launch_ms", 0) * 1e3) for d in v))
PY
