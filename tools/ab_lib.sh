#!/bin/bash
# Same-box A/B of two libgmz.so builds on the bench's self-play legs (alternated, ROUNDS rounds):
#   bash tools/ab_lib.sh TAG OLD_LIB [ROUNDS] [bench.py args...]   (OLD_LIB: a path; the new one is the in-tree build)
# -> gpurun_out/TAG/{old,new}_<i>.json and a one-line summary per build (moves/s, tower ms per launch, C1 / C5 lines)
set -o pipefail
TAG=$1; OLD=$2; ROUNDS=${3:-2}; shift 3
ARGS=${@:---no-cpu-baseline --trainer-steps 0 --loop-iters 0 --worker-moves 0 --sublines c1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for i in $(seq 1 $ROUNDS); do
  GMZ_LIB=$OLD timeout -k 10 400 python bench.py $ARGS > $OUT/old_$i.json 2> $OUT/old_$i.err || { echo "old bench failed"; tail -3 $OUT/old_$i.err; exit 1; }
  timeout -k 10 400 python bench.py $ARGS > $OUT/new_$i.json 2> $OUT/new_$i.err || { echo "new bench failed"; tail -3 $OUT/new_$i.err; exit 1; }
done
python3 - "$OUT" <<'PY'
import json, sys, glob
for kind in ("old", "new"):
    for f in sorted(glob.glob(sys.argv[1] + "/%s_*.json" % kind)):
        d = json.load(open(f))
        sub = d.get("sublines", {})
        extra = " ".join("%s %.0f (tower %.3f ms)" % (k, v["value"], v["roofline"]["mean_launch_ms"]) for k, v in sub.items()
                         if isinstance(v, dict) and "value" in v)
        print(kind, "%.0f moves/s" % d["value"], "tower %.3f ms" % d["roofline"]["mean_launch_ms"],
              "single-stream tower %.3f ms" % d.get("single_stream_kernels", {}).get("tower", {}).get("mean_launch_ms", float("nan")), extra)
PY
