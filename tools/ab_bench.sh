#!/bin/bash
# Same-box A/B of bench.py: the current tree against a git worktree of an older commit built in
# _ab_old/ (git worktree add _ab_old <rev>; make -C _ab_old/datou-gomoku-muzero_amd/csrc).
# Alternates the two 3 times.  Usage: bash tools/ab_bench.sh TAG [bench.py args]
TAG=${1:-ab}
shift
ARGS=${@:---steps 6 --warmup 1}
OUT=$PWD/gpurun_out/ab_$TAG
mkdir -p $OUT
for i in 1 2 3; do
  (cd _ab_old && timeout -k 10 400 python bench.py $ARGS --no-cpu-baseline > $OUT/old_$i.json 2> $OUT/old_$i.err) || { echo "old bench failed"; tail -3 $OUT/old_$i.err; exit 1; }
  timeout -k 10 400 python bench.py $ARGS --no-cpu-baseline > $OUT/new_$i.json 2> $OUT/new_$i.err || { echo "new bench failed"; tail -3 $OUT/new_$i.err; exit 1; }
done
python - "$OUT" <<'PY'
import json, sys, glob
for kind in ("old", "new"):
    v = [json.load(open(f)) for f in sorted(glob.glob(sys.argv[1] + "/%s_*.json" % kind))]
    print(kind, " ".join("%.0f" % d["value"] for d in v), v[0]["unit"], "; tower ms", " ".join("%.3f" % d["roofline"]["mean_launch_ms"] for d in v))
PY
