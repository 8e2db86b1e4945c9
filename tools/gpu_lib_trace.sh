#!/bin/bash
# Per-library kernel averages under rocprofv3 (self-play bench, two streams) + the bench's moves/s.
# Usage: bash tools/gpu_lib_trace.sh TAG "lib1 lib2 ..." [KERNEL_REGEX]  (cur = in-tree libgmz.so)
TAG=$1; LIBS=$2; KRE=${3:-"k_head_gemm|k_head_finish|k_expand_select|k_tower3"}
OUT=$PWD/gpurun_out/lt_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
SP="--steps 4 --warmup 1 --no-cpu-baseline --trainer-steps 0 --loop-iters 0 --single-stream-moves 0"
for r in 1 2; do
  for n in $LIBS; do
    L=$PWD/datou-gomoku-muzero_amd/_alt/libgmz_$n.so
    [ "$n" = cur ] && L=$PWD/datou-gomoku-muzero_amd/libgmz.so
    GMZ_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${n}_$r -o run -- \
      python3 bench.py $SP > $OUT/${n}_$r.json 2> $OUT/${n}_$r.err || { echo "$n failed"; tail -3 $OUT/${n}_$r.err; exit 1; }
    python3 - "$OUT/${n}_$r" "$n" "$KRE" <<'PY'
import csv, glob, json, re, sys
d, n, kre = sys.argv[1], sys.argv[2], sys.argv[3]
st = list(csv.DictReader(open(glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0])))
b = json.load(open(d + ".json"))
parts = ["%s %.1f" % (re.sub(r"<.*", "", r["Name"]).split("::")[-1][:18], float(r["AverageNs"]) / 1e3) for r in st if re.search(kre, r["Name"])]
print("%-8s %.0f moves/s | %s" % (n, b["value"], " | ".join(parts)))
PY
  done
done
