#!/bin/bash
# Round-2 evidence on the GPU box: kernel-trace stats of the default self-play bench, PMC HBM traffic
# (separate FETCH_SIZE / WRITE_SIZE passes) of the f16 dynamics tower and the fused tree kernel, a G
# sweep of the self-play step (tree-kernel HBM fraction vs games per GPU), C5 / C9 lines.
OUT=gpurun_out/r2prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
SP="--no-cpu-baseline --trainer-steps 0 --loop-iters 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --steps 3 --warmup 1 $SP > $OUT/bench_under_trace.json 2> $OUT/trace.err || { echo "trace failed"; tail -5 $OUT/trace.err; exit 1; }
echo "trace done"
for CTR in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $CTR --kernel-include-regex "k_tower3|k_expand_select" --output-format csv -d $OUT/pmc_$CTR -o pmc -- \
    python3 bench.py --steps 1 --warmup 0 $SP > $OUT/pmc_$CTR.json 2> $OUT/pmc_$CTR.err || { echo "pmc $CTR failed"; tail -3 $OUT/pmc_$CTR.err; exit 1; }
  echo "pmc $CTR done"
done
python3 tools/pmc_summary.py $OUT "k_tower3<15, true" fp16 > $OUT/pmc_tower.txt
python3 tools/pmc_summary.py $OUT "k_expand_select" fp16 > $OUT/pmc_expand_select.txt
cat $OUT/pmc_tower.txt $OUT/pmc_expand_select.txt
for G in 2048 4096; do
  timeout -k 10 400 python3 bench.py --games $G --steps 4 --warmup 1 $SP > $OUT/bench_G$G.json 2> $OUT/bench_G$G.err || { echo "G=$G failed"; tail -5 $OUT/bench_G$G.err; exit 1; }
  echo "G=$G done"
done
timeout -k 10 500 python3 bench.py --size 19 --sims 800 --blocks 16 --steps 3 --warmup 1 $SP > $OUT/c5.json 2> $OUT/c5.err || { echo "c5 failed"; tail -3 $OUT/c5.err; exit 1; }
timeout -k 10 300 python3 bench.py --size 9 --sims 50 --mode AlphaZero --steps 10 --warmup 2 $SP > $OUT/c9.json 2> $OUT/c9.err || { echo "c9 failed"; tail -3 $OUT/c9.err; exit 1; }
python3 - <<'PY'
import json
for f in ("bench_under_trace", "bench_G2048", "bench_G4096", "c5", "c9"):
    d = json.load(open("gpurun_out/r2prof/%s.json" % f)); r = d["roofline"]; t = d.get("roofline_tree", {})
    print("%-18s %9.1f moves/s  tower %.3f ms frac %.3f | tree %.1f us %.0f GB/s frac %.3f" % (
        f, d["value"], r["mean_launch_ms"], r["frac"], t.get("mean_launch_ms", 0) * 1e3, t.get("achieved", 0), t.get("frac", 0)))
PY
