#!/bin/bash
# Round-end evidence (run on the GPU box from the repo root): kernel-trace stats, PMC HBM traffic of the
# dynamics tower (separate FETCH_SIZE / WRITE_SIZE passes), full default bench.  -> gpurun_out/round_<TAG>/
TAG=${1:-r01}
OUT=gpurun_out/round_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_under_trace.json 2> $OUT/trace.err || { echo "trace failed"; exit 1; }
for CTR in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $CTR --kernel-include-regex "k_tower" --output-format csv -d $OUT/pmc_$CTR -o pmc -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc_$CTR.json 2> $OUT/pmc_$CTR.err || { echo "pmc $CTR failed"; exit 1; }
done
python3 tools/pmc_summary.py $OUT "k_tower3<15, true" > $OUT/pmc_summary.txt && cat $OUT/pmc_summary.txt
cp $OUT/pmc_tower.json profiles/pmc_tower_latest.json 2>/dev/null
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail $OUT/bench_default.err; exit 1; }
cat $OUT/bench_default.json
