#!/bin/bash
# The one GPU-box runner (replaces the round-1/2 one-off gpu_*.sh / round*_profile.sh / pmc_round*.sh
# scripts; their commands are the subcommands below).  Run on the box through gpurun, e.g.
#   gpurun --timeout 1200 -- bash tools/gpu.sh tests r03a 'large or c4'
#   gpurun --timeout 900  -- bash tools/gpu.sh bench r03a [bench.py args...]
#   gpurun --timeout 900  -- bash tools/gpu.sh trace r03a        # rocprofv3 kernel stats of the default step
#   gpurun --timeout 900  -- bash tools/gpu.sh pmc r03a          # PMC passes: tower + tree kernel
# Every GPU step runs under its own timeout and the steps chain with &&: after a failure, nothing
# further touches the GPU.  Output: gpurun_out/<tag>/.
set -o pipefail
CMD=$1
TAG=${2:-x}
shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
SP="--no-cpu-baseline --trainer-steps 0 --loop-iters 0 --sublines= --worker-moves 0"

case $CMD in
  tests)  # GPU test suite (optionally -k EXPR)
    K=()
    [ -n "$1" ] && K=(-k "$1")
    # a heartbeat under gpurun_out/ while pytest runs: single tests (e.g. the fp32 agreement search) can run
    # for minutes without a result line; pytest's own --timeout and the outer timeout bound any hang
    ( while sleep 60; do date >> $OUT/heartbeat; done ) &
    HB=$!
    timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > $OUT/pytest.log 2>&1
    rc=$?
    kill $HB
    echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"
    grep -E "FAILED|^E  |differing searches" $OUT/pytest.log | head -30
    exit $rc ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
    rc=$?; tail -2 $OUT/smoke.log; exit $rc ;;
  bench)  # bench.py with the given arguments (default: the driver's default line)
    timeout -k 10 800 python -u bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
    rc=$?
    tail -3 $OUT/bench.err
    python3 tools/summarize_bench.py $OUT/bench.json
    exit $rc ;;
  trace)  # rocprofv3 kernel-trace stats of the default self-play step (+ the bench line under the tracer)
    cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
      python3 bench.py --steps 3 --warmup 1 $SP "$@" > $OUT/bench_under_trace.json 2> $OUT/trace.err || { echo "trace failed"; tail -5 $OUT/trace.err; exit 1; }
    find $OUT/trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
    python3 - "$OUT" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1] + "/kernel_stats.csv")))
for r in rows[:8]:
    print("%-60s %6s calls avg %9.1f us %5.1f%%" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
PY
    ;;
  pmc)  # one counter group per rocprofv3 run (MI355X_MICROARCH.md: separate passes) on the self-play step
    cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
    for CTR in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS"; do
      NAME=$(echo $CTR | tr ' ' '_' | cut -c1-40)
      timeout -s KILL 240 rocprofv3 --pmc $CTR --kernel-include-regex "k_tower3|k_expand_select" --output-format csv -d $OUT/$NAME -o pmc -- \
        python3 bench.py --steps 1 --warmup 0 --single-stream-moves 0 $SP "$@" > $OUT/$NAME.json 2> $OUT/$NAME.err || { echo "pmc $CTR failed"; tail -3 $OUT/$NAME.err; exit 1; }
      echo "pass $NAME done"
    done
    for K in "k_tower3<15, true" "k_expand_select"; do
      echo "== $K"; python3 tools/pmc_summary.py $OUT "$K" fp16 2
    done > $OUT/summary.txt
    cat $OUT/summary.txt ;;
  layout)  # tree-kernel A/B: dense vs compact child lists, hint on/off, per game count (one stream)
    for G in ${1:-1024 8192}; do
      for L in dense lists; do
        for H in on off; do
          timeout -k 10 300 python -u bench.py --games $G --streams 1 --steps 3 --warmup 1 --layout $L --hint $H \
            --single-stream-moves 0 $SP > $OUT/G${G}_${L}_${H}.json 2> $OUT/G${G}_${L}_${H}.err || { echo "G=$G $L $H failed"; tail -5 $OUT/G${G}_${L}_${H}.err; exit 1; }
          python3 -c "import json,sys; d=json.load(open(sys.argv[1])); t=d['roofline_tree']; print('G=%5d %-5s hint=%-3s moves/s %8.0f  tree %7.1f us  %6.0f GB/s  frac %.3f  levels %.1f' % (d['config']['games_per_gpu'], t['layout'], sys.argv[2], d['value'], t['mean_launch_ms']*1e3, t['achieved'], t['frac'], t['mean_select_levels']))" $OUT/G${G}_${L}_${H}.json $H | tee -a $OUT/summary.txt
        done
      done
    done ;;
  tree_curve)  # the default engine per game count: headline (two streams) + the tree kernel alone (one engine)
    for G in ${1:-1024 2048 4096 8192}; do
      timeout -k 10 400 python -u bench.py --games $G --steps 3 --warmup 1 $SP > $OUT/G$G.json 2> $OUT/G$G.err || { echo "G=$G failed"; tail -5 $OUT/G$G.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); t=d['roofline_tree']; s=d['single_stream_kernels']; print('G=%5d moves/s %8.0f | tree alone (%s, hint %s) %7.1f us %6.0f GB/s frac %.3f | in the step %6.1f us frac %.3f | tower alone frac %.3f' % (d['config']['games_per_gpu'], d['value'], t['layout'], t['descent_hint'], s['tree']['mean_launch_ms']*1e3, s['tree']['achieved_gbs'], s['tree']['frac'], t['mean_launch_ms']*1e3, t['frac'], s['tower']['frac']))" $OUT/G$G.json | tee -a $OUT/summary.txt
    done ;;
  layout_libs)  # k_expand_select of the list layout per occupancy build (GMZ_LIB) at each G, one stream
    for G in ${1:-4096 8192}; do
      for LIB in libgmz.so ${LIBS:-_alt/libgmz_cl6.so _alt/libgmz_cl8.so}; do
        for H in off on; do
          N=G${G}_$(basename $LIB .so)_$H
          GMZ_LIB=$PWD/datou-gomoku-muzero_amd/$LIB timeout -k 10 300 python -u bench.py --games $G --streams 1 --steps 3 --warmup 1 \
            --layout lists --hint $H --single-stream-moves 0 $SP > $OUT/$N.json 2> $OUT/$N.err || { echo "$N failed"; tail -5 $OUT/$N.err; exit 1; }
          python3 -c "import json,sys; d=json.load(open(sys.argv[1])); t=d['roofline_tree']; print('%-32s moves/s %8.0f  tree %7.1f us  %6.0f GB/s  frac %.3f' % (sys.argv[2], d['value'], t['mean_launch_ms']*1e3, t['achieved'], t['frac']))" $OUT/$N.json $N | tee -a $OUT/summary.txt
        done
      done
    done ;;
  *)
    echo "usage: tools/gpu.sh tests|smoke|bench|trace|pmc TAG [args]"; exit 2 ;;
esac
