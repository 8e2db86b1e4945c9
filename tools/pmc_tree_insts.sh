#!/bin/bash
# Instruction mix of the tree kernel (k_expand_select) at G games, one stream: per launch and per tree level.
G=${1:-8192}
TAG=${2:-x}
shift 2
OUT=gpurun_out/pmc_tree_insts_${G}_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
SP="--games $G --streams 1 --steps 1 --warmup 0 --no-cpu-baseline --trainer-steps 0 --loop-iters 0 --single-stream-moves 0 --sublines= --worker-moves 0 $*"
i=0
for CTR in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SMEM SQ_WAVE_CYCLES" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $CTR --kernel-include-regex "k_expand_select" --output-format csv -d $OUT/p$i -o pmc -- \
    python3 bench.py $SP > $OUT/p$i.json 2> $OUT/p$i.err || { echo "pmc pass $i failed"; tail -3 $OUT/p$i.err; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, json, sys, collections
root = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(root + "/*/pmc_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in agg.items()}
d = json.load(open(root + "/p1.json"))["roofline_tree"]
waves = m.get("SQ_WAVES", 1)
lv = d["mean_select_levels"] + d["mean_backup_levels"]
for k in sorted(m):
    print("%-26s %14.4g per launch %10.1f per wave" % (k, m[k], m[k] / waves))
print("tree levels per game-wave (select + backup) %.2f; VALU per game-wave %.0f" % (lv, m.get("SQ_INSTS_VALU", 0) / waves))
print("algorithmic bytes per launch (bench model) %.4g MB; FETCH_SIZE x2 + WRITE_SIZE = %.4g MB"
      % (d["bytes_per_launch"] / 1e6, (2 * m.get("FETCH_SIZE", 0) + m.get("WRITE_SIZE", 0)) * 1024 / 1e6))
if "GRBM_GUI_ACTIVE" in m and "SQ_ACTIVE_INST_VALU" in m:
    # SQ_ACTIVE_INST_VALU: cycles a VALU instruction issued, summed over waves (per SIMD-ish); vs the SIMD cycles
    print("VALU issue cycles / (SIMD cycles = GRBM_GUI_ACTIVE/8 x 1024 SIMDs): %.3f"
          % (m["SQ_ACTIVE_INST_VALU"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024)))
PY
