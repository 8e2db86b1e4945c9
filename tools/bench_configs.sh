#!/bin/bash
# Secondary self-play configurations: C5 (19x19, 800 sims, 16 blocks) and 9x9 AlphaZero
# at 50 sims, 1024 games each.  -> gpurun_out/c5.json, gpurun_out/c9.json
timeout -k 10 500 python bench.py --size 19 --sims 800 --blocks 16 --steps 3 --warmup 1 --no-cpu-baseline \
  > gpurun_out/c5.json 2> gpurun_out/c5.err || { echo "c5 failed"; tail -3 gpurun_out/c5.err; exit 1; }
timeout -k 10 300 python bench.py --size 9 --sims 50 --mode AlphaZero --steps 10 --warmup 2 --no-cpu-baseline \
  > gpurun_out/c9.json 2> gpurun_out/c9.err || { echo "c9 failed"; tail -3 gpurun_out/c9.err; exit 1; }
python - <<'PY'
import json
for f in ("c5", "c9"):
    d = json.load(open("gpurun_out/%s.json" % f)); r = d["roofline"]
    print(f, round(d["value"], 1), d["unit"], "tower ms", round(r["mean_launch_ms"], 3), "frac", round(r["frac"], 3), r["kernel"][:40])
PY
