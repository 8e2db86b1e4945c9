#!/bin/bash
# tools/dual_stream_probe.py sweep (one box, alternated): parts x tower grid cap
OUT=gpurun_out/dual3
mkdir -p $OUT
run() { timeout -k 10 200 python tools/dual_stream_probe.py "$@" >> $OUT/r.jsonl 2>>$OUT/err.log; }
for i in 1 2; do
  run --parts 1 || exit 1
  for cap in 160 192 224; do run --parts 2 --max-grid $cap || exit 1; done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/dual3/r.jsonl"):
    r = json.loads(l); d[(r["parts"], r["max_grid"])].append(r["moves_per_s"])
for k, v in sorted(d.items(), key=lambda x: (x[0][0], x[0][1] or 0)):
    print(k, " ".join("%.0f" % x for x in v))
PY
