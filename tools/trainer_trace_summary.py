"""Trainer step kernels from a rocprofv3 kernel trace of tools/bench_trainer.py (tools/trainer_profile.sh):
the steady-state window's per-step launch count and the dominant HIP convolution's mean duration INSIDE the
graph-replayed step, as MFMA roofline fractions -> a JSON summary that bench.py's trainer leg reports as
``roofline_in_step`` (builder-measured, labelled with its source).
  python tools/trainer_trace_summary.py TRACE.csv BENCH.json OUT.json [window_ms]"""
import csv
import json
import sys
from collections import defaultdict

trace, bench_json, out = sys.argv[1], sys.argv[2], sys.argv[3]
win = float(sys.argv[4]) if len(sys.argv) > 4 else 400.0
b = json.load(open(bench_json))
step_ms = b["ms_per_step"]
rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(trace))]
end = max(e for _, e, _ in rows)
t0 = end - win * 1e6
agg = defaultdict(lambda: [0, 0])
n = 0
for s, e, k in rows:
    if s >= t0:
        agg[k][0] += 1
        agg[k][1] += e - s
        n += 1
steps = win / step_ms
B, H = 360, 15
flop = 2.0 * B * H * H * 128 * 128 * 9  # one 128->128 3x3 conv over the batch (forward or input gradient)
peak = 2500.0
res = {"source": "rocprofv3 --kernel-trace of tools/bench_trainer.py --per (B=360, 15x15, 8 blocks, graph-replayed "
                 "step), last %.0f ms = %.1f steps at %.2f ms per step under the tracer" % (win, steps, step_ms),
       "launches_per_step": n / steps, "kernels": {}}
for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
    res["kernels"][k[:90]] = {"launches_per_step": c / steps, "mean_us": t / c / 1e3, "ms_per_step": t / 1e6 / steps}
conv = [(k, v) for k, v in agg.items() if "k_conv3<" in k]
if conv:
    c = sum(v[0] for _, v in conv)
    t = sum(v[1] for _, v in conv)
    us = t / c / 1e3
    ach = flop / (us * 1e-6) / 1e12
    res["dominant"] = {"kernel": "gmz_conv3x3 (k_conv3, 128->128 3x3 conv, forward and input gradient, f16 NHWC, B=360)",
                       "mean_us_in_step": us, "achieved": ach, "peak": peak, "unit": "TFLOP/s", "frac": ach / peak,
                       "launches_per_step": c / steps, "ms_per_step": t / 1e6 / steps}
wg = [(k, v) for k, v in agg.items() if "k_conv3_wgrad<" in k]
if wg:
    # one weight gradient per residual-conv USE: 16 convs x (representation + 5 unroll steps) = 96 per step; with
    # trainer.DEFER_WGRAD one launch covers several uses (segments), so the rate is per use, not per launch
    uses = 2 * 8 * (1 + 5)
    c = sum(v[0] for _, v in wg)
    t = sum(v[1] for _, v in wg)
    red = sum(v[1] for k, v in agg.items() if "k_conv3_wgrad_reduce" in k)
    ms = t / 1e6 / steps
    ach = uses * flop / (ms * 1e-3) / 1e12
    res["weight_gradient"] = {"kernel": "gmz_conv3x3_wgrad (k_conv3_wgrad partials; k_conv3_wgrad_reduce separate)",
                              "uses_per_step": uses, "launches_per_step": c / steps, "ms_per_step": ms,
                              "reduce_ms_per_step": red / 1e6 / steps, "achieved": ach, "unit": "TFLOP/s",
                              "frac": ach / peak}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1)[:2500])
