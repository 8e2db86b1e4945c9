"""Per-kernel breakdown of the last WINDOW_MS of a rocprofv3 kernel trace (steady-state steps only;
the stats CSV also counts warm-up and MIOpen tuning launches).
  python tools/trace_window.py run_kernel_trace.csv [window_ms] [top]"""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
win = float(sys.argv[2]) if len(sys.argv) > 2 else 500.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path))]
end = max(e for _, e, _ in rows)
t0 = end - win * 1e6
agg = defaultdict(lambda: [0, 0])
busy = 0
for s, e, n in rows:
    if s >= t0:
        agg[n][0] += 1
        agg[n][1] += e - s
        busy += e - s
print("window %.1f ms, kernel busy %.1f ms, %d launches" % (win, busy / 1e6, sum(v[0] for v in agg.values())))
for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print("%-100s %6d  avg %8.1f us  tot %7.2f ms %5.1f%%" % (n[:100], c, t / c / 1e3, t / 1e6, 100 * t / busy))
