"""Summarise rocprofv3 PMC csv dirs for the dynamics tower (k_tower3<15, true>)."""
import collections, csv, glob, json, os, sys

root = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "k_tower3<15, true"
precision = sys.argv[3] if len(sys.argv) > 3 else "fp16"  # the towers' operand type in the profiled run
streams = int(sys.argv[4]) if len(sys.argv) > 4 else 1  # engine streams of the profiled bench (rows per launch = G / streams)
games = int(sys.argv[5]) if len(sys.argv) > 5 else 1024  # games per GPU of the profiled bench
agg = collections.defaultdict(list)
dur = []
for f in glob.glob(os.path.join(root, "*", "pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if kern not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
m = {k: sum(v) / len(v) for k, v in agg.items()}
for k in sorted(m):
    print("%-28s %.6g" % (k, m[k]))
d = sum(dur) / max(1, len(dur))
print("mean dispatch duration (profiled) %.4g ms" % (d * 1e3))
if "GRBM_GUI_ACTIVE" in m:
    print("effective clock %.3f GHz" % (m["GRBM_GUI_ACTIVE"] / 8 / d / 1e9))
if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
    # MFMA busy cycles summed over SIMDs; 256 CUs x 4 SIMDs
    print("MFMA busy fraction %.3f" % (m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8) / 1024))
if "SQ_WAVE_CYCLES" in m:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if k in m:
            print("%s / WAVE_CYCLES = %.3f" % (k, m[k] / m["SQ_WAVE_CYCLES"]))
if "FETCH_SIZE" in m:
    print("FETCH_SIZE %.4g MB (x2 gfx950 wide-load correction: %.4g MB)" % (m["FETCH_SIZE"] / 1024, 2 * m["FETCH_SIZE"] / 1024))
if "WRITE_SIZE" in m:
    print("WRITE_SIZE %.4g MB" % (m["WRITE_SIZE"] / 1024))
if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
    print("HBM bytes per launch %.4g MB -> %.1f GB/s over the profiled mean duration"
          % ((2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) / 1024, (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024 / d / 1e9))
    hbm = (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024
    json.dump({"hbm_bytes_per_launch": hbm, "fetch_kb": m["FETCH_SIZE"], "write_kb": m["WRITE_SIZE"],
               "precision": precision, "kernel": kern, "streams": streams, "games": games, "launches_averaged": len(dur),
               "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md HBM section (gfx950 counts 128-B wide reads at 64 B)"},
              open(os.path.join(root, "pmc_tower.json" if "k_tower3" in kern else "pmc_tree.json"), "w"))
