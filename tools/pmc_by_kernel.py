"""Per-kernel means of rocprofv3 --pmc counter passes (one subdirectory per pass under ROOT), with the derived
ratios used in DESIGN.md: MFMA busy fraction (SQ_VALU_MFMA_BUSY_CYCLES over GRBM_GUI_ACTIVE/8 x 1,024 SIMDs),
effective clock (GRBM_GUI_ACTIVE / 8 / duration), LDS bank-conflict share, wait shares of wave cycles.
  python tools/pmc_by_kernel.py ROOT [name-substring ...]"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
keep = sys.argv[2:]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in glob.glob(os.path.join(root, "*", "pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if keep and not any(s in k for s in keep):
            continue
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
for k in sorted(agg):
    m = {c: sum(v) / len(v) for c, v in agg[k].items()}
    d = sum(dur[k]) / len(dur[k])
    print("== %s  (%d dispatch-counter samples, mean %.4f ms)" % (k[:150], len(dur[k]), d * 1e3))
    for c in sorted(m):
        print("   %-30s %.6g" % (c, m[c]))
    if "GRBM_GUI_ACTIVE" in m:
        clk = m["GRBM_GUI_ACTIVE"] / 8 / d
        print("   effective clock %.3f GHz" % (clk / 1e9))
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            print("   MFMA busy fraction %.3f" % (m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8) / 1024))
    if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
        print("   LDS bank-conflict share %.3f" % (m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]))
    if "SQ_WAVE_CYCLES" in m:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if c in m:
                print("   %s / WAVE_CYCLES %.3f" % (c, m[c] / m["SQ_WAVE_CYCLES"]))
