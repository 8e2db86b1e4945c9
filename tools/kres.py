"""Kernel resource table from hipcc -Rpass-analysis=kernel-resource-usage remarks (stdin):
name VGPRs AGPRs spills occupancy LDS, one line per kernel, filtered by an optional regex.
  hipcc ... -c gmz_tree.hip -Rpass-analysis=kernel-resource-usage 2>&1 | python3 tools/kres.py k_expand_select"""
import re
import subprocess
import sys

pat = re.compile(sys.argv[1]) if len(sys.argv) > 1 else None
rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    if cur is None:
        continue
    for key, rx in (("vgpr", r"\bVGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("vspill", r"VGPRs Spill: (\d+)"),
                    ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
        m = re.search(rx, line)
        if m:
            cur[key] = int(m.group(1))
names = [r["name"] for r in rows]
try:
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
except Exception:
    dem = names
for r, d in zip(rows, dem):
    if pat and not pat.search(d):
        continue
    print("%-80s vgpr %3s agpr %3s spill %3s occ %s lds %s" % (d[:80], r.get("vgpr"), r.get("agpr"), r.get("vspill"),
                                                              r.get("occ"), r.get("lds")))
