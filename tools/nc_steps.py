#!/usr/bin/env python3
"""Per-kernel averages of the newcov bench's timed steps (the last 20
dispatches of each kernel) from gpu_nctrace.sh's kernel traces."""
import csv
import glob
import os
import sys

for d in sorted(glob.glob(os.path.join(sys.argv[1], "*/"))):
    tr = list(csv.DictReader(open(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0])))
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    ks = {}
    for r in tr:
        n = r["Kernel_Name"].split("(")[0]
        if n.startswith("syz::") and any(x in n for x in ("newcov", "grp_", "hash_clear")):
            ks.setdefault(n[5:], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("==", d, f"sum {sum(sum(v[-20:]) / 20 for v in ks.values()):.1f} us")
    for n, v in ks.items():
        print(f"  {n:26s} last20avg {sum(v[-20:]) / 20:8.1f} us")
