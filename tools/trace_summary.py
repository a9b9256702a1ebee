#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats directory: top kernels by
total time, and the last step's pass-1 / covered-update dispatches."""
import csv
import glob
import sys

d = sys.argv[1]
ks = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(ks)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:22]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):6d} "
          f"{float(r['AverageNs'])/1e3:10.1f} us  {r['Name'][:100]}")
kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
tr = list(csv.DictReader(open(kt)))
sel = [r for r in tr if any(k in r["Kernel_Name"] for k in
                            ("pass1_kernel", "cover_records", "first_to_bits"))]
print("last step, minimize chunks:")
for r in sel[-17:]:
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f"  {us:8.1f} us  grid {r['Grid_Size_X']:>8}  {r['Kernel_Name'][:50]}")
