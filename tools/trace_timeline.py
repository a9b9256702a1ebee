#!/usr/bin/env python3
"""The last step's dispatch timeline of a rocprofv3 --kernel-trace run: every
dispatch from the last occurrence of MARK (a kernel that starts the step) on,
with its start offset, duration and the idle gap before it, then the idle
total (host read-backs and launch gaps) and per-kernel sums.
Usage: tools/trace_timeline.py <trace_dir> <mark kernel substring> [max rows]"""
import collections
import csv
import glob
import sys

d, mark = sys.argv[1], sys.argv[2]
rows_max = int(sys.argv[3]) if len(sys.argv) > 3 else 400
kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
tr = sorted(csv.DictReader(open(kt)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(tr) if mark in r["Kernel_Name"]]
if not idx:
    sys.exit(f"no dispatch of {mark}")
sel = tr[idx[-1]:]
t0 = int(sel[0]["Start_Timestamp"])
prev_end = t0
idle = 0.0
tot = collections.defaultdict(float)
cnt = collections.Counter()
for k, r in enumerate(sel):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = max(0, s - prev_end) / 1e3
    idle += gap
    prev_end = max(prev_end, e)
    name = r["Kernel_Name"]
    tot[name] += (e - s) / 1e3
    cnt[name] += 1
    if k < rows_max:
        print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  gap {gap:7.1f}  "
              f"grid {r['Grid_Size_X']:>9}  {name[:70]}")
print(f"span {(prev_end - t0) / 1e3:.1f} us, idle {idle:.1f} us, {len(sel)} dispatches")
for n, v in sorted(tot.items(), key=lambda kv: -kv[1])[:25]:
    print(f"{v:9.1f} us {cnt[n]:4d} calls  {n[:100]}")
