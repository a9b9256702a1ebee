#!/usr/bin/env python3
"""Per-kernel time over the last N steps of a rocprofv3 --kernel-trace run:
the dispatches from the N-th last dispatch of STEP_KERNEL on (e.g. C5's timed
batches after its history and warm-up), averaged per step.
Usage: tools/trace_last.py <trace_dir> <step kernel substring> <N>"""
import collections
import csv
import glob
import sys

d, step, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
tr = sorted(csv.DictReader(open(kt)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(tr) if step in r["Kernel_Name"]]
if len(idx) < n:
    sys.exit(f"only {len(idx)} dispatches of {step}")
sel = tr[idx[-n]:]
tot = collections.defaultdict(float)
cnt = collections.Counter()
for r in sel:
    tot[r["Kernel_Name"]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    cnt[r["Kernel_Name"]] += 1
span = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e3
print(f"last {n} steps from {step}: {span / n:.1f} us per step (first dispatch to last end), "
      f"kernel sum {sum(tot.values()) / n:.1f} us per step")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"{v / n:9.1f} us/step {cnt[k] / n:5.1f} calls  {k[:110]}")
