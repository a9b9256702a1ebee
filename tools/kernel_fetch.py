#!/usr/bin/env python3
"""Per-kernel HBM read bytes per step from one rocprofv3 --pmc FETCH_SIZE
pass (x2: gfx950 tallies 128-B requests at 64 B, MI355X_MICROARCH.md 'HBM').
Steps are counted as the dispatches of STEP_KERNEL.
Usage: tools/kernel_fetch.py <dir> [step_kernel]"""
import collections
import csv
import glob
import os
import sys


def main(d, step_kernel="bin_kernel"):
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != "FETCH_SIZE":
                continue
            tot[r["Kernel_Name"]] += float(r["Counter_Value"])
            disp[r["Kernel_Name"]].add(r["Dispatch_Id"])
    steps = max([len(v) for k, v in disp.items() if step_kernel in k] or [1])
    rows = sorted(((2 * v * 1024 / steps, k) for k, v in tot.items()), reverse=True)
    print(f"steps {steps}; read bytes per step: total {sum(b for b, _ in rows) / 1e9:.3f} GB")
    for b, k in rows[:12]:
        print(f"{b / 1e9:9.4f} GB  {len(disp[k]) / steps:6.1f}/step  {k[:90]}")


if __name__ == "__main__":
    main(*sys.argv[1:])
