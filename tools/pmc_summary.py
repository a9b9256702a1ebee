#!/usr/bin/env python3
"""Summarise a tools/kprof.sh output dir: kernel durations + PMC counters
per kernel (summed over dispatches, divided by dispatch count)."""
import collections
import csv
import glob
import os
import sys


def short(name):
    name = name.split("(")[0]
    return name.replace("void ", "").replace("syz::", "")[:48]


def main(d):
    st = os.path.join(d, "trace", "run_kernel_stats.csv")
    if os.path.exists(st):
        print("== kernel durations")
        for r in list(csv.DictReader(open(st)))[:14]:
            print(f'  {short(r["Name"]):48s} calls={r["Calls"]:>4s} '
                  f'avg_us={float(r["AverageNs"]) / 1e3:9.1f} pct={float(r["Percentage"]):5.1f}')
    agg = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
    print("== counters (per dispatch)")
    kern = sorted({k for k, _ in agg})
    for k in kern:
        items = [(c, v / len(disp[(k, c)])) for (kk, c), v in agg.items() if kk == k]
        if max(v for _, v in items) < 1e6:
            continue
        print(" ", k)
        for c, v in sorted(items):
            print(f"      {c:24s} {v:14.4g}")


if __name__ == "__main__":
    main(sys.argv[1])
