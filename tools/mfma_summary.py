#!/usr/bin/env python3
"""MFMA utilisation of the C4 GEMM kernels from rocprofv3 --pmc passes
(SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE per dispatch).
gfx950 counts SQ_VALU_MFMA_BUSY_CYCLES summed over the SIMDs of every CU, so
the busy fraction of the matrix cores is MFMA_BUSY / (GRBM_GUI_ACTIVE x CUs x
4 SIMDs) while the kernel runs.  Usage: tools/mfma_summary.py DIR...  (each
DIR one rocprofv3 -d output)."""
import collections
import csv
import glob
import os
import sys

CUS, SIMDS = 256, 4
for d in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "gemm" not in k:
                continue
            k = k.split("(")[0].replace("void ", "")
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[k].add(r["Dispatch_Id"])
    for k, c in agg.items():
        nd = len(n[k])
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / nd
        gui = c.get("GRBM_GUI_ACTIVE", 0) / nd
        frac = busy / (gui * CUS * SIMDS) if gui else float("nan")
        print(f"{os.path.basename(d)}  {k}: dispatches {nd}, per dispatch "
              + ", ".join(f"{name} {v / nd:.4g}" for name, v in sorted(c.items()))
              + f"; MFMA busy / (GRBM_GUI_ACTIVE x {CUS} CUs x {SIMDS} SIMDs) = {frac:.3f}")
