#!/usr/bin/env python3
"""MFMA utilisation of the C4 GEMM kernels from rocprofv3 --pmc passes
(SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE per dispatch).
On gfx950 SQ_VALU_MFMA_BUSY_CYCLES is summed over all 1024 SIMDs (a
v_mfma_i32_32x32x32_i8 adds its 32 cycles: the C4 dense contraction's 30 M
MFMAs read 9.6e8) and GRBM_GUI_ACTIVE over the 8 XCDs, so the matrix cores'
busy fraction while the kernel runs is MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 x 256
CUs x 4 SIMDs).  Usage: tools/mfma_summary.py DIR...  (each
DIR one rocprofv3 -d output)."""
import collections
import csv
import glob
import os
import sys

CUS, SIMDS, XCDS = 256, 4, 8
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
        frac = busy / (gui / XCDS * CUS * SIMDS) if gui else float("nan")
        print(f"{os.path.basename(d)}  {k}: dispatches {nd}, per dispatch "
              + ", ".join(f"{name} {v / nd:.4g}" for name, v in sorted(c.items()))
              + f"; MFMA busy / (GRBM_GUI_ACTIVE / {XCDS} x {CUS} CUs x {SIMDS} SIMDs) = {frac:.3f}")
