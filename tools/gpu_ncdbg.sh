#!/bin/bash
# timing probes of the LDS candidate pass (SYZCOV_NC_DBG bits; results invalid)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ncd
for d in ${DBGS:-0 1 2 6}; do
  for it in ${ITEMS:-1024}; do
  SYZCOV_NC_DBG=$d SYZCOV_NEWCOV_ITEMS=$it SYZCOV_NEWCOV_PATH=lds timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ncd/d${d}_$it -o run -- python3 bench.py --workload newcov --steps 10 --warmup 2 --no-cpu > gpurun_out/ncd/d${d}_$it.log 2>&1 || echo "bench d=$d exited $?"
  python3 - gpurun_out/ncd/d${d}_$it $d $it <<'PY'
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)
if not f: sys.exit(0)
tr = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r["Start_Timestamp"]))
v = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in tr if "newcov_cand_lds" in r["Kernel_Name"]]
print(f"dbg={sys.argv[2]} items={sys.argv[3]} cand_lds last10 avg {sum(v[-10:]) / 10:.1f} us (n={len(v)})")
PY
  done
done
