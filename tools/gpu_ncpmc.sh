#!/bin/bash
# PMC counters of the newcov candidate kernels (one counter pass per run)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ncp
i=0
for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU" "FETCH_SIZE" "SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  SYZCOV_NEWCOV_PATH=${NCPATH:-lds} timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "newcov_cand|newcov_split" --output-format csv -d gpurun_out/ncp/p$i -o run -- python3 bench.py --workload newcov --steps 5 --warmup 2 --no-cpu > gpurun_out/ncp/p$i.log 2>&1 || { tail -5 gpurun_out/ncp/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/ncp/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        n = len(v)
        print(f"   {c:26s} n={n:4d} last-avg {sum(v[-max(1, n // 4):]) / max(1, n // 4):.4g}")
PY
