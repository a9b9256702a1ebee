#!/bin/bash
# PMC passes over the newcov LDS candidate kernel
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ncp2
i=0
for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_WAVES SQ_LDS_BANK_CONFLICT" "FETCH_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  SYZCOV_NEWCOV_PATH=lds timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "newcov_cand_lds" --output-format csv -d gpurun_out/ncp2/p$i -o run -- python3 bench.py --workload newcov --steps 5 --warmup 2 --no-cpu --history 8 > gpurun_out/ncp2/p$i.log 2>&1 || { tail -5 gpurun_out/ncp2/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/ncp2/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for c, v in sorted(agg.items()):
    print(f"   {c:26s} n={len(v):4d} last5-avg {sum(v[-5:]) / 5:.4g}")
PY
