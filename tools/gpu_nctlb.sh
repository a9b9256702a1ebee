#!/bin/bash
# TLB / latency counters of the newcov candidate kernels (both passes)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/nctlb
for path in lds probe; do
i=0
for ctr in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" "TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_REQUEST_sum"; do
  i=$((i+1))
  SYZCOV_NEWCOV_PATH=$path timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "newcov_cand" --output-format csv -d gpurun_out/nctlb/$path$i -o run -- python3 bench.py --workload newcov --steps 5 --warmup 2 --no-cpu --history 8 > gpurun_out/nctlb/$path$i.log 2>&1 || { tail -5 gpurun_out/nctlb/$path$i.log; exit 1; }
done
echo "== $path"
python3 - $path <<'PY'
import csv, glob, collections, sys
agg = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/nctlb/{sys.argv[1]}*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for c, v in sorted(agg.items()):
    print(f"   {c:44s} last5-avg {sum(v[-5:]) / 5:.4g}")
PY
done
