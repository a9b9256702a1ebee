#!/bin/bash
# kernel trace + stats of a short default bench run -> gpurun_out/tr_<tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-x}; out=gpurun_out/tr_$tag; mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log
f=$(find $out -name 'run_kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:22]:
    print(f'{r["Name"].split("(")[0][:70]:70s} {int(r["Calls"]):5d} {float(r["AverageNs"])/1e3:9.1f} us {float(r["Percentage"]):5.1f}%')
PY
