#!/bin/bash
# key-mode tuning: canon digit width, minimize pass-1 variants, then a kernel trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/b3
run() {  # tag env...
    local tag=$1; shift
    env "$@" timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/b3/$tag.json 2> gpurun_out/b3/$tag.err || { tail -20 gpurun_out/b3/$tag.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/b3/$tag.json'));print('$tag', round(d['ms_per_step'],3), d['phases_ms'])"
}
run hb9 SYZCOV_CANON_HB=9
run mr1 SYZCOV_MR_CFG=1,0
run mr12 SYZCOV_MR_CFG=12,0
run mr13 SYZCOV_MR_CFG=13,0
run mr14 SYZCOV_MR_CFG=14,0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b3/trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/b3/trace.log 2>&1 || { tail -20 gpurun_out/b3/trace.log; exit 1; }
find gpurun_out/b3/trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/b3/kstats.csv
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/b3/kstats.csv')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:25]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:10.1f} us  {r['Name'][:110]}")
PY
