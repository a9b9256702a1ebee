#!/bin/bash
# kernel stats of the newcov bench, one run per candidate pass (lds / probe)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/nct
for p in ${PATHS:-lds probe}; do
  SYZCOV_NEWCOV_PATH=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nct/$p -o run -- python3 bench.py --workload newcov --steps 20 --warmup 5 --no-cpu "$@" > gpurun_out/nct/$p.log 2>&1 || { tail -20 gpurun_out/nct/$p.log; exit 1; }
  echo "== $p"; tail -1 gpurun_out/nct/$p.log | cut -c1-200
  python3 - gpurun_out/nct/$p <<'PY'
import csv, glob, sys
ks = glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(ks)), key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:10.1f} us  {r['Name'][:90]}")
PY
done
