#!/bin/bash
# C4 (priorities) and C5 (new coverage) bench lines + kernel stats -> gpurun_out/other
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/other; mkdir -p $out
timeout -k 10 300 python3 bench.py --workload prio > $out/prio.json 2> $out/prio.err || { tail -20 $out/prio.err; exit 1; }
cat $out/prio.json
timeout -k 10 300 python3 bench.py --workload newcov > $out/newcov.json 2> $out/newcov.err || { tail -20 $out/newcov.err; exit 1; }
cat $out/newcov.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prio_trace -o run -- python3 bench.py --workload prio --steps 3 --warmup 1 --no-cpu > $out/prio_trace.log 2>&1 || { tail -5 $out/prio_trace.log; exit 1; }
echo done
