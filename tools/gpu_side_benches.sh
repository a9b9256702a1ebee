#!/bin/bash
# C4 / C5 bench lines with CPU baselines (not under the profiler)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/side; mkdir -p $o
timeout -k 10 300 python -u bench.py --workload newcov --steps 20 --warmup 5 > $o/newcov.json 2> $o/newcov.err || { tail -5 $o/newcov.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload prio --steps 20 --warmup 5 > $o/prio.json 2> $o/prio.err || { tail -5 $o/prio.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload prio --prio-dense --steps 20 --warmup 5 --no-cpu > $o/prio_dense.json 2> $o/prio_dense.err || { tail -5 $o/prio_dense.err; exit 1; }
for f in newcov prio prio_dense; do python3 -c "import json; d=json.load(open('$o/$f.json')); print('$f', round(d['ms_per_step'],4), d['value'], d['phases_ms'], round(d['roofline']['frac'],4), d.get('cpu_baseline',{}).get('value'))"; done
