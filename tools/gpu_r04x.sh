#!/bin/bash
# Round-4 GPU call X: cover_dedup with per-class occupancy bounds: parity,
# the bench.py dedup line, kernel trace of it.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04x; mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dedup.py > $o/pytest.log 2>&1
rc=$?; tail -3 $o/pytest.log; [ $rc -ne 0 ] && exit 1
timeout -k 10 300 python -u bench.py --workload dedup --steps 20 --warmup 3 > $o/bench_dedup.json 2> $o/bench_dedup.err || { tail -20 $o/bench_dedup.err; exit 1; }
python3 -c "import json; d=json.load(open('$o/bench_dedup.json')); print(round(d['ms_per_step'],4), d['phases_ms'], round(d['roofline']['frac'],4), d['value'], d['cpu_baseline']['value'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$o/prof -o dd -- python3 $GRAFT_REPO_ROOT/bench.py --workload dedup --steps 10 --warmup 2 --no-cpu > $GRAFT_REPO_ROOT/$o/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && f=$(find $o/prof -name "*kernel_stats.csv" | head -1) && head -6 $f | cut -c1-150
