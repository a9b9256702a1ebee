#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
./tools/gpu_tests_all.sh "prio or c4" || exit 1
mkdir -p gpurun_out/pr
timeout -k 10 300 python -u bench.py --workload prio --steps 20 --warmup 5 --no-cpu > gpurun_out/pr/pos.json 2> gpurun_out/pr/pos.err || { tail -20 gpurun_out/pr/pos.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/pr/pos.json'));print('pos', d['ms_per_step'], d['phases_ms'], round(d['roofline']['frac'],3), d['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pr/trace -o run -- python3 bench.py --workload prio --steps 3 --warmup 1 --no-cpu > gpurun_out/pr/trace.log 2>&1 || { tail -20 gpurun_out/pr/trace.log; exit 1; }
python3 tools/trace_summary.py gpurun_out/pr/trace | head -14
