#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
./tools/gpu_tests_all.sh "prio or c4 or choose or normalize or static" || exit 1
mkdir -p gpurun_out/pr
for mode in pos dense; do
  extra=""; [ $mode = dense ] && extra="--prio-dense"
  timeout -k 10 300 python -u bench.py --workload prio --steps 20 --warmup 5 --no-cpu $extra > gpurun_out/pr/$mode.json 2> gpurun_out/pr/$mode.err || { tail -20 gpurun_out/pr/$mode.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/pr/$mode.json'));print('$mode', d['ms_per_step'], d['phases_ms'], round(d['roofline']['frac'],3), d['value'])"
done
