#!/bin/bash
# kernel trace of the default bench step; per-kernel stats + per-dispatch minimize chunks
set -o pipefail
export TMPDIR=/tmp
tag=${1:-t}; shift
mkdir -p gpurun_out/$tag
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag/trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/$tag/trace.log 2>&1 || { tail -20 gpurun_out/$tag/trace.log; exit 1; }
python3 tools/trace_summary.py gpurun_out/$tag/trace
