#!/bin/bash
# kernel trace + stats of one bench command: tools/gpu_trace.sh OUTDIR bench-args...
set -o pipefail
export TMPDIR=/tmp
o=$1; shift; mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace -o run -- python3 bench.py --no-cpu --no-c3 --no-dropin "$@" > $o/trace.log 2>&1 || { tail -20 $o/trace.log; exit 1; }
python3 tools/trace_summary.py $o/trace | head -40
