#!/bin/bash
# rocprofv3 passes for bench.py (run on the GPU box, from the repo root).
#   tools/profile.sh <tag> [bench args...]
# 1) kernel trace + stats (durations)   -> gpurun_out/prof_<tag>/trace
# 2) FETCH_SIZE pass (HBM read bytes)    -> gpurun_out/prof_<tag>/fetch
# 3) WRITE_SIZE pass (HBM write bytes)   -> gpurun_out/prof_<tag>/write
# Each pass is its own run (counters are never combined with tracing).
set -e
tag=${1:-r01}; shift || true
args=${@:---steps 3 --warmup 1 --no-cpu}
out=gpurun_out/prof_$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py $args > $out/trace.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $out/fetch.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $out/write.log 2>&1
echo profile_done
