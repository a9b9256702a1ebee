#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box from the repo root):
#   tools/profile.sh <tag>
# 1) kernel trace + stats of a short bench run  -> gpurun_out/prof_<tag>/trace
# 2) FETCH_SIZE pass, 3) WRITE_SIZE pass (separate runs; counters are never
#    combined with tracing), one step each      -> gpurun_out/prof_<tag>/{fetch,write}
# 4) per-phase HBM traffic                      -> gpurun_out/prof_<tag>/traffic.json
set -o pipefail
tag=${1:-r01}
out=gpurun_out/prof_$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu > $out/trace.log 2>&1 || { tail -20 $out/trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu > $out/fetch.log 2>&1 || { tail -5 $out/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu > $out/write.log 2>&1 || { tail -5 $out/write.log; exit 1; }
python3 tools/traffic.py $out/fetch $out/write $out/traffic.json
echo profile_done
