#!/bin/bash
# One GPU-box pass: parity tests, bench, rocprofv3 evidence.
#   tools/gpu_check.sh <tag> [pytest -k expr]
set -o pipefail
tag=${1:-r01}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    ${2:+-k "$2"} > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
timeout -k 10 300 python3 bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
bash tools/profile.sh $tag || exit 1
