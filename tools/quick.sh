#!/bin/bash
# quick GPU iteration: range-engine parity tests + phase micro-benches
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/q
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -k "${1:-engine}" > gpurun_out/q/pytest.log 2>&1 || { tail -40 gpurun_out/q/pytest.log; exit 1; }
tail -2 gpurun_out/q/pytest.log
for w in canon minimize step; do timeout -k 10 200 python3 tools/kbench.py $w --reps 3 || exit 1; done
