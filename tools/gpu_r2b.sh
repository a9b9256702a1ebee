#!/bin/bash
# full-size parity tests + driver-shaped bench (round 2)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r2b
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r2b/pytest.log 2>&1 || { tail -40 gpurun_out/r2b/pytest.log; exit 1; }
grep -E "PASS|FAIL|SKIP|passed|failed" gpurun_out/r2b/pytest.log | tail -12
t0=$(date +%s)
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2b/bench.json 2> gpurun_out/r2b/bench.err || { tail -30 gpurun_out/r2b/bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - t0 )) s"
cat gpurun_out/r2b/bench.json
