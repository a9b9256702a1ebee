#!/bin/bash
# round-2 first GPU check: parity tests, smoke, driver-shaped bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r2a
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a/pytest.log 2>&1 || { tail -30 gpurun_out/r2a/pytest.log; exit 1; }
tail -2 gpurun_out/r2a/pytest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2a/smoke.log 2>&1 || { cat gpurun_out/r2a/smoke.log; exit 1; }
cat gpurun_out/r2a/smoke.log
/usr/bin/time -v timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2a/bench.json 2> gpurun_out/r2a/bench.err || { tail -30 gpurun_out/r2a/bench.err; exit 1; }
cat gpurun_out/r2a/bench.json
grep -E "Elapsed|Maximum resident" gpurun_out/r2a/bench.err
