#!/bin/bash
# GPU parity tests only (optionally -k expr)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/t
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${1:+-k "$1"} > gpurun_out/t/pytest.log 2>&1 || { tail -40 gpurun_out/t/pytest.log; exit 1; }
tail -3 gpurun_out/t/pytest.log
