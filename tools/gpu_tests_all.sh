#!/bin/bash
# all GPU parity tests + smoke (optionally -k expr)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/t
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${1:+-k "$1"} > gpurun_out/t/pytest.log 2>&1 || { grep -E "PASS|FAIL|ERROR" gpurun_out/t/pytest.log | tail -5; tail -60 gpurun_out/t/pytest.log; exit 1; }
tail -3 gpurun_out/t/pytest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -3
