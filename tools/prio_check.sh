#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pc
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "prio or choice or choose or static" > gpurun_out/pc/pytest.log 2>&1 || { tail -30 gpurun_out/pc/pytest.log; exit 1; }
tail -1 gpurun_out/pc/pytest.log
timeout -k 10 300 python3 bench.py --workload prio --no-cpu | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'], d['phases_ms'], round(d['roofline']['frac'],4))"
