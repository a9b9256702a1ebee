#!/bin/bash
# sort parity, then the order phase vs the read-back interval (SYZCOV_SORT_SYNC)

set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/gs
timeout -k 10 300 python -u -m pytest tests/test_gpu_cover.py tests/test_gpu_fullsize.py tests/test_gpu_manager.py -x -q \
    -k "sort_order or c3_order or c2 or minimize" --timeout 250 --timeout-method thread > gpurun_out/gs/pytest.log 2>&1 \
    || { tail -30 gpurun_out/gs/pytest.log; exit 1; }
tail -1 gpurun_out/gs/pytest.log
for v in 4 8 16; do echo "sync=$v"; SYZCOV_SORT_SYNC=$v timeout -k 10 120 python3 tools/kbench.py order --reps 5 2>&1 | tail -2 || exit 1; done
timeout -k 10 200 python -u bench.py --no-cpu --steps 10 --warmup 3 > /tmp/b.json 2>/dev/null || exit 1
python3 -c "import json; d=json.load(open('/tmp/b.json')); print(round(d['ms_per_step'],3), d['phases_ms'])"
