#!/bin/bash
# Round-4 GPU call Y: cover_dedup + ingest into the device new-coverage check.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04y; mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dedup.py > $o/pytest.log 2>&1
rc=$?; tail -15 $o/pytest.log; [ $rc -ne 0 ] && exit 1
exit 0
