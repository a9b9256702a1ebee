#!/bin/bash
# Round-4 GPU call B: newcov (C5) key-mode LDS membership path: tests, then
# the steady-state bench A/B against the per-PC gather path.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04b; mkdir -p $o
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_keys.py tests/test_gpu_corpus_abi.py "tests/test_gpu_cover.py::test_sort_order_parts_merge_to_go_order" \
  tests/test_gpu_manager.py tests/test_gpu_triage.py "tests/test_gpu_fullsize.py::test_c5_newcov_stream_fullsize" \
  "tests/test_gpu_fullsize.py::test_world8_rehearsal_c2" "tests/test_gpu_fullsize.py::test_world8_rehearsal_c3" > $o/pytest.log 2>&1
rc=$?; tail -5 $o/pytest.log; grep -q "illegal memory access\|HSA_STATUS_ERROR\|Memory access fault" $o/pytest.log && { echo "GPU fault"; exit 1; }
fatal $rc pytest
for v in keym gather; do
  if [ $v = keym ]; then e=""; else e="SYZCOV_FORCE=nc_lds,nc_gather"; fi
  env $e timeout -k 10 300 python -u bench.py --workload newcov --no-cpu --steps 10 --warmup 3 > $o/nc_$v.json 2> $o/nc_$v.err
  rc=$?; [ $rc -ne 0 ] && { tail -10 $o/nc_$v.err; fatal $rc nc_$v; }
  python3 -c "import json; d=json.load(open('$o/nc_$v.json')); print('$v', round(d['ms_per_step'],4), d['phases_ms'], round(d['roofline']['frac'],4), d['results']['new_records_per_batch'])"
done
echo done
