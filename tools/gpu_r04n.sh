#!/bin/bash
# Round-4 GPU call N: C5 candidate items in range-major order (the membership
# table's range slice stays in L2) — parity (C5/C5S streams, newcov tests) and
# the steady-state bench against variants/nco.so (call-major items).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04n; mkdir -p $o
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
timeout -k 10 700 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  "tests/test_gpu_fullsize.py::test_c5_newcov_stream_fullsize" tests/test_gpu_engine.py tests/test_gpu_manager.py tests/test_gpu_triage.py > $o/pytest.log 2>&1
rc=$?; tail -3 $o/pytest.log; grep -q "illegal memory access\|HSA_STATUS_ERROR\|Memory access fault" $o/pytest.log && { echo "GPU fault"; exit 1; }
fatal $rc pytest
[ $rc -ne 0 ] && { grep -E "^E " $o/pytest.log | head -10; exit 1; }
V=$PWD/syzkaller_amd/variants
for v in nco new nco new; do
  if [ $v = new ]; then e=""; else e="SYZCOV_LIB=$V/$v.so"; fi
  env $e timeout -k 10 240 python -u bench.py --workload newcov --steps 20 --warmup 5 --no-cpu > $o/c5_$v.json 2> $o/c5_$v.err || { tail -5 $o/c5_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/c5_$v.json')); print('c5 $v', round(d['ms_per_step'],4), d['results']['new_records_per_batch'][:4])"
done
echo done
