#!/bin/bash
# Round-4 GPU call M: pad-free canon key kernel with past-end chunks wrapped to
# the segment's start — parity (key mode) and timing against variants/g.so
# (the committed kernel) and variants/bq1.so (rank batches of one row quad).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04m; mkdir -p $o
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_keys.py "tests/test_gpu_fullsize.py::test_c2_fullsize_digest" > $o/pytest.log 2>&1
rc=$?; tail -3 $o/pytest.log; grep -q "illegal memory access\|HSA_STATUS_ERROR\|Memory access fault" $o/pytest.log && { echo "GPU fault"; exit 1; }
fatal $rc pytest
[ $rc -ne 0 ] && { grep -E "^E " $o/pytest.log | head -10; exit 1; }
V=$PWD/syzkaller_amd/variants
for v in g new bq1 g new bq1; do
  if [ $v = new ]; then e=""; else e="SYZCOV_LIB=$V/$v.so"; fi
  env $e timeout -k 10 150 python -u tools/kbench.py canon --keys --reps 5 > $o/canon_$v.log 2>&1 || { tail -5 $o/canon_$v.log; exit 1; }
  echo "canon $v: $(tail -3 $o/canon_$v.log | awk '{print $2}' | tr '\n' ' ')"
done
echo done
