#!/bin/bash
# quick GPU iteration: selected parity tests (TESTS, K) then bench probes ("name:env:args" specs)
set -o pipefail
export TMPDIR=/tmp
o=${OUT:-gpurun_out/q}; mkdir -p $o
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TTIME:-400} python -u -m pytest $TESTS -m gpu -x -q --timeout 200 --timeout-method thread ${K:+-k "$K"} > $o/pytest.log 2>&1
  rc=$?; tail -3 $o/pytest.log; [ $rc -ne 0 ] && grep -E "^E |FAIL" $o/pytest.log | head -20
  grep -q "illegal memory access\|HSA_STATUS_ERROR\|Memory access fault" $o/pytest.log && { echo "GPU fault"; exit 1; }
  case $rc in 124|134|137|139) echo "fatal rc=$rc"; exit 1;; esac
fi
[ $# -gt 0 ] && exec_probe=1
[ -n "$exec_probe" ] && tools/gpu_probe.sh $o "$@"
exit 0
