#!/bin/bash
# Go-sort order variants: parity (sort tests) then kbench order, per library:
#   tools/sweep_order.sh variants/a.so ...   (default build first)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/so
for v in default "$@"; do
  echo "== $v"
  lib=""; [ "$v" != default ] && lib=$PWD/syzkaller_amd/$v
  SYZCOV_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_cover.py -x -q --timeout 120 --timeout-method thread -k "sort_order or minimize" > gpurun_out/so/pytest.log 2>&1 || { tail -30 gpurun_out/so/pytest.log; exit 1; }
  tail -1 gpurun_out/so/pytest.log
  SYZCOV_LIB=$lib timeout -k 10 200 python3 tools/kbench.py order --reps 4 || exit 1
done
