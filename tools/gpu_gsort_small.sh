#!/bin/bash
# gosort LDS finisher size (SYZ_GSORT_SMALL variants): sort parity (Go order at
# 20k / 1M / patterns, C3's 10M digest), then the order phase and the C2 step.
#   usage: tools/gpu_gsort_small.sh variants/a.so variants/b.so ...
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/gs
for v in default "$@"; do
  lib=; [ $v != default ] && lib=$PWD/syzkaller_amd/$v
  echo "== $v"
  SYZCOV_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_cover.py tests/test_gpu_fullsize.py tests/test_gpu_manager.py -x -q \
      -k "sort_order or c3_order or c2 or minimize" --timeout 250 --timeout-method thread > gpurun_out/gs/pytest_${v//\//_}.log 2>&1 \
      || { tail -30 gpurun_out/gs/pytest_${v//\//_}.log; exit 1; }
  tail -1 gpurun_out/gs/pytest_${v//\//_}.log
  SYZCOV_LIB=$lib timeout -k 10 120 python3 tools/kbench.py order --reps 6 2>&1 | tail -3 || exit 1
  SYZCOV_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu --steps 10 --warmup 3 > /tmp/b.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('/tmp/b.json')); print('$v', round(d['ms_per_step'],3), d['phases_ms'])"
done
