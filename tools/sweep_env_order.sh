#!/bin/bash
# kbench order under environment settings, after the sort parity tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/seo
for e in "$@"; do
  echo "== env [$e]"
  env $e timeout -k 10 300 python -u -m pytest tests/test_gpu_cover.py -x -q --timeout 120 --timeout-method thread -k "sort_order or minimize" > gpurun_out/seo/pytest.log 2>&1 || { tail -30 gpurun_out/seo/pytest.log; exit 1; }
  tail -1 gpurun_out/seo/pytest.log
  env $e timeout -k 10 200 python3 tools/kbench.py order --reps 4 || exit 1
done
