#!/bin/bash
# C5: new-coverage / triage parity, then the newcov bench line, for the
# default library and each variant:  tools/gpu_newcov.sh [variants/x.so ...]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/nc
for v in default "$@"; do
  lib=; [ $v != default ] && lib=$PWD/syzkaller_amd/$v
  echo "== $v"
  SYZCOV_LIB=$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_manager.py tests/test_gpu_triage.py tests/test_gpu_engine.py -x -q \
      --timeout 250 --timeout-method thread > gpurun_out/nc/pytest.log 2>&1 || { tail -30 gpurun_out/nc/pytest.log; exit 1; }
  tail -1 gpurun_out/nc/pytest.log
  for r in 1 2; do
    SYZCOV_LIB=$lib timeout -k 10 200 python -u bench.py --workload newcov --no-cpu --steps 20 --warmup 5 > gpurun_out/nc/bench.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/nc/bench.json')); print(round(d['ms_per_step'],4), d['phases_ms'], round(d['roofline']['frac'],4))"
  done
done
