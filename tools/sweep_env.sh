#!/bin/bash
# kbench <phase> under environment settings (tuning knobs), after the engine
# parity tests under each setting:  tools/sweep_env.sh canon "" "SYZCOV_X=1" ...
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/se
ph=$1; shift
for e in "$@"; do
  echo "== env [$e]"
  env $e timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/se/pytest.log 2>&1 || { tail -30 gpurun_out/se/pytest.log; exit 1; }
  tail -1 gpurun_out/se/pytest.log
  env $e timeout -k 10 200 python3 tools/kbench.py $ph --reps 4 || exit 1
done
