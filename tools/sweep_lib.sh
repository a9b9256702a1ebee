#!/bin/bash
# Canon parity on the default build, then kbench <phase> for the default and
# each variant library:  tools/sweep_lib.sh <phase> variants/a.so variants/b.so ...
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sw
ph=$1; shift
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sw/pytest.log 2>&1 || { tail -40 gpurun_out/sw/pytest.log; exit 1; }
tail -1 gpurun_out/sw/pytest.log
echo "== default"; timeout -k 10 200 python3 tools/kbench.py $ph --reps 3 || exit 1
for v in "$@"; do
  echo "== $v"; SYZCOV_LIB=$PWD/syzkaller_amd/$v timeout -k 10 200 python3 tools/kbench.py $ph --reps 3 || exit 1
done
