set -o pipefail
export TMPDIR=/tmp
for v in 0 8 9 10 11; do
  SYZCOV_MR_CFG=$v,1 timeout -k 10 200 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -k "engine_step" > gpurun_out/sw_t$v.log 2>&1 || { echo "variant $v FAILED"; tail -5 gpurun_out/sw_t$v.log; }
  echo "== $v $(tail -1 gpurun_out/sw_t$v.log)"
  SYZCOV_MR_CFG=$v,1 timeout -k 10 120 python3 tools/kbench.py minimize --reps 2 2>&1 | grep "ms " || exit 1
done
