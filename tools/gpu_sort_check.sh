set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/gs
timeout -k 10 400 python -u -m pytest tests/test_gpu_cover.py tests/test_gpu_manager.py tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gs/pytest.log 2>&1 || { tail -30 gpurun_out/gs/pytest.log; exit 1; }
tail -1 gpurun_out/gs/pytest.log
timeout -k 10 100 python3 tools/kbench.py order --reps 5 && timeout -k 10 100 python3 tools/kbench.py order --reps 3 --inputs 8000000 && timeout -k 10 100 python3 tools/kbench.py step --reps 3
