#!/bin/bash
# Round-4 last check of the exact final tree: every -m gpu test, smoke, the
# driver-shaped bench line (profiles come from tools/gpu_r04v.sh runs).
set -o pipefail
export TMPDIR=/tmp
o=${1:-gpurun_out/r04fin}; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest.log 2>&1
rc=$?; tail -3 $o/pytest.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $o/pytest.log | head -20; exit 1; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -5 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench.json 2> $o/bench.err || { tail -20 $o/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$o/bench.json')); print(round(d['ms_per_step'],4), d['phases_ms'], round(d['roofline']['frac'],4), d['results'], d['c3_single_gpu']['ms_per_step'])"
# the membership pass with per-lane row descriptors (variants/mb2.so): its
# newcov tests and C5 line beside the product build's
if [ -f syzkaller_amd/variants/mb2.so ]; then
  SYZCOV_LIB=$PWD/syzkaller_amd/variants/mb2.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_manager.py tests/test_gpu_triage.py "tests/test_gpu_engine.py::test_newcov_batch_vs_sequential" "tests/test_gpu_fullsize.py::test_c5_newcov_stream_fullsize" > $o/pytest_mb2.log 2>&1
  rc=$?; tail -1 $o/pytest_mb2.log; [ $rc -ne 0 ] && exit 1
  for v in main mb2; do
    if [ $v = main ]; then unset SYZCOV_LIB; else export SYZCOV_LIB=$PWD/syzkaller_amd/variants/$v.so; fi
    timeout -k 10 300 python -u bench.py --workload newcov --steps 10 --warmup 3 --no-cpu > $o/nc_$v.json 2> $o/nc_$v.err || { tail -5 $o/nc_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('$o/nc_$v.json')); print('$v', round(d['ms_per_step'],4), d['phases_ms'])"
  done
fi
