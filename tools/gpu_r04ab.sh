#!/bin/bash
# Round-4 GPU call AB: C5 membership pass, double-buffered (product build)
# vs single-step with XCD-paired halves (variants/mb1.so): tests, C5 lines.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04ab; mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_manager.py tests/test_gpu_triage.py tests/test_gpu_dedup.py "tests/test_gpu_engine.py::test_newcov_batch_vs_sequential" "tests/test_gpu_fullsize.py::test_c5_newcov_stream_fullsize" > $o/pytest.log 2>&1
rc=$?; tail -3 $o/pytest.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $o/pytest.log | head -20; exit 1; }
for v in ${VARIANTS:-main mb1}; do
  if [ $v = main ]; then unset SYZCOV_LIB; else export SYZCOV_LIB=$PWD/syzkaller_amd/variants/$v.so; fi
  timeout -k 10 300 python -u bench.py --workload newcov --steps 10 --warmup 3 --no-cpu > $o/nc_$v.json 2> $o/nc_$v.err || { tail -5 $o/nc_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/nc_$v.json')); print('$v', round(d['ms_per_step'],4), d['phases_ms'])"
done
unset SYZCOV_LIB
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$o/prof -o nc -- python3 $GRAFT_REPO_ROOT/bench.py --workload newcov --steps 10 --warmup 3 --no-cpu > $GRAFT_REPO_ROOT/$o/prof.log 2>&1 || exit 1
echo done
