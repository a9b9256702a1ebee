#!/bin/bash
# Round-4 GPU call AD: the C5 line and its FETCH/WRITE traffic (timed batches
# only) on the final newcov build, plus its newcov tests.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04ad; mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_manager.py tests/test_gpu_triage.py tests/test_gpu_dedup.py "tests/test_gpu_engine.py::test_newcov_batch_vs_sequential" "tests/test_gpu_fullsize.py::test_c5_newcov_stream_fullsize" > $o/pytest.log 2>&1
rc=$?; tail -2 $o/pytest.log; [ $rc -ne 0 ] && exit 1
N="python3 bench.py --no-cpu --no-c3 --no-dropin --workload newcov"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/newcov_trace -o run -- $N --steps 10 --warmup 3 > $o/newcov_trace.log 2>&1 || { tail -20 $o/newcov_trace.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/newcov_fetch -o run -- $N --steps 10 --warmup 3 > $o/nf.log 2>&1 || { tail -5 $o/nf.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/newcov_write -o run -- $N --steps 10 --warmup 3 > $o/nw.log 2>&1 || { tail -5 $o/nw.log; exit 1; }
python3 tools/traffic.py $o/newcov_fetch $o/newcov_write $o/newcov_traffic.json newcov_own_kernel 10 > /dev/null && cat $o/newcov_traffic.json
timeout -k 10 300 python -u bench.py --workload newcov --steps 10 --warmup 3 > $o/nc.json 2> $o/nc.err || { tail -5 $o/nc.err; exit 1; }
python3 -c "import json; d=json.load(open('$o/nc.json')); print(round(d['ms_per_step'],4), d['phases_ms'], d['roofline'])"
