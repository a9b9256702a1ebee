#!/bin/bash
# Round-4 GPU call AA: C5 with the separate nibble membership pass: the
# newcov / triage / dedup-ingest tests and C5 digests, then the C5 bench line.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04aa; mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_manager.py tests/test_gpu_triage.py tests/test_gpu_dedup.py "tests/test_gpu_engine.py::test_newcov_batch_vs_sequential" "tests/test_gpu_fullsize.py::test_c5_newcov_stream_fullsize" > $o/pytest.log 2>&1
rc=$?; tail -5 $o/pytest.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $o/pytest.log | head -20; exit 1; }
timeout -k 10 300 python -u bench.py --workload newcov --steps 10 --warmup 3 --no-cpu > $o/nc.json 2> $o/nc.err || { tail -5 $o/nc.err; exit 1; }
python3 -c "import json; d=json.load(open('$o/nc.json')); print(round(d['ms_per_step'],4), d['phases_ms'], d['results']['new_records_per_batch'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$o/prof -o nc -- python3 $GRAFT_REPO_ROOT/bench.py --workload newcov --steps 10 --warmup 3 --no-cpu > $GRAFT_REPO_ROOT/$o/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && f=$(find $o/prof -name "*kernel_stats.csv" | head -1) && head -12 $f | cut -c1-160
