#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
./tools/gpu_tests_all.sh "newcov or new_inputs or exec_output or sentinel or test_gpu_manager" || exit 1
mkdir -p gpurun_out/nc
timeout -k 10 300 python -u bench.py --workload newcov --steps 20 --warmup 5 --no-cpu > gpurun_out/nc/keys.json 2> gpurun_out/nc/keys.err || { tail -20 gpurun_out/nc/keys.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/nc/keys.json'));print('keys', d['ms_per_step'], d['phases_ms'], d['roofline']['frac'], d['results']['new_records_per_batch'][:4], d['results']['candidates_per_batch'][:4])"
timeout -k 10 300 python -u bench.py --workload newcov --steps 20 --warmup 5 --no-cpu --no-universe > gpurun_out/nc/win.json 2> gpurun_out/nc/win.err || { tail -20 gpurun_out/nc/win.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/nc/win.json'));print('window', d['ms_per_step'], d['phases_ms'], d['roofline']['frac'], d['results']['new_records_per_batch'][:4], d['results']['candidates_per_batch'][:4])"
SYZCOV_NEWCOV_PATH=probe timeout -k 10 300 python -u bench.py --workload newcov --steps 20 --warmup 5 --no-cpu > gpurun_out/nc/probe.json 2> gpurun_out/nc/probe.err || { tail -20 gpurun_out/nc/probe.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/nc/probe.json'));print('keys-probe', d['ms_per_step'], d['phases_ms'], d['roofline']['frac'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/nc/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload newcov --steps 20 --warmup 5 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/nc/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/nc/prof.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/nc/prof -name "*kernel_stats.csv" -exec head -20 {} \;
