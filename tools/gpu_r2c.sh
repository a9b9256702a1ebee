#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
./tools/gpu_tests_all.sh "test_gpu_keys or test_engine or fullsize or test_gpu_cover" || exit 1
mkdir -p gpurun_out/b3
run() {  # tag args...
    local tag=$1; shift
    env "$@" timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/b3/$tag.json 2> gpurun_out/b3/$tag.err || { tail -20 gpurun_out/b3/$tag.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/b3/$tag.json'));print('$tag', round(d['ms_per_step'],3), d['phases_ms'], d['results'])"
}
run keys0 SYZCOV_MR_CFG=0,0
run keys14 SYZCOV_MR_CFG=14,0
run keys12 SYZCOV_MR_CFG=12,0
