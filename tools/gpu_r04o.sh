#!/bin/bash
# Round-4 GPU call O: the driver's multi-GPU launch rehearsed on the one-GPU
# box (bench.py --gpus 2 starts its own ranks; both on GPU 0, gloo).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04o; mkdir -p $o
timeout -k 10 500 python -u bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu --no-dropin > $o/bench2.json 2> $o/bench2.err
rc=$?; tail -3 $o/bench2.err; [ $rc -ne 0 ] && exit 1
python3 -c "import json; d=json.load(open('$o/bench2.json')); print(d['n_gpus'], d.get('rccl_ranks'), d.get('backend'), round(d['ms_per_step'],3), d['phases_ms'], d['results'], d['config']['workload'])"
