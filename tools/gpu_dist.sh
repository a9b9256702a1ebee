#!/bin/bash
# sharded engine on one GPU: distributed parity tests + a 2-rank C3-sized bench rehearsal (gloo)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/dist; mkdir -p $o
fault() { grep -q "illegal memory access\|Memory access fault\|HSA_STATUS_ERROR" "$1" && { echo "GPU fault in $1"; exit 1; }; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sharded or world8" > $o/pt.log 2>&1
rc=$?; tail -2 $o/pt.log; fault $o/pt.log; [ $rc -ne 0 ] && grep -E "^E " $o/pt.log | head -8
case $rc in 124|134|137|139) exit 1;; esac
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --global-inputs 2000000 > $o/b2.json 2> $o/b2.err || { tail -20 $o/b2.err; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$o/b2.json') if l.startswith('{')][-1]); print(d['ms_per_step'], d['phases_ms'], d['results'], d['config']['workload'])"
