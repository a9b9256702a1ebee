#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ncs
rm -f gpurun_out/ncs/stamps.txt
SYZCOV_NC_DBG=${DBG:-24} SYZCOV_NC_STAMP_FILE=gpurun_out/ncs/stamps.txt SYZCOV_NEWCOV_PATH=lds timeout -k 10 300 python3 bench.py --workload newcov --steps 3 --warmup 1 --no-cpu "$@" > gpurun_out/ncs/b.log 2>&1 || { tail -5 gpurun_out/ncs/b.log; exit 1; }
grep "workgroups/CU" gpurun_out/ncs/b.log | tail -1; python3 tools/nc_stamps.py gpurun_out/ncs/stamps.txt
