#!/bin/bash
# C3 fix check + minimize chunk stamps (debug build) + pool trim check
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r2d; mkdir -p $o
fault() { grep -q "illegal memory access\|Memory access fault\|HSA_STATUS_ERROR" "$1" && { echo "GPU fault in $1"; exit 1; }; }
timeout -k 10 200 python -u -m pytest tests/test_sanitize.py -m gpu -x -q --timeout 240 --timeout-method thread > $o/san.log 2>&1; tail -3 $o/san.log; fault $o/san.log
SYZCOV_LIB=$PWD/syzkaller_amd/variants/mrdbg.so SYZCOV_MR_DBG=2100000000,1000000 timeout -k 10 200 python -u tools/diag_c3.py 1000000 > $o/stamps.log 2>&1; grep -v "^\s*File\|Traceback" $o/stamps.log | tail -40; fault $o/stamps.log
timeout -k 10 400 python -u tools/diag_c3.py > $o/c3.log 2>&1; tail -4 $o/c3.log; fault $o/c3.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_keys.py -x -q --timeout 280 --timeout-method thread > $o/pt.log 2>&1; tail -3 $o/pt.log; fault $o/pt.log
