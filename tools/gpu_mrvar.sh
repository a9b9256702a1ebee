#!/bin/bash
# minimize pass-1 variants: parity (engine / key-mode / full-size C2 tests) for PAR,
# bench phases for BENCH, chunk stamps (debug build) for STAMP
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/mrvar; mkdir -p $o
fault() { grep -q "illegal memory access\|Memory access fault\|HSA_STATUS_ERROR" "$1" && { echo "GPU fault in $1"; exit 1; }; }
for v in $PAR; do
  SYZCOV_MR_CFG=${v%%:*} timeout -k 10 300 python -u -m pytest tests/test_gpu_keys.py tests/test_gpu_engine.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -k "not c3 and not world8 and not c4" > $o/pt_$v.log 2>&1
  rc=$?; echo "variant $v parity: $(tail -1 $o/pt_$v.log)"; fault $o/pt_$v.log; [ $rc -ne 0 ] && { grep -E "^E " $o/pt_$v.log | head -5; }
  case $rc in 124|134|137|139) exit 1;; esac
done
for v in $BENCH; do
  wg=${v#*:}; [ "$wg" = "$v" ] && wg=""
  ch=${v#*@}; [ "$ch" = "$v" ] && ch=""; v0=${v%%@*}
  SYZCOV_MR_CHUNK=$ch SYZCOV_MR_WG=$wg SYZCOV_MR_CFG=${v0%%:*} timeout -k 10 200 python -u bench.py --no-cpu --steps 10 --warmup 3 > $o/b_$v.json 2> $o/b_$v.err || { tail -5 $o/b_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/b_$v.json')); print('variant $v', round(d['ms_per_step'],3), d['phases_ms'], d['results']['kept'])"
done
for v in $STAMP; do
  SYZCOV_MR_CFG=${v%%:*} SYZCOV_LIB=$PWD/syzkaller_amd/variants/mrdbg.so SYZCOV_MR_DBG=2100000000,1000000 \
    timeout -k 10 200 python -u tools/diag_c3.py 1000000 > $o/stamps_$v.log 2>&1
  rc=$?; echo "stamps variant $v"; grep "mr dbg\]   wgs\|minimize ok\|step ok" $o/stamps_$v.log; fault $o/stamps_$v.log
  case $rc in 124|134|137|139) exit 1;; esac
done
