#!/bin/bash
# key-mode canon: 2-pass key sort (default) vs the 3-pass window-offset sort: parity + bench phases
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/ck2; mkdir -p $o
fault() { grep -q "illegal memory access\|Memory access fault\|HSA_STATUS_ERROR" "$1" && { echo "GPU fault in $1"; exit 1; }; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_keys.py tests/test_gpu_fullsize.py tests/test_gpu_engine.py tests/test_gpu_manager.py -x -q --timeout 280 --timeout-method thread -k "not c4" > $o/pt.log 2>&1
rc=$?; tail -2 $o/pt.log; fault $o/pt.log; [ $rc -ne 0 ] && { grep -E "^E " $o/pt.log | head -8; }
case $rc in 124|134|137|139) exit 1;; esac
for k in ${KS:-1 0}; do
  SYZCOV_CANON_KEY2=$k timeout -k 10 200 python -u bench.py --no-cpu --steps 10 --warmup 3 > $o/b_$k.json 2> $o/b_$k.err || { tail -5 $o/b_$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/b_$k.json')); print('key2=$k', round(d['ms_per_step'],3), d['phases_ms'], d['results']['kept'], d['results']['union'])"
done
