#!/bin/bash
# window mode (no universe, 64 ranges): minimize variants, bench phases + parity of the stream
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/wmr; mkdir -p $o
for v in 1,0 4,16 4,4 4,2; do
  SYZCOV_MR_CFG=$v timeout -k 10 200 python -u bench.py --no-cpu --no-universe --steps 6 --warmup 2 > $o/b_$v.json 2> $o/b_$v.err || { tail -5 $o/b_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/b_$v.json')); print('window $v', round(d['ms_per_step'],3), d['phases_ms'], d['results']['kept'])"
done
SYZCOV_MR_CFG=${PV:-4,16} timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_fullsize.py tests/test_gpu_cover.py tests/test_gpu_manager.py -x -q --timeout 280 --timeout-method thread -k "not c3 and not c4" > $o/pt.log 2>&1
rc=$?; tail -2 $o/pt.log; [ $rc -ne 0 ] && grep -E "^E " $o/pt.log | head -5; exit 0
