#!/bin/bash
# Round-4 GPU call J: the engine's order phase without the finisher's host
# read-back (error flag on the device) — parity — and first-chunk sizes of
# Minimize's chunk schedule (variants/first*.so) against the default 64.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04j; mkdir -p $o
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fullsize.py tests/test_gpu_engine.py tests/test_gpu_cover.py > $o/pytest.log 2>&1
rc=$?; tail -3 $o/pytest.log; grep -q "illegal memory access\|HSA_STATUS_ERROR\|Memory access fault" $o/pytest.log && { echo "GPU fault"; exit 1; }
fatal $rc pytest
[ $rc -ne 0 ] && { grep -E "^E " $o/pytest.log | head -10; exit 1; }
V=$PWD/syzkaller_amd/variants
for v in def first1024 first4096 def first1024 first4096; do
  if [ $v = def ]; then e=""; else e="SYZCOV_LIB=$V/$v.so"; fi
  env $e timeout -k 10 150 python -u tools/kbench.py minimize --keys --reps 5 > $o/min_$v.log 2>&1 || { tail -5 $o/min_$v.log; exit 1; }
  echo "min $v: $(tail -3 $o/min_$v.log | awk '{print $2}' | tr '\n' ' ')"
done
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-c3 --no-dropin --no-cpu > $o/bench$r.json 2> $o/bench$r.err
  rc=$?; [ $rc -ne 0 ] && tail -5 $o/bench$r.err; fatal $rc bench
  python3 -c "import json; d=json.load(open('$o/bench$r.json')); print(round(d['ms_per_step'],4), d['phases_ms'], round(d['roofline']['frac'],4))"
done
echo done
