#!/bin/bash
# One GPU iteration: selected parity tests, then selected bench lines.
#   TESTS="tests/test_gpu_keys.py ..." K="-k expr" BENCH="corpus newcov prio" \
#   tools/gpu_iter.sh OUTDIR
# A GPU fault, abort, segfault or time limit ends the script at once.
set -o pipefail
export TMPDIR=/tmp
o=${1:-gpurun_out/iter}
mkdir -p $o
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
fault() { grep -q "illegal memory access\|HSA_STATUS_ERROR\|Memory access fault" "$1" && { echo "GPU fault in $1"; exit 1; }; }
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TTIME:-600} python -u -m pytest $TESTS -m gpu -x -q --timeout 280 \
      --timeout-method thread ${K:+-k "$K"} > $o/pytest.log 2>&1
  rc=$?; tail -3 $o/pytest.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" $o/pytest.log | head -20; }
  fault $o/pytest.log; fatal $rc pytest
fi
for b in $BENCH; do
  timeout -k 10 300 python -u bench.py --workload $b --steps ${STEPS:-20} --warmup 5 --no-cpu \
      $BARGS > $o/bench_$b.json 2> $o/bench_$b.err
  rc=$?; [ $rc -ne 0 ] && tail -20 $o/bench_$b.err; fault $o/bench_$b.err; fatal $rc bench_$b
  python3 -c "import json,sys; d=json.load(open('$o/bench_$b.json')); print('$b', round(d['ms_per_step'],4), d.get('phases_ms'), d['roofline']['frac'], d.get('results',{}).get('kept'), d.get('results',{}).get('union'))"
done
exit 0
