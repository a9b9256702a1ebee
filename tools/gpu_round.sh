#!/bin/bash
# One GPU call per milestone: parity tests, smoke, the driver-shaped bench line,
# then the rocprofv3 evidence (tools/profile_r02.sh).  A crash, abort or time
# limit ends the script; an ordinary test failure is reported and the bench
# still runs.   usage: tools/gpu_round.sh OUTDIR [pytest -k expr]
set -o pipefail
export TMPDIR=/tmp
o=${1:-gpurun_out/round}
mkdir -p $o
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
[ -x tools/probe/scan_dpp ] && { timeout -k 10 60 tools/probe/scan_dpp || exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    ${2:+-k "$2"} > $o/pytest.log 2>&1
rc=$?; tail -3 $o/pytest.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $o/pytest.log | head -20; }
grep -q "illegal memory access\|HSA_STATUS_ERROR\|Memory access fault" $o/pytest.log && { echo "GPU fault in pytest"; exit 1; }
fatal $rc pytest
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
rc=$?; tail -2 $o/smoke.log; fatal $rc smoke
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench.json 2> $o/bench.err
rc=$?; cat $o/bench.json; [ $rc -ne 0 ] && tail -20 $o/bench.err; fatal $rc bench
[ "$NOPROF" = 1 ] && exit 0
[ $SECONDS -gt 650 ] && { echo "no time left for profiles ($SECONDS s)"; exit 0; }
timeout -k 10 $((1100 - SECONDS)) bash tools/profile_r03.sh
