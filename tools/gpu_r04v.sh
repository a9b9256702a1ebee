#!/bin/bash
# Round-4 full validation: every -m gpu test, smoke, the driver-shaped bench
# line, and the rocprofv3 evidence (tools/profile_r04.sh).
# usage: tools/gpu_r04g.sh [OUTDIR]
set -o pipefail
export TMPDIR=/tmp
o=${1:-gpurun_out/r04g}; mkdir -p $o
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest.log 2>&1
rc=$?; tail -3 $o/pytest.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $o/pytest.log | head -20; }
grep -q "illegal memory access\|HSA_STATUS_ERROR\|Memory access fault" $o/pytest.log && { echo "GPU fault in pytest"; exit 1; }
fatal $rc pytest
[ $rc -ne 0 ] && exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
rc=$?; tail -2 $o/smoke.log; fatal $rc smoke
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench.json 2> $o/bench.err
rc=$?; [ $rc -ne 0 ] && tail -20 $o/bench.err; fatal $rc bench
python3 -c "import json; d=json.load(open('$o/bench.json')); print(round(d['ms_per_step'],4), d['phases_ms'], round(d['roofline']['frac'],4), d['results'], d['c3_single_gpu']['ms_per_step'])"
[ $SECONDS -gt 700 ] && { echo "no time left for profiles ($SECONDS s)"; exit 0; }
timeout -k 10 $((1120 - SECONDS)) bash tools/profile_r04.sh $o/prof
