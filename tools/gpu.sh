#!/bin/bash
# The one GPU-box entry point of this repo (run it through gpurun from the repo
# root):   tools/gpu.sh OUTDIR STEP [STEP ...]
# Steps run in the order given; each has its own time limit, and a GPU fault,
# an abort, a segfault or a time limit ends the script (nothing more runs on
# the GPU after it).  An ordinary test failure is reported and ends it too.
#   tests            every -m gpu test (PYTEST_SEL / K narrow it: files, -k expr)
#   smoke            __graft_entry__.smoke()
#   bench            the driver's line: bench.py --gpus 1 (STEPS, WARMUP)
#   newcov | newcov_early | dedup | prio    the other workloads' lines
#   probe:NAME:ENV:ARGS   one bench line (no CPU baseline) with ENV set and
#                    ARGS appended, commas for spaces (e.g.
#                    probe:v1:SYZCOV_LIB=$PWD/syzkaller_amd/variants/v1.so:--workload,newcov)
#   trace:ARGS       rocprofv3 kernel trace + stats of bench.py ARGS
#   kbench:ARGS      tools/kbench.py ARGS (kernel micro-bench)
#   profile          tools/profile.sh OUTDIR/prof $PARTS (rocprofv3 stats + PMC passes)
set -o pipefail
export TMPDIR=/tmp
o=${1:?usage: tools/gpu.sh OUTDIR STEP...}; shift
mkdir -p $o
fatal() {  # rc, step, log
  grep -q "illegal memory access\|HSA_STATUS_ERROR\|Memory access fault" $3 2>/dev/null &&
    { echo "GPU fault in $2"; exit 1; }
  case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit 1;; esac
}
summ() {  # one line of a bench JSON
  python3 - "$1" "$2" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
if "c3_rank_of_8" in d:  # the rank-share leg (alone, or as a sub-record)
    q = d["c3_rank_of_8"]
    print(sys.argv[2], "rank_of_8", round(q["ms_per_step"], 4), q["phases_ms"],
          "canon", round(q["canon_roofline"]["frac"], 4), "min", round(q["minimize_roofline"]["frac"], 4))
    if "ms_per_step" not in d:
        sys.exit(0)
r = d.get("roofline", {})
print(sys.argv[2], round(d["ms_per_step"], 4), d.get("phases_ms"), "frac", round(r.get("frac", 0), 4),
      d.get("results", {}).get("kept"), d.get("results", {}).get("union"),
      "c2", (d.get("c2") or {}).get("ms_per_step"), (d.get("c2") or {}).get("phases_ms"))
EOF
}
for step in "$@"; do
  case $step in
  tests)
    timeout -k 10 ${TTIME:-1000} python -u -m pytest ${PYTEST_SEL:-tests} -m gpu -x -q --timeout 300 \
        --timeout-method thread ${K:+-k "$K"} > $o/pytest.log 2>&1
    rc=$?; tail -3 $o/pytest.log
    [ $rc -ne 0 ] && { grep -E "^E |FAIL|Error" $o/pytest.log | head -30; fatal $rc tests $o/pytest.log; exit 1; }
    ;;
  smoke)
    timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
    rc=$?; tail -2 $o/smoke.log; [ $rc -ne 0 ] && { fatal $rc smoke $o/smoke.log; exit 1; }
    ;;
  bench)
    timeout -k 10 600 python -u bench.py --gpus 1 --steps ${STEPS:-5} --warmup ${WARMUP:-2} \
        > $o/bench.json 2> $o/bench.err
    rc=$?; [ $rc -ne 0 ] && { tail -20 $o/bench.err; fatal $rc bench $o/bench.err; exit 1; }
    summ $o/bench.json bench
    ;;
  newcov|newcov_early|dedup|prio)
    w=${step%_early}; extra=""; [ $step = newcov_early ] && extra="--history 32"
    timeout -k 10 400 python -u bench.py --workload $w --steps 10 --warmup 3 $extra \
        > $o/$step.json 2> $o/$step.err
    rc=$?; [ $rc -ne 0 ] && { tail -20 $o/$step.err; fatal $rc $step $o/$step.err; exit 1; }
    summ $o/$step.json $step
    ;;
  probe:*)
    spec=${step#probe:}; name=${spec%%:*}; rest=${spec#*:}; envs=${rest%%:*}; args=${rest#*:}
    args=${args//,/ }  # commas separate the appended arguments
    env $(eval echo $envs) timeout -k 10 400 python -u bench.py --no-cpu --no-dropin \
        --steps ${STEPS:-10} --warmup 3 $args > $o/$name.json 2> $o/$name.err
    rc=$?; [ $rc -ne 0 ] && { tail -15 $o/$name.err; fatal $rc $name $o/$name.err; exit 1; }
    summ $o/$name.json $name
    ;;
  trace:*)  # kernel trace + stats of one bench command (ARGS appended, commas for spaces)
    targs=${step#trace:}; targs=${targs//,/ }
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace -o run -- \
        python3 bench.py --no-cpu --no-c2 --no-dropin $targs > $o/trace.log 2>&1 ||
        { tail -20 $o/trace.log; exit 1; }
    python3 tools/trace_summary.py $o/trace > $o/trace_summary.txt; head -30 $o/trace_summary.txt
    [ -n "$TL_MARK" ] && python3 tools/trace_timeline.py $o/trace "$TL_MARK" > $o/timeline.txt
    # TL_LAST="KERNEL N": per-step kernel times of the last N steps (trace_last.py)
    [ -n "$TL_LAST" ] && python3 tools/trace_last.py $o/trace $TL_LAST > $o/last.txt && head -8 $o/last.txt
    find $o/trace -name '*kernel_trace.csv' -delete
    ;;
  kbench:*)
    timeout -k 10 300 python -u tools/kbench.py ${step#kbench:} > $o/kbench.log 2>&1
    rc=$?; tail -20 $o/kbench.log; [ $rc -ne 0 ] && { fatal $rc kbench $o/kbench.log; exit 1; }
    ;;
  profile)
    timeout -k 10 ${PTIME:-900} bash tools/profile.sh $o/prof $PARTS || exit 1
    # the raw per-dispatch CSVs stay on the box (gpurun copies back <= 64 MiB)
    find $o/prof \( -name '*kernel_trace.csv' -o -name '*counter_collection.csv' \) -delete
    ;;
  *) echo "unknown step $step"; exit 2;;
  esac
done
echo "gpu.sh done"
