#!/bin/bash
# Round-3 rocprofv3 evidence (run on the GPU box from the repo root):
#   corpus C2 (key mode): kernel trace + stats, FETCH_SIZE and WRITE_SIZE passes -> traffic
#   newcov C5: the same;  prio C4: trace + stats
# counters never combined with tracing; each pass its own run (MI355X_MICROARCH.md)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/prof_r03
mkdir -p $o
B="python3 bench.py --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/corpus_trace -o run -- $B --steps 5 --warmup 2 > $o/corpus_trace.log 2>&1 || { tail -20 $o/corpus_trace.log; exit 1; }
python3 tools/trace_summary.py $o/corpus_trace > $o/corpus_summary.txt && head -12 $o/corpus_summary.txt
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/corpus_fetch -o run -- $B --steps 1 --warmup 0 > $o/cf.log 2>&1 || { tail -5 $o/cf.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/corpus_write -o run -- $B --steps 1 --warmup 0 > $o/cw.log 2>&1 || { tail -5 $o/cw.log; exit 1; }
python3 tools/traffic.py $o/corpus_fetch $o/corpus_write $o/corpus_traffic.json > /dev/null && cat $o/corpus_traffic.json
N="$B --workload newcov"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/newcov_trace -o run -- $N --steps 10 --warmup 3 > $o/newcov_trace.log 2>&1 || { tail -20 $o/newcov_trace.log; exit 1; }
python3 tools/trace_summary.py $o/newcov_trace > $o/newcov_summary.txt && head -10 $o/newcov_summary.txt
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/newcov_fetch -o run -- $N --steps 2 --warmup 0 --history 4 > $o/nf.log 2>&1 || { tail -5 $o/nf.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/newcov_write -o run -- $N --steps 2 --warmup 0 --history 4 > $o/nw.log 2>&1 || { tail -5 $o/nw.log; exit 1; }
python3 tools/traffic.py $o/newcov_fetch $o/newcov_write $o/newcov_traffic.json newcov_own_kernel > /dev/null && cat $o/newcov_traffic.json
P="$B --workload prio"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prio_trace -o run -- $P --steps 10 --warmup 3 > $o/prio_trace.log 2>&1 || { tail -20 $o/prio_trace.log; exit 1; }
python3 tools/trace_summary.py $o/prio_trace > $o/prio_summary.txt && head -8 $o/prio_summary.txt
echo profile_done
