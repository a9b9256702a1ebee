#!/bin/bash
# Round-4 rocprofv3 evidence (run on the GPU box from the repo root):
#   corpus C2 (key mode): kernel trace + stats, FETCH_SIZE and WRITE_SIZE passes -> traffic
#   canon LDS / VALU / wait counters (tools/kbench.py step --keys, one step)
#   newcov C5 (steady state): trace + stats, FETCH / WRITE of the timed batches only
#   prio C4: trace + stats
# counters never combined with tracing; each pass its own run (MI355X_MICROARCH.md)
set -o pipefail
export TMPDIR=/tmp
o=${1:-gpurun_out/prof_r04}
mkdir -p $o
B="python3 bench.py --no-cpu --no-c3 --no-dropin"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/corpus_trace -o run -- $B --steps 5 --warmup 2 > $o/corpus_trace.log 2>&1 || { tail -20 $o/corpus_trace.log; exit 1; }
python3 tools/trace_summary.py $o/corpus_trace > $o/corpus_summary.txt && head -16 $o/corpus_summary.txt
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/corpus_fetch -o run -- $B --steps 1 --warmup 0 > $o/cf.log 2>&1 || { tail -5 $o/cf.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/corpus_write -o run -- $B --steps 1 --warmup 0 > $o/cw.log 2>&1 || { tail -5 $o/cw.log; exit 1; }
python3 tools/traffic.py $o/corpus_fetch $o/corpus_write $o/corpus_traffic.json > /dev/null && cat $o/corpus_traffic.json
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $o/pmc$i -o run -- python3 tools/kbench.py step --keys --reps 1 > $o/pmc$i.log 2>&1 || { tail -3 $o/pmc$i.log; echo "pmc pass $i failed"; }
done
python3 tools/pmc_summary.py $o > $o/pmc_summary.txt 2>&1; grep -A18 "canon_key_kernel<32" $o/pmc_summary.txt | head -20
N="$B --workload newcov"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/newcov_trace -o run -- $N --steps 10 --warmup 3 > $o/newcov_trace.log 2>&1 || { tail -20 $o/newcov_trace.log; exit 1; }
python3 tools/trace_summary.py $o/newcov_trace > $o/newcov_summary.txt && head -10 $o/newcov_summary.txt
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/newcov_fetch -o run -- $N --steps 10 --warmup 3 > $o/nf.log 2>&1 || { tail -5 $o/nf.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/newcov_write -o run -- $N --steps 10 --warmup 3 > $o/nw.log 2>&1 || { tail -5 $o/nw.log; exit 1; }
python3 tools/traffic.py $o/newcov_fetch $o/newcov_write $o/newcov_traffic.json newcov_own_kernel 10 > /dev/null && cat $o/newcov_traffic.json
P="$B --workload prio"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prio_trace -o run -- $P --steps 10 --warmup 3 > $o/prio_trace.log 2>&1 || { tail -20 $o/prio_trace.log; exit 1; }
python3 tools/trace_summary.py $o/prio_trace > $o/prio_summary.txt && head -8 $o/prio_summary.txt
echo profile_done
