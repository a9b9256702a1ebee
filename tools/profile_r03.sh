#!/bin/bash
# Round-3 rocprofv3 evidence (run on the GPU box from the repo root):
#   corpus C2 (key mode): kernel trace + stats, FETCH_SIZE and WRITE_SIZE passes -> traffic
#   canon / minimize LDS + VALU counters (tools/kbench.py step --keys, one step)
#   newcov C5 (steady state): trace + stats, FETCH / WRITE of the timed batches
#   prio C4: trace + stats, MFMA busy counters (positional and dense)
# counters never combined with tracing; each pass its own run (MI355X_MICROARCH.md)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/prof_r03
mkdir -p $o
B="python3 bench.py --no-cpu --no-c3 --no-dropin"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/corpus_trace -o run -- $B --steps 5 --warmup 2 > $o/corpus_trace.log 2>&1 || { tail -20 $o/corpus_trace.log; exit 1; }
python3 tools/trace_summary.py $o/corpus_trace > $o/corpus_summary.txt && head -14 $o/corpus_summary.txt
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/corpus_fetch -o run -- $B --steps 1 --warmup 0 > $o/cf.log 2>&1 || { tail -5 $o/cf.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/corpus_write -o run -- $B --steps 1 --warmup 0 > $o/cw.log 2>&1 || { tail -5 $o/cw.log; exit 1; }
python3 tools/traffic.py $o/corpus_fetch $o/corpus_write $o/corpus_traffic.json > /dev/null && cat $o/corpus_traffic.json
i=0
for set in "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $o/pmc$i -o run -- python3 tools/kbench.py step --keys --reps 1 > $o/pmc$i.log 2>&1 || { tail -3 $o/pmc$i.log; echo "pmc pass $i failed"; }
done
python3 tools/pmc_summary.py $o > $o/pmc_summary.txt 2>&1; head -60 $o/pmc_summary.txt
N="$B --workload newcov"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/newcov_trace -o run -- $N --steps 10 --warmup 3 > $o/newcov_trace.log 2>&1 || { tail -20 $o/newcov_trace.log; exit 1; }
python3 tools/trace_summary.py $o/newcov_trace > $o/newcov_summary.txt && head -10 $o/newcov_summary.txt
P="$B --workload prio"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prio_trace -o run -- $P --steps 10 --warmup 3 > $o/prio_trace.log 2>&1 || { tail -20 $o/prio_trace.log; exit 1; }
python3 tools/trace_summary.py $o/prio_trace > $o/prio_summary.txt && head -8 $o/prio_summary.txt
for pv in "" "--prio-dense"; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $o/prio_mfma${pv:+_dense} -o run -- $P $pv --steps 2 --warmup 1 > $o/pm${pv:+d}.log 2>&1 || { tail -3 $o/pm${pv:+d}.log; echo "mfma pass failed"; }
done
echo profile_done
