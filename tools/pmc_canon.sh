#!/bin/bash
# LDS / instruction counters of the canon kernels (kbench canon, 1 rep), one pass per set
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/pmc_canon; mkdir -p $out
rocprofv3 --list-avail > $out/avail.txt 2>&1 || true
grep -oE 'SQ_[A-Z_]*LDS[A-Z_]*' $out/avail.txt | sort -u > $out/lds_counters.txt || true
i=0
for set in "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE" "SQ_LDS_ATOMIC_RETURN SQ_INSTS_LDS_ATOMIC SQ_INSTS_LDS_STORE SQ_INSTS_LDS_LOAD SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INST_LEVEL_LDS SQ_WAVES" \
           "SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVES GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $out/pmc$i -o run -- python3 tools/kbench.py canon --reps 1 > $out/p$i.log 2>&1 || { tail -5 $out/p$i.log; echo "pass $i failed"; }
done
python3 tools/pmc_summary.py $out > $out/summary.txt 2>&1 || true
cat $out/lds_counters.txt; cat $out/summary.txt | head -60
