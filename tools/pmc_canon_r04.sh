#!/bin/bash
# Where canon's wave time goes (one pass per counter set, kbench canon --keys, one launch):
# parked at s_waitcnt (SQ_WAIT_ANY), issue stalls (SQ_WAIT_INST_ANY), issuing (SQ_ACTIVE_INST_*).
set -o pipefail
export TMPDIR=/tmp
o=${1:-gpurun_out/pmc_canon}; mkdir -p $o
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $o/pmc$i -o run -- python3 tools/kbench.py canon --keys --reps 1 > $o/pmc$i.log 2>&1 || { tail -3 $o/pmc$i.log; echo "pmc pass $i failed"; exit 1; }
done
python3 tools/pmc_summary.py $o > $o/summary.txt 2>&1; grep -A20 "canon_key_kernel<32" $o/summary.txt | head -24
