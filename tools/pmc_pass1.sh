set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r05c; mkdir -p $o
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  for L in 22 17; do
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $o/pmc${i}_L$L -o run -- python3 tools/kbench.py minimize --keys --reps 1 --log2-space $L > $o/pmc${i}_L$L.log 2>&1 || { tail -3 $o/pmc${i}_L$L.log; echo "pmc pass $i L$L failed"; exit 1; }
  done
done
echo done
