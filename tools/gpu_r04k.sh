#!/bin/bash
# Round-4 GPU call K: waves per workgroup of the canon kernels (variants/wpb*.so) against 2.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04k; mkdir -p $o
V=$PWD/syzkaller_amd/variants
for v in def wpb1 wpb4 def wpb1 wpb4; do
  if [ $v = def ]; then e=""; else e="SYZCOV_LIB=$V/$v.so"; fi
  env $e timeout -k 10 150 python -u tools/kbench.py canon --keys --reps 5 > $o/canon_$v.log 2>&1 || { tail -5 $o/canon_$v.log; exit 1; }
  echo "canon $v: $(tail -3 $o/canon_$v.log | awk '{print $2}' | tr '\n' ' ')"
done
echo done
