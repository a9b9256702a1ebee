#!/bin/bash
# Round-4 GPU call C: minimize chunk-cap sweep (C2, key mode) + the copy-peak forms.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04c; mkdir -p $o
for v in base mc131072 mc262144 mc524288; do
  if [ $v = base ]; then e=""; else e="SYZCOV_LIB=$PWD/syzkaller_amd/variants/$v.so"; fi
  env $e timeout -k 10 150 python -u tools/kbench.py minimize --keys --reps 5 > $o/min_$v.log 2>&1 || { tail -5 $o/min_$v.log; exit 1; }
  echo "$v: $(tail -3 $o/min_$v.log | awk '{print $2}' | tr '\n' ' ')"
done
timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0, '.')
import torch, bench
print(bench.stream_peak(torch.device('cuda', 0)))
" > $o/peak.log 2>&1; tail -2 $o/peak.log
echo done
