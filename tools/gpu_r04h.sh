#!/bin/bash
# Round-4 GPU call H: non-temporal stream loads, A/B against this build —
# C5 (newcov PC stream, variants/nt.so: the membership table keeps its L2
# share) and Minimize pass 1 (variants/mrnt.so).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04h; mkdir -p $o
V=$PWD/syzkaller_amd/variants
for v in def nt def nt; do
  if [ $v = def ]; then e=""; else e="SYZCOV_LIB=$V/$v.so"; fi
  env $e timeout -k 10 240 python -u bench.py --workload newcov --steps 20 --warmup 5 --no-cpu > $o/c5_$v.json 2> $o/c5_$v.err || { tail -5 $o/c5_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/c5_$v.json')); print('c5 $v', round(d['ms_per_step'],4), d['results']['new_records_per_batch'][:4])"
done
for v in def mrnt def mrnt; do
  if [ $v = def ]; then e=""; else e="SYZCOV_LIB=$V/$v.so"; fi
  env $e timeout -k 10 150 python -u tools/kbench.py minimize --keys --reps 5 > $o/min_$v.log 2>&1 || { tail -5 $o/min_$v.log; exit 1; }
  echo "min $v: $(tail -3 $o/min_$v.log | awk '{print $2}' | tr '\n' ' ')"
done
echo done
