#!/bin/bash
# Round-4 GPU call Z: C5 candidate pass without the membership gathers
# (timing probe builds variants/nomem*.so) against the product library.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04z; mkdir -p $o
for v in ${VARIANTS:-base nomem nomem8}; do
  if [ $v = base ]; then unset SYZCOV_LIB; else export SYZCOV_LIB=$PWD/syzkaller_amd/variants/$v.so; fi
  timeout -k 10 300 python -u bench.py --workload newcov --steps 10 --warmup 3 --no-cpu > $o/nc_$v.json 2> $o/nc_$v.err || { tail -5 $o/nc_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/nc_$v.json')); print('$v', round(d['ms_per_step'],4), d['phases_ms'])"
done
