#!/bin/bash
# Bench lines for A/B probes: each "name:env-assignments:bench-args" entry
# runs bench.py once (no CPU baseline) and prints its phases.
#   tools/gpu_probe.sh OUTDIR "key::" "nomem:SYZCOV_LIB=\$PWD/syzkaller_amd/variants/nomem.so:" ...
set -o pipefail
export TMPDIR=/tmp
o=${1:-gpurun_out/probe}; shift
mkdir -p $o
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; envs=${rest%%:*}; args=${rest#*:}
  env $(eval echo $envs) timeout -k 10 300 python -u bench.py --no-cpu --steps ${STEPS:-10} --warmup 3 $args \
      > $o/$name.json 2> $o/$name.err
  rc=$?
  if [ $rc -ne 0 ]; then tail -15 $o/$name.err; case $rc in 124|134|137|139) echo "fatal rc=$rc"; exit 1;; esac; fi
  grep -q "illegal memory access\|HSA_STATUS_ERROR\|Memory access fault" $o/$name.err && { echo "GPU fault in $name"; exit 1; }
  python3 -c "import json; d=json.load(open('$o/$name.json')); print('$name', round(d['ms_per_step'],4), d.get('phases_ms'), round(d['roofline']['frac'],3), d.get('results',{}).get('kept'), d.get('results',{}).get('union'))"
done
exit 0
