#!/bin/bash
# newcov bench lines: LDS pass (default choice), probe pass, window mode
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ncb
for cfg in "lds:" "probe:" "auto:--no-universe"; do
  p=${cfg%%:*}; a=${cfg#*:}
  env SYZCOV_NEWCOV_PATH=$([ $p = auto ] && echo "" || echo $p) timeout -k 10 300 python -u bench.py --workload newcov --steps 20 --warmup 5 --no-cpu $a > gpurun_out/ncb/$p.json 2> gpurun_out/ncb/$p.err || { tail -20 gpurun_out/ncb/$p.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ncb/$p.json'));print('$p $a', round(d['ms_per_step'],4), d['phases_ms'], round(d['roofline']['frac'],3))"
done
