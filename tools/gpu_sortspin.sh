#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
for v in 0 1 0 1; do echo "spin=$v"; SYZCOV_SORT_SPIN=$v timeout -k 10 120 python3 tools/kbench.py order --reps 6 2>&1 | tail -4 || exit 1; done
for v in 0 1; do SYZCOV_SORT_SPIN=$v timeout -k 10 200 python -u bench.py --no-cpu --steps 10 --warmup 3 > /tmp/b.json 2>/dev/null || exit 1; python3 -c "import json; d=json.load(open('/tmp/b.json')); print('spin=$v', round(d['ms_per_step'],3), d['phases_ms'])"; done
