#!/bin/bash
# minimize pass-1 tuning sweep (SYZCOV_MR_CFG variants), one process per setting
set -o pipefail
export TMPDIR=/tmp
for cfg in "$@"; do
  echo "== cfg $cfg"
  SYZCOV_MR_CFG=$cfg timeout -k 10 120 python3 tools/kbench.py minimize --reps 2 2>&1 | grep "ms " || exit 1
done
