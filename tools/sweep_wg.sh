#!/bin/bash
# Minimize PCs-per-workgroup sweep (every value is exact): tools/sweep_wg.sh 65536 131072 ...
set -o pipefail
export TMPDIR=/tmp
for v in "$@"; do
  echo "== wg $v"
  SYZCOV_MR_WG=$v timeout -k 10 120 python3 tools/kbench.py minimize --reps 3 2>&1 | grep "ms " || exit 1
done
