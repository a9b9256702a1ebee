#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
for cfg in "0,0" "0,3" "0,4" "0,6"; do
  echo "== cfg $cfg"
  SYZCOV_MR_CFG=$cfg timeout -k 10 120 python3 tools/kbench.py minimize --reps 3 2>&1 | grep "ms " || exit 1
done
