#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
for cfg in "$@"; do
  echo "== chunk $cfg"
  SYZCOV_MR_CFG=0,1 SYZCOV_MR_CHUNK=$cfg timeout -k 10 120 python3 tools/kbench.py minimize --reps 2 2>&1 | grep "ms " || exit 1
done
