#!/bin/bash
# Minimize chunk schedule sweep (first chunk, growth) with the default pass-1
# kernel: tools/sweep_chunk.sh 64,4 1024,4 ...  (every schedule is exact)
set -o pipefail
export TMPDIR=/tmp
for cfg in "$@"; do
  echo "== chunk $cfg"
  SYZCOV_MR_CHUNK=$cfg timeout -k 10 120 python3 tools/kbench.py minimize --reps 3 2>&1 | grep "ms " || exit 1
done
