#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
for alg in "$@"; do
  echo "== canon $alg"
  SYZCOV_CANON=$alg timeout -k 10 120 python3 tools/kbench.py canon --reps 3 2>&1 | grep "ms " || exit 1
done
