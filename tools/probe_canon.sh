#!/bin/bash
# canon phase cost probes (SYZCOV_CANON_PROBE: 1 load, 2 +pass 0, 3 +all passes, 0 full)
set -o pipefail
export TMPDIR=/tmp
for p in 1 2 3 0; do
  echo "== probe $p"
  SYZCOV_CANON_PROBE=$p timeout -k 10 120 python3 tools/kbench.py canon --reps 2 2>&1 | grep "ms " || exit 1
done
