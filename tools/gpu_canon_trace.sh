#!/bin/bash
# per-class canon kernel times: 2-pass key sort vs 3-pass window-offset sort (rocprofv3 kernel trace)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/ckt; mkdir -p $o
for k in 1 0; do
  SYZCOV_CANON_KEY2=$k timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/t$k -o run -- python3 bench.py --no-cpu --steps 5 --warmup 1 > $o/t$k.log 2>&1 || { tail -5 $o/t$k.log; exit 1; }
  echo "== key2=$k"; python3 tools/trace_summary.py $o/t$k | grep -E "canon|bin_kernel" | head -12
done
