#!/bin/bash
# Round-4 GPU call R: cover_dedup (dedup.hip) per-class kernels: parity,
# micro-bench at three buffer-length classes, kernel trace.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04r; mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dedup.py > $o/pytest.log 2>&1
rc=$?; tail -12 $o/pytest.log; [ $rc -ne 0 ] && exit 1
for m in 512 1400 2048; do
  timeout -k 10 200 python -u tools/kbench.py dedup --inputs 65536 --mean $m --sigma $((m/4)) --reps 3 > $o/kb_$m.txt 2>&1 || exit 1
done
timeout -k 10 300 python -u tools/kbench.py dedup --inputs 1000000 --reps 3 > $o/kb_1m.txt 2>&1 || exit 1
grep -h dedup $o/kb_*.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$o/prof -o dd -- python3 $GRAFT_REPO_ROOT/tools/kbench.py dedup --inputs 1000000 --reps 3 > $GRAFT_REPO_ROOT/$o/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && f=$(find $o/prof -name "*kernel_stats.csv" | head -1) && head -8 $f
