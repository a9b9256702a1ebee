#!/bin/bash
# Round-4 GPU call D: grouped minimizeCorpus engine + raw-cover drop-in digests,
# minimize chunk-cap sweep, copy-peak forms, canon wave-time counters.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04d; mkdir -p $o
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  "tests/test_gpu_manager.py::test_minimize_corpus_engine_size" tests/test_gpu_manager.py \
  "tests/test_gpu_fullsize.py::test_c2_dropin_raw_covers_digest" \
  "tests/test_gpu_fullsize.py::test_c2_minimize_corpus_293_groups_digest" > $o/pytest.log 2>&1
rc=$?; tail -4 $o/pytest.log; grep -q "illegal memory access\|HSA_STATUS_ERROR\|Memory access fault" $o/pytest.log && { echo "GPU fault"; exit 1; }
fatal $rc pytest
for v in base mc131072 mc262144 mc524288; do
  if [ $v = base ]; then e=""; else e="SYZCOV_LIB=$PWD/syzkaller_amd/variants/$v.so"; fi
  env $e timeout -k 10 150 python -u tools/kbench.py minimize --keys --reps 5 > $o/min_$v.log 2>&1 || { tail -5 $o/min_$v.log; exit 1; }
  echo "$v: $(tail -3 $o/min_$v.log | awk '{print $2}' | tr '\n' ' ')"
done
timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0, '.')
import torch, bench
print(bench.stream_peak(torch.device('cuda', 0)))
" > $o/peak.log 2>&1; tail -1 $o/peak.log
timeout -k 10 400 bash tools/pmc_canon_r04.sh $o/pmc_canon || exit 1
echo done
