#!/bin/bash
# Round-4 GPU call L: pad-free canon key kernel (every lane loads 4 words of its segment; no pad fills, no gap) — parity, then
# timing against the previous build (variants/g.so).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04l; mkdir -p $o
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_keys.py "tests/test_gpu_fullsize.py::test_c2_fullsize_digest" \
  "tests/test_gpu_fullsize.py::test_c3_fullsize_digest" tests/test_gpu_engine.py tests/test_gpu_corpus_abi.py tests/test_gpu_cover.py > $o/pytest.log 2>&1
rc=$?; tail -4 $o/pytest.log; grep -q "illegal memory access\|HSA_STATUS_ERROR\|Memory access fault" $o/pytest.log && { echo "GPU fault"; exit 1; }
fatal $rc pytest
[ $rc -ne 0 ] && { grep -E "^E " $o/pytest.log | head -10; exit 1; }
for v in g new g new; do
  if [ $v = new ]; then e=""; else e="SYZCOV_LIB=$PWD/syzkaller_amd/variants/$v.so"; fi
  env $e timeout -k 10 150 python -u tools/kbench.py canon --keys --reps 5 > $o/canon_$v.log 2>&1 || { tail -5 $o/canon_$v.log; exit 1; }
  echo "canon $v: $(tail -3 $o/canon_$v.log | awk '{print $2}' | tr '\n' ' ')"
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-c3 --no-dropin --no-cpu > $o/bench.json 2> $o/bench.err
rc=$?; [ $rc -ne 0 ] && tail -5 $o/bench.err; fatal $rc bench
python3 -c "import json; d=json.load(open('$o/bench.json')); print(round(d['ms_per_step'],4), d['phases_ms'], round(d['roofline']['frac'],4), d['results'])"
echo done
