#!/bin/bash
# Round-4 first GPU call: new tests, the C3 two-step rehearsal, the --gpus 2
# launcher on the one-GPU box, and the minimize range sweep (time + FETCH).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04a; mkdir -p $o
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 560 --timeout-method thread -m gpu \
  tests/test_gpu_engine.py tests/test_gpu_keys.py "tests/test_gpu_cover.py::test_minimize_engine_with_caller_order" tests/test_gpu_corpus_abi.py "tests/test_gpu_fullsize.py::test_world8_rehearsal_c3" > $o/pytest.log 2>&1
rc=$?; tail -5 $o/pytest.log; grep -q "illegal memory access\|HSA_STATUS_ERROR\|Memory access fault" $o/pytest.log && { echo "GPU fault"; exit 1; }
fatal $rc pytest
timeout -k 10 400 python -u bench.py --gpus 2 --steps 3 --warmup 1 > $o/bench2.json 2> $o/bench2.err
rc=$?; cat $o/bench2.json; [ $rc -ne 0 ] && tail -20 $o/bench2.err; fatal $rc bench2
for L in 17 18 19 20 21 22; do
  timeout -k 10 120 python -u tools/kbench.py minimize --keys --log2-space $L --reps 4 > $o/kb$L.log 2>&1 || { tail -5 $o/kb$L.log; exit 1; }
  echo "L=$L $(tail -1 $o/kb$L.log)"
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/f$L -o run -- python3 tools/kbench.py minimize --keys --log2-space $L --reps 1 > $o/f$L.log 2>&1 || { tail -3 $o/f$L.log; exit 1; }
  python3 tools/kernel_fetch.py $o/f$L prep_kernel > $o/f$L.txt && head -8 $o/f$L.txt
done
for v in base noconf; do
  if [ $v = base ]; then e=""; else e="SYZCOV_LIB=$PWD/syzkaller_amd/variants/$v.so"; fi
  env $e timeout -k 10 120 python -u tools/kbench.py canon --keys --reps 4 > $o/canon_$v.log 2>&1 || { tail -5 $o/canon_$v.log; exit 1; }
  echo "canon $v: $(tail -2 $o/canon_$v.log | head -1)"
done
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > $o/bench.json 2> $o/bench.err
rc=$?; cat $o/bench.json; [ $rc -ne 0 ] && tail -20 $o/bench.err; fatal $rc bench
echo done
