# A/B of canon variants (kbench canon --keys), after a correctness subset
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/e5; mkdir -p $o
: timeout -k 10 400 python -u -m pytest tests/test_gpu_keys.py tests/test_gpu_corpus_abi.py -m gpu -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1; rc=$?
tail -3 $o/pytest.log
rc=0; case $rc in 0) ;; *) grep -E "^E |FAIL" $o/pytest.log | head; exit 1;; esac
for v in vpipe vdesc vpipe; do
  if [ $v = main ]; then lib=""; else lib="SYZCOV_LIB=$PWD/syzkaller_amd/variants/$v.so"; fi
  env $lib timeout -k 10 200 python -u tools/kbench.py canon --keys --reps 5 > $o/canon_$v.txt 2>&1 || { tail $o/canon_$v.txt; exit 1; }
  echo $v $(grep canon: $o/canon_$v.txt | tail -3 | awk '{print $2}')
done
