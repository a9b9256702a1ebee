#!/bin/bash
# Round-4 GPU call P: cover_dedup (dedup.hip) parity, its micro-bench and
# kernel trace; the bench.py launcher rehearsal (2 ranks on GPU 0, gloo).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04p; mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dedup.py > $o/pytest.log 2>&1
rc=$?; tail -12 $o/pytest.log; [ $rc -ne 0 ] && exit 1
timeout -k 10 200 python -u tools/kbench.py dedup --inputs 65536 --reps 5 > $o/kb_64k.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/kbench.py dedup --inputs 1000000 --reps 5 > $o/kb_1m.txt 2>&1 || exit 1
cat $o/kb_64k.txt $o/kb_1m.txt | grep dedup
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$o/prof -o dd -- python3 $GRAFT_REPO_ROOT/tools/kbench.py dedup --inputs 1000000 --reps 3 > $GRAFT_REPO_ROOT/$o/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && find $o/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -5 {}'
timeout -k 10 500 python -u bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu --no-dropin > $o/bench2.json 2> $o/bench2.err
rc=$?; tail -3 $o/bench2.err; [ $rc -ne 0 ] && exit 1
wc -l $o/bench2.json
python3 -c "import json; d=json.load(open('$o/bench2.json')); print(d['n_gpus'], d.get('rccl_ranks'), d.get('backend'), round(d['ms_per_step'],3), d['results'])"
