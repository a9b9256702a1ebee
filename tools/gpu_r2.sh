#!/bin/bash
# manager/newcov GPU pass: new parity tests, C5 bench line, its kernel stats
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r01d}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_manager.py tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread -k "manager or newcov or minimize_corpus or new_input or universe" > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
timeout -k 10 300 python3 bench.py --workload newcov > $out/newcov.json 2> $out/newcov.err || { tail -20 $out/newcov.err; exit 1; }
cat $out/newcov.json
timeout -k 10 300 python3 bench.py --workload newcov --universe --no-cpu > $out/newcov_universe.json 2> $out/newcov_universe.err || { tail -20 $out/newcov_universe.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_newcov -o run -- python3 bench.py --workload newcov --no-cpu --steps 3 --warmup 1 > $out/prof_newcov.log 2>&1 || { tail -20 $out/prof_newcov.log; exit 1; }
find $out/prof_newcov -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200 | head -20
