#!/bin/bash
# rocprofv3 evidence for the C4 prio bench: kernel stats, MFMA busy counters,
# HBM bytes (separate passes) -> gpurun_out/prof_prio
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/prof_prio; mkdir -p $out
timeout -k 10 300 python3 bench.py --workload prio > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
    python3 bench.py --workload prio --steps 3 --warmup 1 --no-cpu > $out/trace.log 2>&1 || { tail -20 $out/trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_I8 GRBM_GUI_ACTIVE --output-format csv -d $out/pmc1 -o run -- \
    python3 bench.py --workload prio --steps 1 --warmup 0 --no-cpu > $out/pmc1.log 2>&1 || { tail -5 $out/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- \
    python3 bench.py --workload prio --steps 1 --warmup 0 --no-cpu > $out/fetch.log 2>&1 || { tail -5 $out/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- \
    python3 bench.py --workload prio --steps 1 --warmup 0 --no-cpu > $out/write.log 2>&1 || { tail -5 $out/write.log; exit 1; }
python3 tools/pmc_summary.py $out > $out/summary.txt 2>&1 || true
grep -A8 "prio_gemm\|prio_build" $out/summary.txt | head -40
