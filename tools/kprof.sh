#!/bin/bash
# kernel trace + a few PMC passes of tools/kbench.py on the GPU box
#   tools/kprof.sh <tag> <what> [pmc-set ...]   pmc-set = comma-free counter list in quotes
set -o pipefail
tag=$1; what=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
    python3 tools/kbench.py $what --reps 3 > $out/trace.log 2>&1 || { tail -20 $out/trace.log; exit 1; }
grep -h "ms " $out/trace.log || true
i=0
for pmc in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d $out/pmc$i -o run -- \
      python3 tools/kbench.py $what --reps 1 > $out/pmc$i.log 2>&1 || { tail -5 $out/pmc$i.log; exit 1; }
done
echo kprof_done
