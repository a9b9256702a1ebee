#!/bin/bash
# newcov iteration: parity tests of both candidate passes, then kernel stats
set -o pipefail
export TMPDIR=/tmp
./tools/gpu_tests_all.sh "newcov or new_inputs or exec_output or sentinel or test_gpu_manager or triage or add_inputs" || exit 1
./tools/gpu_nctrace.sh "$@" || exit 1
python3 tools/nc_steps.py gpurun_out/nct
