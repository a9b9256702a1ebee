#!/bin/bash
# newcov parity tests (both passes) + LDS-pass timing probes
set -o pipefail
export TMPDIR=/tmp
./tools/gpu_tests_all.sh "newcov or new_inputs or exec_output or sentinel or test_gpu_manager or triage or add_inputs" || exit 1
DBGS="${DBGS:-0 1 2}" ./tools/gpu_ncdbg.sh
