#!/bin/bash
# the concurrent-callers ASan harness alone (plus a HIP-only memory probe)
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
timeout -k 10 100 ./tests/native/build/abi_stress_asan 32 1 hip 2>&1 | tail -4
timeout -k 10 200 ./tests/native/build/abi_stress_asan 32 8 2>&1 | tail -6
