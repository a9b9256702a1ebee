#!/bin/bash
# Host-side ASan + UBSan build of the C-ABI (device code uninstrumented: GPU
# sanitizers are not available here) and the concurrent-callers harness
# tests/native/abi_stress.cc, linked with the CPU oracle as the checker.
# Output: tests/native/build/abi_stress_asan (run by tests/test_sanitize.py, GPU).
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
B="$ROOT/tests/native/build"
mkdir -p "$B/obj"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all"
FLAGS="--offload-arch=gfx950 -O2 -g -fPIC -std=c++17 -ffp-contract=off -w"
OBJS=()
for f in "$ROOT"/syzkaller_amd/csrc/*.hip "$ROOT"/syzkaller_amd/csrc/*.cc; do
    o="$B/obj/$(basename "$f").o"
    if [ ! -f "$o" ] || [ "$f" -nt "$o" ] || [ "$ROOT/syzkaller_amd/csrc/common.h" -nt "$o" ] || [ "$ROOT/include/syzcov.h" -nt "$o" ]; then
        "$HIPCC" $FLAGS $SAN -c "$f" -o "$o" &
    fi
    OBJS+=("$o")
done
wait
for f in cover_oracle gosort_oracle; do
    gcc -O2 -fPIC -std=c11 -ffp-contract=off -c "$ROOT/oracle/$f.c" -o "$B/obj/$f.o"
    OBJS+=("$B/obj/$f.o")
done
"$HIPCC" $FLAGS $SAN -c "$ROOT/tests/native/abi_stress.cc" -o "$B/obj/abi_stress.o"
"$HIPCC" --offload-arch=gfx950 $SAN -o "$B/abi_stress_asan" "$B/obj/abi_stress.o" "${OBJS[@]}" -lpthread
echo "built $B/abi_stress_asan"
