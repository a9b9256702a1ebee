// Probe: xperm<M>(lane) must equal lane ^ M for every mask the bitonic
// canonicalizer uses.
#include <stdio.h>
#include "../../syzkaller_amd/csrc/xperm.h"
using namespace syz;

__global__ void k(uint32_t *bad) {
    const uint32_t l = __lane_id();
    uint32_t b = 0;
#define CHK(M) b |= (xperm<M>(l * 7 + 3) != ((l ^ M) * 7 + 3)) << __COUNTER__;
    CHK(1) CHK(2) CHK(3) CHK(4) CHK(7) CHK(8) CHK(15) CHK(16) CHK(31) CHK(32) CHK(63)
    atomicOr(bad, b);
}

int main() {
    uint32_t *d, h = 0;
    (void)hipMalloc(&d, 4);
    (void)hipMemset(d, 0, 4);
    hipLaunchKernelGGL(k, dim3(4), dim3(256), 0, 0, d);
    (void)hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
    const int ms[] = {1, 2, 3, 4, 7, 8, 15, 16, 31, 32, 63};
    for (int i = 0; i < 11; i++) printf("mask %2d: %s\n", ms[i], (h >> i) & 1 ? "WRONG" : "ok");
    return h != 0;
}
