// probe: the DPP wave scan (common.h) against a serial scan, random inputs,
// partial EXEC masks excluded (every caller runs it with the whole wave)
#include "../../syzkaller_amd/csrc/common.h"
#include <cstdio>
#include <vector>
__global__ void k(const uint32_t *in, uint32_t *out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    out[i] = syz::wave_incl_scan(in[i]);
}
int main() {
    const int n = 64 * 4096;
    std::vector<uint32_t> h(n), r(n);
    uint64_t s = 88172645463325252ull;
    for (auto &x : h) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; x = (uint32_t)(s % 100000); }
    uint32_t *di, *dout;
    hipMalloc(&di, n * 4); hipMalloc(&dout, n * 4);
    hipMemcpy(di, h.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, di, dout, n);
    hipMemcpy(r.data(), dout, n * 4, hipMemcpyDeviceToHost);
    long bad = 0;
    for (int w = 0; w < n / 64; w++) {
        uint32_t acc = 0;
        for (int l = 0; l < 64; l++) { acc += h[w * 64 + l]; bad += r[w * 64 + l] != acc; }
    }
    printf("scan_dpp mismatches: %ld\n", bad);
    return bad != 0;
}
