// DRAM locality probe: read a 528 MB buffer as random chunks of C bytes
// (one wave per chunk, 16 B per lane) vs sequential; reports GB/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
#include <random>
__global__ __launch_bounds__(256) void rd(const uint4 *__restrict__ a, const uint32_t *__restrict__ starts,
                                          uint32_t nchunks, uint32_t vec_per_chunk, uint32_t *out) {
    uint32_t acc = 0;
    const uint32_t l = threadIdx.x & 63;
    for (uint32_t c = blockIdx.x * 4 + (threadIdx.x >> 6); c < nchunks; c += gridDim.x * 4) {
        const uint4 *p = a + starts[c];
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t i = u * 64 + l;
            v[u] = i < vec_per_chunk ? p[i] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < 4; u++) acc += v[u].x ^ v[u].w;
    }
    if (acc == 0x9999) out[0] = acc;
}
int main() {
    const size_t bytes = 528ull << 20;
    uint4 *a;
    uint32_t *out, *dst;
    hipMalloc(&a, bytes);
    hipMalloc(&out, 4);
    hipMemset(a, 1, bytes);
    std::mt19937_64 rng(1);
    for (uint32_t C : {256u, 1024u, 2048u, 4096u, 16384u}) {
        const uint32_t vpc = C / 16;
        if (vpc > 256) continue;
        const uint32_t n = bytes / C;
        std::vector<uint32_t> st(n);
        for (uint32_t i = 0; i < n; i++) st[i] = i * vpc;
        for (int mode = 0; mode < 2; mode++) {
            if (mode == 1) std::shuffle(st.begin(), st.end(), rng);
            hipMalloc(&dst, n * 4);
            hipMemcpy(dst, st.data(), n * 4, hipMemcpyHostToDevice);
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            rd<<<4096, 256>>>(a, dst, n, vpc, out);
            hipEventRecord(e0);
            for (int it = 0; it < 5; it++) rd<<<4096, 256>>>(a, dst, n, vpc, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            printf("chunk %6u B %s: %.0f GB/s\n", C, mode ? "random    " : "sequential", 5.0 * bytes / (ms * 1e-3) / 1e9);
            hipFree(dst);
        }
    }
    return 0;
}
