// Probe: are same-address LDS ds_add_rtn results ordered by lane within one
// wave instruction?  Prints violation counts per digit-range D.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

__global__ void probe(uint32_t D, uint32_t trials, unsigned long long *viol) {
    __shared__ uint32_t hist[4][512];
    __shared__ uint32_t ret[4][64];
    __shared__ uint32_t dig[4][64];
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63;
    unsigned long long v = 0;
    for (uint32_t t = 0; t < trials; t++) {
        for (uint32_t q = l; q < 512; q += 64) hist[w][q] = 0;
        __builtin_amdgcn_wave_barrier();
        uint32_t s = mix(blockIdx.x * 7919u + w * 104729u + t * 15485863u);
        for (int row = 0; row < 8; row++) {
            uint32_t d = mix(s + row * 64 + l) % D;
            uint32_t r = atomicAdd(&hist[w][d], 1u);
            ret[w][l] = r;
            dig[w][l] = d;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            // lane l checks all lower lanes with the same digit
            for (uint32_t j = 0; j < l; j++)
                if (dig[w][j] == d && ret[w][j] > r) v++;
            __builtin_amdgcn_wave_barrier();
        }
    }
    atomicAdd(viol, v);
}

int main() {
    unsigned long long *dv;
    hipMalloc(&dv, 8);
    uint32_t Ds[] = {1, 2, 3, 8, 64, 512};
    for (uint32_t D : Ds) {
        hipMemset(dv, 0, 8);
        hipLaunchKernelGGL(probe, dim3(1024), dim3(256), 0, 0, D, 64u, dv);
        unsigned long long h = 0;
        hipMemcpy(&h, dv, 8, hipMemcpyDeviceToHost);
        printf("D=%u violations=%llu\n", D, h);
    }
    return 0;
}
