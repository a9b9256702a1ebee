// Probe: cycles per wave-instruction of LDS primitives on gfx950, with
// random addresses over a 512-entry table, 1..16 waves per CU.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

template <int OP>
__global__ void probe(uint32_t iters, uint32_t bins, unsigned long long *cyc, uint32_t *sink) {
    __shared__ uint32_t tab[16][2048];
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63;
    uint32_t *t = tab[w];
    for (uint32_t q = l; q < 2048; q += 64) t[q] = q;
    __syncthreads();
    uint32_t a[16];
    for (int i = 0; i < 16; i++) a[i] = mix(l * 131 + i * 7919 + blockIdx.x) % bins;
    uint32_t acc = 0;
    __syncthreads();
    const long long t0 = clock64();
    for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const uint32_t ad = (a[i] + it) & (bins - 1);
            if (OP == 0) acc += atomicAdd(&t[ad], 1u);          // ds_add_rtn
            if (OP == 1) atomicAdd(&t[ad], 1u);                 // ds_add (no return)
            if (OP == 2) t[ad] = acc + i;                       // ds_write random
            if (OP == 3) acc += t[ad];                          // ds_read random
            if (OP == 4) acc += t[(it * 64 + l + i * 64) & 2047]; // ds_read linear
            if (OP == 5) t[(it * 64 + l + i * 64) & 2047] = acc;  // ds_write linear
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    const long long t1 = clock64();
    if (l == 0) atomicAdd(cyc, (unsigned long long)(t1 - t0));
    if (acc == 0x12345678) sink[0] = acc;
}

int main() {
    unsigned long long *dc; uint32_t *ds;
    (void)hipMalloc(&dc, 8); (void)hipMalloc(&ds, 4);
    const char *names[] = {"ds_add_rtn rand", "ds_add rand", "ds_write rand", "ds_read rand",
                           "ds_read lin", "ds_write lin"};
    for (int waves : {1, 4, 8, 16}) {
        for (uint32_t bins : {512u, 2048u}) {
            for (int op = 0; op < 6; op++) {
                (void)hipMemset(dc, 0, 8);
                const uint32_t iters = 256;
                dim3 g(256), b(64 * waves);
                switch (op) {
                case 0: hipLaunchKernelGGL(probe<0>, g, b, 0, 0, iters, bins, dc, ds); break;
                case 1: hipLaunchKernelGGL(probe<1>, g, b, 0, 0, iters, bins, dc, ds); break;
                case 2: hipLaunchKernelGGL(probe<2>, g, b, 0, 0, iters, bins, dc, ds); break;
                case 3: hipLaunchKernelGGL(probe<3>, g, b, 0, 0, iters, bins, dc, ds); break;
                case 4: hipLaunchKernelGGL(probe<4>, g, b, 0, 0, iters, bins, dc, ds); break;
                case 5: hipLaunchKernelGGL(probe<5>, g, b, 0, 0, iters, bins, dc, ds); break;
                }
                unsigned long long h = 0;
                (void)hipMemcpy(&h, dc, 8, hipMemcpyDeviceToHost);
                // clock64 = s_memtime (constant 100 MHz on gfx9?) -> report raw ticks per instr per wave
                double per = (double)h / (256.0 * waves) / (iters * 16.0);
                // CU-level: waves share one LDS: CU ticks per instr = per / waves
                printf("waves/CU=%2d bins=%4u %-16s ticks/instr/wave=%8.3f  CU ticks/instr=%7.3f\n",
                       waves, bins, names[op], per, per / waves);
            }
        }
    }
    return 0;
}
