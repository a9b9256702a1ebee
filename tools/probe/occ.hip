// occupancy probe: how many 1024-thread workgroups of a given LDS size share a CU
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(1024) void k(int *out, int spin) {
    extern __shared__ unsigned s[];
    __shared__ unsigned st[2048];
    s[threadIdx.x] = threadIdx.x;
    st[threadIdx.x] = 1;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin) {}
    if (threadIdx.x == 0) out[blockIdx.x] = s[5] + st[7];
}
int main() {
    int *d;
    hipMalloc(&d, 1 << 20);
    for (int dyn : {32768, 57344, 65536, 69632, 73728}) {
        hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, dyn);
        int nb = 0;
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, 1024, dyn);
        // wall time of 1024 blocks x 20 us spin: 256 CUs -> 4 rounds at 1/CU, 2 at 2/CU
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipLaunchKernelGGL(k, dim3(1024), dim3(1024), dyn, 0, d, 2000);
        hipEventRecord(a);
        hipLaunchKernelGGL(k, dim3(1024), dim3(1024), dyn, 0, d, 2000);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        printf("dyn %6d + 8 KB static: occupancy API %d blocks/CU, 1024 blocks x 20us: %.1f us\n", dyn, nb, ms * 1000);
    }
    return 0;
}
