// synth.hip — counter-based synthetic corpus generator, written
// directly into HBM.  Integer-exact, so the CPU twin (oracle/synth_oracle.c)
// regenerates bit-identical inputs for parity checks and the CPU baseline
// without shipping tens of GB.
#include "common.h"

namespace syz {

// SYNTH_X86 (mode bit 1): an x86-like universe, neighbouring KCOV return
// addresses 5..14 bytes apart: PCs in pairs per 16-byte block, the first at
// 16m + a, the second 5 + b bytes later (a, b < 4, hashed per pair), so some
// pairs share an 8-byte block: kshift 2 and 2 keys per PC.  Otherwise one PC
// per 16-byte slot (kshift 4, a key per PC).
constexpr int SYNTH_UNIFORM = 1, SYNTH_X86 = 2;
__device__ __forceinline__ uint32_t synth_universe(uint64_t seed, uint32_t k, int mode = 0) {
    if (mode & SYNTH_X86) {
        const uint64_t h = splitmix64(seed ^ 0xA0761D6478BD642Full ^ (uint64_t)(k >> 1));
        return 0x81000000u + 16u * (k >> 1) + (uint32_t)(h & 3u) +
               (k & 1u) * (5u + (uint32_t)((h >> 2) & 3u));
    }
    const uint64_t h = splitmix64(seed ^ 0xA0761D6478BD642Full ^ (uint64_t)k);
    return 0x81000000u + 16u * k + (uint32_t)(h & 15u);
}

__global__ void synth_lens_kernel(uint64_t seed, uint64_t first, uint64_t n, uint32_t mean,
                                  uint32_t sigma, uint32_t *__restrict__ lens) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t base = splitmix64(seed ^ splitmix64((first + i) ^ 0x5851F42D4C957F2Dull));
        int64_t sum = 0;
#pragma unroll
        for (int t = 0; t < 3; t++) {
            const uint64_t h = splitmix64(base + (uint64_t)(t + 1) * 0x9E3779B97F4A7C15ull);
            sum += (int64_t)(h & 0xFFFF) + (int64_t)((h >> 16) & 0xFFFF) +
                   (int64_t)((h >> 32) & 0xFFFF) + (int64_t)(h >> 48);
        }
        const int64_t num = (int64_t)sigma * (sum - 6 * 65536) + 32768;
        const int64_t off = num >= 0 ? num / 65536 : -((-num + 65535) / 65536);
        int64_t L = (int64_t)mean + off;
        L = L < 1 ? 1 : (L > 65535 ? 65535 : L);
        lens[i] = (uint32_t)L;
    }
}

__global__ void synth_pcs_kernel(uint64_t seed, uint64_t first, uint64_t n,
                                 const uint64_t *__restrict__ off, uint32_t log2_space,
                                 int mode, uint32_t *__restrict__ pcs) {
    for (uint64_t i = blockIdx.x; i < n; i += gridDim.x) {
        const uint64_t base = splitmix64(seed ^ splitmix64((first + i) + 0x632BE59BD9B4E019ull));
        const uint64_t b = off[i], len = off[i + 1] - b;
        for (uint64_t j = threadIdx.x; j < len; j += blockDim.x) {
            const uint64_t h = splitmix64(base + (j + 1) * 0x9E3779B97F4A7C15ull);
            uint32_t k;
            if (mode & SYNTH_UNIFORM) {
                k = (uint32_t)(h >> (64 - log2_space));
            } else {
                // u = x / 2^32 (32 hash bits: every one of the 2^S keys is
                // reachable); k = floor(2^S u^3) = x^3 >> (96 - S), and
                // x^3 < 2^96 so that is the high 64 bits of x^2 * x >> (32 - S)
                const uint64_t x = h >> 32;
                k = (uint32_t)(__umul64hi(x * x, x) >> (32 - log2_space));
            }
            pcs[b + j] = synth_universe(seed, k, mode);
        }
    }
}

// C5 call records: CallID of record `first + i`, uniform over [0, ncalls)
__global__ void synth_callids_kernel(uint64_t seed, uint64_t first, uint64_t n, uint32_t ncalls,
                                     int32_t *__restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t h = splitmix64(seed ^ splitmix64((first + i) ^ 0xC2B2AE3D27D4EB4Full));
        out[i] = (int32_t)(((h >> 32) * (uint64_t)ncalls) >> 32);
    }
}

__global__ void synth_universe_kernel(uint64_t seed, uint32_t n, int mode,
                                      uint32_t *__restrict__ out) {
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x)
        out[k] = synth_universe(seed, k, mode);
}

// Streaming copy, 16 B per lane: the measured HBM peak the bench reports
// next to the 8 TB/s vendor figure (roofline.peak_measured).  Each workgroup
// copies whole contiguous 8 x 16 KB tiles (8 loads of 16 B per lane in flight
// before the first store) with non-temporal stores, so the written lines do
// not evict the lines being read.
constexpr int SC_THREADS = 1024, SC_U = 8;
typedef unsigned int sc_v4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(SC_THREADS) void stream_copy_kernel(const uint4 *__restrict__ src,
                                                                 uint4 *__restrict__ dst,
                                                                 uint64_t n4) {
    constexpr uint64_t TILE = (uint64_t)SC_THREADS * SC_U;
    const uint64_t ntile = n4 / TILE;
    for (uint64_t t = blockIdx.x; t < ntile; t += gridDim.x) {
        const uint64_t b = t * TILE + threadIdx.x;
        const sc_v4 *s4 = reinterpret_cast<const sc_v4 *>(src);
        sc_v4 *d4 = reinterpret_cast<sc_v4 *>(dst);
        sc_v4 v[SC_U];
#pragma unroll
        for (int u = 0; u < SC_U; u++) v[u] = s4[b + (uint64_t)u * SC_THREADS];
#pragma unroll
        for (int u = 0; u < SC_U; u++) __builtin_nontemporal_store(v[u], d4 + b + (uint64_t)u * SC_THREADS);
    }
    for (uint64_t i = ntile * TILE + (uint64_t)blockIdx.x * SC_THREADS + threadIdx.x; i < n4;
         i += (uint64_t)gridDim.x * SC_THREADS)
        dst[i] = src[i];
}

// The plain form (one 16-byte element per thread, one pass, default cache
// policy), the shape of the guide's float4 copy (MI355X_MICROARCH.md, HBM3E
// measured bandwidth): the bench reports the better of the two forms.
__global__ __launch_bounds__(256) void flat_copy_kernel(const uint4 *__restrict__ src,
                                                        uint4 *__restrict__ dst, uint64_t n4) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n4) dst[i] = src[i];
}

}  // namespace syz

using namespace syz;

extern "C" int syzcov_dev_copy_peak(const void *src, void *dst, size_t nbytes, int form,
                                    void *stream) {
    if (!src || !dst || nbytes % 16 || ((uintptr_t)src | (uintptr_t)dst) % 16 || form < 0 ||
        form > 1)
        return SYZCOV_EINVAL;
    if (nbytes == 0) return 0;
    const uint64_t n4 = nbytes / 16;
    if (form == 0)
        hipLaunchKernelGGL(stream_copy_kernel, dim3(256 * 2), dim3(SC_THREADS), 0,
                           (hipStream_t)stream, (const uint4 *)src, (uint4 *)dst, n4);
    else
        hipLaunchKernelGGL(flat_copy_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0,
                           (hipStream_t)stream, (const uint4 *)src, (uint4 *)dst, n4);
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" int syzcov_dev_stream_copy(const void *src, void *dst, size_t nbytes, void *stream) {
    if (!src || !dst || nbytes % 16 || ((uintptr_t)src | (uintptr_t)dst) % 16) return SYZCOV_EINVAL;
    if (nbytes == 0) return 0;
    hipLaunchKernelGGL(stream_copy_kernel, dim3(256 * 2), dim3(SC_THREADS), 0, (hipStream_t)stream,
                       (const uint4 *)src, (uint4 *)dst, (uint64_t)(nbytes / 16));
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" int syzcov_dev_synth_universe_mode(uint64_t seed, uint32_t log2_space, int mode,
                                              uint32_t *out, void *stream) {
    if (!out || log2_space < 1 || log2_space > 26 || mode < 0 || mode > 3) return SYZCOV_EINVAL;
    const uint32_t n = 1u << log2_space;
    hipLaunchKernelGGL(synth_universe_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0,
                       (hipStream_t)stream, seed, n, mode, out);
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" int syzcov_dev_synth_universe(uint64_t seed, uint32_t log2_space, uint32_t *out,
                                         void *stream) {
    return syzcov_dev_synth_universe_mode(seed, log2_space, 0, out, stream);
}

extern "C" int syzcov_dev_synth_lens(uint64_t seed, uint64_t first, size_t n, uint32_t mean,
                                     uint32_t sigma, uint32_t *lens, void *stream) {
    if (n == 0) return 0;
    if (!lens) return SYZCOV_EINVAL;
    hipLaunchKernelGGL(synth_lens_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0,
                       (hipStream_t)stream, seed, first, (uint64_t)n, mean, sigma, lens);
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" int syzcov_dev_synth_pcs(uint64_t seed, uint64_t first, size_t n, const uint64_t *off,
                                    uint32_t log2_space, int mode, uint32_t *pcs,
                                    void *stream) {
    if (n == 0) return 0;
    if (!off || !pcs || log2_space < 1 || log2_space > 26 || mode < 0 || mode > 3)
        return SYZCOV_EINVAL;
    hipLaunchKernelGGL(synth_pcs_kernel, dim3(grid_for(n, 1, 16384)), dim3(256), 0,
                       (hipStream_t)stream, seed, first, (uint64_t)n, off, log2_space, mode,
                       pcs);
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" int syzcov_dev_synth_callids(uint64_t seed, uint64_t first, size_t n, uint32_t ncalls,
                                        int32_t *out, void *stream) {
    if (n == 0) return 0;
    if (!out || ncalls == 0) return SYZCOV_EINVAL;
    hipLaunchKernelGGL(synth_callids_kernel, dim3(grid_for(n, 256, 4096)), dim3(256), 0,
                       (hipStream_t)stream, seed, first, (uint64_t)n, ncalls, out);
    SYZ_LAUNCH_CHECK();
    return 0;
}
