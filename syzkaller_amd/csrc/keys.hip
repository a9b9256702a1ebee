// keys.hip — the engine's dense key space over a registered PC universe.
//
// The manager knows every PC the kernel can report: the call sites of
// __sanitizer_cov_trace_pc (allCoverPCs, syz-manager/cover.go:57-69).  With
// kshift = the largest shift that keeps that universe collision-free
// (no two universe PCs share pc >> kshift) and kbase = U[0] >> kshift,
//     key(pc) = (pc >> kshift) - kbase
// is injective on the universe and maps it onto [0, nkeys): a dense key space
// computed with a shift and a subtract, no dictionary lookup (a per-PC
// lookup is a random access, which a 2 G-PC corpus cannot afford).  The
// synthetic universe gives kshift = 4 and nkeys = 2^22 instead
// of 2^26 window offsets; an x86 kernel's call sites are >= 5 bytes apart, so
// kshift >= 2 there.  Canonicalize emits keys (canon_wave.hip, key mode),
// Minimize's LDS ranges, the union bitmap and the first-cover array are over
// keys, and the union list maps back through pc_of_key.
#include "common.h"

namespace syz {

__global__ void keymap_kernel(const uint32_t *__restrict__ univ, uint64_t n, uint32_t kshift,
                              uint32_t kbase, uint64_t nkeys, uint32_t *__restrict__ pc_of_key,
                              uint32_t *__restrict__ err) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t pc = univ[i];
        const uint32_t key = (pc >> kshift) - kbase;
        if (key >= nkeys || (i && (univ[i - 1] >> kshift) >= (pc >> kshift))) {
            atomicOr(err, 1u);  // not sorted / not collision-free / outside the key range
            continue;
        }
        pc_of_key[key] = pc;
    }
}

// out[i] = pc_of_key[keys[i]] for i < *n_dev (device count, e.g. a union
// size still on the device) or n_max; in place allowed (out == keys).  A
// value outside [0, nkeys) (a stale slot) maps to 0xFFFFFFFF, never read.
__global__ void keys_to_pcs_kernel(const uint32_t *__restrict__ pc_of_key, uint64_t nkeys,
                                   const uint32_t *keys, uint32_t *out,
                                   const uint32_t *__restrict__ n_dev, uint64_t n_max) {
    const uint64_t n = n_dev ? (uint64_t)*n_dev : n_max;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n && i < n_max;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t k = keys[i];
        out[i] = k < nkeys ? pc_of_key[k] : 0xFFFFFFFFu;
    }
}

// covered[w] = bits of the keys with a first cover (first < INT32_MAX): the
// corpus union, from the MIN-merged first-cover array of a sharded step.
__global__ void first_to_bits_kernel(const int32_t *__restrict__ first, uint64_t span,
                                     uint32_t *__restrict__ covered) {
    const uint64_t nw = (span + 31) / 32;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw * 32;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const bool set = i < span && first[i] != INT32_MAX;
        const uint64_t m = __ballot(set);
        if ((threadIdx.x & 31) == 0) covered[i >> 5] = (uint32_t)(m >> (threadIdx.x & 32));
    }
}

}  // namespace syz

using namespace syz;

extern "C" int syzcov_dev_first_to_bits(const int32_t *first, uint64_t span, uint32_t *covered,
                                        void *stream) {
    if (span == 0) return 0;
    if (!first || !covered) return SYZCOV_EINVAL;
    hipLaunchKernelGGL(first_to_bits_kernel, dim3(grid_for((span + 31) / 32 * 32, 256, 8192)),
                       dim3(256), 0, (hipStream_t)stream, first, span, covered);
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" int syzcov_dev_universe_keymap(const uint32_t *univ, size_t n, uint32_t kshift,
                                          uint32_t kbase, uint64_t nkeys, uint32_t *pc_of_key,
                                          uint32_t *err_flag, void *stream) {
    if (n == 0) return 0;
    if (!univ || !pc_of_key || !err_flag || kshift > 31 || nkeys == 0) return SYZCOV_EINVAL;
    hipLaunchKernelGGL(keymap_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0,
                       (hipStream_t)stream, univ, (uint64_t)n, kshift, kbase, nkeys, pc_of_key,
                       err_flag);
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" int syzcov_dev_keys_to_pcs(const uint32_t *pc_of_key, uint64_t nkeys,
                                      const uint32_t *keys, uint32_t *out, const uint32_t *n_dev,
                                      size_t n_max, void *stream) {
    if (n_max == 0) return 0;
    if (!pc_of_key || !keys || !out) return SYZCOV_EINVAL;
    hipLaunchKernelGGL(keys_to_pcs_kernel, dim3(grid_for(n_max, 256, 4096)), dim3(256), 0,
                       (hipStream_t)stream, pc_of_key, nkeys, keys, out, n_dev,
                       (uint64_t)n_max);
    SYZ_LAUNCH_CHECK();
    return 0;
}
