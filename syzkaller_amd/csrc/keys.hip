// keys.hip — the engine's dense key space over a registered PC universe.
//
// The universe is the set of PCs KCOV can REPORT: the return address of every
// `call __sanitizer_cov_trace_pc` (the call sites objdump lists for
// allCoverPCs, syz-manager/cover.go:274-306, plus the call's length — KCOV
// records the return address, which is why cover.go:82 subtracts 1 again),
// truncated to u32 as the executor does (executor.cc:455-466).  With
// kshift = the largest shift (capped at KSHIFT_MAX) that keeps that universe
// collision-free (no two universe PCs share pc >> kshift) and
// kbase = U[0] >> kshift,
//     key(pc) = (pc >> kshift) - kbase
// is injective on the universe and maps it onto [0, nkeys): a dense key space
// computed with a shift and a subtract.  The synthetic universe
// gives kshift = 4 and nkeys = 2^22 instead of 2^26 window offsets; an x86
// kernel's return addresses are >= 5 bytes apart, so kshift >= 2 there.
//
// EXACT ON ANY INPUT.  Two PCs can share a key only if one of them is not in
// the universe, so a key never stands for a PC by itself: canonical lists hold
// KEY WORDS, key | (pc & lowmask) << SYZ_KEY_BITS (common.h), and whatever
// indexes by key also checks membership,
//     low_of_key[key] == (pc & lowmask),  lowmask = 2^kshift - 1
// (one byte per key: the universe PC's low kshift bits, 0x7F for a key with no
// universe PC; kshift <= 6 keeps 0x7F out of reach and bit 7 free for
// Minimize's covered flag).  A PC that fails it sets SYZCOV_ERR_UNIVERSE and
// the step / batch raises instead of aliasing it with its neighbour:
// Minimize pass 1 checks every canonical word against the table staged in LDS
// next to its covered bits (minimize_range.hip); the fuzzer state's pc_index
// checks every PC it indexes (cover_state.h).
#include "common.h"

namespace syz {

__global__ void keymap_kernel(const uint32_t *__restrict__ univ, uint64_t n, uint32_t kshift,
                              uint32_t kbase, uint64_t nkeys, uint32_t *__restrict__ pc_of_key,
                              uint8_t *__restrict__ low_of_key, uint32_t *__restrict__ err) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t pc = univ[i];
        const uint32_t key = (pc >> kshift) - kbase;
        if (key >= nkeys || (i && (univ[i - 1] >> kshift) >= (pc >> kshift))) {
            atomicOr(err, 1u);  // not sorted / not collision-free / outside the key range
            continue;
        }
        if (pc_of_key) pc_of_key[key] = pc;
        if (low_of_key) low_of_key[key] = (uint8_t)(pc & ((1u << kshift) - 1u));
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

// out[i] = the PC of key word words[i] (common.h): exact for any word, no
// table (the canonical lists of a key-mode step back as PCs).
__global__ void words_to_pcs_kernel(const uint32_t *words, uint64_t n, uint32_t kshift,
                                    uint32_t kbase, uint32_t *out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t w = words[i];
        out[i] = (((w & SYZ_KEY_MASK) + kbase) << kshift) | (w >> SYZ_KEY_BITS);
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
                                          uint8_t *low_of_key, uint32_t *err_flag, void *stream) {
    if (!univ || (!pc_of_key && !low_of_key) || !err_flag || kshift > SYZCOV_KSHIFT_MAX ||
        nkeys == 0)
        return SYZCOV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    // keys without a universe PC: pc_of_key 0 (never read for a valid key),
    // low_of_key 0x7F (no PC's low kshift <= 6 bits equal it)
    if (pc_of_key) SYZ_HIP(hipMemsetAsync(pc_of_key, 0, nkeys * 4, s));
    if (low_of_key) SYZ_HIP(hipMemsetAsync(low_of_key, 0x7F, nkeys, s));
    if (n == 0) return 0;
    hipLaunchKernelGGL(keymap_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, univ,
                       (uint64_t)n, kshift, kbase, nkeys, pc_of_key, low_of_key, err_flag);
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

extern "C" int syzcov_dev_words_to_pcs(const uint32_t *words, size_t n, uint32_t kshift,
                                       uint32_t kbase, uint32_t *out, void *stream) {
    if (n == 0) return 0;
    if (!words || !out || kshift > SYZCOV_KSHIFT_MAX) return SYZCOV_EINVAL;
    hipLaunchKernelGGL(words_to_pcs_kernel, dim3(grid_for(n, 256, 16384)), dim3(256), 0,
                       (hipStream_t)stream, words, (uint64_t)n, kshift, kbase, out);
    SYZ_LAUNCH_CHECK();
    return 0;
}
