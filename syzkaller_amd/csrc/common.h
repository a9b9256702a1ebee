// common.h — shared device/host helpers for the syzcov HIP kernels (gfx950).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include <atomic>
#include <type_traits>

#include "../../include/syzcov.h"
#include "force.h"

#define SYZ_SENT 0xFFFFFFFFu
#define SYZ_WAVE 64

namespace syz {

void set_error(const char *fmt, ...);

#define SYZ_HIP(expr)                                                                  \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess) {                                                        \
            ::syz::set_error("%s:%d %s: %s", __FILE__, __LINE__, #expr,                \
                             hipGetErrorString(e_));                                   \
            return SYZCOV_EHIP;                                                        \
        }                                                                              \
    } while (0)

#define SYZ_LAUNCH_CHECK()                                                             \
    do {                                                                               \
        hipError_t e_ = hipGetLastError();                                             \
        if (e_ != hipSuccess) {                                                        \
            ::syz::set_error("%s:%d launch: %s", __FILE__, __LINE__,                   \
                             hipGetErrorString(e_));                                   \
            return SYZCOV_EHIP;                                                        \
        }                                                                              \
    } while (0)

static inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device):
// `done` holds one bit per device (function attributes are per device, and
// the C-ABI serves up to 16 devices from concurrent threads).
static inline int set_dyn_lds_once(const void *fn, int bytes, std::atomic<uint32_t> &done) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return SYZCOV_EHIP;
    const uint32_t bit = 1u << (dev & 31);
    if (done.load(std::memory_order_acquire) & bit) return 0;
    SYZ_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
    done.fetch_or(bit, std::memory_order_release);
    return 0;
}
static inline unsigned grid_for(size_t n, unsigned block, unsigned cap = 1u << 16) {
    size_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

// ---------------------------------------------------------------- device side
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// Issue fence of a software-pipelined loop: loads issued before it stay
// before it (memory clobber), and code that reads the returned value stays
// after it.  Without it the scheduler sinks the next batch's loads below the
// current batch's consumers, so the in-order vmcnt wait for the current batch
// also drains the next one (one batch in flight instead of two).
// -DSYZ_NO_ISSUE_FENCE builds the unfenced schedule for A/B runs.
template <typename T>
__device__ __forceinline__ T issue_fence(T x) {
#ifndef SYZ_NO_ISSUE_FENCE
    asm volatile("" : "+s"(x) : : "memory");
#endif
    return x;
}

// The ONLY door to the readlane builtins (tests/test_source_guards.py fails
// on any other use).  They move 32
// bits and return int: a 64-bit value or a pointer passed straight in loses
// its high half, and an int result widened to 64 bits sign-extends a low half
// >= 2^31 (two GPU faults).  These keep the caller's 32-bit
// type, reject anything else at compile time, and 64-bit values go through
// uniform_u64 / wave_readlane_u64 (both halves as uint32_t).
template <class T>
__device__ __forceinline__ T wave_readfirstlane(T v) {
    static_assert(sizeof(T) == 4 && std::is_integral<T>::value,
                  "readfirstlane moves 32 bits: use uniform_u64 for 64-bit values / pointers");
    return (T)__builtin_amdgcn_readfirstlane((int)v);  // readlane-door
}
template <class T>
__device__ __forceinline__ T wave_readlane(T v, int lane) {
    static_assert(sizeof(T) == 4 && std::is_integral<T>::value,
                  "readlane moves 32 bits: use wave_readlane_u64 for 64-bit values / pointers");
    return (T)__builtin_amdgcn_readlane((int)v, lane);  // readlane-door
}
__device__ __forceinline__ uint64_t wave_readlane_u64(uint64_t v, int lane) {
    return ((uint64_t)wave_readlane((uint32_t)(v >> 32), lane) << 32) |
           wave_readlane((uint32_t)v, lane);
}

// A wave-uniform value into scalar registers
__device__ __forceinline__ uint32_t uniform_u32(uint32_t v) { return wave_readfirstlane(v); }
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
    return ((uint64_t)uniform_u32((uint32_t)(v >> 32)) << 32) | uniform_u32((uint32_t)v);
}

// Wave-wide inclusive scan of a u32 (64 lanes) in DPP, no LDS: row_shr 1, 2,
// 4, 8 scan each row of 16 lanes (lanes shifted in from outside the row read
// the identity 0), then row_bcast:15 adds row r-1's total to rows 1 and 3 and
// row_bcast:31 adds rows 0-1's total to rows 2 and 3 (gfx9 DPP broadcasts).
// The __shfl_up form compiled to a ds_bpermute round trip per step.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return v;
}

// Histograms of u16 PAIRS (bins 2w and 2w + 1 in the halves of word w) for
// the wave radix sorts (canon_wave.hip, dedup.hip).
// exclusive scan of the 2048 u16 counts in bin order, in place
// (WQ uint4 of words per lane: 4 for the 1024 words of 2048 bins, 8 for the
// 2048 words of a 12-bit digit's 4096 bins).  Lane l holds chunks q * 64 + l
// (lane-contiguous 16-byte accesses, conflict-free; a lane-contiguous run of
// WQ chunks put lanes 4 (WQ 8: 2) apart on the same banks, a 4-way (8-way)
// conflict on every read and write), so chunk row q's prefix is the rows
// before it plus a wave scan within the row: two rows per scan, packed as
// u16 pairs (a segment's counts stay below 2^16).
template <int WQ = 4>
__device__ __forceinline__ void hist16_scan(uint32_t *h, uint32_t l) {
    static_assert(WQ % 2 == 0, "rows are scanned in pairs");
    uint4 *h4 = reinterpret_cast<uint4 *>(h);
    uint4 v[WQ];
    uint32_t s[WQ];
#pragma unroll
    for (int q = 0; q < WQ; q++) {
        v[q] = h4[q * 64 + l];
        const uint32_t w4[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
        s[q] = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) s[q] += (w4[i] & 0xFFFFu) + (w4[i] >> 16);
    }
    uint32_t base = 0;
#pragma unroll
    for (int q = 0; q < WQ; q += 2) {
        const uint32_t inc = wave_incl_scan(s[q] | (s[q + 1] << 16));
        const uint32_t tot = wave_readlane(inc, 63);
        uint32_t pq[2];
        pq[0] = base + (inc & 0xFFFFu) - s[q];
        base += tot & 0xFFFFu;
        pq[1] = base + (inc >> 16) - s[q + 1];
        base += tot >> 16;
#pragma unroll
        for (int r = 0; r < 2; r++) {
            const uint4 vv = v[q + r];
            uint32_t w4[4] = {vv.x, vv.y, vv.z, vv.w};
            uint32_t p = pq[r];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint32_t lo = w4[i] & 0xFFFFu, hi = w4[i] >> 16;
                w4[i] = p | ((p + lo) << 16);
                p += lo + hi;
            }
            h4[(q + r) * 64 + l] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
        }
    }
}

template <int NQ, int WQ = 4>
__device__ __forceinline__ void hist16_zero(uint32_t *h, uint32_t l) {
    uint4 *h4 = reinterpret_cast<uint4 *>(h);
#pragma unroll
    for (int q = 0; q < WQ; q++) h4[q * 64 + l] = make_uint4(0, 0, 0, 0);
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// Block-wide exclusive scan; `tmp` is LDS with >= blockDim/64 + 1 entries.
// Returns the exclusive prefix of v; *total receives the block total.
template <int THREADS>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *tmp, uint32_t *total) {
    constexpr int NW = THREADS / 64;
    const uint32_t w = threadIdx.x >> 6, l = __lane_id();
    uint32_t inc = wave_incl_scan(v);
    if (l == 63) tmp[w] = inc;
    __syncthreads();
    if (w == 0) {
        uint32_t s = (l < NW) ? tmp[l] : 0u;
        uint32_t si = wave_incl_scan(s);
        if (l < NW) tmp[l] = si - s;
        if (l == NW - 1) tmp[NW] = si;
    }
    __syncthreads();
    uint32_t res = tmp[w] + inc - v;
    *total = tmp[NW];
    __syncthreads();
    return res;
}

// Key mode (keys.hip): a canonical PC travels as the WORD
//     key(pc) | (pc & (2^kshift - 1)) << SYZ_KEY_BITS,  key(pc) = (pc >> kshift) - kbase,
// i.e. the dense key plus the low bits the shift drops, so the PC itself is
// never lost (keys < 2^25, kshift <= SYZCOV_KSHIFT_MAX = 6: 31 bits).
constexpr uint32_t SYZ_KEY_BITS = 26;
constexpr uint32_t SYZ_KEY_MASK = (1u << SYZ_KEY_BITS) - 1u;
__host__ __device__ __forceinline__ uint32_t key_word(uint32_t pc, uint32_t kshift,
                                                      uint32_t kbase) {
    return ((pc >> kshift) - kbase) | ((pc & ((1u << kshift) - 1u)) << SYZ_KEY_BITS);
}

// Line-aligned canonical layout: every (input, range) sub-run
// of the canonical lists starts on its own 128-byte line, so Minimize's pass 1
// (minimize_range.hip), which reads range j of an input in a different
// workgroup than range j + 1, never fetches a line twice.  With R ranges and
// ak = SYZ_ALIGN_K(R) = 31 (R + 1):
//   input i's words start at   aligned_base(off[i], i, ak) = align32(off[i] + ak i)
//   range j's sub-run at       + aligned_sub(s_{j-1}, j)   = align32(s_{j-1} + 31 j)
// (s_j = split[i][j], s_{-1} = 0).  Sub-run j ends at or below s_j + 31 (j + 1),
// so sub-runs never overlap, and input i ends below aligned_base of i + 1:
// the buffer holds p + ak n + 32 words for n inputs of p raw PCs.  ak = 0 is
// the plain CSR layout (input i at off[i], sub-run j at s_{j-1}).
__host__ __device__ constexpr uint32_t SYZ_ALIGN_K(uint32_t nrange) { return 31u * (nrange + 1u); }
__host__ __device__ __forceinline__ uint64_t aligned_base(uint64_t off_i, uint64_t i, uint32_t ak) {
    return ak ? (off_i + (uint64_t)ak * i + 31u) & ~31ull : off_i;
}
__host__ __device__ __forceinline__ uint32_t aligned_sub(uint32_t s_prev, uint32_t j, uint32_t ak) {
    return ak ? (s_prev + 31u * j + 31u) & ~31u : s_prev;
}
static inline uint64_t aligned_words(uint64_t p, uint64_t n, uint32_t ak) {
    return ak ? p + (uint64_t)ak * n + 32 : p;
}

// 64-bit splitmix (synthetic generator; identical to oracle/synth_oracle.c).
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Dense PC-id lookup: tab[w] = prefix(lo 32) | bits(hi 32).
__device__ __forceinline__ uint32_t dense_id(const uint64_t *__restrict__ tab, uint32_t pc,
                                             uint32_t pc_lo) {
    uint32_t off = pc - pc_lo;
    uint64_t e = tab[off >> 5];
    uint32_t bits = (uint32_t)(e >> 32);
    uint32_t mask = (1u << (off & 31)) - 1u;
    return (uint32_t)e + __popc(bits & mask);
}

}  // namespace syz
