// dedup.hip — the executor's cover_dedup (executor/executor.cc:574-587) over a
// batch of raw u64 KCOV buffers, on the GPU.
//
// Reference semantics, per buffer: std::sort ascending, then keep pc iff
// pc != last with `last` starting at 0 — so the result is the sorted distinct
// nonzero PCs, compacted to the front of the buffer in place, and the new
// count.  executor.cc:459-463 then writes each kept PC truncated to u32; the
// optional out32 array receives exactly those words.
//
// One workgroup (256 threads = 4 waves) per buffer.  Sorting is the
// all-ascending ("flip") bitonic network, with its compare-exchanges in
// registers: each thread holds E keys whose indices differ in a log2(E)-bit
// window of index bits, so log2(E) stages run without LDS traffic and the LDS
// is touched only when the window moves.  The flip stage of a merge level
// whose partners are not register-local is done as a reversal of the block's
// upper half inside that move, so every compare-exchange is the same
// ascending min/max (no direction bits).
//
// Keys.  A kernel's text spans far less than 4 GB, so a buffer's PCs almost
// always satisfy max - min < 2^32: those buffers sort the u32 offsets
// pc - min (v_min_u32 / v_max_u32 per compare-exchange, half the LDS bytes
// and registers of u64 keys) and add min back when they store.  Buffers whose
// PCs span more (any u64 input is legal) are marked and sorted with u64 keys
// by a second kernel, as are buffers longer than one tile.
//
// Kernels, all walking every buffer and taking those of their class (so each
// has the register and LDS budget of its own tile):
//  - narrow<E>, E = 4, 8, 16: buffers of up to 1024, 2048, 4096 PCs, tile of
//    next_pow2(n) u32 keys (pads +inf in LDS), so all 256 threads work on a
//    buffer of 1-4K PCs;
//  - wide: the marked buffers (u64 keys, one tile), and the buffers longer
//    than 4096 (KCOV holds up to kCoverSize = 64K, executor.cc:50): their
//    4096-tiles are sorted in LDS and merged in place in HBM by the same
//    network, whose virtual +inf pads past n never move (no workspace); the
//    merge stages with strides below 4096 run in LDS per tile.
// Compaction: keep = pc != predecessor (0 before the first), wave ballots
// per register row, a 64-entry scan, coalesced in-place stores.
#include "common.h"

namespace syz {
namespace dd {

constexpr uint32_t NT = 256;  // threads per workgroup
constexpr uint32_t LT = 12;   // log2 of the LDS tile
constexpr uint32_t T = 1u << LT;
constexpr uint32_t WIDE = 0xFFFFFFFEu;  // new_len mark: left to the wide kernel

template <int E> struct Lg;
template <> struct Lg<4> { static constexpr uint32_t v = 2; };
template <> struct Lg<8> { static constexpr uint32_t v = 3; };
template <> struct Lg<16> { static constexpr uint32_t v = 4; };

__device__ __forceinline__ void cx(uint32_t &a, uint32_t &b) {
    const uint32_t x = a, y = b;
    a = x < y ? x : y;
    b = x < y ? y : x;
}

__device__ __forceinline__ void cx(uint64_t &a, uint64_t &b) {
    const uint64_t x = a, y = b;
    const bool sw = x > y;
    a = sw ? y : x;
    b = sw ? x : y;
}

__device__ __forceinline__ uint32_t ceil_log2(uint32_t n) { return n <= 1 ? 0 : 32 - __clz(n - 1); }

template <typename K, int E>
struct Shared {
    K tile[E * NT + NT];  // + one pad key per E (bank spread)
    uint64_t red[8];
    uint32_t cnt[64];
    uint32_t pre[64];
    uint32_t tot;
    uint32_t nsel;
    uint32_t sel[NT];
};

// The network over one tile of 2^LGT keys, E registers per thread, R threads
// active.  Register e of thread t in the window at s holds index
// idx(t, e, s) = (t mod 2^s) | e << s | (t >> s) << (s + log2 E); windows sit
// at multiples of log2 E (or at LGT - log2 E), and the LDS keeps one pad key
// per E, at lds_at(i) = i + (i >> log2 E), so every register's LDS address is
// a per-thread base plus a compile-time offset.
template <typename K, int E, int LGT>
struct Net {
    static constexpr int LG = Lg<E>::v;
    static_assert(LGT >= 2 * LG && LGT <= LG + 8, "tile shape");
    static constexpr uint32_t R = 1u << (LGT - LG);
    static constexpr int win(int b) {
        return b / LG * LG < LGT - LG ? b / LG * LG : LGT - LG;
    }
    static __device__ __forceinline__ uint32_t lds_at(uint32_t i) { return i + (i >> LG); }
    template <int S>
    static __device__ __forceinline__ uint32_t base(uint32_t t) {
        return (t & ((1u << S) - 1)) | ((t >> S) << (S + LG));
    }
    // lds_at(b + (e << S)) for b with bits [S, S + LG) clear
    template <int S>
    static constexpr uint32_t step() {
        return (1u << S) + (S >= LG ? (1u << (S - LG)) : 0u);
    }

    template <int LB>
    static __device__ __forceinline__ void half_clean(K (&v)[E]) {
#pragma unroll
        for (int e = 0; e < E; e++)
            if (!(e & (1 << LB))) cx(v[e], v[e | (1 << LB)]);
    }
    template <int B>
    static __device__ __forceinline__ void flip(K (&v)[E]) {
#pragma unroll
        for (int e = 0; e < E; e++)
            if (!(e & (1 << B))) cx(v[e], v[e ^ ((2 << B) - 1)]);
    }
    // half-cleaners on index bits BHI .. W in the window at W
    template <int W, int BHI>
    static __device__ __forceinline__ void stages(K (&v)[E]) {
        if constexpr (BHI >= W) {
            half_clean<BHI - W>(v);
            stages<W, BHI - 1>(v);
        }
    }
    // the merge levels whose blocks fit in one thread's registers (window 0)
    template <int B>
    static __device__ __forceinline__ void reg_levels(K (&v)[E]) {
        if constexpr (B < LG) {
            flip<B>(v);
            stages<0, B - 1>(v);
            reg_levels<B + 1>(v);
        }
    }

    // registers from the window at SF to the window at ST through LDS; with
    // RB > 0, the reads reverse the lower RB bits of every index whose bit RB
    // (inside the window at ST) is set: the flip stage of merge level RB
    template <int SF, int ST, int RB>
    static __device__ __forceinline__ void relayout(K (&v)[E], K *lds, uint32_t t, bool act) {
        if (act) {
            K *w = lds + lds_at(base<SF>(t));
#pragma unroll
            for (int e = 0; e < E; e++) w[e * step<SF>()] = v[e];
        }
        __syncthreads();
        if (act) {
            const K *r = lds + lds_at(base<ST>(t));
            if constexpr (RB > 0) {
                static_assert(RB >= ST && RB < ST + LG, "reversal bit in the window");
                const K *rr = lds + lds_at((~t & ((1u << ST) - 1)) | ((t >> ST) << (ST + LG)));
                constexpr int EB = RB - ST, EM = (1 << EB) - 1;
#pragma unroll
                for (int e = 0; e < E; e++)
                    v[e] = (e >> EB) & 1 ? rr[(e ^ EM) * step<ST>()] : r[e * step<ST>()];
            } else {
#pragma unroll
                for (int e = 0; e < E; e++) v[e] = r[e * step<ST>()];
            }
        }
        __syncthreads();
    }

    // stages BHI .. W in the window at W, then down through the lower windows
    template <int BHI, int W>
    static __device__ __forceinline__ void chain(K (&v)[E], K *lds, uint32_t t, bool act) {
        if (act) stages<W, BHI>(v);
        if constexpr (W > 0) {
            constexpr int W2 = win(W - 1);
            relayout<W, W2, 0>(v, lds, t, act);
            chain<W - 1, W2>(v, lds, t, act);
        }
    }
    template <int B>
    static __device__ __forceinline__ void levels(K (&v)[E], K *lds, uint32_t t, bool act) {
        if constexpr (B < LGT) {
            constexpr int W = win(B);
            relayout<0, W, B>(v, lds, t, act);
            chain<B, W>(v, lds, t, act);
            levels<B + 1>(v, lds, t, act);
        }
    }
    // full sort from the coalesced window (LGT - LG) back to it
    static __device__ void sort(K (&v)[E], K *lds, uint32_t t, bool act) {
        relayout<LGT - LG, 0, 0>(v, lds, t, act);
        if (act) reg_levels<0>(v);
        levels<LG>(v, lds, t, act);
        relayout<0, LGT - LG, 0>(v, lds, t, act);
    }
    // the merge stages with strides 2^(LGT-1) .. 1, coalesced window to itself
    static __device__ void clean(K (&v)[E], K *lds, uint32_t t) {
        chain<LGT - 1, win(LGT - 1)>(v, lds, t, true);
        relayout<0, LGT - LG, 0>(v, lds, t, true);
    }

    // Append the kept PCs of the sorted tile.  v: its keys in the coalesced
    // window (register e of thread t = index e * R + t) and the LDS holding
    // the same keys; PC = key + kbase; n_t real keys; carry: the PC before
    // index 0 (0 for a buffer's first tile, executor.cc:579).
    static __device__ void compact(const K (&v)[E], Shared<K, E> &sh, uint32_t t, uint32_t n_t,
                                   uint64_t kbase, uint64_t &carry, uint32_t &wpos, uint64_t *g,
                                   uint32_t *o32) {
        const uint32_t wave = t >> 6, lane = t & 63;
        uint64_t m[E];
#pragma unroll
        for (int e = 0; e < E; e++) {
            const uint32_t i = e * R + t;
            bool keep = false;
            if (t < R && i < n_t)
                keep = (uint64_t)v[e] + kbase !=
                       (i ? (uint64_t)sh.tile[lds_at(i - 1)] + kbase : carry);
            m[e] = __ballot(keep);
            if (lane == 0) sh.cnt[e * 4 + wave] = (uint32_t)__popcll(m[e]);
        }
        __syncthreads();
        if (wave == 0) {
            // rows are index-ordered (e, wave, lane): an exclusive scan over 4E
            const uint32_t x = lane < E * 4 ? sh.cnt[lane] : 0u;
            uint32_t inc = x;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(inc, d, 64);
                if ((int)lane >= d) inc += y;
            }
            sh.pre[lane] = inc - x;
            if (lane == 63) sh.tot = inc;
        }
        __syncthreads();
        const uint64_t lt = (1ull << lane) - 1;
#pragma unroll
        for (int e = 0; e < E; e++) {
            if ((m[e] >> lane) & 1) {
                const uint32_t pos = wpos + sh.pre[e * 4 + wave] + (uint32_t)__popcll(m[e] & lt);
                const uint64_t pc = (uint64_t)v[e] + kbase;
                g[pos] = pc;
                if (o32) o32[pos] = (uint32_t)pc;
            }
        }
        carry = (uint64_t)sh.tile[lds_at(n_t - 1)] + kbase;
        wpos += sh.tot;
        __syncthreads();
    }
};

// A buffer of n PCs (n <= 2^LGT) with max - min < 2^32: u32 keys pc - min.
// Returns false (nothing written) when its PCs span more.
template <int E, int LGT>
__device__ bool narrow_buffer(Shared<uint32_t, E> &sh, uint32_t t, uint32_t n, uint64_t *g,
                              uint32_t *o32, uint32_t &wpos) {
    using N = Net<uint32_t, E, LGT>;
    constexpr uint32_t R = N::R;
    uint64_t pc[E];
    uint64_t mn = ~0ull, mx = 0;
#pragma unroll
    for (int e = 0; e < E; e++) {
        const uint32_t i = e * R + t;  // the coalesced window
        const bool in = t < R && i < n;
        pc[e] = in ? g[i] : 0;
        if (in) {
            mn = pc[e] < mn ? pc[e] : mn;
            mx = pc[e] > mx ? pc[e] : mx;
        }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t a = __shfl_xor(mn, d, 64), b = __shfl_xor(mx, d, 64);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
    }
    const uint32_t wave = t >> 6;
    if ((t & 63) == 0) {
        sh.red[wave] = mn;
        sh.red[4 + wave] = mx;
    }
    __syncthreads();
    mn = sh.red[0];
    mx = sh.red[4];
#pragma unroll
    for (int w = 1; w < 4; w++) {
        mn = sh.red[w] < mn ? sh.red[w] : mn;
        mx = sh.red[4 + w] > mx ? sh.red[4 + w] : mx;
    }
    __syncthreads();  // sh.red is read by every thread before reuse
    if (mx - mn > 0xFFFFFFFFull) return false;
    uint32_t v[E];
#pragma unroll
    for (int e = 0; e < E; e++) {
        const uint32_t i = e * R + t;
        v[e] = (t < R && i < n) ? (uint32_t)(pc[e] - mn) : 0xFFFFFFFFu;
    }
    N::sort(v, sh.tile, t, t < R);
    uint64_t carry = 0;
    N::compact(v, sh, t, n, mn, carry, wpos, g, o32);
    return true;
}

using W16 = Net<uint64_t, 16, LT>;

// a buffer of n <= 4096 PCs with u64 keys (one full tile)
__device__ void wide_buffer(Shared<uint64_t, 16> &sh, uint32_t t, uint32_t n, uint64_t *g,
                            uint32_t *o32, uint32_t &wpos) {
    uint64_t v[16];
#pragma unroll
    for (int e = 0; e < 16; e++) {
        const uint32_t i = e * NT + t;
        v[e] = i < n ? g[i] : ~0ull;
    }
    W16::sort(v, sh.tile, t, true);
    uint64_t carry = 0;
    W16::compact(v, sh, t, n, 0, carry, wpos, g, o32);
}

// the coalesced tile [base, base + T) of g, pads +inf
__device__ __forceinline__ void load_tile(uint64_t (&v)[16], const uint64_t *g, uint32_t base,
                                          uint32_t n, uint32_t t) {
#pragma unroll
    for (int e = 0; e < 16; e++) {
        const uint32_t i = base + e * NT + t;
        v[e] = i < n ? g[i] : ~0ull;
    }
}

__device__ __forceinline__ void store_tile(const uint64_t (&v)[16], uint64_t *g, uint32_t base,
                                           uint32_t n, uint32_t t) {
#pragma unroll
    for (int e = 0; e < 16; e++) {
        const uint32_t i = base + e * NT + t;
        if (i < n) g[i] = v[e];
    }
}

__device__ __forceinline__ void cmpswap(uint64_t *g, uint32_t i, uint32_t q) {
    const uint64_t a = g[i], b = g[q];
    if (a > b) {
        g[i] = b;
        g[q] = a;
    }
}

// global stages of one workgroup: the writes of a stage must be seen by the
// other waves' loads of the next (the L1 is invalidated by the fence)
__device__ __forceinline__ void gsync() {
    __threadfence();
    __syncthreads();
}

// a buffer of n > 4096 PCs: u64 tiles sorted in LDS, merged in HBM
__device__ void large_buffer(Shared<uint64_t, 16> &sh, uint32_t t, uint32_t n, uint64_t *g,
                             uint32_t *o32, uint32_t &wpos) {
    uint64_t v[16];
    const uint32_t ntiles = (n + T - 1) / T;
    for (uint32_t c = 0; c < ntiles; c++) {
        load_tile(v, g, c * T, n, t);
        W16::sort(v, sh.tile, t, true);
        store_tile(v, g, c * T, n, t);
    }
    gsync();
    // the merges of blocks of 2^lk
    const uint32_t lgP = ceil_log2(n);
    for (uint32_t lk = LT + 1; lk <= lgP; lk++) {
        const uint32_t half = 1u << (lk - 1), npair = 1u << (lgP - 1);
        for (uint32_t p = t; p < npair; p += NT) {  // flip: i <-> block end - 1 - r
            const uint32_t r = p & (half - 1), blk = (p >> (lk - 1)) << lk;
            const uint32_t q = blk + 2 * half - 1 - r;
            if (q < n) cmpswap(g, blk + r, q);
        }
        gsync();
        for (uint32_t lj = lk - 2; lj >= LT; lj--) {
            const uint32_t j = 1u << lj;
            for (uint32_t p = t; p < npair; p += NT) {
                const uint32_t i = ((p >> lj) << (lj + 1)) | (p & (j - 1));
                if (i + j < n) cmpswap(g, i, i + j);
            }
            gsync();
        }
        for (uint32_t c = 0; c < ntiles; c++) {
            load_tile(v, g, c * T, n, t);
            W16::clean(v, sh.tile, t);
            store_tile(v, g, c * T, n, t);
        }
        gsync();
    }
    uint64_t carry = 0;
    for (uint32_t c = 0; c < ntiles; c++) {
        load_tile(v, g, c * T, n, t);
        uint64_t *w = sh.tile + W16::lds_at(W16::base<8>(t));
#pragma unroll
        for (int e = 0; e < 16; e++) w[e * W16::step<8>()] = v[e];
        __syncthreads();
        const uint32_t nt = n - c * T < T ? n - c * T : T;
        W16::compact(v, sh, t, nt, 0, carry, wpos, g, o32);
    }
}

// Buffers blockIdx.x + k * gridDim.x, k = 0, 1, ...: each round the 256
// threads classify 256 of them at once, then the workgroup dedups the
// selected ones in order.
template <typename K, int E, typename Sel, typename Run>
__device__ __forceinline__ void walk(Shared<K, E> &sh, uint32_t t, uint64_t nseg, Sel sel,
                                     Run run) {
    const uint64_t stride = gridDim.x;
    for (uint64_t k0 = 0; blockIdx.x + k0 * stride < nseg; k0 += NT) {
        const uint64_t seg = blockIdx.x + (k0 + t) * stride;
        const bool mine = seg < nseg && sel(seg);
        if (t == 0) sh.nsel = 0;
        __syncthreads();
        const uint64_t bal = __ballot(mine);
        uint32_t wbase = 0;
        if ((t & 63) == 0 && bal) wbase = atomicAdd(&sh.nsel, (uint32_t)__popcll(bal));
        wbase = __shfl(wbase, 0, 64);
        if (mine) sh.sel[wbase + __popcll(bal & ((1ull << (t & 63)) - 1))] = t;
        __syncthreads();
        const uint32_t ns = sh.nsel;
        // (the order within a round is free: the buffers are independent)
        for (uint32_t j = 0; j < ns; j++) run(blockIdx.x + (k0 + sh.sel[j]) * stride);
        __syncthreads();
    }
}

// (occupancy: E = 16 at 128 VGPRs and E = 8 at 96 run 4 and 5 waves per SIMD
// without spills; E = 4 spills below its 136)
template <int E>
__global__ __launch_bounds__(NT, E == 16 ? 4 : E == 8 ? 5 : 1) void narrow_kernel(uint64_t *pcs, const uint64_t *off,
                                                    uint64_t nseg, uint32_t *new_len,
                                                    uint32_t *out32) {
    __shared__ Shared<uint32_t, E> sh;
    const uint32_t t = threadIdx.x;
    constexpr uint64_t lo = E == 4 ? 0 : E == 8 ? 4 * NT : 8 * NT, hi = E * NT;
    walk(
        sh, t, nseg,
        [&](uint64_t seg) {
            const uint64_t b0 = off[seg], b1 = off[seg + 1];
            return b1 >= b0 && b1 - b0 <= hi && (b1 - b0 > lo || (E == 4 && b1 == b0));
        },
        [&](uint64_t seg) {
            const uint64_t b0 = off[seg];
            const uint32_t n = (uint32_t)(off[seg + 1] - b0);
            uint64_t *g = pcs + b0;
            uint32_t *o32 = out32 ? out32 + b0 : nullptr;
            uint32_t wpos = 0;
            bool done = true;
            if constexpr (E == 4) {
                switch (ceil_log2(n)) {  // tiles of 16 .. 1024 keys
                case 0: case 1: case 2: case 3: case 4:
                    if (n) done = narrow_buffer<4, 4>(sh, t, n, g, o32, wpos);
                    break;
                case 5: done = narrow_buffer<4, 5>(sh, t, n, g, o32, wpos); break;
                case 6: done = narrow_buffer<4, 6>(sh, t, n, g, o32, wpos); break;
                case 7: done = narrow_buffer<4, 7>(sh, t, n, g, o32, wpos); break;
                case 8: done = narrow_buffer<4, 8>(sh, t, n, g, o32, wpos); break;
                case 9: done = narrow_buffer<4, 9>(sh, t, n, g, o32, wpos); break;
                default: done = narrow_buffer<4, 10>(sh, t, n, g, o32, wpos); break;
                }
            } else {
                done = narrow_buffer<E, Lg<E>::v + 8>(sh, t, n, g, o32, wpos);
            }
            if (t == 0) new_len[seg] = done ? wpos : WIDE;
        });
}

__global__ __launch_bounds__(NT) void wide_kernel(uint64_t *pcs, const uint64_t *off,
                                                  uint64_t nseg, uint32_t *new_len,
                                                  uint32_t *out32) {
    __shared__ Shared<uint64_t, 16> sh;
    const uint32_t t = threadIdx.x;
    walk(
        sh, t, nseg,
        [&](uint64_t seg) {
            const uint64_t b0 = off[seg], b1 = off[seg + 1];
            return b1 < b0 || b1 - b0 > T || new_len[seg] == WIDE;
        },
        [&](uint64_t seg) {
            const uint64_t b0 = off[seg], b1 = off[seg + 1];
            if (b1 < b0 || b1 - b0 > (1ull << 31)) {  // malformed or beyond the u32 network
                if (t == 0) new_len[seg] = UINT32_MAX;
                return;
            }
            const uint32_t n = (uint32_t)(b1 - b0);
            uint32_t wpos = 0;
            uint32_t *o32 = out32 ? out32 + b0 : nullptr;
            if (n <= T)
                wide_buffer(sh, t, n, pcs + b0, o32, wpos);
            else
                large_buffer(sh, t, n, pcs + b0, o32, wpos);
            if (t == 0) new_len[seg] = wpos;
        });
}

// ---------------------------------------------------------------------
// Executor buffers straight into the new-coverage check: the
// deduped buffers' u32 words packed into a CSR of records.
constexpr uint32_t IB = 1024;  // buffers per scan block

__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t v) {
    const uint32_t l = __lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(v, d, 64);
        if ((int)l >= d) v += y;
    }
    return v;
}

// exclusive scan over IB threads (u64); *total = the block's sum
__device__ __forceinline__ uint64_t block_excl_scan64(uint64_t v, uint64_t *tmp, uint64_t *total) {
    const uint32_t w = threadIdx.x >> 6, l = __lane_id();
    const uint64_t inc = wave_incl_scan64(v);
    if (l == 63) tmp[w] = inc;
    __syncthreads();
    if (w == 0) {
        const uint64_t x = l < IB / 64 ? tmp[l] : 0ull;
        const uint64_t xi = wave_incl_scan64(x);
        if (l < IB / 64) tmp[l] = xi - x;
        if (l == IB / 64 - 1) tmp[IB / 64] = xi;
    }
    __syncthreads();
    const uint64_t r = tmp[w] + inc - v;
    *total = tmp[IB / 64];
    __syncthreads();
    return r;
}

// a malformed buffer (new_len UINT32_MAX) contributes no record PCs
__device__ __forceinline__ uint64_t rec_len(const uint32_t *nl, uint64_t b, uint64_t nbuf) {
    return b < nbuf && nl[b] != UINT32_MAX ? nl[b] : 0u;
}

__global__ __launch_bounds__(IB) void ingest_bsum_kernel(const uint32_t *nl, uint64_t nbuf,
                                                         uint64_t *bsum) {
    __shared__ uint64_t tmp[IB / 64 + 1];
    uint64_t total;
    block_excl_scan64(rec_len(nl, (uint64_t)blockIdx.x * IB + threadIdx.x, nbuf), tmp, &total);
    if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

__global__ __launch_bounds__(IB) void ingest_bscan_kernel(uint64_t *bsum, uint64_t nblk) {
    __shared__ uint64_t tmp[IB / 64 + 1];
    uint64_t carry = 0;
    for (uint64_t c = 0; c < nblk; c += IB) {
        const uint64_t i = c + threadIdx.x;
        uint64_t total;
        const uint64_t p = block_excl_scan64(i < nblk ? bsum[i] : 0ull, tmp, &total);
        if (i < nblk) bsum[i] = carry + p;
        carry += total;
    }
}

__global__ __launch_bounds__(IB) void ingest_off_kernel(const uint32_t *nl, uint64_t nbuf,
                                                        const uint64_t *bsum, uint64_t *rec_off,
                                                        uint32_t *err) {
    __shared__ uint64_t tmp[IB / 64 + 1];
    const uint64_t b = (uint64_t)blockIdx.x * IB + threadIdx.x;
    const uint64_t len = rec_len(nl, b, nbuf);
    uint64_t total;
    const uint64_t p = bsum[blockIdx.x] + block_excl_scan64(len, tmp, &total);
    if (b < nbuf) {
        rec_off[b] = p;
        if (nl[b] == UINT32_MAX && err) atomicOr(err, 1u);
    }
    if (b == nbuf - 1) rec_off[nbuf] = p + len;
}

// record b's words from their buffer slot to their CSR slot
__global__ __launch_bounds__(NT) void ingest_copy_kernel(const uint32_t *words, const uint64_t *off,
                                                         const uint32_t *nl, uint64_t nbuf,
                                                         const uint64_t *rec_off,
                                                         uint32_t *rec_pcs) {
    for (uint64_t b = blockIdx.x; b < nbuf; b += gridDim.x) {
        const uint64_t len = rec_len(nl, b, nbuf);
        const uint32_t *src = words + off[b];
        uint32_t *dst = rec_pcs + rec_off[b];
        for (uint64_t i = threadIdx.x; i < len; i += NT) dst[i] = src[i];
    }
}

}  // namespace dd
}  // namespace syz

using namespace syz;

// executor.cc:574-587 over nseg buffers [off[s], off[s + 1]) of pcs, in place
extern "C" int syzcov_dev_cover_dedup64(uint64_t *pcs, const uint64_t *off, size_t nseg,
                                        uint32_t *new_len, uint32_t *out32, void *stream) {
    if (nseg == 0) return 0;
    if (!pcs || !off || !new_len) return SYZCOV_EINVAL;
    // a few resident workgroups per CU walk the buffers of each class
    const unsigned grid = nseg < 4096 ? (unsigned)nseg : 4096u;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(dd::narrow_kernel<4>, dim3(grid), dim3(dd::NT), 0, s, pcs, off,
                       (uint64_t)nseg, new_len, out32);
    hipLaunchKernelGGL(dd::narrow_kernel<8>, dim3(grid), dim3(dd::NT), 0, s, pcs, off,
                       (uint64_t)nseg, new_len, out32);
    hipLaunchKernelGGL(dd::narrow_kernel<16>, dim3(grid), dim3(dd::NT), 0, s, pcs, off,
                       (uint64_t)nseg, new_len, out32);
    hipLaunchKernelGGL(dd::wide_kernel, dim3(grid), dim3(dd::NT), 0, s, pcs, off, (uint64_t)nseg,
                       new_len, out32);
    SYZ_LAUNCH_CHECK();
    return 0;
}

static size_t ingest_part(size_t n) { return (n + 255) / 256 * 256; }

extern "C" size_t syzcov_dev_cover_ingest64_ws_size(size_t nbuf, uint64_t total) {
    const size_t nblk = (nbuf + dd::IB - 1) / dd::IB;
    return ingest_part(nbuf * 4) + ingest_part(total * 4) + ingest_part(nblk * 8);
}

// executor.cc:574-587 + :459-463 over nbuf raw KCOV buffers, the
// kept words packed into the records syzcov_state_newcov_dev takes
extern "C" int syzcov_dev_cover_ingest64(uint64_t *pcs64, const uint64_t *off, size_t nbuf,
                                         uint64_t total, uint64_t *rec_off, uint32_t *rec_pcs,
                                         uint32_t *err, void *ws, size_t ws_size, void *stream) {
    if (nbuf == 0) return 0;
    if (!pcs64 || !off || !rec_off || !rec_pcs || !ws ||
        ws_size < syzcov_dev_cover_ingest64_ws_size(nbuf, total))
        return SYZCOV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    uint8_t *w = (uint8_t *)ws;
    uint32_t *nl = (uint32_t *)w;
    uint32_t *words = (uint32_t *)(w + ingest_part(nbuf * 4));
    uint64_t *bsum = (uint64_t *)(w + ingest_part(nbuf * 4) + ingest_part(total * 4));
    if (int rc = syzcov_dev_cover_dedup64(pcs64, off, nbuf, nl, words, stream)) return rc;
    const uint64_t nblk = (nbuf + dd::IB - 1) / dd::IB;
    hipLaunchKernelGGL(dd::ingest_bsum_kernel, dim3(nblk), dim3(dd::IB), 0, s, nl, (uint64_t)nbuf,
                       bsum);
    hipLaunchKernelGGL(dd::ingest_bscan_kernel, dim3(1), dim3(dd::IB), 0, s, bsum, nblk);
    hipLaunchKernelGGL(dd::ingest_off_kernel, dim3(nblk), dim3(dd::IB), 0, s, nl, (uint64_t)nbuf,
                       bsum, rec_off, err);
    const unsigned grid = nbuf < 8192 ? (unsigned)nbuf : 8192u;
    hipLaunchKernelGGL(dd::ingest_copy_kernel, dim3(grid), dim3(dd::NT), 0, s, words, off, nl,
                       (uint64_t)nbuf, rec_off, rec_pcs);
    SYZ_LAUNCH_CHECK();
    return 0;
}
