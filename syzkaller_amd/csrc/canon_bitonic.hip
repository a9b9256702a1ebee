// canon_bitonic.hip — cover.Canonicalize (cover/cover.go:27-40) as a bitonic
// sorting network held entirely in VGPRs.
//
// The radix canonicalizer (canon_wave.hip) is bound by the LDS pipe: three
// random LDS operations per key and pass, and the skewed PC distribution
// turns the histogram atomics into same-address conflicts.  Here a wave
// keeps NK = 32 keys per lane (2048 keys) in registers and sorts them with
// the all-ascending ("flip") bitonic network: 66 compare-exchange stages, 45
// of them between registers of one lane (v_min/v_max), 21 between lanes,
// whose partner values come from DPP row patterns and v_permlane16/32_swap
// (xperm.h) — no LDS, no data-dependent conflicts, deterministic.  Segments
// up to 4093 / 8189 keys take 2 / 4 waves; only the flip stages between
// waves (and one half-cleaner stage for 4 waves) go through LDS.
//
// Keys are window offsets (pc - pc_lo); slots beyond the segment hold
// 0xFFFFFFFF and sort last.  The raw list is read with coalesced 16-byte
// loads in any order (a network does not care where keys start); the sorted
// keys sit in blocked order (wave w, lane l, register i = position
// 2048 w + 32 l + i).  Unique keeps the reference loop (`last := sent`), and
// each lane writes its kept run to the segment's own CSR slots (in place is
// safe: every raw key is in registers before the first write).  Split points
// per PC range (for minimize_range.hip) come from the range transitions of
// the kept stream.
#include "common.h"
#include "xperm.h"

#include <algorithm>

namespace syz {
namespace cbt {

constexpr int NK = 32;       // keys per lane
constexpr int MAX_R = 256;   // ranges (split columns)

struct Params {
    const uint64_t *off;
    const uint32_t *raw;
    uint32_t *out;
    uint32_t *new_len;
    uint32_t pc_lo;
    uint32_t span_m1;
    uint32_t sent_key;        // window offset of PC 0xFFFFFFFF (or 0xFFFFFFFF if outside)
    uint32_t *split;          // nullable: [nseg][nrange]
    uint32_t nrange, rshift;
    unsigned long long *range_tot;
    uint32_t *err;
};

__device__ __forceinline__ void cmpx(uint32_t &a, uint32_t &b) {
    const uint32_t lo = min(a, b);
    b = max(a, b);
    a = lo;
}

// --- stages inside one lane (register index pairs)
template <int K>  // flip: i <-> i ^ (K-1) within blocks of K registers
__device__ __forceinline__ void flip_regs(uint32_t (&k)[NK]) {
#pragma unroll
    for (int i = 0; i < NK; i++) {
        const int j = i ^ (K - 1);
        if (i < j) cmpx(k[i], k[j]);
    }
}

template <int J>  // half-cleaner: i <-> i ^ J
__device__ __forceinline__ void half_regs(uint32_t (&k)[NK]) {
#pragma unroll
    for (int i = 0; i < NK; i++)
        if (!(i & J)) cmpx(k[i], k[i | J]);
}

template <int J>  // half-cleaners J, J/2, ..., 1 inside the lane
__device__ __forceinline__ void half_regs_down(uint32_t (&k)[NK]) {
    half_regs<J>(k);
    if constexpr (J > 1) half_regs_down<J / 2>(k);
}

// --- stages between lanes
template <int M>  // flip: (lane, i) <-> (lane ^ M, NK-1-i); the lower lane keeps the min
__device__ __forceinline__ void flip_lanes(uint32_t (&k)[NK]) {
    const bool lower = !(__lane_id() & ((M + 1) >> 1));
#pragma unroll
    for (int i = 0; i < NK / 2; i++) {
        const uint32_t a = k[i], b = k[NK - 1 - i];
        const uint32_t pa = xperm<M>(b), pb = xperm<M>(a);
        k[i] = lower ? min(a, pa) : max(a, pa);
        k[NK - 1 - i] = lower ? min(b, pb) : max(b, pb);
    }
}

template <int M>  // half-cleaner: (lane, i) <-> (lane ^ M, i)
__device__ __forceinline__ void half_lanes(uint32_t (&k)[NK]) {
    const bool lower = !(__lane_id() & M);
#pragma unroll
    for (int i = 0; i < NK; i++) {
        const uint32_t p = xperm<M>(k[i]);
        k[i] = lower ? min(k[i], p) : max(k[i], p);
    }
}

template <int M>  // lane half-cleaners M, M/2, ..., 1
__device__ __forceinline__ void half_lanes_down(uint32_t (&k)[NK]) {
    half_lanes<M>(k);
    if constexpr (M > 1) half_lanes_down<M / 2>(k);
}

// the half-cleaners of a level whose blocks span LB lanes: lane part, then registers
template <int LB>
__device__ __forceinline__ void merge_tail(uint32_t (&k)[NK]) {
    if constexpr (LB >= 4) half_lanes_down<LB / 4>(k);
    half_regs_down<NK / 2>(k);
}

template <int K>
__device__ __forceinline__ void levels_in_lane(uint32_t (&k)[NK]) {
    flip_regs<K>(k);
    if constexpr (K >= 4) half_regs_down<K / 4>(k);
    if constexpr (K < NK) levels_in_lane<K * 2>(k);
}

template <int LB>
__device__ __forceinline__ void levels_across_lanes(uint32_t (&k)[NK]) {
    flip_lanes<LB - 1>(k);
    merge_tail<LB>(k);
    if constexpr (LB < 64) levels_across_lanes<LB * 2>(k);
}

// Sort the wave's 64 * NK keys ascending in blocked order.
__device__ __forceinline__ void sort_wave(uint32_t (&k)[NK]) {
    levels_in_lane<2>(k);
    levels_across_lanes<2>(k);
}

// Exchange with another wave of the workgroup through LDS: p[i] = partner
// wave's key at (lane ^ lmask, register i ^ rmask).
template <int W>
__device__ __forceinline__ void wave_exchange(const uint32_t (&k)[NK], uint32_t (&p)[NK],
                                              uint32_t *xbuf, uint32_t w, uint32_t pw,
                                              uint32_t lmask, int rmask) {
    const uint32_t l = __lane_id();
#pragma unroll
    for (int i = 0; i < NK; i++) xbuf[(w * NK + i) * 64 + l] = k[i];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NK; i++) p[i] = xbuf[(pw * NK + (i ^ rmask)) * 64 + (l ^ lmask)];
    __syncthreads();
}

template <int W>
__global__ __launch_bounds__(64 * W) void canon_bitonic_kernel(Params P, const uint32_t *list,
                                                               const uint32_t *count) {
    constexpr int NQ = NK / 4;
    __shared__ uint32_t xbuf[W > 1 ? W * 64 * NK : 1];
    __shared__ uint32_t s_last[W], s_cnt[W], s_lastr[W];
    __shared__ unsigned long long s_rt[MAX_R];
    const uint32_t t = threadIdx.x;
    const uint32_t w = __builtin_amdgcn_readfirstlane(t >> 6);
    const uint32_t l = __lane_id();
    for (uint32_t j = t; j < MAX_R; j += 64 * W) s_rt[j] = 0;
    __syncthreads();
    const uint32_t nl = *count;
    for (uint32_t li = blockIdx.x; li < nl; li += gridDim.x) {
        const uint32_t seg = list[li];
        const uint64_t base = P.off[seg];
        const uint32_t n = (uint32_t)(P.off[seg + 1] - base);
        const uint64_t a0 = base & ~3ull;
        const uint32_t head = (uint32_t)(base - a0), end = head + n;
        const uint4 *src = reinterpret_cast<const uint4 *>(P.raw + a0);
        uint32_t k[NK];
        bool oob = false;
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            const uint32_t chunk = (w * NQ + q) * 64 + l;
            const uint32_t e4 = chunk * 4u;
            const uint4 v = src[e4 < end ? chunk : 0];  // chunk 0 is always valid
            const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const uint32_t idx = e4 + c;
                const uint32_t key = vv[c] - P.pc_lo;
                const bool valid = idx >= head && idx < end;
                oob |= valid && key > P.span_m1;
                k[q * 4 + c] = valid ? key : 0xFFFFFFFFu;
            }
        }
        if (__ballot(oob) && l == 0) *P.err = 1u;
        sort_wave(k);
        if constexpr (W > 1) {
            // levels spanning waves: blocks of KW waves
#pragma unroll
            for (int KW = 2; KW <= W; KW *= 2) {
                uint32_t p[NK];
                {   // flip: (w, l, i) <-> (w ^ (KW-1), l ^ 63, NK-1-i)
                    wave_exchange<W>(k, p, xbuf, w, w ^ (KW - 1), 63u, NK - 1);
                    const bool lower = !(w & (KW >> 1));
#pragma unroll
                    for (int i = 0; i < NK; i++) k[i] = lower ? min(k[i], p[i]) : max(k[i], p[i]);
                }
#pragma unroll
                for (int JW = KW / 4; JW >= 1; JW /= 2) {  // wave half-cleaners
                    wave_exchange<W>(k, p, xbuf, w, w ^ JW, 0u, 0);
                    const bool lower = !(w & JW);
#pragma unroll
                    for (int i = 0; i < NK; i++) k[i] = lower ? min(k[i], p[i]) : max(k[i], p[i]);
                }
                merge_tail<128>(k);  // every half-cleaner inside the wave
            }
        }
        // ------------------------------------------------ unique
        // position of (w, l, i) = 64 NK w + NK l + i; prev of i = 0 is the
        // previous lane's last key (the previous wave's for lane 0).
        if constexpr (W > 1) {
            if (l == 63) s_last[w] = k[NK - 1];
            __syncthreads();
        }
        const uint32_t wfirst = w == 0 ? P.sent_key : s_last[w - 1];
        uint32_t prev = shift_up(k[NK - 1], wfirst);
        const uint32_t pos0 = (w * 64 + l) * NK;
        uint32_t keepm = 0, c = 0;
#pragma unroll
        for (int i = 0; i < NK; i++) {
            const bool keep = pos0 + i < n && k[i] != prev;
            keepm |= (uint32_t)keep << i;
            c += keep;
            prev = k[i];
        }
        const uint32_t incl = wave_incl_scan(c);
        uint32_t lbase = incl - c, total = __shfl(incl, 63, 64), wbase = 0;
        if constexpr (W > 1) {
            if (l == 63) s_cnt[w] = total;
            __syncthreads();
            total = 0;
            for (uint32_t j = 0; j < W; j++) {
                const uint32_t cj = s_cnt[j];
                wbase += j < w ? cj : 0u;
                total += cj;
            }
        }
        uint32_t *outp = P.out + base + wbase + lbase;
        uint32_t o = 0;
#pragma unroll
        for (int i = 0; i < NK; i++)
            if ((keepm >> i) & 1u) outp[o++] = k[i] + P.pc_lo;
        if (t == 0) P.new_len[seg] = total;
        // ------------------------------------------------ range splits
        // split[j] = # kept keys with range <= j: written at every range
        // transition of the kept stream, the tail up to R-1 gets `total`.
        {
            uint32_t lastr = 0;  // range of this lane's last kept key (0 if none)
#pragma unroll
            for (int i = 0; i < NK; i++)
                if ((keepm >> i) & 1u) lastr = k[i] >> P.rshift;
            // ranges are non-decreasing along the stream: prefix max = carry-in
            uint32_t mx = lastr;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t up = __shfl_up(mx, d, 64);
                if (l >= (uint32_t)d) mx = max(mx, up);
            }
            uint32_t rin = shift_up(mx, 0u);  // lanes before this one
            if constexpr (W > 1) {
                if (l == 63) s_lastr[w] = mx;
                __syncthreads();
                uint32_t wr = 0;
                for (uint32_t j = 0; j < w; j++) wr = max(wr, s_lastr[j]);
                rin = max(rin, wr);
            }
            uint32_t pos = wbase + lbase, r = rin, run = 0;
#pragma unroll
            for (int i = 0; i < NK; i++)
                if ((keepm >> i) & 1u) {
                    const uint32_t ri = k[i] >> P.rshift;
                    if (ri != r) {
                        if (P.split)
                            for (uint32_t j = r; j < ri; j++) P.split[(uint64_t)seg * P.nrange + j] = pos;
                        if (run) atomicAdd(&s_rt[r], (unsigned long long)run);
                        r = ri;
                        run = 0;
                    }
                    pos++;
                    run++;
                }
            if (run) atomicAdd(&s_rt[r], (unsigned long long)run);
            // the last kept key's lane closes the stream: ranges r..R-1 end at total
            const uint64_t has = __ballot(keepm != 0);
            const bool lastw = W == 1 || total == wbase + (uint32_t)__shfl(incl, 63, 64);
            if (P.split) {
                if (has) {
                    const uint32_t ll = 63 - __clzll(has);
                    if (lastw && l == ll)
                        for (uint32_t j = r; j < P.nrange; j++)
                            P.split[(uint64_t)seg * P.nrange + j] = total;
                } else if (total == 0 && t == 0) {
                    for (uint32_t j = 0; j < P.nrange; j++) P.split[(uint64_t)seg * P.nrange + j] = 0;
                }
            }
        }
        __syncthreads();  // xbuf / s_* reuse by the next segment
    }
    __syncthreads();
    for (uint32_t j = t; j < P.nrange; j += 64 * W)
        if (s_rt[j]) atomicAdd(&P.range_tot[j], s_rt[j]);
}

}  // namespace cbt

// Launch the bitonic canonicalizer over class lists: W = 1 (n <= 2045),
// 2 (<= 4093), 4 (<= 8189).  lists/counts as produced by the binning kernel.
int canon_bitonic_launch(int W, const uint64_t *off, const uint32_t *raw, uint32_t *out,
                         uint32_t *new_len, uint32_t pc_lo, uint64_t pc_span, uint32_t sent_key,
                         uint32_t *split, uint32_t nrange, uint32_t rshift, uint64_t *range_tot,
                         uint32_t *err, const uint32_t *list, const uint32_t *cnt, uint64_t nseg,
                         hipStream_t s) {
    cbt::Params P;
    P.off = off;
    P.raw = raw;
    P.out = out;
    P.new_len = new_len;
    P.pc_lo = pc_lo;
    P.span_m1 = (uint32_t)(pc_span - 1);
    P.sent_key = sent_key;
    P.split = split;
    P.nrange = nrange;
    P.rshift = rshift;
    P.range_tot = (unsigned long long *)range_tot;
    P.err = err;
    const unsigned grid = (unsigned)std::min<uint64_t>(std::max<uint64_t>(nseg, 1), 8192);
    switch (W) {
    case 1: hipLaunchKernelGGL(cbt::canon_bitonic_kernel<1>, dim3(grid), dim3(64), 0, s, P, list, cnt); break;
    case 2: hipLaunchKernelGGL(cbt::canon_bitonic_kernel<2>, dim3(grid), dim3(128), 0, s, P, list, cnt); break;
    case 4: hipLaunchKernelGGL(cbt::canon_bitonic_kernel<4>, dim3(grid), dim3(256), 0, s, P, list, cnt); break;
    default: return SYZCOV_EINVAL;
    }
    SYZ_LAUNCH_CHECK();
    return 0;
}

}  // namespace syz
