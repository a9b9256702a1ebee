// canon_wave.hip — corpus-scale cover.Canonicalize (cover/cover.go:27-40):
// one WAVEFRONT per segment, no workgroup barriers.
//
// A segment of n <= 8189 raw PCs is sorted by an LSD radix sort over its
// window offsets (pc - pc_lo, nbits = bit_length(span - 1), <= 9-bit digits)
// entirely in the wave's private LDS slice.  Key mode (a registered PC
// universe, keys.hip) writes each canonical PC as its dense key
// (pc >> kshift) - kbase: the map is monotone and injective on the universe,
// so the sorted unique PCs give the sorted unique keys, and the split points
// are taken over key ranges.  The sort itself stays on window offsets:
//   load     16-byte vector loads of the raw list (head/tail masked);
//   pass 0   lowest digit, unstable: count (ds_add), exclusive scan of the
//            512-entry histogram, scatter with ds_add_rtn positions;
//   pass k   stable: the keys are re-read row-major from LDS (row r = slots
//            64r..64r+63) and ranked with ds_add_rtn one row after another.
//            Stability needs same-address LDS atomics of ONE wave instruction
//            to be applied in lane order.  gfx950 does that
//            (tools/probe/lds_order.hip: 0 violations in 3M rows), but the
//            ISA does not promise it, so the result is CHECKED: a segment
//            whose final keys are not non-decreasing is not written and goes
//            to the workgroup bitonic fallback (canon.hip) instead.
//   unique   the reference loop (`last := sent`: the key of PC 0xFFFFFFFF is
//            dropped only in first position), ballot-compacted, written back
//            to the segment's own CSR slots (in place is safe: the wave holds
//            its keys before it writes) as PCs, or as keys in key mode.
// Optional outputs for the range-partitioned Minimize (minimize_range.hip):
//   split[seg * R + j] = number of canonical PCs with offset < (j+1) << rshift
//   range_tot[j]      += canonical PCs of range j over the corpus.
// Segments longer than 8189 keys are listed for the workgroup paths.
#include "common.h"
#include "xperm.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace syz {

int canon_list_path(const uint64_t *off, const uint32_t *in, uint32_t *out, uint32_t *new_len,
                    const uint32_t *list, const uint32_t *count, hipStream_t s, uint32_t ak);
int canon_large_path(const uint64_t *off, const uint32_t *in, uint32_t *out, uint32_t *new_len,
                     const uint32_t *dlist, uint32_t nlarge, uint8_t *pres, uint32_t pc_lo,
                     uint64_t pc_span, uint32_t *err, hipStream_t s, uint32_t ak);

#ifndef SYZ_CANON_W32
#define SYZ_CANON_W32 3
#endif
#ifndef SYZ_CANON_W40
#define SYZ_CANON_W40 3
#endif
#ifndef SYZ_CANON_W48
#define SYZ_CANON_W48 3
#endif
namespace cw {

constexpr int WPB = 2;        // waves per workgroup (independent segments)
constexpr int MAX_RPL = 4;    // ranges per lane (R <= 256)
constexpr uint32_t WAVE_MAX = 8192 - 3;  // a CAP-slot wave holds head (<= 3) + n keys

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// The histogram is PACKED: one u32 per digit holds the current pass's running
// slot in its low 16 bits and the next pass's digit count in its high 16 bits
// (a segment holds < 2^16 keys, so neither half overflows into the other).
// One 2 KB array per wave instead of two raises LDS-limited residency.
constexpr uint32_t CNT1 = 1u << 16;  // +1 on the high (count) half

// Exclusive scan of the counts (high halves) into slots (low halves), with the
// high halves cleared for the next pass's counts (HIST / 64 entries per lane).
// Lane l holds chunks q * 64 + l, conflict-free as in hist16_scan below: two
// chunk rows per wave scan, packed as u16 pairs.
template <int HIST>
__device__ __forceinline__ void hist_scan(uint32_t *hist, uint32_t l) {
    constexpr int PL = HIST / 256;  // uint4 chunks per lane
    static_assert(PL % 2 == 0, "rows are scanned in pairs");
    uint4 *h4 = reinterpret_cast<uint4 *>(hist);
    uint4 v[PL];
    uint32_t s[PL];
#pragma unroll
    for (int q = 0; q < PL; q++) {
        v[q] = h4[q * 64 + l];
        v[q].x >>= 16; v[q].y >>= 16; v[q].z >>= 16; v[q].w >>= 16;
        s[q] = v[q].x + v[q].y + v[q].z + v[q].w;
    }
    uint32_t base = 0;
#pragma unroll
    for (int q = 0; q < PL; q += 2) {
        const uint32_t inc = wave_incl_scan(s[q] | (s[q + 1] << 16));
        const uint32_t tot = wave_readlane(inc, 63);
        uint32_t pq[2];
        pq[0] = base + (inc & 0xFFFFu) - s[q];
        base += tot & 0xFFFFu;
        pq[1] = base + (inc >> 16) - s[q + 1];
        base += tot >> 16;
#pragma unroll
        for (int r = 0; r < 2; r++) {
            uint32_t p = pq[r];
            const uint4 vv = v[q + r];
            uint4 o;
            o.x = p; p += vv.x; o.y = p; p += vv.y; o.z = p; p += vv.z; o.w = p;
            h4[(q + r) * 64 + l] = o;
        }
    }
}

template <int HIST>
__device__ __forceinline__ void hist_zero(uint32_t *hist, uint32_t l) {
    constexpr int PL = HIST / 256;
    uint4 *h4 = reinterpret_cast<uint4 *>(hist);
#pragma unroll
    for (int q = 0; q < PL; q++) h4[q * 64 + l] = make_uint4(0, 0, 0, 0);
}

// One radix scatter over the active rows: ranks by ds_add_rtn on the low
// halves, writes each key to its slot, and counts the next pass's digit into
// the high halves.  The atomics of BQ row quads are issued before their
// stores: a store's address depends on its atomic's return, and the compiler
// does not move a later atomic above an earlier store, so one store per
// atomic would expose a full LDS round trip per row.  Atomics of a wave apply
// in program order, so the row-major ranking order (stability) is unchanged.
#ifndef SYZ_CANON_BQ
#define SYZ_CANON_BQ 2
#endif
#ifndef SYZ_CANON_BQK  // row quads per rank batch of the key kernel
#define SYZ_CANON_BQK SYZ_CANON_BQ
#endif
#ifndef SYZ_CANON_BQ_AL
#define SYZ_CANON_BQ_AL SYZ_CANON_BQK
#endif
// Only REAL keys take part: slots outside the segment (the aligned head, the
// tail of the last row quad) are skipped rather than ranked as maximal pads,
// which would all hit ONE histogram address (serialised same-address LDS
// atomics).  RAW: the keys are in the raw-load layout (slot (q*64+l)*4+c,
// real iff in [lo, hi)); otherwise row-major (slot (q*4+c)*64+l, real iff
// < hi).  Real keys always sort to [0, n), so later passes see them there.
template <bool RAW, int NK>
__device__ __forceinline__ bool real_slot(int j, uint32_t l, uint32_t lo, uint32_t hi) {
    if (RAW) {
        const uint32_t idx = (uint32_t)(((j >> 2) * 64 + l) * 4 + (j & 3));
        return idx >= lo && idx < hi;
    }
    return (uint32_t)(j * 64) + l < hi;
}

// Pad slots are sent, branch-free, to a private dummy word of their lane
// (hist[HIST + l], buf[cap + l]): distinct addresses, so they cost no
// same-address serialisation, and they never touch the real counters/slots.
template <bool RAW, int NK, int HIST, int BQ = SYZ_CANON_BQ>
__device__ __forceinline__ void scatter_rows(const uint32_t (&k)[NK], uint32_t nq, uint32_t l,
                                             uint32_t lo, uint32_t hi, uint32_t *buf,
                                             uint32_t *hist, uint32_t sh, uint32_t dmask,
                                             uint32_t dbits, bool count_next) {
    constexpr int NQ = NK / 4;
    constexpr uint32_t CAP = 64 * NK;
    static_assert(NQ % BQ == 0, "row quads per batch");
#pragma unroll
    for (int q0 = 0; q0 < NQ; q0 += BQ) {
        if ((uint32_t)q0 >= nq) continue;
        uint32_t pos[4 * BQ];
        bool ok[4 * BQ];
#pragma unroll
        for (int j = 0; j < 4 * BQ; j++) {
            ok[j] = real_slot<RAW, NK>(q0 * 4 + j, l, lo, hi);
            if ((uint32_t)(q0 + j / 4) < nq)
                pos[j] = atomicAdd(&hist[ok[j] ? (k[q0 * 4 + j] >> sh) & dmask : HIST + l], 1u);
        }
#pragma unroll
        for (int j = 0; j < 4 * BQ; j++)
            if ((uint32_t)(q0 + j / 4) < nq) buf[ok[j] ? pos[j] & 0xFFFFu : CAP + l] = k[q0 * 4 + j];
        if (count_next) {
#pragma unroll
            for (int j = 0; j < 4 * BQ; j++)
                if ((uint32_t)(q0 + j / 4) < nq)
                    atomicAdd(&hist[ok[j] ? (k[q0 * 4 + j] >> (sh + dbits)) & dmask : HIST + l], CNT1);
        }
    }
}

struct Params {
    const uint64_t *off;
    const uint32_t *raw;
    uint32_t *out;
    uint32_t *new_len;
    uint64_t nseg;
    uint32_t pc_lo;
    uint64_t span;
    uint32_t nbits;
    uint32_t kshift, kbase;   // output key = (pc >> kshift) - kbase (key mode)
    uint64_t nkeys;
    uint32_t lowmask;           // 2^kshift - 1 (key mode: the word's low bits)
    int key_out;              // write keys (key mode) instead of PCs
    uint32_t sent_key;        // key of PC 0xFFFFFFFF (or 0xFFFFFFFF if outside)
    uint32_t *split;          // nullable: [nseg][nrange]
    uint32_t nrange, rshift;
    unsigned long long *range_tot;  // nullable: [nrange]
    uint32_t *redo_list, *redo_cnt;  // wave sort failed its order check
    uint32_t *big_list, *big_cnt;    // n > WAVE_MAX (listed by bin_kernel)
    uint32_t *err;
    uint32_t force_redo;             // SYZCOV_FORCE=redo: every segment takes the redo path
    uint32_t ak;                     // line-aligned sub-runs (common.h SYZ_ALIGN_K), 0 = CSR slots
};

// Line-aligned writes (common.h): the output position of the kept word at
// canonical index pos is pos + delta, delta = aligned_sub(s, j, ak) - s for the
// range j the word falls in (s = the index of j's first word).  Words arrive in
// sorted order, a row of 64 at a time; a lane whose word is the first of its
// range (`start`) derives the delta, and it holds until the next start (at
// most R per segment, so the uniform loop over a row's starts is short).
__device__ __forceinline__ uint32_t aligned_delta(uint64_t start_mask, uint32_t pos, uint32_t rng,
                                                  uint32_t ak, uint32_t l, uint32_t &dcar) {
    uint32_t delta = dcar;
    if (start_mask) {  // wave-uniform
        const uint32_t dl = aligned_sub(pos, rng, ak) - pos;
        uint64_t rem = start_mask;
        while (rem) {
            const uint32_t b = (uint32_t)__builtin_ctzll(rem);
            rem &= rem - 1;
            const uint32_t db = wave_readlane(dl, b);
            if (l >= b) delta = db;
            dcar = db;
        }
    }
    return delta;
}

// Wave-aggregated binning of segments into capacity classes (one atomic per
// wave and class): lists[c][..] = segments with cls_lo[c] <= n <= cls_hi[c].
constexpr int NCLS = 5;
struct Classes { uint32_t lo[NCLS], hi[NCLS]; };

// BIN_K segments per thread per round, so a round takes one global atomic per
// class for 256 * BIN_K segments (per 256 the six class counters saw 39 K
// contended atomics each at C3: 0.45 ms)
constexpr int BIN_K = 16;
__global__ __launch_bounds__(256) void bin_kernel(const uint64_t *__restrict__ off, uint64_t nseg,
                                                  Classes C, uint32_t *__restrict__ counts,
                                                  uint32_t *__restrict__ lists, uint64_t stride,
                                                  uint32_t *__restrict__ big_list,
                                                  uint32_t *__restrict__ big_cnt,
                                                  uint64_t max_len, uint32_t *__restrict__ err) {
    // block-aggregated: LDS counts per class, ONE global atomic per round and class
    __shared__ uint32_t s_cnt[NCLS + 1], s_base[NCLS + 1];
    __shared__ uint32_t s_wofs[4][BIN_K][NCLS + 1];  // each wave's slots in the round
    const uint32_t l = __lane_id(), wv = threadIdx.x >> 6;
    const uint64_t lt = (1ull << l) - 1ull;
    const uint64_t per = (uint64_t)blockDim.x * BIN_K;
    for (uint64_t b0 = (uint64_t)blockIdx.x * per; b0 < nseg; b0 += (uint64_t)gridDim.x * per) {
        if (threadIdx.x <= NCLS) s_cnt[threadIdx.x] = 0;
        __syncthreads();
        int cj[BIN_K];
#pragma unroll
        for (int j = 0; j < BIN_K; j++) {
            const uint64_t i = b0 + (uint64_t)j * blockDim.x + threadIdx.x;
            int c = -1;
            if (i < nseg) {
                const uint64_t n = off[i + 1] - off[i];
                // the host launches only the classes the declared bound reaches:
                // a longer segment would be left uncanonicalized, so it fails loudly
                if (n > max_len) atomicOr(err, SYZCOV_ERR_SEGLEN);
                c = n > WAVE_MAX ? NCLS : -1;  // NCLS = big list
#pragma unroll
                for (int k = 0; k < NCLS; k++)
                    if (n >= C.lo[k] && n <= C.hi[k]) c = k;
            }
            cj[j] = c;
        }
#pragma unroll
        for (int j = 0; j < BIN_K; j++)
#pragma unroll
            for (int k = 0; k <= NCLS; k++) {
                const uint64_t msk = __ballot(cj[j] == k);
                if (l == 0) s_wofs[wv][j][k] = msk ? atomicAdd(&s_cnt[k], (uint32_t)__popcll(msk)) : 0u;
            }
        __syncthreads();
        if (threadIdx.x <= NCLS) {
            const uint32_t k = threadIdx.x;
            s_base[k] = s_cnt[k] ? atomicAdd(k < NCLS ? &counts[k] : big_cnt, s_cnt[k]) : 0u;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < BIN_K; j++) {
            const uint64_t i = b0 + (uint64_t)j * blockDim.x + threadIdx.x;
#pragma unroll
            for (int k = 0; k <= NCLS; k++) {
                const uint64_t msk = __ballot(cj[j] == k);
                if (cj[j] == k) {
                    const uint32_t slot = s_base[k] + s_wofs[wv][j][k] + (uint32_t)__popcll(msk & lt);
                    if (k < NCLS) lists[k * stride + slot] = (uint32_t)i; else big_list[slot] = (uint32_t)i;
                }
            }
        }
        __syncthreads();
    }
}

// Window offset below which a canonical PC falls in range j of the split
// (ranges of 2^rshift KEYS in key mode, of window offsets otherwise).
__device__ __forceinline__ uint32_t split_bound(const Params &P, uint32_t j) {
    if (!P.key_out) return (j + 1) << P.rshift;
    const uint64_t pc = ((uint64_t)P.kbase + ((uint64_t)(j + 1) << P.rshift)) << P.kshift;
    if (pc <= P.pc_lo) return 0;
    const uint64_t o = pc - P.pc_lo;
    return o > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)o;
}

// NK = keys per lane (CAP = 64 * NK, NK a multiple of 4); MINW = waves per
// SIMD the register budget must allow (LDS caps residency anyway).  Segments
// come from a class list.  Only the n real keys are ranked (real_slot), so
// after every pass the sorted keys are buf[0, n); slots past n are stale and
// never read as keys.  Each pass counts the NEXT pass's digits while it
// scatters (packed histogram), so a pass is one read-back and one scatter
// loop; the keys of the pass being scattered live in registers only between
// those two loops.
// Wave priority by how far the wave is into its segment (s_setprio): 0
// converting the raw rows (and issuing the next segment's loads), 1 in the
// low-digit pass, 2 in the high-digit pass, 3 in unique + output + split.  Of
// the 3 waves a SIMD holds, the one furthest along issues first, so the
// waves spread over the phases and one wave's LDS-bound ranks overlap another's
// VALU-bound conversion or unique loop instead of all three queueing on the
// LDS together.  C3 canon 57.2 → 48.9 ms (DESIGN.md §4.1 with the other
// placements measured; the window-mode kernel: its first pass, later passes,
// unique).  SYZ_CANON_AGE_PRIO=0 builds leave every wave at 0.
#ifndef SYZ_CANON_AGE_PRIO
#define SYZ_CANON_AGE_PRIO 1
#endif
template <int P>
__device__ __forceinline__ void age_prio() {
    if constexpr (SYZ_CANON_AGE_PRIO != 0) __builtin_amdgcn_s_setprio(P);
}

template <int NK, int MINW, int HB>
__global__ __launch_bounds__(64 * WPB, MINW) void canon_wave_kernel(Params P, const uint32_t *list,
                                                                    const uint32_t *count) {
    constexpr int CAP = 64 * NK;
    constexpr int HIST = 1 << HB;
    constexpr int NQ = NK / 4;  // 16-byte loads per lane = row quads
    __shared__ uint32_t s_buf[WPB][CAP + 64];  // + one pad dummy per lane
    __shared__ __attribute__((aligned(16))) uint32_t s_hist[WPB][HIST + 64];
    const uint32_t w = wave_readfirstlane(threadIdx.x >> 6);
    const uint32_t l = __lane_id();
    uint32_t *buf = s_buf[w];
    const uint32_t nbits = P.nbits < 1 ? 1 : P.nbits;
    const uint32_t npass = (nbits + HB - 1) / HB;
    const uint32_t dbits = (nbits + npass - 1) / npass;  // <= HB
    const uint32_t dmask = (1u << dbits) - 1u;
    const uint32_t PAD = npass * dbits >= 32 ? 0xFFFFFFFFu : (1u << (npass * dbits)) - 1u;
    const uint64_t lt = (1ull << l) - 1ull;
    const uint32_t span_m1 = (uint32_t)(P.span - 1);
    const bool inplace = P.out == P.raw;
    uint32_t racc[MAX_RPL];
#pragma unroll
    for (int q = 0; q < MAX_RPL; q++) racc[q] = 0;
    const uint32_t nl = *count;
    const uint32_t nw = gridDim.x * WPB;
    // Software pipeline: the raw rows of the NEXT segment are loaded into
    // registers (vn) while this one is sorted in LDS, so the HBM latency of a
    // segment's load is hidden behind the previous segment's sort (the load
    // alone measured 3.0 of 12.0 ms at C2 when it was not overlapped).
    uint4 vn[NQ];
    uint32_t seg_n = 0, n_n = 0;
    uint64_t base_n = 0;
    auto issue = [&](uint32_t li_) {
        seg_n = list[li_];
        base_n = P.off[seg_n];
        n_n = (uint32_t)(P.off[seg_n + 1] - base_n);
        const uint64_t a0 = base_n & ~3ull;
        const uint32_t end = (uint32_t)(base_n - a0) + n_n;
        const uint32_t nq = (end + 255) >> 8;
        const uint4 *src = reinterpret_cast<const uint4 *>(P.raw + a0);
#pragma unroll
        for (int q = 0; q < NQ; q++)
            if ((uint32_t)q < nq) {
                const uint32_t e4 = (uint32_t)(q * 64 + l) * 4u;
                // chunks past the end re-read chunk 0 (always inside the buffer)
                vn[q] = src[e4 < end ? q * 64 + l : 0];
            }
    };
    uint32_t li = blockIdx.x * WPB + w;
    if (li < nl) issue(li);
    for (; li < nl; li += nw) {
        // wave-uniform descriptor in scalar registers (canon_key_kernel)
        age_prio<0>();
        const uint32_t seg = uniform_u32(seg_n);
        const uint64_t base = uniform_u64(base_n);
        const uint32_t n = uniform_u32(n_n);
        const uint64_t a0 = base & ~3ull;
        const uint32_t head = (uint32_t)(base - a0), end = head + n;
        const uint32_t nq = (end + 255) >> 8;  // active row quads (256 keys each)
        uint32_t k[NK];
        bool oob = false;
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            if ((uint32_t)q < nq) {
                const uint32_t e4 = (uint32_t)(q * 64 + l) * 4u;
                const uint32_t vv[4] = {vn[q].x, vn[q].y, vn[q].z, vn[q].w};
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    const uint32_t idx = e4 + c;
                    const uint32_t key = vv[c] - P.pc_lo;  // window offset: the sort key
                    const bool valid = idx >= head && idx < end;
                    oob |= valid && key > span_m1;
                    k[q * 4 + c] = valid ? key : PAD;
                }
            }
        }
        if (li + nw < nl) issue(li + nw);
        if (__ballot(oob) && l == 0) atomicOr(P.err, SYZCOV_ERR_WINDOW);
        age_prio<1>();
        // ------------------------------------------- pass 0 (unstable)
        hist_zero<HIST>(s_hist[w], l);
        wave_sync();
#pragma unroll
        for (int q = 0; q < NQ; q++)
            if ((uint32_t)q < nq) {
#pragma unroll
                for (int c = 0; c < 4; c++)
                    atomicAdd(&s_hist[w][real_slot<true, NK>(q * 4 + c, l, head, end)
                                             ? k[q * 4 + c] & dmask : HIST + l], CNT1);
            }
        wave_sync();
        hist_scan<HIST>(s_hist[w], l);
        wave_sync();
        const bool two = npass > 1;
        scatter_rows<true, NK, HIST>(k, nq, l, head, end, buf, s_hist[w], 0, dmask, dbits, two);
        wave_sync();
        age_prio<2>();
        // --------------------------------------------- stable passes
        for (uint32_t p = 1; p < npass; p++) {
            const uint32_t sh = p * dbits;
            const bool more = p + 1 < npass;
#pragma unroll
            for (int q = 0; q < NQ; q++)
                if ((uint32_t)q < nq) {
#pragma unroll
                    for (int c = 0; c < 4; c++) k[q * 4 + c] = buf[(q * 4 + c) * 64 + l];
                }
            hist_scan<HIST>(s_hist[w], l);
            wave_sync();
            scatter_rows<false, NK, HIST>(k, nq, l, 0, n, buf, s_hist[w], sh, dmask, dbits, more);
            wave_sync();
        }
        age_prio<3>();
        // --------------------------------- order check + unique + write
        // prev of slot e is slot e-1 (lane l-1 of the row, or lane 63 of the
        // previous row); the reference's `last := sent` for e == 0.
        // The sorted rows are read once into registers: the LDS writes of the
        // compaction below may not be reordered ahead of LDS reads, so reading
        // row by row there would expose one LDS round trip per row.
#pragma unroll
        for (int q = 0; q < NQ; q++)
            if ((uint32_t)q < nq) {
#pragma unroll
                for (int c = 0; c < 4; c++) k[q * 4 + c] = buf[(q * 4 + c) * 64 + l];
            }
        uint32_t bad = P.force_redo;
        if (inplace) {  // nothing may be written before the order is known
            uint32_t rprev = P.sent_key;  // predecessors as in canon_key_kernel
#pragma unroll
            for (int q = 0; q < NQ; q++)
                if ((uint32_t)q < nq) {
#pragma unroll
                    for (int c = 0; c < 4; c++) {
                        const uint32_t e = (uint32_t)((q * 4 + c) * 64) + l;
                        const uint32_t v = k[q * 4 + c];
                        const uint32_t r = rotate_up(v);
                        const uint32_t prev = l == 0 ? rprev : r;
                        rprev = r;
                        bad |= (uint32_t)(v < prev) & (uint32_t)(e - 1u < n - 1u);
                    }
                }
            if (__ballot(bad)) {
                if (l == 0) P.redo_list[atomicAdd(P.redo_cnt, 1u)] = seg;
                continue;
            }
        }
        uint32_t cnt = 0, rprev = P.sent_key, dcar = 0;
        uint32_t *outp = P.out + aligned_base(base, seg, P.ak);
#pragma unroll
        for (int q = 0; q < NQ; q++)
            if ((uint32_t)q < nq) {
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    const uint32_t e = (uint32_t)((q * 4 + c) * 64) + l;
                    const uint32_t v = k[q * 4 + c];
                    const uint32_t r = rotate_up(v);
                    const uint32_t prev = l == 0 ? rprev : r;
                    rprev = r;
                    bad |= (uint32_t)(v < prev) & (uint32_t)(e - 1u < n - 1u);
                    // keys outside [0, span) (flagged at load) sort last and are
                    // dropped, so nothing downstream indexes past the key range
                    const uint32_t keep =
                        (uint32_t)(e < n) & (uint32_t)(v != prev) & (uint32_t)(v <= span_m1);
                    const uint64_t m = __ballot(keep);
                    const uint32_t pos = cnt + (uint32_t)__popcll(m & lt);
                    // key mode: the PC's key word (common.h); the key map is
                    // monotone, so sorted unique PCs give sorted words
                    const uint32_t wo = P.key_out ? key_word(v + P.pc_lo, P.kshift, P.kbase)
                                                  : v + P.pc_lo;
                    uint32_t delta = 0;
                    if (P.ak) {  // uniform: the range of each word (keys or offsets)
                        const uint32_t rv = (P.key_out ? wo & SYZ_KEY_MASK : v) >> P.rshift;
                        const uint32_t rp = (P.key_out ? key_word(prev + P.pc_lo, P.kshift, P.kbase)
                                                             & SYZ_KEY_MASK
                                                       : prev) >> P.rshift;
                        const uint64_t sm = __ballot(keep && (pos == 0 || rv != rp));
                        delta = aligned_delta(sm, pos, rv, P.ak, l, dcar);
                    }
                    if (keep) {
                        outp[pos + delta] = wo;
                        buf[pos] = v;
                    }
                    cnt += (uint32_t)__popcll(m);
                }
            }
        if (__ballot(bad)) {  // out-of-place: the fallback rewrites this segment
            if (l == 0) P.redo_list[atomicAdd(P.redo_cnt, 1u)] = seg;
            continue;
        }
        if (l == 0) P.new_len[seg] = cnt;
        // ------------------------------------------- range splits
        if (!P.split) {
            if (l == 0) racc[0] += cnt;  // one range: its total is the PC count
        } else {
            wave_sync();
            uint32_t carry = 0;
            uint32_t *sp = P.split + (uint64_t)seg * P.nrange;
#pragma unroll
            for (int q = 0; q < MAX_RPL; q++) {
                const uint32_t j = q * 64 + l;
                if (q * 64 < (int)P.nrange) {
                    uint32_t s = cnt;
                    if (j + 1 < P.nrange) {
                        const uint32_t b = split_bound(P, j);
                        uint32_t lo = 0, hi = cnt;  // lower_bound(b) in buf[0, cnt)
                        while (lo < hi) {
                            const uint32_t mid = (lo + hi) >> 1;
                            if (buf[mid] < b) lo = mid + 1; else hi = mid;
                        }
                        s = lo;
                    }
                    const uint32_t prev_s = __shfl_up(s, 1, 64);
                    const uint32_t c = s - (l == 0 ? carry : prev_s);
                    carry = __shfl(s, 63, 64);
                    if (j < P.nrange) {
                        sp[j] = s;
                        racc[q] += c;
                    }
                }
            }
        }
    }
    if (P.range_tot) {
#pragma unroll
        for (int q = 0; q < MAX_RPL; q++) {
            const uint32_t j = q * 64 + l;
            if (j < P.nrange && racc[q]) atomicAdd(&P.range_tot[j], (unsigned long long)racc[q]);
        }
    }
}

// ---------------------------------------------------------------------------
// Key mode, <= 2^22 keys: the wave sorts the dense KEYS themselves in 2 LSD
// passes of 11-bit digits (the window offsets take 3 passes of 9 bits).
// The 2048-bin histogram is held as u16 PAIRS, bin d in half (d & 1) of word
// d >> 1 (4 KB; a segment holds < 2^16 keys, so a half never carries into the
// other), and the next pass's digit is counted after the scatter instead of
// during it, so one 4 KB array serves both passes: 12.3 KB of LDS per wave
// against 10.5 KB for the 3-pass sort, within the 3 waves per SIMD the
// registers allow anyway (the packed u32 format needed 8 KB of histogram and
// halved the resident waves, 9.45 vs 7.9 ms).  Random-address LDS operations
// per key: 6 (2 x count, rank, scatter) instead of 9.
// A PC outside the window is flagged (SYZCOV_ERR_WINDOW: the step's results
// are invalid and the engine raises) and sorts as the last key, so nothing
// downstream indexes past the key range.
// Key words: the sorted word is key | (pc & lowmask) << SYZ_KEY_BITS
// (common.h), the PC's low kshift bits riding above the key bits as payload
// (the digits never read them).  Unique compares whole words, i.e. PCs, so
// two PCs that share a key both stay; Minimize checks every word against the
// universe (minimize_range.hip, key mode).
constexpr int KB = 11;
constexpr uint32_t KEY_BITS = SYZ_KEY_BITS;   // keys < 2^22 here: two 11-bit digits
constexpr uint32_t KEY_MASK = SYZ_KEY_MASK;
constexpr uint32_t KWORDS = 1u << (KB - 1);  // 2048 u16 bins in 1024 words

__device__ __forceinline__ uint32_t hinc(uint32_t d) { return 1u << ((d & 1u) << 4); }

// hist16_scan / hist16_zero: common.h (shared with dedup.hip's radix kernel)

// Gapped key words (the sort's register/LDS form in canon_key_kernel): the
// 22-bit key's digits 12 bits apart, lo11 | hi11 << 12, and the PC's low bits
// at bit 26 as in the output word (common.h), so that the output word is one
// shift and one bit-field insert away (ungap_word).  A real key's 12-bit digit
// (k >> sh) & 4095 (sh 0 or 12) is its 11-bit digit; a PAD slot's word has
// digit 2048 + 2l in both passes, whose histogram word KWORDS + l is its
// lane's private dummy: pads need no per-slot select in the count and scatter
// loops (they rank on the dummy, which starts each scatter at CAP, so they
// land past the real keys).
__device__ __forceinline__ uint32_t gap_key(uint32_t key, uint32_t low) {
    return key + (key & ~2047u) + (low << SYZ_KEY_BITS);  // key < 2^22
}
// D12 (keys < 2^23): the high digit has 12 bits (bits 12-23 of the gapped
// word, 4096 bins in 2048 words); a pad's high field is 4096 + 2l (bit 24), so
// its dummy word is 2048 + l
template <bool D12 = false>
__device__ __forceinline__ uint32_t pad_word(uint32_t l) {
    const uint32_t d = 2048u + 2u * l;
    return d | ((D12 ? 4096u + 2u * l : d) << 12);
}
// the key word of common.h (key | low << SYZ_KEY_BITS) of a gapped word: bits
// 0-10 and 25-31 stay, bits 12-25 move down by one (bits 23-25 are zero)
__device__ __forceinline__ uint32_t ungap_word(uint32_t g) {
    constexpr uint32_t KEEP = 0x7FFu | (0x7Fu << 25);
    return (g & KEEP) | ((g >> 1) & ~KEEP);  // one v_bfi_b32
}
constexpr uint32_t GAP_KEY_MASK = 2047u | (2047u << 12);
constexpr uint32_t GAP_KEY_MASK12 = 2047u | (4095u << 12);
static_assert(SYZ_KEY_BITS == 26, "gapped words keep the low bits in place");

// the histogram word of digit field x (bins 2w, 2w + 1 share word w): one
// bit-field extract and one shift-add (the compiler rewrites a constant
// extract as (x << 1) & 0x1FFC plus the base, three operations)
template <int WB = 11>
__device__ __forceinline__ uint32_t *pair_word(uint32_t *h, uint32_t x) {
    uint32_t w;
    if (WB == 12)
        asm("v_bfe_u32 %0, %1, 1, 12" : "=v"(w) : "v"(x));
    else
        asm("v_bfe_u32 %0, %1, 1, 11" : "=v"(w) : "v"(x));
    return &h[w];
}

// count / rank+scatter over gapped words: no validity tests (pads carry
// their lane's dummy digit).  Inactive row quads hold pads too.  The bin
// pair's half is selected by hs = digit << 4: shifts and v_bfe_u32 read only
// its low 5 bits, (digit & 1) << 4.
template <int NK, int WB = 11>
__device__ __forceinline__ void count_gap(const uint32_t (&k)[NK], uint32_t nq, uint32_t *h,
                                          uint32_t sh) {
    constexpr int NQ = NK / 4;
#pragma unroll
    for (int q = 0; q < NQ; q++)
        if ((uint32_t)q < nq) {
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const uint32_t x = k[q * 4 + c] >> sh;
                atomicAdd(pair_word<WB>(h, x), 1u << ((x << 4) & 31u));
            }
        }
}

template <int NK, int BQ = SYZ_CANON_BQ, int WB = 11>
__device__ __forceinline__ void scatter_gap(const uint32_t (&k)[NK], uint32_t nq, uint32_t *buf,
                                            uint32_t *h, uint32_t sh) {
    constexpr int NQ = NK / 4;
#pragma unroll
    for (int q0 = 0; q0 < NQ; q0 += BQ) {
        if ((uint32_t)q0 >= nq) continue;
        uint32_t r[4 * BQ];
        // (a last batch may be partial: NQ need not be a multiple of BQ)
#pragma unroll
        for (int j = 0; j < 4 * BQ; j++) {
            if (q0 * 4 + j >= NK) break;
            const uint32_t x = k[q0 * 4 + j] >> sh;
            r[j] = atomicAdd(pair_word<WB>(h, x), 1u << ((x << 4) & 31u));
        }
        // every rank atomic of the batch is in flight before the first result
        // is used (interleaved, the extracts waited on each atomic in turn)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 4 * BQ; j++) {
            if (q0 * 4 + j >= NK) break;
            const uint32_t hs = (k[q0 * 4 + j] >> sh) << 4;
            buf[__builtin_amdgcn_ubfe(r[j], hs, 16)] = k[q0 * 4 + j];  // offset = hs & 31
        }
    }
}


template <int NK, int MINW, bool ALIGNED = false, int BQK = ALIGNED ? SYZ_CANON_BQ_AL : SYZ_CANON_BQK,
          bool D12 = false>
__global__ __launch_bounds__(64 * WPB, MINW) void canon_key_kernel(Params P, const uint32_t *list,
                                                                   const uint32_t *count) {
    constexpr uint32_t HW = D12 ? 2 * KWORDS : KWORDS;  // the high pass's histogram words
    constexpr int HQ = D12 ? 8 : 4, HB = D12 ? 12 : 11;
    constexpr uint32_t GMASK = D12 ? GAP_KEY_MASK12 : GAP_KEY_MASK;
    constexpr int CAP = 64 * NK;
    constexpr int NQ = NK / 4;
    __shared__ uint32_t s_buf[WPB][CAP + NK];  // + the lane's pads (<= NK) past CAP
    __shared__ __attribute__((aligned(16))) uint32_t s_h[WPB][HW + 64];
    const uint32_t w = wave_readfirstlane(threadIdx.x >> 6);
    const uint32_t l = __lane_id();
    uint32_t *buf = s_buf[w];
    uint32_t *h = s_h[w];
    const uint32_t span_m1 = (uint32_t)(P.span - 1);
    const uint32_t kmax = (uint32_t)(P.nkeys - 1);
    const bool inplace = P.out == P.raw;
    const uint32_t pad = pad_word<D12>(l);
    // the previous word of slot 0: the sentinel's key word (cover.go:31,
    // `last := sent`), gapped; ~0 never equals a gapped word
    const uint32_t sent_g = P.sent_key == 0xFFFFFFFFu
                                ? 0xFFFFFFFFu
                                : gap_key(P.sent_key & SYZ_KEY_MASK, P.sent_key >> SYZ_KEY_BITS);
    uint32_t racc[MAX_RPL];
#pragma unroll
    for (int q = 0; q < MAX_RPL; q++) racc[q] = 0;
    const uint32_t nl = *count;
    const uint32_t nw = gridDim.x * WPB;
    uint4 vn[NQ];
    uint32_t seg_n = 0, n_n = 0;
    uint64_t base_n = 0;
    auto issue = [&](uint32_t li_) {
        seg_n = list[li_];
        base_n = P.off[seg_n];
        n_n = (uint32_t)(P.off[seg_n + 1] - base_n);
        const uint64_t a0 = base_n & ~3ull;
        const uint32_t end = (uint32_t)(base_n - a0) + n_n;
        const uint4 *src = reinterpret_cast<const uint4 *>(P.raw + a0);
        // every row quad, straight-line (the conversion below is branch-free
        // and reads them all); chunks past the end re-read chunk 0
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            const uint32_t e4 = (uint32_t)(q * 64 + l) * 4u;
            vn[q] = src[e4 < end ? q * 64 + l : 0];
        }
    };
    uint32_t li = blockIdx.x * WPB + w;
    if (li < nl) issue(li);
    for (; li < nl; li += nw) {
        // the descriptor is wave-uniform: scalar registers, so the output
        // pointer is not re-read from a VGPR (v_readfirstlane + s_nop) per store
        age_prio<0>();
        const uint32_t seg = uniform_u32(seg_n);
        const uint64_t base = uniform_u64(base_n);
        const uint32_t n = uniform_u32(n_n);
        const uint64_t a0 = base & ~3ull;
        const uint32_t head = (uint32_t)(base - a0), end = head + n;
        // (an empty segment sorts nothing: with an unaligned start its one row
        // quad would hold only pads, which the unique loop would keep)
        const uint32_t nq = n ? (end + 255) >> 8 : 0u;
        // gapped words, branch-free; slots outside the segment are pads
        // (slot (q, l, c) holds raw index 4 (64 q + l) + c - head)
        // (a slot is real iff head <= 4 (64 q + l) + c < end: the upper bound
        // is one signed compare against a uniform value, the lower one only
        // concerns lane 0's first row quad)
        uint32_t k[NK];
        bool oob = false;
        const int l4 = (int)(4u * l);
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            const uint32_t vv[4] = {vn[q].x, vn[q].y, vn[q].z, vn[q].w};
#pragma unroll
            for (int c = 0; c < 4; c++) {
                bool valid = l4 < (int)end - (256 * q + c);
                if (q == 0 && c < 3) valid &= l4 + c >= (int)head;
                const bool out = vv[c] - P.pc_lo > span_m1;
                oob |= valid & out;
                // an out-of-window word sorts as the last key (its low bits
                // are kept: the step fails on SYZCOV_ERR_WINDOW anyway)
                const uint32_t g = gap_key(out ? kmax : (vv[c] >> P.kshift) - P.kbase,
                                           vv[c] & P.lowmask);
                k[q * 4 + c] = valid ? g : pad;
                // materialised here: sunk into the count loop, the selects kept
                // every slot's masks alive (SGPR spills through VGPR lanes)
                asm volatile("" : "+v"(k[q * 4 + c]));
            }
        }
        // (before the next segment's loads: deferred, the slots' masks stayed alive)
        if (__builtin_amdgcn_ballot_w64(oob) && l == 0) atomicOr(P.err, SYZCOV_ERR_WINDOW);
        if (li + nw < nl) issue(li + nw);
        age_prio<1>();
        // ---------------------------------------- pass 0: low 11 bits
        hist16_zero<NQ>(h, l);
        wave_sync();
        count_gap<NK>(k, nq, h, 0);
        wave_sync();
        hist16_scan(h, l);
        h[KWORDS + l] = CAP;  // the lane's pads rank from CAP on
        wave_sync();
        scatter_gap<NK, BQK>(k, nq, buf, h, 0);
        wave_sync();
        // slots [n, 256 nq) are read back by pass 1: pads of the reading lane
        // (fewer than 260 slots: at most 5 per lane, unrolled)
#pragma unroll
        for (uint32_t t = 0; t < 5; t++) {
            const uint32_t p = (n & ~63u) + l + 64 * t;
            if (p >= n && p < nq * 256u) buf[p] = pad;
        }
        wave_sync();
        // ---------------------------- pass 1: high 11 bits, stable (row-major)
        age_prio<2>();
#pragma unroll
        for (int q = 0; q < NQ; q++)
            if ((uint32_t)q < nq) {
#pragma unroll
                for (int c = 0; c < 4; c++) k[q * 4 + c] = buf[(q * 4 + c) * 64 + l];
            }
        hist16_zero<NQ, HQ>(h, l);
        wave_sync();
        count_gap<NK, HB>(k, nq, h, 12);
        wave_sync();
        hist16_scan<HQ>(h, l);
        h[HW + l] = CAP;
        wave_sync();
        scatter_gap<NK, BQK, HB>(k, nq, buf, h, 12);
        wave_sync();
        age_prio<3>();
        // slots [n, 256 nq) take the last key: the unique loop drops them as
        // repeats and the order check passes them, with no per-slot bound test
        if (n) {
            const uint32_t last = buf[n - 1];  // (not among the slots written)
#pragma unroll
            for (uint32_t t = 0; t < 5; t++) {
                const uint32_t p = (n & ~63u) + l + 64 * t;
                if (p >= n && p < nq * 256u) buf[p] = last;
            }
            wave_sync();
        }
        // --------------------------------- order check + unique + write
#pragma unroll
        for (int q = 0; q < NQ; q++)
            if ((uint32_t)q < nq) {
#pragma unroll
                for (int c = 0; c < 4; c++) k[q * 4 + c] = buf[(q * 4 + c) * 64 + l];
            }
        bool bad = P.force_redo != 0;
        // a slot's predecessor words: the slot rotated up one lane, lane 0 taking
        // the previous slot's rotated word (its lane 63) — two VALU operations,
        // where a shift with the carry read out by v_readlane took three
        const bool lane0 = l == 0;
        if (inplace) {  // nothing may be written before the order is known
            uint32_t rprev = sent_g;
#pragma unroll
            for (int q = 0; q < NQ; q++)
                if ((uint32_t)q < nq) {
#pragma unroll
                    for (int c = 0; c < 4; c++) {
                        const uint32_t v = k[q * 4 + c];
                        const uint32_t r = rotate_up(v);
                        const uint32_t prev = lane0 ? rprev : r;
                        rprev = r;
                        // (slot 0's predecessor is the sentinel: no order)
                        bad |= ((v & GMASK) < (prev & GMASK)) & (q + c > 0 || l > 0);
                    }
                }
            if (__ballot(bad)) {
                if (l == 0) P.redo_list[atomicAdd(P.redo_cnt, 1u)] = seg;
                continue;
            }
        }
        uint32_t cnt = 0, rprev = sent_g, dcar = 0;
        uint32_t *outp = P.out + aligned_base(base, seg, P.ak);
        // line-aligned: each kept word straight to its aligned sub-run (the
        // range transitions of a row by one ballot, aligned_delta), or with
        // SYZ_CANON_AL_COPY from buf after the split search (round 5's form)
#ifdef SYZ_CANON_AL_COPY
        constexpr bool direct = !ALIGNED;
        constexpr bool al_direct = false;
#else
        constexpr bool direct = true;
        constexpr bool al_direct = ALIGNED;
#endif
        // a gapped word's range: key bits rshift.. sit one bit higher (bits 12+)
        const uint32_t rsh1 = P.rshift + 1;
        const uint32_t rmask = (GMASK >> rsh1) << rsh1;
#pragma unroll
        for (int q = 0; q < NQ; q++)
            if ((uint32_t)q < nq) {
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    const uint32_t v = k[q * 4 + c];
                    const uint32_t r = rotate_up(v);
                    const uint32_t prev = lane0 ? rprev : r;
                    rprev = r;
                    bad |= ((v & GMASK) < (prev & GMASK)) & (q + c > 0 || l > 0);
                    // whole words: distinct PCs stay distinct even if they share a key
                    const bool keep = v != prev;
                    const uint64_t m = __builtin_amdgcn_ballot_w64(keep);
                    const uint32_t pos = cnt + __builtin_amdgcn_mbcnt_hi(
                                                   (uint32_t)(m >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    uint32_t delta = dcar;
                    if (al_direct) {
                        // a range starts where a kept word's range bits differ
                        // from its predecessor's (a non-kept slot repeats the
                        // previous kept word); the segment's first word always
                        const bool st = keep & ((((v ^ prev) & rmask) != 0u) |
                                                (q == 0 && c == 0 && lane0));
                        uint64_t sm = __builtin_amdgcn_ballot_w64(st);
                        while (sm) {  // uniform; about one start per row of 64
                            const uint32_t b = (uint32_t)__builtin_ctzll(sm);
                            sm &= sm - 1;
                            const uint32_t pb = wave_readlane(pos, (int)b);
                            const uint32_t jb = ((wave_readlane(v, (int)b) & GMASK) >> rsh1);
                            const uint32_t db = aligned_sub(pb, jb, P.ak) - pb;
                            delta = l >= b ? db : delta;
                            dcar = db;
                        }
                    }
                    if (keep) {
                        const uint32_t w = ungap_word(v);
                        // the key word: the PC is kept exactly
                        if (direct) outp[pos + (al_direct ? delta : 0u)] = w;
                        buf[pos] = w;  // (the split search masks the key)
                    }
                    cnt += (uint32_t)__popcll(m);
                }
            }
        if (__ballot(bad)) {
            if (l == 0) P.redo_list[atomicAdd(P.redo_cnt, 1u)] = seg;
            continue;
        }
        if (l == 0) P.new_len[seg] = cnt;
        if (!P.split) {
            if (l == 0) racc[0] += cnt;
        } else {
            wave_sync();
            uint32_t carry2 = 0;
            uint32_t *sp = P.split + (uint64_t)seg * P.nrange;
#pragma unroll
            for (int q = 0; q < MAX_RPL; q++) {
                const uint32_t j = q * 64 + l;
                if (q * 64 < (int)P.nrange) {
                    uint32_t s2 = cnt;
                    if (j + 1 < P.nrange) {
                        const uint32_t b = (j + 1) << P.rshift;  // keys below range j + 1
                        uint32_t lo2 = 0, hi2 = cnt;
                        while (lo2 < hi2) {
                            const uint32_t mid = (lo2 + hi2) >> 1;
                            if ((buf[mid] & KEY_MASK) < b) lo2 = mid + 1; else hi2 = mid;
                        }
                        s2 = lo2;
                    }
                    const uint32_t prev_s = __shfl_up(s2, 1, 64);
                    const uint32_t sprev = l == 0 ? carry2 : prev_s;  // keys below range j
                    const uint32_t c2 = s2 - sprev;
                    carry2 = __shfl(s2, 63, 64);
                    if (j < P.nrange) {
                        sp[j] = s2;
                        racc[q] += c2;
                        // line-aligned: range j's words move up by this much (the
                        // histogram is free once the sort is done)
                        if (!direct) h[j] = aligned_sub(sprev, j, P.ak) - sprev;
                    }
                }
            }
            if (!direct) {  // the sorted words from buf to their aligned sub-runs
                wave_sync();
                for (uint32_t p0 = 0; p0 < cnt; p0 += 64) {
                    const uint32_t p = p0 + l;
                    if (p < cnt) {
                        const uint32_t w = buf[p];
                        outp[p + h[(w & KEY_MASK) >> P.rshift]] = w;
                    }
                }
            }
        }
    }
    if (P.range_tot) {
#pragma unroll
        for (int q = 0; q < MAX_RPL; q++) {
            const uint32_t j = q * 64 + l;
            if (j < P.nrange && racc[q]) atomicAdd(&P.range_tot[j], (unsigned long long)racc[q]);
        }
    }
}

// Splits + range totals of listed segments (fallback / long paths), from the
// canonical lists already in `out`.  One wave per listed segment.
__global__ __launch_bounds__(64) void split_list_kernel(Params P, const uint32_t *list,
                                                        const uint32_t *count, int big_only) {
    const uint32_t l = __lane_id();
    const uint32_t nl = *count;
    for (uint32_t li = blockIdx.x; li < nl; li += gridDim.x) {
        const uint32_t seg = list[li];
        if (big_only && P.off[seg + 1] - P.off[seg] <= WAVE_MAX) continue;
        const uint32_t *c = P.out + aligned_base(P.off[seg], seg, P.ak);  // contiguous still
        const uint32_t cnt = P.new_len[seg];
        uint32_t carry = 0;
        for (uint32_t jb = 0; jb < P.nrange; jb += 64) {
            const uint32_t j = jb + l;
            uint32_t s = cnt;
            if (j + 1 < P.nrange) {
                const uint32_t b = (j + 1) << P.rshift;
                uint32_t lo = 0, hi = cnt;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    const uint32_t x = P.key_out ? c[mid] & SYZ_KEY_MASK : c[mid] - P.pc_lo;
                    if (x < b) lo = mid + 1; else hi = mid;
                }
                s = lo;
            }
            const uint32_t prev_s = __shfl_up(s, 1, 64);
            const uint32_t cc = s - (l == 0 ? carry : prev_s);
            carry = __shfl(s, 63, 64);
            if (j < P.nrange) {
                P.split[(uint64_t)seg * P.nrange + j] = s;
                if (P.range_tot && cc) atomicAdd(&P.range_tot[j], (unsigned long long)cc);
            }
        }
    }
}

// Segments canonicalized by the workgroup paths (canon.hip) hold PCs: check
// them against the key range and, in key mode, turn them into keys (in place)
// before their split points are taken.  A key outside [0, span) sets
// SYZCOV_ERR_WINDOW and drops the segment, so Minimize never indexes past the
// range (the wave path drops such keys itself).
__global__ __launch_bounds__(64) void keyify_list_kernel(Params P, const uint32_t *list,
                                                         const uint32_t *count, int big_only) {
    const uint32_t nl = *count;
    for (uint32_t li = blockIdx.x; li < nl; li += gridDim.x) {
        const uint32_t seg = list[li];
        if (big_only && P.off[seg + 1] - P.off[seg] <= WAVE_MAX) continue;
        uint32_t *c = P.out + aligned_base(P.off[seg], seg, P.ak);
        const uint32_t cnt = P.new_len[seg];
        bool bad = false;
        for (uint32_t i = __lane_id(); i < cnt; i += 64) {
            const uint32_t pc = c[i];
            const bool out = pc - P.pc_lo > (uint32_t)(P.span - 1);
            bad |= out;
            if (P.key_out && !out) c[i] = key_word(pc, P.kshift, P.kbase);
        }
        if (__ballot(bad)) {  // flagged; the segment is dropped (memory-safe downstream)
            if (__lane_id() == 0) {
                atomicOr(P.err, SYZCOV_ERR_WINDOW);
                P.new_len[seg] = 0;
            }
        }
    }
}

// The workgroup paths write a segment contiguously at its line-aligned base;
// once its split points are known its range sub-runs move up to their aligned
// starts (common.h), in place: every word moves to an equal or higher index,
// so the ranges go last to first and each range's words top chunk first, the
// whole chunk read before any of it is written (a workgroup per segment).
__global__ __launch_bounds__(256) void spread_list_kernel(Params P, const uint32_t *list,
                                                          const uint32_t *count, int big_only) {
    const uint32_t nl = *count;
    for (uint32_t li = blockIdx.x; li < nl; li += gridDim.x) {
        const uint32_t seg = list[li];
        if (big_only && P.off[seg + 1] - P.off[seg] <= WAVE_MAX) continue;
        uint32_t *c = P.out + aligned_base(P.off[seg], seg, P.ak);
        const uint32_t *sp = P.split + (uint64_t)seg * P.nrange;
        for (int j = (int)P.nrange - 1; j > 0; j--) {
            const uint32_t s0 = sp[j - 1], s1 = sp[j];
            const uint32_t d = aligned_sub(s0, (uint32_t)j, P.ak) - s0;
            if (s1 == s0 || d == 0) continue;
            for (uint32_t top = s1; top > s0;) {
                const uint32_t lo = top - s0 > blockDim.x ? top - blockDim.x : s0;
                const uint32_t i = lo + threadIdx.x;
                uint32_t v = 0;
                if (i < top) v = c[i];
                __syncthreads();
                if (i < top) c[i + d] = v;
                __syncthreads();
                top = lo;
            }
        }
    }
}

}  // namespace cw
}  // namespace syz

using namespace syz;

// Workgroups that fit on the whole chip at once for a class kernel: the grid
// is never larger, so every wave owns an equal share of the class (+-1
// segment) instead of a fixed 1/4096 of it run in 2-3 partly empty rounds.
template <int NK, int MW, int HB>
static unsigned resident_grid(uint64_t nseg) {
    static unsigned cap = 0;
    if (!cap) {
        int dev = 0, ncu = 256, nb = 0;
        if (hipGetDevice(&dev) == hipSuccess) {
            hipDeviceProp_t pr;
            if (hipGetDeviceProperties(&pr, dev) == hipSuccess) ncu = pr.multiProcessorCount;
        }
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &nb, reinterpret_cast<const void *>(cw::canon_wave_kernel<NK, MW, HB>), 64 * cw::WPB,
                0) != hipSuccess || nb < 1)
            nb = 1;
        cap = (unsigned)(nb * ncu);
    }
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((nseg + cw::WPB - 1) / cw::WPB, cap));
}

template <int NK, int MW, bool AL, bool D12 = false>
static unsigned resident_grid_key(uint64_t nseg) {
    static unsigned cap = 0;
    if (!cap) {
        int dev = 0, ncu = 256, nb = 0;
        if (hipGetDevice(&dev) == hipSuccess) {
            hipDeviceProp_t pr;
            if (hipGetDeviceProperties(&pr, dev) == hipSuccess) ncu = pr.multiProcessorCount;
        }
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &nb, reinterpret_cast<const void *>(
                         cw::canon_key_kernel<NK, MW, AL, AL ? SYZ_CANON_BQ_AL : SYZ_CANON_BQK, D12>),
                64 * cw::WPB, 0) != hipSuccess || nb < 1)
            nb = 1;
        cap = (unsigned)(nb * ncu);
    }
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((nseg + cw::WPB - 1) / cw::WPB, cap));
}

template <int NK, int MW>
static void launch_key_class(const cw::Params &P, const uint32_t *lc, const uint32_t *cnt,
                             uint64_t nseg, hipStream_t s) {
    // keys < 2^23: a 12-bit high digit (its 8.4 KB histogram leaves LDS for
    // at most 2 waves per SIMD, so that is the register budget too)
    constexpr int MW12 = MW > 2 ? 2 : MW;
    if (P.nkeys > (1ull << 22) && !P.ak)
        hipLaunchKernelGGL((cw::canon_key_kernel<NK, MW12, false, SYZ_CANON_BQK, true>),
                           dim3(resident_grid_key<NK, MW12, false, true>(nseg)), dim3(64 * cw::WPB),
                           0, s, P, lc, cnt);
    else if (P.ak)  // line-aligned sub-runs: a separate build of the kernel (no per-word branch)
        hipLaunchKernelGGL((cw::canon_key_kernel<NK, MW, true>),
                           dim3(resident_grid_key<NK, MW, true>(nseg)), dim3(64 * cw::WPB), 0, s,
                           P, lc, cnt);
    else
        hipLaunchKernelGGL((cw::canon_key_kernel<NK, MW, false>),
                           dim3(resident_grid_key<NK, MW, false>(nseg)), dim3(64 * cw::WPB), 0,
                           s, P, lc, cnt);
}

extern "C" size_t syzcov_dev_canon_split_ws_size(size_t nseg) {
    // counters | redo list | big list | class lists
    return 256 + (2 + cw::NCLS) * align_up(nseg * sizeof(uint32_t), 256);
}

// One class launch of the 3-pass sort (9-bit digits; window mode, or key
// spaces above 2^22).  (2 passes of 11-bit digits with packed u32 histograms
// measured 9.45 vs 7.9 ms at C2: 8 KB histograms halve the resident waves; the
// key mode's 2-pass sort holds them as u16 pairs instead, canon_key_kernel.)
template <int NK, int MW>
static void launch_class(const cw::Params &P, const uint32_t *lc, const uint32_t *cnt,
                         uint64_t nseg, hipStream_t s) {
    hipLaunchKernelGGL((cw::canon_wave_kernel<NK, MW, 9>), dim3(resident_grid<NK, MW, 9>(nseg)),
                       dim3(64 * cw::WPB), 0, s, P, lc, cnt);
}

static int canon_split_impl(const uint64_t *off, const uint32_t *raw, uint32_t *out,
                            uint32_t *new_len, size_t nseg, size_t max_seg_len, uint32_t pc_lo,
                            uint64_t pc_span, uint32_t kshift, uint32_t kbase, uint64_t nkeys,
                            int key_out, uint32_t range_shift,
                            uint32_t *split,
                            uint64_t *range_tot, uint32_t *err_flag, void *ws, size_t ws_size,
                            void *stream, int aligned = 0) {
    if (nseg == 0) return 0;
    if (!off || !raw || !out || !new_len || !err_flag || !ws) return SYZCOV_EINVAL;
    if (pc_span == 0 || pc_span > (1ull << 32) || (uint64_t)pc_lo + pc_span > (1ull << 32))
        return SYZCOV_ERANGE;
    if (key_out) {  // every window PC must map into [0, nkeys)
        // key words (common.h): keys < 2^25, the low bits above them
        if (kshift > SYZCOV_KSHIFT_MAX || nkeys > (1ull << 25)) return SYZCOV_EINVAL;
        const uint64_t k0 = pc_lo >> kshift, k1 = (pc_lo + pc_span - 1) >> kshift;
        if (nkeys == 0 || k0 < kbase || k1 - kbase >= nkeys) return SYZCOV_ERANGE;
    } else {
        nkeys = pc_span;
    }
    if (ws_size < syzcov_dev_canon_split_ws_size(nseg) || nseg > 0xFFFFFFFFull)
        return SYZCOV_EINVAL;
    if (out == raw && max_seg_len > 16384) return SYZCOV_EINVAL;  // large path is out of place
    if (range_shift > 20) return SYZCOV_EINVAL;
    const uint64_t nrange = (nkeys + (1ull << range_shift) - 1) >> range_shift;
    if (split && nrange > (uint64_t)cw::MAX_RPL * 64) return SYZCOV_ERANGE;
    // the line-aligned layout needs the split points and its own buffer
    if (aligned && (!split || out == raw)) return SYZCOV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    uint8_t *w = (uint8_t *)ws;
    uint32_t *cnts = (uint32_t *)w;  // [0] redo, [1] big, [2..] classes
    uint32_t *redo = (uint32_t *)(w + 256);
    uint32_t *big = (uint32_t *)(w + 256 + align_up(nseg * sizeof(uint32_t), 256));
    SYZ_HIP(hipMemsetAsync(cnts, 0, 2 * sizeof(uint32_t), s));
    cw::Params P{};
    P.off = off;
    P.raw = raw;
    P.out = out;
    P.new_len = new_len;
    P.nseg = nseg;
    P.pc_lo = pc_lo;
    P.span = pc_span;
    P.kshift = kshift;
    P.kbase = kbase;
    P.nkeys = nkeys;
    P.key_out = key_out;
    P.lowmask = (1u << kshift) - 1u;
    P.nbits = pc_span <= 1 ? 1 : 64 - __builtin_clzll(pc_span - 1);
    const uint64_t so = (uint64_t)(uint32_t)(0xFFFFFFFFu - pc_lo);
    P.sent_key = so < pc_span ? (uint32_t)so : 0xFFFFFFFFu;
    P.split = split;
    P.nrange = (uint32_t)nrange;
    P.rshift = range_shift;
    P.range_tot = (unsigned long long *)range_tot;
    P.redo_list = redo;
    P.redo_cnt = cnts;
    P.big_list = big;
    P.big_cnt = cnts + 1;
    P.err = err_flag;
    // key mode over <= 2^22 keys: sort the keys themselves, 2 passes of 11
    // bits with u16-pair histograms (canon_key_kernel).  C2 canon ms: 8.03 with
    // the 3-pass window-offset sort in every class, 7.66 with the key sort in
    // the 2048-key class only, 7.23 in every class once the scatter batches
    // were branch-free (3072 keys run at 2 waves per SIMD: 48 keys per lane do
    // not fit 168 VGPRs).  SYZ_CANON_KEY2=0 builds keep the 3-pass sort.
#ifndef SYZ_CANON_KEY2
#define SYZ_CANON_KEY2 2
#endif
    const uint32_t force = force_flags();
    // 2 passes: 11 + 11 bits up to 2^22 keys, 11 + 12 (CSR) up to 2^23
    const int key2 = (key_out && !(force & FORCE_CANON3) &&
                      (nkeys <= (1ull << 22) || (nkeys <= (1ull << 23) && !aligned)))
                         ? SYZ_CANON_KEY2
                         : 0;
    P.force_redo = (force & FORCE_REDO) ? 1u : 0u;
    P.ak = aligned ? SYZ_ALIGN_K((uint32_t)nrange) : 0u;
    cw::Params PK = P;  // the key kernel's unique loop compares (key | low bits) words
    PK.sent_key = so < pc_span ? ((0xFFFFFFFFu >> kshift) - kbase) | (P.lowmask << cw::KEY_BITS)
                               : 0xFFFFFFFFu;  // a word's key is < 2^25: never equal
    // bin by capacity class (wave-aggregated atomics), one launch per class
    // (a register bitonic network measured 20.3 ms at C2 against the LDS
    // radix's 7.8: 147 VALU ops per key)
    cw::Classes C;
    // (a 1024-key class for the segments of <= 1021 keys measured slower than
    // sending them to the 2048-key class: 7.85 vs 7.79 ms at C2; its short
    // kernel was mostly ramp and tail)
    const uint32_t nk[cw::NCLS] = {32, 40, 48, 64, 128};
    for (int c = 0; c < cw::NCLS; c++) {
        C.lo[c] = c ? nk[c - 1] * 64 - 2 : 0;  // CAP - 3 + 1 of the previous class
        C.hi[c] = nk[c] * 64 - 3;
    }
    uint32_t *clists = (uint32_t *)(w + 256 + 2 * align_up(nseg * sizeof(uint32_t), 256));
    uint32_t *ccnt = cnts + 2;
    SYZ_HIP(hipMemsetAsync(ccnt, 0, cw::NCLS * sizeof(uint32_t), s));
    hipLaunchKernelGGL(cw::bin_kernel, dim3(grid_for(nseg, 256 * cw::BIN_K, 2048)), dim3(256), 0, s, off,
                       (uint64_t)nseg, C, ccnt, clists, (uint64_t)nseg, big, cnts + 1,
                       (uint64_t)max_seg_len, err_flag);
    for (int c = 0; c < cw::NCLS; c++) {
        if (max_seg_len < C.lo[c]) break;
        const uint32_t *lc = clists + (size_t)c * nseg;
        if (key2 == 2 || (key2 == 1 && c == 0)) {
            switch (c) {
            case 0: launch_key_class<32, SYZ_CANON_W32>(PK, lc, ccnt + c, nseg, s); break;
            case 1: launch_key_class<40, SYZ_CANON_W40>(PK, lc, ccnt + c, nseg, s); break;
            case 2: launch_key_class<48, 2>(PK, lc, ccnt + c, nseg, s); break;  // 168 VGPRs do not fit
            case 3: launch_key_class<64, 2>(PK, lc, ccnt + c, nseg, s); break;
            case 4: launch_key_class<128, 1>(PK, lc, ccnt + c, nseg, s); break;
            }
        } else {
            switch (c) {
            case 0: launch_class<32, SYZ_CANON_W32>(P, lc, ccnt + c, nseg, s); break;
            case 1: launch_class<40, SYZ_CANON_W40>(P, lc, ccnt + c, nseg, s); break;
            case 2: launch_class<48, SYZ_CANON_W48>(P, lc, ccnt + c, nseg, s); break;
            case 3: launch_class<64, 2>(P, lc, ccnt + c, nseg, s); break;
            case 4: launch_class<128, 1>(P, lc, ccnt + c, nseg, s); break;
            }
        }
        SYZ_LAUNCH_CHECK();
    }
    // the workgroup paths write PCs: keys for them in key mode, then splits
    auto finish_list = [&](const uint32_t *list, const uint32_t *cnt, int big_only,
                           unsigned grid) {
        hipLaunchKernelGGL(cw::keyify_list_kernel, dim3(grid), dim3(64), 0, s, P, list, cnt,
                           big_only);
        if (split)
            hipLaunchKernelGGL(cw::split_list_kernel, dim3(grid), dim3(64), 0, s, P, list, cnt,
                               big_only);
        if (P.ak)
            hipLaunchKernelGGL(cw::spread_list_kernel, dim3(grid), dim3(256), 0, s, P, list, cnt,
                               big_only);
    };
    // segments whose wave sort failed the order check (not expected on gfx950)
    int rc = canon_list_path(off, raw, out, new_len, redo, cnts, s, P.ak);
    if (rc) return rc;
    finish_list(redo, cnts, 0, 64);
    if (max_seg_len > cw::WAVE_MAX) {
        if (max_seg_len <= 16384) {
            rc = canon_list_path(off, raw, out, new_len, big, cnts + 1, s, P.ak);
            if (rc) return rc;
        } else {
            uint32_t nbig = 0;
            SYZ_HIP(hipMemcpyAsync(&nbig, cnts + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
            SYZ_HIP(hipStreamSynchronize(s));
            if (nbig) {
                // the window is checked by keyify_list_kernel
                rc = canon_large_path(off, raw, out, new_len, big, nbig, nullptr, pc_lo,
                                      pc_span, err_flag, s, P.ak);
                if (rc) return rc;
            }
        }
        finish_list(big, cnts + 1, 1, 256);
    }
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" int syzcov_dev_canon_split(const uint64_t *off, const uint32_t *raw, uint32_t *out,
                                      uint32_t *new_len, size_t nseg, size_t max_seg_len,
                                      uint32_t pc_lo, uint64_t pc_span, uint32_t range_shift,
                                      uint32_t *split, uint64_t *range_tot, uint32_t *err_flag,
                                      void *ws, size_t ws_size, void *stream) {
    return canon_split_impl(off, raw, out, new_len, nseg, max_seg_len, pc_lo, pc_span, 0, pc_lo,
                            pc_span, 0, range_shift, split, range_tot, err_flag, ws, ws_size,
                            stream);
}

extern "C" int syzcov_dev_canon_split_keys(const uint64_t *off, const uint32_t *raw, uint32_t *out,
                                           uint32_t *new_len, size_t nseg, size_t max_seg_len,
                                           uint32_t pc_lo, uint64_t pc_span, uint32_t kshift,
                                           uint32_t kbase, uint64_t nkeys, uint32_t range_shift,
                                           uint32_t *split, uint64_t *range_tot,
                                           uint32_t *err_flag, void *ws, size_t ws_size,
                                           void *stream) {
    return canon_split_impl(off, raw, out, new_len, nseg, max_seg_len, pc_lo, pc_span, kshift,
                            kbase, nkeys, 1, range_shift, split, range_tot, err_flag, ws, ws_size,
                            stream);
}

extern "C" int syzcov_dev_canon_split_aligned(const uint64_t *off, const uint32_t *raw,
                                              uint32_t *out, uint32_t *new_len, size_t nseg,
                                              size_t max_seg_len, uint32_t pc_lo,
                                              uint64_t pc_span, uint32_t kshift, uint32_t kbase,
                                              uint64_t nkeys, int key_out, uint32_t range_shift,
                                              uint32_t *split, uint64_t *range_tot,
                                              uint32_t *err_flag, void *ws, size_t ws_size,
                                              void *stream) {
    return canon_split_impl(off, raw, out, new_len, nseg, max_seg_len, pc_lo, pc_span,
                            key_out ? kshift : 0, key_out ? kbase : pc_lo,
                            key_out ? nkeys : pc_span, key_out ? 1 : 0, range_shift, split,
                            range_tot, err_flag, ws, ws_size, stream, 1);
}

extern "C" uint64_t syzcov_dev_canon_aligned_words(uint64_t p_max, uint64_t nseg,
                                                   uint64_t nrange) {
    return aligned_words(p_max, nseg, SYZ_ALIGN_K((uint32_t)nrange));
}
