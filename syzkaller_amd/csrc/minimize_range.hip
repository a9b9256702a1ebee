// minimize_range.hip — cover.Minimize (cover/cover.go:104-131) as a
// first-cover problem whose per-PC test never leaves LDS.
//
// kept(r) <=> some pc of cov_r has first(pc) == r, first(pc) = min rank
// covering pc.  Items (inputs in rank order) are processed in
// geometrically growing chunks.  Before chunk c, `covered` holds every PC
// whose first cover lies in an earlier chunk; inside the chunk a PC that is
// covered cannot be first for any rank of the chunk, so it costs one LDS bit
// test.  Every uncovered occurrence (rank, pc) is RECORDED and atomicMin-ed
// into first_w[pc - pc_lo]; the first cover of every PC is always recorded
// (nothing before it covers the PC).  Hence, after the last chunk:
//   first_w[pc]  = first(pc) for every recorded pc,
//   covered      = the union of the corpus (the maxCover merge operand),
//   kept(r)      <=> some record (r, pc) has first_w[pc] == r   (pass 2),
// and pass 2 touches only the records (a few per distinct PC), not the corpus.
//
// LDS residency: the PC window is cut into ranges of 2^rshift PCs (128 KB of
// bitmap at rshift 20).  A workgroup owns one range for a slice of the
// chunk's items, loads that range's covered bitmap into LDS, and streams the
// items' sub-runs inside the range (canonical lists are sorted, so a sub-run
// is contiguous: split[] from canon_wave.hip).  Ranges get workgroups in
// proportion to their PC counts (range_tot), so a hot range is cut into many
// short item slices.  Each wave flattens the sub-runs of 64 items into full
// 64-lane rows (a scalar walk over the items starting inside each row) and
// keeps ROWS row loads in flight before it tests them.
//
// Record overflow (more uncovered occurrences than rec_cap, only for
// adversarial corpora) is detected on the device; the fallback kernels then
// rescan candidate items and derive the union from first_w, so the result
// stays exact for every input.
#include "common.h"

#include <algorithm>

namespace syz {
namespace mr {

constexpr int THREADS = 1024;
constexpr int NWAVE = THREADS / 64;
constexpr int ROWS = 16;         // row loads in flight per wave
constexpr int MAX_R = 256;

struct Args {
    const uint64_t *off;
    const uint32_t *len;       // canonical lengths (used when split == NULL)
    const uint32_t *pcs;
    const uint32_t *split;     // [nseg][nrange] or NULL (nrange == 1)
    const int32_t *order;      // item -> local input index
    const int32_t *ranks;      // item -> rank (NULL: item index)
    uint32_t pc_lo;
    uint32_t rshift, nrange;
    const unsigned long long *range_tot;
    const uint32_t *covered;   // window bitmap (nrange << rshift bits)
    int32_t *first_w;          // [span], INT32_MAX outside records
    unsigned long long *rec;   // (rank << 32) | window offset
    uint64_t rec_cap;
    unsigned long long *rec_cnt;  // may exceed rec_cap (overflow)
    uint8_t *cand;             // [items] item had an uncovered PC
    // rank-ordered descriptors (prep_kernel): coalesced per (range, item slice)
    const uint64_t *base_r;    // [items] off[order[j]]
    const uint32_t *split_t;   // [nrange][items] split[order[j]][rho]
    uint32_t n_items;
};

// Gather the items' CSR bases and split columns into rank order, transposed
// so that a workgroup owning range rho reads split_t[rho][i0..i1) contiguously.
__global__ __launch_bounds__(256) void prep_kernel(Args A, uint64_t *base_r, uint32_t *split_t) {
    const uint32_t n = A.n_items;
    for (uint32_t t0 = blockIdx.x * 64; t0 < n; t0 += gridDim.x * 64) {
        const uint32_t j = t0 + (threadIdx.x & 63);
        if (j >= n) continue;
        const uint32_t seg = (uint32_t)A.order[j];
        if (threadIdx.x < 64) base_r[j] = A.off[seg];
        for (uint32_t rho = threadIdx.x >> 6; rho < A.nrange; rho += 4)
            split_t[(uint64_t)rho * n + j] =
                A.split ? A.split[(uint64_t)seg * A.nrange + rho] : A.len[seg];
    }
}

// Workgroup -> (range, item slice [i0, i1)) with pieces proportional to the
// range's weight: p_j = 1 + floor(w_j * (G - R) / W).
__device__ bool piece_of(const Args &A, uint32_t G, uint32_t a, uint32_t b, uint32_t *rho,
                         uint32_t *i0, uint32_t *i1, uint32_t *sh) {
    // sh: LDS scratch of MAX_R + 1 entries; computed by wave 0
    const uint32_t l = __lane_id();
    if (threadIdx.x < 64) {
        unsigned long long wsum = 0;
        for (uint32_t j = l; j < A.nrange; j += 64) wsum += A.range_tot[j];
        for (int d = 32; d >= 1; d >>= 1) wsum += __shfl_xor(wsum, d, 64);
        const uint64_t spare = G > A.nrange ? G - A.nrange : 0;
        uint32_t carry = 0;
        for (uint32_t jb = 0; jb < A.nrange; jb += 64) {
            const uint32_t j = jb + l;
            uint32_t p = 0;
            if (j < A.nrange)  // integer: the pieces never exceed G
                p = 1u + (wsum ? (uint32_t)(A.range_tot[j] * spare / wsum) : 0u);
            const uint32_t inc = wave_incl_scan(p);
            if (j < A.nrange) sh[j + 1] = carry + inc;
            carry += __shfl(inc, 63, 64);
        }
        if (l == 0) sh[0] = 0;
    }
    __syncthreads();
    const uint32_t g = blockIdx.x;
    if (g >= sh[A.nrange]) return false;
    uint32_t lo = 0, hi = A.nrange;  // largest j with sh[j] <= g
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (sh[mid] <= g) lo = mid; else hi = mid;
    }
    const uint32_t p = sh[lo + 1] - sh[lo], q = g - sh[lo];
    const uint64_t n = b - a;
    *rho = lo;
    *i0 = a + (uint32_t)(n * q / p);
    *i1 = a + (uint32_t)(n * (q + 1) / p);
    return true;
}

// Pass 1 over items [a, b) (one chunk).
__global__ __launch_bounds__(THREADS) void pass1_kernel(Args A, uint32_t a, uint32_t b,
                                                        int load_cov) {
    extern __shared__ uint32_t s_cov[];          // (1 << rshift) / 32 words
    __shared__ uint32_t s_plan[MAX_R + 1];
    uint32_t rho, i0, i1;
    if (!piece_of(A, gridDim.x, a, b, &rho, &i0, &i1, s_plan)) return;
    const uint32_t nwords = (1u << A.rshift) >> 5;
    {
        const uint4 *g4 = reinterpret_cast<const uint4 *>(A.covered + (uint64_t)rho * nwords);
        uint4 *s4 = reinterpret_cast<uint4 *>(s_cov);
        if (load_cov) {
            for (uint32_t q = threadIdx.x; q < nwords / 4; q += THREADS) s4[q] = g4[q];
        } else {  // first chunk: nothing is covered yet
            for (uint32_t q = threadIdx.x; q < nwords / 4; q += THREADS)
                s4[q] = make_uint4(0, 0, 0, 0);
        }
    }
    __syncthreads();
    const uint32_t l = __lane_id();
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t lt = (1ull << l) - 1ull;
    const uint32_t rbase = rho << A.rshift;  // window offset of the range
    // the slice is split evenly over the waves, 64 items per batch
    const uint32_t per = (i1 - i0 + NWAVE - 1) / NWAVE;
    const uint32_t w0 = i0 + w * per, w1 = min(i1, w0 + per);
    for (uint32_t ib = w0; ib < w1; ib += 64) {
        // ---- per-lane item descriptor: sub-run of range rho
        const uint32_t item = ib + l;
        uint64_t st = 0;
        uint32_t m = 0;
        int32_t rk = 0;
        if (item < w1) {
            rk = A.ranks ? A.ranks[item] : (int32_t)item;
            const uint32_t s1 = A.split_t[(uint64_t)rho * A.n_items + item];
            const uint32_t s0 = rho ? A.split_t[(uint64_t)(rho - 1) * A.n_items + item] : 0u;
            st = A.base_r[item] + s0;
            m = s1 - s0;
        }
        const uint32_t incl = wave_incl_scan(m);
        const uint32_t pre = incl - m;                      // exclusive prefix
        const uint32_t T = __shfl(incl, 63, 64);            // flattened length
        if (T == 0) continue;
        // per-lane state: item containing flattened element R0 + l
        uint64_t my_st = 0;
        uint32_t my_pre = 0, my_item = 0;
        int32_t my_rk = 0;
        for (uint32_t R0 = 0; R0 < T; R0 += ROWS * 64) {
            uint32_t v[ROWS], ix[ROWS], rkv[ROWS];
            bool act[ROWS];
#pragma unroll
            for (int u = 0; u < ROWS; u++) {
                const uint32_t r0 = R0 + u * 64;
                act[u] = false;
                if (r0 < T) {
                    // carry the item of the previous row's last element
                    my_st = (uint64_t)__builtin_amdgcn_readlane((uint32_t)my_st, 63) |
                            ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(my_st >> 32), 63) << 32);
                    my_pre = __builtin_amdgcn_readlane(my_pre, 63);
                    my_item = __builtin_amdgcn_readlane(my_item, 63);
                    my_rk = __builtin_amdgcn_readlane(my_rk, 63);
                    uint64_t starts = __ballot(m > 0 && pre >= r0 && pre < r0 + 64);
                    while (starts) {
                        const uint32_t i = __builtin_ctzll(starts);
                        starts &= starts - 1;
                        const uint32_t pi = __builtin_amdgcn_readlane(pre, i);
                        if (l >= pi - r0) {
                            my_st = (uint64_t)__builtin_amdgcn_readlane((uint32_t)st, i) |
                                    ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(st >> 32), i) << 32);
                            my_pre = pi;
                            my_item = ib + i;
                            my_rk = __builtin_amdgcn_readlane(rk, i);
                        }
                    }
                    const uint32_t f = r0 + l;
                    act[u] = f < T;
                    ix[u] = my_item;
                    rkv[u] = (uint32_t)my_rk;
                    v[u] = act[u] ? A.pcs[my_st + (f - my_pre)] : 0u;
                }
            }
            // LDS bit tests; one record reservation per batch of ROWS rows
            uint64_t um[ROWS];
            uint32_t nunc = 0;
#pragma unroll
            for (int u = 0; u < ROWS; u++) {
                um[u] = 0;
                if (R0 + u * 64 < T) {
                    const uint32_t bit = act[u] ? v[u] - A.pc_lo - rbase : 0u;  // < 2^rshift
                    const bool unc = act[u] && !((s_cov[bit >> 5] >> (bit & 31)) & 1u);
                    um[u] = __ballot(unc);
                    nunc += (uint32_t)__popcll(um[u]);
                }
            }
            if (nunc) {
                unsigned long long basei = 0;
                if (l == 0) basei = atomicAdd(A.rec_cnt, (unsigned long long)nunc);
                basei = __shfl(basei, 0, 64);
#pragma unroll
                for (int u = 0; u < ROWS; u++) {
                    if ((um[u] >> l) & 1u) {
                        const uint32_t wo = v[u] - A.pc_lo;
                        atomicMin(&A.first_w[wo], (int32_t)rkv[u]);
                        const uint64_t slot = basei + (uint64_t)__popcll(um[u] & lt);
                        if (slot < A.rec_cap)
                            A.rec[slot] = ((unsigned long long)rkv[u] << 32) | wo;
                        A.cand[ix[u]] = 1;
                    }
                    basei += (uint64_t)__popcll(um[u]);
                }
            }
        }
    }
}

// covered |= records [*done, min(*cnt, cap)); then *done advances (next kernel).
__global__ void cover_records_kernel(const unsigned long long *rec, uint64_t cap,
                                     const unsigned long long *cnt, const unsigned long long *done,
                                     uint32_t *covered) {
    const uint64_t lo = *done, hi = std::min<uint64_t>(*cnt, cap);
    for (uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < hi;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t wo = (uint32_t)rec[i];
        const uint32_t mbit = 1u << (wo & 31);
        if (!(covered[wo >> 5] & mbit)) atomicOr(&covered[wo >> 5], mbit);
    }
}

__global__ void advance_kernel(const unsigned long long *cnt, unsigned long long *done,
                               uint64_t cap) {
    if (threadIdx.x == 0) *done = std::min<uint64_t>(*cnt, cap);
}

// The first-cover rank of window offset wo: first_w[wo] on one GPU; across
// shards the MIN-merged dense table first_d[id(wo)] (tab: dictionary of the
// merged union, syzcov_dev_dict_build_bits layout).
__device__ __forceinline__ int32_t first_of(const int32_t *first_w, const uint64_t *tab,
                                            const int32_t *first_d, uint32_t wo) {
    if (!tab) return first_w[wo];
    const uint64_t e = tab[wo >> 5];
    const uint32_t bits = (uint32_t)(e >> 32), b = wo & 31;
    if (!((bits >> b) & 1u)) return INT32_MAX;
    return first_d[(uint32_t)e + __popc(bits & ((1u << b) - 1u))];
}

// Pass 2 over the records: kept[rank] = 1 iff first(pc) == rank.
__global__ void pass2_kernel(const unsigned long long *rec, uint64_t cap,
                             const unsigned long long *cnt, const int32_t *first_w,
                             const uint64_t *tab, const int32_t *first_d, uint8_t *kept) {
    const uint64_t hi = std::min<uint64_t>(*cnt, cap);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < hi;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long r = rec[i];
        const int32_t rank = (int32_t)(r >> 32);
        if (first_of(first_w, tab, first_d, (uint32_t)r) == rank) kept[rank] = 1;
    }
}

// first_w back to INT32_MAX at every recorded offset (after pass 2).
__global__ void reset_kernel(const unsigned long long *rec, uint64_t cap,
                             const unsigned long long *cnt, int32_t *first_w) {
    const uint64_t hi = std::min<uint64_t>(*cnt, cap);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < hi;
         i += (uint64_t)gridDim.x * blockDim.x)
        first_w[(uint32_t)rec[i]] = INT32_MAX;
}

// ---- overflow fallbacks (early exit unless *cnt > cap)
__global__ void ovf_pass2_kernel(Args A, uint32_t n_items, const int32_t *first_w,
                                 const uint64_t *tab, const int32_t *first_d, uint8_t *kept) {
    if (*A.rec_cnt <= A.rec_cap) return;
    for (uint32_t j = blockIdx.x; j < n_items; j += gridDim.x) {
        if (!A.cand[j]) continue;
        const int32_t rank = A.ranks ? A.ranks[j] : (int32_t)j;
        const uint64_t o = A.base_r[j];
        const uint32_t n = A.split_t[(uint64_t)(A.nrange - 1) * A.n_items + j];
        bool hit = false;
        for (uint32_t q = threadIdx.x; q < n; q += blockDim.x)
            hit |= first_of(first_w, tab, first_d, A.pcs[o + q] - A.pc_lo) == rank;
        if (__syncthreads_or(hit) && threadIdx.x == 0) kept[rank] = 1;
    }
}

__global__ void ovf_union_kernel(const unsigned long long *cnt, uint64_t cap, const int32_t *first_w,
                                 uint64_t span, uint32_t *covered) {
    if (*cnt <= cap) return;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < span;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const bool set = first_w[i] != INT32_MAX;
        const uint64_t m = __ballot(set);
        if ((threadIdx.x & 31) == 0) {
            const uint32_t word = (uint32_t)(m >> (threadIdx.x & 32));
            if (word) atomicOr(&covered[i >> 5], word);
        }
    }
}

__global__ void ovf_reset_kernel(const unsigned long long *cnt, uint64_t cap, int32_t *first_w,
                                 uint64_t span) {
    if (*cnt <= cap) return;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < span;
         i += (uint64_t)gridDim.x * blockDim.x)
        first_w[i] = INT32_MAX;
}

// window-indexed first_w <-> dense table over a dictionary (shard exchange)
__global__ void first_dense_kernel(const uint64_t *__restrict__ tab, uint64_t nwords,
                                   int32_t *__restrict__ first_w, int32_t *__restrict__ dense,
                                   int to_dense) {
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords;
         w += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t e = tab[w];
        uint32_t bits = (uint32_t)(e >> 32), pos = (uint32_t)e;
        while (bits) {
            const int b = __ffs(bits) - 1;
            bits &= bits - 1;
            if (to_dense)
                dense[pos++] = first_w[w * 32 + b];
            else
                first_w[w * 32 + b] = dense[pos++];
        }
    }
}

}  // namespace mr
}  // namespace syz

using namespace syz;

/* ws: rec_done (u64) | base_r [n_items] u64 | split_t [nrange][n_items] u32 */
static uint64_t mr_nrange(uint64_t span, uint32_t rshift) {
    return (span + (1ull << rshift) - 1) >> rshift;
}

extern "C" size_t syzcov_dev_minimize_range_ws_size(size_t n_items, uint64_t pc_span,
                                                    uint32_t range_shift) {
    if (range_shift > 20) range_shift = 20;
    return 256 + align_up(n_items * 8, 256) +
           align_up(mr_nrange(pc_span, range_shift) * n_items * 4, 256);
}

static int mr_args(mr::Args &A, const uint64_t *off, const uint32_t *len, const uint32_t *pcs,
                   const uint32_t *split, const int32_t *order, const int32_t *ranks,
                   size_t n_items, uint32_t pc_lo, uint64_t pc_span, uint32_t range_shift,
                   const uint64_t *range_tot, uint32_t *covered, int32_t *first_w, uint64_t *rec,
                   uint64_t rec_cap, uint64_t *rec_cnt, uint8_t *cand, void *ws) {
    if (!off || !pcs || !order || !range_tot || !covered || !first_w || !rec || !rec_cnt || !cand ||
        !ws || n_items > 0x7FFFFFFF)
        return SYZCOV_EINVAL;
    if (range_shift < 10 || range_shift > 20 || pc_span == 0 || pc_span > (1ull << 32))
        return SYZCOV_EINVAL;
    const uint64_t nrange = mr_nrange(pc_span, range_shift);
    if (nrange > (uint64_t)mr::MAX_R) return SYZCOV_ERANGE;
    if (!split && nrange != 1) return SYZCOV_EINVAL;
    if (!split && !len) return SYZCOV_EINVAL;
    A.off = off;
    A.len = len;
    A.pcs = pcs;
    A.split = split;
    A.order = order;
    A.ranks = ranks;
    A.pc_lo = pc_lo;
    A.rshift = range_shift;
    A.nrange = (uint32_t)nrange;
    A.range_tot = (const unsigned long long *)range_tot;
    A.covered = covered;
    A.first_w = first_w;
    A.rec = (unsigned long long *)rec;
    A.rec_cap = rec_cap;
    A.rec_cnt = (unsigned long long *)rec_cnt;
    A.cand = cand;
    A.n_items = (uint32_t)n_items;
    A.base_r = (uint64_t *)((uint8_t *)ws + 256);
    A.split_t = (uint32_t *)((uint8_t *)A.base_r + align_up(n_items * 8, 256));
    return 0;
}

// pass 2 + resets (first_w back to INT32_MAX)
static int mr_pass2(const mr::Args &A, uint64_t pc_span, const uint64_t *tab,
                    const int32_t *first_d, uint8_t *kept, hipStream_t s) {
    const unsigned long long *rec = A.rec, *cnt = A.rec_cnt;
    hipLaunchKernelGGL(mr::pass2_kernel, dim3(1024), dim3(256), 0, s, rec, A.rec_cap, cnt,
                       (const int32_t *)A.first_w, tab, first_d, kept);
    hipLaunchKernelGGL(mr::ovf_pass2_kernel, dim3(1024), dim3(256), 0, s, A, A.n_items,
                       (const int32_t *)A.first_w, tab, first_d, kept);
    hipLaunchKernelGGL(mr::reset_kernel, dim3(1024), dim3(256), 0, s, rec, A.rec_cap, cnt,
                       A.first_w);
    hipLaunchKernelGGL(mr::ovf_reset_kernel, dim3(2048), dim3(256), 0, s, cnt, A.rec_cap, A.first_w,
                       pc_span);
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" int syzcov_dev_minimize_range(
    const uint64_t *off, const uint32_t *len, const uint32_t *pcs, const uint32_t *split,
    const int32_t *order, const int32_t *ranks, size_t n_items, uint32_t pc_lo, uint64_t pc_span,
    uint32_t range_shift, const uint64_t *range_tot, uint32_t *covered, int32_t *first_w,
    uint64_t *rec, uint64_t rec_cap, uint64_t *rec_cnt, uint8_t *cand, uint8_t *kept, int do_pass2,
    size_t first_chunk, uint32_t growth, uint64_t pcs_per_wg_hint, void *ws, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    if (n_items == 0) {
        if (rec_cnt) SYZ_HIP(hipMemsetAsync(rec_cnt, 0, sizeof(uint64_t), s));
        return 0;
    }
    if (do_pass2 && !kept) return SYZCOV_EINVAL;
    mr::Args A;
    int rc = mr_args(A, off, len, pcs, split, order, ranks, n_items, pc_lo, pc_span, range_shift,
                     range_tot, covered, first_w, rec, rec_cap, rec_cnt, cand, ws);
    if (rc) return rc;
    const uint64_t nrange = A.nrange;
    unsigned long long *done = (unsigned long long *)ws;
    SYZ_HIP(hipMemsetAsync(done, 0, sizeof(uint64_t), s));
    SYZ_HIP(hipMemsetAsync(rec_cnt, 0, sizeof(uint64_t), s));
    hipLaunchKernelGGL(mr::prep_kernel, dim3(grid_for(n_items, 64, 8192)), dim3(256), 0, s, A,
                       (uint64_t *)A.base_r, (uint32_t *)A.split_t);
    const size_t lds = ((size_t)1 << range_shift) / 8;
    static bool attr_set = false;  // idempotent; races only repeat the call
    if (!attr_set) {
        SYZ_HIP(hipFuncSetAttribute((const void *)mr::pass1_kernel,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024));
        attr_set = true;
    }
    if (first_chunk == 0) first_chunk = 64;
    if (growth < 2) growth = 4;
    if (pcs_per_wg_hint == 0) pcs_per_wg_hint = 1 << 18;
    const uint64_t avg_len = 2048;  // only sizes the grid; any value is exact
    uint64_t a = 0, step = first_chunk;
    while (a < n_items) {
        const uint64_t b = std::min<uint64_t>(n_items, a + step);
        uint64_t G = (b - a) * avg_len / pcs_per_wg_hint;
        G = std::max<uint64_t>(G, std::max<uint64_t>(4 * nrange, 1024));
        G = std::min<uint64_t>(G, 8192);
        hipLaunchKernelGGL(mr::pass1_kernel, dim3((unsigned)G), dim3(mr::THREADS), lds, s, A,
                           (uint32_t)a, (uint32_t)b, (int)(a != 0));
        hipLaunchKernelGGL(mr::cover_records_kernel, dim3(1024), dim3(256), 0, s,
                           (const unsigned long long *)rec, rec_cap,
                           (const unsigned long long *)rec_cnt, (const unsigned long long *)done,
                           covered);
        hipLaunchKernelGGL(mr::advance_kernel, dim3(1), dim3(64), 0, s,
                           (const unsigned long long *)rec_cnt, done, rec_cap);
        a = b;
        step *= growth;
    }
    // record overflow: the union comes from first_w instead
    hipLaunchKernelGGL(mr::ovf_union_kernel, dim3(2048), dim3(256), 0, s,
                       (const unsigned long long *)rec_cnt, rec_cap, (const int32_t *)first_w,
                       pc_span, covered);
    SYZ_LAUNCH_CHECK();
    if (!do_pass2) return 0;
    return mr_pass2(A, pc_span, nullptr, nullptr, kept, s);
}

extern "C" int syzcov_dev_minimize_range_pass2(
    const uint64_t *off, const uint32_t *len, const uint32_t *pcs, const uint32_t *split,
    const int32_t *order, const int32_t *ranks, size_t n_items, uint32_t pc_lo, uint64_t pc_span,
    uint32_t range_shift, const uint64_t *range_tot, uint32_t *covered, int32_t *first_w,
    uint64_t *rec, uint64_t rec_cap, uint64_t *rec_cnt, uint8_t *cand, const uint64_t *tab,
    const int32_t *first_dense, uint8_t *kept, void *ws, void *stream) {
    if (n_items == 0) return 0;
    if (!kept || (tab && !first_dense)) return SYZCOV_EINVAL;
    mr::Args A;
    int rc = mr_args(A, off, len, pcs, split, order, ranks, n_items, pc_lo, pc_span, range_shift,
                     range_tot, covered, first_w, rec, rec_cap, rec_cnt, cand, ws);
    if (rc) return rc;
    return mr_pass2(A, pc_span, tab, first_dense, kept, (hipStream_t)stream);
}

extern "C" int syzcov_dev_first_dense(const uint64_t *tab, uint64_t pc_span, int32_t *first_w,
                                      int32_t *dense, int to_dense, void *stream) {
    if (!tab || !first_w || !dense || pc_span == 0) return SYZCOV_EINVAL;
    const uint64_t nwords = (pc_span + 31) / 32;
    hipLaunchKernelGGL(mr::first_dense_kernel, dim3(grid_for(nwords, 256, 16384)), dim3(256), 0,
                       (hipStream_t)stream, tab, nwords, first_w, dense, to_dense);
    SYZ_LAUNCH_CHECK();
    return 0;
}
