// minimize.hip — cover.Minimize (cover/cover.go:104-131) as a first-cover
// problem on gfx950.
//
// The reference scans inputs in sort.Sort order (len desc, cover.go:113) and
// keeps an input iff it holds a PC not yet in `covered`.  By induction
// `covered` before rank r equals the union of all inputs of rank < r, so
//     kept(r)  <=>  exists pc in cov_r with first(pc) == r,
//     first(pc) = min{ rank j : pc in cov_j }.
// Pass 1 computes first[] with a read-before-atomicMin per PC over the dense
// id space (MALL/L2-resident: 4 B per distinct PC), walking ranks in order
// across the grid so that nearly every PC is filtered by the plain read;
// an input that never lowered an entry can not be first for anything and is
// dropped on the spot.  Pass 2 re-scans only the candidates (early exit on
// the first PC it owns).  An ordered compaction then yields the kept input
// indices in processing order — the reference's output order.
#include "common.h"

#include <algorithm>

namespace syz {

constexpr int MINI_THREADS = 256;

__global__ __launch_bounds__(MINI_THREADS) void minimize_pass1_kernel(
    const uint64_t *__restrict__ off, const uint32_t *__restrict__ len,
    const uint32_t *__restrict__ pcs, const int32_t *__restrict__ order,
    const int32_t *__restrict__ ranks, uint32_t n, const uint64_t *__restrict__ tab,
    uint32_t pc_lo, int32_t *__restrict__ first, uint8_t *__restrict__ cand) {
    for (uint32_t j = blockIdx.x; j < n; j += gridDim.x) {
        const int32_t idx = order[j];
        const int32_t r = ranks ? ranks[j] : (int32_t)j;
        const uint64_t b = off[idx];
        const uint32_t l = len ? len[idx] : (uint32_t)(off[idx + 1] - b);
        bool won = false;
        for (uint32_t k = threadIdx.x; k < l; k += MINI_THREADS) {
            const uint32_t id = dense_id(tab, pcs[b + k], pc_lo);
            if (first[id] > r) {
                const int32_t old = atomicMin(&first[id], r);
                won |= old > r;
            }
        }
        won = __syncthreads_or(won);
        if (threadIdx.x == 0) cand[j] = won ? 1 : 0;
    }
}

__global__ __launch_bounds__(MINI_THREADS) void minimize_pass2_kernel(
    const uint64_t *__restrict__ off, const uint32_t *__restrict__ len,
    const uint32_t *__restrict__ pcs, const int32_t *__restrict__ order,
    const int32_t *__restrict__ ranks, uint32_t n, const uint64_t *__restrict__ tab,
    uint32_t pc_lo, const int32_t *__restrict__ first, const uint8_t *__restrict__ cand,
    uint8_t *__restrict__ kept) {
    for (uint32_t j = blockIdx.x; j < n; j += gridDim.x) {
        if (!cand[j]) continue;  // kept[] is pre-zeroed
        const int32_t idx = order[j];
        const int32_t r = ranks ? ranks[j] : (int32_t)j;
        const uint64_t b = off[idx];
        const uint32_t l = len ? len[idx] : (uint32_t)(off[idx + 1] - b);
        bool found = false;
        for (uint32_t k0 = 0; k0 < l; k0 += MINI_THREADS) {
            const uint32_t k = k0 + threadIdx.x;
            bool f = false;
            if (k < l) f = first[dense_id(tab, pcs[b + k], pc_lo)] == r;
            if (__syncthreads_or(f)) {
                found = true;
                break;
            }
        }
        if (threadIdx.x == 0 && found) kept[r] = 1;
    }
}

// Ordered compaction of byte flags: pass A counts per 1024-flag block,
// pass B scans the block counts, pass C scatters order[r] for kept r.
constexpr int CMP_THREADS = 256, CMP_PER = 4, CMP_BLK = CMP_THREADS * CMP_PER;

__global__ __launch_bounds__(CMP_THREADS) void compact_count_kernel(const uint8_t *__restrict__ f,
                                                                     uint64_t n,
                                                                     uint32_t *__restrict__ bsum) {
    __shared__ uint32_t tmp[CMP_THREADS / 64 + 1];
    const uint64_t base = (uint64_t)blockIdx.x * CMP_BLK + threadIdx.x * CMP_PER;
    uint32_t c = 0;
#pragma unroll
    for (int q = 0; q < CMP_PER; q++) c += (base + q < n) && f[base + q];
    uint32_t total;
    block_excl_scan<CMP_THREADS>(c, tmp, &total);
    if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

__global__ __launch_bounds__(1024) void scan_blocks_kernel(uint32_t *__restrict__ bsum,
                                                            uint64_t nblk,
                                                            uint32_t *__restrict__ total_out) {
    __shared__ uint32_t tmp[1024 / 64 + 1];
    uint32_t carry = 0;
    for (uint64_t c = 0; c < nblk; c += 1024) {
        const uint64_t i = c + threadIdx.x;
        const uint32_t v = i < nblk ? bsum[i] : 0u;
        uint32_t total;
        const uint32_t p = block_excl_scan<1024>(v, tmp, &total);
        if (i < nblk) bsum[i] = carry + p;
        carry += total;
    }
    if (threadIdx.x == 0 && total_out) *total_out = carry;
}

__global__ __launch_bounds__(CMP_THREADS) void compact_scatter_kernel(
    const uint8_t *__restrict__ f, uint64_t n, const uint32_t *__restrict__ bsum,
    const int32_t *__restrict__ order, int32_t *__restrict__ out) {
    __shared__ uint32_t tmp[CMP_THREADS / 64 + 1];
    const uint64_t base = (uint64_t)blockIdx.x * CMP_BLK + threadIdx.x * CMP_PER;
    uint32_t c = 0;
#pragma unroll
    for (int q = 0; q < CMP_PER; q++) c += (base + q < n) && f[base + q];
    uint32_t total;
    uint32_t p = bsum[blockIdx.x] + block_excl_scan<CMP_THREADS>(c, tmp, &total);
#pragma unroll
    for (int q = 0; q < CMP_PER; q++)
        if (base + q < n && f[base + q]) out[p++] = order ? order[base + q] : (int32_t)(base + q);
}

// A shard's work items in one ordered compaction (corpus.hip items_of): the
// global ranks r whose input order[r] lives in [base, base + n_local), as
// (rank, local input) pairs, flags derived from the order on the fly (was a
// flag pass and two compactions of the same flags: 7 launches, 94 us at C3/8).
__device__ __forceinline__ uint32_t sel_of(const int32_t *order, uint64_t i, uint64_t n,
                                           uint32_t base, uint32_t n_local) {
    return i < n && (uint32_t)order[i] - base < n_local;
}
__global__ __launch_bounds__(CMP_THREADS) void sel_count_kernel(const int32_t *__restrict__ order,
                                                                uint64_t n, uint32_t base,
                                                                uint32_t n_local,
                                                                uint32_t *__restrict__ bsum) {
    __shared__ uint32_t tmp[CMP_THREADS / 64 + 1];
    const uint64_t b0 = (uint64_t)blockIdx.x * CMP_BLK + threadIdx.x * CMP_PER;
    uint32_t c = 0;
#pragma unroll
    for (int q = 0; q < CMP_PER; q++) c += sel_of(order, b0 + q, n, base, n_local);
    uint32_t total;
    block_excl_scan<CMP_THREADS>(c, tmp, &total);
    if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}
__global__ __launch_bounds__(CMP_THREADS) void sel_scatter_kernel(
    const int32_t *__restrict__ order, uint64_t n, uint32_t base, uint32_t n_local,
    const uint32_t *__restrict__ bsum, int32_t *__restrict__ ranks, int32_t *__restrict__ items) {
    __shared__ uint32_t tmp[CMP_THREADS / 64 + 1];
    const uint64_t b0 = (uint64_t)blockIdx.x * CMP_BLK + threadIdx.x * CMP_PER;
    uint32_t f[CMP_PER], c = 0;
#pragma unroll
    for (int q = 0; q < CMP_PER; q++) c += f[q] = sel_of(order, b0 + q, n, base, n_local);
    uint32_t total;
    uint32_t p = bsum[blockIdx.x] + block_excl_scan<CMP_THREADS>(c, tmp, &total);
#pragma unroll
    for (int q = 0; q < CMP_PER; q++)
        if (f[q]) {
            ranks[p] = (int32_t)(b0 + q);
            items[p++] = order[b0 + q] - (int32_t)base;
        }
}

// ---------------------------------------------------------------------
// Manager.minimizeCorpus (syz-manager/manager.go:504-524): cover.Minimize
// runs once per call group, so first-cover is keyed by (group, pc).  Ranks
// are grouped (group g owns ranks [goff[g], goff[g+1]), each group in its own
// Go sort.Sort order) and a batch of groups [g0, g1) gets a first-cover slab
// first[(g - g0) * nids + id].  ord_g[j] is the grouped index of rank j and
// perm[] maps grouped indices to corpus indices.
__global__ void grp_order_kernel(const int32_t *__restrict__ ord_g, const int32_t *__restrict__ perm,
                                 const uint64_t *__restrict__ goff, uint32_t ngroups, uint32_t n,
                                 int32_t *__restrict__ order_c, uint32_t *__restrict__ rank_grp) {
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
        order_c[j] = perm[ord_g[j]];
        uint32_t lo = 0, hi = ngroups;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (goff[mid] <= j) lo = mid; else hi = mid;
        }
        rank_grp[j] = lo;
    }
}

__global__ __launch_bounds__(MINI_THREADS) void grp_pass1_kernel(
    const uint64_t *__restrict__ off, const uint32_t *__restrict__ pcs,
    const int32_t *__restrict__ order, const uint32_t *__restrict__ rank_grp, uint32_t r0,
    uint32_t r1, uint32_t g0, uint32_t nids, const uint64_t *__restrict__ tab, uint32_t pc_lo,
    int32_t *__restrict__ first, uint8_t *__restrict__ cand) {
    for (uint32_t j = r0 + blockIdx.x; j < r1; j += gridDim.x) {
        const int32_t idx = order[j];
        int32_t *fg = first + (size_t)(rank_grp[j] - g0) * nids;
        const int32_t r = (int32_t)j;
        const uint64_t b = off[idx];
        const uint32_t l = (uint32_t)(off[idx + 1] - b);
        bool won = false;
        for (uint32_t k = threadIdx.x; k < l; k += MINI_THREADS) {
            const uint32_t id = dense_id(tab, pcs[b + k], pc_lo);
            if (fg[id] > r) won |= atomicMin(&fg[id], r) > r;
        }
        won = __syncthreads_or(won);
        if (threadIdx.x == 0) cand[j] = won ? 1 : 0;
    }
}

__global__ __launch_bounds__(MINI_THREADS) void grp_pass2_kernel(
    const uint64_t *__restrict__ off, const uint32_t *__restrict__ pcs,
    const int32_t *__restrict__ order, const uint32_t *__restrict__ rank_grp, uint32_t r0,
    uint32_t r1, uint32_t g0, uint32_t nids, const uint64_t *__restrict__ tab, uint32_t pc_lo,
    const int32_t *__restrict__ first, const uint8_t *__restrict__ cand, uint8_t *__restrict__ kept) {
    for (uint32_t j = r0 + blockIdx.x; j < r1; j += gridDim.x) {
        if (!cand[j]) continue;
        const int32_t idx = order[j];
        const int32_t *fg = first + (size_t)(rank_grp[j] - g0) * nids;
        const uint64_t b = off[idx];
        const uint32_t l = (uint32_t)(off[idx + 1] - b);
        bool found = false;
        for (uint32_t k0 = 0; k0 < l; k0 += MINI_THREADS) {
            const uint32_t k = k0 + threadIdx.x;
            const bool f = k < l && fg[dense_id(tab, pcs[b + k], pc_lo)] == (int32_t)j;
            if (__syncthreads_or(f)) {
                found = true;
                break;
            }
        }
        if (threadIdx.x == 0 && found) kept[j] = 1;
    }
}

static unsigned mini_grid(size_t n) {
    // enough workgroups to fill 256 CUs several times over while keeping the
    // in-flight rank window narrow (read-before-atomic filtering)
    return (unsigned)std::min<size_t>(std::max<size_t>(n, 1), 2048);
}

}  // namespace syz

using namespace syz;

extern "C" int syzcov_dev_minimize_pass1(const uint64_t *off, const uint32_t *len,
                                         const uint32_t *pcs, const int32_t *order,
                                         const int32_t *ranks, size_t n,
                                         const uint64_t *tab, uint32_t pc_lo, int32_t *first,
                                         uint8_t *cand, void *stream) {
    if (n == 0) return 0;
    if (!off || !pcs || !order || !tab || !first || !cand || n > 0x7FFFFFFF) return SYZCOV_EINVAL;
    hipLaunchKernelGGL(minimize_pass1_kernel, dim3(mini_grid(n)), dim3(MINI_THREADS), 0,
                       (hipStream_t)stream, off, len, pcs, order, ranks, (uint32_t)n, tab, pc_lo,
                       first, cand);
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" int syzcov_dev_minimize_pass2(const uint64_t *off, const uint32_t *len,
                                         const uint32_t *pcs, const int32_t *order,
                                         const int32_t *ranks, size_t n,
                                         const uint64_t *tab, uint32_t pc_lo, const int32_t *first,
                                         const uint8_t *cand, uint8_t *kept, void *stream) {
    if (n == 0) return 0;
    if (!off || !pcs || !order || !tab || !first || !cand || !kept || n > 0x7FFFFFFF)
        return SYZCOV_EINVAL;
    hipLaunchKernelGGL(minimize_pass2_kernel, dim3(mini_grid(n)), dim3(MINI_THREADS), 0,
                       (hipStream_t)stream, off, len, pcs, order, ranks, (uint32_t)n, tab, pc_lo,
                       first, cand, kept);
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" size_t syzcov_dev_compact_ws_size(size_t n) {
    return align_up(((n + CMP_BLK - 1) / CMP_BLK + 1) * sizeof(uint32_t), 256);
}

extern "C" int syzcov_dev_compact_kept(const uint8_t *kept, const int32_t *order, size_t n,
                                       int32_t *out_idx, uint32_t *n_out, void *ws,
                                       void *stream) {
    if (!n_out || !ws) return SYZCOV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) {
        SYZ_HIP(hipMemsetAsync(n_out, 0, sizeof(uint32_t), s));
        return 0;
    }
    if (!kept || !out_idx) return SYZCOV_EINVAL;
    const uint64_t nblk = (n + CMP_BLK - 1) / CMP_BLK;
    uint32_t *bsum = (uint32_t *)ws;
    hipLaunchKernelGGL(compact_count_kernel, dim3((unsigned)nblk), dim3(CMP_THREADS), 0, s, kept,
                       (uint64_t)n, bsum);
    SYZ_LAUNCH_CHECK();
    hipLaunchKernelGGL(scan_blocks_kernel, dim3(1), dim3(1024), 0, s, bsum, nblk, n_out);
    SYZ_LAUNCH_CHECK();
    hipLaunchKernelGGL(compact_scatter_kernel, dim3((unsigned)nblk), dim3(CMP_THREADS), 0, s,
                       kept, (uint64_t)n, bsum, order, out_idx);
    SYZ_LAUNCH_CHECK();
    return 0;
}

namespace syz {
// (rank, local input) of every global rank whose input lives in [base, base +
// n_local), in rank order; *n_out = their number; ws: syzcov_dev_compact_ws_size(n)
int compact_shard_items(const int32_t *order, size_t n, uint32_t base, uint32_t n_local,
                        int32_t *ranks, int32_t *items, uint32_t *n_out, void *ws, hipStream_t s) {
    if (!n_out || !ws || !order || !ranks || !items) return SYZCOV_EINVAL;
    if (n == 0) {
        SYZ_HIP(hipMemsetAsync(n_out, 0, sizeof(uint32_t), s));
        return 0;
    }
    const uint64_t nblk = (n + CMP_BLK - 1) / CMP_BLK;
    uint32_t *bsum = (uint32_t *)ws;
    hipLaunchKernelGGL(sel_count_kernel, dim3((unsigned)nblk), dim3(CMP_THREADS), 0, s, order,
                       (uint64_t)n, base, n_local, bsum);
    hipLaunchKernelGGL(scan_blocks_kernel, dim3(1), dim3(1024), 0, s, bsum, nblk, n_out);
    hipLaunchKernelGGL(sel_scatter_kernel, dim3((unsigned)nblk), dim3(CMP_THREADS), 0, s, order,
                       (uint64_t)n, base, n_local, (const uint32_t *)bsum, ranks, items);
    SYZ_LAUNCH_CHECK();
    return 0;
}

// Grouped Minimize over ranks [r0, r1) whose groups are [g0, g1); `first`
// holds (g1 - g0) * nids entries.  kept[] must be zeroed by the caller.
// order_c[j] = corpus index of rank j, rank_grp[j] = its group
int minimize_groups_order(const int32_t *ord_g, const int32_t *perm, const uint64_t *goff_dev,
                          uint32_t ngroups, uint32_t n, int32_t *order_c, uint32_t *rank_grp,
                          hipStream_t s) {
    hipLaunchKernelGGL(grp_order_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, ord_g, perm,
                       goff_dev, ngroups, n, order_c, rank_grp);
    SYZ_LAUNCH_CHECK();
    return 0;
}

int minimize_groups_batch(const uint64_t *off, const uint32_t *pcs, const int32_t *order_c,
                          const uint32_t *rank_grp, uint32_t r0, uint32_t r1, uint32_t g0,
                          uint32_t nids, const uint64_t *tab, uint32_t pc_lo, int32_t *first,
                          size_t first_n, uint8_t *cand, uint8_t *kept, hipStream_t s) {
    if (r1 <= r0) return 0;
    SYZ_HIP(hipMemsetD32Async((hipDeviceptr_t)first, 0x7FFFFFFF, first_n, s));
    const unsigned g = mini_grid(r1 - r0);
    hipLaunchKernelGGL(grp_pass1_kernel, dim3(g), dim3(MINI_THREADS), 0, s, off, pcs, order_c,
                       rank_grp, r0, r1, g0, nids, tab, pc_lo, first, cand);
    hipLaunchKernelGGL(grp_pass2_kernel, dim3(g), dim3(MINI_THREADS), 0, s, off, pcs, order_c,
                       rank_grp, r0, r1, g0, nids, tab, pc_lo, (const int32_t *)first,
                       (const uint8_t *)cand, kept);
    SYZ_LAUNCH_CHECK();
    return 0;
}
}  // namespace syz
