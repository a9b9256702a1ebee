// newcov.hip — streaming new-coverage check of syz-fuzzer execute()
// (syz-fuzzer/fuzzer.go:456-480) against resident per-CallID maxCover
// bitmaps and the global flakes bitmap.
//
// The reference walks executed calls one at a time:
//   diff = Difference(Difference(cov, maxCover[c]), flakes)
//   if diff != ∅ { maxCover[c] = Union(maxCover[c], diff); triage(cov) }
// Over a batch in order that is exactly
//   new(k) <=> exists pc in cov_k: pc ∉ F, pc ∉ M0[c_k], and no earlier
//              record j < k with c_j = c_k holds pc,
//   M1[c]  =  M0[c] ∪ (∪_{j: c_j = c} cov_j \ F),
// i.e. first-cover on the key (CallID, pc) after masking F ∪ M0.  Pass 1
// tests every PC against the bitmaps and compacts each record's survivors
// into its own slots (few once maxCover saturates); a hash table keyed by
// (CallID, pc) takes an atomicMin of the record index; pass 2 marks a record
// new iff it owns one of its keys and ORs the owned keys into maxCover.
//
// The bitmaps are indexed by window offset (pc - pc_lo), or, once the PC
// universe is registered (syzcov_state_set_universe), by the dense key
// (pc >> kshift) - kbase of keys.hip: one probe per PC into a per-call bitmap
// of nkeys bits (512 KB at the synthetic 2^22-PC universe instead of 8 MB of
// window bits), so a call's bitmap stays in its XCD's L2 while that XCD
// walks the call's records.
#include "cover_state.h"

namespace syz {

constexpr int NC_THREADS = 256;
constexpr int NC_WPB = NC_THREADS / 64;
constexpr int NC_U = 8;  // rows of 64 PCs in flight per wave
constexpr uint32_t SENT = 0xFFFFFFFFu;

// Candidates: (record k, pc) pairs that pass the maxCover and flakes
// bitmaps, appended to one list (few once maxCover saturates); stats[1] is
// the list length.  One atomic per wave-row that has any.
__device__ __forceinline__ void emit_cands(bool cand, uint32_t k, uint32_t pc,
                                           uint2 *__restrict__ clist,
                                           uint32_t *__restrict__ stats) {
    const uint64_t m = __ballot(cand);
    if (!m) return;
    const uint32_t l = __lane_id();
    uint32_t base = 0;
    if (l == 0) base = atomicAdd(&stats[1], (uint32_t)__popcll(m));
    base = __shfl(base, 0, 64);
    if (cand) clist[base + (uint32_t)__popcll(m & ((1ull << l) - 1ull))] = make_uint2(k, pc);
}

// ---------------------------------------------------------------------------
// Records grouped by CallID (counting sort over three kernels): both
// candidate passes walk a call's records together.
//   grp_hist: per-call counts   grp_scan: offsets coff   grp_scatter: perm/pos
constexpr int GRP_MAX_CALLS = 16384;  // LDS counters; above, global atomics
constexpr int GS_THREADS = 1024, GS_PER = 4;  // scatter: records per thread

__global__ __launch_bounds__(256) void grp_hist_kernel(const int32_t *__restrict__ callid,
                                                       uint32_t nrec, int ncalls,
                                                       uint32_t *__restrict__ ccnt,
                                                       uint32_t *__restrict__ stats) {
    extern __shared__ uint32_t h[];  // ncalls counters, or none above GRP_MAX_CALLS
    const bool sh = ncalls <= GRP_MAX_CALLS;
    if (sh)
        for (int c = threadIdx.x; c < ncalls; c += blockDim.x) h[c] = 0;
    __syncthreads();
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < nrec; k += gridDim.x * blockDim.x) {
        const int c = callid[k];
        if (c >= 0 && c < ncalls) atomicAdd(sh ? &h[c] : &ccnt[c], 1u);
        else stats[0] = 2u;
    }
    __syncthreads();
    if (sh)
        for (int c = threadIdx.x; c < ncalls; c += blockDim.x)
            if (h[c]) atomicAdd(&ccnt[c], h[c]);
}

// call offsets coff[0..ncalls] (exclusive scan); cursors = coff
__global__ __launch_bounds__(1024) void grp_scan_kernel(const uint32_t *__restrict__ ccnt,
                                                        int ncalls, uint32_t *__restrict__ coff,
                                                        uint32_t *__restrict__ cursor) {
    __shared__ uint32_t tmp[1024 / 64 + 1];
    uint32_t carry = 0;
    for (int c0 = 0; c0 < ncalls; c0 += 1024) {
        const int c = c0 + (int)threadIdx.x;
        const uint32_t v = c < ncalls ? ccnt[c] : 0u;
        uint32_t tot;
        const uint32_t p = block_excl_scan<1024>(v, tmp, &tot);
        if (c < ncalls) coff[c] = cursor[c] = carry + p;
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) coff[ncalls] = carry;
}

// perm[j] = k with j from the call's cursor (order inside a call
// is free: perm is only a visiting order, ownership uses the batch index).
// Each workgroup reserves one range per call it holds (LDS counts, one
// global atomic per (workgroup, call)) instead of one atomic per record.
__global__ __launch_bounds__(GS_THREADS) void grp_scatter_kernel(
    const int32_t *__restrict__ callid, uint32_t nrec, int ncalls, uint32_t *__restrict__ cursor,
    uint32_t *__restrict__ perm) {
    extern __shared__ uint32_t h[];  // ncalls local counts, then bases
    const bool sh = ncalls <= GRP_MAX_CALLS;
    const uint32_t k0 = blockIdx.x * GS_THREADS * GS_PER;
    if (!sh) {  // many calls: one global atomic per record
        for (uint32_t i = threadIdx.x; i < GS_THREADS * GS_PER; i += GS_THREADS) {
            const uint32_t k = k0 + i;
            if (k >= nrec) break;
            const int c = callid[k];
            if (c >= 0 && c < ncalls) perm[atomicAdd(&cursor[c], 1u)] = k;
        }
        return;
    }
    for (int c = threadIdx.x; c < ncalls; c += GS_THREADS) h[c] = 0;
    __syncthreads();
    uint32_t rank[GS_PER];
    int cc[GS_PER];
#pragma unroll
    for (int u = 0; u < GS_PER; u++) {
        const uint32_t k = k0 + u * GS_THREADS + threadIdx.x;
        cc[u] = k < nrec ? callid[k] : -1;
        if (cc[u] >= ncalls) cc[u] = -1;
        rank[u] = cc[u] >= 0 ? atomicAdd(&h[cc[u]], 1u) : 0u;
    }
    __syncthreads();
    for (int c = threadIdx.x; c < ncalls; c += GS_THREADS)
        if (h[c]) h[c] = atomicAdd(&cursor[c], h[c]);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < GS_PER; u++) {
        const uint32_t k = k0 + u * GS_THREADS + threadIdx.x;
        if (cc[u] >= 0) perm[h[cc[u]] + rank[u]] = k;
    }
}

// ---------------------------------------------------------------------------
// Probing candidate pass (any index space).  One WAVEFRONT per record in
// call-grouped order, coalesced 64-PC rows, both bitmap probes per PC.
// XCD-aware: workgroups are dispatched round-robin over the 8 XCDs, so the
// workgroups of XCD x (blockIdx % 8 == x) take the x-th eighth of the
// grouped records and a call's records share that XCD's L2 copy of its
// bitmap.  stats[0] = error (1 outside the index space, 2 call id, 3
// unsorted).
__global__ __launch_bounds__(NC_THREADS) void newcov_cand_kernel(
    const int32_t *__restrict__ callid, const uint64_t *__restrict__ rec_off,
    const uint32_t *__restrict__ pcs, uint32_t nrec, const uint32_t *__restrict__ maxcov,
    uint64_t words_per_call, const uint32_t *__restrict__ flakes, Index X,
    const uint32_t *__restrict__ perm, const uint32_t *__restrict__ coff, int ncalls,
    uint2 *__restrict__ clist, uint32_t *__restrict__ stats) {
    const uint32_t l = __lane_id();
    const uint32_t ng = coff[ncalls];  // grouped (valid) records; the rest: grp_hist flagged
    const uint32_t x = blockIdx.x & 7, nbx = gridDim.x >> 3;
    const uint32_t j0 = (uint32_t)((uint64_t)ng * x / 8), j1 = (uint32_t)((uint64_t)ng * (x + 1) / 8);
    const uint32_t nw = nbx * NC_WPB;
    for (uint32_t j = j0 + (blockIdx.x >> 3) * NC_WPB + (threadIdx.x >> 6); j < j1; j += nw) {
        const uint32_t k = perm[j];
        const uint32_t *M = maxcov + (uint64_t)(uint32_t)callid[k] * words_per_call;
        const uint64_t b = rec_off[k], n = rec_off[k + 1] - b;
        uint32_t bad = 0, carry = 0;
        // NC_U rows per step: all their loads and maxCover probes in flight together
        for (uint64_t q0 = 0; q0 < n; q0 += 64 * NC_U) {
            uint32_t pc[NC_U], w[NC_U], ix[NC_U];
            bool ok[NC_U];
#pragma unroll
            for (int u = 0; u < NC_U; u++) {
                const uint64_t q = q0 + u * 64 + l;
                pc[u] = q < n ? pcs[b + q] : 0u;
            }
#pragma unroll
            for (int u = 0; u < NC_U; u++) {
                const uint64_t q = q0 + u * 64 + l;
                const bool inw = pc_index(X, pc[u], &ix[u]);
                // 0xFFFFFFFF is Difference's end sentinel: never part of a
                // diff (cover.go:43-48,97), so never a candidate, never an error
                const bool sent = pc[u] == SENT;
                ok[u] = q < n && inw && !sent;
                bad |= (uint32_t)(q < n && !inw && !sent);
                w[u] = ok[u] ? M[ix[u] >> 5] : 0xFFFFFFFFu;
            }
#pragma unroll
            for (int u = 0; u < NC_U; u++) {
                const uint64_t q = q0 + u * 64 + l;
                // sortedness: the previous PC is lane l-1 of this row, or the
                // last PC of the previous row for lane 0
                uint32_t prev = __shfl_up(pc[u], 1, 64);
                if (l == 0) prev = carry;
                carry = wave_readlane(pc[u], 63);
                if (q < n && q > 0 && prev > pc[u]) bad |= 2u;
                // maxCover first: once it saturates, flakes are rarely probed
                const bool cand =
                    ok[u] && !((w[u] >> (ix[u] & 31)) & 1u) && !bit_test(flakes, ix[u]);
                emit_cands(cand, k, pc[u], clist, stats);
            }
        }
        if (bad) stats[0] = (bad & 1u) ? 1u : 3u;
    }
}

// ---------------------------------------------------------------------------
// LDS-staged candidate pass.  Probing a per-call bitmap in global memory is
// one scattered request per PC into a 150 MB set of bitmaps that no L2 holds
// (C5: 132 M probes per batch).  Instead the index space is cut into ranges
// of 2^19 keys (64 KB of bitmap): a workgroup stages one range of one call's
// maxCover (| flakes) in LDS and tests a chunk of that (call, range)'s PCs
// there.
//   records grouped by call:   grp_hist -> grp_scan -> grp_scatter (perm)
//   sub-runs:                  nq[q][j] = grouped record j's PC count in range
//                              q, Bq[q][j] = where that sub-run starts in pcs
//   row streams:               each sub-run cut into rows of <= 256 PCs (16-byte
//                              aligned: one dwordx4 per lane); Rq[q][j]
//                              = exclusive prefix of row counts (range_scan),
//                              one 16-byte row descriptor each (row_fill)
//   work items:                (call, range, chunk of CHR rows of its stream)
// The synthetic coverage is skewed (40% of PCs in range 0), so chunking by
// rows, not by records, is what balances the workgroups.
constexpr uint32_t NR_MAX = 32;          // ranges (index space <= 2^24)
constexpr uint32_t RSH = 19;             // 2^19 indices (64 KB of bitmap) per range:
                                         // two workgroups per CU
constexpr uint32_t ITEMS_MAX = 65536;    // chunk-count cap (items_target)
constexpr int LC_THREADS = 1024;         // LDS: two workgroups per CU
constexpr uint32_t LC_CBW = 16;          // candidates buffered per wave
constexpr int LC_U = 4;                  // 256-PC rows per step (two steps in flight)
#ifndef SYZ_NC_SQG
#define SYZ_NC_SQG 8
#endif
constexpr int SQ_G = SYZ_NC_SQG;         // split queries in flight per wave
#ifndef SYZ_NC_SPLIT_LNS
#define SYZ_NC_SPLIT_LNS 5
#endif
constexpr uint32_t SPLIT_LNS = SYZ_NC_SPLIT_LNS;  // log2 of the samples per record
constexpr uint32_t SPLIT_NS = 1u << SPLIT_LNS;    // (each sample fetches its own line)
static_assert(SPLIT_NS <= 64, "one sample per lane");

// Range boundaries of every grouped record, one wave per record, by
// SPLIT_NS-way search: SPLIT_NS evenly spaced samples bracket each query to a
// bucket of ceil(n / SPLIT_NS) PCs, whose elements are then counted (SQ_G
// queries' bucket loads in flight together).  32 samples: 32 sample lines +
// ~2 lines per query's bucket, against 64 + ~1 at 64 samples.  Queries: "index < (q+1) << RSH" for q < nr-1
// and "not the sentinel" (the record's length without its trailing
// 0xFFFFFFFF, which is never a candidate, cover.go:43-48).  Sorted records
// only: a record out of order is caught here at the boundaries (stats 3)
// or inside its sub-runs by the candidate pass; non-monotone boundaries
// become empty sub-runs.  An end outside the index space: stats 1.  Key
// positions only (pc_index_range): the candidate pass checks every PC's
// membership in the universe.
__global__ __launch_bounds__(256) void newcov_split_kernel(
    const uint64_t *__restrict__ rec_off, const uint32_t *__restrict__ pcs,
    const uint32_t *__restrict__ perm, const uint32_t *__restrict__ coff, int ncalls, Index X,
    uint32_t nr, uint32_t rsh, uint32_t stride, uint32_t *__restrict__ nq, uint64_t *__restrict__ Bq,
    uint32_t *__restrict__ stats) {
    const uint32_t l = __lane_id(), ng = coff[ncalls];
    for (uint32_t j = blockIdx.x * 4 + (threadIdx.x >> 6); j < ng; j += gridDim.x * 4) {
        const uint32_t k = perm[j];
        const uint64_t b = rec_off[k];
        const uint32_t n = (uint32_t)(rec_off[k + 1] - b);
        const uint32_t *p = pcs + b;
        // samples: s_l = floor(l n / NS) (every element when n <= NS)
        const uint32_t ns = min(n, SPLIT_NS);
        const uint32_t sl = n <= SPLIT_NS ? l : (uint32_t)(((uint64_t)l * n) >> SPLIT_LNS);
        const uint32_t x = l < ns ? p[sl] : SENT;
        uint32_t kx;
        const bool xin = pc_index_range(X, x, &kx);
        uint32_t bad = (uint32_t)(l < ns && x != SENT && !xin);
        if (x == SENT || !xin) kx = 0xFFFFFFFFu;  // sorts after every query
        const uint32_t nqry = nr;  // queries 0..nr-2: range bounds; nr-1: the sentinel
        uint32_t res_mine = 0;     // lane q < nr ends with query q's answer
        for (uint32_t g0 = 0; g0 < nqry; g0 += SQ_G) {
            uint32_t lo[SQ_G], hi[SQ_G], cnt[SQ_G], v[SQ_G];
#pragma unroll
            for (int g = 0; g < SQ_G; g++) {
                const uint32_t qy = g0 + g;
                v[g] = qy + 1 < nqry ? (qy + 1) << rsh : 0xFFFFFFFFu;
                const uint32_t c = qy < nqry ? (uint32_t)__popcll(__ballot(l < ns && kx < v[g])) : 0u;
                if (n <= SPLIT_NS) {
                    lo[g] = c;
                    hi[g] = c;
                } else {
                    lo[g] = c == 0 ? 0u : (uint32_t)(((uint64_t)(c - 1) * n) >> SPLIT_LNS) + 1;
                    hi[g] = c == SPLIT_NS ? n : (uint32_t)(((uint64_t)c * n) >> SPLIT_LNS);
                    if (qy >= nqry) hi[g] = lo[g];
                }
                cnt[g] = 0;
            }
            for (uint32_t o = 0;; o += 64) {
                bool more = false;
                uint32_t e[SQ_G];
#pragma unroll
                for (int g = 0; g < SQ_G; g++) {
                    const uint32_t i = lo[g] + o + l;
                    e[g] = i < hi[g] ? p[i] : SENT;
                    more |= lo[g] + o + 64 < hi[g];
                }
#pragma unroll
                for (int g = 0; g < SQ_G; g++) {
                    uint32_t ke;
                    const bool ein = pc_index_range(X, e[g], &ke);
                    if (e[g] == SENT || !ein) ke = 0xFFFFFFFFu;
                    cnt[g] += (uint32_t)__popcll(__ballot(lo[g] + o + l < hi[g] && ke < v[g]));
                }
                if (!__ballot(more)) break;
            }
#pragma unroll
            for (int g = 0; g < SQ_G; g++)
                if (l == g0 + g) res_mine = lo[g] + cnt[g];
        }
        // lane q < nr holds boundary q; the last is the length without sentinels
        const uint32_t neff = __shfl(res_mine, nr - 1, 64);
        uint32_t prev = __shfl_up(res_mine, 1, 64);
        if (l == 0) prev = 0;
        // the record's last PC, and each boundary's neighbours
        if (l == 0 && neff) {
            uint32_t kl;
            bad |= (uint32_t)!pc_index_range(X, p[neff - 1], &kl);
        }
        if (l + 1 < nr && res_mine > 0 && res_mine < neff && p[res_mine - 1] > p[res_mine])
            bad |= 2u;
        const bool mono = !__ballot(l < nr && res_mine < prev);
        const uint64_t eb = __ballot(bad & 1u), eo = __ballot(bad & 2u);
        if (l == 0 && (eb || eo || !mono)) stats[0] = eb ? 1u : 3u;
        if (l < nr) {
            const bool ok = mono && !eb;
            const uint64_t i = (uint64_t)l * stride + j;
            nq[i] = ok ? res_mine - prev : 0u;
            Bq[i] = b + (ok ? prev : 0u);
        }
    }
}

// rows of a sub-run of n PCs starting at pcs index b: 256-PC rows aligned to 4
__device__ __forceinline__ uint32_t sub_rows(uint32_t n, uint64_t b) {
    return n ? (uint32_t)(((b & 3) + n + 255) >> 8) : 0u;
}

// Row counts scanned exclusively into Rq[q][0..m) for every
// range q, in chunks of RS_CHUNK: pass 1 sums each chunk, pass 2 scans a
// chunk from the sum of the chunks before it; Rq[q][m] = the range's rows.
constexpr uint32_t RS_CHUNK = 8192;

__global__ __launch_bounds__(1024) void range_sum_kernel(const uint32_t *__restrict__ nq,
                                                         const uint64_t *__restrict__ Bq,
                                                         uint32_t m, uint32_t stride,
                                                         uint32_t *__restrict__ csum) {
    __shared__ uint32_t tmp[1024 / 64 + 1];
    const uint32_t q = blockIdx.y, b = blockIdx.x, nb = gridDim.x;
    const uint32_t *a = nq + (uint64_t)q * stride + (uint64_t)b * RS_CHUNK;
    const uint64_t *bb = Bq + (uint64_t)q * stride + (uint64_t)b * RS_CHUNK;
    const uint32_t n = min(RS_CHUNK, m - b * RS_CHUNK);
    uint32_t v = 0;
    for (uint32_t i = threadIdx.x; i < n; i += 1024) v += sub_rows(a[i], bb[i]);
    uint32_t tot;
    block_excl_scan<1024>(v, tmp, &tot);
    if (threadIdx.x == 0) csum[q * nb + b] = tot;
}

__global__ __launch_bounds__(1024) void range_scan_kernel(const uint32_t *__restrict__ nq,
                                                          const uint64_t *__restrict__ Bq,
                                                          uint32_t m, uint32_t stride,
                                                          const uint32_t *__restrict__ csum,
                                                          uint32_t *__restrict__ Rq) {
    __shared__ uint32_t tmp[1024 / 64 + 1];
    const uint32_t q = blockIdx.y, b = blockIdx.x, nb = gridDim.x;
    const uint32_t *a = nq + (uint64_t)q * stride;
    const uint64_t *bb = Bq + (uint64_t)q * stride;
    uint32_t *R = Rq + (uint64_t)q * stride;
    uint32_t carry = 0;
    for (uint32_t i = 0; i < b; i++) carry += csum[q * nb + i];
    constexpr uint32_t PT = RS_CHUNK / 1024;
    const uint32_t i0 = b * RS_CHUNK + threadIdx.x * PT;
    uint32_t v[PT], sum = 0;
#pragma unroll
    for (uint32_t u = 0; u < PT; u++) {
        v[u] = i0 + u < m ? sub_rows(a[i0 + u], bb[i0 + u]) : 0u;
        sum += v[u];
    }
    uint32_t tot;
    uint32_t run = carry + block_excl_scan<1024>(sum, tmp, &tot);
#pragma unroll
    for (uint32_t u = 0; u < PT; u++) {
        if (i0 + u < m) R[i0 + u] = run;
        run += v[u];
    }
    if (b == nb - 1 && threadIdx.x == 1023) R[m] = run;
}

// Work-item prefix over (call, range) pairs in RANGE-major order, p = q *
// ncalls + c: ceil(rows / CHR) items each.  Items run in that order, so the
// workgroups resident at any time test PCs of one key range, and the range's
// slice of the membership table (2^RSH bytes) stays in L2 for their byte
// gathers (call-major, the gathers spread over the whole table).
__global__ __launch_bounds__(1024) void item_scan_kernel(const uint32_t *__restrict__ coff,
                                                         int ncalls, uint32_t nr,
                                                         const uint32_t *__restrict__ Rq,
                                                         uint32_t stride, uint32_t CHR,
                                                         uint32_t *__restrict__ ipre) {
    __shared__ uint32_t tmp[1024 / 64 + 1];
    const uint32_t ne = (uint32_t)ncalls * nr;
    uint32_t carry = 0;
    for (uint32_t e0 = 0; e0 < ne; e0 += 1024) {
        const uint32_t e = e0 + threadIdx.x;
        uint32_t v = 0;
        if (e < ne) {
            const uint32_t q = e / (uint32_t)ncalls, c = e - q * (uint32_t)ncalls;
            const uint32_t *R = Rq + (uint64_t)q * stride;
            v = (R[coff[c + 1]] - R[coff[c]] + CHR - 1) / CHR;
        }
        uint32_t tot;
        const uint32_t p = block_excl_scan<1024>(v, tmp, &tot);
        if (e < ne) ipre[e] = carry + p;
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) ipre[ne] = carry;
}

// Where each range's rows start in the row array: qoff[q] = sum of the
// earlier ranges' row counts.
__global__ void row_offsets_kernel(const uint32_t *__restrict__ Rq, uint32_t m, uint32_t stride,
                                   uint32_t nr, uint32_t *__restrict__ qoff) {
    if (threadIdx.x == 0) {
        uint32_t o = 0;
        for (uint32_t q = 0; q < nr; q++) {
            qoff[q] = o;
            o += Rq[(uint64_t)q * stride + m];
        }
        qoff[nr] = o;
    }
}

// Work-item descriptors {e = c * nr + q, first row, end row}: thread per pair,
// items placed in range-major order (item_scan_kernel).
__global__ __launch_bounds__(256) void desc_kernel(const uint32_t *__restrict__ coff, int ncalls,
                                                   uint32_t nr, const uint32_t *__restrict__ Rq,
                                                   uint32_t stride, uint32_t CHR,
                                                   const uint32_t *__restrict__ ipre,
                                                   uint4 *__restrict__ desc) {
    const uint32_t ne = (uint32_t)ncalls * nr;
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < ne; p += gridDim.x * blockDim.x) {
        const uint32_t q = p / (uint32_t)ncalls, c = p - q * (uint32_t)ncalls, e = c * nr + q;
        const uint32_t *R = Rq + (uint64_t)q * stride;
        const uint32_t r0 = R[coff[c]], r1 = R[coff[c + 1]], base = ipre[p];
        for (uint32_t i = 0; r0 + i * CHR < r1; i++)
            desc[base + i] = make_uint4(e, r0 + i * CHR, min(r0 + (i + 1) * CHR, r1), 0u);
    }
}

// Row descriptors of range q's stream, one thread per (grouped record, q):
// {pcs index of the row's first element (a multiple of 4), record k, first
// valid element | end element << 9 | "the row starts the sub-run" << 18
// (its first valid PC has no predecessor to compare with), 0}.
__global__ __launch_bounds__(256) void row_fill_kernel(const uint32_t *__restrict__ nq,
                                                       const uint64_t *__restrict__ Bq,
                                                       const uint32_t *__restrict__ Rq,
                                                       const uint32_t *__restrict__ perm,
                                                       const uint32_t *__restrict__ coff,
                                                       int ncalls, uint32_t nr, uint32_t stride,
                                                       const uint32_t *__restrict__ qoff,
                                                       uint4 *__restrict__ rows) {
    const uint32_t ng = coff[ncalls];
    const uint64_t total = (uint64_t)ng * nr;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t q = (uint32_t)(i / ng), j = (uint32_t)(i - (uint64_t)q * ng);
        const uint64_t x = (uint64_t)q * stride + j;
        const uint32_t n = nq[x], r = Rq[x];
        if (!n) continue;
        const uint32_t b = (uint32_t)Bq[x], k = perm[j], a0 = b & ~3u, end = b + n;
        uint4 *out = rows + qoff[q] + r;
        for (uint32_t st = a0, i = 0; st < end; st += 256, i++) {
            const uint32_t lo = st == a0 ? b - a0 : 0u, hi = min(256u, end - st);
            out[i] = make_uint4(st, k, lo | hi << 9 | (st == a0 ? 1u << 18 : 0u), 0u);
        }
    }
}

// The candidate pass.  Work item w -> (call c, range q, rows [r0, r1) of
// range q's row stream).  The workgroup stages (maxCover[c] | flakes) over
// range q in LDS; each wave takes 64 consecutive rows at a time (one
// descriptor per lane, read back wave-uniform with readlane) and streams
// them NC_U rows per step through buffer loads (row base in an SGPR, lane
// offset constant), the next step's loads in flight while the current step
// is tested.  The staging loads and each wave's first step are in flight
// together.  Per PC: one subtract (index relative to the range), one LDS
// bit test, one compare with its predecessor (DPP wave shift).
// Validity: the split pass checks each record's ends against the index
// space and its range boundaries; a sorted record then has every PC of
// sub-run q inside range q, so the only per-PC check is sortedness (stats
// 3), which every unsorted record fails somewhere (the LDS index is masked,
// so a stray PC of an unsorted record stays in bounds until the batch is
// rejected).  KEY: dense keys (pc >> kshift) - kbase, else pc - pc_lo.
// lanes [a, b) of a wave as a mask (a <= b <= 64)
__device__ __forceinline__ uint64_t lane_range(uint32_t a, uint32_t b) {
    const uint64_t hi = b >= 64 ? ~0ull : ((1ull << b) - 1ull);
    const uint64_t lo = a >= 64 ? ~0ull : ((1ull << a) - 1ull);
    return hi & ~lo;
}

// SGPRs capped: above 80 the hardware admits one 1024-thread workgroup per
// CU instead of two (MI355X_MICROARCH.md, residency), whatever the
// occupancy API reports.
// cache policy of the candidate pass's PC stream loads: nt (2), the stream
// is read once and the membership table keeps more of its L2 share (C5
// steady state 0.967 vs 0.991 ms per batch; the same policy on Minimize's
// chunk stream: 2.96 vs 2.88 ms, not used there)
#ifndef SYZ_NC_PC_AUX
#define SYZ_NC_PC_AUX 2
#endif
#ifndef SYZ_NC_KEY_WPE
#define SYZ_NC_KEY_WPE 4  // key mode: 128 VGPRs (the deferred membership bytes) at one workgroup per CU: 0.97 vs 1.41 ms per C5 batch at 8
#endif
// SEP (key mode, kshift <= 4): no per-PC membership gathers here; the
// separate pass (newcov_memb_kernel) checks every PC from LDS, and this pass
// checks its candidates only (the keys of maxCover | flakes all hold a
// universe PC, so a PC whose key has none is always a candidate).
template <bool KEY, bool SEP>
__global__ __launch_bounds__(LC_THREADS, KEY ? SYZ_NC_KEY_WPE : 8) __attribute__((amdgpu_num_sgpr(72))) void newcov_cand_lds_kernel(
    const uint32_t *__restrict__ pcs, uint32_t npc, const uint32_t *__restrict__ mfl,
    uint64_t words_per_call, Index X, uint32_t nr, const uint32_t *__restrict__ ipre, uint32_t ne,
    const uint4 *__restrict__ desc, const uint4 *__restrict__ rows,
    const uint32_t *__restrict__ qoff, uint2 *__restrict__ clist, uint32_t *__restrict__ stats) {
    extern __shared__ uint4 s_m4[];  // (1 << RSH) / 128 uint4
    __shared__ uint2 s_cb[LC_THREADS / 64 * LC_CBW];  // per wave: pending candidates
    const uint32_t t = threadIdx.x, w = blockIdx.x, l = __lane_id(), wv = t >> 6;
    if (w >= ipre[ne]) return;  // grid is an upper bound
    const uint4 d = desc[w];
    const uint32_t e = d.x, c = e / nr, q = e - c * nr, r0 = d.y, r1 = d.z;
    const uint4 *R = rows + qoff[q];
    const __amdgpu_buffer_rsrc_t pr =
        __builtin_amdgcn_make_buffer_rsrc((void *)pcs, 0, npc * 4u, 0x00020000);
    // staging loads of (maxCover[c] | flakes) over indices [q << RSH, (q+1) << RSH)
    // (words_per_call is a multiple of 4)
    const uint64_t wbase = (uint64_t)q << (RSH - 5);
    const uint32_t nv = (uint32_t)(min<uint64_t>((uint64_t)1 << (RSH - 5), words_per_call - wbase) >> 2);
    const uint4 *M4 = (const uint4 *)(mfl + (uint64_t)c * words_per_call + wbase);
    constexpr int SV = (1 << (RSH - 7)) / LC_THREADS;  // uint4 per thread
    uint4 sv[SV];
#pragma unroll
    for (int i = 0; i < SV; i++) {
        const uint32_t j = t + i * LC_THREADS;
        sv[i] = M4[j < nv ? j : 0u];  // (selected at the LDS store)
    }
    const uint32_t *s_m = (const uint32_t *)s_m4;
    const uint32_t obase = (KEY ? X.kbase : X.pc_lo) + (q << RSH);
    const uint32_t ks = KEY ? X.kshift : 0u;
    // key mode: every PC is checked against the universe (keys.hip), one byte
    // gather per PC with a 32-bit offset (a lane past the sub-run reads past
    // the table's end: 0, no fetch)
    const __amdgpu_buffer_rsrc_t lr = __builtin_amdgcn_make_buffer_rsrc(
        (void *)X.low_of_key, 0, KEY ? (int)X.span : 0, 0x00020000);
    const uint32_t lowmask = (1u << ks) - 1u;
    uint32_t badv = 0;  // this lane saw a PC below its predecessor
    uint32_t nonv = 0;  // this lane saw a PC outside the universe
    uint4 my = make_uint4(0, 0, 0, 0);
    uint32_t nrow = 0, p0v = 0;
    uint2 *cb = s_cb + wv * LC_CBW;
    uint32_t nc = 0;  // candidates in cb (wave-uniform)
    auto flush = [&]() {
        uint32_t base = 0;
        if (l == 0) base = atomicAdd(&stats[1], nc);
        base = wave_readfirstlane(base);
        if (l < nc) clist[base + l] = cb[l];
        nc = 0;
    };
    auto emit = [&](bool cand, uint32_t k, uint32_t pc) {
        // candidates collect in the wave's LDS buffer (no global atomic round
        // trip in the loop)
        const uint64_t m = __ballot(cand);
        if (m) {
            const uint32_t n = (uint32_t)__popcll(m);
            const uint32_t rank = (uint32_t)__popcll(m & ((1ull << l) - 1ull));
            if (nc + n > LC_CBW) flush();
            if (n > LC_CBW) {  // a row with many: straight to the list
                uint32_t base = 0;
                if (l == 0) base = atomicAdd(&stats[1], n);
                base = wave_readfirstlane(base);
                if (cand) clist[base + rank] = make_uint2(k, pc);
            } else {
                if (cand) cb[nc + rank] = make_uint2(k, pc);
                nc += n;
            }
        }
    };
    // the 64 rows' descriptors (lane i: row rb + i) and the PC before each
    // row (0 when the row starts its sub-run: nothing to compare against)
    // this wave's rows: an even share of the item's, contiguous
    const uint32_t per = (r1 - r0 + LC_THREADS / 64 - 1) / (LC_THREADS / 64);
    const uint32_t w0 = min(r1, r0 + wv * per), w1 = min(r1, w0 + per);
    auto rows64 = [&](uint32_t rb_) {
        nrow = min(64u, w1 - rb_);
        const uint4 dsc = R[rb_ + min(l, nrow - 1)];
        my = l < nrow ? dsc : make_uint4(dsc.x, 0, 0, 0);  // past the end: no valid element
        const bool need = l < nrow && !(my.z >> 18 & 1u);
        const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(pr, need ? (my.x - 1) * 4u : 0xFFFFFFF0u, 0, 0);
        p0v = need ? v : 0u;
    };
    // loads of rows [s0, s0 + NC_U) of the current 64: lane l holds elements
    // 4l .. 4l+3 of a row; a lane with none valid reads past the buffer's end
    // (returns 0, fetches nothing)
    auto issue = [&](uint32_t s0, uint4 *pc) {
#pragma unroll
        for (int u = 0; u < LC_U; u++) {
            const uint32_t i = (s0 + u) & 63;
            const uint32_t ra = wave_readlane(my.x, i);
            const uint32_t z = wave_readlane(my.z, i);
            const uint32_t lo = z & 511u, hi = (z >> 9) & 511u;
            const bool any = s0 + u < nrow && 4 * l + 3 >= lo && 4 * l < hi;
            pc[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  pr, any ? l * 16u : 0xFFFFFFF0u, any ? ra * 4u : 0u,
                                                  SYZ_NC_PC_AUX));
        }
    };
    // key mode: the membership bytes of a step's rows, gathered BEFORE the next
    // step's loads are issued, so testing them waits for this step's loads
    // only (gathered inside the test, each wait also drained the prefetched
    // next step: C5 1.23 ms per batch)
    uint32_t mb[LC_U * 4];
    auto gather = [&](uint32_t s0, const uint4 *pc) {
        if (!KEY || SEP) return;
#pragma unroll
        for (int u = 0; u < LC_U; u++) {
            const uint32_t i = (s0 + u) & 63;
            const uint32_t z = wave_readlane(my.z, i);
            const uint32_t lo = z & 511u, hi = (z >> 9) & 511u;
            const bool row = s0 + u < nrow;  // wave-uniform
            const uint32_t v[4] = {pc[u].x, pc[u].y, pc[u].z, pc[u].w};
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const bool in = row && 4 * l + c >= lo && 4 * l + c < hi;
                mb[u * 4 + c] = __builtin_amdgcn_raw_buffer_load_b8(
                    lr, in ? (v[c] >> ks) - obase + (q << RSH) : 0xFFFFFFF0u, 0, 0);
            }
        }
    };
    // per-lane flags over a row's four components, one ballot per row
    // (a ballot and two lane masks per component made the test SALU-bound)
    auto test = [&](uint32_t s0, const uint4 *pc) {
#pragma unroll
        for (int u = 0; u < LC_U; u++) {
            if (s0 + u >= nrow) break;  // wave-uniform
            const uint32_t i = (s0 + u) & 63;
            const uint32_t z = wave_readlane(my.z, i);
            const uint32_t lo = z & 511u, hi = (z >> 9) & 511u, first = z >> 18 & 1u;
            const uint32_t lo1 = lo + first, n = hi - lo, n1 = hi - lo1;
            const uint32_t v[4] = {pc[u].x, pc[u].y, pc[u].z, pc[u].w};
            // bitmap words of the four components (the word index is masked
            // into the staged range, so reads are unconditional and in flight
            // together)
            uint32_t o[4], wd[4];
#pragma unroll
            for (int c = 0; c < 4; c++) {
                o[c] = (KEY ? v[c] >> ks : v[c]) - obase;
                wd[c] = s_m[(o[c] >> 5) & ((1u << (RSH - 5)) - 1)];
            }
            // element 4l's predecessor: lane l-1's last element (DPP wave shift),
            // for lane 0 the PC before the row
            const uint32_t p0 =
                __builtin_amdgcn_update_dpp(wave_readlane(p0v, i), v[3], 0x138, 0xF, 0xF, false);
            uint32_t cand = 0;
#pragma unroll
            for (int c = 0; c < 4; c++) {
                // element 4l + c is valid / has a predecessor in the sub-run
                const uint32_t el = 4 * l + c;
                const bool valid = el - lo < n, pv = el - lo1 < n1;
                badv |= (uint32_t)(pv & ((c ? v[c - 1] : p0) > v[c]));
                if (KEY && !SEP) nonv |= (uint32_t)(valid & (mb[u * 4 + c] != (v[c] & lowmask)));
                cand |= (uint32_t)(valid & !((wd[c] >> (o[c] & 31)) & 1u)) << c;
            }
            if (__ballot(cand != 0)) {  // rare
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    const uint64_t cm = __ballot((cand >> c) & 1u);
                    if (!cm) continue;
                    const bool mine = (cm >> l) & 1u;
                    if (KEY && SEP) {  // the candidates' membership, one byte each
                        const uint32_t mc = __builtin_amdgcn_raw_buffer_load_b8(
                            lr, mine ? (v[c] >> ks) - obase + (q << RSH) : 0xFFFFFFF0u, 0, 0);
                        nonv |= (uint32_t)(mine & (mc != (v[c] & lowmask)));
                    }
                    emit(mine, wave_readlane(my.y, i), v[c]);
                }
            }
        }
    };
    uint4 pcA[LC_U], pcB[LC_U];
    uint32_t rb = w0;
    if (rb < w1) {  // this wave's first step, in flight with the staging loads
        rows64(rb);
        issue(0, pcA);
    }
#pragma unroll
    for (int i = 0; i < SV; i++) {
        const uint32_t j = t + i * LC_THREADS;
        s_m4[j] = j < nv ? sv[i] : make_uint4(~0u, ~0u, ~0u, ~0u);
    }
    __syncthreads();
    for (; rb < w1; rb += 64) {
        if (rb != w0) {
            rows64(rb);
            issue(0, pcA);
        }
        // unconditional issues: a load under a branch makes the compiler drain
        // every load at the loop head, which would serialise the two buffers
        for (uint32_t s0 = 0; s0 < nrow; s0 += 2 * LC_U) {
            gather(s0, pcA);
            issue(s0 + LC_U, pcB);
            test(s0, pcA);
            gather(s0 + LC_U, pcB);
            issue(s0 + 2 * LC_U, pcA);
            test(s0 + LC_U, pcB);
        }
    }
    if (nc) flush();
    if (__ballot(badv) && l == 0) stats[0] = 3u;
    if (__ballot(nonv) && l == 0) stats[0] = 1u;  // not in the universe: rejected like a PC out of range
}

// ---------------------------------------------------------------------------
// Fused candidate + membership pass (key mode, kshift <= 4): every PC of the
// batch is read once.  Ranges of 2^RSF = 2^18 keys: a workgroup holds the
// range's universe low bits as nibbles (128 KB, nib_build_kernel) and one
// call's maxCover | flakes bits over the range (32 KB) — the whole 160 KB of
// LDS — and tests each PC of its rows against both:
//   covered, nibble == the PC's low bits   nothing (the common case)
//   covered, nibble != low bits            not a universe PC: batch rejected
//   uncovered                              candidate; its membership is
//                                          checked exactly from low_of_key
// (a key of maxCover | flakes always holds a universe PC, so a PC on a key
// with none is uncovered and goes the exact way).
// Persistent slices: workgroup g takes the g-th of G equal slices of the row
// stream (range-major, calls in order inside a range: row_fill_kernel), so
// its rows are a run of SEGMENTS (call c, range q).  It restages the nibbles
// when the range changes (once or twice per slice) and the call's bits per
// segment; the next segment's bits are loaded into registers while the
// current one streams, so a segment switch is two barriers and a 32 KB LDS
// store (a workgroup per (call, range) item paid its launch, staging and
// first loads in series per item: 0.49 ms per C5 batch).  With no LDS left, a
// wave buffers up to 64 candidates in registers (lane j holds the j-th),
// appended by a full-wave ds_permute that is a bijection (candidate lanes to
// the free slots after the buffered ones, the others to the rest).
constexpr uint32_t RSF = 18;
constexpr size_t FUSED_LDS = ((size_t)1 << (RSF - 1)) + ((size_t)1 << (RSF - 3));  // 160 KB
constexpr uint32_t FG_MAX = 4096;  // slices
#ifndef SYZ_NC_FU
#define SYZ_NC_FU 4
#endif
constexpr int FU = SYZ_NC_FU;  // rows per step of the fused pass (two steps in flight)
#ifndef SYZ_NC_CBD
#define SYZ_NC_CBD 4
#endif
constexpr int CBD = SYZ_NC_CBD;  // candidate buffer rows per wave (fused pass): 1/4/8 ->
                                 // early-regime fused pass 1083/774/850 us per batch

// The ranges' row offsets (row_offsets_kernel's qoff), the segment starts in
// the row stream, flat s = q * nc + c: segb[q * (nc + 1) + c] = qoff[q] +
// Rq[q][coff[c]] (c <= nc), and for each slice g the segment holding its first
// row (the last s starting at or before it).  One workgroup.
__global__ __launch_bounds__(1024) void fused_seg_kernel(const uint32_t *__restrict__ coff,
                                                         int ncalls, uint32_t nr,
                                                         const uint32_t *__restrict__ Rq,
                                                         uint32_t m, uint32_t stride,
                                                         uint32_t *__restrict__ qoff,
                                                         uint32_t G, uint32_t *__restrict__ segb,
                                                         uint32_t *__restrict__ wg_seg) {
    // qoff: one wave, lane q loads range q's row count (nr <= NR_MAX = 32),
    // a DPP scan (thread 0 walking the ranges paid a dependent load each)
    __shared__ uint32_t s_qoff[NR_MAX + 1];
    if (threadIdx.x < 64) {
        const uint32_t q = threadIdx.x;
        const uint32_t rc = q < nr ? Rq[(uint64_t)q * stride + m] : 0u;
        const uint32_t inc = wave_incl_scan(rc);
        if (q <= nr) {
            qoff[q] = inc - rc;
            s_qoff[q] = inc - rc;
        }
    }
    __syncthreads();
    // the segment starts also go to LDS when they fit: the slices' binary
    // searches then wait on LDS reads, not on ~13 dependent global loads each
    // (17 us of the C5 batch with the table read from L2)
    constexpr uint32_t SB_LDS = 12288;
    __shared__ uint32_t s_sb[SB_LDS];
    const uint32_t nc = (uint32_t)ncalls, n = nr * (nc + 1);
    const bool in_lds = n <= SB_LDS;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t q = i / (nc + 1), c = i - q * (nc + 1);
        const uint32_t v = s_qoff[q] + Rq[(uint64_t)q * stride + coff[c]];
        segb[i] = v;
        if (in_lds) s_sb[i] = v;
    }
    __syncthreads();
    const uint32_t *sb = in_lds ? s_sb : segb;
    const uint32_t rt = s_qoff[nr], ns = nr * nc;
    for (uint32_t g = threadIdx.x; g < G; g += blockDim.x) {
        const uint32_t a = (uint32_t)((uint64_t)rt * g / G);
        uint32_t lo = 0, hi = ns;  // largest s with start(s) <= a (start(0) = 0)
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1, q = mid / nc;
            if (sb[q * (nc + 1) + (mid - q * nc)] <= a) lo = mid; else hi = mid;
        }
        wg_seg[g] = lo;
    }
}

__global__ __launch_bounds__(LC_THREADS, 1) void newcov_fused_kernel(
    const uint32_t *__restrict__ pcs, uint32_t npc, const uint32_t *__restrict__ mfl_,
    const uint32_t *__restrict__ maxc, const uint32_t *__restrict__ flk,
    const uint32_t *__restrict__ mode,
    uint64_t words_per_call, const uint32_t *__restrict__ nib, uint64_t nib_words, Index X,
    uint32_t nr, int ncalls, const uint32_t *__restrict__ segb,
    const uint32_t *__restrict__ wg_seg, const uint4 *__restrict__ rows,
    const uint32_t *__restrict__ qoff, uint2 *__restrict__ clist, uint32_t *__restrict__ stats) {
    extern __shared__ uint4 s_f4[];  // nibbles [0, 128 KB), then the call's bits
    constexpr uint32_t NBW = 1u << (RSF - 3), MBW = 1u << (RSF - 5);  // words
    constexpr int SVM = MBW / 4 / LC_THREADS, SVN = NBW / 4 / LC_THREADS;
    const uint32_t *s_nb = (const uint32_t *)s_f4;
    const uint32_t *s_m = s_nb + NBW;
    const uint32_t t = threadIdx.x, l = __lane_id(), wv = t >> 6;
    const uint32_t nc = (uint32_t)ncalls, ns = nr * nc;
    const uint32_t rt = qoff[nr];
    const uint32_t a = (uint32_t)((uint64_t)rt * blockIdx.x / gridDim.x);
    const uint32_t b = (uint32_t)((uint64_t)rt * (blockIdx.x + 1) / gridDim.x);
    if (a >= b) return;
    const __amdgpu_buffer_rsrc_t pr =
        __builtin_amdgcn_make_buffer_rsrc((void *)pcs, 0, npc * 4u, 0x00020000);
    const uint32_t ks = X.kshift, lowmask = (1u << ks) - 1u;
    const __amdgpu_buffer_rsrc_t lr =
        __builtin_amdgcn_make_buffer_rsrc((void *)X.low_of_key, 0, (int)X.span, 0x00020000);
    // segment s clipped to the slice (empty if it lies outside)
    auto seg = [&](uint32_t s, uint32_t &q, uint32_t &c, uint32_t &lo, uint32_t &hi) {
        q = s / nc;
        c = s - q * nc;
        const uint32_t *sb = segb + q * (nc + 1) + c;
        lo = max(sb[0], a);
        hi = min(sb[1], b);
    };
    // mfl mode 1 (nc_zero_kernel): mfl is stale, stage maxCover | flakes
    const bool stale = mode && mode[0] == 1u;
    const uint32_t *mfl = stale ? maxc : mfl_;
    auto load_bits = [&](uint32_t q, uint32_t c, uint4 (&sm)[SVM]) {
        const uint64_t mb = (uint64_t)q * MBW;
        const uint32_t nvm = (uint32_t)(min<uint64_t>(MBW, words_per_call - mb) >> 2);
        const uint4 *M4 = (const uint4 *)(mfl + (uint64_t)c * words_per_call + mb);
        if (stale) {  // flakes: one bitmap for every call, L2-resident
            const uint4 *F4 = (const uint4 *)(flk + mb);
            uint4 fv[SVM];
#pragma unroll
            for (int i = 0; i < SVM; i++) {
                const uint32_t j = t + i * LC_THREADS;
                sm[i] = j < nvm ? M4[j] : make_uint4(~0u, ~0u, ~0u, ~0u);  // past the keys: covered
                fv[i] = j < nvm ? F4[j] : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int i = 0; i < SVM; i++)
                sm[i] = make_uint4(sm[i].x | fv[i].x, sm[i].y | fv[i].y, sm[i].z | fv[i].z,
                                   sm[i].w | fv[i].w);
            return;
        }
#pragma unroll
        for (int i = 0; i < SVM; i++) {
            const uint32_t j = t + i * LC_THREADS;
            sm[i] = j < nvm ? M4[j] : make_uint4(~0u, ~0u, ~0u, ~0u);  // past the keys: covered
        }
    };
    auto store_bits = [&](const uint4 (&sm)[SVM]) {
#pragma unroll
        for (int i = 0; i < SVM; i++) s_f4[NBW / 4 + t + i * LC_THREADS] = sm[i];
    };
    auto stage_nib = [&](uint32_t q) {  // (a short last range reads its real words only)
        const uint64_t nbb = (uint64_t)q * NBW;
        const uint32_t nvn = (uint32_t)(min<uint64_t>(NBW, nib_words - nbb) >> 2);
        const uint4 *N4 = (const uint4 *)(nib + nbb);
        uint4 sn[SVN];
#pragma unroll
        for (int i = 0; i < SVN; i++) {
            const uint32_t j = t + i * LC_THREADS;
            sn[i] = j < nvn ? N4[j] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < SVN; i++) s_f4[t + i * LC_THREADS] = sn[i];
    };
    uint4 my = make_uint4(0, 0, 0, 0);
    uint32_t nrow = 0, p0v = 0, obase = 0, w1 = 0;
    // candidate buffer, CBD rows of 64: the j-th candidate sits in lane j % 64
    // of row j / 64, so a wave appends to the batch's list (one atomic on one
    // counter for the whole GPU) once per up to 64 CBD candidates: in the
    // early regime (~8 M candidates per batch) one append per 64 serialised
    // ~120 K atomics on that address
    uint32_t cbk[CBD], cbp[CBD], ncb = 0;
    auto flush = [&]() {
        uint32_t base = 0;
        if (l == 0) base = atomicAdd(&stats[1], ncb);
        base = wave_readfirstlane(base);
#pragma unroll
        for (int d = 0; d < CBD; d++)
            if (d * 64 + l < ncb) clist[base + d * 64 + l] = make_uint2(cbk[d], cbp[d]);
        ncb = 0;
    };
    auto emit = [&](uint64_t m, uint32_t k, uint32_t pc) {
        const uint32_t n = (uint32_t)__popcll(m);
        if (ncb + n > 64u * CBD) flush();
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        const bool cand = (m >> l) & 1u;
        // a bijection on the lanes: candidates to the lanes of slots ncb.., the
        // others to the rest
        const uint32_t dst = (cand ? ncb + rank : ncb + n + (l - rank)) & 63u;
        const uint32_t pk = (uint32_t)__builtin_amdgcn_ds_permute((int)(dst * 4u), (int)k);
        const uint32_t pp = (uint32_t)__builtin_amdgcn_ds_permute((int)(dst * 4u), (int)pc);
        const uint32_t off = (l - ncb) & 63u;  // this lane's slot ncb + off, if off < n
        const uint32_t row = (ncb + off) >> 6;
#pragma unroll
        for (int d = 0; d < CBD; d++) {
            const bool here = off < n && row == (uint32_t)d;
            cbk[d] = here ? pk : cbk[d];
            cbp[d] = here ? pp : cbp[d];
        }
        ncb += n;
    };
    auto rows64 = [&](uint32_t rb_) {
        nrow = min(64u, w1 - rb_);
        const uint4 dsc = rows[rb_ + min(l, nrow - 1)];
        my = l < nrow ? dsc : make_uint4(dsc.x, 0, 0, 0);
        const bool need = l < nrow && !(my.z >> 18 & 1u);
        const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(pr, need ? (my.x - 1) * 4u : 0xFFFFFFF0u, 0, 0);
        p0v = need ? v : 0u;
    };
    auto issue = [&](uint32_t s0, uint4 *pc) {
#pragma unroll
        for (int u = 0; u < FU; u++) {
            const uint32_t i = (s0 + u) & 63;
            const uint32_t ra = wave_readlane(my.x, i);
            const uint32_t z = wave_readlane(my.z, i);
            const uint32_t lo = z & 511u, hi = (z >> 9) & 511u;
            const bool any = s0 + u < nrow && 4 * l + 3 >= lo && 4 * l < hi;
            pc[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  pr, any ? l * 16u : 0xFFFFFFF0u, any ? ra * 4u : 0u,
                                                  SYZ_NC_PC_AUX));
        }
    };
    // per-lane flags over the row's four components, one ballot per row
    // (ballots and lane masks per component made the test SALU-bound)
    uint32_t badv = 0, nonv = 0;
    auto test = [&](uint32_t s0, const uint4 *pc) {
#pragma unroll
        for (int u = 0; u < FU; u++) {
            if (s0 + u >= nrow) break;  // wave-uniform
            const uint32_t i = (s0 + u) & 63;
            const uint32_t z = wave_readlane(my.z, i);
            const uint32_t lo = z & 511u, hi = (z >> 9) & 511u, first = z >> 18 & 1u;
            const uint32_t lo1 = lo + first, n = hi - lo, n1 = hi - lo1;  // (hi > lo)
            const uint32_t v[4] = {pc[u].x, pc[u].y, pc[u].z, pc[u].w};
            uint32_t o[4], wd[4], nw[4], nbs[4];
#pragma unroll
            for (int c = 0; c < 4; c++) {
                o[c] = (v[c] >> ks) - obase;
                wd[c] = s_m[(o[c] >> 5) & (MBW - 1)];
                nw[c] = s_nb[(o[c] >> 3) & (NBW - 1)];
            }
            const uint32_t p0 =
                __builtin_amdgcn_update_dpp(wave_readlane(p0v, i), v[3], 0x138, 0xF, 0xF, false);
            uint32_t cand = 0;
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const uint32_t el = 4 * l + c;
                const bool valid = el - lo < n, pv = el - lo1 < n1;
                badv |= (uint32_t)(pv & ((c ? v[c - 1] : p0) > v[c]));
                const bool cov = (wd[c] >> (o[c] & 31)) & 1u;
                const uint32_t nb = (nw[c] >> ((o[c] & 7u) * 4u)) & 15u;
                nbs[c] = nb;
                nonv |= (uint32_t)(valid & cov & (nb != (v[c] & lowmask)));
                cand |= (uint32_t)(valid & !cov) << c;
            }
            if (__ballot(cand != 0)) {  // rare in steady state
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    const uint64_t cm = __ballot((cand >> c) & 1u);
                    if (!cm) continue;
                    // the candidates' membership: the staged nibble settles it
                    // unless it reads 15, which a key with no universe PC also
                    // stages (0x7F & 15): only then the exact byte (every
                    // candidate's byte load was ~1/3 of the early regime's
                    // extra fused-pass time)
                    const bool mine = (cm >> l) & 1u;
                    const uint32_t lw = v[c] & lowmask;
                    const bool exact = mine && nbs[c] == 15u && lw == 15u;
                    nonv |= (uint32_t)(mine & !exact & (nbs[c] != lw));
                    if (__ballot(exact)) {
                        const uint32_t mc = __builtin_amdgcn_raw_buffer_load_b8(
                            lr, exact ? (v[c] >> ks) - X.kbase : 0xFFFFFFF0u, 0, 0);
                        nonv |= (uint32_t)(exact & (mc != lw));
                    }
                    emit(cm, wave_readlane(my.y, i), v[c]);
                }
            }
        }
    };
    // a wave's share of segment rows [lo_, hi_): an even split over the waves
    uint32_t w0 = 0;
    auto share = [&](uint32_t lo_, uint32_t hi_) {
        const uint32_t per = (hi_ - lo_ + LC_THREADS / 64 - 1) / (LC_THREADS / 64);
        w0 = min(hi_, lo_ + wv * per);
        w1 = min(hi_, w0 + per);
    };
    uint4 pcA[FU], pcB[FU];
    uint32_t s = wg_seg[blockIdx.x], q, c, lo, hi;
    seg(s, q, c, lo, hi);
    share(lo, hi);
    if (w0 < w1) {  // the first rows' loads, in flight with the staging
        rows64(w0);
        issue(0, pcA);
    }
    {
        uint4 sm[SVM];
        load_bits(q, c, sm);
        stage_nib(q);
        store_bits(sm);
    }
    uint32_t cur_q = q;
    __syncthreads();
    for (;;) {
        // the next segment of the slice (calls with no rows in a range are
        // skipped); its bits load while this one streams
        uint32_t s2 = s + 1, q2 = 0, c2 = 0, lo2 = 0, hi2 = 0;
        bool more = false;
        for (; s2 < ns; s2++) {
            seg(s2, q2, c2, lo2, hi2);
            if (lo2 >= b) break;
            if (hi2 > lo2) {
                more = true;
                break;
            }
        }
        uint4 sm[SVM];
        if (more) load_bits(q2, c2, sm);
        obase = X.kbase + (q << RSF);
        // this wave's rows of the segment; the first 64's descriptors and first
        // step were issued before the segment's barrier
        for (uint32_t rb = w0; rb < w1; rb += 64) {
            if (rb != w0) {
                rows64(rb);
                issue(0, pcA);
            }
            for (uint32_t s0 = 0; s0 < nrow; s0 += 2 * FU) {
                issue(s0 + FU, pcB);
                test(s0, pcA);
                issue(s0 + 2 * FU, pcA);
                test(s0 + FU, pcB);
            }
        }
        if (more) {  // the next segment's first loads, before the barrier
            share(lo2, hi2);
            if (w0 < w1) {
                rows64(w0);
                issue(0, pcA);
            }
        }
        __syncthreads();
        if (!more) break;
        if (q2 != cur_q) {
            stage_nib(q2);
            cur_q = q2;
        }
        store_bits(sm);
        __syncthreads();
        s = s2;
        q = q2;
        c = c2;
        lo = lo2;
        hi = hi2;
    }
    if (ncb) flush();
    if (__ballot(badv) && l == 0) stats[0] = 3u;
    if (__ballot(nonv) && l == 0) stats[0] = 1u;  // not in the universe: rejected like a PC out of range
}

// ---------------------------------------------------------------------------
// Separate membership pass (key mode, kshift <= 4): every PC of the row
// streams against the universe's low bits, staged as nibbles in LDS half a
// range (2^(RSH-1) keys, 128 KB) at a time.  Workgroup (g, h) takes the g-th
// of MB_G equal slices of the whole row stream (ranges in order; the coverage
// is skewed, 40% of the PCs in range 0, so slicing by range left most CUs
// idle: 0.89 ms) and checks their PCs of half h of each range it crosses,
// restaging the table per range: the rows are read once per half, 2 x 4 B per
// PC, instead of one L2 byte request per PC in the candidate pass (those
// requests bound it: 0.92 vs 0.44 ms per C5 batch without them).  A PC whose
// key holds no universe PC is a candidate (its maxCover | flakes bit is
// clear) and checked there exactly.
constexpr int MB_THREADS = 1024;
// (128 / 256 / 384 / 512 slices: 0.645-0.647 / 0.644-0.648 / 0.661 / 0.649-0.650
// ms per steady-state C5 batch)
#ifndef SYZ_NC_MB_G
#define SYZ_NC_MB_G 256
#endif
constexpr uint32_t MB_G = SYZ_NC_MB_G;  // row slices per half (a multiple of 8)
constexpr int MB_U = 4;         // rows per wave step (two steps in flight)

__global__ void nib_build_kernel(const uint8_t *__restrict__ low_of_key, uint64_t nkeys,
                                 uint64_t nwords, uint32_t *__restrict__ nib) {
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords;
         w += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t x = 0;
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) {
            const uint64_t k = w * 8 + j;
            x |= (k < nkeys ? low_of_key[k] & 15u : 0u) << (4 * j);
        }
        nib[w] = x;
    }
}

__global__ __launch_bounds__(MB_THREADS) void newcov_memb_kernel(
    const uint32_t *__restrict__ pcs, uint32_t npc, const uint32_t *__restrict__ nib, Index X,
    uint32_t nr, const uint4 *__restrict__ rows, const uint32_t *__restrict__ qoff,
    uint32_t *__restrict__ stats) {
    extern __shared__ uint4 s_nb4[];  // 2^(RSH-1) nibbles
    constexpr uint32_t HW = 1u << (RSH - 4);  // words per half range
    // workgroups i and i + 8 share an XCD (round-robin dispatch): the two
    // halves of a slice run there together and the second read of the rows
    // hits that XCD's L2
    const uint32_t i16 = blockIdx.x & 15u;
    const uint32_t g = (blockIdx.x >> 4) * 8 + (i16 & 7u), h = i16 >> 3;
    const uint32_t t = threadIdx.x, l = __lane_id(), wv = t >> 6;
    const uint32_t *s_nb = (const uint32_t *)s_nb4;
    const uint32_t rt = qoff[nr];
    uint32_t a = (uint32_t)((uint64_t)rt * g / MB_G);
    const uint32_t b = (uint32_t)((uint64_t)rt * (g + 1) / MB_G);
    uint32_t q = 0;
    while (q + 1 < nr && qoff[q + 1] <= a) q++;
    const uint32_t ks = X.kshift, lowmask = (1u << ks) - 1u;
    const __amdgpu_buffer_rsrc_t pr =
        __builtin_amdgcn_make_buffer_rsrc((void *)pcs, 0, npc * 4u, 0x00020000);
    bool bad = false;
    for (; a < b; q++) {
        const uint32_t e = min(b, qoff[q + 1]);
        if (a >= e) continue;
        // this range's half of the table (the previous one's readers are done)
        __syncthreads();
        const uint4 *src = (const uint4 *)(nib + ((uint64_t)q << (RSH - 3)) + (uint64_t)h * HW);
#pragma unroll
        for (uint32_t i = 0; i < HW / 4 / MB_THREADS; i++)
            s_nb4[t + i * MB_THREADS] = src[t + i * MB_THREADS];
        __syncthreads();
        const uint32_t hb = X.kbase + (q << RSH) + (h << (RSH - 1));  // the half's first key
        // each wave takes 64 consecutive rows at a time, their descriptors
        // one per lane (a single vector load, read back with readlane), and
        // streams them MB_U rows per step, the next step's loads issued before
        // this step is tested (rows past the block load nothing)
        for (uint32_t rb = a + wv * 64; rb < e; rb += (MB_THREADS / 64) * 64) {
            const uint32_t nrow = min(64u, e - rb);
            const uint4 dsc = rows[rb + min(l, nrow - 1)];
            uint4 pa[MB_U], pb[MB_U];
            auto load = [&](uint32_t s0, uint4 (&pc)[MB_U]) {
#pragma unroll
                for (int u = 0; u < MB_U; u++) {
                    const uint32_t i = (s0 + u) & 63;
                    const uint32_t st = wave_readlane(dsc.x, i);
                    const uint32_t z = wave_readlane(dsc.z, i);
                    const bool row = s0 + u < nrow;  // wave-uniform
                    const uint32_t lo = z & 511u, hi = row ? (z >> 9) & 511u : 0u;
                    const bool any = 4 * l + 3 >= lo && 4 * l < hi;
                    pc[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                          pr, any ? l * 16u : 0xFFFFFFF0u,
                                                          any ? st * 4u : 0u, 0));
                }
            };
            auto check = [&](uint32_t s0, const uint4 (&pc)[MB_U]) {
#pragma unroll
                for (int u = 0; u < MB_U; u++) {
                    const uint32_t i = (s0 + u) & 63;
                    const uint32_t z = wave_readlane(dsc.z, i);
                    const bool row = s0 + u < nrow;
                    const uint32_t lo = z & 511u, hi = row ? (z >> 9) & 511u : 0u;
                    const uint32_t v[4] = {pc[u].x, pc[u].y, pc[u].z, pc[u].w};
#pragma unroll
                    for (int c = 0; c < 4; c++) {
                        const uint32_t el = 4 * l + c;
                        const uint32_t rel = (v[c] >> ks) - hb;
                        const bool in = el >= lo && el < hi && rel < (1u << (RSH - 1));
                        const uint32_t nb = (s_nb[(rel >> 3) & (HW - 1)] >> ((rel & 7) * 4)) & 15u;
                        bad |= in & (nb != (v[c] & lowmask));
                    }
                }
            };
            load(0, pa);
            for (uint32_t s0 = 0; s0 < nrow; s0 += 2 * MB_U) {
                load(s0 + MB_U, pb);
                check(s0, pa);
                load(s0 + 2 * MB_U, pa);
                check(s0 + MB_U, pb);
            }
        }
        a = e;
    }
    if (__ballot(bad) && l == 0) stats[0] = 1u;  // not in the universe: the batch is rejected
}

// ---------------------------------------------------------------------------
// First cover over the candidate list: hval[(call, pc)] = min record index,
// then a record is new iff it owns one of its candidates, and each owned
// candidate is OR-ed into maxCover once.

// table capacity for ncand candidates (power of two, load <= 1/2)
__device__ __forceinline__ uint64_t hash_cap(uint32_t ncand) {
    uint64_t cap = 1024;
    while (cap < 2ull * ncand) cap <<= 1;
    return cap;
}

__global__ void hash_clear_kernel(const uint32_t *__restrict__ stats,
                                  unsigned long long *__restrict__ hkey,
                                  uint32_t *__restrict__ hval) {
    if (stats[0] || !stats[1]) return;  // rejected batch / nothing to insert
    const uint64_t cap = hash_cap(stats[1]);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap;
         i += (uint64_t)gridDim.x * blockDim.x) {
        hkey[i] = ~0ull;
        hval[i] = 0xFFFFFFFFu;
    }
}

__device__ __forceinline__ uint64_t hash64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xFF51AFD7ED558CCDull;
    k ^= k >> 33;
    k *= 0xC4CEB9FE1A85EC53ull;
    k ^= k >> 33;
    return k;
}

constexpr uint64_t EMPTY_KEY = ~0ull;

__global__ __launch_bounds__(256) void newcov_insert_kernel(
    const int32_t *__restrict__ callid, const uint2 *__restrict__ clist,
    const uint32_t *__restrict__ stats, unsigned long long *__restrict__ hkey,
    uint32_t *__restrict__ hval) {
    if (stats[0] || !stats[1]) return;
    const uint32_t n = stats[1];
    const uint64_t mask = hash_cap(n) - 1;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint2 kp = clist[i];
        const uint64_t key = (uint64_t)(uint32_t)callid[kp.x] << 32 | kp.y;
        uint64_t h = hash64(key) & mask;
        for (;;) {
            const unsigned long long prev = atomicCAS(&hkey[h], EMPTY_KEY, key);
            if (prev == EMPTY_KEY || prev == key) {
                atomicMin(&hval[h], kp.x);
                break;
            }
            h = (h + 1) & mask;
        }
    }
}

// The batch's zero fills in one launch: stats, the per-call counters, is_new
// The mfl mode (fused pass, key mode).  In the early regime (millions of
// candidates per batch) the ownership pass's atomicOr into mfl = maxCover |
// flakes, one per owned candidate beside the one into maxCover, cost ~0.2 ms
// of a 1.9 ms batch; in the steady state (no candidates) staging maxCover |
// flakes per segment instead of mfl cost 14 us of 0.57 ms.  So the device
// picks per batch, with no host round trip (mode[0] = this batch's, mode[1]
// = the next one's, written by the ownership pass's block 0):
//   0  mfl fresh: the fused pass stages mfl, the ownership pass keeps it;
//   1  mfl stale: the fused pass stages maxCover | flakes, mfl untouched;
//   3  stale, rebuild asked (a batch with few candidates saw mode 1): this
//      kernel rebuilds mfl before the batch's fused pass, mode[0] = 0.
// A batch above NOMFL_CANDS candidates leaves mfl stale (next mode 1).
constexpr uint32_t NOMFL_CANDS = 1u << 19;
__global__ __launch_bounds__(256) void nc_zero_kernel(uint32_t *__restrict__ stats,
                                                      uint32_t *__restrict__ ccnt, uint32_t nc,
                                                      uint8_t *__restrict__ is_new, uint32_t nrec,
                                                      uint32_t *__restrict__ mode,
                                                      const uint4 *__restrict__ maxcov,
                                                      const uint4 *__restrict__ flakes,
                                                      uint64_t vec_per_call, uint64_t nv,
                                                      uint4 *__restrict__ mfl) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, nt = gridDim.x * blockDim.x;
    if (t < 4) stats[t] = 0u;
    for (uint32_t c = t; c < nc; c += nt) ccnt[c] = 0u;
    for (uint32_t k = t; k < nrec; k += nt) is_new[k] = 0;
    if (mode) {
        const uint32_t nx = mode[1];  // (written only by the ownership pass)
        if (nx == 3u)
            for (uint64_t i = t; i < nv; i += nt) {
                const uint4 m = maxcov[i], f = flakes[i % vec_per_call];
                mfl[i] = make_uint4(m.x | f.x, m.y | f.y, m.z | f.z, m.w | f.w);
            }
        if (t == 0) mode[0] = nx == 1u ? 1u : 0u;
    }
}

// stats_out (nullable): the caller's copy of stats[0..2), taken here (the
// last kernel of the batch) instead of by a separate device copy
__global__ __launch_bounds__(256) void newcov_own_kernel(
    const int32_t *__restrict__ callid, const uint2 *__restrict__ clist,
    const uint32_t *__restrict__ stats, const unsigned long long *__restrict__ hkey,
    const uint32_t *__restrict__ hval, uint8_t *__restrict__ is_new,
    uint32_t *__restrict__ maxcov, uint32_t *__restrict__ mfl, uint64_t words_per_call, Index X,
    uint32_t *__restrict__ stats_out) {
    if (stats_out && blockIdx.x == 0 && threadIdx.x < 2) stats_out[threadIdx.x] = stats[threadIdx.x];
    if (stats[0] || !stats[1]) return;
    const uint32_t n = stats[1];
    const uint64_t mask = hash_cap(n) - 1;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint2 kp = clist[i];
        const uint32_t c = (uint32_t)callid[kp.x];
        const uint64_t key = (uint64_t)c << 32 | kp.y;
        uint64_t h = hash64(key) & mask;
        while (hkey[h] != key) h = (h + 1) & mask;
        if (hval[h] == kp.x) {
            is_new[kp.x] = 1;
            uint32_t ix;
            pc_index(X, kp.y, &ix);  // candidates are inside (checked by the cand pass)
            atomicOr(&maxcov[(uint64_t)c * words_per_call + (ix >> 5)], 1u << (ix & 31));
            if (mfl) atomicOr(&mfl[(uint64_t)c * words_per_call + (ix >> 5)], 1u << (ix & 31));
        }
    }
}

// Packed slots, when ncalls x span < 2^32 (C5: 293 x 2^22): one u64 per slot,
// (call x span + index) << 32 | min record, so a probe, its insert (CAS, then
// atomicMin on the same word) and the owner test touch one line, where the
// key and value arrays took two; the clear writes 8 bytes per slot, not 12.
__device__ __forceinline__ uint32_t slot_key(const Index &X, uint32_t c, uint32_t pc) {
    uint32_t ix;
    pc_index_range(X, pc, &ix);  // candidates are inside (checked by the cand pass)
    return c * (uint32_t)X.span + ix;
}

__global__ void hash_clear32_kernel(const uint32_t *__restrict__ stats,
                                    unsigned long long *__restrict__ slots) {
    if (stats[0] || !stats[1]) return;
    const uint64_t cap = hash_cap(stats[1]);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap;
         i += (uint64_t)gridDim.x * blockDim.x)
        slots[i] = EMPTY_KEY;
}

__global__ __launch_bounds__(256) void newcov_insert32_kernel(
    const int32_t *__restrict__ callid, const uint2 *__restrict__ clist,
    const uint32_t *__restrict__ stats, unsigned long long *__restrict__ slots, Index X) {
    if (stats[0] || !stats[1]) return;
    const uint32_t n = stats[1];
    const uint64_t mask = hash_cap(n) - 1;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint2 kp = clist[i];
        const uint32_t key = slot_key(X, (uint32_t)callid[kp.x], kp.y);
        const unsigned long long mine = (unsigned long long)key << 32 | kp.x;
        uint64_t h = hash64(key) & mask;
        for (;;) {
            const unsigned long long prev = atomicCAS(&slots[h], EMPTY_KEY, mine);
            if (prev == EMPTY_KEY) break;
            if ((uint32_t)(prev >> 32) == key) {  // same key: the smaller record stays
                if (prev > mine) atomicMin(&slots[h], mine);
                break;
            }
            h = (h + 1) & mask;
        }
    }
}

__global__ __launch_bounds__(256) void newcov_own32_kernel(
    const int32_t *__restrict__ callid, const uint2 *__restrict__ clist,
    const uint32_t *__restrict__ stats, const unsigned long long *__restrict__ slots,
    uint8_t *__restrict__ is_new, uint32_t *__restrict__ maxcov, uint32_t *__restrict__ mfl,
    uint64_t words_per_call, Index X, uint32_t *__restrict__ stats_out, uint32_t *__restrict__ mode) {
    if (stats_out && blockIdx.x == 0 && threadIdx.x < 2) stats_out[threadIdx.x] = stats[threadIdx.x];
    // the mfl mode (nc_zero_kernel): mode[0] is this batch's for every block
    const uint32_t cand = stats[0] ? 0u : stats[1], cur = mode ? mode[0] : 0u;
    if (mode && blockIdx.x == 0 && threadIdx.x == 0)
        mode[1] = cand > NOMFL_CANDS ? 1u : cur == 1u ? 3u : 0u;
    if (mode && (cand > NOMFL_CANDS || cur == 1u)) mfl = nullptr;  // left stale
    if (stats[0] || !stats[1]) return;
    const uint32_t n = stats[1];
    const uint64_t mask = hash_cap(n) - 1;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint2 kp = clist[i];
        const uint32_t c = (uint32_t)callid[kp.x];
        const uint32_t key = slot_key(X, c, kp.y);
        uint64_t h = hash64(key) & mask;
        unsigned long long v;
        while ((uint32_t)((v = slots[h]) >> 32) != key) h = (h + 1) & mask;
        if ((uint32_t)v == kp.x) {
            is_new[kp.x] = 1;
            const uint32_t ix = key - c * (uint32_t)X.span;
            atomicOr(&maxcov[(uint64_t)c * words_per_call + (ix >> 5)], 1u << (ix & 31));
            if (mfl) atomicOr(&mfl[(uint64_t)c * words_per_call + (ix >> 5)], 1u << (ix & 31));
        }
    }
}

// mfl[c] = maxcov[c] | flakes for every call
__global__ void mfl_build_kernel(const uint4 *__restrict__ maxcov, const uint4 *__restrict__ flakes,
                                 uint64_t vec_per_call, uint64_t n, uint4 *__restrict__ mfl) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 m = maxcov[i], f = flakes[i % vec_per_call];
        mfl[i] = make_uint4(m.x | f.x, m.y | f.y, m.z | f.z, m.w | f.w);
    }
}

__global__ void bits_set_kernel(const uint32_t *__restrict__ pcs, uint64_t n,
                                uint32_t *__restrict__ bm, Index X, uint32_t *__restrict__ err) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t pc = pcs[i];
        if (pc == 0xFFFFFFFFu) continue;  // Union drops the sentinel (cover.go:97)
        uint32_t ix;
        if (!pc_index(X, pc, &ix)) {
            *err = 1u;
            continue;
        }
        atomicOr(&bm[ix >> 5], 1u << (ix & 31));
    }
}

// kshift of a sorted unique universe: min over neighbours of the highest
// differing bit (keys.hip); *out pre-set to 31.
__global__ void universe_shift_kernel(const uint32_t *__restrict__ u, uint32_t n,
                                      uint32_t *__restrict__ out) {
    uint32_t m = 31;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i + 1 < n;
         i += gridDim.x * blockDim.x)
        m = min(m, 31u - (uint32_t)__clz(u[i] ^ u[i + 1]));
    for (int d = 32; d >= 1; d >>= 1) m = min(m, (uint32_t)__shfl_xor(m, d, 64));
    if (__lane_id() == 0) atomicMin(out, m);
}

// kshift of a sorted unique PC list on the device (*d_ks = min over
// neighbours of the highest differing bit; 31 for a single PC): the host
// caps it at SYZCOV_KSHIFT_MAX (corpus.hip's grouped drop-in)
int universe_shift_dev(const uint32_t *u, uint32_t n, uint32_t *d_ks, hipStream_t s) {
    SYZ_HIP(hipMemsetD32Async((hipDeviceptr_t)d_ks, 31, 1, s));
    if (n > 1)
        hipLaunchKernelGGL(universe_shift_kernel, dim3(grid_for(n, 256, 1024)), dim3(256), 0, s, u,
                           n, d_ks);
    SYZ_LAUNCH_CHECK();
    return 0;
}

// addInput (fuzzer.go:372-373): an accepted input's whole cover (flakes
// included, the sentinel excluded) joins corpusCover and maxCover.  One wave
// per record; nothing on a rejected batch.
__global__ __launch_bounds__(256) void accept_or_kernel(const int32_t *__restrict__ callid,
                                                        const uint64_t *__restrict__ rec_off,
                                                        const uint32_t *__restrict__ pcs,
                                                        uint32_t nrec,
                                                        const uint8_t *__restrict__ is_new,
                                                        const uint32_t *__restrict__ stats,
                                                        uint32_t *__restrict__ maxcov,
                                                        uint32_t *__restrict__ corpus,
                                                        uint64_t words, Index X) {
    if (stats[0]) return;
    const uint32_t l = __lane_id();
    for (uint32_t k = blockIdx.x * 4 + (threadIdx.x >> 6); k < nrec; k += gridDim.x * 4) {
        if (!is_new[k]) continue;
        const uint64_t c = (uint32_t)callid[k], b = rec_off[k], n = rec_off[k + 1] - b;
        for (uint64_t i = l; i < n; i += 64) {
            const uint32_t pc = pcs[b + i];
            uint32_t ix;
            if (pc == 0xFFFFFFFFu || !pc_index(X, pc, &ix)) continue;
            atomicOr(&maxcov[c * words + (ix >> 5)], 1u << (ix & 31));
            atomicOr(&corpus[c * words + (ix >> 5)], 1u << (ix & 31));
        }
    }
}

}  // namespace syz

// ------------------------------------------------ host-side orchestration
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

using namespace syz;


static int grow(CoverState *st, size_t need) {
    if (need <= st->scap) return 0;
    if (st->scratch) {
        hipStreamSynchronize(st->s);
        hipFree(st->scratch);
    }
    st->scratch = nullptr;
    st->scap = 0;
    size_t cap = need + need / 2;
    if (hipMalloc(&st->scratch, cap) != hipSuccess) return SYZCOV_ENOMEM;
    st->scap = cap;
    return 0;
}

// CoverState::grp: 3 x (ncalls + 1) + ncalls * NR_MAX + 1 u32, then the
// descriptors (<= ITEMS_MAX + ncalls * NR_MAX + 1 uint4, 16-byte aligned)
static size_t grp_desc_off(int ncalls) {
    return align_up(4 * (3 * ((size_t)ncalls + 1) + (size_t)ncalls * NR_MAX + 1), 256);
}
static size_t grp_bytes(int ncalls) {
    return grp_desc_off(ncalls) + 16 * ((size_t)ITEMS_MAX + (size_t)ncalls * NR_MAX + 1);
}

// (re)allocate the bitmaps for the current index space, zeroed
static int alloc_maps(CoverState *st) {
    if (st->maxcov) hipFree(st->maxcov);
    if (st->flakes) hipFree(st->flakes);
    if (st->corpus) hipFree(st->corpus);
    if (st->mfl) hipFree(st->mfl);
    st->maxcov = st->flakes = st->corpus = st->mfl = nullptr;
    st->mfl_stale = true;
    st->words = ((st->X.span + 127) / 128) * 4;  // 16-byte rows (LDS staging)
    if (!st->grp && hipMalloc(&st->grp, grp_bytes(st->ncalls)) != hipSuccess)
        return SYZCOV_ENOMEM;
    if (hipMalloc(&st->maxcov, (size_t)st->ncalls * st->words * 4) != hipSuccess ||
        hipMalloc(&st->flakes, st->words * 4) != hipSuccess)
        return SYZCOV_ENOMEM;
    SYZ_HIP(hipMemsetAsync(st->maxcov, 0, (size_t)st->ncalls * st->words * 4, st->s));
    SYZ_HIP(hipMemsetAsync(st->flakes, 0, st->words * 4, st->s));
    SYZ_HIP(hipStreamSynchronize(st->s));
    return 0;
}

extern "C" int syzcov_state_create(int ncalls, uint32_t pc_lo, uint64_t pc_span,
                                   syzcov_cover_state *out) {
    if (ncalls <= 0 || pc_span == 0 || pc_span > (1ull << 32) || !out) return SYZCOV_EINVAL;
    if ((uint64_t)pc_lo + pc_span > (1ull << 32)) return SYZCOV_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        set_error("no HIP device");
        return SYZCOV_ENODEV;
    }
    CoverState *st = new (std::nothrow) CoverState();
    if (!st) return SYZCOV_ENOMEM;
    hipGetDevice(&st->dev);
    st->ncalls = ncalls;
    st->pc_lo = pc_lo;
    st->pc_span = pc_span;
    st->X = Index{0, pc_lo, 0, 0, pc_span, nullptr};
    int rc = hipStreamCreateWithFlags(&st->s, hipStreamNonBlocking) == hipSuccess
                 ? alloc_maps(st) : SYZCOV_EHIP;
    if (rc) {
        if (st->maxcov) hipFree(st->maxcov);
        if (st->flakes) hipFree(st->flakes);
        if (st->grp) hipFree(st->grp);
        if (st->s) hipStreamDestroy(st->s);
        delete st;
        return rc;
    }
    *out = (syzcov_cover_state)(uintptr_t)st;
    return 0;
}

extern "C" int syzcov_state_destroy(syzcov_cover_state h) {
    CoverState *st = (CoverState *)(uintptr_t)h;
    if (!st) return SYZCOV_EINVAL;
    hipStreamSynchronize(st->s);
    hipFree(st->maxcov);
    hipFree(st->flakes);
    if (st->corpus) hipFree(st->corpus);
    if (st->mfl) hipFree(st->mfl);
    if (st->pc_of_key) hipFree(st->pc_of_key);
    if (st->low_of_key) hipFree(st->low_of_key);
    if (st->nib) hipFree(st->nib);
    if (st->grp) hipFree(st->grp);
    if (st->scratch) hipFree(st->scratch);
    if (st->ev_state) hipEventDestroy(st->ev_state);
    if (st->ev_dev) hipEventDestroy(st->ev_dev);
    hipStreamDestroy(st->s);
    delete st;
    return 0;
}

static int set_bits(CoverState *st, uint32_t *bm, const uint32_t *pcs, size_t n) {
    if (n == 0) return 0;
    size_t need = align_up(n * 4, 256) + 256;
    int rc = grow(st, need);
    if (rc) return rc;
    uint32_t *dp = (uint32_t *)st->scratch;
    uint32_t *derr = (uint32_t *)((uint8_t *)st->scratch + align_up(n * 4, 256));
    SYZ_HIP(hipMemsetAsync(derr, 0, 4, st->s));
    SYZ_HIP(hipMemcpyAsync(dp, pcs, n * 4, hipMemcpyHostToDevice, st->s));
    hipLaunchKernelGGL(bits_set_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0, st->s, dp,
                       (uint64_t)n, bm, st->X, derr);
    SYZ_LAUNCH_CHECK();
    uint32_t herr = 0;
    SYZ_HIP(hipMemcpyAsync(&herr, derr, 4, hipMemcpyDeviceToHost, st->s));
    SYZ_HIP(hipStreamSynchronize(st->s));
    if (herr) {
        set_error(st->X.key_mode ? "PC outside the registered universe's key range"
                                 : "PC outside the state's PC window");
        return SYZCOV_ERANGE;
    }
    return 0;
}

namespace syz {
int state_grow(CoverState *st, size_t need) { return grow(st, need); }
int state_set_bits(CoverState *st, uint32_t *bm, const uint32_t *pcs, size_t n) {
    return set_bits(st, bm, pcs, n);
}
// corpusCover bitmaps, zeroed, on first use (fuzzer.go:372, 451)
int state_ensure_corpus(CoverState *st) {
    if (st->corpus) return 0;
    const size_t bytes = (size_t)st->ncalls * st->words * 4;
    if (hipMalloc(&st->corpus, bytes) != hipSuccess) {
        st->corpus = nullptr;
        return SYZCOV_ENOMEM;
    }
    SYZ_HIP(hipMemsetAsync(st->corpus, 0, bytes, st->s));
    return 0;
}
// one per-call bitmap back as a sorted PC list (keys mapped to PCs)
int state_bitmap_get(CoverState *st, const uint32_t *bm, uint32_t *out, size_t cap,
                     int64_t *count) {
    return st->X.key_mode
               ? bitmap_to_list(bm, st->X.span, 0, out, cap, count, st->s, st->pc_of_key)
               : bitmap_to_list(bm, st->pc_span, st->pc_lo, out, cap, count, st->s, nullptr);
}
}  // namespace syz

extern "C" int syzcov_state_add(syzcov_cover_state h, int call, const uint32_t *pcs, size_t n) {
    CoverState *st = (CoverState *)(uintptr_t)h;
    if (!st || call < 0 || call >= st->ncalls || (n && !pcs)) return SYZCOV_EINVAL;
    std::lock_guard<std::mutex> g(st->mu);
    hipSetDevice(st->dev);
    st->dirty = true;
    st->mfl_stale = true;
    return set_bits(st, st->maxcov + (size_t)call * st->words, pcs, n);
}

// Key mode (keys.hip): the PC universe (every PC KCOV can report: the return
// addresses of the __sanitizer_cov_trace_pc calls, syz-manager/cover.go:
// 274-306 and :82; inside the window, any order, duplicates allowed) fixes
// kshift / kbase / nkeys; maxCover and flakes become bitmaps over its dense
// keys.  Allowed only while maxCover is empty.  From then on every PC passed
// in is checked against the universe (pc_index): one outside it is rejected
// (the whole batch, or the call), never aliased with the universe PC that
// owns its key.
extern "C" int syzcov_state_set_universe(syzcov_cover_state h, const uint32_t *pcs, size_t n) {
    CoverState *st = (CoverState *)(uintptr_t)h;
    if (!st || (n && !pcs)) return SYZCOV_EINVAL;
    std::lock_guard<std::mutex> g(st->mu);
    hipSetDevice(st->dev);
    if (st->dirty) {
        set_error("set_universe after maxCover was filled");
        return SYZCOV_EINVAL;
    }
    if (st->pc_of_key) hipFree(st->pc_of_key);
    if (st->low_of_key) hipFree(st->low_of_key);
    if (st->nib) hipFree(st->nib);
    st->pc_of_key = nullptr;
    st->low_of_key = nullptr;
    st->nib = nullptr;
    st->X = Index{0, st->pc_lo, 0, 0, st->pc_span, nullptr};  // back to window mode
    if (n == 0) return alloc_maps(st);
    // the sorted unique universe on the device: window bits -> list
    uint32_t *bm = nullptr, *lst = nullptr, *sc = nullptr;
    void *ws = nullptr;
    const uint64_t wwords = (st->pc_span + 31) / 32;
    const size_t wsz = syzcov_dev_dict_ws_size(st->pc_span);
    uint64_t *tab = nullptr;
    int rc = 0;
    do {
        if (hipMalloc(&bm, wwords * 4) != hipSuccess || hipMalloc(&tab, wwords * 8) != hipSuccess ||
            hipMalloc(&ws, wsz + 256) != hipSuccess || hipMalloc(&lst, n * 4 + 4) != hipSuccess ||
            hipMalloc(&sc, 256) != hipSuccess) {
            rc = SYZCOV_ENOMEM;
            break;
        }
        if (hipMemsetAsync(bm, 0, wwords * 4, st->s) != hipSuccess) { rc = SYZCOV_EHIP; break; }
        if ((rc = set_bits(st, bm, pcs, n))) break;  // window mode: bits over offsets
        uint32_t *d_n = sc, *d_ks = sc + 1;
        if ((rc = syzcov_dev_dict_build_bits(bm, st->pc_span, tab, d_n, ws, st->s))) break;
        if ((rc = syzcov_dev_dict_to_list(tab, st->pc_span, st->pc_lo, lst, d_n, st->s))) break;
        uint32_t hn = 0;
        if (hipMemcpyAsync(&hn, d_n, 4, hipMemcpyDeviceToHost, st->s) != hipSuccess ||
            hipStreamSynchronize(st->s) != hipSuccess) { rc = SYZCOV_EHIP; break; }
        if (hn == 0) break;  // only sentinels: stay in window mode
        const uint32_t kmax = SYZCOV_KSHIFT_MAX;  // the shift is capped (keys.hip)
        if (hipMemcpyAsync(d_ks, &kmax, 4, hipMemcpyHostToDevice, st->s) != hipSuccess) {
            rc = SYZCOV_EHIP;
            break;
        }
        hipLaunchKernelGGL(universe_shift_kernel, dim3(grid_for(hn, 256, 1024)), dim3(256), 0,
                           st->s, (const uint32_t *)lst, hn, d_ks);
        uint32_t ks = 0, ends[2] = {0, 0};
        if (hipMemcpyAsync(&ks, d_ks, 4, hipMemcpyDeviceToHost, st->s) != hipSuccess ||
            hipMemcpyAsync(&ends[0], lst, 4, hipMemcpyDeviceToHost, st->s) != hipSuccess ||
            hipMemcpyAsync(&ends[1], lst + hn - 1, 4, hipMemcpyDeviceToHost, st->s) != hipSuccess ||
            hipStreamSynchronize(st->s) != hipSuccess) { rc = SYZCOV_EHIP; break; }
        const uint32_t kbase = ends[0] >> ks;
        const uint64_t nkeys = (uint64_t)(ends[1] >> ks) - kbase + 1;
        if (hipMalloc(&st->pc_of_key, nkeys * 4) != hipSuccess ||
            hipMalloc(&st->low_of_key, nkeys) != hipSuccess) {
            rc = SYZCOV_ENOMEM;
            break;
        }
        if (hipMemsetAsync(d_n, 0, 4, st->s) != hipSuccess) { rc = SYZCOV_EHIP; break; }
        // (the keymap zero-fills pc_of_key and 0x7F-fills low_of_key first)
        if ((rc = syzcov_dev_universe_keymap(lst, hn, ks, kbase, nkeys, st->pc_of_key,
                                             st->low_of_key, d_n, st->s)))
            break;
        uint32_t kerr = 0;
        if (hipMemcpyAsync(&kerr, d_n, 4, hipMemcpyDeviceToHost, st->s) != hipSuccess ||
            hipStreamSynchronize(st->s) != hipSuccess) { rc = SYZCOV_EHIP; break; }
        if (kerr) {  // cannot happen for a sorted unique list under its own shift
            set_error("universe keymap failed");
            rc = SYZCOV_EINVAL;
            break;
        }
        if (ks <= 4) {  // the separate membership pass's nibbles, whole ranges
            const uint64_t nwords = ((nkeys + (1ull << RSH) - 1) >> RSH) << (RSH - 3);
            if (hipMalloc(&st->nib, nwords * 4) != hipSuccess) {
                st->nib = nullptr;
                rc = SYZCOV_ENOMEM;
                break;
            }
            hipLaunchKernelGGL(nib_build_kernel, dim3(grid_for(nwords, 256, 8192)), dim3(256), 0,
                               st->s, (const uint8_t *)st->low_of_key, nkeys, nwords, st->nib);
        }
        st->X = Index{1, st->pc_lo, ks, kbase, nkeys, st->low_of_key};
        rc = alloc_maps(st);
    } while (0);
    if (bm) hipFree(bm);
    if (tab) hipFree(tab);
    if (ws) hipFree(ws);
    if (lst) hipFree(lst);
    if (sc) hipFree(sc);
    if (rc) {
        if (st->pc_of_key) hipFree(st->pc_of_key);
        if (st->low_of_key) hipFree(st->low_of_key);
        if (st->nib) hipFree(st->nib);
        st->pc_of_key = nullptr;
        st->low_of_key = nullptr;
        st->nib = nullptr;
        st->X = Index{0, st->pc_lo, 0, 0, st->pc_span, nullptr};
        alloc_maps(st);
    }
    return rc;
}

extern "C" int syzcov_state_set_flakes(syzcov_cover_state h, const uint32_t *pcs, size_t n) {
    CoverState *st = (CoverState *)(uintptr_t)h;
    if (!st || (n && !pcs)) return SYZCOV_EINVAL;
    std::lock_guard<std::mutex> g(st->mu);
    hipSetDevice(st->dev);
    SYZ_HIP(hipMemsetAsync(st->flakes, 0, st->words * 4, st->s));
    st->mfl_stale = true;
    return set_bits(st, st->flakes, pcs, n);
}

extern "C" int64_t syzcov_state_get(syzcov_cover_state h, int call, uint32_t *out, size_t cap) {
    CoverState *st = (CoverState *)(uintptr_t)h;
    if (!st || call < 0 || call >= st->ncalls) return SYZCOV_EINVAL;
    std::lock_guard<std::mutex> g(st->mu);
    hipSetDevice(st->dev);
    int64_t count = 0;
    int rc = state_bitmap_get(st, st->maxcov + (size_t)call * st->words, out, cap, &count);
    return rc ? rc : count;
}

// device workspace: clist uint2[npc] | perm u32[nrec] | nq u32[NR_MAX x (nrec + 1)] |
//   Bq u64[NR_MAX x (nrec + 1)] | Rq u32[NR_MAX x (nrec + 1)] | csum u32[chunks x NR_MAX] |
//   qoff u32[NR_MAX + 1] | rows uint4[npc / 64 + min(npc, nrec x NR_MAX)] | hkey u64[cap] |
//   hval u32[cap] | stats
struct NcLayout {
    size_t perm, nq, bq, rq, csum, qoff, rows, hkey, hval, stats, end;
};
static NcLayout nc_layout(size_t nrec, uint64_t npc) {
    uint64_t cap = 1024;
    while (cap < 2ull * npc) cap <<= 1;
    NcLayout L;
    L.perm = align_up(npc * 8 + 8, 256);
    L.nq = align_up(L.perm + nrec * 4 + 4, 256);
    L.bq = align_up(L.nq + (nrec + 1) * NR_MAX * 4, 256);
    L.rq = align_up(L.bq + (nrec + 1) * NR_MAX * 8, 256);
    L.csum = align_up(L.rq + (nrec + 1) * NR_MAX * 4, 256);
    L.qoff = align_up(L.csum + ((nrec + RS_CHUNK - 1) / RS_CHUNK) * NR_MAX * 4 + 4, 256);
    L.rows = align_up(L.qoff + (NR_MAX + 1) * 4, 256);
    const uint64_t nrows = npc / 256 + 2 * std::min<uint64_t>(npc, (uint64_t)nrec * NR_MAX) + 1;
    L.hkey = align_up(L.rows + nrows * 16, 256);
    L.hval = align_up(L.hkey + cap * 8, 256);
    L.stats = align_up(L.hval + cap * 4, 256);
    L.end = L.stats + 256;
    return L;
}

extern "C" size_t syzcov_state_newcov_ws_size(size_t nrec, uint64_t npc) {
    return nc_layout(nrec, npc).end;
}

// Candidate pass choice.  LDS staging (ranges of 2^19 indices, nr <= 32)
// pays when the bitmap bytes staged (about nr x calls x 64 KB) stay well
// under the PCs streamed; otherwise (sparse calls, huge windows) every PC
// probes the bitmap in global memory.  SYZCOV_FORCE=nc_lds|nc_probe forces one.
static int dev_cus() {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        n = 256;
    return n > 0 ? n : 256;
}
static int forced_path() {
    const uint32_t f = force_flags();
    return (f & FORCE_NC_LDS) ? 1 : (f & FORCE_NC_PROBE) ? 2 : 0;
}
// work items of the LDS pass per batch (64 rows at least per item)
// work items per batch: 512 / 1024 / 2048 / 4096 measured 0.642-0.646 /
// 0.671-0.675 / 0.644-0.649 / 0.70 ms per steady-state C5 batch
#ifndef SYZ_NC_ITEMS
#define SYZ_NC_ITEMS 512
#endif
constexpr uint32_t NC_ITEMS = SYZ_NC_ITEMS;

static int newcov_launch(CoverState *st, const int32_t *callid, const uint64_t *rec_off,
                         const uint32_t *pcs, size_t nrec, uint64_t npc, uint8_t *is_new,
                         uint8_t *ws, uint32_t **stats_out, uint32_t *stats_user, hipStream_t s) {
    const NcLayout Lw = nc_layout(nrec, npc);
    uint2 *clist = (uint2 *)ws;
    uint32_t *perm = (uint32_t *)(ws + Lw.perm);
    unsigned long long *hkey = (unsigned long long *)(ws + Lw.hkey);
    uint32_t *hval = (uint32_t *)(ws + Lw.hval);
    uint32_t *stats = (uint32_t *)(ws + Lw.stats);
    *stats_out = stats;
    const uint32_t nc = (uint32_t)st->ncalls;
    uint32_t *ccnt = st->grp, *coff = ccnt + nc + 1, *cur = coff + nc + 1, *ipre = cur + nc + 1;
    // the mfl mode words (nc_zero_kernel) sit past mfl's bitmaps
    // (this batch's fused and ownership passes get them only on the fused path)
    uint32_t *mfl_mode = nullptr;
    hipLaunchKernelGGL(nc_zero_kernel, dim3(grid_for(std::max<uint64_t>(nrec, nc), 256, 256)),
                       dim3(256), 0, s, stats, ccnt, nc, is_new, (uint32_t)nrec,
                       st->mfl ? st->mfl + (size_t)st->ncalls * st->words : nullptr,
                       (const uint4 *)st->maxcov, (const uint4 *)st->flakes, st->words / 4,
                       st->words / 4 * st->ncalls, (uint4 *)st->mfl);
    // records grouped by call (both passes)
    static std::atomic<uint32_t> gs_done{0};
    if (nc <= GRP_MAX_CALLS) {
        int rc = set_dyn_lds_once((const void *)grp_scatter_kernel, GRP_MAX_CALLS * 4, gs_done);
        if (rc) return rc;
    }
    hipLaunchKernelGGL(grp_hist_kernel, dim3(grid_for(nrec, 256, 1024)), dim3(256),
                       nc <= GRP_MAX_CALLS ? (size_t)nc * 4 : 0, s, callid, (uint32_t)nrec,
                       st->ncalls, ccnt, stats);
    hipLaunchKernelGGL(grp_scan_kernel, dim3(1), dim3(1024), 0, s, (const uint32_t *)ccnt,
                       st->ncalls, coff, cur);
    hipLaunchKernelGGL(grp_scatter_kernel,
                       dim3((unsigned)((nrec + GS_THREADS * GS_PER - 1) / (GS_THREADS * GS_PER))),
                       dim3(GS_THREADS), nc <= GRP_MAX_CALLS ? (size_t)nc * 4 : 0, s, callid,
                       (uint32_t)nrec, st->ncalls, cur, perm);
    // key mode with the universe's nibbles: the fused pass over 2^18-key ranges
    // (SYZCOV_FORCE=nc_sep: the candidate pass, then the separate membership pass)
    const uint32_t ff = force_flags();
    const bool fused = st->X.key_mode && st->nib && !(ff & FORCE_NC_SEP) &&
                       ((st->X.span + (1ull << RSF) - 1) >> RSF) <= NR_MAX;
    const uint32_t rsh = fused ? RSF : RSH;
    const uint64_t nr64 = (st->X.span + (1ull << rsh) - 1) >> rsh;
    const int forced = forced_path();
    const uint64_t range_bytes = std::min<uint64_t>(st->words * 4, 1u << (rsh - 3));
    const bool lds = nr64 <= NR_MAX && npc < (1ull << 30) &&  // buffer offsets: 4 GB of PCs
                     (forced == 1 ||
                      (forced == 0 && 2 * nr64 * (uint64_t)nc * range_bytes <= npc * 4));
    if (lds) {
        if (!st->mfl) {  // + the mfl mode words
            if (hipMalloc(&st->mfl, (size_t)st->ncalls * st->words * 4 + 256) != hipSuccess) {
                st->mfl = nullptr;
                return SYZCOV_ENOMEM;
            }
            st->mfl_stale = true;
        }
        // a non-fused batch reads mfl itself: rebuild it if a fused batch may
        // have left it stale
        if (!fused && st->mfl_dev_mode) st->mfl_stale = true;
        st->mfl_dev_mode = fused;
        if (st->mfl_stale) {
            const uint64_t vpc = st->words / 4, nv = vpc * st->ncalls;
            hipLaunchKernelGGL(mfl_build_kernel, dim3(grid_for(nv, 256, 16384)), dim3(256), 0, s,
                               (const uint4 *)st->maxcov, (const uint4 *)st->flakes, vpc, nv,
                               (uint4 *)st->mfl);
            SYZ_HIP(hipMemsetAsync(st->mfl + (size_t)st->ncalls * st->words, 0, 8, s));  // mode 0
            st->mfl_stale = false;
        }
        mfl_mode = fused ? st->mfl + (size_t)st->ncalls * st->words : nullptr;
        static std::atomic<uint32_t> lds_done[3], memb_done, fused_done;
        const bool sep = st->X.key_mode && st->nib && !fused;
        const int kv = !st->X.key_mode ? 0 : sep ? 2 : 1;
        auto kfn = kv == 0 ? newcov_cand_lds_kernel<false, false>
                   : kv == 1 ? newcov_cand_lds_kernel<true, false>
                             : newcov_cand_lds_kernel<true, true>;
        int rc = fused ? set_dyn_lds_once((const void *)newcov_fused_kernel, (int)FUSED_LDS, fused_done)
                       : set_dyn_lds_once((const void *)kfn, 1 << (RSH - 3), lds_done[kv]);
        if (rc) return rc;
        if (sep && (rc = set_dyn_lds_once((const void *)newcov_memb_kernel, 1 << (RSH - 2), memb_done)))
            return rc;
        const uint32_t nr = (uint32_t)nr64, stride = (uint32_t)nrec + 1;
        uint4 *desc = (uint4 *)((uint8_t *)st->grp + grp_desc_off(st->ncalls));
        uint32_t *nq = (uint32_t *)(ws + Lw.nq), *csum = (uint32_t *)(ws + Lw.csum);
        uint32_t *rq = (uint32_t *)(ws + Lw.rq), *qoff = (uint32_t *)(ws + Lw.qoff);
        uint64_t *bq = (uint64_t *)(ws + Lw.bq);
        uint4 *rows = (uint4 *)(ws + Lw.rows);
        // chunk: about NC_ITEMS work items over the batch, >= 64 rows, and
        // rows <= nrows / CHR <= ITEMS_MAX, so the descriptors fit ITEMS_MAX +
        // the pairs
        const uint64_t nrows = npc / 256 + 2 * std::min<uint64_t>(npc, (uint64_t)nrec * nr) + 1;
        const uint64_t est = npc / 256 + (uint64_t)nrec * nr / 2;  // ~half a row of slack per sub-run
        const uint32_t CHR = (uint32_t)std::max<uint64_t>(
            std::max<uint64_t>(64, (est + NC_ITEMS - 1) / NC_ITEMS),
            (nrows + ITEMS_MAX - 1) / ITEMS_MAX);
        // sub-runs of the grouped records (records with a bad call id are not
        // grouped: coff[nc] <= nrec)
        hipLaunchKernelGGL(newcov_split_kernel, dim3(grid_for(nrec, 4, 16384)), dim3(256), 0, s,
                           rec_off, pcs, (const uint32_t *)perm, (const uint32_t *)coff, st->ncalls,
                           st->X, nr, rsh, stride, nq, bq, stats);
        const uint32_t nb = (uint32_t)((nrec + RS_CHUNK - 1) / RS_CHUNK);
        hipLaunchKernelGGL(range_sum_kernel, dim3(nb, nr), dim3(1024), 0, s, (const uint32_t *)nq,
                           (const uint64_t *)bq, (uint32_t)nrec, stride, csum);
        hipLaunchKernelGGL(range_scan_kernel, dim3(nb, nr), dim3(1024), 0, s, (const uint32_t *)nq,
                           (const uint64_t *)bq, (uint32_t)nrec, stride, (const uint32_t *)csum, rq);
        if (!fused)
            hipLaunchKernelGGL(item_scan_kernel, dim3(1), dim3(1024), 0, s, (const uint32_t *)coff,
                               st->ncalls, nr, (const uint32_t *)rq, stride, CHR, ipre);
        // the segment table lives in the item descriptors' space (unused here)
        uint32_t *segb = (uint32_t *)desc, *wg_seg = segb + nr * (nc + 1);
        const uint32_t fused_g = (uint32_t)std::min<int>(dev_cus(), (int)FG_MAX);
        if (fused)  // qoff and the fused pass's segment table
            hipLaunchKernelGGL(fused_seg_kernel, dim3(1), dim3(1024), 0, s, (const uint32_t *)coff,
                               st->ncalls, nr, (const uint32_t *)rq, (uint32_t)nrec, stride, qoff,
                               fused_g, segb, wg_seg);
        else
            hipLaunchKernelGGL(row_offsets_kernel, dim3(1), dim3(64), 0, s, (const uint32_t *)rq,
                               (uint32_t)nrec, stride, nr, qoff);
        const uint32_t ne = nc * nr;
        if (!fused)
            hipLaunchKernelGGL(desc_kernel, dim3(grid_for(ne, 256, 4096)), dim3(256), 0, s,
                               (const uint32_t *)coff, st->ncalls, nr, (const uint32_t *)rq, stride,
                               CHR, (const uint32_t *)ipre, desc);
        hipLaunchKernelGGL(row_fill_kernel, dim3(grid_for((uint64_t)nrec * nr, 256, 16384)),
                           dim3(256), 0, s, (const uint32_t *)nq, (const uint64_t *)bq,
                           (const uint32_t *)rq, (const uint32_t *)perm, (const uint32_t *)coff,
                           st->ncalls, nr, stride, (const uint32_t *)qoff, rows);
        // items <= rows / CHR + non-empty (call, range) pairs; the excess exits
        const uint64_t items = nrows / CHR + std::min<uint64_t>((uint64_t)nc, nrec) * nr + 1;
        if (fused) {
            const uint64_t nib_words = ((st->X.span + (1ull << RSH) - 1) >> RSH) << (RSH - 3);
            hipLaunchKernelGGL(newcov_fused_kernel, dim3(fused_g), dim3(LC_THREADS), FUSED_LDS, s,
                               pcs, (uint32_t)npc, (const uint32_t *)st->mfl,
                               (const uint32_t *)st->maxcov, (const uint32_t *)st->flakes,
                               (const uint32_t *)mfl_mode, st->words,
                               (const uint32_t *)st->nib, nib_words, st->X, nr, st->ncalls,
                               (const uint32_t *)segb, (const uint32_t *)wg_seg,
                               (const uint4 *)rows, (const uint32_t *)qoff, clist, stats);
        } else {
            hipLaunchKernelGGL(kfn, dim3((unsigned)items), dim3(LC_THREADS), (size_t)(1u << (RSH - 3)), s, pcs,
                               (uint32_t)npc, (const uint32_t *)st->mfl, st->words,
                               st->X, nr, (const uint32_t *)ipre, ne, (const uint4 *)desc,
                               (const uint4 *)rows, (const uint32_t *)qoff, clist, stats);
        }
        if (sep)
            hipLaunchKernelGGL(newcov_memb_kernel, dim3(MB_G * 2), dim3(MB_THREADS),
                               (size_t)(1u << (RSH - 2)), s, pcs, (uint32_t)npc,
                               (const uint32_t *)st->nib, st->X, nr, (const uint4 *)rows,
                               (const uint32_t *)qoff, stats);
    } else {
        const unsigned gx = (grid_for(nrec, NC_WPB, 4096) + 7) & ~7u;  // a multiple of the 8 XCDs
        hipLaunchKernelGGL(newcov_cand_kernel, dim3(gx), dim3(NC_THREADS), 0, s, callid, rec_off,
                           pcs, (uint32_t)nrec, st->maxcov, st->words, st->flakes, st->X,
                           (const uint32_t *)perm, (const uint32_t *)coff, st->ncalls, clist, stats);
    }
    const unsigned gh = grid_for(std::max<uint64_t>(npc, 512), 256, 8192);
    if ((uint64_t)st->ncalls * st->X.span <= 0xFFFFFFFFull && !(ff & FORCE_NC_HASH64)) {
        hipLaunchKernelGGL(hash_clear32_kernel, dim3(gh), dim3(256), 0, s, (const uint32_t *)stats,
                           hkey);
        hipLaunchKernelGGL(newcov_insert32_kernel, dim3(gh), dim3(256), 0, s, callid,
                           (const uint2 *)clist, (const uint32_t *)stats, hkey, st->X);
        hipLaunchKernelGGL(newcov_own32_kernel, dim3(gh), dim3(256), 0, s, callid,
                           (const uint2 *)clist, (const uint32_t *)stats,
                           (const unsigned long long *)hkey, is_new, st->maxcov, st->mfl,
                           st->words, st->X, stats_user, mfl_mode);
    } else {
        hipLaunchKernelGGL(hash_clear_kernel, dim3(gh), dim3(256), 0, s, (const uint32_t *)stats,
                           hkey, hval);
        hipLaunchKernelGGL(newcov_insert_kernel, dim3(gh), dim3(256), 0, s, callid,
                           (const uint2 *)clist, (const uint32_t *)stats, hkey, hval);
        hipLaunchKernelGGL(newcov_own_kernel, dim3(gh), dim3(256), 0, s, callid,
                           (const uint2 *)clist, (const uint32_t *)stats,
                           (const unsigned long long *)hkey, (const uint32_t *)hval, is_new,
                           st->maxcov, st->mfl, st->words, st->X, stats_user);
    }
    SYZ_LAUNCH_CHECK();
    return 0;
}

// Device-resident batch (all pointers device memory; rec_off[0] == 0,
// rec_off[nrec] == npc).
// stats (device u32[2], nullable): [0] error code (1 PC outside the window,
// 2 call id out of range, 3 unsorted record), [1] candidates after the
// bitmap filter.  Errors are reported there, not returned: the launch is
// asynchronous on `stream`.
extern "C" int syzcov_state_newcov_dev(syzcov_cover_state h, const int32_t *callid,
                                       const uint64_t *rec_off, const uint32_t *pcs, size_t nrec,
                                       uint64_t npc, uint8_t *is_new, uint32_t *stats, void *ws,
                                       size_t ws_size, void *stream) {
    CoverState *st = (CoverState *)(uintptr_t)h;
    if (!st || !callid || !rec_off || !is_new || !ws || nrec > 0x7FFFFFFF || npc > 0xFFFFFFFFull)
        return SYZCOV_EINVAL;
    if (ws_size < syzcov_state_newcov_ws_size(nrec, npc)) return SYZCOV_EINVAL;
    if (nrec == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    // the handle's lock (the reference's coverMu) for the launch: the batch
    // uses the handle's grouping scratch and maxCover.  The caller's stream
    // waits for the handle's earlier work, and the handle's stream (the host
    // tier: state_add, triage, ...) for this batch.
    std::lock_guard<std::mutex> g(st->mu);
    hipSetDevice(st->dev);
    if (!st->ev_state) {
        SYZ_HIP(hipEventCreateWithFlags(&st->ev_state, hipEventDisableTiming));
        SYZ_HIP(hipEventCreateWithFlags(&st->ev_dev, hipEventDisableTiming));
    }
    if (s != st->s) {
        SYZ_HIP(hipEventRecord(st->ev_state, st->s));
        SYZ_HIP(hipStreamWaitEvent(s, st->ev_state, 0));
    }
    st->dirty = true;
    uint32_t *dstats = nullptr;
    const int rc = newcov_launch(st, callid, rec_off, pcs, nrec, npc, is_new, (uint8_t *)ws,
                                 &dstats, stats, s);
    if (s != st->s) {
        SYZ_HIP(hipEventRecord(st->ev_dev, s));
        SYZ_HIP(hipStreamWaitEvent(st->s, st->ev_dev, 0));
    }
    return rc;
}

// The host-buffer batch of execute() (add_input false) or addInput
// (add_input true: accepted inputs then OR their whole cover into maxCover
// and corpusCover).
static int64_t newcov_host(CoverState *st, const int32_t *callid, const uint64_t *rec_off,
                           const uint32_t *rec_pcs, size_t nrec, uint8_t *is_new, bool add_input) {
    if (!st || (nrec && (!callid || !rec_off || !is_new))) return SYZCOV_EINVAL;
    if (nrec == 0) return 0;
    if (nrec > 0x7FFFFFFF) return SYZCOV_EINVAL;
    std::lock_guard<std::mutex> g(st->mu);
    hipSetDevice(st->dev);
    const uint64_t base0 = rec_off[0];
    const uint64_t npc = rec_off[nrec] - base0;
    if (npc && !rec_pcs) return SYZCOV_EINVAL;
    if (npc > 0xFFFFFFFFull) return SYZCOV_EINVAL;
    int rc = add_input ? state_ensure_corpus(st) : 0;
    if (rc) return rc;
    // staging: callid | off | pcs | is_new | newcov workspace
    const size_t o_off = align_up(nrec * 4, 256), o_pcs = align_up(o_off + (nrec + 1) * 8, 256),
                 o_new = align_up(o_pcs + npc * 4 + 4, 256), o_ws = align_up(o_new + nrec, 256),
                 o_end = o_ws + syzcov_state_newcov_ws_size(nrec, npc);
    rc = grow(st, o_end);
    if (rc) return rc;
    uint8_t *S = (uint8_t *)st->scratch;
    hipStream_t s = st->s;
    st->dirty = true;
    std::vector<uint64_t> hoff(nrec + 1);  // offsets rebased to 0
    for (size_t k = 0; k <= nrec; k++) hoff[k] = rec_off[k] - base0;
    SYZ_HIP(hipMemcpyAsync(S, callid, nrec * 4, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(S + o_off, hoff.data(), (nrec + 1) * 8, hipMemcpyHostToDevice, s));
    if (npc) SYZ_HIP(hipMemcpyAsync(S + o_pcs, rec_pcs + base0, npc * 4, hipMemcpyHostToDevice, s));
    uint32_t *dstats = nullptr;
    rc = newcov_launch(st, (const int32_t *)S, (const uint64_t *)(S + o_off),
                       (const uint32_t *)(S + o_pcs), nrec, npc, S + o_new, S + o_ws, &dstats, nullptr,
                       s);
    if (rc) return rc;
    if (add_input) {
        hipLaunchKernelGGL(accept_or_kernel, dim3(grid_for(nrec, 4, 8192)), dim3(256), 0, s,
                           (const int32_t *)S, (const uint64_t *)(S + o_off),
                           (const uint32_t *)(S + o_pcs), (uint32_t)nrec,
                           (const uint8_t *)(S + o_new), (const uint32_t *)dstats, st->maxcov,
                           st->corpus, st->words, st->X);
        SYZ_LAUNCH_CHECK();
        st->mfl_stale = true;
    }
    uint32_t hs[2];
    SYZ_HIP(hipMemcpyAsync(hs, dstats, 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipMemcpyAsync(is_new, S + o_new, nrec, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    if (hs[0]) {
        set_error(hs[0] == 1 ? "PC outside the state's PC window"
                  : hs[0] == 2 ? "call id out of range"
                               : "record cover not sorted");
        return hs[0] == 1 ? SYZCOV_ERANGE : hs[0] == 2 ? SYZCOV_EINVAL : SYZCOV_ENOTSORTED;
    }
    int64_t nnew = 0;
    for (size_t k = 0; k < nrec; k++) nnew += is_new[k];
    return nnew;
}

extern "C" int64_t syzcov_newcov_batch(syzcov_cover_state h, const int32_t *callid,
                                       const uint64_t *rec_off, const uint32_t *rec_pcs,
                                       size_t nrec, uint8_t *is_new) {
    return newcov_host((CoverState *)(uintptr_t)h, callid, rec_off, rec_pcs, nrec, is_new, false);
}

extern "C" int64_t syzcov_state_add_inputs(syzcov_cover_state h, const int32_t *callid,
                                           const uint64_t *rec_off, const uint32_t *rec_pcs,
                                           size_t nrec, uint8_t *accepted) {
    return newcov_host((CoverState *)(uintptr_t)h, callid, rec_off, rec_pcs, nrec, accepted, true);
}
