// triage.hip — triageInput's coverage steps (syz-fuzzer/fuzzer.go:377-417)
// for a batch of inputs against the resident corpusCover / flakes bitmaps,
// plus the corpusCover accessors.
//
// Per input t (call c, sorted cover A, three re-execution covers R_i):
//   newCover  = Difference(Difference(A, corpusCover[c]), flakes)     :384-385
//   if newCover == ∅: stop                                            :387-389
//   minCover  = A;  for each executed run R_i (len > 0, :401-404):
//       minCover = Intersection(minCover, R_i)                        :408
//       flakes   = Union(flakes, SymmetricDifference(A, R_i))         :407-415
//   stableNewCover = Intersection(newCover, minCover)                 :417
// The updateFlakes predicate (:409) only skips a Union that would change
// nothing, so flakes grows by every executed run's symmetric difference.
// Over canonical lists (sorted; 0xFFFFFFFF only as a trailing sentinel)
// every one of these set ops drops the sentinel (cover.go:81-102).
//
// Batch schedule: every input's newCover is read before any flakes update
// (kernel 1, then kernel 2) — one interleaving the reference's concurrent
// triage goroutines can produce (they take coverMu.RLock for :383-386 and
// coverMu.Lock per update, :412-414).  Inside kernel 2 the updates are
// atomic ORs: the union is order-independent, and no step of kernel 2 reads
// flakes.
//
// Kernel 1: one wave per input: validates the cover and its runs (sorted,
// inside the index space), marks newCover positions (bit 0) and sets the
// "in every run" bit (bit 1) for kernel 2 to clear.
// Kernel 2: one workgroup per input with a non-empty newCover: the cover
// and each run are staged in LDS (when <= TR_CAP PCs) and each side is
// binary-searched in the other: PCs of one side missing from the other are
// the symmetric difference (OR-ed into flakes); cover PCs missing from a run
// leave minCover.  The stable PCs are then compacted in order.
#include "cover_state.h"

namespace syz {

constexpr int TR_THREADS = 256;
constexpr uint32_t TR_CAP = 8192;  // PCs per side staged in LDS (2 x 32 KB)
constexpr uint32_t SENT = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t strip_sent(const uint32_t *p, uint32_t n) {
    while (n && p[n - 1] == SENT) n--;
    return n;
}

__device__ __forceinline__ bool contains(const uint32_t *a, uint32_t n, uint32_t v) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo < n && a[lo] == v;
}

// A sorted list (trailing sentinels excluded) inside the index space?  0 ok,
// 1 outside, 3 unsorted.  One wave.
__device__ uint32_t check_list(const uint32_t *p, uint32_t n, const Index &X) {
    const uint32_t l = __lane_id();
    uint32_t bad = 0;
    for (uint32_t i = l; i < n; i += 64) {
        uint32_t ix;
        if (!pc_index(X, p[i], &ix)) bad |= 1u;
        if (i > 0 && p[i - 1] > p[i]) bad |= 2u;
    }
    const uint64_t b1 = __ballot(bad & 1u), b2 = __ballot(bad & 2u);
    return b1 ? 1u : b2 ? 3u : 0u;
}

__global__ __launch_bounds__(256) void triage_new_kernel(
    const int32_t *__restrict__ callid, uint32_t ntri, int ncalls,
    const uint64_t *__restrict__ cov_off, const uint32_t *__restrict__ cov_pcs,
    const uint64_t *__restrict__ run_off, const uint32_t *__restrict__ run_pcs,
    const uint32_t *__restrict__ corpus, const uint32_t *__restrict__ flakes, uint64_t words,
    Index X, uint8_t *__restrict__ mark, uint32_t *__restrict__ new_cnt,
    uint32_t *__restrict__ err) {
    const uint32_t l = __lane_id();
    for (uint32_t t = blockIdx.x * 4 + (threadIdx.x >> 6); t < ntri; t += gridDim.x * 4) {
        const int c = callid[t];
        if (c < 0 || c >= ncalls) {
            if (l == 0) {
                *err = 2u;
                new_cnt[t] = 0;
            }
            continue;
        }
        const uint64_t a0 = cov_off[t];
        const uint32_t *A = cov_pcs + a0;
        const uint32_t nraw = (uint32_t)(cov_off[t + 1] - a0), nA = strip_sent(A, nraw);
        uint32_t e = check_list(A, nA, X);
        for (int i = 0; i < 3; i++) {
            const uint64_t r0 = run_off[3 * t + i];
            const uint32_t *R = run_pcs + r0;
            const uint32_t e2 = check_list(R, strip_sent(R, (uint32_t)(run_off[3 * t + i + 1] - r0)), X);
            e = e ? e : e2;
        }
        if (e) {
            if (l == 0) {
                *err = e;
                new_cnt[t] = 0;
            }
            continue;
        }
        const uint32_t *CC = corpus + (uint64_t)c * words;
        uint32_t cnt = 0;
        for (uint32_t i = l; i - l < nraw; i += 64) {
            bool nw = false;
            if (i < nA) {
                uint32_t ix;
                pc_index(X, A[i], &ix);
                nw = !bit_test(CC, ix) && !bit_test(flakes, ix);
            }
            if (i < nraw) mark[a0 + i] = (uint8_t)((nw ? 1u : 0u) | (i < nA ? 2u : 0u));
            cnt += (uint32_t)__popcll(__ballot(nw));
        }
        if (l == 0) new_cnt[t] = cnt;
    }
}

__global__ __launch_bounds__(TR_THREADS) void triage_runs_kernel(
    uint32_t ntri, const uint64_t *__restrict__ cov_off, const uint32_t *__restrict__ cov_pcs,
    const uint64_t *__restrict__ run_off, const uint32_t *__restrict__ run_pcs,
    uint32_t *__restrict__ flakes, Index X, uint8_t *__restrict__ mark,
    const uint32_t *__restrict__ new_cnt, uint32_t *__restrict__ stable_cnt,
    uint32_t *__restrict__ stable_pcs, const uint32_t *__restrict__ err) {
    __shared__ uint32_t sA[TR_CAP], sR[TR_CAP];
    __shared__ uint32_t tmp[TR_THREADS / 64 + 1];
    const uint32_t t = blockIdx.x, tid = threadIdx.x;
    if (t >= ntri) return;
    if (*err || new_cnt[t] == 0) {  // rejected batch / nothing new: no re-executions
        if (tid == 0) stable_cnt[t] = 0;
        return;
    }
    const uint64_t a0 = cov_off[t];
    const uint32_t nraw = (uint32_t)(cov_off[t + 1] - a0);
    const uint32_t nA = strip_sent(cov_pcs + a0, nraw);
    const uint32_t *A = cov_pcs + a0;
    if (nA <= TR_CAP) {
        for (uint32_t i = tid; i < nA; i += TR_THREADS) sA[i] = A[i];
        A = sA;
    }
    for (int r = 0; r < 3; r++) {
        const uint64_t r0 = run_off[3 * t + r], r1 = run_off[3 * t + r + 1];
        if (r1 == r0) continue;  // the call was not executed (:401-404)
        const uint32_t nR = strip_sent(run_pcs + r0, (uint32_t)(r1 - r0));
        const uint32_t *R = run_pcs + r0;
        __syncthreads();  // previous run's readers of sR are done
        if (nR <= TR_CAP) {
            for (uint32_t i = tid; i < nR; i += TR_THREADS) sR[i] = R[i];
            R = sR;
        }
        __syncthreads();
        for (uint32_t i = tid; i < nA; i += TR_THREADS) {
            const uint32_t p = A[i];
            if (!contains(R, nR, p)) {  // p in A \ R: leaves minCover, joins flakes
                mark[a0 + i] &= (uint8_t)~2u;
                uint32_t ix;
                pc_index(X, p, &ix);
                atomicOr(&flakes[ix >> 5], 1u << (ix & 31));
            }
        }
        for (uint32_t i = tid; i < nR; i += TR_THREADS) {
            const uint32_t q = R[i];
            if (!contains(A, nA, q)) {  // q in R \ A: joins flakes
                uint32_t ix;
                pc_index(X, q, &ix);
                atomicOr(&flakes[ix >> 5], 1u << (ix & 31));
            }
        }
    }
    __syncthreads();
    // stableNewCover = newCover ∩ minCover, in cover order
    uint32_t base = 0;
    for (uint32_t i0 = 0; i0 < nA; i0 += TR_THREADS) {
        const uint32_t i = i0 + tid;
        const bool keep = i < nA && (mark[a0 + i] & 3u) == 3u;
        uint32_t tot;
        const uint32_t rank = block_excl_scan<TR_THREADS>(keep ? 1u : 0u, tmp, &tot);
        if (keep) stable_pcs[a0 + base + rank] = A[i];
        base += tot;
        __syncthreads();
    }
    if (tid == 0) stable_cnt[t] = base;
}

}  // namespace syz

// ------------------------------------------------ host-side orchestration
#include <vector>

using namespace syz;

extern "C" int syzcov_state_corpus_add(syzcov_cover_state h, int call, const uint32_t *pcs,
                                       size_t n) {
    CoverState *st = (CoverState *)(uintptr_t)h;
    if (!st || call < 0 || call >= st->ncalls || (n && !pcs)) return SYZCOV_EINVAL;
    std::lock_guard<std::mutex> g(st->mu);
    hipSetDevice(st->dev);
    int rc = state_ensure_corpus(st);
    if (rc) return rc;
    st->dirty = true;
    return state_set_bits(st, st->corpus + (size_t)call * st->words, pcs, n);
}

extern "C" int64_t syzcov_state_corpus_get(syzcov_cover_state h, int call, uint32_t *out,
                                           size_t cap) {
    CoverState *st = (CoverState *)(uintptr_t)h;
    if (!st || call < 0 || call >= st->ncalls) return SYZCOV_EINVAL;
    std::lock_guard<std::mutex> g(st->mu);
    hipSetDevice(st->dev);
    int rc = state_ensure_corpus(st);
    if (rc) return rc;
    int64_t count = 0;
    rc = state_bitmap_get(st, st->corpus + (size_t)call * st->words, out, cap, &count);
    return rc ? rc : count;
}

extern "C" int64_t syzcov_state_flakes_get(syzcov_cover_state h, uint32_t *out, size_t cap) {
    CoverState *st = (CoverState *)(uintptr_t)h;
    if (!st) return SYZCOV_EINVAL;
    std::lock_guard<std::mutex> g(st->mu);
    hipSetDevice(st->dev);
    int64_t count = 0;
    const int rc = state_bitmap_get(st, st->flakes, out, cap, &count);
    return rc ? rc : count;
}

extern "C" int64_t syzcov_state_triage(syzcov_cover_state h, size_t ntri, const int32_t *callid,
                                       const uint64_t *cov_off, const uint32_t *cov_pcs,
                                       const uint64_t *run_off, const uint32_t *run_pcs,
                                       uint32_t *new_cnt, uint32_t *stable_cnt,
                                       uint32_t *stable_pcs) {
    CoverState *st = (CoverState *)(uintptr_t)h;
    if (!st || (ntri && (!callid || !cov_off || !run_off || !new_cnt || !stable_cnt)))
        return SYZCOV_EINVAL;
    if (ntri == 0) return 0;
    if (ntri > 0x7FFFFFFF) return SYZCOV_EINVAL;
    const uint64_t c0 = cov_off[0], nc = cov_off[ntri] - c0;
    const uint64_t r0 = run_off[0], nr = run_off[3 * ntri] - r0;
    if ((nc && (!cov_pcs || !stable_pcs)) || (nr && !run_pcs)) return SYZCOV_EINVAL;
    if (nc > 0xFFFFFFFFull || nr > 0xFFFFFFFFull) return SYZCOV_EINVAL;
    for (size_t t = 0; t < ntri; t++)
        if (cov_off[t + 1] < cov_off[t] || cov_off[t + 1] - cov_off[t] > 0xFFFFFFFFull)
            return SYZCOV_EINVAL;
    for (size_t k = 0; k < 3 * ntri; k++)
        if (run_off[k + 1] < run_off[k] || run_off[k + 1] - run_off[k] > 0xFFFFFFFFull)
            return SYZCOV_EINVAL;
    std::lock_guard<std::mutex> g(st->mu);
    hipSetDevice(st->dev);
    int rc = state_ensure_corpus(st);
    if (rc) return rc;
    // staging: callid | cov_off | run_off | cov_pcs | run_pcs | mark | new_cnt |
    //          stable_cnt | stable_pcs | err
    auto A = [](size_t x) { return align_up(x, 256); };
    const size_t o_coff = A(ntri * 4), o_roff = o_coff + A((ntri + 1) * 8),
                 o_cpcs = o_roff + A((3 * ntri + 1) * 8), o_rpcs = o_cpcs + A(nc * 4 + 4),
                 o_mark = o_rpcs + A(nr * 4 + 4), o_new = o_mark + A(nc + 1),
                 o_scnt = o_new + A(ntri * 4), o_spcs = o_scnt + A(ntri * 4),
                 o_err = o_spcs + A(nc * 4 + 4), o_end = o_err + 256;
    if ((rc = state_grow(st, o_end))) return rc;
    uint8_t *S = (uint8_t *)st->scratch;
    hipStream_t s = st->s;
    std::vector<uint64_t> hco(ntri + 1), hro(3 * ntri + 1);
    for (size_t t = 0; t <= ntri; t++) hco[t] = cov_off[t] - c0;
    for (size_t k = 0; k <= 3 * ntri; k++) hro[k] = run_off[k] - r0;
    SYZ_HIP(hipMemcpyAsync(S, callid, ntri * 4, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(S + o_coff, hco.data(), (ntri + 1) * 8, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(S + o_roff, hro.data(), (3 * ntri + 1) * 8, hipMemcpyHostToDevice, s));
    if (nc) SYZ_HIP(hipMemcpyAsync(S + o_cpcs, cov_pcs + c0, nc * 4, hipMemcpyHostToDevice, s));
    if (nr) SYZ_HIP(hipMemcpyAsync(S + o_rpcs, run_pcs + r0, nr * 4, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemsetAsync(S + o_err, 0, 4, s));
    st->dirty = true;
    const int32_t *d_cid = (const int32_t *)S;
    const uint64_t *d_coff = (const uint64_t *)(S + o_coff), *d_roff = (const uint64_t *)(S + o_roff);
    const uint32_t *d_cpcs = (const uint32_t *)(S + o_cpcs), *d_rpcs = (const uint32_t *)(S + o_rpcs);
    uint8_t *d_mark = S + o_mark;
    uint32_t *d_new = (uint32_t *)(S + o_new), *d_scnt = (uint32_t *)(S + o_scnt),
             *d_spcs = (uint32_t *)(S + o_spcs), *d_err = (uint32_t *)(S + o_err);
    hipLaunchKernelGGL(triage_new_kernel, dim3(grid_for(ntri, 4, 8192)), dim3(256), 0, s, d_cid,
                       (uint32_t)ntri, st->ncalls, d_coff, d_cpcs, d_roff, d_rpcs,
                       (const uint32_t *)st->corpus, (const uint32_t *)st->flakes, st->words, st->X,
                       d_mark, d_new, d_err);
    hipLaunchKernelGGL(triage_runs_kernel, dim3((unsigned)ntri), dim3(TR_THREADS), 0, s,
                       (uint32_t)ntri, d_coff, d_cpcs, d_roff, d_rpcs, st->flakes, st->X, d_mark,
                       (const uint32_t *)d_new, d_scnt, d_spcs, (const uint32_t *)d_err);
    SYZ_LAUNCH_CHECK();
    st->mfl_stale = true;  // flakes may have grown
    uint32_t herr = 0;
    SYZ_HIP(hipMemcpyAsync(&herr, d_err, 4, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipMemcpyAsync(new_cnt, d_new, ntri * 4, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipMemcpyAsync(stable_cnt, d_scnt, ntri * 4, hipMemcpyDeviceToHost, s));
    if (nc) SYZ_HIP(hipMemcpyAsync(stable_pcs + c0, d_spcs, nc * 4, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    if (herr) {  // kernel 2 did nothing: flakes unchanged
        set_error(herr == 1 ? "PC outside the state's index space"
                  : herr == 2 ? "call id out of range"
                              : "cover not sorted");
        return herr == 1 ? SYZCOV_ERANGE : herr == 2 ? SYZCOV_EINVAL : SYZCOV_ENOTSORTED;
    }
    int64_t n = 0;
    for (size_t t = 0; t < ntri; t++) n += stable_cnt[t] != 0;
    return n;
}
