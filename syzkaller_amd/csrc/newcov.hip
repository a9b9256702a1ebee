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
// tests every PC against the cache-resident bitmaps and compacts the
// survivors (few once maxCover saturates); a hash table keyed by
// (CallID, pc) takes an atomicMin of the record index; pass 2 marks a record
// new iff it owns one of its keys; the survivors are OR-ed into maxCover.
#include "common.h"

namespace syz {

__device__ __forceinline__ bool bit_test(const uint32_t *__restrict__ bm, uint64_t o) {
    return (bm[o >> 5] >> (o & 31)) & 1u;
}

constexpr int NC_THREADS = 256;

// per record: count candidates
__global__ __launch_bounds__(NC_THREADS) void newcov_count_kernel(
    const int32_t *__restrict__ callid, const uint64_t *__restrict__ rec_off,
    const uint32_t *__restrict__ pcs, uint32_t nrec, const uint32_t *__restrict__ maxcov,
    uint64_t words_per_call, const uint32_t *__restrict__ flakes, uint32_t pc_lo,
    uint64_t pc_span, int ncalls, uint32_t *__restrict__ rec_cnt, uint32_t *__restrict__ err) {
    __shared__ uint32_t tmp[NC_THREADS / 64 + 1];
    for (uint32_t k = blockIdx.x; k < nrec; k += gridDim.x) {
        const int c = callid[k];
        const uint64_t b = rec_off[k], n = rec_off[k + 1] - b;
        uint32_t cnt = 0;
        if (c < 0 || c >= ncalls) {
            if (threadIdx.x == 0) *err = 2u;
        } else {
            const uint32_t *M = maxcov + (uint64_t)c * words_per_call;
            for (uint64_t q = threadIdx.x; q < n; q += NC_THREADS) {
                const uint32_t pc = pcs[b + q];
                const uint64_t o = (uint64_t)(uint32_t)(pc - pc_lo);
                if (pc < pc_lo || o >= pc_span) {
                    *err = 1u;
                    continue;
                }
                if (q > 0 && pcs[b + q - 1] > pc) *err = 3u;  // not sorted
                cnt += !bit_test(flakes, o) && !bit_test(M, o);
            }
        }
        uint32_t total;
        block_excl_scan<NC_THREADS>(cnt, tmp, &total);
        if (threadIdx.x == 0) rec_cnt[k] = total;
    }
}

// exclusive scan of rec_cnt in one workgroup; total -> *tot
__global__ __launch_bounds__(1024) void newcov_scan_kernel(uint32_t *__restrict__ a, uint32_t n,
                                                            uint32_t *__restrict__ tot) {
    __shared__ uint32_t tmp[1024 / 64 + 1];
    uint32_t carry = 0;
    for (uint32_t c = 0; c < n; c += 1024) {
        const uint32_t i = c + threadIdx.x;
        const uint32_t v = i < n ? a[i] : 0u;
        uint32_t total;
        const uint32_t p = block_excl_scan<1024>(v, tmp, &total);
        if (i < n) a[i] = carry + p;
        carry += total;
    }
    if (threadIdx.x == 0) *tot = carry;
}

// per record: write candidate (key, record) pairs at rec_base[k] + rank
__global__ __launch_bounds__(NC_THREADS) void newcov_compact_kernel(
    const int32_t *__restrict__ callid, const uint64_t *__restrict__ rec_off,
    const uint32_t *__restrict__ pcs, uint32_t nrec, const uint32_t *__restrict__ maxcov,
    uint64_t words_per_call, const uint32_t *__restrict__ flakes, uint32_t pc_lo,
    uint64_t pc_span, int ncalls, const uint32_t *__restrict__ rec_base,
    uint64_t *__restrict__ ckey, uint32_t *__restrict__ crec) {
    __shared__ uint32_t tmp[NC_THREADS / 64 + 1];
    for (uint32_t k = blockIdx.x; k < nrec; k += gridDim.x) {
        const int c = callid[k];
        if (c < 0 || c >= ncalls) continue;  // block-uniform
        const uint32_t *M = maxcov + (uint64_t)c * words_per_call;
        const uint64_t b = rec_off[k], n = rec_off[k + 1] - b;
        uint32_t wpos = rec_base[k];
        for (uint64_t q0 = 0; q0 < n; q0 += NC_THREADS) {
            const uint64_t q = q0 + threadIdx.x;
            bool cand = false;
            uint32_t pc = 0;
            if (q < n) {
                pc = pcs[b + q];
                const uint64_t o = (uint64_t)(uint32_t)(pc - pc_lo);
                cand = pc >= pc_lo && o < pc_span && !bit_test(flakes, o) && !bit_test(M, o);
            }
            uint32_t total;
            const uint32_t p = block_excl_scan<NC_THREADS>(cand ? 1u : 0u, tmp, &total);
            if (cand) {
                ckey[wpos + p] = ((uint64_t)(uint32_t)c << 32) | pc;
                crec[wpos + p] = k;
            }
            wpos += total;
        }
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

__global__ void newcov_insert_kernel(const uint64_t *__restrict__ ckey,
                                     const uint32_t *__restrict__ crec, uint32_t ncand,
                                     unsigned long long *__restrict__ hkey,
                                     uint32_t *__restrict__ hval, uint64_t mask) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < ncand;
         i += gridDim.x * blockDim.x) {
        const uint64_t key = ckey[i];
        uint64_t h = hash64(key) & mask;
        for (;;) {
            const unsigned long long prev = atomicCAS(&hkey[h], EMPTY_KEY, key);
            if (prev == EMPTY_KEY || prev == key) {
                atomicMin(&hval[h], crec[i]);
                break;
            }
            h = (h + 1) & mask;
        }
    }
}

__global__ void newcov_own_kernel(const uint64_t *__restrict__ ckey,
                                  const uint32_t *__restrict__ crec, uint32_t ncand,
                                  const unsigned long long *__restrict__ hkey,
                                  const uint32_t *__restrict__ hval, uint64_t mask,
                                  uint8_t *__restrict__ is_new, uint32_t *__restrict__ maxcov,
                                  uint64_t words_per_call, uint32_t pc_lo) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < ncand;
         i += gridDim.x * blockDim.x) {
        const uint64_t key = ckey[i];
        uint64_t h = hash64(key) & mask;
        while (hkey[h] != key) h = (h + 1) & mask;
        if (hval[h] == crec[i]) is_new[crec[i]] = 1;
        const uint32_t c = (uint32_t)(key >> 32), pc = (uint32_t)key;
        const uint64_t o = (uint64_t)(uint32_t)(pc - pc_lo);
        atomicOr(&maxcov[(uint64_t)c * words_per_call + (o >> 5)], 1u << (o & 31));
    }
}

__global__ void bits_set_kernel(const uint32_t *__restrict__ pcs, uint64_t n,
                                uint32_t *__restrict__ bm, uint32_t pc_lo, uint64_t pc_span,
                                uint32_t *__restrict__ err) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t pc = pcs[i];
        const uint64_t o = (uint64_t)(uint32_t)(pc - pc_lo);
        if (pc < pc_lo || o >= pc_span) {
            *err = 1u;
            continue;
        }
        atomicOr(&bm[o >> 5], 1u << (o & 31));
    }
}

}  // namespace syz

// ------------------------------------------------ host-side orchestration
#include <mutex>
#include <new>

using namespace syz;

namespace syz {
struct CoverState {
    int dev = 0;
    int ncalls = 0;
    uint32_t pc_lo = 0;
    uint64_t pc_span = 0, words = 0;
    uint32_t *maxcov = nullptr;  // ncalls x words
    uint32_t *flakes = nullptr;  // words
    hipStream_t s = nullptr;
    std::mutex mu;  // the reference's coverMu
    // grow-only scratch
    void *scratch = nullptr;
    size_t scap = 0;
};

int bitmap_to_list(const uint32_t *bm, uint64_t pc_span, uint32_t pc_lo, uint32_t *out,
                   size_t cap, int64_t *count, hipStream_t s);
}  // namespace syz

static int grow(CoverState *st, size_t need) {
    if (need <= st->scap) return 0;
    if (st->scratch) hipFree(st->scratch);
    st->scratch = nullptr;
    st->scap = 0;
    size_t cap = need + need / 2;
    if (hipMalloc(&st->scratch, cap) != hipSuccess) return SYZCOV_ENOMEM;
    st->scap = cap;
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
    st->words = (pc_span + 31) / 32;
    if (hipStreamCreateWithFlags(&st->s, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&st->maxcov, (size_t)ncalls * st->words * 4) != hipSuccess ||
        hipMalloc(&st->flakes, st->words * 4) != hipSuccess) {
        if (st->maxcov) hipFree(st->maxcov);
        if (st->s) hipStreamDestroy(st->s);
        delete st;
        return SYZCOV_ENOMEM;
    }
    hipMemsetAsync(st->maxcov, 0, (size_t)ncalls * st->words * 4, st->s);
    hipMemsetAsync(st->flakes, 0, st->words * 4, st->s);
    if (hipStreamSynchronize(st->s) != hipSuccess) return SYZCOV_EHIP;
    *out = (syzcov_cover_state)(uintptr_t)st;
    return 0;
}

extern "C" int syzcov_state_destroy(syzcov_cover_state h) {
    CoverState *st = (CoverState *)(uintptr_t)h;
    if (!st) return SYZCOV_EINVAL;
    hipStreamSynchronize(st->s);
    hipFree(st->maxcov);
    hipFree(st->flakes);
    if (st->scratch) hipFree(st->scratch);
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
                       (uint64_t)n, bm, st->pc_lo, st->pc_span, derr);
    SYZ_LAUNCH_CHECK();
    uint32_t herr = 0;
    SYZ_HIP(hipMemcpyAsync(&herr, derr, 4, hipMemcpyDeviceToHost, st->s));
    SYZ_HIP(hipStreamSynchronize(st->s));
    if (herr) {
        set_error("PC outside the state's PC window");
        return SYZCOV_ERANGE;
    }
    return 0;
}

extern "C" int syzcov_state_add(syzcov_cover_state h, int call, const uint32_t *pcs, size_t n) {
    CoverState *st = (CoverState *)(uintptr_t)h;
    if (!st || call < 0 || call >= st->ncalls || (n && !pcs)) return SYZCOV_EINVAL;
    std::lock_guard<std::mutex> g(st->mu);
    hipSetDevice(st->dev);
    return set_bits(st, st->maxcov + (size_t)call * st->words, pcs, n);
}

extern "C" int syzcov_state_set_flakes(syzcov_cover_state h, const uint32_t *pcs, size_t n) {
    CoverState *st = (CoverState *)(uintptr_t)h;
    if (!st || (n && !pcs)) return SYZCOV_EINVAL;
    std::lock_guard<std::mutex> g(st->mu);
    hipSetDevice(st->dev);
    SYZ_HIP(hipMemsetAsync(st->flakes, 0, st->words * 4, st->s));
    return set_bits(st, st->flakes, pcs, n);
}

extern "C" int64_t syzcov_state_get(syzcov_cover_state h, int call, uint32_t *out, size_t cap) {
    CoverState *st = (CoverState *)(uintptr_t)h;
    if (!st || call < 0 || call >= st->ncalls) return SYZCOV_EINVAL;
    std::lock_guard<std::mutex> g(st->mu);
    hipSetDevice(st->dev);
    int64_t count = 0;
    int rc = bitmap_to_list(st->maxcov + (size_t)call * st->words, st->pc_span, st->pc_lo, out,
                            cap, &count, st->s);
    return rc ? rc : count;
}

extern "C" int64_t syzcov_newcov_batch(syzcov_cover_state h, const int32_t *callid,
                                       const uint64_t *rec_off, const uint32_t *rec_pcs,
                                       size_t nrec, uint8_t *is_new) {
    CoverState *st = (CoverState *)(uintptr_t)h;
    if (!st || (nrec && (!callid || !rec_off || !is_new))) return SYZCOV_EINVAL;
    if (nrec == 0) return 0;
    if (nrec > 0x7FFFFFFF) return SYZCOV_EINVAL;
    std::lock_guard<std::mutex> g(st->mu);
    hipSetDevice(st->dev);
    const uint64_t base0 = rec_off[0];
    const uint64_t npc = rec_off[nrec] - base0;
    if (npc && !rec_pcs) return SYZCOV_EINVAL;
    // layout: callid | off | pcs | rec_cnt | err,tot | is_new | ckey | crec | hkey | hval
    size_t o_cid = 0, o_off = align_up(o_cid + nrec * 4, 256),
           o_pcs = align_up(o_off + (nrec + 1) * 8, 256), o_cnt = align_up(o_pcs + npc * 4 + 4, 256),
           o_misc = align_up(o_cnt + nrec * 4, 256), o_new = align_up(o_misc + 16, 256),
           o_ckey = align_up(o_new + nrec, 256), o_crec = align_up(o_ckey + npc * 8 + 8, 256),
           o_end = align_up(o_crec + npc * 4 + 4, 256);
    int rc = grow(st, o_end);
    if (rc) return rc;
    uint8_t *S = (uint8_t *)st->scratch;
    int32_t *d_cid = (int32_t *)(S + o_cid);
    uint64_t *d_off = (uint64_t *)(S + o_off);
    uint32_t *d_pcs = (uint32_t *)(S + o_pcs), *d_cnt = (uint32_t *)(S + o_cnt);
    uint32_t *d_err = (uint32_t *)(S + o_misc), *d_tot = d_err + 1;
    uint8_t *d_new = S + o_new;
    uint64_t *d_ckey = (uint64_t *)(S + o_ckey);
    uint32_t *d_crec = (uint32_t *)(S + o_crec);
    hipStream_t s = st->s;
    // offsets rebased to 0
    uint64_t *hoff = (uint64_t *)malloc((nrec + 1) * 8);
    if (!hoff) return SYZCOV_ENOMEM;
    for (size_t k = 0; k <= nrec; k++) hoff[k] = rec_off[k] - base0;
    SYZ_HIP(hipMemsetAsync(d_err, 0, 16, s));
    SYZ_HIP(hipMemsetAsync(d_new, 0, nrec, s));
    SYZ_HIP(hipMemcpyAsync(d_cid, callid, nrec * 4, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(d_off, hoff, (nrec + 1) * 8, hipMemcpyHostToDevice, s));
    if (npc) SYZ_HIP(hipMemcpyAsync(d_pcs, rec_pcs + base0, npc * 4, hipMemcpyHostToDevice, s));
    const unsigned gr = grid_for(nrec, 1, 8192);
    hipLaunchKernelGGL(newcov_count_kernel, dim3(gr), dim3(NC_THREADS), 0, s, d_cid, d_off, d_pcs,
                       (uint32_t)nrec, st->maxcov, st->words, st->flakes, st->pc_lo, st->pc_span,
                       st->ncalls, d_cnt, d_err);
    hipLaunchKernelGGL(newcov_scan_kernel, dim3(1), dim3(1024), 0, s, d_cnt, (uint32_t)nrec, d_tot);
    hipLaunchKernelGGL(newcov_compact_kernel, dim3(gr), dim3(NC_THREADS), 0, s, d_cid, d_off, d_pcs,
                       (uint32_t)nrec, st->maxcov, st->words, st->flakes, st->pc_lo, st->pc_span,
                       st->ncalls, d_cnt, d_ckey, d_crec);
    SYZ_LAUNCH_CHECK();
    uint32_t hmisc[2];
    SYZ_HIP(hipMemcpyAsync(hmisc, d_err, 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    free(hoff);
    if (hmisc[0]) {
        set_error(hmisc[0] == 1 ? "PC outside the state's PC window"
                  : hmisc[0] == 2 ? "call id out of range"
                                  : "record cover not sorted");
        return hmisc[0] == 1 ? SYZCOV_ERANGE : hmisc[0] == 2 ? SYZCOV_EINVAL : SYZCOV_ENOTSORTED;
    }
    const uint32_t ncand = hmisc[1];
    if (ncand) {
        uint64_t cap = 1024;
        while (cap < 2ull * ncand) cap <<= 1;
        const size_t o_hkey = o_end, o_hval = align_up(o_hkey + cap * 8, 256),
                     o_fin = align_up(o_hval + cap * 4, 256);
        // grow preserving the candidate arrays: allocate fresh if needed
        if (o_fin > st->scap) {
            void *nb = nullptr;
            if (hipMalloc(&nb, o_fin + o_fin / 2) != hipSuccess) return SYZCOV_ENOMEM;
            SYZ_HIP(hipMemcpyAsync(nb, st->scratch, o_end, hipMemcpyDeviceToDevice, s));
            SYZ_HIP(hipStreamSynchronize(s));
            hipFree(st->scratch);
            st->scratch = nb;
            st->scap = o_fin + o_fin / 2;
            S = (uint8_t *)nb;
            d_new = S + o_new;
            d_ckey = (uint64_t *)(S + o_ckey);
            d_crec = (uint32_t *)(S + o_crec);
        }
        unsigned long long *d_hkey = (unsigned long long *)(S + o_hkey);
        uint32_t *d_hval = (uint32_t *)(S + o_hval);
        SYZ_HIP(hipMemsetAsync(d_hkey, 0xFF, cap * 8, s));
        SYZ_HIP(hipMemsetAsync(d_hval, 0xFF, cap * 4, s));
        hipLaunchKernelGGL(newcov_insert_kernel, dim3(grid_for(ncand, 256, 8192)), dim3(256), 0, s,
                           d_ckey, d_crec, ncand, d_hkey, d_hval, cap - 1);
        hipLaunchKernelGGL(newcov_own_kernel, dim3(grid_for(ncand, 256, 8192)), dim3(256), 0, s,
                           d_ckey, d_crec, ncand, d_hkey, d_hval, cap - 1, d_new, st->maxcov,
                           st->words, st->pc_lo);
        SYZ_LAUNCH_CHECK();
    }
    SYZ_HIP(hipMemcpyAsync(is_new, d_new, nrec, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    int64_t nnew = 0;
    for (size_t k = 0; k < nrec; k++) nnew += is_new[k];
    return nnew;
}
