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
#include "common.h"

namespace syz {

__device__ __forceinline__ bool bit_test(const uint32_t *__restrict__ bm, uint64_t o) {
    return (bm[o >> 5] >> (o & 31)) & 1u;
}

// Where a PC lives in the bitmaps: its window offset, or its dense key.
struct Index {
    int key_mode;
    uint32_t pc_lo, kshift, kbase;
    uint64_t span;  // window span, or nkeys
};

// Bitmap index of pc; false if pc is outside the window / key range.
__device__ __forceinline__ bool pc_index(const Index &X, uint32_t pc, uint32_t *idx) {
    if (X.key_mode) {
        const uint32_t k = (pc >> X.kshift) - X.kbase;  // wraps past span below kbase
        *idx = k;
        return k < X.span;
    }
    const uint32_t o = pc - X.pc_lo;
    *idx = o;
    return pc >= X.pc_lo && (uint64_t)o < X.span;
}

constexpr int NC_THREADS = 256;
constexpr int NC_WPB = NC_THREADS / 64;
constexpr int NC_U = 8;  // rows of 64 PCs in flight per wave

// Records grouped by CallID (counting sort in one workgroup): the candidate
// pass walks them in this order so the records of one call run together on
// one XCD and share its L2 copy of maxCover[call] (the probes of one record
// touch ~2k random lines of an 8 MB bitmap; a call's records hit mostly the
// same hot lines).  perm[] is only a visiting order: ownership still uses
// the batch index k.
constexpr int GRP_MAX_CALLS = 16384;

__global__ __launch_bounds__(1024) void newcov_group_kernel(const int32_t *__restrict__ callid,
                                                             uint32_t nrec, int ncalls,
                                                             uint32_t *__restrict__ perm) {
    __shared__ uint32_t h[GRP_MAX_CALLS];
    __shared__ uint32_t tmp[1024 / 64 + 1];
    const uint32_t t = threadIdx.x;
    if (ncalls > GRP_MAX_CALLS) {
        for (uint32_t k = t; k < nrec; k += 1024) perm[k] = k;
        return;
    }
    for (int c = t; c < ncalls; c += 1024) h[c] = 0;
    __syncthreads();
    for (uint32_t k = t; k < nrec; k += 1024) {
        const int c = callid[k];
        if (c >= 0 && c < ncalls) atomicAdd(&h[c], 1u);
    }
    __syncthreads();
    uint32_t carry = 0;  // exclusive scan; bad call ids go last
    for (int c0 = 0; c0 < ncalls; c0 += 1024) {
        const int c = c0 + (int)t;
        const uint32_t v = c < ncalls ? h[c] : 0u;
        uint32_t total;
        const uint32_t p = block_excl_scan<1024>(v, tmp, &total);
        __syncthreads();
        if (c < ncalls) h[c] = carry + p;
        carry += total;
        __syncthreads();
    }
    __shared__ uint32_t bad_pos;
    if (t == 0) bad_pos = carry;
    __syncthreads();
    for (uint32_t k = t; k < nrec; k += 1024) {
        const int c = callid[k];
        const uint32_t pos = (c >= 0 && c < ncalls) ? atomicAdd(&h[c], 1u) : atomicAdd(&bad_pos, 1u);
        perm[pos] = k;
    }
}

// stats[0] = error (1 window, 2 call id, 3 unsorted), stats[1] = candidates.
// One WAVEFRONT per record: coalesced 64-PC rows, both bitmap probes per PC,
// ballot compaction of the survivors into the record's OWN slots of cpc
// (cpc is indexed like pcs), so no global atomics per row; one atomic per
// wave for the batch total.  Once maxCover saturates (a fuzzer's steady
// state) almost every record has zero survivors.
__global__ __launch_bounds__(NC_THREADS) void newcov_cand_kernel(
    const int32_t *__restrict__ callid, const uint64_t *__restrict__ rec_off,
    const uint32_t *__restrict__ pcs, uint32_t nrec, const uint32_t *__restrict__ maxcov,
    uint64_t words_per_call, const uint32_t *__restrict__ flakes, Index X, int ncalls,
    const uint32_t *__restrict__ perm, uint8_t *__restrict__ is_new, uint32_t *__restrict__ cpc,
    uint32_t *__restrict__ rec_cnt, uint32_t *__restrict__ stats) {
    const uint32_t l = __lane_id();
    const uint64_t lt = (1ull << l) - 1ull;
    // XCD-aware: workgroups are dispatched round-robin over the 8 XCDs, so
    // the workgroups of XCD x (blockIdx % 8 == x) take the x-th eighth of
    // the call-grouped records
    const uint32_t x = blockIdx.x & 7, nbx = gridDim.x >> 3;
    const uint32_t j0 = (uint32_t)((uint64_t)nrec * x / 8), j1 = (uint32_t)((uint64_t)nrec * (x + 1) / 8);
    const uint32_t nw = nbx * NC_WPB;
    uint32_t wave_tot = 0;
    for (uint32_t j = j0 + (blockIdx.x >> 3) * NC_WPB + (threadIdx.x >> 6); j < j1; j += nw) {
        const uint32_t k = perm[j];
        const int c = callid[k];
        if (l == 0) is_new[k] = 0;
        if (c < 0 || c >= ncalls) {
            if (l == 0) {
                stats[0] = 2u;
                rec_cnt[k] = 0;
            }
            continue;
        }
        const uint32_t *M = maxcov + (uint64_t)c * words_per_call;
        const uint64_t b = rec_off[k], n = rec_off[k + 1] - b;
        uint32_t bad = 0, cnt = 0, carry = 0;
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
                const bool sent = pc[u] == 0xFFFFFFFFu;
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
                carry = __builtin_amdgcn_readlane(pc[u], 63);
                if (q < n && q > 0 && prev > pc[u]) bad |= 2u;
                // maxCover first: once it saturates, flakes are rarely probed
                const bool cand =
                    ok[u] && !((w[u] >> (ix[u] & 31)) & 1u) && !bit_test(flakes, ix[u]);
                const uint64_t m = __ballot(cand);
                if (cand) cpc[b + cnt + (uint32_t)__popcll(m & lt)] = pc[u];
                cnt += (uint32_t)__popcll(m);
            }
        }
        if (bad) stats[0] = (bad & 1u) ? 1u : 3u;
        if (l == 0) rec_cnt[k] = cnt;
        wave_tot += cnt;
    }
    if (l == 0 && wave_tot) atomicAdd(&stats[1], wave_tot);
}

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

// first-cover of every candidate key (CallID, pc): hval = min record index
__global__ __launch_bounds__(NC_THREADS) void newcov_insert_kernel(
    const int32_t *__restrict__ callid, const uint64_t *__restrict__ rec_off,
    const uint32_t *__restrict__ cpc, const uint32_t *__restrict__ rec_cnt, uint32_t nrec,
    const uint32_t *__restrict__ stats, unsigned long long *__restrict__ hkey,
    uint32_t *__restrict__ hval) {
    if (stats[0] || !stats[1]) return;
    const uint64_t mask = hash_cap(stats[1]) - 1;
    const uint32_t l = __lane_id(), nw = gridDim.x * NC_WPB;
    for (uint32_t k = blockIdx.x * NC_WPB + (threadIdx.x >> 6); k < nrec; k += nw) {
        const uint32_t cnt = rec_cnt[k];
        if (!cnt) continue;
        const uint64_t hi = (uint64_t)(uint32_t)callid[k] << 32, b = rec_off[k];
        for (uint32_t i = l; i < cnt; i += 64) {
            const uint64_t key = hi | cpc[b + i];
            uint64_t h = hash64(key) & mask;
            for (;;) {
                const unsigned long long prev = atomicCAS(&hkey[h], EMPTY_KEY, key);
                if (prev == EMPTY_KEY || prev == key) {
                    atomicMin(&hval[h], k);
                    break;
                }
                h = (h + 1) & mask;
            }
        }
    }
}

// record k is new iff it owns (first-covers) one of its keys; each owned key
// is OR-ed into maxCover once
__global__ __launch_bounds__(NC_THREADS) void newcov_own_kernel(
    const int32_t *__restrict__ callid, const uint64_t *__restrict__ rec_off,
    const uint32_t *__restrict__ cpc, const uint32_t *__restrict__ rec_cnt, uint32_t nrec,
    const uint32_t *__restrict__ stats, const unsigned long long *__restrict__ hkey,
    const uint32_t *__restrict__ hval, uint8_t *__restrict__ is_new,
    uint32_t *__restrict__ maxcov, uint64_t words_per_call, Index X) {
    if (stats[0] || !stats[1]) return;
    const uint64_t mask = hash_cap(stats[1]) - 1;
    const uint32_t l = __lane_id(), nw = gridDim.x * NC_WPB;
    for (uint32_t k = blockIdx.x * NC_WPB + (threadIdx.x >> 6); k < nrec; k += nw) {
        const uint32_t cnt = rec_cnt[k];
        if (!cnt) continue;
        const uint32_t c = (uint32_t)callid[k];
        const uint64_t hi = (uint64_t)c << 32, b = rec_off[k];
        uint32_t *M = maxcov + (uint64_t)c * words_per_call;
        bool own = false;
        for (uint32_t i = l; i < cnt; i += 64) {
            const uint32_t pc = cpc[b + i];
            const uint64_t key = hi | pc;
            uint64_t h = hash64(key) & mask;
            while (hkey[h] != key) h = (h + 1) & mask;
            if (hval[h] == k) {
                own = true;
                uint32_t ix;
                pc_index(X, pc, &ix);  // candidates are inside (checked by the cand pass)
                atomicOr(&M[ix >> 5], 1u << (ix & 31));
            }
        }
        if (__ballot(own) && l == 0) is_new[k] = 1;
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

}  // namespace syz

// ------------------------------------------------ host-side orchestration
#include <algorithm>
#include <mutex>
#include <new>
#include <vector>

using namespace syz;

namespace syz {
struct CoverState {
    int dev = 0;
    int ncalls = 0;
    uint32_t pc_lo = 0;
    uint64_t pc_span = 0;
    // bitmap index space: window offsets, or dense keys of the registered
    // universe (key mode); words = 32-bit words per bitmap
    Index X{};
    uint64_t words = 0;
    uint32_t *maxcov = nullptr;  // ncalls x words
    uint32_t *flakes = nullptr;  // words
    uint32_t *pc_of_key = nullptr;  // key mode: key -> PC (reads of maxCover)
    bool dirty = false;          // maxCover touched: the universe can no longer change
    hipStream_t s = nullptr;
    std::mutex mu;  // the reference's coverMu
    // grow-only scratch
    void *scratch = nullptr;
    size_t scap = 0;
};

int bitmap_to_list(const uint32_t *bm, uint64_t pc_span, uint32_t pc_lo, uint32_t *out,
                   size_t cap, int64_t *count, hipStream_t s, const uint32_t *pc_of_key);
}  // namespace syz

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

// (re)allocate the bitmaps for the current index space, zeroed
static int alloc_maps(CoverState *st) {
    if (st->maxcov) hipFree(st->maxcov);
    if (st->flakes) hipFree(st->flakes);
    st->maxcov = st->flakes = nullptr;
    st->words = (st->X.span + 31) / 32;
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
    st->X = Index{0, pc_lo, 0, 0, pc_span};
    int rc = hipStreamCreateWithFlags(&st->s, hipStreamNonBlocking) == hipSuccess
                 ? alloc_maps(st) : SYZCOV_EHIP;
    if (rc) {
        if (st->maxcov) hipFree(st->maxcov);
        if (st->flakes) hipFree(st->flakes);
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
    if (st->pc_of_key) hipFree(st->pc_of_key);
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

extern "C" int syzcov_state_add(syzcov_cover_state h, int call, const uint32_t *pcs, size_t n) {
    CoverState *st = (CoverState *)(uintptr_t)h;
    if (!st || call < 0 || call >= st->ncalls || (n && !pcs)) return SYZCOV_EINVAL;
    std::lock_guard<std::mutex> g(st->mu);
    hipSetDevice(st->dev);
    st->dirty = true;
    return set_bits(st, st->maxcov + (size_t)call * st->words, pcs, n);
}

// Key mode (keys.hip): the PC universe (allCoverPCs, syz-manager/cover.go:57-69;
// inside the window, any order, duplicates allowed) fixes kshift / kbase /
// nkeys; maxCover and flakes become bitmaps over its dense keys.  Allowed
// only while maxCover is empty.  Contract from then on: every PC passed in
// belongs to the universe (KCOV reports only its call sites); a PC outside
// the universe's key range is rejected, one inside it is trusted.
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
    st->pc_of_key = nullptr;
    st->X = Index{0, st->pc_lo, 0, 0, st->pc_span};  // back to window mode
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
        const uint32_t k31 = 31;
        if (hipMemcpyAsync(d_ks, &k31, 4, hipMemcpyHostToDevice, st->s) != hipSuccess) {
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
        if (hipMalloc(&st->pc_of_key, nkeys * 4) != hipSuccess) { rc = SYZCOV_ENOMEM; break; }
        if (hipMemsetAsync(d_n, 0, 4, st->s) != hipSuccess) { rc = SYZCOV_EHIP; break; }
        if ((rc = syzcov_dev_universe_keymap(lst, hn, ks, kbase, nkeys, st->pc_of_key, d_n, st->s)))
            break;
        st->X = Index{1, st->pc_lo, ks, kbase, nkeys};
        rc = alloc_maps(st);
    } while (0);
    if (bm) hipFree(bm);
    if (tab) hipFree(tab);
    if (ws) hipFree(ws);
    if (lst) hipFree(lst);
    if (sc) hipFree(sc);
    if (rc) {
        if (st->pc_of_key) hipFree(st->pc_of_key);
        st->pc_of_key = nullptr;
        st->X = Index{0, st->pc_lo, 0, 0, st->pc_span};
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
    return set_bits(st, st->flakes, pcs, n);
}

extern "C" int64_t syzcov_state_get(syzcov_cover_state h, int call, uint32_t *out, size_t cap) {
    CoverState *st = (CoverState *)(uintptr_t)h;
    if (!st || call < 0 || call >= st->ncalls) return SYZCOV_EINVAL;
    std::lock_guard<std::mutex> g(st->mu);
    hipSetDevice(st->dev);
    int64_t count = 0;
    const uint32_t *bm = st->maxcov + (size_t)call * st->words;
    int rc = st->X.key_mode
                 ? bitmap_to_list(bm, st->X.span, 0, out, cap, &count, st->s, st->pc_of_key)
                 : bitmap_to_list(bm, st->pc_span, st->pc_lo, out, cap, &count, st->s, nullptr);
    return rc ? rc : count;
}

// device workspace: cpc u32[npc] | rec_cnt u32[nrec] | perm u32[nrec] | hkey u64[cap] |
//                   hval u32[cap] | stats
static void nc_layout(size_t nrec, uint64_t npc, size_t *o_cnt, size_t *o_hkey, size_t *o_hval,
                      size_t *o_stats, size_t *end) {
    uint64_t cap = 1024;
    while (cap < 2ull * npc) cap <<= 1;
    *o_cnt = align_up(npc * 4 + 4, 256);
    *o_hkey = align_up(*o_cnt + 2 * align_up(nrec * 4 + 4, 256), 256);
    *o_hval = align_up(*o_hkey + cap * 8, 256);
    *o_stats = align_up(*o_hval + cap * 4, 256);
    *end = *o_stats + 256;
}

extern "C" size_t syzcov_state_newcov_ws_size(size_t nrec, uint64_t npc) {
    size_t a, b, c, d, e;
    nc_layout(nrec, npc, &a, &b, &c, &d, &e);
    return e;
}

static int newcov_launch(CoverState *st, const int32_t *callid, const uint64_t *rec_off,
                         const uint32_t *pcs, size_t nrec, uint64_t npc, uint8_t *is_new,
                         uint8_t *ws, uint32_t **stats_out, hipStream_t s) {
    size_t o_cnt, o_hkey, o_hval, o_stats, end;
    nc_layout(nrec, npc, &o_cnt, &o_hkey, &o_hval, &o_stats, &end);
    uint32_t *cpc = (uint32_t *)ws;
    uint32_t *cnt = (uint32_t *)(ws + o_cnt);
    uint32_t *perm = (uint32_t *)(ws + o_cnt + align_up(nrec * 4 + 4, 256));
    unsigned long long *hkey = (unsigned long long *)(ws + o_hkey);
    uint32_t *hval = (uint32_t *)(ws + o_hval);
    uint32_t *stats = (uint32_t *)(ws + o_stats);
    *stats_out = stats;
    SYZ_HIP(hipMemsetAsync(stats, 0, 16, s));
    const unsigned gr = grid_for(nrec, NC_WPB, 4096);
    hipLaunchKernelGGL(newcov_group_kernel, dim3(1), dim3(1024), 0, s, callid, (uint32_t)nrec,
                       st->ncalls, perm);
    const unsigned gx = (grid_for(nrec, NC_WPB, 4096) + 7) & ~7u;  // a multiple of the 8 XCDs
    hipLaunchKernelGGL(newcov_cand_kernel, dim3(gx), dim3(NC_THREADS), 0, s, callid, rec_off, pcs,
                       (uint32_t)nrec, st->maxcov, st->words, st->flakes, st->X, st->ncalls,
                       (const uint32_t *)perm, is_new, cpc, cnt, stats);
    const unsigned gh = grid_for(std::max<uint64_t>(npc, 512), 256, 8192);
    hipLaunchKernelGGL(hash_clear_kernel, dim3(gh), dim3(256), 0, s, (const uint32_t *)stats, hkey,
                       hval);
    hipLaunchKernelGGL(newcov_insert_kernel, dim3(gr), dim3(NC_THREADS), 0, s, callid, rec_off,
                       (const uint32_t *)cpc, (const uint32_t *)cnt, (uint32_t)nrec,
                       (const uint32_t *)stats, hkey, hval);
    hipLaunchKernelGGL(newcov_own_kernel, dim3(gr), dim3(NC_THREADS), 0, s, callid, rec_off,
                       (const uint32_t *)cpc, (const uint32_t *)cnt, (uint32_t)nrec,
                       (const uint32_t *)stats, (const unsigned long long *)hkey,
                       (const uint32_t *)hval, is_new, st->maxcov, st->words, st->X);
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
    st->dirty = true;
    uint32_t *dstats = nullptr;
    int rc = newcov_launch(st, callid, rec_off, pcs, nrec, npc, is_new, (uint8_t *)ws, &dstats, s);
    if (rc) return rc;
    if (stats) SYZ_HIP(hipMemcpyAsync(stats, dstats, 8, hipMemcpyDeviceToDevice, s));
    return 0;
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
    if (npc > 0xFFFFFFFFull) return SYZCOV_EINVAL;
    // staging: callid | off | pcs | is_new | newcov workspace
    const size_t o_off = align_up(nrec * 4, 256), o_pcs = align_up(o_off + (nrec + 1) * 8, 256),
                 o_new = align_up(o_pcs + npc * 4 + 4, 256), o_ws = align_up(o_new + nrec, 256),
                 o_end = o_ws + syzcov_state_newcov_ws_size(nrec, npc);
    int rc = grow(st, o_end);
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
                       (const uint32_t *)(S + o_pcs), nrec, npc, S + o_new, S + o_ws, &dstats, s);
    if (rc) return rc;
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
