// canon_ids.hip — corpus-scale Canonicalize into the dense PC-id space, and
// the chunked first-cover Minimize over it (engine fast path).
//
// Canonicalize (cover/cover.go:27-40) of a whole corpus once the dictionary
// exists (dict.hip): every raw PC becomes its dense id (ids are ranks in PC
// order, so sorting ids sorts PCs), and each segment is sorted by an
// LDS-staged LSD radix sort and de-duplicated by ONE workgroup:
//   pass 0  low <= 11 bits, unstable (LDS atomic slots) — LSD only needs the
//           later passes to be stable;
//   pass k  next <= 10 bits, stable: keys in wave-striped order, ranks from a
//           wave-level match (10 ballots) + per-(digit, wave) LDS counters,
//           digit-major/wave-minor exclusive scan.
// Padding lanes never take part, so no key value is reserved.  Unique keeps
// the `last := sent` quirk in id space (the id of PC 0xFFFFFFFF, when
// present, is dropped iff it is the first key).  Output: canonical ids in the
// input's CSR slot + new lengths; PCs are materialised on demand through the
// dictionary (syzcov_dev_gather_u32 over syzcov_dev_dict_pcs).
//
// Minimize pass 1 then reads ids directly.  Ranks are processed in
// geometrically growing chunks; between chunks a covered bitmap (ids with
// first < INT32_MAX, n_ids bits, L2-resident) is rebuilt, and inside a chunk a
// PC whose bit is set cannot be first for any rank of the chunk and costs one
// cached bit test — the atomic path only sees PCs not yet covered.
#include "common.h"

#include <algorithm>

namespace syz {

int canon_large_path(const uint64_t *off, const uint32_t *in, uint32_t *out, uint32_t *new_len,
                     const uint32_t *dlist, uint32_t nlarge, uint8_t *pres, uint32_t pc_lo,
                     uint64_t pc_span, uint32_t *err, hipStream_t s);

__device__ __forceinline__ int bit_length(uint32_t x) { return x ? 32 - __clz(x) : 0; }

// exclusive scan of cnt entries of LDS array h in place (contiguous runs per
// thread); needs THREADS | cnt.
template <int THREADS>
__device__ __forceinline__ void lds_excl_scan(uint32_t *h, uint32_t cnt, uint32_t *tmp) {
    const uint32_t per = cnt / THREADS;
    const uint32_t b = threadIdx.x * per;
    uint32_t s = 0;
    for (uint32_t q = 0; q < per; q++) s += h[b + q];
    uint32_t total;
    uint32_t pre = block_excl_scan<THREADS>(s, tmp, &total);
    for (uint32_t q = 0; q < per; q++) {
        const uint32_t v = h[b + q];
        h[b + q] = pre;
        pre += v;
    }
    __syncthreads();
}

// IDS = true: keys are dense ids (dictionary built beforehand, `tab`).
// IDS = false: keys are window offsets pc - pc_lo (no dictionary needed), the
// canonical list is written as PCs, and every kept PC is marked in the
// presence bitmap `pres` (test-before-atomicOr) — mark fused into the sort.
template <int THREADS, int ITEMS, bool IDS>
__global__ __launch_bounds__(THREADS) void canon_ids_kernel(
    const uint64_t *__restrict__ off, const uint32_t *__restrict__ raw, uint32_t *__restrict__ out,
    uint32_t *__restrict__ new_len, const uint32_t *__restrict__ list,
    const uint32_t *__restrict__ count, const uint64_t *__restrict__ tab, uint32_t pc_lo,
    uint64_t pc_span, const uint32_t *__restrict__ n_ids_ptr, uint32_t *__restrict__ pres,
    uint32_t *__restrict__ err) {
    constexpr int NW = THREADS / 64, CAP = THREADS * ITEMS;
    constexpr int UB = 11, SB = 10;  // unstable / stable digit widths
    constexpr int HSZ = (1 << UB) > (NW << SB) ? (1 << UB) : (NW << SB);
    __shared__ uint32_t keys[CAP];
    __shared__ uint32_t hist[HSZ];
    __shared__ uint32_t tmp[THREADS / 64 + 1];
    const uint32_t t = threadIdx.x, w = t >> 6, l = __lane_id();
    const uint64_t ltmask = (1ull << l) - 1ull;
    int nbits;
    // key of PC 0xFFFFFFFF (dropped iff first: `last := sent`), or none
    uint32_t sent_id = 0xFFFFFFFFu;
    const uint64_t so = (uint64_t)(uint32_t)(SYZ_SENT - pc_lo);
    if (IDS) {
        const uint32_t nids = *n_ids_ptr;
        nbits = max(1, bit_length(nids - 1));
        // present sentinel = max PC -> max id
        if (so < pc_span && ((uint32_t)(tab[so >> 5] >> 32) >> (so & 31)) & 1u) sent_id = nids - 1;
    } else {
        nbits = max(1, bit_length((uint32_t)(pc_span - 1)));
        if (so < pc_span) sent_id = (uint32_t)so;
    }
    const uint32_t nlist = *count;
    for (uint32_t li = blockIdx.x; li < nlist; li += gridDim.x) {
        const uint32_t seg = list[li];
        const uint64_t base = off[seg];
        const uint32_t n = (uint32_t)(off[seg + 1] - base);
        uint32_t k[ITEMS], r[ITEMS];
        // load raw PCs (wave-striped, coalesced) and map to dense ids
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            const uint32_t e = w * 64 * ITEMS + i * 64 + l;
            k[i] = 0;
            if (e < n) {
                const uint32_t pc = raw[base + e];
                const uint64_t o = (uint64_t)(uint32_t)(pc - pc_lo);
                if (pc < pc_lo || o >= pc_span)
                    *err = 1u;
                else
                    k[i] = IDS ? dense_id(tab, pc, pc_lo) : (uint32_t)o;
            }
        }
        // ---- pass 0: low UB bits, unstable
        const int b0 = min(UB, nbits);
        const uint32_t m0 = (1u << b0) - 1u;
        for (uint32_t q = t; q < (1u << UB); q += THREADS) hist[q] = 0;
        __syncthreads();
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            const uint32_t e = w * 64 * ITEMS + i * 64 + l;
            if (e < n) r[i] = atomicAdd(&hist[k[i] & m0], 1u);
        }
        __syncthreads();
        lds_excl_scan<THREADS>(hist, 1u << UB, tmp);
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            const uint32_t e = w * 64 * ITEMS + i * 64 + l;
            if (e < n) keys[hist[k[i] & m0] + r[i]] = k[i];
        }
        __syncthreads();
        // ---- stable passes
        for (int shift = b0; shift < nbits; shift += SB) {
            const uint32_t ms = (1u << min(SB, nbits - shift)) - 1u;
#pragma unroll
            for (int i = 0; i < ITEMS; i++) {
                const uint32_t e = w * 64 * ITEMS + i * 64 + l;
                k[i] = e < n ? keys[e] : 0u;
            }
            for (uint32_t q = t; q < (uint32_t)(NW << SB); q += THREADS) hist[q] = 0;
            __syncthreads();
#pragma unroll
            for (int i = 0; i < ITEMS; i++) {
                const uint32_t e = w * 64 * ITEMS + i * 64 + l;
                const bool act = e < n;
                const uint32_t d = (k[i] >> shift) & ms;
                uint64_t peers = __ballot(act);
#pragma unroll
                for (int b = 0; b < SB; b++) {
                    const bool bit = (d >> b) & 1u;
                    const uint64_t m = __ballot(bit);
                    peers &= bit ? m : ~m;
                }
                if (act) {
                    const uint32_t slot = d * NW + w;
                    const uint32_t cnt = hist[slot];
                    r[i] = cnt + __popcll(peers & ltmask);
                    if ((peers & ltmask) == 0) hist[slot] = cnt + __popcll(peers);
                }
            }
            __syncthreads();
            lds_excl_scan<THREADS>(hist, (uint32_t)(NW << SB), tmp);
#pragma unroll
            for (int i = 0; i < ITEMS; i++) {
                const uint32_t e = w * 64 * ITEMS + i * 64 + l;
                if (e < n) keys[hist[((k[i] >> shift) & ms) * NW + w] + r[i]] = k[i];
            }
            __syncthreads();
        }
        // ---- unique (blocked) + compaction in LDS + coalesced write
        uint32_t v[ITEMS], keepmask = 0, cnt = 0;
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            const uint32_t e = t * ITEMS + i;
            v[i] = keys[e];
            const uint32_t prev = e == 0 ? sent_id : (i == 0 ? keys[e - 1] : v[i - 1]);
            const bool keep = e < n && v[i] != prev;
            keepmask |= (uint32_t)keep << i;
            cnt += keep;
        }
        uint32_t total;
        uint32_t pos = block_excl_scan<THREADS>(cnt, tmp, &total);
#pragma unroll
        for (int i = 0; i < ITEMS; i++)
            if (keepmask & (1u << i)) keys[pos++] = v[i];
        __syncthreads();
        for (uint32_t q = t; q < total; q += THREADS) {
            const uint32_t key = keys[q];
            if (IDS) {
                out[base + q] = key;
            } else {
                out[base + q] = pc_lo + key;
                const uint32_t m = 1u << (key & 31);
                if (!(pres[key >> 5] & m)) atomicOr(&pres[key >> 5], m);
            }
        }
        if (t == 0) new_len[seg] = total;
        __syncthreads();
    }
}

// Large segments in the PC-space engine: mark the canonical PCs the generic
// large path produced.
__global__ void mark_large_kernel(const uint64_t *__restrict__ off,
                                  const uint32_t *__restrict__ list, uint32_t nlarge,
                                  const uint32_t *__restrict__ new_len,
                                  const uint32_t *__restrict__ data, uint32_t *__restrict__ pres,
                                  uint32_t pc_lo) {
    for (uint32_t li = blockIdx.x; li < nlarge; li += gridDim.x) {
        const uint32_t seg = list[li];
        const uint64_t b = off[seg];
        for (uint32_t q = threadIdx.x; q < new_len[seg]; q += blockDim.x) {
            const uint32_t o = data[b + q] - pc_lo;
            atomicOr(&pres[o >> 5], 1u << (o & 31));
        }
    }
}

// Large segments (> 16384 raw PCs): canonical PCs via the generic large path,
// then each PC is replaced by its id in place.
__global__ void pcs_to_ids_kernel(const uint64_t *__restrict__ off, const uint32_t *__restrict__ list,
                                  uint32_t nlarge, const uint32_t *__restrict__ new_len,
                                  uint32_t *__restrict__ data, const uint64_t *__restrict__ tab,
                                  uint32_t pc_lo) {
    for (uint32_t li = blockIdx.x; li < nlarge; li += gridDim.x) {
        const uint32_t seg = list[li];
        const uint64_t b = off[seg];
        for (uint32_t q = threadIdx.x; q < new_len[seg]; q += blockDim.x)
            data[b + q] = dense_id(tab, data[b + q], pc_lo);
    }
}

// ---------------------------------------------------------------- Minimize
constexpr int MI_THREADS = 256;

__global__ __launch_bounds__(MI_THREADS) void mini_ids_pass1_kernel(
    const uint64_t *__restrict__ off, const uint32_t *__restrict__ len,
    const uint32_t *__restrict__ ids, const int32_t *__restrict__ order,
    const int32_t *__restrict__ ranks, uint32_t j0, uint32_t j1,
    const uint32_t *__restrict__ covered, int32_t *__restrict__ first,
    uint8_t *__restrict__ cand) {
    for (uint32_t j = j0 + blockIdx.x; j < j1; j += gridDim.x) {
        const int32_t idx = order[j];
        const int32_t r = ranks ? ranks[j] : (int32_t)j;
        const uint64_t b = off[idx];
        const uint32_t l = len[idx];
        bool won = false;
        for (uint32_t k = threadIdx.x; k < l; k += MI_THREADS) {
            const uint32_t id = ids[b + k];
            if (covered && ((covered[id >> 5] >> (id & 31)) & 1u)) continue;
            const int32_t f = __hip_atomic_load(&first[id], __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
            if (f > r) won |= atomicMin(&first[id], r) > r;
        }
        won = __syncthreads_or(won);
        if (threadIdx.x == 0) cand[j] = won ? 1 : 0;
    }
}

__global__ void covered_update_kernel(const int32_t *__restrict__ first,
                                      const uint32_t *__restrict__ n_ids_ptr, uint32_t nwords,
                                      uint32_t *__restrict__ covered) {
    const uint32_t nids = *n_ids_ptr;
    for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < nwords;
         w += gridDim.x * blockDim.x) {
        uint32_t bits = 0;
        const uint32_t id0 = w * 32;
        if (id0 < nids) {
            const uint32_t m = min(32u, nids - id0);
            for (uint32_t q = 0; q < m; q++) bits |= (uint32_t)(first[id0 + q] != 0x7FFFFFFF) << q;
        }
        covered[w] = bits;
    }
}

__global__ __launch_bounds__(MI_THREADS) void mini_ids_pass2_kernel(
    const uint64_t *__restrict__ off, const uint32_t *__restrict__ len,
    const uint32_t *__restrict__ ids, const int32_t *__restrict__ order,
    const int32_t *__restrict__ ranks, uint32_t n, const int32_t *__restrict__ first,
    const uint8_t *__restrict__ cand, uint8_t *__restrict__ kept) {
    for (uint32_t j = blockIdx.x; j < n; j += gridDim.x) {
        if (!cand[j]) continue;
        const int32_t idx = order[j];
        const int32_t r = ranks ? ranks[j] : (int32_t)j;
        const uint64_t b = off[idx];
        const uint32_t l = len[idx];
        bool found = false;
        for (uint32_t k0 = 0; k0 < l; k0 += MI_THREADS) {
            const uint32_t k = k0 + threadIdx.x;
            const bool f = k < l && first[ids[b + k]] == r;
            if (__syncthreads_or(f)) {
                found = true;
                break;
            }
        }
        if (threadIdx.x == 0 && found) kept[r] = 1;
    }
}

// ---- window-space Minimize (PC-space engine): first[] indexed by pc - pc_lo.
// `covered` = PCs with a first-cover rank before the current chunk (read only
// inside a chunk), `touched` = PCs that got their first rank during it
// (covered |= touched between chunks).
__global__ __launch_bounds__(MI_THREADS) void mini_win_pass1_kernel(
    const uint64_t *__restrict__ off, const uint32_t *__restrict__ len,
    const uint32_t *__restrict__ pcs, const int32_t *__restrict__ order,
    const int32_t *__restrict__ ranks, uint32_t j0, uint32_t j1, uint32_t pc_lo,
    const uint32_t *__restrict__ covered, uint32_t *__restrict__ touched,
    int32_t *__restrict__ first, uint8_t *__restrict__ cand) {
    for (uint32_t j = j0 + blockIdx.x; j < j1; j += gridDim.x) {
        const int32_t idx = order[j];
        const int32_t r = ranks ? ranks[j] : (int32_t)j;
        const uint64_t b = off[idx];
        const uint32_t l = len[idx];
        bool won = false;
        for (uint32_t k = threadIdx.x; k < l; k += MI_THREADS) {
            const uint32_t o = pcs[b + k] - pc_lo;
            const uint32_t m = 1u << (o & 31);
            if (covered[o >> 5] & m) continue;
            const int32_t f = __hip_atomic_load(&first[o], __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
            if (f > r) {
                const int32_t old = atomicMin(&first[o], r);
                won |= old > r;
                if (old == 0x7FFFFFFF) atomicOr(&touched[o >> 5], m);
            }
        }
        won = __syncthreads_or(won);
        if (threadIdx.x == 0) cand[j] = won ? 1 : 0;
    }
}

__global__ void or_words_kernel(uint32_t *__restrict__ dst, const uint32_t *__restrict__ src,
                                uint64_t nwords) {
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords;
         w += (uint64_t)gridDim.x * blockDim.x)
        dst[w] |= src[w];
}

__global__ __launch_bounds__(MI_THREADS) void mini_win_pass2_kernel(
    const uint64_t *__restrict__ off, const uint32_t *__restrict__ len,
    const uint32_t *__restrict__ pcs, const int32_t *__restrict__ order,
    const int32_t *__restrict__ ranks, uint32_t n, uint32_t pc_lo,
    const int32_t *__restrict__ first, const uint8_t *__restrict__ cand,
    uint8_t *__restrict__ kept) {
    for (uint32_t j = blockIdx.x; j < n; j += gridDim.x) {
        if (!cand[j]) continue;
        const int32_t idx = order[j];
        const int32_t r = ranks ? ranks[j] : (int32_t)j;
        const uint64_t b = off[idx];
        const uint32_t l = len[idx];
        bool found = false;
        for (uint32_t k0 = 0; k0 < l; k0 += MI_THREADS) {
            const uint32_t k = k0 + threadIdx.x;
            const bool f = k < l && first[pcs[b + k] - pc_lo] == r;
            if (__syncthreads_or(f)) {
                found = true;
                break;
            }
        }
        if (threadIdx.x == 0 && found) kept[r] = 1;
    }
}

// window-indexed first[] <-> dense-id first[] (compact form for the RCCL MIN)
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

__global__ void gather_u32_kernel(const uint32_t *__restrict__ table,
                                  const uint64_t *__restrict__ off, const uint32_t *__restrict__ len,
                                  const uint32_t *__restrict__ in, size_t nseg,
                                  uint32_t *__restrict__ out) {
    for (size_t s = blockIdx.x; s < nseg; s += gridDim.x) {
        const uint64_t b = off[s];
        const uint32_t l = len[s];
        for (uint32_t q = threadIdx.x; q < l; q += blockDim.x) out[b + q] = table[in[b + q]];
    }
}

// full id -> PC list (sentinel kept), the inverse of dense_id
__global__ void dict_pcs_kernel(const uint64_t *__restrict__ tab, uint64_t nwords, uint32_t pc_lo,
                                uint32_t *__restrict__ out) {
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords;
         w += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t e = tab[w];
        uint32_t bits = (uint32_t)(e >> 32), pos = (uint32_t)e;
        while (bits) {
            const int b = __ffs(bits) - 1;
            bits &= bits - 1;
            out[pos++] = pc_lo + (uint32_t)(w * 32 + b);
        }
    }
}

template <int THREADS, int ITEMS, bool IDS>
static void launch_ids(int c, const uint64_t *off, const uint32_t *raw, uint32_t *out,
                       uint32_t *new_len, const uint32_t *lists, size_t stride,
                       const uint32_t *counts, const uint64_t *tab, uint32_t pc_lo,
                       uint64_t pc_span, const uint32_t *n_ids, uint32_t *pres, uint32_t *err,
                       size_t nseg, hipStream_t s) {
    const unsigned grid = (unsigned)std::min<size_t>(std::max<size_t>(nseg, 1), 16384);
    hipLaunchKernelGGL((canon_ids_kernel<THREADS, ITEMS, IDS>), dim3(grid), dim3(THREADS), 0, s, off,
                       raw, out, new_len, lists + (size_t)c * stride, counts + c, tab, pc_lo,
                       pc_span, n_ids, pres, err);
}

__global__ void canon_bin_kernel2(const uint64_t *__restrict__ off, size_t nseg,
                                  uint32_t *__restrict__ counts, uint32_t *__restrict__ lists,
                                  size_t list_stride) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nseg;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint64_t n = off[i + 1] - off[i];
        const int c = n <= 256 ? 0 : n <= 512 ? 1 : n <= 1024 ? 2 : n <= 2048 ? 3
                    : n <= 4096 ? 4 : n <= 8192 ? 5 : n <= 16384 ? 6 : 7;
        const uint32_t slot = atomicAdd(&counts[c], 1u);
        lists[(size_t)c * list_stride + slot] = (uint32_t)i;
    }
}

}  // namespace syz

using namespace syz;

// Shared driver of the two canonical forms: bin segments by raw length, one
// launch per size class, segments > 16384 through the generic large path.
template <bool IDS>
static int canon_keys(const uint64_t *off, const uint32_t *raw, uint32_t *out, uint32_t *new_len,
                      size_t nseg, size_t max_seg_len, const uint64_t *tab, uint32_t pc_lo,
                      uint64_t pc_span, const uint32_t *n_ids, uint32_t *pres, uint32_t *err_flag,
                      void *ws, hipStream_t s) {
    uint32_t *counts = (uint32_t *)ws;
    uint32_t *lists = (uint32_t *)((uint8_t *)ws + align_up(8 * sizeof(uint32_t), 256));
    SYZ_HIP(hipMemsetAsync(counts, 0, 8 * sizeof(uint32_t), s));
    hipLaunchKernelGGL(canon_bin_kernel2, dim3(grid_for(nseg, 256, 4096)), dim3(256), 0, s, off,
                       nseg, counts, lists, nseg);
#define SYZ_CLASS(c, T, I)                                                                      \
    launch_ids<T, I, IDS>(c, off, raw, out, new_len, lists, nseg, counts, tab, pc_lo, pc_span, \
                          n_ids, pres, err_flag, nseg, s)
    SYZ_CLASS(0, 64, 4);
    if (max_seg_len > 256) SYZ_CLASS(1, 64, 8);
    if (max_seg_len > 512) SYZ_CLASS(2, 128, 8);
    if (max_seg_len > 1024) SYZ_CLASS(3, 256, 8);
    if (max_seg_len > 2048) SYZ_CLASS(4, 256, 16);
    if (max_seg_len > 4096) SYZ_CLASS(5, 512, 16);
    if (max_seg_len > 8192) SYZ_CLASS(6, 1024, 16);
#undef SYZ_CLASS
    SYZ_LAUNCH_CHECK();
    if (max_seg_len > 16384) {
        uint32_t nlarge = 0;
        SYZ_HIP(hipMemcpyAsync(&nlarge, counts + 7, 4, hipMemcpyDeviceToHost, s));
        SYZ_HIP(hipStreamSynchronize(s));
        if (nlarge) {
            const uint32_t *dl = lists + 7 * nseg;
            int rc = canon_large_path(off, raw, out, new_len, dl, nlarge, nullptr, pc_lo, pc_span,
                                      err_flag, s);
            if (rc) return rc;
            if (IDS)
                hipLaunchKernelGGL(pcs_to_ids_kernel, dim3(std::min<uint32_t>(nlarge, 4096)),
                                   dim3(256), 0, s, off, dl, nlarge, new_len, out, tab, pc_lo);
            else
                hipLaunchKernelGGL(mark_large_kernel, dim3(std::min<uint32_t>(nlarge, 4096)),
                                   dim3(256), 0, s, off, dl, nlarge, new_len, out, pres, pc_lo);
            SYZ_LAUNCH_CHECK();
        }
    }
    return 0;
}

extern "C" int syzcov_dev_canon_ids(const uint64_t *off, const uint32_t *raw, uint32_t *out_ids,
                                    uint32_t *new_len, size_t nseg, size_t max_seg_len,
                                    const uint64_t *tab, uint32_t pc_lo, uint64_t pc_span,
                                    const uint32_t *n_ids, uint32_t *err_flag, void *ws,
                                    size_t ws_size, void *stream) {
    if (nseg == 0) return 0;
    if (!off || !raw || !out_ids || !new_len || !tab || !n_ids || !err_flag || !ws)
        return SYZCOV_EINVAL;
    if (ws_size < syzcov_dev_canon_ws_size(nseg, max_seg_len)) return SYZCOV_EINVAL;
    if (out_ids == raw && max_seg_len > 16384) return SYZCOV_EINVAL;  // large path is out of place
    return canon_keys<true>(off, raw, out_ids, new_len, nseg, max_seg_len, tab, pc_lo, pc_span,
                            n_ids, nullptr, err_flag, ws, (hipStream_t)stream);
}

extern "C" int syzcov_dev_canon_pcs(const uint64_t *off, const uint32_t *raw, uint32_t *out_pcs,
                                    uint32_t *new_len, size_t nseg, size_t max_seg_len,
                                    uint32_t pc_lo, uint64_t pc_span, uint32_t *pres_bits,
                                    uint32_t *err_flag, void *ws, size_t ws_size, void *stream) {
    if (nseg == 0) return 0;
    if (!off || !raw || !out_pcs || !new_len || !pres_bits || !err_flag || !ws)
        return SYZCOV_EINVAL;
    if (pc_span == 0 || pc_span > (1ull << 32)) return SYZCOV_ERANGE;
    if (ws_size < syzcov_dev_canon_ws_size(nseg, max_seg_len)) return SYZCOV_EINVAL;
    if (out_pcs == raw && max_seg_len > 16384) return SYZCOV_EINVAL;
    return canon_keys<false>(off, raw, out_pcs, new_len, nseg, max_seg_len, nullptr, pc_lo,
                             pc_span, nullptr, pres_bits, err_flag, ws, (hipStream_t)stream);
}

extern "C" size_t syzcov_dev_minimize_win_ws_size(uint64_t pc_span) {
    return 2 * align_up((pc_span + 31) / 32 * 4, 256);
}

extern "C" int syzcov_dev_minimize_win(const uint64_t *off, const uint32_t *len,
                                       const uint32_t *pcs, const int32_t *order,
                                       const int32_t *ranks, size_t n, uint32_t pc_lo,
                                       uint64_t pc_span, int32_t *first_w, uint8_t *cand,
                                       uint8_t *kept, int do_pass2, void *ws, void *stream) {
    if (n == 0) return 0;
    if (!off || !len || !pcs || !order || !first_w || !cand || !ws || n > 0x7FFFFFFF)
        return SYZCOV_EINVAL;
    if (do_pass2 && !kept) return SYZCOV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const uint64_t nwords = (pc_span + 31) / 32;
    const size_t half = align_up(nwords * 4, 256);
    uint32_t *covered = (uint32_t *)ws;
    uint32_t *touched = (uint32_t *)((uint8_t *)ws + half);
    SYZ_HIP(hipMemsetAsync(ws, 0, 2 * half, s));
    const unsigned grid = 2048;
    uint64_t j0 = 0, step = 4096;
    while (j0 < n) {
        const uint64_t j1 = std::min<uint64_t>(n, j0 + step);
        hipLaunchKernelGGL(mini_win_pass1_kernel, dim3((unsigned)std::min<uint64_t>(grid, j1 - j0)),
                           dim3(MI_THREADS), 0, s, off, len, pcs, order, ranks, (uint32_t)j0,
                           (uint32_t)j1, pc_lo, (const uint32_t *)covered, touched, first_w, cand);
        j0 = j1;
        step *= 2;
        if (j0 < n)
            hipLaunchKernelGGL(or_words_kernel, dim3(grid_for(nwords, 256, 4096)), dim3(256), 0, s,
                               covered, (const uint32_t *)touched, nwords);
    }
    SYZ_LAUNCH_CHECK();
    if (do_pass2) {
        hipLaunchKernelGGL(mini_win_pass2_kernel, dim3((unsigned)std::min<size_t>(n, 2048)),
                           dim3(MI_THREADS), 0, s, off, len, pcs, order, ranks, (uint32_t)n, pc_lo,
                           (const int32_t *)first_w, (const uint8_t *)cand, kept);
        SYZ_LAUNCH_CHECK();
    }
    return 0;
}

extern "C" int syzcov_dev_minimize_win_pass2(const uint64_t *off, const uint32_t *len,
                                             const uint32_t *pcs, const int32_t *order,
                                             const int32_t *ranks, size_t n, uint32_t pc_lo,
                                             const int32_t *first_w, const uint8_t *cand,
                                             uint8_t *kept, void *stream) {
    if (n == 0) return 0;
    if (!off || !len || !pcs || !order || !first_w || !cand || !kept) return SYZCOV_EINVAL;
    hipLaunchKernelGGL(mini_win_pass2_kernel, dim3((unsigned)std::min<size_t>(n, 2048)),
                       dim3(MI_THREADS), 0, (hipStream_t)stream, off, len, pcs, order, ranks,
                       (uint32_t)n, pc_lo, first_w, cand, kept);
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" int syzcov_dev_first_dense(const uint64_t *tab, uint64_t pc_span, int32_t *first_w,
                                      int32_t *dense, int to_dense, void *stream) {
    if (!tab || !first_w || !dense || pc_span == 0) return SYZCOV_EINVAL;
    const uint64_t nwords = (pc_span + 31) / 32;
    hipLaunchKernelGGL(first_dense_kernel, dim3(grid_for(nwords, 256, 16384)), dim3(256), 0,
                       (hipStream_t)stream, tab, nwords, first_w, dense, to_dense);
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" size_t syzcov_dev_minimize_ws_size(size_t n_ids_cap) {
    return align_up((n_ids_cap + 31) / 32 * 4, 256);
}

extern "C" int syzcov_dev_minimize_ids(const uint64_t *off, const uint32_t *len,
                                       const uint32_t *ids, const int32_t *order,
                                       const int32_t *ranks, size_t n, const uint32_t *n_ids,
                                       size_t n_ids_cap, int32_t *first, uint8_t *cand,
                                       uint8_t *kept, int do_pass2, void *ws, void *stream) {
    if (n == 0) return 0;
    if (!off || !len || !ids || !order || !n_ids || !first || !cand || !ws || n > 0x7FFFFFFF)
        return SYZCOV_EINVAL;
    if (do_pass2 && !kept) return SYZCOV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const uint32_t nwords = (uint32_t)((n_ids_cap + 31) / 32);
    uint32_t *covered = (uint32_t *)ws;
    SYZ_HIP(hipMemsetAsync(covered, 0, (size_t)nwords * 4, s));
    const unsigned grid = 2048;
    // chunk 0 without filter, then doubling chunks with the covered filter
    uint64_t j0 = 0, step = 4096;
    while (j0 < n) {
        const uint64_t j1 = std::min<uint64_t>(n, j0 + step);
        hipLaunchKernelGGL(mini_ids_pass1_kernel, dim3((unsigned)std::min<uint64_t>(grid, j1 - j0)),
                           dim3(MI_THREADS), 0, s, off, len, ids, order, ranks, (uint32_t)j0,
                           (uint32_t)j1, j0 ? (const uint32_t *)covered : nullptr, first, cand);
        j0 = j1;
        step *= 2;
        if (j0 < n)
            hipLaunchKernelGGL(covered_update_kernel, dim3(grid_for(nwords, 256, 4096)), dim3(256), 0,
                               s, first, n_ids, nwords, covered);
    }
    SYZ_LAUNCH_CHECK();
    if (do_pass2) {
        hipLaunchKernelGGL(mini_ids_pass2_kernel, dim3((unsigned)std::min<size_t>(n, 2048)),
                           dim3(MI_THREADS), 0, s, off, len, ids, order, ranks, (uint32_t)n, first,
                           cand, kept);
        SYZ_LAUNCH_CHECK();
    }
    return 0;
}

extern "C" int syzcov_dev_minimize_ids_pass2(const uint64_t *off, const uint32_t *len,
                                             const uint32_t *ids, const int32_t *order,
                                             const int32_t *ranks, size_t n, const int32_t *first,
                                             const uint8_t *cand, uint8_t *kept, void *stream) {
    if (n == 0) return 0;
    if (!off || !len || !ids || !order || !first || !cand || !kept) return SYZCOV_EINVAL;
    hipLaunchKernelGGL(mini_ids_pass2_kernel, dim3((unsigned)std::min<size_t>(n, 2048)),
                       dim3(MI_THREADS), 0, (hipStream_t)stream, off, len, ids, order, ranks,
                       (uint32_t)n, first, cand, kept);
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" int syzcov_dev_dict_pcs(const uint64_t *tab, uint64_t pc_span, uint32_t pc_lo,
                                   uint32_t *out, void *stream) {
    if (!tab || !out || pc_span == 0) return SYZCOV_EINVAL;
    const uint64_t nwords = (pc_span + 31) / 32;
    hipLaunchKernelGGL(dict_pcs_kernel, dim3(grid_for(nwords, 256, 16384)), dim3(256), 0,
                       (hipStream_t)stream, tab, nwords, pc_lo, out);
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" int syzcov_dev_gather_u32(const uint32_t *table, const uint64_t *off,
                                     const uint32_t *len, const uint32_t *in, size_t nseg,
                                     uint32_t *out, void *stream) {
    if (nseg == 0) return 0;
    if (!table || !off || !len || !in || !out) return SYZCOV_EINVAL;
    hipLaunchKernelGGL(gather_u32_kernel, dim3(grid_for(nseg, 1, 16384)), dim3(256), 0,
                       (hipStream_t)stream, table, off, len, in, nseg, out);
    SYZ_LAUNCH_CHECK();
    return 0;
}
