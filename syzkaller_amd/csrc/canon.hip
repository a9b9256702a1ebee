// canon.hip — segmented cover.Canonicalize (cover/cover.go:27-40) for gfx950.
//
// Each CSR segment (one raw KCOV cover) is sorted and de-duplicated by ONE
// workgroup, entirely on chip: a bitonic network whose short strides run in
// registers (blocked arrangement, ITEMS consecutive keys per lane), whose
// in-wave strides are lane exchanges (__shfl_xor -> ds_bpermute/DPP) and only
// whose cross-wave strides touch LDS.  Keys are staged through LDS once in and
// once out so both global streams are coalesced.  Unique keeps the
// reference's `last := sent` quirk (a leading 0xFFFFFFFF is only possible
// when every key is 0xFFFFFFFF, and is then dropped).  The canonical list is
// written to out[off[i] ..) (same CSR slots: the device analogue of the
// reference's in-place cov[:i]), and optionally each kept PC is marked in a
// uint8 presence map over the PC window (test-then-store: idempotent, no
// atomics) for the dense-id dictionary.
//
// Segments are binned by length into power-of-two capacity classes so each
// class runs a kernel whose CAP = THREADS*ITEMS fits the segment; segments
// longer than 16384 keys take the multi-pass path (chunk sort + merge-path
// merges in global memory + segment-level unique).
#include "common.h"

#include <algorithm>
#include <cstdlib>

namespace syz {

enum { NCLASS = 7, CLASS_LARGE = 7, LARGE_CHUNK = 16384 };
// class c handles n <= 256 << c
__host__ __device__ inline int len_class(uint64_t n) {
    if (n <= 256) return 0;
    if (n <= 512) return 1;
    if (n <= 1024) return 2;
    if (n <= 2048) return 3;
    if (n <= 4096) return 4;
    if (n <= 8192) return 5;
    if (n <= 16384) return 6;
    return CLASS_LARGE;
}

// ------------------------------------------------------------------ binning
__global__ void canon_bin_kernel(const uint64_t *__restrict__ off, size_t nseg,
                                 uint32_t *__restrict__ counts, uint32_t *__restrict__ lists,
                                 size_t list_stride) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i < nseg; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t n = off[i + 1] - off[i];
        int c = len_class(n);
        uint32_t slot = atomicAdd(&counts[c], 1u);
        lists[(size_t)c * list_stride + slot] = (uint32_t)i;
    }
}

// ---------------------------------------------------------- bitonic network
template <int THREADS, int ITEMS>
__device__ __forceinline__ void bitonic_sort(uint32_t (&v)[ITEMS], uint32_t *sm) {
    constexpr int CAP = THREADS * ITEMS;
    const uint32_t t = threadIdx.x;
#pragma unroll
    for (int k = 2; k <= CAP; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j < ITEMS) {
                // in-register compare-exchange
#pragma unroll
                for (int i = 0; i < ITEMS; i++) {
                    if ((i & j) == 0) {
                        const uint32_t e = t * ITEMS + i;
                        const bool asc = (e & k) == 0;
                        uint32_t a = v[i], b = v[i | j];
                        uint32_t lo = min(a, b), hi = max(a, b);
                        v[i] = asc ? lo : hi;
                        v[i | j] = asc ? hi : lo;
                    }
                }
            } else if (j < ITEMS * 64) {
                // partner lane t ^ m, same register slot
                const int m = j / ITEMS;
                const bool lower = (t & m) == 0;
                const bool asc = ((t * ITEMS) & k) == 0;
                const bool keep_min = lower == asc;
#pragma unroll
                for (int i = 0; i < ITEMS; i++) {
                    uint32_t p = __shfl_xor(v[i], m, 64);
                    v[i] = keep_min ? min(v[i], p) : max(v[i], p);
                }
            } else {
                // cross-wave stride: exchange through LDS
#pragma unroll
                for (int i = 0; i < ITEMS; i++) sm[t * ITEMS + i] = v[i];
                __syncthreads();
                const uint32_t m = (uint32_t)(j / ITEMS);
                const bool lower = (t & m) == 0;
                const bool asc = ((t * ITEMS) & k) == 0;
                const bool keep_min = lower == asc;
#pragma unroll
                for (int i = 0; i < ITEMS; i++) {
                    uint32_t p = sm[(t ^ m) * ITEMS + i];
                    v[i] = keep_min ? min(v[i], p) : max(v[i], p);
                }
                __syncthreads();
            }
        }
    }
}

__device__ __forceinline__ void mark_pc(uint8_t *__restrict__ pres, uint32_t pc, uint32_t pc_lo,
                                        uint64_t pc_span, uint32_t *__restrict__ err) {
    uint64_t o = (uint64_t)(uint32_t)(pc - pc_lo);
    if (pc < pc_lo || o >= pc_span) {
        *err = 1u;  // benign race: any writer sets 1
        return;
    }
    if (pres[o] == 0) pres[o] = 1;
}

// One segment per workgroup iteration.  SORT_ONLY: write the sorted keys of
// the whole CAP-wide chunk (padding included) to out_chunk (large path).
template <int THREADS, int ITEMS>
__global__ __launch_bounds__(THREADS) void canon_class_kernel(
    const uint64_t *__restrict__ off, const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
    uint32_t *__restrict__ new_len, const uint32_t *__restrict__ list,
    const uint32_t *__restrict__ count, uint8_t *__restrict__ pres, uint32_t pc_lo,
    uint64_t pc_span, uint32_t *__restrict__ err, uint32_t ak = 0) {
    constexpr int CAP = THREADS * ITEMS;
    __shared__ uint32_t sm[CAP];
    __shared__ uint32_t scan_tmp[THREADS / 64 + 1];
    const uint32_t t = threadIdx.x;
    const uint32_t nlist = *count;
    for (uint32_t li = blockIdx.x; li < nlist; li += gridDim.x) {
        const uint32_t seg = list[li];
        const uint64_t base = off[seg];
        if (off[seg + 1] - base > (uint64_t)CAP) continue;  // belongs to the large path
        const uint32_t n = (uint32_t)(off[seg + 1] - base);
        // coalesced striped load -> LDS -> blocked registers
        for (uint32_t k = t; k < (uint32_t)CAP; k += THREADS) sm[k] = k < n ? in[base + k] : SYZ_SENT;
        __syncthreads();
        uint32_t v[ITEMS];
#pragma unroll
        for (int i = 0; i < ITEMS; i++) v[i] = sm[t * ITEMS + i];
        __syncthreads();
        bitonic_sort<THREADS, ITEMS>(v, sm);
        // unique (cover.go:30-37): keep e < n && v != prev (prev of e=0 is sent)
#pragma unroll
        for (int i = 0; i < ITEMS; i++) sm[t * ITEMS + i] = v[i];
        __syncthreads();
        uint32_t keepmask = 0, cnt = 0;
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            const uint32_t e = t * ITEMS + i;
            const uint32_t prev = e == 0 ? SYZ_SENT : (i == 0 ? sm[e - 1] : v[i - 1]);
            const bool keep = e < n && v[i] != prev;
            keepmask |= (uint32_t)keep << i;
            cnt += keep;
        }
        uint32_t total;
        uint32_t pos = block_excl_scan<THREADS>(cnt, scan_tmp, &total);  // has barriers
#pragma unroll
        for (int i = 0; i < ITEMS; i++)
            if (keepmask & (1u << i)) sm[pos++] = v[i];
        __syncthreads();
        // (ak: contiguous at the input's line-aligned base, common.h; the
        // caller spreads the ranges' sub-runs apart once their splits are known)
        uint32_t *o = out + aligned_base(base, seg, ak);
        for (uint32_t k = t; k < total; k += THREADS) {
            const uint32_t pc = sm[k];
            o[k] = pc;
            if (pres) mark_pc(pres, pc, pc_lo, pc_span, err);
        }
        if (t == 0) new_len[seg] = total;
        __syncthreads();
    }
}

// ------------------------------------------------------------- large path
// (1) sort every LARGE_CHUNK-wide chunk of every large segment into scratch.
template <int THREADS, int ITEMS>
__global__ __launch_bounds__(THREADS) void large_chunk_sort_kernel(
    const uint64_t *__restrict__ off, const uint32_t *__restrict__ in,
    const uint32_t *__restrict__ list, const uint32_t *__restrict__ count,
    const uint64_t *__restrict__ scratch_off, uint32_t *__restrict__ scratch) {
    constexpr int CAP = THREADS * ITEMS;
    __shared__ uint32_t sm[CAP];
    const uint32_t t = threadIdx.x;
    const uint32_t nlist = *count;
    // work items: (list entry, chunk) flattened; chunk counts are per segment,
    // so walk segments and their chunks with a grid-stride over a global chunk id
    for (uint32_t li = 0; li < nlist; li++) {
        const uint32_t seg = list[li];
        const uint64_t base = off[seg];
        const uint64_t n = off[seg + 1] - base;
        const uint64_t nchunks = (n + CAP - 1) / CAP;
        for (uint64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
            const uint64_t cb = c * CAP;
            for (uint32_t k = t; k < (uint32_t)CAP; k += THREADS)
                sm[k] = (cb + k < n) ? in[base + cb + k] : SYZ_SENT;
            __syncthreads();
            uint32_t v[ITEMS];
#pragma unroll
            for (int i = 0; i < ITEMS; i++) v[i] = sm[t * ITEMS + i];
            __syncthreads();
            bitonic_sort<THREADS, ITEMS>(v, sm);
#pragma unroll
            for (int i = 0; i < ITEMS; i++) sm[t * ITEMS + i] = v[i];
            __syncthreads();
            const uint64_t sb = scratch_off[li] + cb;
            for (uint32_t k = t; k < (uint32_t)CAP; k += THREADS)
                if (cb + k < n) scratch[sb + k] = sm[k];
            __syncthreads();
        }
    }
}

// (2) merge pass: within every large segment, merge adjacent sorted runs of
// width w into runs of 2w.  One thread per output element, co-rank search.
__global__ void large_merge_kernel(const uint64_t *__restrict__ seg_len,
                                   const uint64_t *__restrict__ scratch_off, uint32_t nlarge,
                                   const uint32_t *__restrict__ src, uint32_t *__restrict__ dst,
                                   uint64_t w) {
    for (uint32_t li = 0; li < nlarge; li++) {
        const uint64_t n = seg_len[li];
        const uint32_t *s = src + scratch_off[li];
        uint32_t *d = dst + scratch_off[li];
        for (uint64_t o = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; o < n;
             o += (uint64_t)gridDim.x * blockDim.x) {
            const uint64_t pb = o / (2 * w) * (2 * w);
            const uint64_t na = (pb + w < n) ? w : n - pb;
            const uint64_t nb = (pb + w < n) ? ((pb + 2 * w <= n) ? w : n - pb - w) : 0;
            const uint32_t *A = s + pb, *B = s + pb + na;
            const uint64_t dd = o - pb;  // diagonal
            // co-rank: smallest i with i + j = dd such that A[i] > B[j-1] ... (stable: A first on ties)
            uint64_t lo = dd > nb ? dd - nb : 0, hi = dd < na ? dd : na;
            while (lo < hi) {
                uint64_t i = (lo + hi) >> 1;
                uint64_t j = dd - i;
                // take more from A if A[i] <= B[j-1]
                if (j > 0 && i < na && A[i] <= B[j - 1])
                    lo = i + 1;
                else
                    hi = i;
            }
            const uint64_t i = lo, j = dd - lo;
            uint32_t val;
            if (i < na && (j >= nb || A[i] <= B[j]))
                val = A[i];
            else
                val = B[j];
            d[o] = val;
        }
    }
}

// (3) unique + compact + mark for each large segment; one workgroup walks a
// segment in chunks, carrying the output position.
__global__ __launch_bounds__(256) void large_unique_kernel(
    const uint64_t *__restrict__ off, const uint32_t *__restrict__ list, uint32_t nlarge,
    const uint64_t *__restrict__ scratch_off, const uint32_t *__restrict__ sorted,
    uint32_t *__restrict__ out, uint32_t *__restrict__ new_len, uint8_t *__restrict__ pres,
    uint32_t pc_lo, uint64_t pc_span, uint32_t *__restrict__ err, uint32_t ak) {
    __shared__ uint32_t scan_tmp[256 / 64 + 1];
    for (uint32_t li = blockIdx.x; li < nlarge; li += gridDim.x) {
        const uint32_t seg = list[li];
        const uint64_t base = aligned_base(off[seg], seg, ak);
        const uint64_t n = off[seg + 1] - off[seg];
        const uint32_t *s = sorted + scratch_off[li];
        uint64_t wpos = 0;
        for (uint64_t cb = 0; cb < n; cb += 256) {
            const uint64_t e = cb + threadIdx.x;
            bool keep = false;
            uint32_t v = 0;
            if (e < n) {
                v = s[e];
                const uint32_t prev = e == 0 ? SYZ_SENT : s[e - 1];
                keep = v != prev;
            }
            uint32_t total;
            uint32_t p = block_excl_scan<256>(keep ? 1u : 0u, scan_tmp, &total);
            if (keep) {
                out[base + wpos + p] = v;
                if (pres) mark_pc(pres, v, pc_lo, pc_span, err);
            }
            wpos += total;
        }
        if (threadIdx.x == 0) new_len[seg] = (uint32_t)wpos;
    }
}

template <int THREADS, int ITEMS>
static int launch_class(int c, const uint64_t *off, const uint32_t *in, uint32_t *out,
                        uint32_t *new_len, const uint32_t *lists, size_t stride,
                        const uint32_t *counts, uint8_t *pres, uint32_t pc_lo, uint64_t pc_span,
                        uint32_t *err, size_t nseg_class_bound, hipStream_t s) {
    unsigned grid = (unsigned)std::min<size_t>(std::max<size_t>(nseg_class_bound, 1), 8192);
    hipLaunchKernelGGL((canon_class_kernel<THREADS, ITEMS>), dim3(grid), dim3(THREADS), 0, s, off,
                       in, out, new_len, lists + (size_t)c * stride, counts + c, pres, pc_lo,
                       pc_span, err);
    SYZ_LAUNCH_CHECK();
    return 0;
}

}  // namespace syz

using namespace syz;

// Workspace: counts[8] | lists[8][nseg].  The large-segment path allocates
// its own scratch (it is off the hot path: see syzcov_dev_canonicalize).
extern "C" size_t syzcov_dev_canon_ws_size(size_t nseg, size_t max_seg_len) {
    (void)max_seg_len;
    return align_up(8 * sizeof(uint32_t), 256) + align_up(8 * nseg * sizeof(uint32_t), 256);
}

namespace syz {
int canon_large_path(const uint64_t *off, const uint32_t *in, uint32_t *out, uint32_t *new_len,
                     const uint32_t *dlist, uint32_t nlarge, uint8_t *pres, uint32_t pc_lo,
                     uint64_t pc_span, uint32_t *err, hipStream_t s, uint32_t ak = 0);
}

extern "C" int syzcov_dev_canonicalize(const uint64_t *off, const uint32_t *in, uint32_t *out,
                                       uint32_t *new_len, size_t nseg, size_t max_seg_len,
                                       uint8_t *pres, uint32_t pc_lo, uint64_t pc_span,
                                       uint32_t *err_flag, void *ws, size_t ws_size,
                                       void *stream) {
    if (nseg == 0) return 0;
    if (!off || !in || !out || !new_len || !ws) return SYZCOV_EINVAL;
    if (ws_size < syzcov_dev_canon_ws_size(nseg, max_seg_len)) return SYZCOV_EINVAL;
    if (pres && !err_flag) return SYZCOV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    uint8_t *w = (uint8_t *)ws;
    uint32_t *counts = (uint32_t *)w;
    uint32_t *lists = (uint32_t *)(w + align_up(8 * sizeof(uint32_t), 256));
    SYZ_HIP(hipMemsetAsync(counts, 0, 8 * sizeof(uint32_t), s));
    hipLaunchKernelGGL(canon_bin_kernel, dim3(grid_for(nseg, 256, 4096)), dim3(256), 0, s, off,
                       nseg, counts, lists, nseg);
    SYZ_LAUNCH_CHECK();
    // Each class kernel is a grid-stride loop over its device-side list; the
    // grid is bounded by nseg so no host round trip is needed.
    int r = 0;
    r |= launch_class<64, 4>(0, off, in, out, new_len, lists, nseg, counts, pres, pc_lo, pc_span,
                             err_flag, nseg, s);
    if (max_seg_len > 256)
        r |= launch_class<64, 8>(1, off, in, out, new_len, lists, nseg, counts, pres, pc_lo,
                                 pc_span, err_flag, nseg, s);
    if (max_seg_len > 512)
        r |= launch_class<128, 8>(2, off, in, out, new_len, lists, nseg, counts, pres, pc_lo,
                                  pc_span, err_flag, nseg, s);
    if (max_seg_len > 1024)
        r |= launch_class<256, 8>(3, off, in, out, new_len, lists, nseg, counts, pres, pc_lo,
                                  pc_span, err_flag, nseg, s);
    if (max_seg_len > 2048)
        r |= launch_class<256, 16>(4, off, in, out, new_len, lists, nseg, counts, pres, pc_lo,
                                   pc_span, err_flag, nseg, s);
    if (max_seg_len > 4096)
        r |= launch_class<512, 16>(5, off, in, out, new_len, lists, nseg, counts, pres, pc_lo,
                                   pc_span, err_flag, nseg, s);
    if (max_seg_len > 8192)
        r |= launch_class<1024, 16>(6, off, in, out, new_len, lists, nseg, counts, pres, pc_lo,
                                    pc_span, err_flag, nseg, s);
    if (r) return SYZCOV_EHIP;
    if (max_seg_len > LARGE_CHUNK) {
        // Large segments are rare (KCOV caps a call at 65535 PCs; huge lists
        // only come through the single-list drop-in).  Their count is read
        // back once; this is the only host synchronisation in the call.
        uint32_t nlarge = 0;
        SYZ_HIP(hipMemcpyAsync(&nlarge, counts + CLASS_LARGE, sizeof(uint32_t),
                               hipMemcpyDeviceToHost, s));
        SYZ_HIP(hipStreamSynchronize(s));
        if (nlarge) {
            int rc = canon_large_path(off, in, out, new_len, lists + (size_t)CLASS_LARGE * nseg,
                                      nlarge, pres, pc_lo, pc_span, err_flag, s);
            if (rc) return rc;
        }
    }
    return 0;
}

namespace syz {
// Listed segments of up to 16384 keys (a device-side list and count), one
// workgroup each: the fallback of the wavefront canonicalizer (canon_wave.hip)
// for segments too long for a wave and for any segment whose wave sort failed
// its order check.  Longer listed segments are skipped (large path).
int canon_list_path(const uint64_t *off, const uint32_t *in, uint32_t *out, uint32_t *new_len,
                    const uint32_t *list, const uint32_t *count, hipStream_t s, uint32_t ak) {
    hipLaunchKernelGGL((canon_class_kernel<1024, 16>), dim3(256), dim3(1024), 0, s, off, in, out,
                       new_len, list, count, nullptr, 0u, (uint64_t)0, nullptr, ak);
    SYZ_LAUNCH_CHECK();
    return 0;
}

int canon_large_path(const uint64_t *off, const uint32_t *in, uint32_t *out, uint32_t *new_len,
                     const uint32_t *dlist, uint32_t nlarge, uint8_t *pres, uint32_t pc_lo,
                     uint64_t pc_span, uint32_t *err, hipStream_t s, uint32_t ak) {
    // host copies of the large-segment list and lengths (small)
    uint32_t *hlist = (uint32_t *)malloc(nlarge * sizeof(uint32_t));
    if (!hlist) return SYZCOV_ENOMEM;
    int rc = 0;
    uint64_t *hoff = nullptr, *hsoff = nullptr, *hlen = nullptr;
    void *dbuf = nullptr;
    do {
        if (hipMemcpyAsync(hlist, dlist, nlarge * sizeof(uint32_t), hipMemcpyDeviceToHost, s) !=
                hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            rc = SYZCOV_EHIP;
            break;
        }
        hoff = (uint64_t *)malloc(2 * sizeof(uint64_t));
        hsoff = (uint64_t *)malloc(nlarge * sizeof(uint64_t));
        hlen = (uint64_t *)malloc(nlarge * sizeof(uint64_t));
        uint64_t total = 0, maxn = 0;
        for (uint32_t i = 0; i < nlarge; i++) {
            if (hipMemcpy(hoff, off + hlist[i], 2 * sizeof(uint64_t), hipMemcpyDeviceToHost) !=
                hipSuccess) {
                rc = SYZCOV_EHIP;
                break;
            }
            hsoff[i] = total;
            hlen[i] = hoff[1] - hoff[0];
            total += hlen[i];
            if (hlen[i] > maxn) maxn = hlen[i];
        }
        if (rc) break;
        // device: [soff u64 x nlarge][len u64 x nlarge][A keys][B keys]
        size_t meta = align_up(2 * nlarge * sizeof(uint64_t), 256);
        if (hipMalloc(&dbuf, meta + 2 * align_up(total * sizeof(uint32_t), 256)) != hipSuccess) {
            rc = SYZCOV_ENOMEM;
            break;
        }
        uint64_t *dsoff = (uint64_t *)dbuf;
        uint64_t *dlen = dsoff + nlarge;
        uint32_t *A = (uint32_t *)((uint8_t *)dbuf + meta);
        uint32_t *B = (uint32_t *)((uint8_t *)A + align_up(total * sizeof(uint32_t), 256));
        if (hipMemcpyAsync(dsoff, hsoff, nlarge * sizeof(uint64_t), hipMemcpyHostToDevice, s) !=
                hipSuccess ||
            hipMemcpyAsync(dlen, hlen, nlarge * sizeof(uint64_t), hipMemcpyHostToDevice, s) !=
                hipSuccess) {
            rc = SYZCOV_EHIP;
            break;
        }
        uint32_t *dcount = nullptr;
        // count pointer for the chunk-sort kernel: reuse dlen region? pass a device copy
        if (hipMalloc(&dcount, sizeof(uint32_t)) != hipSuccess) {
            rc = SYZCOV_ENOMEM;
            break;
        }
        hipMemcpyAsync(dcount, &nlarge, sizeof(uint32_t), hipMemcpyHostToDevice, s);
        unsigned g = (unsigned)std::min<uint64_t>((maxn + LARGE_CHUNK - 1) / LARGE_CHUNK, 4096);
        hipLaunchKernelGGL((large_chunk_sort_kernel<1024, 16>), dim3(g), dim3(1024), 0, s, off, in,
                           dlist, dcount, dsoff, A);
        uint32_t *src = A, *dst = B;
        for (uint64_t w = LARGE_CHUNK; w < maxn; w *= 2) {
            hipLaunchKernelGGL(large_merge_kernel, dim3(grid_for(maxn, 256, 8192)), dim3(256), 0, s,
                               dlen, dsoff, nlarge, src, dst, w);
            uint32_t *tswap = src;
            src = dst;
            dst = tswap;
        }
        hipLaunchKernelGGL(large_unique_kernel, dim3(std::min<uint32_t>(nlarge, 1024)), dim3(256),
                           0, s, off, dlist, nlarge, dsoff, src, out, new_len, pres, pc_lo,
                           pc_span, err, ak);
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
            rc = SYZCOV_EHIP;
        hipFree(dcount);
    } while (0);
    if (dbuf) hipFree(dbuf);
    free(hlist);
    free(hoff);
    free(hsoff);
    free(hlen);
    return rc;
}
}  // namespace syz

