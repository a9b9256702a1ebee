// setops.hip — cover.Difference / SymmetricDifference / Union / Intersection
// (cover/cover.go:42-102) for gfx950.
//
// foreach (cover.go:81-102) is a two-pointer merge that advances both sides
// on equal heads.  For operands sorted non-decreasing that is multiset
// algebra on value counts ca(x), cb(x):
//   Union max(ca,cb) · Intersection min(ca,cb) · Difference (ca-cb)+ ·
//   SymmetricDifference |ca-cb|,  and 0xFFFFFFFF never survives (f's `sent`
//   result is dropped, :97).
// Fully parallel form: every element finds its run in the other operand by
// binary search, decides from its occurrence index whether it is emitted,
// and lands at its position in the stable merge (a before b on ties); an
// ordered compaction of the emitted slots yields foreach's exact output.
#include "common.h"

namespace syz {

__device__ __forceinline__ uint64_t lower_bound(const uint32_t *__restrict__ x, uint64_t n,
                                                uint32_t v) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        uint64_t m = (lo + hi) >> 1;
        if (x[m] < v)
            lo = m + 1;
        else
            hi = m;
    }
    return lo;
}

__device__ __forceinline__ uint64_t upper_bound(const uint32_t *__restrict__ x, uint64_t n,
                                                uint32_t v) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        uint64_t m = (lo + hi) >> 1;
        if (x[m] <= v)
            lo = m + 1;
        else
            hi = m;
    }
    return lo;
}

// op: 0 Difference, 1 SymmetricDifference, 2 Union, 3 Intersection
__global__ void setop_place_kernel(int op, const uint32_t *__restrict__ a, uint64_t na,
                                   const uint32_t *__restrict__ b, uint64_t nb,
                                   uint8_t *__restrict__ flag, uint32_t *__restrict__ val,
                                   uint32_t *__restrict__ err) {
    const uint64_t total = na + nb;
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (uint64_t)gridDim.x * blockDim.x) {
        if (e < na) {
            const uint64_t i = e;
            const uint32_t x = a[i];
            if (i > 0 && a[i - 1] > x) *err = 1u;
            const uint64_t occ = i - lower_bound(a, na, x);
            const uint64_t lb = lower_bound(b, nb, x);
            const uint64_t cnt = upper_bound(b, nb, x) - lb;
            bool emit;
            switch (op) {
            case 0: emit = occ >= cnt; break;
            case 1: emit = occ >= cnt; break;
            case 2: emit = true; break;
            default: emit = occ < cnt; break;
            }
            const uint64_t pos = i + lb;
            flag[pos] = emit && x != SYZ_SENT;
            val[pos] = x;
        } else {
            const uint64_t j = e - na;
            const uint32_t x = b[j];
            if (j > 0 && b[j - 1] > x) *err = 1u;
            const uint64_t occ = j - lower_bound(b, nb, x);
            const uint64_t ub = upper_bound(a, na, x);
            const uint64_t cnt = ub - lower_bound(a, na, x);
            const bool emit = (op == 1 || op == 2) && occ >= cnt;
            const uint64_t pos = j + ub;
            flag[pos] = emit && x != SYZ_SENT;
            val[pos] = x;
        }
    }
}

}  // namespace syz

using namespace syz;

extern "C" int syzcov_dev_compact_kept(const uint8_t *kept, const int32_t *order, size_t n,
                                       int32_t *out_idx, uint32_t *n_out, void *ws, void *stream);
extern "C" size_t syzcov_dev_compact_ws_size(size_t n);

namespace syz {
// Device-level set op: a, b, out device pointers; ws >= setop_ws_size(na+nb).
size_t setop_ws_size(size_t ntot) {
    return align_up(ntot + 1, 256) + align_up((ntot + 1) * 4, 256) + align_up(4, 256) +
           syzcov_dev_compact_ws_size(ntot + 1);
}

int dev_setop(int op, const uint32_t *a, size_t na, const uint32_t *b, size_t nb, uint32_t *out,
              uint32_t *n_out, uint32_t *err, void *ws, hipStream_t s) {
    const size_t ntot = na + nb;
    uint8_t *w = (uint8_t *)ws;
    uint8_t *flag = w;
    uint32_t *val = (uint32_t *)(w + align_up(ntot + 1, 256));
    void *cws = (uint8_t *)val + align_up((ntot + 1) * 4, 256) + align_up(4, 256);
    if (ntot == 0) {
        SYZ_HIP(hipMemsetAsync(n_out, 0, sizeof(uint32_t), s));
        return 0;
    }
    hipLaunchKernelGGL(setop_place_kernel, dim3(grid_for(ntot, 256, 8192)), dim3(256), 0, s, op, a,
                       (uint64_t)na, b, (uint64_t)nb, flag, val, err);
    SYZ_LAUNCH_CHECK();
    return syzcov_dev_compact_kept(flag, (const int32_t *)val, ntot, (int32_t *)out, n_out, cws,
                                   s);
}
}  // namespace syz
