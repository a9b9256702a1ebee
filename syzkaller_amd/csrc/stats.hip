// stats.hip — the manager UI's coverage statistics (syz-manager/html.go).
//
// uniqueCover (html.go:213-238) counts, per PC, how often the corpus holds it
// and keeps the PCs counted exactly once:
//   perCall = false: every occurrence counts (duplicates inside one cover too,
//                    :224-230 iterate inp.Cover as given);
//   perCall = true:  a (call, pc) pair counts once (:220-228), so a PC is
//                    unique iff exactly one call group holds it.
// Over the corpus' dense id space (dict.hip): perCall = false is a
// saturating per-id counter; perCall = true keeps the first call seen per id
// (atomicCAS) and a "second call" mark.  The selected ids are compacted in id
// order, i.e. sorted PC order, which is the reference's final Canonicalize.
#include "common.h"

namespace syz {

constexpr int32_t UC_NONE = INT32_MIN;  // no call seen yet (call keys must differ)

__global__ __launch_bounds__(256) void uc_count_kernel(const uint64_t *__restrict__ off,
                                                       const uint32_t *__restrict__ pcs, uint32_t n,
                                                       const int32_t *__restrict__ call,
                                                       const uint64_t *__restrict__ tab,
                                                       uint32_t pc_lo, uint32_t *__restrict__ cnt,
                                                       int32_t *__restrict__ owner) {
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        const uint64_t b = off[i], l = off[i + 1] - b;
        const int32_t c = call ? call[i] : 0;
        for (uint64_t k = threadIdx.x; k < l; k += blockDim.x) {
            const uint32_t id = dense_id(tab, pcs[b + k], pc_lo);
            if (!call) {
                if (cnt[id] < 2) atomicAdd(&cnt[id], 1u);  // 0, 1 or "more"
            } else if (cnt[id] < 2) {
                const int32_t o = owner[id];
                if (o == c) continue;
                const int32_t prev = o == UC_NONE ? atomicCAS(&owner[id], UC_NONE, c) : o;
                if (prev != UC_NONE && prev != c) cnt[id] = 2;  // a second call group
            }
        }
    }
}

// flag[id] = id is unique; pc_of[id] = its PC (the dictionary inverted)
__global__ void uc_select_kernel(const uint64_t *__restrict__ tab, uint64_t nwords, uint32_t pc_lo,
                                 const uint32_t *__restrict__ cnt, const int32_t *__restrict__ owner,
                                 int per_call, uint8_t *__restrict__ flag,
                                 int32_t *__restrict__ pc_of) {
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords;
         w += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t e = tab[w];
        uint32_t bits = (uint32_t)(e >> 32), id = (uint32_t)e;
        while (bits) {
            const uint32_t b = (uint32_t)__builtin_ctz(bits);
            bits &= bits - 1;
            pc_of[id] = (int32_t)(pc_lo + (uint32_t)(w * 32 + b));
            flag[id] = per_call ? (owner[id] != UC_NONE && cnt[id] < 2) : (cnt[id] == 1);
            id++;
        }
    }
}

int unique_cover_launch(const uint64_t *off, const uint32_t *pcs, uint32_t n, const int32_t *call,
                        const uint64_t *tab, uint64_t span, uint32_t pc_lo, uint32_t nids,
                        uint32_t *cnt, int32_t *owner, uint8_t *flag, int32_t *pc_of,
                        hipStream_t s) {
    SYZ_HIP(hipMemsetAsync(cnt, 0, (size_t)nids * 4 + 4, s));
    SYZ_HIP(hipMemsetD32Async((hipDeviceptr_t)owner, (int)UC_NONE, (size_t)nids + 1, s));
    hipLaunchKernelGGL(uc_count_kernel, dim3(grid_for(n, 1, 8192)), dim3(256), 0, s, off, pcs, n,
                       call, tab, pc_lo, cnt, owner);
    const uint64_t nwords = (span + 31) / 32;
    hipLaunchKernelGGL(uc_select_kernel, dim3(grid_for(nwords, 256, 16384)), dim3(256), 0, s, tab,
                       nwords, pc_lo, (const uint32_t *)cnt, (const int32_t *)owner,
                       call ? 1 : 0, flag, pc_of);
    SYZ_LAUNCH_CHECK();
    return 0;
}

}  // namespace syz
