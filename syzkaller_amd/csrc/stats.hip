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

#include <algorithm>

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


// ---------------------------------------------------------------- UI stats
// httpSummary (html.go:67-99): per call group, len(Union of its covers) and
// len(Intersection(that union, uniqueCover(true))); httpCorpus (:157-175):
// per input, len(Intersection(inp.Cover, uniqueCover(false))).  Covers are
// canonical, so both are counts over dense ids; the sentinel PC (sent_id) is
// never counted, as Union/Intersection drop it (cover.go:97).

// presence slab of call groups [g0, g0 + gb): bits[(g - g0) * wpg + id / 32]
__global__ __launch_bounds__(256) void ui_call_bits_kernel(
    const uint64_t *__restrict__ off, const uint32_t *__restrict__ pcs, uint32_t n,
    const int32_t *__restrict__ call, const uint64_t *__restrict__ tab, uint32_t pc_lo,
    uint32_t sent_id, uint32_t g0, uint32_t gb, uint64_t wpg, uint32_t *__restrict__ bits) {
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        const uint32_t g = (uint32_t)call[i] - g0;
        if (g >= gb) continue;
        const uint64_t b = off[i], l = off[i + 1] - b;
        uint32_t *row = bits + (uint64_t)g * wpg;
        for (uint64_t k = threadIdx.x; k < l; k += blockDim.x) {
            const uint32_t id = dense_id(tab, pcs[b + k], pc_lo);
            if (id == sent_id) continue;
            const uint32_t m = 1u << (id & 31);
            if (!(row[id >> 5] & m)) atomicOr(&row[id >> 5], m);
        }
    }
}

// cover[g0 + g] = popcount of slab row g (one workgroup per row)
__global__ __launch_bounds__(256) void ui_popc_kernel(const uint32_t *__restrict__ bits,
                                                      uint64_t wpg, uint32_t *__restrict__ cover) {
    __shared__ uint32_t part[4];
    const uint32_t *row = bits + (uint64_t)blockIdx.x * wpg;
    uint32_t c = 0;
    for (uint64_t w = threadIdx.x; w < wpg; w += blockDim.x) c += __popc(row[w]);
    c = wave_sum(c);
    if (__lane_id() == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) cover[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

// flag_all[id] = the id is in uniqueCover(false); ucov[owner] += id is in
// uniqueCover(true) (its only group is `owner`)
__global__ void ui_unique_kernel(const uint32_t *__restrict__ cnt_all,
                                 const uint32_t *__restrict__ cnt_call,
                                 const int32_t *__restrict__ owner, uint32_t nids, uint32_t sent_id,
                                 uint8_t *__restrict__ flag_all, uint32_t *__restrict__ ucov) {
    for (uint32_t id = blockIdx.x * blockDim.x + threadIdx.x; id < nids;
         id += gridDim.x * blockDim.x) {
        const bool real = id != sent_id;
        flag_all[id] = real && cnt_all[id] == 1;
        if (ucov && real && owner[id] != UC_NONE && cnt_call[id] < 2)
            atomicAdd(&ucov[owner[id]], 1u);
    }
}

// out[i] = PCs of input i in uniqueCover(false) (one wavefront per input)
__global__ __launch_bounds__(256) void ui_input_unique_kernel(
    const uint64_t *__restrict__ off, const uint32_t *__restrict__ pcs, uint32_t n,
    const uint64_t *__restrict__ tab, uint32_t pc_lo, const uint8_t *__restrict__ flag_all,
    uint32_t *__restrict__ out) {
    const uint32_t nw = gridDim.x * (blockDim.x / 64);
    for (uint32_t i = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); i < n; i += nw) {
        const uint64_t b = off[i], l = off[i + 1] - b;
        uint32_t c = 0;
        for (uint64_t k = __lane_id(); k < l; k += 64) c += flag_all[dense_id(tab, pcs[b + k], pc_lo)];
        c = wave_sum(c);
        if (__lane_id() == 0) out[i] = c;
    }
}

int ui_stats_launch(const uint64_t *off, const uint32_t *pcs, uint32_t n, const int32_t *call,
                    uint32_t ncalls, const uint64_t *tab, uint32_t pc_lo, uint32_t nids,
                    uint32_t sent_id, uint32_t *cnt_all, int32_t *own_all, uint32_t *cnt_call,
                    int32_t *own_call, uint8_t *flag_all, uint32_t *slab, uint64_t slab_words,
                    uint32_t *cover, uint32_t *ucov, uint32_t *in_unique, hipStream_t s) {
    const unsigned gin = grid_for(n, 1, 8192);
    SYZ_HIP(hipMemsetAsync(cnt_all, 0, (size_t)nids * 4 + 4, s));
    hipLaunchKernelGGL(uc_count_kernel, dim3(gin), dim3(256), 0, s, off, pcs, n,
                       (const int32_t *)nullptr, tab, pc_lo, cnt_all, own_all);
    if (call) {
        SYZ_HIP(hipMemsetAsync(cnt_call, 0, (size_t)nids * 4 + 4, s));
        SYZ_HIP(hipMemsetD32Async((hipDeviceptr_t)own_call, (int)UC_NONE, (size_t)nids + 1, s));
        SYZ_HIP(hipMemsetAsync(ucov, 0, (size_t)ncalls * 4, s));
        hipLaunchKernelGGL(uc_count_kernel, dim3(gin), dim3(256), 0, s, off, pcs, n, call, tab,
                           pc_lo, cnt_call, own_call);
    }
    hipLaunchKernelGGL(ui_unique_kernel, dim3(grid_for(nids, 256, 8192)), dim3(256), 0, s,
                       (const uint32_t *)cnt_all, (const uint32_t *)cnt_call,
                       (const int32_t *)own_call, nids, sent_id, flag_all, call ? ucov : nullptr);
    hipLaunchKernelGGL(ui_input_unique_kernel, dim3(grid_for(n, 4, 8192)), dim3(256), 0, s, off,
                       pcs, n, tab, pc_lo, (const uint8_t *)flag_all, in_unique);
    if (call) {
        const uint64_t wpg = ((uint64_t)nids + 31) / 32;
        const uint32_t gb = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(ncalls, slab_words / wpg));
        for (uint32_t g0 = 0; g0 < ncalls; g0 += gb) {
            const uint32_t nb = std::min(gb, ncalls - g0);
            SYZ_HIP(hipMemsetAsync(slab, 0, (size_t)nb * wpg * 4, s));
            hipLaunchKernelGGL(ui_call_bits_kernel, dim3(gin), dim3(256), 0, s, off, pcs, n, call,
                               tab, pc_lo, sent_id, g0, nb, wpg, slab);
            hipLaunchKernelGGL(ui_popc_kernel, dim3(nb), dim3(256), 0, s, (const uint32_t *)slab,
                               wpg, cover + g0);
        }
    }
    SYZ_LAUNCH_CHECK();
    return 0;
}

}  // namespace syz
