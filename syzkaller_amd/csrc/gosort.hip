// gosort.hip — the processing order of cover.Minimize: Go's
// sort.Sort(minInputArray) (cover/cover.go:113; Less = len desc, :141-143).
//
// sort.Sort is not stable, so equal-length inputs are ordered by the exact
// swap sequence of Go's algorithm (pdqsort in Go >= 1.19, quickSort + gap-6
// ShellSort in Go 1.8-1.18).
//
// Go >= 1.19 (pdqsort, the default) runs on the GPU, level-synchronously:
// every round advances all live segments by one iteration of pdqsort's loop.
// Per segment the O(1) control steps (breakPatterns, choosePivot, the
// partitionEqual test) run in one lane; the O(n) steps are data-parallel:
// Hoare's partition pairs the k-th left-misplaced element with the k-th
// right-misplaced one, so both sides' ranks come from prefix sums and the m
// swaps run independently — exactly the swaps Go performs.  Segments of up to
// SMALL elements finish inside one workgroup in LDS; leaves of up to TINY
// elements run gosort_core.h's sequential loop in one lane.  Segments never
// touch anything outside [a, b) but the finished pivot at a-1, so their
// processing order does not change the result.
//
// Only Go >= 1.19's pdqsort is restated.  The legacy Go 1.8-1.18 quickSort
// order is not computed here (sort_variant 1 -> SYZCOV_EINVAL): a caller on
// an old Go passes its own sort.Sort order (`order` of syzcov_minimize), as
// the drop-in Go shim does anyway.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdint>
#include <vector>

#include "common.h"

#include <cstring>
#include <mutex>
#include <vector>
#include "gosort_core.h"

namespace syz {
namespace gsort {

#ifndef SYZ_GSORT_SMALL
#define SYZ_GSORT_SMALL 4096
#endif
constexpr int SMALL = SYZ_GSORT_SMALL;  // segment finished in one workgroup's LDS
#ifndef SYZ_GSORT_TINY
#define SYZ_GSORT_TINY 32
#endif
constexpr int TINY = SYZ_GSORT_TINY;  // leaf finished by one lane
static_assert(TINY <= 64, "leaf pdqsort: BitStack holds 3 parked tasks of a <= 64-element leaf");
#ifndef SYZ_GSORT_SPLIT_MUL
#define SYZ_GSORT_SPLIT_MUL 4  // sharded order: split once >= this many large segments per part
#endif
constexpr int CH = 4096;     // elements per work item in the global rounds
constexpr unsigned ITEM_GRID = 1024;  // workgroups looping over a round's work items
constexpr int WG = 256;

struct Seg {
    int a, b, limit, flags;  // flags: bit0 wasBalanced, bit1 wasPartitioned
};
enum { M_DONE = 0, M_ACTIVE = 2 };
struct Plan {
    int mode, pivot, rev, pis, eq, cnt, m;
    uint32_t kp;
};

// accessor over the global key/index arrays
struct GAcc {
    uint32_t *K;
    int32_t *I;
    __device__ bool less(int i, int j) const { return K[i] > K[j]; }
    __device__ void swap(int i, int j) const {
        uint32_t k = K[i];
        K[i] = K[j];
        K[j] = k;
        int32_t x = I[i];
        I[i] = I[j];
        I[j] = x;
    }
};

// accessor over an LDS window holding global positions [base-1, base+len)
struct LAcc {
    uint32_t *K;  // K[g - base + 1]
    int32_t *I;
    int base;
    __device__ bool less(int i, int j) const { return K[i - base + 1] > K[j - base + 1]; }
    __device__ void swap(int i, int j) const {
        const int p = i - base + 1, q = j - base + 1;
        uint32_t k = K[p];
        K[p] = K[q];
        K[q] = k;
        int32_t x = I[p];
        I[p] = I[q];
        I[q] = x;
    }
};

struct Ctl {
    Seg *next;
    uint32_t *next_count, *next_maxlen;
    Seg *small;
    uint32_t *small_count;
    uint32_t small_cap, next_cap;
    uint32_t *err;
};

__device__ __forceinline__ void push_seg(const Ctl &c, Seg s) {
    const int n = s.b - s.a;
    if (n <= 1) return;
    if (n <= SMALL) {
        const uint32_t slot = atomicAdd(c.small_count, 1u);
        if (slot < c.small_cap)
            c.small[slot] = s;
        else
            *c.err = 2u;
    } else {
        const uint32_t slot = atomicAdd(c.next_count, 1u);
        if (slot < c.next_cap)
            c.next[slot] = s;
        else
            *c.err = 3u;
        atomicMax(c.next_maxlen, (uint32_t)n);
    }
}

__global__ void init_kernel(const int64_t *__restrict__ lens, uint32_t n, uint32_t *__restrict__ K,
                            int32_t *__restrict__ I, uint32_t *__restrict__ err) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int64_t l = lens[i];
        if (l < 0 || l > 0xFFFFFFFFll) *err = 1u;
        K[i] = (uint32_t)l;
        I[i] = (int32_t)i;
    }
}

__global__ void seed_kernel(uint32_t n, Ctl c) {
    push_seg(c, Seg{0, (int)n, gocore::bits_len(n), 3});
}

// Segmented form (one independent Go sort.Sort per group, as
// manager.minimizeCorpus runs cover.Minimize per call, manager.go:516-524):
// group g occupies positions [goff[g] + g, goff[g+1] + g) and the position
// after it holds a GAP key 0xFFFFFFFF.  pdqsort reads outside its segment
// only at a-1 (`a > 0 && !less(data[a-1], pivot)`, the partitionEqual test):
// at a group start that reads the gap, and less(gap, pivot) is true for every
// real length (< 0xFFFFFFFF), which is exactly the reference's a == 0 branch
// of a separate slice.  Gaps are never inside a segment, so never move.
__global__ void seg_init_kernel(const int64_t *__restrict__ lens, const uint64_t *__restrict__ goff,
                                uint32_t ngroups, uint32_t *__restrict__ K,
                                int32_t *__restrict__ I, uint32_t *__restrict__ err) {
    const uint32_t n = (uint32_t)goff[ngroups];
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        uint32_t lo = 0, hi = ngroups;  // group of i: last g with goff[g] <= i
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (goff[mid] <= i) lo = mid; else hi = mid;
        }
        const int64_t l = lens[i];
        if (l < 0 || l >= 0xFFFFFFFFll) *err = 1u;
        K[i + lo] = (uint32_t)l;
        I[i + lo] = (int32_t)i;
        if (i + 1 == goff[lo + 1] && lo + 1 < ngroups) {
            K[i + lo + 1] = 0xFFFFFFFFu;
            I[i + lo + 1] = -1;
        }
    }
}

__global__ void seg_seed_kernel(const uint64_t *__restrict__ goff, uint32_t ngroups, Ctl c) {
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < ngroups; g += gridDim.x * blockDim.x) {
        const uint32_t a = (uint32_t)goff[g] + g, b = (uint32_t)goff[g + 1] + g;
        push_seg(c, Seg{(int)a, (int)b, gocore::bits_len(b - a), 3});
    }
}

// order[p - g] = I[p] for every non-gap position p of group g (an element
// never leaves its group, so g is the group of the grouped index I[p])
__global__ void seg_gather_kernel(const int32_t *__restrict__ I, const uint64_t *__restrict__ goff,
                                  uint32_t ngroups, uint32_t npos, int32_t *__restrict__ order) {
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < npos; p += gridDim.x * blockDim.x) {
        const int32_t v = I[p];
        if (v < 0) continue;
        uint32_t lo = 0, hi = ngroups;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (goff[mid] <= (uint64_t)v) lo = mid; else hi = mid;
        }
        order[p - lo] = v;
    }
}

// WG-cooperative first index i in [from, b) with K[i] > K[i-1], or b
__device__ int wg_find_first_descent(const uint32_t *K, int from, int b, int *sh) {
    for (int c0 = from; c0 < b; c0 += WG) {
        const int i = c0 + threadIdx.x;
        const bool hit = i < b && K[i] > K[i - 1];
        const uint64_t m = __ballot(hit);
        if (__lane_id() == 0)
            sh[threadIdx.x >> 6] = m ? (int)(c0 + (threadIdx.x & ~63u) + __builtin_ctzll(m)) : b;
        __syncthreads();
        int best = b;
        for (int w = 0; w < WG / 64; w++) best = min(best, sh[w]);
        __syncthreads();
        if (best < b) return best;
    }
    return b;
}

// The control steps of one pdqsort loop iteration for each segment of the
// round, one workgroup per segment (gocore's sequential form, pdqsort in
// sort/zsortinterface.go): lane 0 runs the O(1) steps (breakPatterns,
// choosePivot; heapSort at limit 0), the workgroup reverses a decreasing
// segment and runs partialInsertionSort's scans, then lane 0 takes the
// partitionEqual test and the Swap(a, pivot) both partition forms start with.
// (Was three launches per round: plan, reverse, partial insertion sort.)
__global__ __launch_bounds__(WG) void lead_kernel(Seg *__restrict__ cur,
                                                   const uint32_t *__restrict__ ncur_p,
                                                   Plan *__restrict__ plan,
                                                   uint32_t *__restrict__ K,
                                                   int32_t *__restrict__ I, Ctl c,
                                                   uint32_t *__restrict__ items_cur,
                                                   uint32_t *__restrict__ items_next,
                                                   uint2 *__restrict__ items, uint32_t item_cap) {
    __shared__ int sh[WG / 64 + 2];
    __shared__ Plan sp;
    __shared__ uint32_t ibase;
    const uint32_t s = blockIdx.x;
    if (s == 0 && threadIdx.x == 0) {  // the children of this round are pushed by swap_kernel
        *c.next_count = 0u;
        *c.next_maxlen = 0u;
        *items_next = 0u;  // the next round's work items (this round's were zeroed before it)
    }
    if (s >= *ncur_p) return;
    Seg g = cur[s];
    const int a = g.a, b = g.b, n = b - a;
    GAcc d{K, I};
    if (threadIdx.x == 0) {
        Plan p{};
        if (n <= SMALL) {  // (only the seed can be small here)
            push_seg(c, g);
            p.mode = M_DONE;
        } else if (g.limit == 0) {  // `if limit == 0 { heapSort(data, a, b); return }`
            gocore::heap_sort(d, a, b);
            p.mode = M_DONE;
        } else {
            const bool wb = g.flags & 1, wp = g.flags & 2;
            if (!wb) {
                gocore::break_patterns(d, a, b);
                g.limit--;
                cur[s].limit = g.limit;
            }
            int hint;
            int pivot = gocore::choose_pivot(d, a, b, &hint);
            if (hint == gocore::kDecreasing) {
                p.rev = 1;
                pivot = (b - 1) - (pivot - a);
                hint = gocore::kIncreasing;
            }
            p.pis = wb && wp && hint == gocore::kIncreasing;
            p.pivot = pivot;
            p.mode = M_ACTIVE;
        }
        sp = p;
    }
    __threadfence_block();
    __syncthreads();
    Plan p = sp;
    if (p.mode == M_ACTIVE && p.rev) {  // reverseRange
        for (int i = threadIdx.x; i < n / 2; i += WG) d.swap(a + i, b - 1 - i);
        __threadfence_block();
        __syncthreads();
    }
    bool sorted = false;
    int i = a + 1;
    for (int step = 0; p.mode == M_ACTIVE && p.pis && step < 5; step++) {
        i = wg_find_first_descent(K, i, b, sh);
        if (i == b) {
            sorted = true;
            break;
        }
        if (n < 50) break;
        // the three moves of one step run on lane 0 (bounded by the segment)
        if (threadIdx.x == 0) {
            d.swap(i, i - 1);
            if (i - a >= 2)
                for (int j = i - 1; j >= 1 && d.less(j, j - 1); j--) d.swap(j, j - 1);
            if (b - i >= 2)
                for (int j = i + 1; j < b && d.less(j, j - 1); j++) d.swap(j, j - 1);
        }
        __threadfence_block();
        __syncthreads();
    }
    // the partition's work items: (segment, chunk of CH elements of (a, b))
    const uint32_t nch = (uint32_t)((n - 1 + CH - 1) / CH);
    if (threadIdx.x == 0) {
        if (p.mode == M_ACTIVE) {
            if (sorted) {
                p.mode = M_DONE;
            } else {
                // the partitionEqual test, then Swap(a, pivot) (lane 0 made the
                // moves above: no fence needed)
                p.eq = a > 0 && !d.less(a - 1, p.pivot);
                d.swap(a, p.pivot);
                p.kp = K[a];
            }
        }
        plan[s] = p;
        uint32_t b0 = item_cap;
        if (p.mode == M_ACTIVE) {
            b0 = atomicAdd(items_cur, nch);
            if (b0 + nch > item_cap) *c.err = 6u;
        }
        ibase = b0;
    }
    __syncthreads();
    const uint32_t b0 = ibase;
    if (b0 + nch <= item_cap)
        for (uint32_t j = threadIdx.x; j < nch; j += WG) items[b0 + j] = make_uint2(s, j);
}

// f(x): x belongs to the left group (partition: Less(x, a) = K[x] > kp;
// partitionEqual: !Less(a, x) = K[x] >= kp)
__device__ __forceinline__ bool left_group(uint32_t k, uint32_t kp, int eq) {
    return eq ? k >= kp : k > kp;
}

// count, rank and swap loop over the round's work items (lead_kernel's
// (segment, chunk) list) with a grid of at most ITEM_GRID workgroups, so the
// host's loose bounds on the segment count and length never size a grid.
__global__ __launch_bounds__(WG) void count_kernel(const Seg *__restrict__ cur,
                                                    const uint32_t *__restrict__ nitems_p,
                                                    const uint2 *__restrict__ items,
                                                    const Plan *__restrict__ plan,
                                                    const uint32_t *__restrict__ K,
                                                    uint32_t *__restrict__ cc, uint32_t stride) {
    __shared__ uint32_t tmp[WG / 64 + 1];
    const uint32_t nitems = *nitems_p;
    for (uint32_t t = blockIdx.x; t < nitems; t += gridDim.x) {
        const uint2 it = items[t];
        const uint32_t s = it.x, j = it.y;
        const Plan p = plan[s];
        const Seg g = cur[s];
        const int x0 = g.a + 1 + (int)j * CH;
        const int x1 = min(g.b, x0 + CH);
        uint32_t c = 0;
        for (int x = x0 + threadIdx.x; x < x1; x += WG) c += left_group(K[x], p.kp, p.eq);
        uint32_t total;
        block_excl_scan<WG>(c, tmp, &total);
        if (threadIdx.x == 0) cc[(size_t)s * stride + j] = total;
    }
}

// ranks of the misplaced elements: PL[a + k] / PR[a + k] = position of the
// k-th left-misplaced (from the left) / right-misplaced (from the right).
// The block sums the segment's block counts itself (its prefix and the total
// cnt; block 0 stores cnt for swap_kernel).  Each wave owns a contiguous
// quarter of the block's chunk: it counts its left-group elements, one
// barrier gives the waves' offsets, and it then ranks its rows with ballots
// (no block scans inside the loop).
__global__ __launch_bounds__(WG) void rank_kernel(const Seg *__restrict__ cur,
                                                   const uint32_t *__restrict__ nitems_p,
                                                   const uint2 *__restrict__ items,
                                                   Plan *__restrict__ plan,
                                                   const uint32_t *__restrict__ K,
                                                   const uint32_t *__restrict__ cc,
                                                   uint32_t stride, int32_t *__restrict__ PL,
                                                   int32_t *__restrict__ PR) {
    constexpr int NW = WG / 64, WCH = CH / NW;  // elements per wave
    __shared__ uint32_t wcnt[NW], wpre[NW], wtot[NW];
    const uint32_t nitems = *nitems_p;
    for (uint32_t t = blockIdx.x; t < nitems; t += gridDim.x) {
        const uint2 it = items[t];
        const uint32_t s = it.x, j = it.y;
        const Plan p = plan[s];
        const Seg g = cur[s];
        const int x0 = g.a + 1 + (int)j * CH;
        const int x1 = min(g.b, x0 + CH);
        const uint32_t w = threadIdx.x >> 6, l = __lane_id();
        const uint64_t lt = (1ull << l) - 1ull;
        const int w0 = x0 + (int)w * WCH, w1 = min(x1, w0 + WCH);
        uint32_t c = 0;
        for (int x = w0 + (int)l; x < w1; x += 64) c += left_group(K[x], p.kp, p.eq);
        c = wave_sum(c);
        const uint32_t nch = (uint32_t)((g.b - g.a - 1 + CH - 1) / CH);
        uint32_t pre = 0, tot = 0;
        for (uint32_t q = threadIdx.x; q < nch; q += WG) {
            const uint32_t v = cc[(size_t)s * stride + q];
            tot += v;
            pre += q < j ? v : 0u;
        }
        pre = wave_sum(pre);
        tot = wave_sum(tot);
        if (l == 0) {
            wcnt[w] = c;
            wpre[w] = pre;
            wtot[w] = tot;
        }
        __syncthreads();
        uint32_t base = 0, cnt = 0;
        for (uint32_t v = 0; v < (uint32_t)NW; v++) {
            base += wpre[v] + (v < w ? wcnt[v] : 0u);
            cnt += wtot[v];
        }
        __syncthreads();  // wcnt / wpre / wtot are rewritten by the next item
        if (j == 0 && threadIdx.x == 0) plan[s].cnt = (int)cnt;
        const int L = g.a + (int)cnt;  // left region [a+1, L]
        for (int c0 = w0; c0 < w1; c0 += 64) {
            const int x = c0 + (int)l;
            const bool in = x < w1;
            const bool f = in && left_group(K[x], p.kp, p.eq);
            const uint64_t m = __ballot(f);
            const uint32_t pf = base + (uint32_t)__popcll(m & lt);
            if (in) {
                if (x > L && f) PR[g.a + ((int)cnt - (int)pf - 1)] = x;
                if (x <= L && !f) PL[g.a + ((x - (g.a + 1)) - (int)pf)] = x;
                // m = the left-misplaced elements = the positions of [a+1, L]
                // less the left-group elements among them, known at x = L with
                // no atomic (one per wave and item on ONE address serialised
                // at L2: 10 K of them made the first round's ranking 167 us)
                if (x == L) plan[s].m = (L - g.a) - (int)(pf + (f ? 1u : 0u));
            }
            base += (uint32_t)__popcll(m);
        }
    }
}

// lane 0 of the owner block
__device__ void swap_tail(const Ctl &c, const Plan &p, const Seg &g, const GAcc &d, int mid) {
    if (p.eq) {  // partitionEqual returns a + 1 + cnt; the loop continues
        push_seg(c, Seg{g.a + 1 + p.cnt, g.b, g.limit, g.flags});
        return;
    }
    d.swap(mid, g.a);
    const int already = p.m == 0;
    const int n = g.b - g.a, ln = mid - g.a, rn = g.b - mid, thr = n / 8;
    if (ln < rn) {
        push_seg(c, Seg{g.a, mid, g.limit, 3});
        push_seg(c, Seg{mid + 1, g.b, g.limit, (ln >= thr) | (already << 1)});
    } else {
        push_seg(c, Seg{mid + 1, g.b, g.limit, 3});
        push_seg(c, Seg{g.a, mid, g.limit, (rn >= thr) | (already << 1)});
    }
}

// The m swaps of the partition, then the tail of the loop iteration:
// partitionEqual's `a = mid` continue, or the pivot swap and the two
// recursions (smaller side first, as Go recurses on it).  The tail touches
// only positions a (never swapped: PL, PR lie in (a, b)) and mid = a + cnt,
// which a swap moves only if it is the last left-misplaced element
// (PL[m - 1] == mid).  So the block that owns swap m - 1 runs the tail after
// its own swaps (block 0 if mid does not move): no cross-block hand-off.
__global__ __launch_bounds__(WG) void swap_kernel(const Seg *__restrict__ cur,
                                                   const uint32_t *__restrict__ nitems_p,
                                                   const uint2 *__restrict__ items,
                                                   Plan *__restrict__ plan, uint32_t *__restrict__ K,
                                                   int32_t *__restrict__ I,
                                                   const int32_t *__restrict__ PL,
                                                   const int32_t *__restrict__ PR, Ctl c) {
    const uint32_t nitems = *nitems_p;
    for (uint32_t t = blockIdx.x; t < nitems; t += gridDim.x) {
        const uint2 it = items[t];
        const uint32_t s = it.x, j = it.y;
        const Plan p = plan[s];
        const uint32_t nparts = p.m > 0 ? (uint32_t)((p.m + CH - 1) / CH) : 1u;
        if (j >= nparts) continue;  // (m <= (n - 1) / 2: never more parts than chunks)
        const Seg g = cur[s];
        GAcc d{K, I};
        for (int k = (int)j * CH + threadIdx.x; k < min(p.m, (int)(j + 1) * CH); k += blockDim.x)
            d.swap(PL[g.a + k], PR[g.a + k]);
        const int mid = g.a + p.cnt;
        const bool moved = !p.eq && p.m > 0 && PL[g.a + p.m - 1] == mid;
        const uint32_t owner = moved ? (uint32_t)((p.m - 1) / CH) : 0u;
        if (j != owner) continue;
        __syncthreads();  // this block's swaps (incl. the one moving mid) before the tail
        if (threadIdx.x == 0) swap_tail(c, p, g, d, mid);
    }
}


// ------------------------------------------------------ sharded order
// One part of `nparts` (a rank of a sharded corpus, dist.py): from the round
// that first holds >= 4 * nparts large segments (or the finisher, whichever
// comes first), this part keeps only the live segments that START in its block
// of positions [part * n / nparts, (part + 1) * n / nparts), with their
// descendants (the owner is fixed at that round), and sets the positions of
// every other live segment to -1.  Every position is then final on at least
// one part, with the same value wherever it is (segments are independent:
// pdqsort reads nothing outside [a, b) but the finished pivot at a-1), so an
// int32 MAX all-reduce of the parts' arrays is Go's order.
__device__ __forceinline__ bool seg_mine(const Seg &g, uint32_t n, uint32_t part, uint32_t nparts) {
    return (uint32_t)(((uint64_t)(uint32_t)g.a * nparts) / n) == part;
}

// positions of the segments this part drops: -1 (block per segment)
__global__ __launch_bounds__(WG) void shard_fill_kernel(const Seg *__restrict__ cur,
                                                        const uint32_t *__restrict__ ccount,
                                                        const Seg *__restrict__ small,
                                                        const uint32_t *__restrict__ scount,
                                                        uint32_t small_cap, uint32_t n,
                                                        uint32_t part, uint32_t nparts,
                                                        int32_t *__restrict__ I) {
    const uint32_t nc = *ccount, ns = min(*scount, small_cap);
    for (uint32_t i = blockIdx.x; i < nc + ns; i += gridDim.x) {
        const Seg g = i < nc ? cur[i] : small[i - nc];
        if (seg_mine(g, n, part, nparts)) continue;
        for (int p = g.a + (int)threadIdx.x; p < g.b; p += WG) I[p] = -1;
    }
}

// the lists compacted to this part's segments (one workgroup; list order is
// free: segments are independent)
__device__ void shard_compact(Seg *list, uint32_t *count, uint32_t cap, uint32_t n, uint32_t part,
                              uint32_t nparts, uint32_t *s_n) {
    const uint32_t tot = min(*count, cap);
    if (threadIdx.x == 0) *s_n = 0;
    __syncthreads();
    for (uint32_t i0 = 0; i0 < tot; i0 += WG) {
        const uint32_t i = i0 + threadIdx.x;
        Seg g{};
        const bool keep = i < tot && seg_mine(g = list[i], n, part, nparts);
        __syncthreads();  // the chunk is read before any slot of it is written
        if (keep) list[atomicAdd(s_n, 1u)] = g;
        __syncthreads();
    }
    if (threadIdx.x == 0) *count = *s_n;
}

__global__ __launch_bounds__(WG) void shard_compact_kernel(Seg *cur, uint32_t *ccount, Seg *small,
                                                           uint32_t *scount, uint32_t small_cap,
                                                           uint32_t cur_cap, uint32_t n,
                                                           uint32_t part, uint32_t nparts) {
    __shared__ uint32_t s_n;
    shard_compact(cur, ccount, cur_cap, n, part, nparts, &s_n);
    __syncthreads();
    shard_compact(small, scount, small_cap, n, part, nparts, &s_n);
}

// ------------------------------------------------------- in-LDS finisher
// One workgroup per segment of <= SMALL elements: tasks are popped by lane 0
// (O(1) control steps), partitions of tasks longer than MID run WG-parallel;
// tasks of TINY < n <= MID are then dealt to the 4 waves, each running its
// own loop with wave-parallel partitions (no workgroup barriers; tasks are
// disjoint and read only the finished pivot left of them); leaves of <= TINY
// elements are collected and finished one per lane at the end.
struct LTask {
    int16_t a, b;  // relative to the segment start
    int16_t limit, flags;
};
#ifndef SYZ_GSORT_MID
#define SYZ_GSORT_MID 1024
#endif
constexpr int MID = SYZ_GSORT_MID;  // tasks up to MID run on one wave
constexpr int MCAP = SMALL / TINY * 2;  // mid tasks per segment
constexpr int WSTK = SMALL / TINY / 4 + 32;  // per-wave stack (its share + depth)

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// One loop of pdqsort on a wave over the tasks in its stack (lane 0: control
// steps; all lanes: the Hoare partition with wave prefix sums).  PL / PR are
// indexed by the task's own positions, so waves never share them.
__device__ void wave_tasks(LAcc d, int a, LTask *stk, int depth, LTask *tiny, int *ntiny,
                           int16_t *PL, int16_t *PR, uint32_t *err) {
    const uint32_t l = __lane_id();
    int sp = depth;  // stack size (uniform)
    while (sp > 0) {
        int mode = 3, ta = 0, tb = 0, limit = 0, flags = 0;
        if (l == 0) {
            const LTask lt = stk[--sp];
            ta = a + lt.a;
            tb = a + lt.b;
            const int tn = lt.b - lt.a;
            limit = lt.limit;
            flags = lt.flags;
            if (tn <= TINY) {
                if (tn > 1) {
                    const int q = atomicAdd(ntiny, 1);
                    if (q < SMALL / 2) tiny[q] = lt; else *err = 4u;
                }
            } else if (limit == 0) {
                gocore::heap_sort(d, ta, tb);
            } else {
                const bool wb = flags & 1, wp = flags & 2;
                if (!wb) {
                    gocore::break_patterns(d, ta, tb);
                    limit--;
                }
                int hint;
                int pivot = gocore::choose_pivot(d, ta, tb, &hint);
                if (hint == gocore::kDecreasing) {
                    gocore::reverse_range(d, ta, tb);
                    pivot = (tb - 1) - (pivot - ta);
                    hint = gocore::kIncreasing;
                }
                if (!(wb && wp && hint == gocore::kIncreasing &&
                      gocore::partial_insertion_sort(d, ta, tb))) {
                    const int eq = ta > 0 && !d.less(ta - 1, pivot);
                    d.swap(ta, pivot);
                    mode = eq ? 2 : 1;
                }
            }
        }
        sp = __shfl(sp, 0, 64);
        mode = __shfl(mode, 0, 64);
        wave_sync_lds();
        if (mode == 3) continue;
        ta = __shfl(ta, 0, 64);
        tb = __shfl(tb, 0, 64);
        const int eq = mode == 2;
        const uint32_t kp = d.K[ta - a + 1];
        const int len = tb - ta - 1;
        const int per = (len + 63) / 64;
        const int x0 = ta + 1 + (int)l * per, x1 = min(tb, x0 + per);
        uint32_t c = 0;
        for (int x = x0; x < x1; x++) c += left_group(d.K[x - a + 1], kp, eq);
        const uint32_t inc = wave_incl_scan(c);
        const uint32_t cnt = __shfl(inc, 63, 64);
        uint32_t pf = inc - c;
        const int L = ta + (int)cnt;
        const int base = ta - a;  // this task's PL / PR window
        uint32_t mine = 0;
        for (int x = x0; x < x1; x++) {
            const bool f = left_group(d.K[x - a + 1], kp, eq);
            if (x > L && f) PR[base + (int)cnt - (int)pf - 1] = (int16_t)(x - a);
            if (x <= L && !f) {
                PL[base + (x - (ta + 1)) - (int)pf] = (int16_t)(x - a);
                mine++;
            }
            pf += f;
        }
        const uint32_t m = wave_sum(mine);
        wave_sync_lds();
        for (int k = (int)l; k < (int)m; k += 64) d.swap(a + PL[base + k], a + PR[base + k]);
        wave_sync_lds();
        if (l == 0) {
            if (eq) {
                const int na = ta + 1 + (int)cnt;
                if (tb - na > 1)
                    stk[sp++] = LTask{(int16_t)(na - a), (int16_t)(tb - a), (int16_t)limit,
                                      (int16_t)flags};
            } else {
                const int mid = ta + (int)cnt;
                d.swap(mid, ta);
                const int already = m == 0;
                const int tn = tb - ta, ln = mid - ta, rn = tb - mid, thr = tn / 8;
                LTask cont, fresh;
                if (ln < rn) {
                    cont = LTask{(int16_t)(mid + 1 - a), (int16_t)(tb - a), (int16_t)limit,
                                 (int16_t)((ln >= thr) | (already << 1))};
                    fresh = LTask{(int16_t)(ta - a), (int16_t)(mid - a), (int16_t)limit, 3};
                } else {
                    cont = LTask{(int16_t)(ta - a), (int16_t)(mid - a), (int16_t)limit,
                                 (int16_t)((rn >= thr) | (already << 1))};
                    fresh = LTask{(int16_t)(mid + 1 - a), (int16_t)(tb - a), (int16_t)limit, 3};
                }
                if (cont.b - cont.a > 1 && sp < WSTK) stk[sp++] = cont;
                else if (cont.b - cont.a > 1) *err = 5u;
                if (fresh.b - fresh.a > 1 && sp < WSTK) stk[sp++] = fresh;
                else if (fresh.b - fresh.a > 1) *err = 5u;
            }
        }
        sp = __shfl(sp, 0, 64);
        wave_sync_lds();
    }
}

__global__ __launch_bounds__(WG) void small_kernel(const Seg *__restrict__ small,
                                                    const uint32_t *__restrict__ nsmall_p,
                                                    uint32_t *__restrict__ Kg,
                                                    int32_t *__restrict__ Ig,
                                                    uint32_t *__restrict__ err) {
    constexpr int TCAP = SMALL / 2;
    __shared__ uint32_t K[SMALL + 1];
    __shared__ int32_t I[SMALL + 1];
    __shared__ int16_t PL[SMALL];  // positions relative to the segment start
    __shared__ int16_t PR[SMALL];  // (int16: two workgroups per CU fit in LDS)
    __shared__ LTask tiny[TCAP];
    __shared__ LTask stk[40];
    __shared__ LTask mids[MCAP];
    __shared__ LTask wstk[WG / 64][WSTK];
    __shared__ int sh[8];
    __shared__ uint32_t tmp[WG / 64 + 1];
    const uint32_t nsmall = *nsmall_p;
    for (uint32_t si = blockIdx.x; si < nsmall; si += gridDim.x) {
        const Seg g = small[si];
        const int a = g.a, n = g.b - g.a;
        for (int q = threadIdx.x; q < n; q += WG) {
            K[q + 1] = Kg[a + q];
            I[q + 1] = Ig[a + q];
        }
        if (threadIdx.x == 0) {
            K[0] = a > 0 ? Kg[a - 1] : 0u;  // the finished pivot left of the segment
            I[0] = -1;
            stk[0] = LTask{0, (int16_t)n, (int16_t)g.limit, (int16_t)g.flags};
            sh[0] = 1;  // stack size
            sh[1] = 0;  // tiny count
            sh[7] = 0;  // mid count
        }
        __syncthreads();
        LAcc d{K, I, a};
        for (;;) {
            // ---- lane 0: pop and run the O(1) control steps
            if (threadIdx.x == 0) {
                int mode = 3;  // 0 stop, 1 partition, 2 partitionEqual, 3 next task
                if (sh[0] == 0) {
                    mode = 0;
                } else {
                    const LTask lt = stk[--sh[0]];
                    const int ta = a + lt.a, tb = a + lt.b, tn = lt.b - lt.a;
                    int limit = lt.limit;
                    if (tn <= TINY) {
                        if (tn > 1) {
                            if (sh[1] < TCAP)
                                tiny[sh[1]++] = lt;
                            else
                                *err = 4u;
                        }
                    } else if (tn <= MID) {  // to the wave phase
                        if (sh[7] < MCAP)
                            mids[sh[7]++] = lt;
                        else
                            *err = 4u;
                    } else if (limit == 0) {
                        gocore::heap_sort(d, ta, tb);
                    } else {
                        const bool wb = lt.flags & 1, wp = lt.flags & 2;
                        if (!wb) {
                            gocore::break_patterns(d, ta, tb);
                            limit--;
                        }
                        int hint;
                        int pivot = gocore::choose_pivot(d, ta, tb, &hint);
                        if (hint == gocore::kDecreasing) {
                            gocore::reverse_range(d, ta, tb);
                            pivot = (tb - 1) - (pivot - ta);
                            hint = gocore::kIncreasing;
                        }
                        if (!(wb && wp && hint == gocore::kIncreasing &&
                              gocore::partial_insertion_sort(d, ta, tb))) {
                            const int eq = ta > 0 && !d.less(ta - 1, pivot);
                            d.swap(ta, pivot);
                            mode = eq ? 2 : 1;
                            sh[2] = ta;
                            sh[3] = tb;
                            sh[4] = limit;
                            sh[5] = lt.flags;
                        }
                    }
                }
                sh[6] = mode;
            }
            __syncthreads();
            const int mode = sh[6];
            if (mode == 0) break;
            if (mode == 3) continue;
            // ---- WG-parallel Hoare partition of [ta+1, tb) around K[ta]
            const int ta = sh[2], tb = sh[3], eq = mode == 2;
            const uint32_t kp = K[ta - a + 1];
            const int len = tb - ta - 1;
            const int per = (len + WG - 1) / WG;
            const int x0 = ta + 1 + (int)threadIdx.x * per, x1 = min(tb, x0 + per);
            uint32_t c = 0;
            for (int x = x0; x < x1; x++) c += left_group(K[x - a + 1], kp, eq);
            uint32_t cnt;
            uint32_t pf = block_excl_scan<WG>(c, tmp, &cnt);
            const int L = ta + (int)cnt;
            uint32_t mine = 0;
            for (int x = x0; x < x1; x++) {
                const bool f = left_group(K[x - a + 1], kp, eq);
                if (x > L && f) PR[(int)cnt - (int)pf - 1] = (int16_t)(x - a);
                if (x <= L && !f) {
                    PL[(x - (ta + 1)) - (int)pf] = (int16_t)(x - a);
                    mine++;
                }
                pf += f;
            }
            uint32_t m;
            block_excl_scan<WG>(mine, tmp, &m);  // total misplaced pairs (barriers)
            for (int k = threadIdx.x; k < (int)m; k += WG) d.swap(a + PL[k], a + PR[k]);
            __syncthreads();
            if (threadIdx.x == 0) {
                const int limit = sh[4], flags = sh[5];
                if (eq) {
                    const int na = ta + 1 + (int)cnt;
                    if (tb - na > 1)
                        stk[sh[0]++] = LTask{(int16_t)(na - a), (int16_t)(tb - a), (int16_t)limit,
                                             (int16_t)flags};
                } else {
                    const int mid = ta + (int)cnt;
                    d.swap(mid, ta);
                    const int already = m == 0;
                    const int tn = tb - ta, ln = mid - ta, rn = tb - mid, thr = tn / 8;
                    LTask cont, fresh;
                    if (ln < rn) {
                        cont = LTask{(int16_t)(mid + 1 - a), (int16_t)(tb - a), (int16_t)limit,
                                     (int16_t)((ln >= thr) | (already << 1))};
                        fresh = LTask{(int16_t)(ta - a), (int16_t)(mid - a), (int16_t)limit, 3};
                    } else {
                        cont = LTask{(int16_t)(ta - a), (int16_t)(mid - a), (int16_t)limit,
                                     (int16_t)((rn >= thr) | (already << 1))};
                        fresh = LTask{(int16_t)(mid + 1 - a), (int16_t)(tb - a), (int16_t)limit, 3};
                    }
                    // larger side parked, smaller side next (depth <= log2 n)
                    if (cont.b - cont.a > 1) stk[sh[0]++] = cont;
                    if (fresh.b - fresh.a > 1) stk[sh[0]++] = fresh;
                }
            }
            __syncthreads();
        }
        // ---- mid tasks: dealt round-robin to the waves, one loop per wave
        {
            const uint32_t w = threadIdx.x >> 6;
            const int nm = sh[7];
            int depth = 0;
            for (int q = (int)w; q < nm; q += WG / 64) {
                if (depth < WSTK) {
                    if (__lane_id() == 0) wstk[w][depth] = mids[q];
                } else if (__lane_id() == 0) {
                    *err = 5u;
                }
                depth++;
            }
            wave_sync_lds();
            wave_tasks(d, a, wstk[w], min(depth, WSTK), tiny, &sh[1], PL, PR, err);
        }
        __syncthreads();
        // ---- leaves: one lane each, Go's sequential loop
        const int nt = sh[1];
        for (int q = threadIdx.x; q < nt; q += WG) {
            const LTask lt = tiny[q];
            gocore::pdq_loop<LAcc, 3, gocore::BitStack>(d, gocore::Task{a + lt.a, a + lt.b, lt.limit,
                                                       (bool)(lt.flags & 1),
                                                       (bool)(lt.flags & 2)});
        }
        __syncthreads();
        for (int q = threadIdx.x; q < n; q += WG) Ig[a + q] = I[q + 1];
        __syncthreads();
    }
}

}  // namespace gsort
}  // namespace syz

using namespace syz;
using namespace syz::gsort;

// workspace layout (all 256-B aligned)
struct SortWs {
    uint32_t *K;
    int32_t *I, *PL, *PR;
    Seg *segA, *segB, *small;
    Plan *plan;
    uint32_t *cc;
    uint2 *items;   // the round's (segment, chunk) work items
    uint32_t *ctl;  // [0] err [1] countA [2] countB [3] small count [4] maxA [5] maxB
                    // [6] itemsA [7] itemsB
    uint32_t seg_cap, small_cap, cc_stride, item_cap;
    size_t n;  // positions
};

static size_t ws_layout(size_t n, size_t ngroups, SortWs *w, uint8_t *base) {
    const uint32_t seg_cap = (uint32_t)(2 * (n / SMALL) + 16);
    const uint32_t small_cap = (uint32_t)(2 * (n / SMALL + 1) * 64 + 64 + ngroups);
    const uint32_t cc_stride = (uint32_t)(n / CH + 2);
    const uint32_t item_cap = (uint32_t)(n / CH + seg_cap + 16);
    size_t o = 0;
    auto take = [&](size_t bytes) {
        size_t r = o;
        o += align_up(bytes, 256);
        return r;
    };
    size_t oK = take(n * 4), oI = take(n * 4), oPL = take(n * 4), oPR = take(n * 4),
           oA = take(seg_cap * sizeof(Seg)), oB = take(seg_cap * sizeof(Seg)),
           oS = take(small_cap * sizeof(Seg)), oP = take(seg_cap * sizeof(Plan)),
           oC = take((size_t)seg_cap * cc_stride * 4), oIt = take((size_t)item_cap * 8),
           oT = take(64);
    if (w) {
        w->K = (uint32_t *)(base + oK);
        w->I = (int32_t *)(base + oI);
        w->PL = (int32_t *)(base + oPL);
        w->PR = (int32_t *)(base + oPR);
        w->segA = (Seg *)(base + oA);
        w->segB = (Seg *)(base + oB);
        w->small = (Seg *)(base + oS);
        w->plan = (Plan *)(base + oP);
        w->cc = (uint32_t *)(base + oC);
        w->items = (uint2 *)(base + oIt);
        w->ctl = (uint32_t *)(base + oT);
        w->item_cap = item_cap;
        w->seg_cap = seg_cap;
        w->small_cap = small_cap;
        w->cc_stride = cc_stride;
        w->n = n;
    }
    return o;
}

extern "C" size_t syzcov_dev_sort_ws_size(size_t n) {
    return ws_layout(n ? n : 1, 0, nullptr, nullptr);
}

extern "C" size_t syzcov_dev_sort_seg_ws_size(size_t n, size_t ngroups) {
    return ws_layout((n ? n : 1) + ngroups, ngroups, nullptr, nullptr);
}

// Level-synchronous pdqsort rounds over the segments already seeded into
// segA / small (ctl[1], ctl[3]); the result is left in w.I.
// seeded >= 0: the host already knows the seed (one segment of `seeded`
// elements), so the first read-back is skipped; an input error flagged by the
// init kernel is then reported by the final read-back.
// Pinned host words for the round read-backs: a copy into pageable memory
// (a stack array) is staged by the runtime and left the GPU idle ~35 us per
// read-back.  Leased from a process-wide pool for the call's duration.
class PinnedCtl {
  public:
    PinnedCtl() {
        std::lock_guard<std::mutex> g(mu());
        if (!free_list().empty()) {
            p_ = free_list().back();
            free_list().pop_back();
        } else if (hipHostMalloc((void **)&p_, 64, hipHostMallocDefault) != hipSuccess) {
            p_ = nullptr;
        }
    }
    ~PinnedCtl() {
        if (!p_) return;
        std::lock_guard<std::mutex> g(mu());
        free_list().push_back(p_);
    }
    uint32_t *get() const { return p_; }

  private:
    static std::mutex &mu() {
        static std::mutex *m = new std::mutex();
        return *m;
    }
    static std::vector<uint32_t *> &free_list() {
        static std::vector<uint32_t *> *v = new std::vector<uint32_t *>();
        return *v;
    }
    uint32_t *p_ = nullptr;
};

// ctl[0..n) -> h through the pinned words (or directly, if none could be had)
static int read_ctl(uint32_t *h, const uint32_t *ctl, size_t n, uint32_t *pin, hipStream_t s) {
    SYZ_HIP(hipMemcpyAsync(pin ? pin : h, ctl, n * 4, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    if (pin) memcpy(h, pin, n * 4);
    return 0;
}

// The sort's internal error word (ctl[0]) into a step's error flags, on the
// device: no host turnaround after the finisher (the caller's result()
// reports it).
__global__ void sort_err_kernel(const uint32_t *ctl, uint32_t *err) {
    if (ctl[0]) atomicOr(err, SYZCOV_ERR_ORDER);
}

static int run_rounds(SortWs &w, hipStream_t s, int64_t seeded = -1, uint32_t part = 0,
                      uint32_t nparts = 1, uint32_t *err_dev = nullptr) {
    PinnedCtl pin;
    bool split = nparts <= 1;  // this part's segments selected (or nothing to split)
    auto split_now = [&](Seg *cur_, uint32_t *ccount_, uint32_t ncur_) {
        hipLaunchKernelGGL(shard_fill_kernel, dim3(std::min<uint32_t>(ncur_ + 4096, 8192)), dim3(WG),
                           0, s, (const Seg *)cur_, (const uint32_t *)ccount_, (const Seg *)w.small,
                           (const uint32_t *)(w.ctl + 3), w.small_cap, (uint32_t)w.n, part, nparts,
                           w.I);
        hipLaunchKernelGGL(shard_compact_kernel, dim3(1), dim3(WG), 0, s, cur_, ccount_, w.small,
                           w.ctl + 3, w.small_cap, w.seg_cap, (uint32_t)w.n, part, nparts);
        SYZ_LAUNCH_CHECK();
        split = true;
        return 0;
    };
    Seg *cur = w.segA, *nxt = w.segB;
    uint32_t *ccount = w.ctl + 1, *ncount = w.ctl + 2, *cmax = w.ctl + 4, *nmax = w.ctl + 5;
    uint32_t *citems = w.ctl + 6, *nitems = w.ctl + 7;
    uint32_t h[6] = {0, 0, 0, 0, 0, 0};
    if (seeded < 0) {
        if (int rc = read_ctl(h, w.ctl, 6, pin.get(), s)) return rc;
    } else if (seeded > SMALL) {
        h[1] = 1;
        h[4] = (uint32_t)seeded;
    } else if (seeded > 1) {
        h[3] = 1;
    }
    // The kernels read the live segment count from the device (ccount), so
    // rounds are queued without a host round trip: the host keeps only UPPER
    // BOUNDS for the grids (a segment has at most two large children, each
    // shorter than it, and at most total/(SMALL+1) large segments exist) and
    // reads the true count back every SYNC_EVERY rounds.  Rounds queued after
    // the last large segment finished find no work items and return at once
    // (≈5 µs a round against ≈50 µs of host turnaround per read-back; a
    // pipelined read-back, the next rounds queued behind an event before the
    // host waits, measured slower: its bounds are a batch older).
    // The first SYNC_EVERY-round batches hold the long rounds; past them the
    // rounds are short and few are left, and a batch of 8 queued past the
    // last large segment cost ~8 x 4 dispatches of ~7 us each (a C3/8 rank:
    // ~0.23 ms of empty rounds), so the tail reads back every SYNC_TAIL.
    constexpr int SYNC_EVERY = 8;  // 4 and 16 measured no faster
#ifndef SYZ_GSORT_SYNC_TAIL
#define SYZ_GSORT_SYNC_TAIL 2  // 1 / 2 / 4 / 8: C3/8 rank order 1.57 / 1.55 / 1.62 / 1.62 ms
#endif
#ifndef SYZ_GSORT_SYNC_HEAD
#define SYZ_GSORT_SYNC_HEAD 16  // rounds before the tail interval applies
#endif
    const uint32_t cap_seg = std::min<uint32_t>(w.seg_cap, w.n / (SMALL + 1) + 1);
    uint32_t ncur = h[1], maxlen = h[4];
    bool exact = true;  // ncur is the device's count (a read-back), not a bound
    int next_sync = SYNC_EVERY;
    for (int round = 0; ncur > 0 && !h[0]; round++) {
        if (round > 4096) return SYZCOV_EHIP;
        if (!split && exact && ncur >= SYZ_GSORT_SPLIT_MUL * nparts) split_now(cur, ccount, ncur);
        exact = false;
        // the children of this round go to nxt
        // (lead_kernel zeroes ncount / nmax)
        Ctl cn{nxt, ncount, nmax, w.small, w.ctl + 3, w.small_cap, w.seg_cap, w.ctl};
        const uint64_t nch = (maxlen + CH - 1) / CH;
        // work items: at most ncur * nch, and sum ceil((n_s - 1) / CH) <= n / CH + ncur
        const unsigned gi = (unsigned)std::min<uint64_t>(
            std::min<uint64_t>(nch * ncur, w.n / CH + ncur), ITEM_GRID);
        hipLaunchKernelGGL(lead_kernel, dim3(ncur), dim3(WG), 0, s, cur, ccount, w.plan, w.K, w.I, cn,
                           citems, nitems, w.items, w.item_cap);
        hipLaunchKernelGGL(count_kernel, dim3(gi), dim3(WG), 0, s, cur, citems, w.items, w.plan, w.K,
                           w.cc, w.cc_stride);
        hipLaunchKernelGGL(rank_kernel, dim3(gi), dim3(WG), 0, s, cur, citems, w.items, w.plan, w.K,
                           w.cc, w.cc_stride, w.PL, w.PR);
        hipLaunchKernelGGL(swap_kernel, dim3(gi), dim3(WG), 0, s, cur, citems, w.items, w.plan, w.K,
                           w.I, w.PL, w.PR, cn);
        SYZ_LAUNCH_CHECK();
        std::swap(cur, nxt);
        std::swap(ccount, ncount);
        std::swap(cmax, nmax);
        std::swap(citems, nitems);
        // bounds for the next round (exact after a read-back)
        ncur = std::min(2 * ncur, cap_seg);
        maxlen = maxlen > 1 ? maxlen - 1 : 0;
        if (round + 1 == next_sync || maxlen <= SMALL) {
            next_sync = round + 1 + (round + 1 < SYZ_GSORT_SYNC_HEAD ? SYNC_EVERY : SYZ_GSORT_SYNC_TAIL);
            if (int rc = read_ctl(h, w.ctl, 6, pin.get(), s)) return rc;
            ncur = h[ccount - w.ctl];
            maxlen = h[cmax - w.ctl];
            exact = true;
        }
    }
    if (!split && !h[0]) {  // the finisher's segments are split at least
        split_now(cur, ccount, 0);
        if (int rc = read_ctl(h, w.ctl, 6, pin.get(), s)) return rc;
    }
    if (!h[0] && h[3]) {
        hipLaunchKernelGGL(small_kernel, dim3(std::min<uint32_t>(h[3], 8192)), dim3(WG), 0, s, w.small,
                           w.ctl + 3, w.K, w.I, w.ctl);
        SYZ_LAUNCH_CHECK();
    }
    if (!h[0] && (h[3] || seeded >= 0)) {
        if (err_dev) {
            hipLaunchKernelGGL(sort_err_kernel, dim3(1), dim3(1), 0, s, (const uint32_t *)w.ctl,
                               err_dev);
            SYZ_LAUNCH_CHECK();
            return 0;
        }
        if (int rc = read_ctl(h, w.ctl, 1, pin.get(), s)) return rc;
    }
    if (h[0]) {
        set_error("device sort: internal error %u", h[0]);
        return h[0] == 1 ? SYZCOV_EINVAL : SYZCOV_EHIP;
    }
    return 0;
}

static int sort_order_part(const int64_t *lens, size_t n, int sort_variant, uint32_t part,
                           uint32_t nparts, int32_t *order, void *ws, size_t ws_size, void *stream,
                           uint32_t *err_dev = nullptr);

namespace syz {
// syzcov_dev_sort_order_part with the finisher's error check left on the
// device (err_dev |= SYZCOV_ERR_ORDER): the corpus handle's order phase
int sort_order_part_dev(const int64_t *lens, size_t n, uint32_t part, uint32_t nparts,
                        int32_t *order, void *ws, size_t ws_size, uint32_t *err_dev,
                        hipStream_t s) {
    if (nparts == 0 || part >= nparts || !err_dev) return SYZCOV_EINVAL;
    return sort_order_part(lens, n, 0, part, nparts, order, ws, ws_size, s, err_dev);
}
}  // namespace syz

extern "C" int syzcov_dev_sort_order(const int64_t *lens, size_t n, int sort_variant,
                                     int32_t *order, void *ws, size_t ws_size, void *stream) {
    return sort_order_part(lens, n, sort_variant, 0, 1, order, ws, ws_size, stream);
}

extern "C" int syzcov_dev_sort_order_part(const int64_t *lens, size_t n, uint32_t part,
                                          uint32_t nparts, int32_t *order, void *ws,
                                          size_t ws_size, void *stream) {
    if (nparts == 0 || part >= nparts) return SYZCOV_EINVAL;
    return sort_order_part(lens, n, 0, part, nparts, order, ws, ws_size, stream);
}

static int sort_order_part(const int64_t *lens, size_t n, int sort_variant, uint32_t part,
                           uint32_t nparts, int32_t *order, void *ws, size_t ws_size, void *stream,
                           uint32_t *err_dev) {
    if (n == 0) return 0;
    if (!lens || !order || n > 0x7FFFFFFF) return SYZCOV_EINVAL;
    if (sort_variant != 0) {
        set_error("only Go >= 1.19 pdqsort order is computed; pass the caller's order instead");
        return SYZCOV_EINVAL;
    }
    hipStream_t s = (hipStream_t)stream;
    if (!ws || ws_size < syzcov_dev_sort_ws_size(n)) return SYZCOV_EINVAL;
    SortWs w;
    ws_layout(n, 0, &w, (uint8_t *)ws);
    SYZ_HIP(hipMemsetAsync(w.ctl, 0, 64, s));
    hipLaunchKernelGGL(init_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, lens, (uint32_t)n,
                       w.K, w.I, w.ctl);
    Ctl c{w.segA, w.ctl + 1, w.ctl + 4, w.small, w.ctl + 3, w.small_cap, w.seg_cap, w.ctl};
    if (n > 1) hipLaunchKernelGGL(seed_kernel, dim3(1), dim3(1), 0, s, (uint32_t)n, c);
    SYZ_LAUNCH_CHECK();
    if (int rc = run_rounds(w, s, (int64_t)n, part, nparts, err_dev)) return rc;
    SYZ_HIP(hipMemcpyAsync(order, w.I, n * 4, hipMemcpyDeviceToDevice, s));
    return 0;
}

extern "C" int syzcov_dev_sort_order_segmented(const int64_t *lens, const uint64_t *goff,
                                               size_t ngroups, size_t n, int sort_variant,
                                               int32_t *order, void *ws, size_t ws_size,
                                               void *stream) {
    if (n == 0) return 0;
    if (!lens || !goff || !order || ngroups == 0 || n + ngroups > 0x7FFFFFFF)
        return SYZCOV_EINVAL;
    if (sort_variant != 0) {
        set_error("only Go >= 1.19 pdqsort order is computed");
        return SYZCOV_EINVAL;
    }
    hipStream_t s = (hipStream_t)stream;
    if (!ws || ws_size < syzcov_dev_sort_seg_ws_size(n, ngroups)) return SYZCOV_EINVAL;
    const size_t npos = n + ngroups - 1;
    SortWs w;
    ws_layout(npos + 1, ngroups, &w, (uint8_t *)ws);
    SYZ_HIP(hipMemsetAsync(w.ctl, 0, 64, s));
    hipLaunchKernelGGL(seg_init_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, lens, goff,
                       (uint32_t)ngroups, w.K, w.I, w.ctl);
    Ctl c{w.segA, w.ctl + 1, w.ctl + 4, w.small, w.ctl + 3, w.small_cap, w.seg_cap, w.ctl};
    hipLaunchKernelGGL(seg_seed_kernel, dim3(grid_for(ngroups, 256, 1024)), dim3(256), 0, s, goff,
                       (uint32_t)ngroups, c);
    SYZ_LAUNCH_CHECK();
    if (int rc = run_rounds(w, s)) return rc;
    hipLaunchKernelGGL(seg_gather_kernel, dim3(grid_for(npos, 256, 8192)), dim3(256), 0, s,
                       (const int32_t *)w.I, goff, (uint32_t)ngroups, (uint32_t)npos, order);
    SYZ_LAUNCH_CHECK();
    return 0;
}
