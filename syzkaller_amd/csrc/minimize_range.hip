// minimize_range.hip — cover.Minimize (cover/cover.go:104-131) as a
// first-cover problem whose per-PC test never leaves LDS.
//
// kept(r) <=> some pc of cov_r has first(pc) == r, first(pc) = min rank
// covering pc.  Items (inputs in rank order) are processed in
// geometrically growing chunks.  Before chunk c, `covered` holds every PC
// whose first cover lies in an earlier chunk; inside the chunk a PC that is
// covered cannot be first for any rank of the chunk, so it costs one LDS bit
// test.  Every uncovered occurrence (rank, pc) is RECORDED and atomicMin-ed
// into first_w[pc - pc_lo]; the first cover of every PC is always recorded
// (nothing before it covers the PC).  Hence, after the last chunk:
//   first_w[pc]  = first(pc) for every recorded pc,
//   covered      = the union of the corpus (the maxCover merge operand),
//   kept(r)      <=> some record (r, pc) has first_w[pc] == r   (pass 2),
// and pass 2 touches only the records (a few per distinct PC), not the corpus.
//
// LDS residency: the PC window is cut into ranges of 2^rshift PCs (128 KB of
// bitmap at rshift 20).  A workgroup owns one range for a slice of the
// chunk's items, loads that range's covered bitmap into LDS, and streams the
// items' sub-runs inside the range (canonical lists are sorted, so a sub-run
// is contiguous: split[] from canon_wave.hip).  Ranges get workgroups in
// proportion to their PC counts (range_tot), so a hot range is cut into many
// short item slices.  A wave takes 64 items at a time and reads each item's
// sub-run with a group of 4 lanes (16 items per step, 16-byte chunks, 4 in
// flight per lane), so a load instruction covers 16 sub-runs in 64-B pieces
// instead of 64 scattered 16-B pieces; the per-PC work is a subtract, a shift
// and one LDS test.
//
// Records go to NCTR regions of the record buffer, each with its own counter
// (workgroup b appends to region b mod NCTR): one counter for the whole chip
// serialised every wave's reservation on a single address, which dominated the
// early chunks, where nearly every PC is a record.
//
// Record overflow (more uncovered occurrences than a region holds, only for
// adversarial corpora) is detected on the device; the fallback kernels then
// rescan candidate items and derive the union from first_w, so the result
// stays exact for every input.
#include "common.h"

#include <algorithm>

#define RC_(expr)                 \
    do {                          \
        int r_ = (expr);          \
        if (r_ < 0) return r_;    \
    } while (0)

namespace syz {
namespace mr {

constexpr int THREADS = 1024;
constexpr int NWAVE = THREADS / 64;

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = max(v, (uint32_t)__shfl_xor(v, d, 64));
    return v;
}
// inclusive prefix max over the wave's lanes (DPP, as wave_incl_scan)
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false));
    return v;
}
constexpr int MAX_R = 256;
constexpr int NCTR = 64;        // record regions (counters)
constexpr int CTR_STRIDE = 32;  // u64s between counters (256 B: separate lines)

struct Args {
    const uint64_t *off;
    const uint32_t *len;       // canonical lengths (used when split == NULL)
    const uint32_t *pcs;
    const uint32_t *split;     // [nseg][nrange] or NULL (nrange == 1)
    const int32_t *order;      // item -> local input index
    const int32_t *ranks;      // item -> rank (NULL: item index)
    uint32_t pc_lo;
    uint32_t rshift, nrange;
    const unsigned long long *range_tot;
    const uint32_t *covered;   // window bitmap (nrange << rshift bits)
    int32_t *first_w;          // [span], INT32_MAX outside records
    unsigned long long *rec;   // (rank << 32) | window offset
    uint64_t rec_cap;
    unsigned long long *rec_cnt;  // total (ABI); > rec_cap if a region overflowed
    unsigned long long *ctr;   // [NCTR * CTR_STRIDE] records appended per region
    unsigned long long *done;  // [NCTR * CTR_STRIDE] records already in `covered`
    uint64_t cap_k;            // records per region: rec[k * cap_k ...]
    uint8_t *cand;             // [items] item had an uncovered PC
    // rank-ordered descriptors (prep_kernel): coalesced per (range, item slice)
    const uint64_t *base_r;    // [items] off[order[j]]
    const uint32_t *split_t;   // [nrange][items] split[order[j]][rho]
    uint32_t n_items;
    uint32_t *pctr;            // dynamic pieces: this chunk's next-piece counter
    uint32_t npieces;          // dynamic pieces: pieces of this chunk (G)
    // key mode: pcs are key words (common.h); every word is checked against the
    // universe's membership table (keys.hip) staged with the covered bits
    uint32_t keymask;          // SYZ_KEY_MASK in key mode, ~0 otherwise
    const uint8_t *low_of_key; // [nrange << rshift] bytes, 0x7F past the keys
    uint32_t *err;             // SYZCOV_ERR_UNIVERSE
    uint32_t ak;               // line-aligned sub-runs (common.h), 0: CSR slots
    // bucketed first covers (bmin_kernel): per-chunk record counts per bucket
    // of 2^BSH keys [2][nb] (chunk parity), scatter cursors [2][nb], the
    // records sorted by bucket; bh == nullptr: min_records_kernel's atomics
    uint32_t *bh, *bcur;
    unsigned long long *rsort;
    uint32_t nb;
};
constexpr uint32_t BSH = 14;          // keys per bucket: 2^14 (64 KB of int32 in LDS)
constexpr uint32_t MAX_NB = 1024;     // key spaces up to 2^24 (cover_from_first)


// Gather the items' CSR bases and split columns into rank order, transposed
// so that a workgroup owning range rho reads split_t[rho][i0..i1) contiguously.
// A tile of 64 items is read row by row (each item's nrange split points are
// contiguous, so a wave reads whole rows), transposed in LDS (row stride
// nrange + 1: conflict-free column reads for even nrange) and written one
// range column of 64 items at a time.  Dynamic LDS: 64 * (nrange + 1) u32.
__global__ __launch_bounds__(256) void prep_kernel(Args A, uint64_t *base_r, uint32_t *split_t) {
    extern __shared__ uint32_t s_tile[];
    __shared__ uint32_t s_seg[64];
    const uint32_t n = A.n_items, R = A.nrange, ld = R + 1;
    // the next tile's order entries are loaded while this tile moves (one
    // dependent global round trip fewer per tile: order -> rows)
    const uint32_t tstride = gridDim.x * 64;
    uint32_t segc = 0;
    if (threadIdx.x < 64 && blockIdx.x * 64 + threadIdx.x < n)
        segc = (uint32_t)A.order[blockIdx.x * 64 + threadIdx.x];
    for (uint32_t t0 = blockIdx.x * 64; t0 < n; t0 += tstride) {
        const uint32_t rows = min(64u, n - t0);
        uint32_t segn = 0;
        if (threadIdx.x < 64 && (uint64_t)t0 + tstride + threadIdx.x < n)
            segn = (uint32_t)A.order[t0 + tstride + threadIdx.x];
        if (threadIdx.x < rows) {
            const uint32_t seg = segc;
            s_seg[threadIdx.x] = seg;
            base_r[t0 + threadIdx.x] = aligned_base(A.off[seg], seg, A.ak);
        }
        segc = segn;
        __syncthreads();
        if (!A.split) {  // one range: the column is the canonical length
            if (threadIdx.x < rows) split_t[t0 + threadIdx.x] = A.len[s_seg[threadIdx.x]];
        } else {
            if ((R & 3u) == 0 && ((uintptr_t)A.split & 15u) == 0) {
                // 16-byte pieces of the rows, every load of the tile issued
                // before the LDS stores (a load-store loop waited on each
                // load in turn: 112 us for a C3/8 rank's 1.25 M items)
                const uint32_t R4 = R >> 2, ne = rows * R4;
                constexpr uint32_t PB = 4;
                for (uint32_t e0 = 0; e0 < ne; e0 += PB * 256) {
                    uint4 v[PB];
#pragma unroll
                    for (uint32_t u = 0; u < PB; u++) {
                        const uint32_t e = e0 + u * 256 + threadIdx.x;
                        const uint32_t r = e / R4, c4 = e - r * R4;
                        v[u] = e < ne ? reinterpret_cast<const uint4 *>(A.split + (uint64_t)s_seg[r] * R)[c4]
                                      : make_uint4(0, 0, 0, 0);
                    }
#pragma unroll
                    for (uint32_t u = 0; u < PB; u++) {
                        const uint32_t e = e0 + u * 256 + threadIdx.x;
                        const uint32_t r = e / R4, c = (e - r * R4) * 4;
                        if (e < ne) {
                            uint32_t *d = s_tile + r * ld + c;
                            d[0] = v[u].x;
                            d[1] = v[u].y;
                            d[2] = v[u].z;
                            d[3] = v[u].w;
                        }
                    }
                }
            } else {
                for (uint32_t e = threadIdx.x; e < rows * R; e += blockDim.x) {
                    const uint32_t r = e / R, c = e - r * R;
                    s_tile[r * ld + c] = A.split[(uint64_t)s_seg[r] * R + c];
                }
            }
            __syncthreads();
            for (uint32_t e = threadIdx.x; e < 64 * R; e += blockDim.x) {
                const uint32_t rho = e >> 6, jj = e & 63;
                if (jj < rows) split_t[(uint64_t)rho * n + t0 + jj] = s_tile[jj * ld + rho];
            }
        }
        __syncthreads();
    }
}

// The range plan of a chunk: sh[j] = first piece position of range j (wave 0
// computes it into LDS; every thread waits).
__device__ void plan_pieces(const Args &A, uint32_t G, uint32_t P, uint32_t *sh) {
    const uint32_t l = __lane_id();
    if (threadIdx.x < 64) {
        unsigned long long wsum = 0;
        for (uint32_t j = l; j < A.nrange; j += 64) wsum += A.range_tot[j];
        for (int d = 32; d >= 1; d >>= 1) wsum += __shfl_xor(wsum, d, 64);
        const uint64_t spare = P > A.nrange ? P - A.nrange : 0;
        uint32_t carry = 0;
        for (uint32_t jb = 0; jb < A.nrange; jb += 64) {
            const uint32_t j = jb + l;
            uint32_t p = 0;
            if (j < A.nrange)  // integer: the pieces never exceed P
                p = 1u + (wsum ? (uint32_t)(A.range_tot[j] * spare / wsum) : 0u);
            const uint32_t inc = wave_incl_scan(p);
            if (j < A.nrange) sh[j + 1] = carry + inc;
            carry += __shfl(inc, 63, 64);
        }
        if (l == 0) sh[0] = 0;
    }
    __syncthreads();
}

// Piece g (slice-major: slice g / P, position g % P) -> (range, item slice
// [i0, i1)).  The chunk's items are cut into S = G / P slices; each slice is
// covered by P consecutive pieces, range j getting p_j = 1 + floor(w_j * (P -
// R) / W) of them (w_j: its key count), so a hot range's part of a slice is
// split further.
__device__ bool map_piece(const Args &A, uint32_t G, uint32_t P, uint32_t a, uint32_t b, uint32_t g,
                          uint32_t *rho, uint32_t *i0, uint32_t *i1, const uint32_t *sh) {
    const uint32_t S = G / P;  // slices
    const uint32_t sl = g / P, r = g % P;
    if (sl >= S || r >= sh[A.nrange]) return false;
    uint32_t lo = 0, hi = A.nrange;  // largest j with sh[j] <= r
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (sh[mid] <= r) lo = mid; else hi = mid;
    }
    const uint32_t p = sh[lo + 1] - sh[lo], q = r - sh[lo];
    const uint64_t n = b - a;
    const uint64_t s0 = n * sl / S, s1 = n * (sl + 1) / S;  // the slice
    *rho = lo;
    *i0 = a + (uint32_t)(s0 + (s1 - s0) * q / p);
    *i1 = a + (uint32_t)(s0 + (s1 - s0) * (q + 1) / p);
    return true;
}

// The next piece for the calling workgroup (key-mode pass 1), XCD-LOCAL
// SLICES: slice sl belongs to XCD sl mod 8 (workgroup b runs on XCD b mod 8,
// the dispatcher's round robin), and an XCD's workgroups draw its slices'
// pieces in slice order from its own counter (pctr[8x]), so the pieces of one
// item slice (every range of the same items) run at the same time on one XCD.
// The 128-byte line where an item's range-rho sub-run ends and its rho+1
// sub-run starts is then read twice from that XCD's L2, not twice from HBM:
// the range-major order (all workgroups on one range, the next range a whole
// range's bytes later) fetched every such line twice, 1.70x the algorithmic
// bytes of a C3/8 rank's Minimize; here 1.41x (C3 Minimize 21.5 -> 17.3 ms).
// A workgroup whose XCD has no pieces left takes the other XCDs' (every piece
// is drawn exactly once, so the assignment never affects the result).  The
// price is a table restage at nearly every piece (the next piece is another
// range), which the unrolled loads below keep to a few microseconds.
// Returns G when every piece is drawn.  (SYZ_MR_RANGE_MAJOR: one counter,
// range-major order.)
__device__ uint32_t draw_piece(uint32_t *pctr, uint32_t G, uint32_t P, uint32_t *xdone) {
    const uint32_t S = G / P;
#ifdef SYZ_MR_RANGE_MAJOR
    (void)xdone;
    const uint32_t g = atomicAdd(pctr, 1u);
    return g < G ? (g % S) * P + g / S : G;  // g = position * S + slice
#else
    const uint32_t me = blockIdx.x & 7u;
    for (uint32_t j = 0; j < 8; j++) {
        const uint32_t x = (me + j) & 7u;
        if (*xdone >> x & 1u) continue;
        const uint32_t nk = x < S ? ((S - 1 - x) / 8 + 1) * P : 0u;  // XCD x's pieces
        const uint32_t k = nk ? atomicAdd(pctr + 8 * x, 1u) : 0u;
        if (k < nk) return (x + 8 * (k / P)) * P + k % P;
        *xdone |= 1u << x;
    }
    return G;
#endif
}

// Pass 1 as a CHUNK STREAM (first covers deferred to min_records_kernel).
// A wave takes 64 items at a time and concatenates their sub-runs into one
// list of 16-byte chunks (an exclusive scan of the per-item chunk counts;
// lane j holds item j's start); lane l then loads chunks l, l + 64, l + 128,
// ... of that list.  Every load instruction is a full wave of useful 16-byte
// pieces whatever the sub-run lengths (lane groups per item idle the lanes of
// short or ragged sub-runs: 4.82 against 3.99 ms in window mode at C2's 64
// ranges), and consecutive lanes read consecutive chunks of one sub-run.
// The item of a chunk: the items starting inside a 64-chunk window mark
// their start in a per-wave LDS row, and a DPP prefix max over the lanes
// carries each mark forward — branch-free, three LDS operations per window.
// (A wave-uniform walk over the item starts by readlane, serial scalar loops
// of ~10 steps per window at 32 ranges, held pass 1 at 3.4 ms of C2's
// 3.95 ms Minimize; the marks: 2.87 ms.)  Loads and covered tests are
// branch-free straight-line code, so the next UG x 64 chunks stay in flight
// while the current ones are tested (a conditional load or test made the
// compiler wait for every outstanding load, vmcnt(0), and for each LDS read
// in turn).  UG = 2 (UG 2 / 3 / 4: 2.85 / 2.89 / 2.95 ms key mode).
// A grid of one workgroup per CU takes pieces from a counter in range-major
// order (a piece of the same range keeps the LDS bitmap), so the chunk has no
// tail of late, unevenly sized workgroups (dynamic pieces).
// KEYM (key mode): LDS holds one byte per key of the range, the universe
// PC's low bits (0x7F: no universe PC) | covered << 7, so the per-PC work is
// still one LDS read: covered = byte >> 7, and the word's low bits must equal
// byte & 0x7F (membership, keys.hip); a word that fails sets
// SYZCOV_ERR_UNIVERSE.  Ranges are 2^17 keys (128 KB of bytes).
// The next batch's item descriptors are loaded while the current batch
// streams (short sub-runs at 32 ranges made their round trip per batch show).
template <int UG, bool KEYM = false>
__global__ __launch_bounds__(THREADS) void pass1_stream_kernel(Args A, uint32_t a, uint32_t b,
                                                               uint32_t P, int load_cov) {
    extern __shared__ uint32_t s_cov[];
    __shared__ uint32_t s_plan[MAX_R + 1];
    __shared__ uint64_t s_a0[NWAVE][64];   // 16-byte aligned base of the sub-run
    __shared__ uint32_t s_he[NWAVE][64];   // (end << 2) | head, in PCs from s_a0
    __shared__ uint32_t s_ex[NWAVE][64];   // first chunk of the item in the stream
    __shared__ int32_t s_rk[NWAVE][64];
    __shared__ uint32_t s_own[NWAVE][64];  // item + 1 starting at each chunk of a window
    __shared__ uint32_t s_next;
    const uint32_t G = A.npieces;
    s_own[threadIdx.x >> 6][__lane_id()] = 0u;
    plan_pieces(A, G, P, s_plan);
    const uint32_t region = blockIdx.x % NCTR;
    unsigned long long *const rctr = A.ctr + region * CTR_STRIDE;
    unsigned long long *const rrec = A.rec + region * A.cap_k;
    const uint32_t nwords = (1u << A.rshift) >> 5;
    const uint8_t *const s_cov8 = reinterpret_cast<const uint8_t *>(s_cov);
    uint32_t cur_rho = 0xFFFFFFFFu;
    uint32_t nonmem = 0;  // lanes that saw a word outside the universe (KEYM)
    for (;;) {
    if (threadIdx.x == 0) s_next = atomicAdd(A.pctr, 1u);
    __syncthreads();
    uint32_t g = s_next;
    __syncthreads();
    if (g >= G) break;
    {
        const uint32_t S = G / P;  // range-major: g = position * S + slice
        g = (g % S) * P + g / S;
    }
    uint32_t rho, i0, i1;
    if (!map_piece(A, G, P, a, b, g, &rho, &i0, &i1, s_plan)) continue;
    if (rho != cur_rho) {
        uint4 *s4 = reinterpret_cast<uint4 *>(s_cov);
        if (KEYM) {  // table bytes | covered << 7, 16 keys per uint4
            const uint32_t nq = (1u << A.rshift) >> 4;
            const uint4 *t4 = reinterpret_cast<const uint4 *>(A.low_of_key + ((uint64_t)rho << A.rshift));
            const uint32_t *cw = A.covered + (uint64_t)rho * nwords;
            for (uint32_t q = threadIdx.x; q < nq; q += THREADS) {
                uint4 t = t4[q];
                if (load_cov) {
                    const uint32_t cb = (cw[q >> 1] >> ((q & 1) * 16)) & 0xFFFFu;
                    auto spread = [](uint32_t x) {  // bit i -> bit 8i + 7
                        return ((x & 1u) << 7) | ((x & 2u) << 14) | ((x & 4u) << 21) |
                               ((x & 8u) << 28);
                    };
                    t.x |= spread(cb);
                    t.y |= spread(cb >> 4);
                    t.z |= spread(cb >> 8);
                    t.w |= spread(cb >> 12);
                }
                s4[q] = t;
            }
        } else {
            const uint4 *g4 = reinterpret_cast<const uint4 *>(A.covered + (uint64_t)rho * nwords);
            if (load_cov) {
                for (uint32_t q = threadIdx.x; q < nwords / 4; q += THREADS) s4[q] = g4[q];
            } else {
                for (uint32_t q = threadIdx.x; q < nwords / 4; q += THREADS)
                    s4[q] = make_uint4(0, 0, 0, 0);
            }
        }
        cur_rho = rho;
        __syncthreads();
    }
    const uint32_t l = __lane_id();
    const uint32_t w = wave_readfirstlane(threadIdx.x >> 6);
    const uint32_t rbase = rho << A.rshift;
    const uint32_t bmask = (1u << A.rshift) - 1u;
    const uint32_t per = (i1 - i0 + NWAVE - 1) / NWAVE;
    const uint32_t w0 = i0 + w * per, w1 = min(i1, w0 + per);
    // item descriptors of batch ib (lane l: item ib + l), loaded one batch ahead
    uint32_t d_s0 = 0, d_s1 = 0;
    uint64_t d_base = 0;
    int32_t d_rk = 0;
    auto load_desc = [&](uint32_t ib_) {
        const uint32_t item = ib_ + l;
        d_s0 = d_s1 = 0;
        d_base = 0;
        d_rk = 0;
        if (item < w1) {
            d_rk = A.ranks ? A.ranks[item] : (int32_t)item;
            d_s1 = A.split_t[(uint64_t)rho * A.n_items + item];
            d_s0 = rho ? A.split_t[(uint64_t)(rho - 1) * A.n_items + item] : 0u;
            d_base = A.base_r[item];
        }
    };
    if (w0 < w1) load_desc(w0);
    for (uint32_t ib = w0; ib < w1; ib += 64) {
        const uint32_t item = ib + l;
        uint32_t m = 0, nch = 0, he = 0;
        uint64_t a0 = 0;
        const int32_t rk = d_rk;
        if (item < w1) {
            // line-aligned: the sub-run owns its lines and starts on one (head 0)
            const uint64_t st = d_base + aligned_sub(d_s0, rho, A.ak);
            m = d_s1 - d_s0;
            a0 = st & ~3ull;
            const uint32_t head = (uint32_t)(st - a0);
            he = ((head + m) << 2) | head;
            nch = m ? (head + m + 3) >> 2 : 0u;
        }
        if (ib + 64 < w1) load_desc(ib + 64);
        const uint32_t incl = wave_incl_scan(nch);
        const uint32_t ex_l = incl - nch;  // lane j: item j's first chunk
        const uint32_t tot = wave_readlane(incl, 63);
        s_a0[w][l] = a0;
        s_he[w][l] = he;
        s_ex[w][l] = ex_l;
        s_rk[w][l] = rk;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        uint32_t sj = 0;  // uniform: the item covering the window's first chunk
        uint4 v[UG];
        uint32_t cj[UG], co[UG], hv[UG];  // item (64: past the end), chunk in it, its (end, head)
        auto issue = [&](uint32_t c0, uint4 (&dst)[UG], uint32_t (&dj)[UG], uint32_t (&dc)[UG],
                         uint32_t (&dh)[UG]) {
            uint32_t jj[UG];
#pragma unroll
            for (int u = 0; u < UG; u++) {
                const uint32_t cb = c0 + u * 64;  // uniform
                const uint32_t c = cb + l;
                // the item of chunk c is the last item starting at or before c:
                // items starting inside the window mark their start (max
                // index + 1: empty sub-runs share a start with the next item),
                // a prefix max over the lanes carries each mark forward, and
                // the item covering the previous window's last chunk (sj)
                // covers the chunks before the first mark
                if (ex_l - cb < 64u) atomicMax(&s_own[w][ex_l - cb], l + 1u);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
                const uint32_t mk = s_own[w][l];
                s_own[w][l] = 0u;
                const uint32_t pm = wave_incl_max(mk);
                const uint32_t j = pm ? max(sj, pm - 1u) : sj;
                sj = wave_readlane(j, 63);
                jj[u] = j;
                dj[u] = c < tot ? j : 64u;
            }
            uint64_t ba[UG];
            uint32_t bx[UG];
#pragma unroll
            for (int u = 0; u < UG; u++) {
                ba[u] = s_a0[w][jj[u]];
                bx[u] = s_ex[w][jj[u]];
                dh[u] = s_he[w][jj[u]];
            }
#pragma unroll
            for (int u = 0; u < UG; u++) {
                const uint32_t c = c0 + u * 64 + l;
                dc[u] = dj[u] < 64 ? c - bx[u] : 0u;  // past the end: chunk 0, never tested
                dst[u] = reinterpret_cast<const uint4 *>(A.pcs + ba[u])[dc[u]];
            }
        };
        // unconditional: chunks past the end load a valid line and are never
        // tested, and straight-line loads keep the compiler's vmcnt exact
        issue(0, v, cj, co, hv);
        for (uint32_t c0 = 0; c0 < tot; c0 += 64 * UG) {
            uint4 vn[UG];
            uint32_t nj[UG], nc[UG], nh[UG];
            issue(c0 + 64 * UG, vn, nj, nc, nh);
            // the next chunks' loads stay ahead of the current ones' tests
            const uint32_t kmask = issue_fence(A.keymask);
            uint32_t um = 0;
            uint32_t wv[UG * 4], bit[UG * 4];
#pragma unroll
            for (int u = 0; u < UG; u++) {
                const uint32_t vv[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    bit[u * 4 + k] = ((vv[k] & kmask) - A.pc_lo - rbase) & bmask;
                    wv[u * 4 + k] = KEYM ? (uint32_t)s_cov8[bit[u * 4 + k]]
                                         : s_cov[bit[u * 4 + k] >> 5];
                }
            }
#pragma unroll
            for (int u = 0; u < UG; u++) {
                const uint32_t head = hv[u] & 3u, end = hv[u] >> 2;
                const uint32_t vv[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t idx = co[u] * 4 + k;
                    const uint32_t valid =
                        (uint32_t)(cj[u] < 64) & (uint32_t)(idx >= head) & (uint32_t)(idx < end);
                    uint32_t unc;
                    if (KEYM) {
                        const uint32_t t = wv[u * 4 + k];
                        unc = (~t >> 7) & 1u;
                        nonmem |= valid & (uint32_t)((t & 0x7Fu) != (vv[k] >> SYZ_KEY_BITS));
                    } else {
                        unc = ~(wv[u * 4 + k] >> (bit[u * 4 + k] & 31)) & 1u;
                    }
                    um |= (valid & unc) << (u * 4 + k);
                }
            }
            if (__ballot(um != 0)) {
                const uint32_t cnt = (uint32_t)__popc(um);
                const uint32_t inc2 = wave_incl_scan(cnt);
                const uint32_t t2 = __shfl(inc2, 63, 64);
                unsigned long long basei = 0;
                if (l == 0) basei = atomicAdd(rctr, (unsigned long long)t2);
                uint64_t slot = __shfl(basei, 0, 64) + (inc2 - cnt);
                if (um) {
#pragma unroll
                    for (int u = 0; u < UG; u++) {
                        if (!((um >> (u * 4)) & 15u)) continue;
                        const int32_t rki = s_rk[w][cj[u]];
                        A.cand[ib + cj[u]] = 1;
                        const uint32_t vv[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                        for (int k = 0; k < 4; k++)
                            if ((um >> (u * 4 + k)) & 1u) {
                                const uint32_t wo =
                                    (vv[k] & A.keymask) - A.pc_lo;
                                if (slot < A.cap_k)
                                    rrec[slot] = ((unsigned long long)(uint32_t)rki << 32) | wo;
                                else  // no room: its min cannot wait
                                    atomicMin(&A.first_w[wo], rki);
                                slot++;
                            }
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < UG; u++) {
                v[u] = vn[u];
                cj[u] = nj[u];
                co[u] = nc[u];
                hv[u] = nh[u];
            }
        }
        // the next batch rewrites this wave's descriptors
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();  // every wave is done before the LDS bitmap is replaced
    }
    if (KEYM && __ballot(nonmem) && __lane_id() == 0) atomicOr(A.err, SYZCOV_ERR_UNIVERSE);
}

// Key mode pass 1 (the corpus engine's path), the chunk stream above with
// fewer vector operations per PC (pass 1 measured VALU-bound: ~18 VALU
// instructions per PC per lane, 57% of wave cycles waiting, at C2):
//  - 32-byte lane chunks (two 16-byte loads), so the per-chunk item lookup
//    (marks, DPP prefix max, descriptor reads) is paid once per 8 PCs;
//  - the staged byte is low | UNcovered << 7 (bit 7 set for a key no earlier
//    chunk covered), so "covered and a universe PC" is one compare of the
//    byte with the word's low bits: the byte index is the word & (2^17 - 1)
//    (key - range base, the low bits above bit 25 masked off), and the common
//    case (every PC covered and valid) costs an and, a shift, a compare and the
//    element's bounds test;
//  - anything else (uncovered: a record; covered but not the universe PC:
//    SYZCOV_ERR_UNIVERSE) is sorted out on a rare, wave-uniform slow path.
// A record's membership is checked there too (its byte's low 7 bits).
// N4 (kshift <= 2, ranges of 2^18 keys): the table entry is a NIBBLE, the
// universe PC's low bits (7: none) | UNcovered << 3, 2^18 of them in the same
// 128 KB — half the ranges of the byte table, so half the sub-run boundary
// lines (C2X: 32 ranges instead of 64); a low value never reaches 7.
template <int UG, bool N4 = false>
__global__ __launch_bounds__(THREADS) void pass1_keys_kernel(Args A, uint32_t a, uint32_t b,
                                                             uint32_t P, int load_cov) {
    constexpr uint32_t CW = 8;  // words per lane chunk
    constexpr uint32_t LOWM = N4 ? 7u : 0x7Fu, USH = N4 ? 3u : 7u;  // entry: low | unc << USH
    // one dynamic block, the range's table at LDS address 0 so that a
    // table read is ds_read_u8 of (word & mask) with no base add; then
    // (KEYS_LDS_EXTRA bytes) the wave descriptors and the piece plan
    extern __shared__ uint32_t s_cov[];
    auto *s_a0 = reinterpret_cast<uint64_t(*)[64]>(
        reinterpret_cast<uint8_t *>(s_cov) + ((size_t)1 << 17));   // 32-byte aligned base
    auto *s_he = reinterpret_cast<uint32_t(*)[64]>(s_a0 + NWAVE);  // (end << 3) | head
    auto *s_ex = s_he + NWAVE;                                     // first chunk of the item
    auto *s_rk = reinterpret_cast<int32_t(*)[64]>(s_ex + NWAVE);
    auto *s_own = reinterpret_cast<uint32_t(*)[64]>(s_rk + NWAVE); // item + 1 per chunk
    uint32_t *s_plan = reinterpret_cast<uint32_t *>(s_own + NWAVE);
    uint32_t &s_next = s_plan[MAX_R + 1];
    uint32_t *s_bh = s_plan + MAX_R + 2;  // this workgroup's records per key bucket
    const uint32_t G = A.npieces;
    s_own[threadIdx.x >> 6][__lane_id()] = 0u;
    if (A.bh)
        for (uint32_t i = threadIdx.x; i < A.nb; i += THREADS) s_bh[i] = 0u;
    plan_pieces(A, G, P, s_plan);
    const uint32_t region = blockIdx.x % NCTR;
    unsigned long long *const rctr = A.ctr + region * CTR_STRIDE;
    unsigned long long *const rrec = A.rec + region * A.cap_k;
    const uint8_t *const s_cov8 = reinterpret_cast<const uint8_t *>(s_cov);
    const uint32_t bmask = (1u << A.rshift) - 1u;
    uint32_t cur_rho = 0xFFFFFFFFu;
    uint32_t nonmem = 0;
    uint32_t xdone = 0;  // (thread 0) XCDs whose slices are all drawn
    for (;;) {
    if (threadIdx.x == 0) s_next = draw_piece(A.pctr, G, P, &xdone);
    __syncthreads();
    uint32_t g = s_next;
    __syncthreads();
    if (g >= G) break;
    uint32_t rho, i0, i1;
    if (!map_piece(A, G, P, a, b, g, &rho, &i0, &i1, s_plan)) continue;
    if (N4 && rho != cur_rho) {  // nibbles: 8 keys per word from 8 bytes + a covered byte
        const uint32_t nq = (1u << A.rshift) >> 3;
        const uint2 *t2 = reinterpret_cast<const uint2 *>(A.low_of_key + ((uint64_t)rho << A.rshift));
        const uint8_t *cb8 =
            reinterpret_cast<const uint8_t *>(A.covered) + (((uint64_t)rho << A.rshift) >> 3);
        constexpr uint32_t TL = 8;  // all of a thread's loads first (below)
        for (uint32_t q0 = 0; q0 < nq; q0 += TL * THREADS) {
            uint2 lb[TL];
            uint32_t unc[TL];
#pragma unroll
            for (uint32_t u = 0; u < TL; u++) {
                const uint32_t q = q0 + u * THREADS + threadIdx.x;
                lb[u] = q < nq ? t2[q] : make_uint2(0, 0);
                unc[u] = load_cov && q < nq ? ~(uint32_t)cb8[q] : 0xFFu;
            }
#pragma unroll
            for (uint32_t u = 0; u < TL; u++) {
                const uint32_t q = q0 + u * THREADS + threadIdx.x;
                uint32_t x = 0;
#pragma unroll
                for (uint32_t j = 0; j < 8; j++) {
                    const uint32_t low =
                        ((j < 4 ? lb[u].x >> (8 * j) : lb[u].y >> (8 * (j - 4)))) & 7u;
                    x |= (low | (((unc[u] >> j) & 1u) << 3)) << (4 * j);
                }
                if (q < nq) s_cov[q] = x;
            }
        }
        cur_rho = rho;
        __syncthreads();
    }
    if (!N4 && rho != cur_rho) {  // table bytes | UNcovered << 7, 16 keys per uint4
        uint4 *s4 = reinterpret_cast<uint4 *>(s_cov);
        const uint32_t nq = (1u << A.rshift) >> 4;
        const uint4 *t4 = reinterpret_cast<const uint4 *>(A.low_of_key + ((uint64_t)rho << A.rshift));
        const uint32_t *cw = A.covered + ((uint64_t)rho << A.rshift) / 32;
        auto spread = [](uint32_t x) {  // bit i -> bit 8i + 7
            return ((x & 1u) << 7) | ((x & 2u) << 14) | ((x & 4u) << 21) | ((x & 8u) << 28);
        };
        // all of a thread's loads first (8 per thread at 2^17 keys): a piece
        // change reloads the table, and a loop of dependent round trips made
        // that a visible share of a 2 MB piece
        constexpr uint32_t TL = 8;
        for (uint32_t q0 = 0; q0 < nq; q0 += TL * THREADS) {
            uint4 t[TL];
            uint32_t cv[TL];
#pragma unroll
            for (uint32_t u = 0; u < TL; u++) {
                const uint32_t q = q0 + u * THREADS + threadIdx.x;
                t[u] = q < nq ? t4[q] : make_uint4(0, 0, 0, 0);
                cv[u] = load_cov && q < nq ? cw[q >> 1] : 0u;
            }
#pragma unroll
            for (uint32_t u = 0; u < TL; u++) {
                const uint32_t q = q0 + u * THREADS + threadIdx.x;
                const uint32_t ub = ~(cv[u] >> ((q & 1) * 16)) & 0xFFFFu;
                t[u].x |= spread(ub);
                t[u].y |= spread(ub >> 4);
                t[u].z |= spread(ub >> 8);
                t[u].w |= spread(ub >> 12);
                if (q < nq) s4[q] = t[u];
            }
        }
        cur_rho = rho;
        __syncthreads();
    }
    const uint32_t l = __lane_id();
    const uint32_t w = wave_readfirstlane(threadIdx.x >> 6);
    const uint32_t per = (i1 - i0 + NWAVE - 1) / NWAVE;
    const uint32_t w0 = i0 + w * per, w1 = min(i1, w0 + per);
    uint32_t d_s0 = 0, d_s1 = 0;
    uint64_t d_base = 0;
    int32_t d_rk = 0;
    auto load_desc = [&](uint32_t ib_) {
        const uint32_t item = ib_ + l;
        d_s0 = d_s1 = 0;
        d_base = 0;
        d_rk = 0;
        if (item < w1) {
            d_rk = A.ranks ? A.ranks[item] : (int32_t)item;
            d_s1 = A.split_t[(uint64_t)rho * A.n_items + item];
            d_s0 = rho ? A.split_t[(uint64_t)(rho - 1) * A.n_items + item] : 0u;
            d_base = A.base_r[item];
        }
    };
    if (w0 < w1) load_desc(w0);
    for (uint32_t ib = w0; ib < w1; ib += 64) {
        const uint32_t item = ib + l;
        uint32_t m = 0, nch = 0, he = 0;
        uint64_t a0 = 0;
        const int32_t rk = d_rk;
        if (item < w1) {
            const uint64_t st = d_base + aligned_sub(d_s0, rho, A.ak);
            m = d_s1 - d_s0;
            a0 = st & ~7ull;
            const uint32_t head = (uint32_t)(st - a0);
            he = ((head + m) << 3) | head;
            nch = m ? (head + m + CW - 1) / CW : 0u;
        }
        if (ib + 64 < w1) load_desc(ib + 64);
        const uint32_t incl = wave_incl_scan(nch);
        const uint32_t ex_l = incl - nch;
        const uint32_t tot = wave_readlane(incl, 63);
        s_a0[w][l] = a0;
        s_he[w][l] = he;
        s_ex[w][l] = ex_l;
        s_rk[w][l] = rk;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        uint32_t sj = 0;
        uint4 v0[UG], v1[UG];
        uint32_t cj[UG], co[UG], hv[UG];
        auto issue = [&](uint32_t c0, uint4 (&d0)[UG], uint4 (&d1)[UG], uint32_t (&dj)[UG],
                         uint32_t (&dc)[UG], uint32_t (&dh)[UG]) {
            uint32_t jj[UG];
#pragma unroll
            for (int u = 0; u < UG; u++) {
                const uint32_t cb = c0 + u * 64;
                const uint32_t c = cb + l;
                if (ex_l - cb < 64u) atomicMax(&s_own[w][ex_l - cb], l + 1u);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
                const uint32_t mk = s_own[w][l];
                s_own[w][l] = 0u;
                const uint32_t pm = wave_incl_max(mk);
                const uint32_t j = pm ? max(sj, pm - 1u) : sj;
                sj = wave_readlane(j, 63);
                jj[u] = j;
                dj[u] = c < tot ? j : 64u;
            }
            uint64_t ba[UG];
            uint32_t bx[UG];
#pragma unroll
            for (int u = 0; u < UG; u++) {
                ba[u] = s_a0[w][jj[u]];
                bx[u] = s_ex[w][jj[u]];
                dh[u] = s_he[w][jj[u]];
            }
#pragma unroll
            for (int u = 0; u < UG; u++) {
                const uint32_t c = c0 + u * 64 + l;
                dc[u] = dj[u] < 64 ? c - bx[u] : 0u;  // past the end: chunk 0, never tested
                const uint4 *p = reinterpret_cast<const uint4 *>(A.pcs + ba[u]) + 2 * dc[u];
                d0[u] = p[0];
                // the second half only if it holds words of the sub-run (no
                // read further past a sub-run's end than a 16-byte chunk's)
                d1[u] = p[dc[u] * CW + 4 < (dh[u] >> 3) ? 1 : 0];
            }
        };
        issue(0, v0, v1, cj, co, hv);
        for (uint32_t c0 = 0; c0 < tot; c0 += 64 * UG) {
            uint4 n0[UG], n1[UG];
            uint32_t nj[UG], nc[UG], nh[UG];
            issue(c0 + 64 * UG, n0, n1, nj, nc, nh);
            const uint32_t bm = issue_fence(bmask);
            uint32_t wd[UG * CW], tb[UG * CW];
#pragma unroll
            for (int u = 0; u < UG; u++) {
                const uint32_t vv[CW] = {v0[u].x, v0[u].y, v0[u].z, v0[u].w,
                                         v1[u].x, v1[u].y, v1[u].z, v1[u].w};
#pragma unroll
                for (int k = 0; k < (int)CW; k++) {
                    wd[u * CW + k] = vv[k];
                    if (N4) {
                        const uint32_t o = vv[k] & bm;
                        tb[u * CW + k] = (s_cov[o >> 3] >> ((o & 7u) << 2)) & 15u;
                    } else {
                        tb[u * CW + k] = s_cov8[vv[k] & bm];
                    }
                }
            }
            // element k of a lane's chunk is in its sub-run iff lo <= k < hi
            int lo[UG];
            uint32_t span[UG];
#pragma unroll
            for (int u = 0; u < UG; u++) {
                lo[u] = (int)(hv[u] & 7u) - (int)(co[u] * CW);
                const int hi = cj[u] < 64 ? (int)(hv[u] >> 3) - (int)(co[u] * CW) : lo[u];
                span[u] = (uint32_t)(hi - lo[u]);
            }
            bool any = false;
#pragma unroll
            for (int u = 0; u < UG; u++)
#pragma unroll
                for (int k = 0; k < (int)CW; k++)
                    any |= ((uint32_t)(k - lo[u]) < span[u]) &
                           (tb[u * CW + k] != (wd[u * CW + k] >> SYZ_KEY_BITS));
            if (__ballot(any)) {  // rare once the early chunks are done
                uint32_t um = 0;  // records: uncovered elements
#pragma unroll
                for (int u = 0; u < UG; u++)
#pragma unroll
                    for (int k = 0; k < (int)CW; k++) {
                        const uint32_t t = tb[u * CW + k], lw = wd[u * CW + k] >> SYZ_KEY_BITS;
                        const uint32_t in = (uint32_t)((uint32_t)(k - lo[u]) < span[u]) &
                                            (uint32_t)(t != lw);
                        nonmem |= in & (uint32_t)((t & LOWM) != lw);
                        um |= (in & (t >> USH)) << (u * CW + k);
                    }
                if (__ballot(um != 0)) {
                    const uint32_t cnt = (uint32_t)__popc(um);
                    const uint32_t inc2 = wave_incl_scan(cnt);
                    const uint32_t t2 = __shfl(inc2, 63, 64);
                    unsigned long long basei = 0;
                    if (l == 0) basei = atomicAdd(rctr, (unsigned long long)t2);
                    uint64_t slot = __shfl(basei, 0, 64) + (inc2 - cnt);
                    if (um) {
#pragma unroll
                        for (int u = 0; u < UG; u++) {
                            if (!((um >> (u * CW)) & 0xFFu)) continue;
                            const int32_t rki = s_rk[w][cj[u]];
                            A.cand[ib + cj[u]] = 1;
#pragma unroll
                            for (int k = 0; k < (int)CW; k++)
                                if ((um >> (u * CW + k)) & 1u) {
                                    const uint32_t wo = wd[u * CW + k] & SYZ_KEY_MASK;
                                    if (slot < A.cap_k) {
                                        rrec[slot] = ((unsigned long long)(uint32_t)rki << 32) | wo;
                                        if (A.bh) atomicAdd(&s_bh[wo >> BSH], 1u);
                                    } else {  // no room: its min cannot wait
                                        atomicMin(&A.first_w[wo], rki);
                                    }
                                    slot++;
                                }
                        }
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < UG; u++) {
                v0[u] = n0[u];
                v1[u] = n1[u];
                cj[u] = nj[u];
                co[u] = nc[u];
                hv[u] = nh[u];
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    }
    if (__ballot(nonmem) && __lane_id() == 0) atomicOr(A.err, SYZCOV_ERR_UNIVERSE);
    if (A.bh) {  // (the piece loop ended on a barrier)
        for (uint32_t i = threadIdx.x; i < A.nb; i += THREADS)
            if (s_bh[i]) atomicAdd(&A.bh[i], s_bh[i]);
    }
}

// ---- The initial block: exact first covers of items [a, a + K) in LDS.
// The geometric chunks start small because every uncovered occurrence of a
// chunk becomes a record, and at the start nearly every occurrence is
// uncovered: at a C3/8 rank the first five chunks (21.8 K items, 1.7 % of
// the bytes) took 0.47 ms of pass 1 + rec_scatter + bmin, ~17 % of its
// Minimize.  Nothing precedes the block, so a key's first cover there is the
// minimum item holding it, which a min table finds without records:
// init_min_kernel: workgroup (piece, q) streams the range-rho sub-runs of
// one part of the block's items (pass1_keys_kernel's chunk stream; a range
// gets parts in proportion to its key count, plan_pieces) and keeps, for
// each key of part q of the range (2^IQ_SH keys, 128 KB of u32),
// min((item - a) << 7 | low bits) in LDS.  An entry starts as
// (INIT_NONE << 7) | low_of_key, so a word whose low bits differ from its
// entry's is not a universe PC (SYZCOV_ERR_UNIVERSE, as pass 1).  The parts
// of a range meet in the scratch table tab[key] by a global atomicMin per
// held key.  The q parts of one range read the same sub-runs: they and the
// neighbouring ranges run on one XCD (workgroup b on XCD b mod 8), so the
// re-reads are L2 hits.
// init_flush_kernel: per key, tab's minimum is the key's first cover ->
// first_w, the covered words, and ONE record (rank, key) per covered
// key, pass 2's evidence (kept(r) <=> first(k) == r for some key k; across
// shards, a key's global first cover on this shard is its local one).  A
// record that finds its region full flags its item as a candidate (the
// overflow fallback rescans candidates), as in pass 1.
constexpr uint32_t IQ_SH = 15;             // keys per init table: 2^15 u32 (128 KB)
constexpr uint32_t INIT_NONE = 0xFFFFFFu;  // entry >> 7 of a key no item of the block holds
constexpr size_t INIT_LDS_EXTRA = NWAVE * 64 * (8 + 3 * 4) + (MAX_R + 2) * 4;

template <int UG>
__global__ __launch_bounds__(THREADS) void init_min_kernel(Args A, uint32_t a, uint32_t K, uint32_t P,
                                                           uint32_t *__restrict__ tab) {
    constexpr uint32_t CW = 8;  // words per lane chunk
    extern __shared__ uint32_t s_tab[];  // 2^IQ_SH entries at LDS 0, then the wave descriptors
    auto *s_a0 = reinterpret_cast<uint64_t(*)[64]>(
        reinterpret_cast<uint8_t *>(s_tab) + ((size_t)4 << IQ_SH));
    auto *s_he = reinterpret_cast<uint32_t(*)[64]>(s_a0 + NWAVE);  // (end << 3) | head
    auto *s_ex = s_he + NWAVE;                                     // first chunk of the item
    auto *s_own = s_ex + NWAVE;                                    // item + 1 per chunk
    uint32_t *s_plan = reinterpret_cast<uint32_t *>(s_own + NWAVE);
    // workgroup -> (piece, part q of the range's keys); the pieces of a range
    // and its neighbours' on one XCD
    const uint32_t nq = 1u << (A.rshift - IQ_SH);
    uint32_t idx = blockIdx.x;
    if ((gridDim.x & 7u) == 0) idx = (blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    const uint32_t pi = idx / nq, q = idx % nq;
    // P pieces over the ranges by their key counts (plan_pieces): range j's
    // items are cut into p_j parts (one range per workgroup took 6.1 ms for
    // 87 K items, the hot ranges' workgroups alone)
    plan_pieces(A, 0, P, s_plan);
    if (pi >= s_plan[A.nrange]) return;
    uint32_t rho = 0, hi_ = A.nrange;  // largest j with sh[j] <= pi
    while (hi_ - rho > 1) {
        const uint32_t mid = (rho + hi_) >> 1;
        if (s_plan[mid] <= pi) rho = mid; else hi_ = mid;
    }
    const uint32_t parts = s_plan[rho + 1] - s_plan[rho], part = pi - s_plan[rho];
    const uint32_t k0 = (rho << A.rshift) + (q << IQ_SH);  // the table's first key
    s_own[threadIdx.x >> 6][__lane_id()] = 0u;
    {  // entries (INIT_NONE << 7) | low, 16 keys per 16-byte load
        const uint4 *lk = reinterpret_cast<const uint4 *>(A.low_of_key + k0);
        for (uint32_t i = threadIdx.x; i < (1u << IQ_SH) / 16; i += THREADS) {
            const uint4 v = lk[i];
            const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
            uint4 *d = reinterpret_cast<uint4 *>(s_tab + 16 * i);
#pragma unroll
            for (int j = 0; j < 4; j++)
                d[j] = make_uint4(INIT_NONE << 7 | (w4[j] & 0xFFu), INIT_NONE << 7 | (w4[j] >> 8 & 0xFFu),
                                  INIT_NONE << 7 | (w4[j] >> 16 & 0xFFu), INIT_NONE << 7 | (w4[j] >> 24));
        }
    }
    __syncthreads();
    const uint32_t i0 = a + (uint32_t)((uint64_t)K * part / parts),
                   i1 = a + (uint32_t)((uint64_t)K * (part + 1) / parts);
    const uint32_t bmask = (1u << A.rshift) - 1u, qoff = q << IQ_SH;
    uint32_t nonmem = 0;
    const uint32_t l = __lane_id();
    const uint32_t w = wave_readfirstlane(threadIdx.x >> 6);
    const uint32_t per = (i1 - i0 + NWAVE - 1) / NWAVE;
    const uint32_t w0 = i0 + w * per, w1 = min(i1, w0 + per);
    uint32_t d_s0 = 0, d_s1 = 0;
    uint64_t d_base = 0;
    auto load_desc = [&](uint32_t ib_) {
        const uint32_t item = ib_ + l;
        d_s0 = d_s1 = 0;
        d_base = 0;
        if (item < w1) {
            d_s1 = A.split_t[(uint64_t)rho * A.n_items + item];
            d_s0 = rho ? A.split_t[(uint64_t)(rho - 1) * A.n_items + item] : 0u;
            d_base = A.base_r[item];
        }
    };
    if (w0 < w1) load_desc(w0);
    for (uint32_t ib = w0; ib < w1; ib += 64) {
        const uint32_t item = ib + l;
        uint32_t m = 0, nch = 0, he = 0;
        uint64_t a0 = 0;
        if (item < w1) {
            const uint64_t st = d_base + aligned_sub(d_s0, rho, A.ak);
            m = d_s1 - d_s0;
            a0 = st & ~7ull;
            const uint32_t head = (uint32_t)(st - a0);
            he = ((head + m) << 3) | head;
            nch = m ? (head + m + CW - 1) / CW : 0u;
        }
        if (ib + 64 < w1) load_desc(ib + 64);
        const uint32_t incl = wave_incl_scan(nch);
        const uint32_t ex_l = incl - nch;
        const uint32_t tot = wave_readlane(incl, 63);
        s_a0[w][l] = a0;
        s_he[w][l] = he;
        s_ex[w][l] = ex_l;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        uint32_t sj = 0;
        uint4 v0[UG], v1[UG];
        uint32_t cj[UG], co[UG], hv[UG];
        auto issue = [&](uint32_t c0, uint4 (&d0)[UG], uint4 (&d1)[UG], uint32_t (&dj)[UG],
                         uint32_t (&dc)[UG], uint32_t (&dh)[UG]) {
            uint32_t jj[UG];
#pragma unroll
            for (int u = 0; u < UG; u++) {
                const uint32_t cb = c0 + u * 64;
                const uint32_t c = cb + l;
                if (ex_l - cb < 64u) atomicMax(&s_own[w][ex_l - cb], l + 1u);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
                const uint32_t mk = s_own[w][l];
                s_own[w][l] = 0u;
                const uint32_t pm = wave_incl_max(mk);
                const uint32_t j = pm ? max(sj, pm - 1u) : sj;
                sj = wave_readlane(j, 63);
                jj[u] = j;
                dj[u] = c < tot ? j : 64u;
            }
            uint64_t ba[UG];
            uint32_t bx[UG];
#pragma unroll
            for (int u = 0; u < UG; u++) {
                ba[u] = s_a0[w][jj[u]];
                bx[u] = s_ex[w][jj[u]];
                dh[u] = s_he[w][jj[u]];
            }
#pragma unroll
            for (int u = 0; u < UG; u++) {
                const uint32_t c = c0 + u * 64 + l;
                dc[u] = dj[u] < 64 ? c - bx[u] : 0u;  // past the end: chunk 0, never used
                const uint4 *p = reinterpret_cast<const uint4 *>(A.pcs + ba[u]) + 2 * dc[u];
                d0[u] = p[0];
                d1[u] = p[dc[u] * CW + 4 < (dh[u] >> 3) ? 1 : 0];
            }
        };
        issue(0, v0, v1, cj, co, hv);
        for (uint32_t c0 = 0; c0 < tot; c0 += 64 * UG) {
            uint4 n0[UG], n1[UG];
            uint32_t nj[UG], nc[UG], nh[UG];
            issue(c0 + 64 * UG, n0, n1, nj, nc, nh);
            const uint32_t bm = issue_fence(bmask);
            // every table read unconditional and issued together (a read or
            // an atomic under a per-element branch waits for each LDS access,
            // and for every outstanding load, in turn): entries at a clamped
            // index, then the element tests; a lower value than the entry's
            // (the first items of a key, rare past the start) takes ds_min on
            // a wave-uniform slow path.  The read first also spares the hot
            // keys (in nearly every item) whole wave instructions of ds_min
            // serialised on one address.
            uint32_t wd[UG * CW], tb[UG * CW], vl[UG * CW];
            uint32_t need = 0;
#pragma unroll
            for (int u = 0; u < UG; u++) {
                const uint32_t vv[CW] = {v0[u].x, v0[u].y, v0[u].z, v0[u].w,
                                         v1[u].x, v1[u].y, v1[u].z, v1[u].w};
#pragma unroll
                for (int k = 0; k < (int)CW; k++) {
                    wd[u * CW + k] = (vv[k] & bm) - qoff;
                    tb[u * CW + k] = s_tab[wd[u * CW + k] & ((1u << IQ_SH) - 1u)];
                }
                // element k of the lane's chunk is in its sub-run iff lo <= k < hi
                const int lo = (int)(hv[u] & 7u) - (int)(co[u] * CW);
                const int hi = cj[u] < 64 ? (int)(hv[u] >> 3) - (int)(co[u] * CW) : lo;
                const uint32_t lr = ib + cj[u] - a;  // the item, block-relative
#pragma unroll
                for (int k = 0; k < (int)CW; k++) {
                    const uint32_t lw = vv[k] >> SYZ_KEY_BITS, v = lr << 7 | lw;
                    const uint32_t in = (uint32_t)(k >= lo) & (uint32_t)(k < hi) &
                                        (uint32_t)(wd[u * CW + k] < (1u << IQ_SH));
                    nonmem |= in & (uint32_t)((tb[u * CW + k] & 0x7Fu) != lw);
                    need |= (in & (uint32_t)(v < tb[u * CW + k])) << (u * CW + k);
                    vl[u * CW + k] = v;
                }
            }
            if (__ballot(need != 0)) {
#pragma unroll
                for (int j = 0; j < UG * (int)CW; j++)
                    if ((need >> j) & 1u) atomicMin(&s_tab[wd[j]], vl[j]);
            }
#pragma unroll
            for (int u = 0; u < UG; u++) {
                v0[u] = n0[u];
                v1[u] = n1[u];
                cj[u] = nj[u];
                co[u] = nc[u];
                hv[u] = nh[u];
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    if (__ballot(nonmem) && __lane_id() == 0) atomicOr(A.err, SYZCOV_ERR_UNIVERSE);
    __syncthreads();
    // the parts of a range meet in tab (all ones before the kernel)
    for (uint32_t i = threadIdx.x; i < (1u << IQ_SH); i += THREADS) {
        const uint32_t e = s_tab[i];
        if ((e >> 7) != INIT_NONE) atomicMin(&tab[k0 + i], e);
    }
}

__global__ __launch_bounds__(256) void init_flush_kernel(Args A, uint32_t a,
                                                         const uint32_t *__restrict__ tab, uint64_t T,
                                                         uint64_t span) {
    const uint32_t region = blockIdx.x % NCTR;
    unsigned long long *const rctr = A.ctr + region * CTR_STRIDE;
    unsigned long long *const rrec = A.rec + region * A.cap_k;
    uint32_t *const covered = const_cast<uint32_t *>(A.covered);
    const uint32_t l = __lane_id();
    for (uint64_t key = (uint64_t)blockIdx.x * 256 + threadIdx.x; key - threadIdx.x < T;
         key += (uint64_t)gridDim.x * 256) {
        const uint32_t lr = key < T ? tab[key] >> 7 : INIT_NONE;
        const bool has = key < span && lr < INIT_NONE;  // (past the span: flagged by init_min)
        const int32_t rank = has ? (A.ranks ? A.ranks[a + lr] : (int32_t)(a + lr)) : INT32_MAX;
        if (key < span) A.first_w[key] = rank;
        const uint64_t m = __ballot(has);
        if ((l & 31) == 0 && key < T) covered[key >> 5] = (uint32_t)(m >> (l & 32));
        if (m) {  // one reservation per wave
            unsigned long long b0 = 0;
            if (l == 0) b0 = atomicAdd(rctr, (unsigned long long)__popcll(m));
            b0 = __shfl(b0, 0, 64);
            if (has) {
                const uint64_t slot = b0 + __popcll(m & ((1ull << l) - 1ull));
                if (slot < A.cap_k)
                    rrec[slot] = (unsigned long long)(uint32_t)rank << 32 | (uint32_t)key;
                else
                    A.cand[a + lr] = 1;  // no room: the overflow fallback rescans the item
            }
        }
    }
}

// the first chunk's records start after the block's: done marks (parity 0) = ctr
__global__ void init_done_kernel(Args A) {
    const uint32_t k = threadIdx.x;
    if (k < NCTR) A.done[k * CTR_STRIDE] = std::min<uint64_t>(A.ctr[k * CTR_STRIDE], A.cap_k);
}

// Manager.minimizeCorpus (syz-manager/manager.go:504-524) when every call
// group is small: per group, exact first covers in LDS, with no chunks and
// no records.  Piece (g, rho): a workgroup streams the range-rho sub-runs of
// every item of group g (ranks [goff[g], goff[g+1]) of the grouped order,
// key words of ranges of 2^rshift <= 2^15 keys) and takes ds_min(first[key -
// rho base], local rank) in a 128 KB table; every entry holding a rank is
// the first cover of its key in the group, so that rank is kept (cover.go:
// 114-129 keeps an input iff it holds a PC no earlier input of its Minimize
// call holds).  Ranks are flagged in an LDS bitmap first (an item is the
// first cover of many keys), then written out once per piece.  The stream is
// pass1_keys_kernel's (32-byte lane chunks, marks + DPP for the item of a
// chunk).
constexpr uint32_t GM_TAB = 1u << 15;           // keys per piece (int32 ranks)
constexpr uint32_t GM_MAX_ITEMS = 1u << 16;     // items per group on this path
struct GmArgs {
    const uint32_t *words;      // key words (common.h), CSR slots
    const uint64_t *base_r;     // [items] off[order[j]] (prep_kernel)
    const uint32_t *split_t;    // [nrange][items] split[order[j]][rho]
    const uint64_t *goff;       // [ngroups + 1] rank intervals of the groups
    uint32_t n_items, ngroups, nrange, rshift;
    uint32_t *pctr;             // next piece
    uint8_t *kept;              // [n_items] by rank
};

__global__ __launch_bounds__(THREADS) void group_min_kernel(GmArgs A) {
    constexpr uint32_t CW = 8;
    extern __shared__ uint32_t s_tab[];  // GM_TAB ranks at LDS 0, then:
    auto *s_a0 = reinterpret_cast<uint64_t(*)[64]>(s_tab + GM_TAB);
    auto *s_he = reinterpret_cast<uint32_t(*)[64]>(s_a0 + NWAVE);
    auto *s_ex = s_he + NWAVE;
    auto *s_own = s_ex + NWAVE;
    uint32_t *s_bits = reinterpret_cast<uint32_t *>(s_own + NWAVE);  // GM_MAX_ITEMS bits
    uint32_t &s_next = s_bits[GM_MAX_ITEMS / 32];
    const uint32_t l = __lane_id();
    const uint32_t w = wave_readfirstlane(threadIdx.x >> 6);
    s_own[w][l] = 0u;
    const uint32_t npieces = A.ngroups * A.nrange;
    const uint32_t kmask = (1u << A.rshift) - 1u;
    for (;;) {
        if (threadIdx.x == 0) s_next = atomicAdd(A.pctr, 1u);
        __syncthreads();
        const uint32_t p = s_next;
        __syncthreads();
        if (p >= npieces) break;
        const uint32_t g = p / A.nrange, rho = p - g * A.nrange;
        const uint32_t i0 = (uint32_t)A.goff[g], i1 = (uint32_t)A.goff[g + 1];
        if (i1 <= i0) continue;
        for (uint32_t q = threadIdx.x; q < GM_TAB / 4; q += THREADS)
            reinterpret_cast<uint4 *>(s_tab)[q] = make_uint4(~0u, ~0u, ~0u, ~0u);
        for (uint32_t q = threadIdx.x; q < (i1 - i0 + 31) / 32; q += THREADS) s_bits[q] = 0u;
        __syncthreads();
        const uint32_t per = (i1 - i0 + NWAVE - 1) / NWAVE;
        const uint32_t w0 = i0 + w * per, w1 = min(i1, w0 + per);
        for (uint32_t ib = w0; ib < w1; ib += 64) {
            const uint32_t item = ib + l;
            uint32_t nch = 0, he = 0;
            uint64_t a0 = 0;
            if (item < w1) {
                const uint32_t s1 = A.split_t[(uint64_t)rho * A.n_items + item];
                const uint32_t s0 = rho ? A.split_t[(uint64_t)(rho - 1) * A.n_items + item] : 0u;
                const uint64_t st = A.base_r[item] + s0;
                const uint32_t m = s1 - s0;
                a0 = st & ~7ull;
                const uint32_t head = (uint32_t)(st - a0);
                he = ((head + m) << 3) | head;
                nch = m ? (head + m + CW - 1) / CW : 0u;
            }
            const uint32_t incl = wave_incl_scan(nch);
            const uint32_t ex_l = incl - nch;
            const uint32_t tot = wave_readlane(incl, 63);
            s_a0[w][l] = a0;
            s_he[w][l] = he;
            s_ex[w][l] = ex_l;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            uint32_t sj = 0;
            for (uint32_t c0 = 0; c0 < tot; c0 += 64) {
                const uint32_t c = c0 + l;
                if (ex_l - c0 < 64u) atomicMax(&s_own[w][ex_l - c0], l + 1u);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
                const uint32_t mk = s_own[w][l];
                s_own[w][l] = 0u;
                const uint32_t pm = wave_incl_max(mk);
                const uint32_t j = pm ? max(sj, pm - 1u) : sj;
                sj = wave_readlane(j, 63);
                if (c < tot) {
                    const uint64_t ba = s_a0[w][j];
                    const uint32_t hv = s_he[w][j];
                    const uint32_t co = c - s_ex[w][j];
                    const uint4 *ptr = reinterpret_cast<const uint4 *>(A.words + ba) + 2 * co;
                    const uint4 v0 = ptr[0];
                    const uint4 v1 = ptr[co * CW + 4 < (hv >> 3) ? 1 : 0];
                    const uint32_t vv[CW] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
                    const int lo = (int)(hv & 7u) - (int)(co * CW);
                    const uint32_t span = (uint32_t)((int)(hv >> 3) - (int)(co * CW) - lo);
                    const uint32_t rank = ib + j - i0;  // local rank in the group
#pragma unroll
                    for (int k = 0; k < (int)CW; k++)
                        if ((uint32_t)(k - lo) < span) atomicMin(&s_tab[vv[k] & kmask], rank);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
        __syncthreads();
        // first covers -> their ranks' bits -> kept bytes
        for (uint32_t q = threadIdx.x; q < GM_TAB; q += THREADS) {
            const uint32_t r = s_tab[q];
            if (r != ~0u) atomicOr(&s_bits[r >> 5], 1u << (r & 31));
        }
        __syncthreads();
        for (uint32_t r = threadIdx.x; r < i1 - i0; r += THREADS)
            if ((s_bits[r >> 5] >> (r & 31)) & 1u) A.kept[i0 + r] = 1;
        __syncthreads();
    }
}
constexpr size_t GM_LDS = GM_TAB * 4 + NWAVE * 64 * (8 + 3 * 4) + GM_MAX_ITEMS / 8 + 16;

// dynamic LDS of pass1_keys_kernel past its 2^17-byte table
constexpr size_t KEYS_LDS_EXTRA =
    NWAVE * 64 * (8 + 4 * 4) + (MAX_R + 2) * 4 + MAX_NB * 4;

// Region loops: block b serves region b % NCTR (the grid is a multiple of
// NCTR), records [lo_k, min(ctr_k, cap_k)) of it.
#define SYZ_FOR_RECORDS(A, LO, i, r)                                                          \
    const uint32_t k_ = blockIdx.x % NCTR, sub_ = blockIdx.x / NCTR, nsub_ = gridDim.x / NCTR; \
    const uint64_t hi_ = std::min<uint64_t>((A).ctr[k_ * CTR_STRIDE], (A).cap_k);             \
    const unsigned long long *rk_ = (A).rec + k_ * (A).cap_k;                                 \
    for (uint64_t i = (LO) + (uint64_t)sub_ * blockDim.x + threadIdx.x; i < hi_;               \
         i += (uint64_t)nsub_ * blockDim.x)                                                   \
        if (const unsigned long long r = rk_[i]; true)

// Deferred first covers: first_w[pc] = min over the records
// appended since the last chunk, and covered |= them unless the caller
// rebuilds covered from first_w.  Pass 1 then never waits on an atomic: on
// gfx950 one counter (vmcnt) tracks loads, stores and atomics together, so an
// atomicMin in the streaming loop made the NEXT iteration's loads wait for it,
// and the early chunks' contended first-cover atomics (every item of the
// chunk holds the hot PCs) set their time (~100 us each at C2).
__global__ void min_records_kernel(Args A, int par, int or_cover) {
    const unsigned long long *done_in = A.done + (par ? 1 : 0) * NCTR * CTR_STRIDE;
    unsigned long long *done_out = A.done + (par ? 0 : 1) * NCTR * CTR_STRIDE;
    if (blockIdx.x < NCTR && threadIdx.x == 0)
        done_out[blockIdx.x * CTR_STRIDE] =
            std::min<uint64_t>(A.ctr[blockIdx.x * CTR_STRIDE], A.cap_k);
    SYZ_FOR_RECORDS(A, done_in[(blockIdx.x % NCTR) * CTR_STRIDE], i, r) {
        const uint32_t wo = (uint32_t)r;
        atomicMin(&A.first_w[wo], (int32_t)(r >> 32));
        if (or_cover) {
            const uint32_t mbit = 1u << (wo & 31);
            if (!(A.covered[wo >> 5] & mbit)) atomicOr((uint32_t *)&A.covered[wo >> 5], mbit);
        }
    }
}

// Bucketed first covers, the chunk's replacement for min_records_kernel +
// first_to_bits (key spaces <= 2^24): min_records' atomicMin per record on
// random first_w words ran at ~19 G/s (0.37 ms of C2's and of a C3/8 rank's
// Minimize), and the covered rebuild read all of first_w after every chunk.
// rec_scatter_kernel copies the chunk's new records into buckets of 2^BSH
// keys (pass 1 counted them per bucket: A.bh, this chunk's parity half);
// bmin_kernel then gives each bucket to one workgroup, which takes the
// minimum rank per key in LDS (ds_min, no global atomics), writes first_w of
// its keys once (min with what is there: a record that found its region full
// took its atomicMin directly) and rebuilds its covered words from first_w.
__device__ uint32_t bucket_scan(const uint32_t *bh, uint32_t nb, uint32_t b, uint32_t *s_tmp) {
    // exclusive prefix of bucket b (one workgroup, nb <= MAX_NB)
    uint32_t v = 0;
    for (uint32_t i = threadIdx.x; i < b; i += blockDim.x) v += bh[i];
    v = wave_sum(v);
    if (__lane_id() == 0) s_tmp[threadIdx.x >> 6] = v;
    __syncthreads();
    uint32_t tot = 0;
    for (uint32_t w = 0; w < blockDim.x / 64; w++) tot += s_tmp[w];
    __syncthreads();
    return tot;
}

constexpr int RS_TILE = 8;  // records per thread per round of rec_scatter_kernel
__global__ __launch_bounds__(256) void rec_scatter_kernel(Args A, int par) {
    __shared__ uint32_t s_pre[MAX_NB], s_cnt[MAX_NB], s_base[MAX_NB];
    const uint32_t *bh = A.bh + par * A.nb;
    uint32_t *cur = A.bcur + par * A.nb;
    // every bucket's exclusive prefix (the scan of the <= 1024 counts, once
    // per workgroup)
    {
        uint32_t run = 0;
        for (uint32_t i0 = 0; i0 < A.nb; i0 += 256) {
            const uint32_t i = i0 + threadIdx.x;
            const uint32_t v = i < A.nb ? bh[i] : 0u;
            __shared__ uint32_t tmp[256 / 64 + 1];
            uint32_t tot;
            const uint32_t ex = block_excl_scan<256>(v, tmp, &tot);
            if (i < A.nb) s_pre[i] = run + ex;
            run += tot;
        }
    }
    const unsigned long long *done_in = A.done + (par ? 1 : 0) * NCTR * CTR_STRIDE;
    unsigned long long *done_out = A.done + (par ? 0 : 1) * NCTR * CTR_STRIDE;
    if (blockIdx.x < NCTR && threadIdx.x == 0)  // (as min_records_kernel)
        done_out[blockIdx.x * CTR_STRIDE] =
            std::min<uint64_t>(A.ctr[blockIdx.x * CTR_STRIDE], A.cap_k);
    const uint32_t k_ = blockIdx.x % NCTR, sub_ = blockIdx.x / NCTR, nsub_ = gridDim.x / NCTR;
    const uint64_t lo = done_in[k_ * CTR_STRIDE];
    const uint64_t hi = std::min<uint64_t>(A.ctr[k_ * CTR_STRIDE], A.cap_k);
    const unsigned long long *rk = A.rec + k_ * A.cap_k;
    const uint64_t per = (uint64_t)256 * RS_TILE;
    for (uint64_t t0 = lo + (uint64_t)sub_ * per; t0 < hi; t0 += (uint64_t)nsub_ * per) {
        for (uint32_t i = threadIdx.x; i < A.nb; i += 256) s_cnt[i] = 0u;
        __syncthreads();
        unsigned long long r[RS_TILE];
        uint32_t slot[RS_TILE];
#pragma unroll
        for (int j = 0; j < RS_TILE; j++) {
            const uint64_t i = t0 + (uint64_t)j * 256 + threadIdx.x;
            r[j] = i < hi ? rk[i] : ~0ull;
            slot[j] = r[j] != ~0ull ? atomicAdd(&s_cnt[(uint32_t)r[j] >> BSH], 1u) : 0u;
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < A.nb; i += 256)
            s_base[i] = s_cnt[i] ? s_pre[i] + atomicAdd(&cur[i], s_cnt[i]) : 0u;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < RS_TILE; j++)
            if (r[j] != ~0ull) A.rsort[s_base[(uint32_t)r[j] >> BSH] + slot[j]] = r[j];
        __syncthreads();
    }
}

__global__ __launch_bounds__(1024) void bmin_kernel(Args A, int par, uint64_t span) {
    __shared__ int32_t s_min[1u << BSH];
    __shared__ uint32_t s_tmp[16];
    const uint32_t b = blockIdx.x;
    const uint32_t *bh = A.bh + par * A.nb;
    const uint32_t r0 = bucket_scan(bh, A.nb, b, s_tmp), n = bh[b];
    const uint64_t k0 = (uint64_t)b << BSH;
    const uint32_t nk = (uint32_t)std::min<uint64_t>(1u << BSH, span - k0);
    if (n) {
        for (uint32_t i = threadIdx.x; i < (1u << BSH); i += 1024) s_min[i] = INT32_MAX;
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < n; i += 1024) {
            const unsigned long long r = A.rsort[r0 + i];
            atomicMin(&s_min[(uint32_t)r & ((1u << BSH) - 1u)], (int32_t)(r >> 32));
        }
        __syncthreads();
    }
    // first_w of the bucket's keys, then its covered words (32 keys each,
    // one ballot half per word): covered = {key : first_w[key] != INT32_MAX}
    for (uint32_t i = threadIdx.x; i < ((nk + 63) & ~63u); i += 1024) {
        int32_t f = INT32_MAX;
        if (i < nk) {
            f = A.first_w[k0 + i];
            if (n && s_min[i] < f) {
                f = s_min[i];
                A.first_w[k0 + i] = f;
            }
        }
        const uint64_t m = __ballot(f != INT32_MAX);
        if ((__lane_id() & 31) == 0 && i < nk)
            const_cast<uint32_t *>(A.covered)[(k0 + i) >> 5] = (uint32_t)(m >> (__lane_id() & 32));
    }
    // the other parity's counts and cursors start the next chunk at zero
    if (threadIdx.x == 0) {
        A.bh[(par ^ 1) * A.nb + b] = 0u;
        A.bcur[(par ^ 1) * A.nb + b] = 0u;
    }
}

// *rec_cnt = total records, or more than rec_cap if any region overflowed
// (the overflow fallbacks key on that).
__global__ void total_kernel(Args A) {
    const uint32_t k = threadIdx.x;
    unsigned long long c = k < NCTR ? A.ctr[k * CTR_STRIDE] : 0ull;
    int ovf = k < NCTR && c > A.cap_k;
    for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
    ovf = __any(ovf);
    if (k == 0) *A.rec_cnt = ovf ? std::max<unsigned long long>(c, A.rec_cap + 1) : c;
}

// The first-cover rank of window offset wo: first_w[wo] on one GPU; across
// shards the MIN-merged dense table first_d[id(wo)] (tab: dictionary of the
// merged union, syzcov_dev_dict_build_bits layout).
__device__ __forceinline__ int32_t first_of(const int32_t *first_w, const uint64_t *tab,
                                            const int32_t *first_d, uint32_t wo) {
    if (!tab) return first_w[wo];
    const uint64_t e = tab[wo >> 5];
    const uint32_t bits = (uint32_t)(e >> 32), b = wo & 31;
    if (!((bits >> b) & 1u)) return INT32_MAX;
    return first_d[(uint32_t)e + __popc(bits & ((1u << b) - 1u))];
}

// Pass 2 over the records: kept[rank] = 1 iff first(pc) == rank.
__global__ void pass2_kernel(Args A, const uint64_t *tab, const int32_t *first_d, uint8_t *kept) {
    SYZ_FOR_RECORDS(A, 0, i, r) {
        const int32_t rank = (int32_t)(r >> 32);
        if (first_of(A.first_w, tab, first_d, (uint32_t)r) == rank)
            kept[(uint32_t)rank] = 1;
    }
}

// first_w back to INT32_MAX at every recorded offset (after pass 2).
__global__ void reset_kernel(Args A) {
    SYZ_FOR_RECORDS(A, 0, i, r) A.first_w[(uint32_t)r] = INT32_MAX;
}

// ---- overflow fallbacks (early exit unless *cnt > cap)
__global__ void ovf_pass2_kernel(Args A, uint32_t n_items, const int32_t *first_w,
                                 const uint64_t *tab, const int32_t *first_d, uint8_t *kept) {
    if (*A.rec_cnt <= A.rec_cap) return;
    for (uint32_t j = blockIdx.x; j < n_items; j += gridDim.x) {
        if (!A.cand[j]) continue;
        const int32_t rank = A.ranks ? A.ranks[j] : (int32_t)j;
        const uint64_t o = A.base_r[j];
        bool hit = false;
        uint32_t s0 = 0;
        for (uint32_t rho = 0; rho < A.nrange; rho++) {  // the item's sub-runs
            const uint32_t s1 = A.split_t[(uint64_t)rho * A.n_items + j];
            const uint64_t a = o + aligned_sub(s0, rho, A.ak);
            for (uint32_t q = threadIdx.x; q < s1 - s0; q += blockDim.x)
                hit |= first_of(first_w, tab, first_d, (A.pcs[a + q] & A.keymask) - A.pc_lo) == rank;
            s0 = s1;
        }
        if (__syncthreads_or(hit) && threadIdx.x == 0) kept[rank] = 1;
    }
}

__global__ void ovf_union_kernel(const unsigned long long *cnt, uint64_t cap, const int32_t *first_w,
                                 uint64_t span, uint32_t *covered) {
    if (*cnt <= cap) return;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < span;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const bool set = first_w[i] != INT32_MAX;
        const uint64_t m = __ballot(set);
        if ((threadIdx.x & 31) == 0) {
            const uint32_t word = (uint32_t)(m >> (threadIdx.x & 32));
            if (word) atomicOr(&covered[i >> 5], word);
        }
    }
}

__global__ void ovf_reset_kernel(const unsigned long long *cnt, uint64_t cap, int32_t *first_w,
                                 uint64_t span) {
    if (*cnt <= cap) return;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < span;
         i += (uint64_t)gridDim.x * blockDim.x)
        first_w[i] = INT32_MAX;
}

// window-indexed first_w <-> dense table over a dictionary (shard exchange)
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

}  // namespace mr
}  // namespace syz

using namespace syz;

/* ws: region counters ctr | done marks x 2 (NCTR * 256 B each) | base_r [n_items] u64 |
 *     split_t [nrange][n_items] u32 */
// region counters | done marks x 2 | per-chunk piece counters (dynamic pieces)
static constexpr int MR_MAX_CHUNKS = 64;
static constexpr size_t MR_BKT = 4 * mr::MAX_NB * sizeof(uint32_t);  // bh[2][nb], bcur[2][nb]
static constexpr size_t MR_HDR = 3 * mr::NCTR * mr::CTR_STRIDE * sizeof(uint64_t) +
                                 MR_MAX_CHUNKS * 256 + MR_BKT;
static uint64_t mr_nrange(uint64_t span, uint32_t rshift) {
    return (span + (1ull << rshift) - 1) >> rshift;
}

extern "C" size_t syzcov_dev_minimize_range_ws_size(size_t n_items, uint64_t pc_span,
                                                    uint32_t range_shift) {
    if (range_shift > 20) range_shift = 20;
    return MR_HDR + align_up(n_items * 8, 256) +
           align_up(mr_nrange(pc_span, range_shift) * n_items * 4, 256);
}

static int dev_cus() {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        n = 256;
    return n > 0 ? n : 256;
}

static int mr_args(mr::Args &A, const uint64_t *off, const uint32_t *len, const uint32_t *pcs,
                   const uint32_t *split, const int32_t *order, const int32_t *ranks,
                   size_t n_items, uint32_t pc_lo, uint64_t pc_span, uint32_t range_shift,
                   const uint64_t *range_tot, uint32_t *covered, int32_t *first_w, uint64_t *rec,
                   uint64_t rec_cap, uint64_t *rec_cnt, uint8_t *cand, void *ws) {
    if (!off || !pcs || !order || !range_tot || !covered || !first_w || !rec || !rec_cnt || !cand ||
        !ws || n_items > 0x7FFFFFFF)
        return SYZCOV_EINVAL;
    if (range_shift < 10 || range_shift > 20 || pc_span == 0 || pc_span > (1ull << 32))
        return SYZCOV_EINVAL;
    const uint64_t nrange = mr_nrange(pc_span, range_shift);
    if (nrange > (uint64_t)mr::MAX_R) return SYZCOV_ERANGE;
    if (!split && nrange != 1) return SYZCOV_EINVAL;
    if (!split && !len) return SYZCOV_EINVAL;
    A.off = off;
    A.len = len;
    A.pcs = pcs;
    A.split = split;
    A.order = order;
    A.ranks = ranks;
    A.pc_lo = pc_lo;
    A.rshift = range_shift;
    A.nrange = (uint32_t)nrange;
    A.range_tot = (const unsigned long long *)range_tot;
    A.covered = covered;
    A.first_w = first_w;
    A.rec = (unsigned long long *)rec;
    A.rec_cap = rec_cap;
    A.rec_cnt = (unsigned long long *)rec_cnt;
    A.cand = cand;
    A.n_items = (uint32_t)n_items;
    A.ctr = (unsigned long long *)ws;
    A.done = A.ctr + mr::NCTR * mr::CTR_STRIDE;
    A.cap_k = rec_cap / mr::NCTR;
    A.base_r = (uint64_t *)((uint8_t *)ws + MR_HDR);
    A.split_t = (uint32_t *)((uint8_t *)A.base_r + align_up(n_items * 8, 256));
    A.pctr = nullptr;
    A.npieces = 0;
    A.keymask = 0xFFFFFFFFu;
    A.low_of_key = nullptr;
    A.err = nullptr;
    A.ak = 0;
    A.bh = A.bcur = nullptr;
    A.rsort = nullptr;
    A.nb = 0;
    return 0;
}

// pass 2 + resets (first_w back to INT32_MAX)
// first_w back to INT32_MAX by a fill below this many PCs/keys
static constexpr uint64_t kFillSpan = 1ull << 24;

static int mr_pass2(const mr::Args &A, uint64_t pc_span, const uint64_t *tab,
                    const int32_t *first_d, uint8_t *kept, hipStream_t s) {
    const unsigned long long *cnt = A.rec_cnt;
    hipLaunchKernelGGL(mr::pass2_kernel, dim3(1024), dim3(256), 0, s, A, tab, first_d, kept);
    hipLaunchKernelGGL(mr::ovf_pass2_kernel, dim3(1024), dim3(256), 0, s, A, A.n_items,
                       (const int32_t *)A.first_w, tab, first_d, kept);
    if (pc_span <= kFillSpan) {
        // a small key space: one coalesced fill (16 MB at 2^22 keys, ~5 us)
        // instead of a scattered reset per record (~40 us at C2) + the
        // overflow reset
        SYZ_HIP(hipMemsetD32Async((hipDeviceptr_t)A.first_w, INT32_MAX, pc_span, s));
    } else {
        hipLaunchKernelGGL(mr::reset_kernel, dim3(1024), dim3(256), 0, s, A);
        hipLaunchKernelGGL(mr::ovf_reset_kernel, dim3(2048), dim3(256), 0, s, cnt, A.rec_cap,
                           A.first_w, pc_span);
    }
    SYZ_LAUNCH_CHECK();
    return 0;
}

static int minimize_range_impl(
    const uint64_t *off, const uint32_t *len, const uint32_t *pcs, const uint32_t *split,
    const int32_t *order, const int32_t *ranks, size_t n_items, uint32_t pc_lo, uint64_t pc_span,
    uint32_t range_shift, const uint64_t *range_tot, uint32_t *covered, int32_t *first_w,
    uint64_t *rec, uint64_t rec_cap, uint64_t *rec_cnt, uint8_t *cand, uint8_t *kept, int do_pass2,
    size_t first_chunk, uint32_t growth, uint64_t pcs_per_wg_hint, const uint8_t *low_of_key,
    uint32_t *err_flag, void *ws, void *stream, const uint64_t *grp_off = nullptr,
    uint32_t ngroups = 0, int aligned = 0, bool n4 = false, uint64_t *rsort = nullptr) {
    hipStream_t s = (hipStream_t)stream;
    if (n_items == 0) {
        if (rec_cnt) SYZ_HIP(hipMemsetAsync(rec_cnt, 0, sizeof(uint64_t), s));
        return 0;
    }
    if (do_pass2 && !kept) return SYZCOV_EINVAL;
    mr::Args A;
    int rc = mr_args(A, off, len, pcs, split, order, ranks, n_items, pc_lo, pc_span, range_shift,
                     range_tot, covered, first_w, rec, rec_cap, rec_cnt, cand, ws);
    if (rc) return rc;
    if (aligned) {  // line-aligned sub-runs (common.h) need the split points
        if (!split) return SYZCOV_EINVAL;
        A.ak = SYZ_ALIGN_K(A.nrange);
    }
    const bool keym = low_of_key != nullptr;
    if (keym) {  // key words over <= 2^25 keys, 2^rshift table bytes (N4: nibbles) in LDS
        if (!err_flag || pc_lo != 0 || range_shift > (n4 ? 18u : 17u) || pc_span > (1ull << 25))
            return SYZCOV_EINVAL;
        A.keymask = SYZ_KEY_MASK;
        A.low_of_key = low_of_key;
        A.err = err_flag;
    }
    const uint64_t nrange = A.nrange;
    SYZ_HIP(hipMemsetAsync(ws, 0, MR_HDR, s));  // region counters and done marks
    static std::atomic<uint32_t> prep_attr{0};  // nrange = 256 needs 65.8 KB of dynamic LDS
    if ((rc = set_dyn_lds_once((const void *)mr::prep_kernel, 80 * 1024, prep_attr))) return rc;
    hipLaunchKernelGGL(mr::prep_kernel, dim3(grid_for(n_items, 64, 8192)), dim3(256),
                       split ? 64 * (nrange + 1) * sizeof(uint32_t) : 0, s, A,
                       (uint64_t *)A.base_r, (uint32_t *)A.split_t);
    const size_t lds = ((size_t)1 << range_shift) / (keym ? 1 : 8);
    using K = void (*)(mr::Args, uint32_t, uint32_t, uint32_t, int);
#ifndef SYZ_MR_KEYS_UG
#define SYZ_MR_KEYS_UG 2
#endif
#ifndef SYZ_MR_OLD_KEYS
    const K k1 = keym && n4 ? mr::pass1_keys_kernel<SYZ_MR_KEYS_UG, true>
                 : keym     ? mr::pass1_keys_kernel<SYZ_MR_KEYS_UG>
                            : mr::pass1_stream_kernel<2, false>;
#else
    const K k1 = keym ? mr::pass1_stream_kernel<2, true> : mr::pass1_stream_kernel<2, false>;
#endif
    static std::atomic<uint32_t> attr_set[3];
#ifndef SYZ_MR_OLD_KEYS
    // (the table at LDS 0 holds 2^range_shift <= 2^17 bytes, the rest past 2^17)
    const size_t lds1 = keym ? ((size_t)1 << 17) + mr::KEYS_LDS_EXTRA : lds;
#else
    const size_t lds1 = lds;
#endif
    if ((rc = set_dyn_lds_once((const void *)k1, (uint32_t)std::max<size_t>(lds1, 128 * 1024),
                               attr_set[keym && n4 ? 2 : keym ? 1 : 0])))
        return rc;
#ifndef SYZ_MR_FIRST
#define SYZ_MR_FIRST 64
#endif
#ifndef SYZ_MR_GROWTH
#define SYZ_MR_GROWTH 4
#endif
    if (first_chunk == 0) first_chunk = SYZ_MR_FIRST;
    if (growth < 2) growth = grp_off ? 8 : SYZ_MR_GROWTH;
    // sweep at C2: 2^17 PCs per workgroup 4.03, 2^19 4.00, 2^20 4.40 ms
#ifndef SYZ_MR_HINT_LOG
#define SYZ_MR_HINT_LOG 19
#endif
#ifndef SYZ_MR_PPS
#define SYZ_MR_PPS 16
#endif
#ifndef SYZ_MR_KEYS_PPS  // key mode, XCD-local slices (draw_piece): 1/2/4/8 -> C3
#define SYZ_MR_KEYS_PPS 2  // Minimize 19.3/17.3/18.3/19.3 ms, C3/8 rank 3.81/2.80/2.83/3.05
#endif
    if (pcs_per_wg_hint == 0) pcs_per_wg_hint = 1 << SYZ_MR_HINT_LOG;
    // pieces per chunk at least: 1 per CU, 4 in key mode, where the slices
    // are XCD-local and a piece's table restage is cheap: the small chunks'
    // few large pieces left a tail (g_min 256 / 512 / 768 / 1024 / 2048:
    // C3/8 rank Minimize 2.63 / 2.60 / 2.60 / 2.59 / 2.71 ms, C2 2.34 / 2.27 /
    // 2.28 / 2.24 / 2.26, pass 2 too: 0.11 -> 0.09)
#ifndef SYZ_MR_GMIN_KEYS
#define SYZ_MR_GMIN_KEYS 1024
#endif
    const uint64_t g_min = keym && !grp_off ? SYZ_MR_GMIN_KEYS : 256;
    const uint64_t avg_len = 2048;  // only sizes the grid; any value is exact
    // below 2^24 keys (64 MB of first_w) the covered set is rebuilt from first_w
    const bool cover_from_first = pc_span <= (1ull << 24);
    // key mode with room for a sorted copy of the records (the corpus engine):
    // first covers by bucket in LDS (bmin_kernel) instead of global atomics
    const bool bucketed = rsort && keym && cover_from_first && !grp_off &&
                          !(force_flags() & FORCE_MIN_ATOMICS);
    if (bucketed) {
        A.nb = (uint32_t)((pc_span + (1ull << mr::BSH) - 1) >> mr::BSH);
        A.bh = (uint32_t *)((uint8_t *)ws + MR_HDR - MR_BKT);
        A.bcur = A.bh + 2 * mr::MAX_NB;
        A.rsort = (unsigned long long *)rsort;
    }
    // pass 1 over the items [a0, a1) in geometric chunks (covered empty at a0)
    auto run_span = [&](uint64_t a0, uint64_t a1, uint64_t step0, bool cov0) -> int {
        uint64_t a = a0, step = step0;
        int par = 0;  // done-mark set of this chunk
        uint32_t nchunk = 0;
        while (a < a1) {
            const uint64_t b = std::min<uint64_t>(a1, a + step);
            // about pcs_per_wg_hint PCs per workgroup, at least one CU's worth;
            // P = 16R pieces per slice (fewer, larger pieces in the small chunks,
            // >= 256 KB of PCs each: 3.52 against 2.87 ms at C2); key mode 2R
            uint64_t G = ((b - a) * avg_len + pcs_per_wg_hint - 1) / pcs_per_wg_hint;
#ifndef SYZ_MR_GMAX
#define SYZ_MR_GMAX 8192
#endif
            G = std::min<uint64_t>(std::max<uint64_t>(G, g_min), SYZ_MR_GMAX);
            const uint64_t P = (keym ? SYZ_MR_KEYS_PPS : SYZ_MR_PPS) * (uint64_t)nrange;
            G = std::max<uint64_t>(G / P, 1) * P;  // whole slices
            // dynamic pieces: one workgroup per CU draws them
            if (nchunk >= MR_MAX_CHUNKS) return SYZCOV_EINVAL;
            A.pctr = (uint32_t *)((uint8_t *)ws + 3 * mr::NCTR * mr::CTR_STRIDE * sizeof(uint64_t) +
                                  (size_t)nchunk * 256);
            A.npieces = (uint32_t)G;
            const unsigned grid = (unsigned)std::min<uint64_t>(G, (uint64_t)dev_cus());
            nchunk++;
            mr::Args A1 = A;  // pass 1 counts this chunk's records per bucket
            if (bucketed) A1.bh = A.bh + par * A.nb;
            hipLaunchKernelGGL(k1, dim3(grid), dim3(mr::THREADS), lds1, s, A1, (uint32_t)a,
                               (uint32_t)b, (uint32_t)P, (int)(a != a0 || cov0));
            if (bucketed) {
                // the chunk's first covers and covered words, bucket by bucket
                hipLaunchKernelGGL(mr::rec_scatter_kernel, dim3(1024), dim3(256), 0, s, A, par);
                hipLaunchKernelGGL(mr::bmin_kernel, dim3(A.nb), dim3(1024), 0, s, A, par,
                                   pc_span);
            } else {
                // the chunk's first covers (+ covered, unless rebuilt below)
                hipLaunchKernelGGL(mr::min_records_kernel, dim3(1024), dim3(256), 0, s, A, par,
                                   (int)!cover_from_first);
                // covered = {pc : first_w[pc] != INT32_MAX}: one coalesced pass over
                // first_w (16 MB at 2^22 keys) instead of an atomicOr per record (C2
                // key mode: 5 vs 74-274 us per early chunk)
                if (cover_from_first && b < a1)
                    RC_(syzcov_dev_first_to_bits(first_w, pc_span, covered, s));
            }
            par ^= 1;
            a = b;
            step *= growth;
        }
        hipLaunchKernelGGL(mr::total_kernel, dim3(1), dim3(64), 0, s, A);
        return 0;
    };
    if (grp_off) {
        // Manager.minimizeCorpus (manager.go:504-524): one cover.Minimize per
        // call group, the groups' processing orders concatenated into one rank
        // space ([grp_off[g], grp_off[g+1]) is group g).  Each group runs pass 1
        // from an empty covered set, its own pass 2, and returns first_w to
        // INT32_MAX at its records, so the next group starts clean.  (Groups
        // are far shorter than a corpus: first chunk 256, growth 8.)
        if (!do_pass2 || ngroups == 0 || grp_off[ngroups] != n_items) return SYZCOV_EINVAL;
        for (uint32_t g = 0; g < ngroups; g++) {
            const uint64_t a0 = grp_off[g], a1 = grp_off[g + 1];
            if (a1 < a0 || a1 > n_items) return SYZCOV_EINVAL;
            if (a1 == a0) continue;
            if (g) SYZ_HIP(hipMemsetAsync(ws, 0, MR_HDR, s));  // region counters, done marks
            if (!cover_from_first)
                SYZ_HIP(hipMemsetAsync(covered, 0, (((uint64_t)nrange << range_shift) + 7) / 8, s));
            RC_(run_span(a0, a1, 256, false));
            hipLaunchKernelGGL(mr::pass2_kernel, dim3(1024), dim3(256), 0, s, A,
                               (const uint64_t *)nullptr, (const int32_t *)nullptr, kept);
            hipLaunchKernelGGL(mr::ovf_pass2_kernel, dim3(1024), dim3(256), 0, s, A, A.n_items,
                               (const int32_t *)A.first_w, (const uint64_t *)nullptr,
                               (const int32_t *)nullptr, kept);
            hipLaunchKernelGGL(mr::reset_kernel, dim3(1024), dim3(256), 0, s, A);
            hipLaunchKernelGGL(mr::ovf_reset_kernel, dim3(2048), dim3(256), 0, s,
                               (const unsigned long long *)rec_cnt, rec_cap, first_w, pc_span);
            SYZ_LAUNCH_CHECK();
        }
        // covered: no union is asked of a grouped step (left empty)
        SYZ_HIP(hipMemsetAsync(covered, 0, (((uint64_t)nrange << range_shift) + 7) / 8, s));
        return 0;
    }
    // the initial block (init_min_kernel): the first SYZ_MR_INIT_CHUNKS chunks'
    // items, exact first covers in LDS; the chunks go on from there
#ifndef SYZ_MR_INIT_CHUNKS
#define SYZ_MR_INIT_CHUNKS 4
#endif
    uint64_t k_init = 0, step0 = first_chunk;
    const int init_chunks = force_flags() & FORCE_SMALL_INIT ? 1 : SYZ_MR_INIT_CHUNKS;
    for (int c = 0; c < init_chunks; c++) {
        k_init += step0;
        step0 *= growth;
    }
    const uint64_t T = nrange << range_shift;  // keys of the tables (covered bits)
    const uint64_t nq = range_shift >= mr::IQ_SH ? 1ull << (range_shift - mr::IQ_SH) : 0;
    const bool init = bucketed && nq && k_init > 0 && T * 4 <= rec_cap * 8 &&
                      nrange <= mr::MAX_R && !(force_flags() & FORCE_NO_INIT_BLOCK);
    if (init) {
        k_init = std::min<uint64_t>(k_init, n_items);
        static std::atomic<uint32_t> init_attr{0};
        const size_t lds_i = ((size_t)4 << mr::IQ_SH) + mr::INIT_LDS_EXTRA;
#ifndef SYZ_MR_INIT_UG  // windows in flight: 1 / 2 / 3 / 4 -> C3/8 rank Minimize
#define SYZ_MR_INIT_UG 2  // 2.61-2.67 / 2.59-2.68 / 2.78 / 2.98 ms (4: 316 B of spills)
#endif
        if ((rc = set_dyn_lds_once((const void *)mr::init_min_kernel<SYZ_MR_INIT_UG>, (uint32_t)lds_i,
                                   init_attr)))
            return rc;
        // pieces: every workgroup slot of the GPU, at least one per range
#ifndef SYZ_MR_INIT_WG
#define SYZ_MR_INIT_WG 1  // workgroups per CU
#endif
        // pieces: every workgroup slot of the GPU, at least two per range (at
        // one per range the hot ranges are not split: C2X, 8 key parts per
        // range, P = R: Minimize 3.40 ms; P = 2R 2.73; no block 2.89)
        const uint64_t P =
            std::max<uint64_t>(2 * nrange, (SYZ_MR_INIT_WG * dev_cus() + nq - 1) / nq);
        uint32_t *tab = (uint32_t *)rsort;  // free until the first chunk's rec_scatter
        SYZ_HIP(hipMemsetAsync(tab, 0xFF, T * 4, s));
        hipLaunchKernelGGL(mr::init_min_kernel<SYZ_MR_INIT_UG>, dim3((unsigned)(nq * P)), dim3(mr::THREADS),
                           lds_i, s, A, 0u, (uint32_t)k_init, (uint32_t)P, tab);
        hipLaunchKernelGGL(mr::init_flush_kernel, dim3((unsigned)std::min<uint64_t>(
                               std::max<uint64_t>(T / 256, mr::NCTR), 4096)),
                           dim3(256), 0, s, A, 0u, (const uint32_t *)tab, T, pc_span);
        hipLaunchKernelGGL(mr::init_done_kernel, dim3(1), dim3(64), 0, s, A);
#ifndef SYZ_MR_POST_INIT_MUL
#define SYZ_MR_POST_INIT_MUL 1
#endif
        RC_(run_span(k_init, n_items, step0 * SYZ_MR_POST_INIT_MUL, true));
    } else {
        RC_(run_span(0, n_items, first_chunk, false));
    }
    if (cover_from_first && !bucketed) RC_(syzcov_dev_first_to_bits(first_w, pc_span, covered, s));
    // record overflow: the union comes from first_w instead (cover_from_first
    // already rebuilt covered from first_w)
    if (!cover_from_first)
        hipLaunchKernelGGL(mr::ovf_union_kernel, dim3(2048), dim3(256), 0, s,
                           (const unsigned long long *)rec_cnt, rec_cap, (const int32_t *)first_w,
                           pc_span, covered);
    SYZ_LAUNCH_CHECK();
    if (!do_pass2) return 0;
    rc = mr_pass2(A, pc_span, nullptr, nullptr, kept, s);
    return rc;
}

// Minimize per call group over one rank space (corpus.hip: the grouped
// drop-in for Manager.minimizeCorpus); key mode when low_of_key is given.
namespace syz {
// Key mode over NIBBLE tables (kshift <= 2: every low value < 4), ranges of
// 2^18 keys (corpus.hip picks it; the public entry keeps byte tables)
int minimize_range_keys_n4(const uint64_t *off, const uint32_t *len, const uint32_t *words,
                           const uint32_t *split, const int32_t *order, const int32_t *ranks,
                           size_t n_items, uint64_t nkeys, uint32_t range_shift,
                           const uint64_t *range_tot, const uint8_t *low_of_key,
                           uint32_t *covered, int32_t *first_w, uint64_t *rec, uint64_t rec_cap,
                           uint64_t *rec_cnt, uint8_t *cand, uint8_t *kept, int do_pass2,
                           uint32_t *err_flag, void *ws, hipStream_t s, uint64_t *rsort) {
    if (!low_of_key) return SYZCOV_EINVAL;
    return minimize_range_impl(off, len, words, split, order, ranks, n_items, 0, nkeys,
                               range_shift, range_tot, covered, first_w, rec, rec_cap, rec_cnt,
                               cand, kept, do_pass2, 0, 0, 0, low_of_key, err_flag, ws, s, nullptr,
                               0, 0, true, rsort);
}
// the corpus engine's key mode with byte tables: rsort (rec_cap records) for
// the bucketed first covers
int minimize_range_keys_sorted(const uint64_t *off, const uint32_t *len, const uint32_t *words,
                               const uint32_t *split, const int32_t *order, const int32_t *ranks,
                               size_t n_items, uint64_t nkeys, uint32_t range_shift,
                               const uint64_t *range_tot, const uint8_t *low_of_key,
                               uint32_t *covered, int32_t *first_w, uint64_t *rec,
                               uint64_t rec_cap, uint64_t *rec_cnt, uint8_t *cand, uint8_t *kept,
                               int do_pass2, uint32_t *err_flag, void *ws, hipStream_t s,
                               uint64_t *rsort) {
    if (!low_of_key) return SYZCOV_EINVAL;
    return minimize_range_impl(off, len, words, split, order, ranks, n_items, 0, nkeys,
                               range_shift, range_tot, covered, first_w, rec, rec_cap, rec_cnt,
                               cand, kept, do_pass2, 0, 0, 0, low_of_key, err_flag, ws, s, nullptr,
                               0, 0, false, rsort);
}

int minimize_range_groups(const uint64_t *off, const uint32_t *len, const uint32_t *pcs,
                          const uint32_t *split, const int32_t *order, size_t n_items,
                          uint32_t pc_lo, uint64_t pc_span, uint32_t range_shift,
                          const uint64_t *range_tot, const uint8_t *low_of_key, uint32_t *covered,
                          int32_t *first_w, uint64_t *rec, uint64_t rec_cap, uint64_t *rec_cnt,
                          uint8_t *cand, uint8_t *kept, uint32_t *err_flag,
                          const uint64_t *grp_off, uint32_t ngroups, void *ws, hipStream_t s,
                          int aligned) {
    return minimize_range_impl(off, len, pcs, split, order, nullptr, n_items, pc_lo, pc_span,
                               range_shift, range_tot, covered, first_w, rec, rec_cap, rec_cnt, cand,
                               kept, 1, 0, 0, 0, low_of_key, err_flag, ws, s, grp_off, ngroups,
                               aligned);
}
}  // namespace syz

// Manager.minimizeCorpus over small groups (group_min_kernel): key words of
// ranges of 2^range_shift <= 2^15 keys (split [n][nrange]), the grouped order
// (rank -> input), the groups' rank intervals on the device.  kept by rank.
namespace syz {
size_t minimize_groups_lds_ws_size(size_t n_items, uint64_t nkeys, uint32_t range_shift) {
    return 256 + align_up(n_items * 8, 256) + align_up(mr_nrange(nkeys, range_shift) * n_items * 4, 256);
}

int minimize_groups_lds(const uint64_t *off, const uint32_t *words, const uint32_t *split,
                        const int32_t *order, size_t n_items, uint64_t nkeys, uint32_t range_shift,
                        const uint64_t *goff_dev, uint32_t ngroups, uint8_t *kept, void *ws,
                        hipStream_t s) {
    if (n_items == 0 || ngroups == 0) return 0;
    if (!off || !words || !split || !order || !goff_dev || !kept || !ws || range_shift > 15 ||
        n_items > 0x7FFFFFFF)
        return SYZCOV_EINVAL;
    const uint64_t nrange = mr_nrange(nkeys, range_shift);
    if (nrange > (uint64_t)mr::MAX_R || nrange * ngroups > 0xFFFFFFFFull) return SYZCOV_ERANGE;
    mr::Args A{};
    A.off = off;
    A.split = split;
    A.order = order;
    A.n_items = (uint32_t)n_items;
    A.nrange = (uint32_t)nrange;
    uint32_t *pctr = (uint32_t *)ws;
    uint64_t *base_r = (uint64_t *)((uint8_t *)ws + 256);
    uint32_t *split_t = (uint32_t *)((uint8_t *)base_r + align_up(n_items * 8, 256));
    SYZ_HIP(hipMemsetAsync(pctr, 0, 4, s));
    SYZ_HIP(hipMemsetAsync(kept, 0, n_items, s));
    static std::atomic<uint32_t> prep_attr{0}, gm_attr{0};
    int rc = set_dyn_lds_once((const void *)mr::prep_kernel, 80 * 1024, prep_attr);
    if (!rc) rc = set_dyn_lds_once((const void *)mr::group_min_kernel, (int)mr::GM_LDS, gm_attr);
    if (rc) return rc;
    hipLaunchKernelGGL(mr::prep_kernel, dim3(grid_for(n_items, 64, 8192)), dim3(256),
                       64 * (nrange + 1) * sizeof(uint32_t), s, A, base_r, split_t);
    mr::GmArgs G{words, base_r, split_t, goff_dev, (uint32_t)n_items, ngroups, (uint32_t)nrange,
                 range_shift, pctr, kept};
    hipLaunchKernelGGL(mr::group_min_kernel, dim3((unsigned)std::min<uint64_t>(nrange * ngroups,
                                                                              (uint64_t)dev_cus())),
                       dim3(mr::THREADS), mr::GM_LDS, s, G);
    SYZ_LAUNCH_CHECK();
    return 0;
}
}  // namespace syz

// The line-aligned layout of syzcov_dev_canon_split_aligned (common.h): key
// mode iff low_of_key (then pc_lo = 0, pc_span = the key count, err_flag).
extern "C" int syzcov_dev_minimize_range_aligned(
    const uint64_t *off, const uint32_t *pcs, const uint32_t *split, const int32_t *order,
    const int32_t *ranks, size_t n_items, uint32_t pc_lo, uint64_t pc_span, uint32_t range_shift,
    const uint64_t *range_tot, const uint8_t *low_of_key, uint32_t *covered, int32_t *first_w,
    uint64_t *rec, uint64_t rec_cap, uint64_t *rec_cnt, uint8_t *cand, uint8_t *kept,
    int do_pass2, uint32_t *err_flag, void *ws, void *stream) {
    return minimize_range_impl(off, nullptr, pcs, split, order, ranks, n_items, pc_lo, pc_span,
                               range_shift, range_tot, covered, first_w, rec, rec_cap, rec_cnt,
                               cand, kept, do_pass2, 0, 0, 0, low_of_key, err_flag, ws, stream,
                               nullptr, 0, 1);
}

extern "C" int syzcov_dev_minimize_range_aligned_pass2(
    const uint64_t *off, const uint32_t *pcs, const uint32_t *split, const int32_t *order,
    const int32_t *ranks, size_t n_items, uint32_t pc_lo, uint64_t pc_span, uint32_t range_shift,
    const uint64_t *range_tot, int key_mode, uint32_t *covered, int32_t *first_w, uint64_t *rec,
    uint64_t rec_cap, uint64_t *rec_cnt, uint8_t *cand, const uint64_t *tab,
    const int32_t *first_dense, uint8_t *kept, void *ws, void *stream) {
    if (n_items == 0) return 0;
    if (!kept || !split || (tab && !first_dense)) return SYZCOV_EINVAL;
    mr::Args A;
    int rc = mr_args(A, off, nullptr, pcs, split, order, ranks, n_items, pc_lo, pc_span,
                     range_shift, range_tot, covered, first_w, rec, rec_cap, rec_cnt, cand, ws);
    if (rc) return rc;
    A.ak = SYZ_ALIGN_K(A.nrange);
    if (key_mode) A.keymask = SYZ_KEY_MASK;  // the overflow fallback reads the words
    return mr_pass2(A, pc_span, tab, first_dense, kept, (hipStream_t)stream);
}

extern "C" int syzcov_dev_minimize_range(
    const uint64_t *off, const uint32_t *len, const uint32_t *pcs, const uint32_t *split,
    const int32_t *order, const int32_t *ranks, size_t n_items, uint32_t pc_lo, uint64_t pc_span,
    uint32_t range_shift, const uint64_t *range_tot, uint32_t *covered, int32_t *first_w,
    uint64_t *rec, uint64_t rec_cap, uint64_t *rec_cnt, uint8_t *cand, uint8_t *kept, int do_pass2,
    size_t first_chunk, uint32_t growth, uint64_t pcs_per_wg_hint, void *ws, void *stream) {
    return minimize_range_impl(off, len, pcs, split, order, ranks, n_items, pc_lo, pc_span,
                               range_shift, range_tot, covered, first_w, rec, rec_cap, rec_cnt,
                               cand, kept, do_pass2, first_chunk, growth, pcs_per_wg_hint, nullptr,
                               nullptr, ws, stream);
}

extern "C" int syzcov_dev_minimize_range_keys(
    const uint64_t *off, const uint32_t *len, const uint32_t *words, const uint32_t *split,
    const int32_t *order, const int32_t *ranks, size_t n_items, uint64_t nkeys,
    uint32_t range_shift, const uint64_t *range_tot, const uint8_t *low_of_key, uint32_t *covered,
    int32_t *first_w, uint64_t *rec, uint64_t rec_cap, uint64_t *rec_cnt, uint8_t *cand,
    uint8_t *kept, int do_pass2, uint32_t *err_flag, void *ws, void *stream) {
    if (!low_of_key) return SYZCOV_EINVAL;
    return minimize_range_impl(off, len, words, split, order, ranks, n_items, 0, nkeys, range_shift,
                               range_tot, covered, first_w, rec, rec_cap, rec_cnt, cand, kept,
                               do_pass2, 0, 0, 0, low_of_key, err_flag, ws, stream);
}

extern "C" int syzcov_dev_minimize_range_pass2(
    const uint64_t *off, const uint32_t *len, const uint32_t *pcs, const uint32_t *split,
    const int32_t *order, const int32_t *ranks, size_t n_items, uint32_t pc_lo, uint64_t pc_span,
    uint32_t range_shift, const uint64_t *range_tot, uint32_t *covered, int32_t *first_w,
    uint64_t *rec, uint64_t rec_cap, uint64_t *rec_cnt, uint8_t *cand, const uint64_t *tab,
    const int32_t *first_dense, uint8_t *kept, void *ws, void *stream) {
    if (n_items == 0) return 0;
    if (!kept || (tab && !first_dense)) return SYZCOV_EINVAL;
    mr::Args A;
    int rc = mr_args(A, off, len, pcs, split, order, ranks, n_items, pc_lo, pc_span, range_shift,
                     range_tot, covered, first_w, rec, rec_cap, rec_cnt, cand, ws);
    if (rc) return rc;
    return mr_pass2(A, pc_span, tab, first_dense, kept, (hipStream_t)stream);
}

extern "C" int syzcov_dev_minimize_range_keys_pass2(
    const uint64_t *off, const uint32_t *len, const uint32_t *words, const uint32_t *split,
    const int32_t *order, const int32_t *ranks, size_t n_items, uint64_t nkeys,
    uint32_t range_shift, const uint64_t *range_tot, uint32_t *covered, int32_t *first_w,
    uint64_t *rec, uint64_t rec_cap, uint64_t *rec_cnt, uint8_t *cand, uint8_t *kept, void *ws,
    void *stream) {
    if (n_items == 0) return 0;
    if (!kept) return SYZCOV_EINVAL;
    mr::Args A;
    int rc = mr_args(A, off, len, words, split, order, ranks, n_items, 0, nkeys, range_shift,
                     range_tot, covered, first_w, rec, rec_cap, rec_cnt, cand, ws);
    if (rc) return rc;
    A.keymask = SYZ_KEY_MASK;  // the overflow fallback reads the words
    return mr_pass2(A, nkeys, nullptr, nullptr, kept, (hipStream_t)stream);
}

extern "C" int syzcov_dev_first_dense(const uint64_t *tab, uint64_t pc_span, int32_t *first_w,
                                      int32_t *dense, int to_dense, void *stream) {
    if (!tab || !first_w || !dense || pc_span == 0) return SYZCOV_EINVAL;
    const uint64_t nwords = (pc_span + 31) / 32;
    hipLaunchKernelGGL(mr::first_dense_kernel, dim3(grid_for(nwords, 256, 16384)), dim3(256), 0,
                       (hipStream_t)stream, tab, nwords, first_w, dense, to_dense);
    SYZ_LAUNCH_CHECK();
    return 0;
}
