// corpus.hip — the resident corpus engine behind one C-ABI handle
// (include/syzcov.h, "resident corpus engine"): the benchmarked C2/C3 path,
// callable from Go over cgo exactly as bench.py drives it.
//
// One step over a raw corpus already in HBM (CSR off u64[n+1], raw KCOV PCs):
//   canon    Canonicalize every input (cover/cover.go:27-40), per-range split
//            points (canon_wave.hip)
//   order    Go sort.Sort(minInputArray) (cover.go:113) over the canonical
//            lengths, or the raw lengths (cover.Minimize on covers as given)
//   minimize first-cover Minimize (cover.go:104-131; minimize_range.hip)
//   finish   kept inputs in processing order, the sorted union (the
//            `Union(total, cov)` fold, manager.go:606-610) and the resident
//            maxCover |= union
// Sharded (one handle per GPU, n_global > n_max): the caller runs the
// collectives between the phase calls (syzkaller_amd/dist.py over RCCL, or the
// Go host's own RCCL calls on the buffers syzcov_corpus_buffer exposes).
//
// Every buffer lives in one device block, carved by a fixed layout, either
// allocated by the handle or handed in by the caller (torch's caching
// allocator in Python), so the exchanged buffers can be wrapped as tensors.
#include <algorithm>
#include <mutex>
#include <new>
#include <vector>

#include "common.h"

namespace syz {

// int64 lengths for the order: canonical (len32) or raw (from the offsets)
__global__ void corpus_lens_kernel(const uint32_t *__restrict__ len32,
                                   const uint64_t *__restrict__ off, uint64_t n,
                                   int64_t *__restrict__ lens) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        lens[i] = len32 ? (int64_t)len32[i] : (int64_t)(off[i + 1] - off[i]);
}

// a caller's order into ORDER; an entry outside [0, N) becomes 0 (no kernel
// indexes past the corpus) and fails the step
__global__ void corpus_order_copy_kernel(const int32_t *__restrict__ src, uint64_t N,
                                         int32_t *__restrict__ dst, uint32_t *err) {
    bool bad = false;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const int32_t v = src[i];
        const bool ok = (uint64_t)(uint32_t)v < N;
        dst[i] = ok ? v : 0;
        bad |= !ok;
    }
    if (__ballot(bad) && __lane_id() == 0) atomicOr(err, SYZCOV_ERR_ORDER);
}

// the union drops the sentinel (cover.go:97): its covered bit goes before the
// maxCover merge
__global__ void corpus_clear_bit_kernel(uint32_t *covered, uint32_t bit) {
    covered[bit >> 5] &= ~(1u << (bit & 31));
}

// sharded: this shard's error flags ride in the spare kept bytes through the
// kept MAX all-reduce, ONE BYTE PER FLAG BIT (kept[N + b] = bit b), so the
// MAX of each byte is the OR of that bit over the shards; finish ORs them back
// (every rank fails a step any shard flagged, with the same flags: its aliased
// first covers went into the MIN merge)
constexpr uint32_t kErrBytes = 4;  // SYZCOV_ERR_WINDOW .. SYZCOV_ERR_ORDER
// a flag bit added past SYZCOV_ERR_ORDER needs a kept byte of its own (and
// KEPT / the exchange grow with it: syzcov.h "N + 4")
static_assert((SYZCOV_ERR_ORDER << 1) == (1u << kErrBytes),
              "one spare kept byte per SYZCOV_ERR_* bit");
__global__ void corpus_err_to_kept_kernel(const uint32_t *err, uint8_t *kept_n) {
    for (uint32_t b = 0; b < kErrBytes; b++) kept_n[b] = (uint8_t)((*err >> b) & 1u);
}
__global__ void corpus_err_from_kept_kernel(uint32_t *err, const uint8_t *kept_n) {
    uint32_t e = 0;
    for (uint32_t b = 0; b < kErrBytes; b++) e |= (kept_n[b] ? 1u : 0u) << b;
    *err |= e;
}

// maxCover |= covered, unless the step saw a PC outside the key space (its
// covered bits may then stand for an aliased PC: the union is recomputed in
// window mode, corpus_fallback); the popcount either way.
__global__ __launch_bounds__(256) void corpus_merge_kernel(uint32_t *__restrict__ maxc,
                                                           const uint32_t *__restrict__ cov,
                                                           uint64_t nwords, const uint32_t *err,
                                                           unsigned long long *pop) {
    const bool skip = (*err & (SYZCOV_ERR_UNIVERSE | SYZCOV_ERR_WINDOW)) != 0;
    uint32_t cnt = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t m = skip ? maxc[i] : (maxc[i] | cov[i]);
        if (!skip) maxc[i] = m;
        cnt += __popc(m);
    }
    for (int d = 32; d >= 1; d >>= 1) cnt += __shfl_xor(cnt, d, 64);
    if (__lane_id() == 0 && cnt) atomicAdd(pop, (unsigned long long)cnt);
}

// The representable PCs of a window-mode fallback union into maxCover: key
// mode, a PC that is its key's universe PC; window mode, a PC in the window.
__global__ void corpus_merge_pcs_kernel(const uint32_t *__restrict__ pcs, uint32_t n,
                                        const uint32_t *__restrict__ pc_of_key, uint32_t kshift,
                                        uint32_t kbase, uint32_t lo, uint64_t span,
                                        uint32_t *__restrict__ maxc,
                                        unsigned long long *missed) {
    uint32_t miss = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t pc = pcs[i];
        uint64_t b;
        if (pc_of_key) {
            b = (uint64_t)(pc >> kshift) - kbase;
            if ((pc >> kshift) < kbase || b >= span || pc_of_key[b] != pc) {
                miss++;
                continue;
            }
        } else {
            b = (uint64_t)pc - lo;
            if (pc < lo || b >= span) {
                miss++;
                continue;
            }
        }
        atomicOr(&maxc[b >> 5], 1u << (b & 31));
    }
    for (int d = 32; d >= 1; d >>= 1) miss += __shfl_xor(miss, d, 64);
    if (__lane_id() == 0 && miss) atomicAdd(missed, (unsigned long long)miss);
}

__global__ __launch_bounds__(256) void corpus_popcount_kernel(const uint32_t *__restrict__ w,
                                                              uint64_t nwords,
                                                              unsigned long long *pop) {
    uint32_t cnt = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords;
         i += (uint64_t)gridDim.x * blockDim.x)
        cnt += __popc(w[i]);
    for (int d = 32; d >= 1; d >>= 1) cnt += __shfl_xor(cnt, d, 64);
    if (__lane_id() == 0 && cnt) atomicAdd(pop, (unsigned long long)cnt);
}

// Minimize's LDS-resident ranges: 2^20 window PCs (128 KB of covered bits);
// in key mode 2^17 keys (128 KB of membership bytes | covered bits), or 2^18
// keys of nibbles when every low value fits 2 bits (kshift <= 2, the x86 shape)
constexpr uint32_t kRangeShiftWindow = 20, kRangeShiftKeys = 17, kRangeShiftKeysN4 = 18;
int minimize_range_keys_n4(const uint64_t *off, const uint32_t *len, const uint32_t *words,
                           const uint32_t *split, const int32_t *order, const int32_t *ranks,
                           size_t n_items, uint64_t nkeys, uint32_t range_shift,
                           const uint64_t *range_tot, const uint8_t *low_of_key,
                           uint32_t *covered, int32_t *first_w, uint64_t *rec, uint64_t rec_cap,
                           uint64_t *rec_cnt, uint8_t *cand, uint8_t *kept, int do_pass2,
                           uint32_t *err_flag, void *ws, hipStream_t s, uint64_t *rsort);
int minimize_range_keys_sorted(const uint64_t *off, const uint32_t *len, const uint32_t *words,
                               const uint32_t *split, const int32_t *order, const int32_t *ranks,
                               size_t n_items, uint64_t nkeys, uint32_t range_shift,
                               const uint64_t *range_tot, const uint8_t *low_of_key,
                               uint32_t *covered, int32_t *first_w, uint64_t *rec,
                               uint64_t rec_cap, uint64_t *rec_cnt, uint8_t *cand, uint8_t *kept,
                               int do_pass2, uint32_t *err_flag, void *ws, hipStream_t s,
                               uint64_t *rsort);

struct Corpus {
    std::mutex mu;
    int dev = 0;
    syzcov_corpus_cfg cfg{};
    bool key_mode = false;
    uint32_t kshift = 0, kbase = 0;
    uint32_t win_lo = 0;    // canonicalize's PC window
    uint64_t win_span = 0;
    uint32_t pc_lo = 0;     // minimize / union / maxCover window (key mode: 0, nkeys)
    uint64_t span = 0;
    uint32_t sent_key = 0xFFFFFFFFu;  // index of PC 0xFFFFFFFF in that window, or none
    uint32_t rshift = kRangeShiftWindow, nrange = 1;
    uint32_t ak = 0;        // line-aligned canonical layout: SYZ_ALIGN_K(nrange), 0 = CSR slots
    uint64_t nwords = 0, n_global = 0, union_cap = 0;
    int world = 1;
    bool shard = false;  // the sharded protocol (cfg.n_global given, even at world 1)
    // layout
    uint8_t *mem = nullptr;
    size_t mem_size = 0;
    bool own_mem = false;
    size_t offs[SYZCOV_CORPUS_NBUF] = {}, sizes[SYZCOV_CORPUS_NBUF] = {};
    size_t ws_size = 0, ws2_size = 0;
    // per-step state
    const uint64_t *off = nullptr;  // the step's offsets (order by raw lengths)
    const uint32_t *raw_in = nullptr;  // the step's raw PCs when canon is out of place
    bool allow_fallback = true;     // a PC outside the key space: window-mode recompute
    bool order_given = false;       // the step's order came from the caller (ORDER)
    bool order_lens_given = false;  // ... or was sorted over the caller's lengths
    uint32_t *fb_union = nullptr;   // a fallback union larger than UNION (grow-only)
    size_t fb_union_cap = 0;
    bool fb_union_used = false;     // this step's union lives in fb_union
    uint32_t *canon = nullptr;      // the step's canonical lists (in place: the raw buffer)
    size_t n = 0;                   // inputs of this shard in the step
    size_t N = 0;                   // inputs ordered (the global corpus when sharded)
    bool dict_ready = false;        // tab holds the dictionary of the merged union
    bool pass2_pending = false;     // sharded pass 1 ran, its pass 2 (which resets FIRST) not yet
    // device staging of the drop-in call (grow-only)
    void *stage = nullptr;
    size_t stage_cap = 0;
    template <class T>
    T *buf(int b) const {
        return sizes[b] ? (T *)(mem + offs[b]) : nullptr;
    }
};

static uint64_t nrange_of(uint64_t span, uint32_t rshift) {
    return (span + (1ull << rshift) - 1) >> rshift;
}

// Largest shift <= SYZCOV_KSHIFT_MAX keeping a sorted unique universe
// collision-free: (a >> s) != (b >> s) iff a ^ b has a bit >= s.
static int universe_shift(const uint32_t *u, size_t n, uint32_t *ks) {
    uint32_t s = SYZCOV_KSHIFT_MAX;
    for (size_t i = 1; i < n; i++) {
        if (u[i] <= u[i - 1]) return SYZCOV_EINVAL;
        const uint32_t x = u[i] ^ u[i - 1];
        const uint32_t hb = 31u - (uint32_t)__builtin_clz(x);
        if (hb < s) s = hb;
    }
    *ks = n < 2 ? 0 : s;
    return 0;
}

// Plans the layout (sizes only); returns the total bytes or < 0.
static int64_t plan(Corpus &c) {
    const syzcov_corpus_cfg &g = c.cfg;
    const size_t n = g.n_max, N = c.n_global;
    size_t *sz = c.sizes;
    for (int b = 0; b < SYZCOV_CORPUS_NBUF; b++) sz[b] = 0;
    sz[SYZCOV_CORPUS_CANON] = g.canon_in_place ? 0 : (aligned_words(g.p_max, n, c.ak) + 1) * 4;
    sz[SYZCOV_CORPUS_NEW_LEN] = (n + 1) * 4;
    sz[SYZCOV_CORPUS_SPLIT] = c.nrange > 1 ? n * c.nrange * 4 : 0;
    sz[SYZCOV_CORPUS_RANGE_TOT] = c.nrange * 8;
    sz[SYZCOV_CORPUS_COVERED] = ((uint64_t)c.nrange << c.rshift) / 8;
    sz[SYZCOV_CORPUS_MAX_COVER] = c.nwords * 4;
    sz[SYZCOV_CORPUS_TAB] = c.nwords * 8;
    sz[SYZCOV_CORPUS_FIRST] = c.span * 4;
    // key mode: the records, then their copy sorted by key bucket (Minimize's
    // bucketed first covers, minimize_range.hip bmin_kernel)
    sz[SYZCOV_CORPUS_REC] = g.rec_cap * 8 * (c.key_mode ? 2 : 1);
    sz[SYZCOV_CORPUS_CAND] = n + 1;
    sz[SYZCOV_CORPUS_KEPT] = N + kErrBytes;
    sz[SYZCOV_CORPUS_LENS] = (N + 1) * 8;
    sz[SYZCOV_CORPUS_ORDER] = (N + 1) * 4;
    sz[SYZCOV_CORPUS_KEPT_IDX] = (N + 1) * 4;
    sz[SYZCOV_CORPUS_UNION] = c.union_cap * 4;
    sz[SYZCOV_CORPUS_SCAL] = 16 * 8;
    sz[SYZCOV_CORPUS_PC_OF_KEY] = c.key_mode ? c.span * 4 : 0;
    sz[SYZCOV_CORPUS_LOW_OF_KEY] = c.key_mode ? (uint64_t)c.nrange << c.rshift : 0;
    if (c.shard) {
        sz[SYZCOV_CORPUS_GLENS] = N * 4;
        sz[SYZCOV_CORPUS_SEL] = 0;   // (unused since the items' one compaction; kept in the ABI)
        sz[SYZCOV_CORPUS_IOTA] = 0;
        sz[SYZCOV_CORPUS_ITEMS] = (n + 1) * 4;
        sz[SYZCOV_CORPUS_RANKS] = (n + 1) * 4;
        sz[SYZCOV_CORPUS_FIRST_DENSE] = c.key_mode ? 0 : c.union_cap * 4;
    }
    c.ws_size = std::max({syzcov_dev_canon_split_ws_size(n), syzcov_dev_dict_ws_size(c.span),
                          syzcov_dev_compact_ws_size(N), syzcov_dev_sort_ws_size(N),
                          syzcov_dev_minimize_range_ws_size(N, c.span, c.rshift)});
    sz[SYZCOV_CORPUS_WS] = c.ws_size;
    // sharded: dictionary / compaction scratch apart from ws, which carries
    // minimize's rank-ordered descriptors from pass 1 to pass 2
    c.ws2_size = c.shard ? std::max(syzcov_dev_dict_ws_size(c.span),
                                        syzcov_dev_compact_ws_size(N))
                             : 0;
    sz[SYZCOV_CORPUS_WS2] = c.ws2_size;
    size_t tot = 0;
    for (int b = 0; b < SYZCOV_CORPUS_NBUF; b++) {
        c.offs[b] = tot;
        tot += align_up(sz[b], 256);
    }
    return (int64_t)tot;
}

// Validates cfg and derives the windows; host reads of the universe only.
static int setup(Corpus &c, const syzcov_corpus_cfg *cfg) {
    if (!cfg || cfg->n_max == 0 || cfg->n_max > 0x7FFFFFFF || cfg->p_max == 0 ||
        cfg->max_seg_len == 0)
        return SYZCOV_EINVAL;
    c.cfg = *cfg;
    syzcov_corpus_cfg &g = c.cfg;
    c.n_global = g.n_global ? g.n_global : g.n_max;
    if (c.n_global < g.n_max || c.n_global > 0x7FFFFFFF) return SYZCOV_EINVAL;
    c.world = (int)((c.n_global + g.n_max - 1) / g.n_max);
    c.shard = g.n_global != 0;
    if (g.canon_in_place && g.max_seg_len > 16384) return SYZCOV_EINVAL;
    c.key_mode = g.universe != nullptr;
    if (c.key_mode) {
        if (g.universe_n == 0) return SYZCOV_EINVAL;
        int rc = universe_shift(g.universe, g.universe_n, &c.kshift);
        if (rc) {
            set_error("the PC universe must be sorted and unique");
            return rc;
        }
        const uint32_t lo = g.universe[0], hi = g.universe[g.universe_n - 1];
        c.kbase = lo >> c.kshift;
        c.win_lo = lo;
        c.win_span = (uint64_t)hi - lo + 1;
        c.pc_lo = 0;
        c.span = (uint64_t)(hi >> c.kshift) - c.kbase + 1;
    } else {
        if (g.pc_span == 0 || (uint64_t)g.pc_lo + g.pc_span > (1ull << 32)) return SYZCOV_ERANGE;
        c.win_lo = c.pc_lo = g.pc_lo;
        c.win_span = c.span = g.pc_span;
    }
    // the key of PC 0xFFFFFFFF, which Union drops (cover.go:97).  In key mode
    // only a universe that holds the sentinel has one: another universe PC
    // sharing its key (pc >= 0xFFFFFFC0 at kshift 6) is an ordinary PC
    if (c.key_mode)
        c.sent_key = g.universe[g.universe_n - 1] == 0xFFFFFFFFu ? (uint32_t)(c.span - 1)
                                                                 : 0xFFFFFFFFu;
    else
        c.sent_key = (uint64_t)(0xFFFFFFFFu - c.pc_lo) < c.span ? 0xFFFFFFFFu - c.pc_lo
                                                                : 0xFFFFFFFFu;
    c.rshift = c.key_mode ? kRangeShiftKeys : kRangeShiftWindow;
    if (c.key_mode && c.span > (1ull << 25)) {
        set_error("key space of %llu keys > 2^25", (unsigned long long)c.span);
        return SYZCOV_ERANGE;
    }
    // nibble tables (CSR key words; SYZCOV_FORCE=mr_bytes keeps the bytes)
    if (c.key_mode && c.kshift <= 2 && g.canon_layout == 0 &&
        !(force_flags() & FORCE_MR_BYTES))
        c.rshift = kRangeShiftKeysN4;
    c.nrange = (uint32_t)nrange_of(c.span, c.rshift);
    if (c.nrange > 256) {
        set_error("PC window too wide for the range engine (> 256 ranges of 2^20)");
        return SYZCOV_ERANGE;
    }
    // canon_layout 1, out of place over more than one range: every (input,
    // range) sub-run on its own 128-B lines (common.h).  Not the default: at
    // C3 it cut Minimize from 22.4 to 20.0 ms but its writes took canon from
    // 62.7 to 71.1 ms (C2: 2.85 -> 2.76 and 6.62 -> 7.44).
    if (g.canon_layout < 0 || g.canon_layout > 1) return SYZCOV_EINVAL;
    c.ak = !g.canon_in_place && c.nrange > 1 && g.canon_layout == 1 ? SYZ_ALIGN_K(c.nrange) : 0;
    c.nwords = (c.span + 31) / 32;
    if (g.rec_cap == 0)
        g.rec_cap = std::max<uint64_t>(1ull << 22, std::min<uint64_t>(g.p_max, 1ull << 26));
    c.union_cap = std::min<uint64_t>(c.span, g.p_max * (uint64_t)c.world) + 1;
    if (g.order_by != 0 && g.order_by != 1) return SYZCOV_EINVAL;
    return 0;
}

static int init_device(Corpus &c, hipStream_t s) {
    const syzcov_corpus_cfg &g = c.cfg;
    SYZ_HIP(hipMemsetAsync(c.mem, 0, c.mem_size, s));
    SYZ_HIP(hipMemsetD32Async((hipDeviceptr_t)c.buf<int32_t>(SYZCOV_CORPUS_FIRST), INT32_MAX,
                              c.span, s));
    if (!c.key_mode) return 0;
    // key tables of the universe (keys.hip), from a staged copy; the
    // membership table is padded to whole ranges with "no universe PC"
    uint32_t *err = (uint32_t *)c.buf<uint64_t>(SYZCOV_CORPUS_SCAL);
    SYZ_HIP(hipMemsetAsync(c.buf<void>(SYZCOV_CORPUS_LOW_OF_KEY), 0x7F,
                           c.sizes[SYZCOV_CORPUS_LOW_OF_KEY], s));
    uint32_t *stage = nullptr;
    SYZ_HIP(hipMalloc(&stage, g.universe_n * 4));
    int rc = 0;
    if (hipMemcpyAsync(stage, g.universe, g.universe_n * 4, hipMemcpyHostToDevice, s) != hipSuccess)
        rc = SYZCOV_EHIP;
    if (!rc)
        rc = syzcov_dev_universe_keymap(stage, g.universe_n, c.kshift, c.kbase, c.span,
                                        c.buf<uint32_t>(SYZCOV_CORPUS_PC_OF_KEY),
                                        c.buf<uint8_t>(SYZCOV_CORPUS_LOW_OF_KEY), err, s);
    uint32_t h = 0;
    if (!rc && (hipMemcpyAsync(&h, err, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipStreamSynchronize(s) != hipSuccess))
        rc = SYZCOV_EHIP;
    hipFree(stage);
    if (rc) return rc;
    if (h) {
        set_error("universe keymap failed (unsorted or colliding universe)");
        return SYZCOV_EINVAL;
    }
    SYZ_HIP(hipMemsetAsync(err, 0, 8, s));
    return 0;
}

static Corpus *get(syzcov_corpus h) { return reinterpret_cast<Corpus *>(h); }

// Scalars (u64 words of SCAL): 0 err flags (u32), 1 n_ids (u32), 2 n_kept
// (u32), 3 n_union (u32), 4 |maxCover| (u64), 5 / 6 local ranks / items
// (u32), 7 record count (u64), 10 fallback min/max PC (2 x u32), 11 fallback
// union PCs maxCover cannot represent (u64).
enum { SC_ERR = 0, SC_NIDS = 1, SC_NKEPT = 2, SC_NUNION = 3, SC_MAXCOV = 4, SC_CR = 5,
       SC_CI = 6, SC_REC = 7, SC_MM = 10, SC_MISSED = 11 };

// SCAL[0] bit: the step was recomputed by corpus_fallback (results valid)
constexpr uint32_t kErrRecomputed = 1u << 31;

static uint64_t *scal(const Corpus &c) { return c.buf<uint64_t>(SYZCOV_CORPUS_SCAL); }
static bool sharded(const Corpus &c) { return c.shard; }
// the canonical lists in the line-aligned layout (common.h): out of place, R > 1
static bool aligned(const Corpus &c) { return c.ak != 0; }

// --------------------------------------------------------------- phases
static int ph_canon(Corpus &c, const uint64_t *off, uint32_t *raw, size_t n, hipStream_t s) {
    if (!off || !raw || n == 0 || n > c.cfg.n_max) return SYZCOV_EINVAL;
    c.off = off;
    c.raw_in = c.cfg.canon_in_place ? nullptr : raw;
    c.fb_union_used = false;
    c.n = n;
    c.N = n;
    c.dict_ready = false;
    if (c.pass2_pending) {
        // a sharded step abandoned between pass 1 and pass 2 (e.g. a failed
        // collective) left its ranks, and in key mode the merged ranks of every
        // shard, in FIRST: pass 1 would atomicMin against them
        SYZ_HIP(hipMemsetD32Async((hipDeviceptr_t)c.buf<int32_t>(SYZCOV_CORPUS_FIRST), INT32_MAX,
                                  c.span, s));
        c.pass2_pending = false;
    }
    uint64_t *sc = scal(c);
    SYZ_HIP(hipMemsetAsync(sc, 0, 16 * 8, s));
    uint64_t *rt = c.buf<uint64_t>(SYZCOV_CORPUS_RANGE_TOT);
    SYZ_HIP(hipMemsetAsync(rt, 0, c.nrange * 8, s));
    c.canon = c.cfg.canon_in_place ? raw : c.buf<uint32_t>(SYZCOV_CORPUS_CANON);
    uint32_t *nl = c.buf<uint32_t>(SYZCOV_CORPUS_NEW_LEN);
    uint32_t *split = c.buf<uint32_t>(SYZCOV_CORPUS_SPLIT);
    void *ws = c.buf<void>(SYZCOV_CORPUS_WS);
    if (aligned(c))  // line-aligned sub-runs for Minimize's pass 1 (common.h)
        return syzcov_dev_canon_split_aligned(off, raw, c.canon, nl, n, c.cfg.max_seg_len,
                                              c.win_lo, c.win_span, c.kshift, c.kbase, c.span,
                                              c.key_mode, c.rshift, split, rt, (uint32_t *)sc, ws,
                                              c.ws_size, s);
    if (c.key_mode)
        return syzcov_dev_canon_split_keys(off, raw, c.canon, nl, n, c.cfg.max_seg_len, c.win_lo,
                                           c.win_span, c.kshift, c.kbase, c.span, c.rshift, split,
                                           rt, (uint32_t *)sc, ws, c.ws_size, s);
    return syzcov_dev_canon_split(off, raw, c.canon, nl, n, c.cfg.max_seg_len, c.pc_lo, c.span,
                                  c.rshift, split, rt, (uint32_t *)sc, ws, c.ws_size, s);
}

// Go's order over N lengths; also clears Minimize's inputs (queued ahead of
// the sort, whose read-backs leave the GPU idle while the host issues).
static int order_begin(Corpus &c, bool global, size_t N, hipStream_t s) {
    if (!c.canon) return SYZCOV_EINVAL;  // no canon phase yet
    if (!global && N != c.n) return SYZCOV_EINVAL;
    if (N < c.n || N > c.n_global) return SYZCOV_EINVAL;
    if (c.shard && (uint64_t)c.cfg.rank * c.cfg.n_max + c.n > N) return SYZCOV_EINVAL;
    c.N = N;
    SYZ_HIP(hipMemsetAsync(c.buf<void>(SYZCOV_CORPUS_COVERED), 0, c.sizes[SYZCOV_CORPUS_COVERED],
                           s));
    SYZ_HIP(hipMemsetAsync(c.buf<void>(SYZCOV_CORPUS_CAND), 0, c.n, s));
    SYZ_HIP(hipMemsetAsync(c.buf<void>(SYZCOV_CORPUS_KEPT), 0, c.sizes[SYZCOV_CORPUS_KEPT], s));
    return 0;
}

// The caller's order (device int32[N]) instead of the restated sort.
static int ph_order_given(Corpus &c, const int32_t *order, size_t N, hipStream_t s) {
    if (!order) return SYZCOV_EINVAL;
    int rc = order_begin(c, c.shard, N, s);
    if (rc) return rc;
    c.order_given = true;
    c.order_lens_given = false;
    hipLaunchKernelGGL(corpus_order_copy_kernel, dim3(grid_for(N, 256, 8192)), dim3(256), 0, s,
                       order, (uint64_t)N, c.buf<int32_t>(SYZCOV_CORPUS_ORDER),
                       (uint32_t *)(scal(c) + SC_ERR));
    SYZ_LAUNCH_CHECK();
    return 0;
}

int sort_order_part_dev(const int64_t *lens, size_t n, uint32_t part, uint32_t nparts,
                        int32_t *order, void *ws, size_t ws_size, uint32_t *err_dev,
                        hipStream_t s);

// nparts > 1: this shard's part of the order only (syzcov_dev_sort_order_part);
// the caller MAX all-reduces ORDER[:N] before minimize
static int ph_order(Corpus &c, const int32_t *lens32, size_t N, hipStream_t s, uint32_t part = 0,
                    uint32_t nparts = 1) {
    int rc = order_begin(c, lens32 != nullptr, N, s);
    if (rc) return rc;
    c.order_given = false;
    c.order_lens_given = lens32 != nullptr && !c.shard;
    int64_t *lens = c.buf<int64_t>(SYZCOV_CORPUS_LENS);
    const uint32_t *l32 = lens32 ? (const uint32_t *)lens32
                                 : (c.cfg.order_by ? nullptr
                                                   : c.buf<uint32_t>(SYZCOV_CORPUS_NEW_LEN));
    hipLaunchKernelGGL(corpus_lens_kernel, dim3(grid_for(N, 256, 8192)), dim3(256), 0, s, l32,
                       c.off, (uint64_t)N, lens);
    SYZ_LAUNCH_CHECK();
    // (an internal sort error fails the step through its flags: no host sync)
    return sort_order_part_dev(lens, N, part, nparts, c.buf<int32_t>(SYZCOV_CORPUS_ORDER),
                               c.buf<void>(SYZCOV_CORPUS_WS), c.ws_size,
                               (uint32_t *)(scal(c) + SC_ERR), s);
}

int compact_shard_items(const int32_t *order, size_t n, uint32_t base, uint32_t n_local,
                        int32_t *ranks, int32_t *items, uint32_t *n_out, void *ws, hipStream_t s);

// Work items: (input, rank).  One GPU: every input, ranks = positions of
// the order.  Sharded: this shard's inputs in global processing order with
// their GLOBAL ranks, by two ordered compactions (no host sync).
static int items_of(Corpus &c, const int32_t **items, const int32_t **ranks, hipStream_t s) {
    if (!sharded(c)) {
        *items = c.buf<int32_t>(SYZCOV_CORPUS_ORDER);
        *ranks = nullptr;
        return 0;
    }
    const uint32_t base = (uint32_t)(c.cfg.rank * c.cfg.n_max);
    int32_t *it = c.buf<int32_t>(SYZCOV_CORPUS_ITEMS), *rk = c.buf<int32_t>(SYZCOV_CORPUS_RANKS);
    const int32_t *order = c.buf<int32_t>(SYZCOV_CORPUS_ORDER);
    // one ordered compaction writes both (minimize.hip compact_shard_items)
    int rc = compact_shard_items(order, c.N, base, (uint32_t)c.n, rk, it,
                                 (uint32_t *)(scal(c) + SC_CR), c.buf<void>(SYZCOV_CORPUS_WS2), s);
    if (rc) return rc;
    *items = it;
    *ranks = rk;
    return 0;
}

static int ph_minimize(Corpus &c, int do_pass2, hipStream_t s) {
    if (!c.canon || !c.N) return SYZCOV_EINVAL;
    if (do_pass2 && sharded(c)) return SYZCOV_EINVAL;  // pass 2 follows the exchange
    const int32_t *items, *ranks;
    int rc = items_of(c, &items, &ranks, s);
    if (rc) return rc;
    const uint32_t *nl = c.buf<uint32_t>(SYZCOV_CORPUS_NEW_LEN);
    const uint32_t *split = c.buf<uint32_t>(SYZCOV_CORPUS_SPLIT);
    const uint64_t *rt = c.buf<uint64_t>(SYZCOV_CORPUS_RANGE_TOT);
    if (!do_pass2) c.pass2_pending = true;
    if (aligned(c))
        return syzcov_dev_minimize_range_aligned(
            c.off, c.canon, split, items, ranks, c.n, c.pc_lo, c.span, c.rshift, rt,
            c.key_mode ? c.buf<uint8_t>(SYZCOV_CORPUS_LOW_OF_KEY) : nullptr,
            c.buf<uint32_t>(SYZCOV_CORPUS_COVERED), c.buf<int32_t>(SYZCOV_CORPUS_FIRST),
            c.buf<uint64_t>(SYZCOV_CORPUS_REC), c.cfg.rec_cap, scal(c) + SC_REC,
            c.buf<uint8_t>(SYZCOV_CORPUS_CAND), c.buf<uint8_t>(SYZCOV_CORPUS_KEPT), do_pass2,
            (uint32_t *)(scal(c) + SC_ERR), c.buf<void>(SYZCOV_CORPUS_WS), s);
    uint64_t *rsort = c.key_mode ? c.buf<uint64_t>(SYZCOV_CORPUS_REC) + c.cfg.rec_cap : nullptr;
    if (c.key_mode && c.rshift == kRangeShiftKeysN4)
        return minimize_range_keys_n4(
            c.off, nl, c.canon, split, items, ranks, c.n, c.span, c.rshift, rt,
            c.buf<uint8_t>(SYZCOV_CORPUS_LOW_OF_KEY), c.buf<uint32_t>(SYZCOV_CORPUS_COVERED),
            c.buf<int32_t>(SYZCOV_CORPUS_FIRST), c.buf<uint64_t>(SYZCOV_CORPUS_REC), c.cfg.rec_cap,
            scal(c) + SC_REC, c.buf<uint8_t>(SYZCOV_CORPUS_CAND),
            c.buf<uint8_t>(SYZCOV_CORPUS_KEPT), do_pass2, (uint32_t *)(scal(c) + SC_ERR),
            c.buf<void>(SYZCOV_CORPUS_WS), s, rsort);
    if (c.key_mode)
        return minimize_range_keys_sorted(
            c.off, nl, c.canon, split, items, ranks, c.n, c.span, c.rshift, rt,
            c.buf<uint8_t>(SYZCOV_CORPUS_LOW_OF_KEY), c.buf<uint32_t>(SYZCOV_CORPUS_COVERED),
            c.buf<int32_t>(SYZCOV_CORPUS_FIRST), c.buf<uint64_t>(SYZCOV_CORPUS_REC), c.cfg.rec_cap,
            scal(c) + SC_REC, c.buf<uint8_t>(SYZCOV_CORPUS_CAND),
            c.buf<uint8_t>(SYZCOV_CORPUS_KEPT), do_pass2, (uint32_t *)(scal(c) + SC_ERR),
            c.buf<void>(SYZCOV_CORPUS_WS), s, rsort);
    return syzcov_dev_minimize_range(
        c.off, nl, c.canon, split, items, ranks, c.n, c.pc_lo, c.span, c.rshift, rt,
        c.buf<uint32_t>(SYZCOV_CORPUS_COVERED), c.buf<int32_t>(SYZCOV_CORPUS_FIRST),
        c.buf<uint64_t>(SYZCOV_CORPUS_REC), c.cfg.rec_cap, scal(c) + SC_REC,
        c.buf<uint8_t>(SYZCOV_CORPUS_CAND), c.buf<uint8_t>(SYZCOV_CORPUS_KEPT), do_pass2, 0, 0, 0,
        c.buf<void>(SYZCOV_CORPUS_WS), s);
}

int minimize_range_groups(const uint64_t *off, const uint32_t *len, const uint32_t *pcs,
                          const uint32_t *split, const int32_t *order, size_t n_items,
                          uint32_t pc_lo, uint64_t pc_span, uint32_t range_shift,
                          const uint64_t *range_tot, const uint8_t *low_of_key, uint32_t *covered,
                          int32_t *first_w, uint64_t *rec, uint64_t rec_cap, uint64_t *rec_cnt,
                          uint8_t *cand, uint8_t *kept, uint32_t *err_flag,
                          const uint64_t *grp_off, uint32_t ngroups, void *ws, hipStream_t s,
                          int aligned);

// Minimize per group of ranks [grp_off[g], grp_off[g+1]) (host offsets), one
// GPU: Manager.minimizeCorpus's per-call cover.Minimize (manager.go:516-524)
// over an order that concatenates the groups' own sort.Sort orders.
static int ph_minimize_groups(Corpus &c, const uint64_t *grp_off, uint32_t ngroups,
                              hipStream_t s) {
    if (!c.canon || !c.N || c.shard) return SYZCOV_EINVAL;
    return minimize_range_groups(
        c.off, c.buf<uint32_t>(SYZCOV_CORPUS_NEW_LEN), c.canon, c.buf<uint32_t>(SYZCOV_CORPUS_SPLIT),
        c.buf<int32_t>(SYZCOV_CORPUS_ORDER), c.n, c.pc_lo, c.span, c.rshift,
        c.buf<uint64_t>(SYZCOV_CORPUS_RANGE_TOT),
        c.key_mode ? c.buf<uint8_t>(SYZCOV_CORPUS_LOW_OF_KEY) : nullptr,
        c.buf<uint32_t>(SYZCOV_CORPUS_COVERED), c.buf<int32_t>(SYZCOV_CORPUS_FIRST),
        c.buf<uint64_t>(SYZCOV_CORPUS_REC), c.cfg.rec_cap, scal(c) + SC_REC,
        c.buf<uint8_t>(SYZCOV_CORPUS_CAND), c.buf<uint8_t>(SYZCOV_CORPUS_KEPT),
        (uint32_t *)(scal(c) + SC_ERR), grp_off, ngroups, c.buf<void>(SYZCOV_CORPUS_WS), s,
        aligned(c));
}

// Window mode, sharded: the dictionary of the merged covered set and this
// shard's first ranks over it (the MIN exchange moves n_ids entries).
static int64_t ph_dense_first(Corpus &c, hipStream_t s) {
    if (c.key_mode || !sharded(c)) return SYZCOV_EINVAL;
    uint64_t *tab = c.buf<uint64_t>(SYZCOV_CORPUS_TAB);
    int rc = syzcov_dev_dict_build_bits(c.buf<uint32_t>(SYZCOV_CORPUS_COVERED), c.span, tab,
                                        (uint32_t *)(scal(c) + SC_NIDS),
                                        c.buf<void>(SYZCOV_CORPUS_WS2), s);
    if (rc) return rc;
    rc = syzcov_dev_first_dense(tab, c.span, c.buf<int32_t>(SYZCOV_CORPUS_FIRST),
                                c.buf<int32_t>(SYZCOV_CORPUS_FIRST_DENSE), 1, s);
    if (rc) return rc;
    uint32_t nids = 0;
    SYZ_HIP(hipMemcpyAsync(&nids, scal(c) + SC_NIDS, 4, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    c.dict_ready = true;
    return nids;
}

// Sharded pass 2 against the exchanged first ranks: key mode reads the MIN
// all-reduced first-cover array itself (its union = keys with a first cover),
// window mode the MIN-merged dense table.
static int ph_pass2(Corpus &c, hipStream_t s) {
    if (!sharded(c)) return SYZCOV_EINVAL;
    const int32_t *items = c.buf<int32_t>(SYZCOV_CORPUS_ITEMS);
    const int32_t *ranks = c.buf<int32_t>(SYZCOV_CORPUS_RANKS);
    int32_t *first = c.buf<int32_t>(SYZCOV_CORPUS_FIRST);
    if (c.key_mode) {
        int rc = syzcov_dev_first_to_bits(first, c.span, c.buf<uint32_t>(SYZCOV_CORPUS_COVERED), s);
        if (rc) return rc;
    } else if (!c.dict_ready) {
        return SYZCOV_EINVAL;
    }
    const uint32_t *nl = c.buf<uint32_t>(SYZCOV_CORPUS_NEW_LEN);
    const uint32_t *split = c.buf<uint32_t>(SYZCOV_CORPUS_SPLIT);
    const uint64_t *rt = c.buf<uint64_t>(SYZCOV_CORPUS_RANGE_TOT);
    uint32_t *cov = c.buf<uint32_t>(SYZCOV_CORPUS_COVERED);
    uint64_t *rec = c.buf<uint64_t>(SYZCOV_CORPUS_REC);
    uint8_t *cand = c.buf<uint8_t>(SYZCOV_CORPUS_CAND), *kept = c.buf<uint8_t>(SYZCOV_CORPUS_KEPT);
    int rc = aligned(c)
                 ? syzcov_dev_minimize_range_aligned_pass2(
                       c.off, c.canon, split, items, ranks, c.n, c.pc_lo, c.span, c.rshift, rt,
                       c.key_mode, cov, first, rec, c.cfg.rec_cap, scal(c) + SC_REC, cand,
                       c.key_mode ? nullptr : c.buf<uint64_t>(SYZCOV_CORPUS_TAB),
                       c.key_mode ? nullptr : c.buf<int32_t>(SYZCOV_CORPUS_FIRST_DENSE), kept,
                       c.buf<void>(SYZCOV_CORPUS_WS), s)
             : c.key_mode
                 ? syzcov_dev_minimize_range_keys_pass2(
                       c.off, nl, c.canon, split, items, ranks, c.n, c.span, c.rshift, rt, cov,
                       first, rec, c.cfg.rec_cap, scal(c) + SC_REC, cand, kept,
                       c.buf<void>(SYZCOV_CORPUS_WS), s)
                 : syzcov_dev_minimize_range_pass2(
                       c.off, nl, c.canon, split, items, ranks, c.n, c.pc_lo, c.span, c.rshift, rt,
                       cov, first, rec, c.cfg.rec_cap, scal(c) + SC_REC, cand,
                       c.buf<uint64_t>(SYZCOV_CORPUS_TAB),
                       c.buf<int32_t>(SYZCOV_CORPUS_FIRST_DENSE), kept,
                       c.buf<void>(SYZCOV_CORPUS_WS), s);
    if (rc) return rc;
    // the other ranks' entries of the merged array too (pass 2 resets only
    // this shard's records above the fill threshold)
    if (c.key_mode) SYZ_HIP(hipMemsetD32Async((hipDeviceptr_t)first, INT32_MAX, c.span, s));
    c.pass2_pending = false;
    hipLaunchKernelGGL(corpus_err_to_kept_kernel, dim3(1), dim3(1), 0, s,
                       (const uint32_t *)(scal(c) + SC_ERR), kept + c.N);
    SYZ_LAUNCH_CHECK();
    return 0;
}

// kept list in processing order, the sorted union, maxCover |= union.
static int ph_finish(Corpus &c, hipStream_t s) {
    if (!c.N) return SYZCOV_EINVAL;
    uint64_t *sc = scal(c);
    if (sharded(c)) {  // the MAX-merged error byte of every shard (ph_pass2)
        hipLaunchKernelGGL(corpus_err_from_kept_kernel, dim3(1), dim3(1), 0, s,
                           (uint32_t *)(sc + SC_ERR), c.buf<uint8_t>(SYZCOV_CORPUS_KEPT) + c.N);
        SYZ_LAUNCH_CHECK();
    }
    void *wsx = sharded(c) ? c.buf<void>(SYZCOV_CORPUS_WS2) : c.buf<void>(SYZCOV_CORPUS_WS);
    uint64_t *tab = c.buf<uint64_t>(SYZCOV_CORPUS_TAB);
    uint32_t *covered = c.buf<uint32_t>(SYZCOV_CORPUS_COVERED);
    int rc = syzcov_dev_compact_kept(c.buf<uint8_t>(SYZCOV_CORPUS_KEPT),
                                     c.buf<int32_t>(SYZCOV_CORPUS_ORDER), c.N,
                                     c.buf<int32_t>(SYZCOV_CORPUS_KEPT_IDX),
                                     (uint32_t *)(sc + SC_NKEPT), wsx, s);
    if (rc) return rc;
    if (!c.dict_ready) {
        rc = syzcov_dev_dict_build_bits(covered, c.span, tab, (uint32_t *)(sc + SC_NIDS), wsx, s);
        if (rc) return rc;
    }
    // Union drops 0xFFFFFFFF (cover.go:97): in key mode, its key
    uint32_t *un = c.buf<uint32_t>(SYZCOV_CORPUS_UNION);
    rc = syzcov_dev_dict_to_list_drop(tab, c.span, c.pc_lo,
                                      c.key_mode ? c.sent_key : 0xFFFFFFFFu, un,
                                      (uint32_t *)(sc + SC_NUNION), s);
    if (rc) return rc;
    if (c.key_mode) {  // sorted keys -> sorted PCs (the key map is monotone)
        rc = syzcov_dev_keys_to_pcs(c.buf<uint32_t>(SYZCOV_CORPUS_PC_OF_KEY), c.span, un, un,
                                    (const uint32_t *)(sc + SC_NUNION), c.union_cap, s);
        if (rc) return rc;
    }
    if (c.sent_key != 0xFFFFFFFFu) {
        hipLaunchKernelGGL(corpus_clear_bit_kernel, dim3(1), dim3(1), 0, s, covered, c.sent_key);
        SYZ_LAUNCH_CHECK();
    }
    SYZ_HIP(hipMemsetAsync(sc + SC_MAXCOV, 0, 8, s));
    hipLaunchKernelGGL(corpus_merge_kernel, dim3(grid_for(c.nwords, 256, 1024)), dim3(256), 0, s,
                       c.buf<uint32_t>(SYZCOV_CORPUS_MAX_COVER), (const uint32_t *)covered,
                       (uint64_t)c.nwords, (const uint32_t *)(sc + SC_ERR),
                       (unsigned long long *)(sc + SC_MAXCOV));
    SYZ_LAUNCH_CHECK();
    return 0;
}

static int ph_order_given(Corpus &c, const int32_t *order, size_t N, hipStream_t s);
static int ph_result(Corpus &c, syzcov_corpus_res *r, hipStream_t s);
int minmax_pcs(const uint32_t *pcs, size_t n, uint32_t *mm, hipStream_t s);

// A step that saw a PC outside the handle's key space (key mode: a PC not in
// the registered universe, which would alias a universe PC; either mode: a PC
// outside the window) is recomputed by a transient window-mode engine over the
// step's own PC extent: cover.Minimize (cover.go:104-131) never fails on a u32
// input, so neither does the handle.  It needs the raw PCs (out-of-place
// canon; the host form restages them) and one GPU (a sharded step fails on
// every rank instead).  The kept list and the union land in this handle's
// buffers; maxCover takes the union's PCs it can represent.  `order`: the
// step's own order when the caller gave it, else canonical / raw lengths as cfg.
static int corpus_fallback(Corpus &c, syzcov_corpus_res *r, hipStream_t s) {
    // the caller's order, or the order the step computed over the caller's
    // lengths (Go's sort over them, exact): either way the step's ORDER
    const int32_t *order =
        c.order_given || c.order_lens_given ? c.buf<int32_t>(SYZCOV_CORPUS_ORDER) : nullptr;
    if (c.shard || !c.raw_in || !c.off || !c.n || !c.allow_fallback) return 1;
    uint64_t ends[2];
    SYZ_HIP(hipMemcpyAsync(&ends[0], c.off, 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipMemcpyAsync(&ends[1], c.off + c.n, 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    if (ends[1] <= ends[0]) return 1;
    uint32_t *mm = (uint32_t *)(scal(c) + SC_MM);
    int rc = minmax_pcs(c.raw_in + ends[0], ends[1] - ends[0], mm, s);
    if (rc) return rc;
    uint32_t hm[2];
    SYZ_HIP(hipMemcpyAsync(hm, mm, 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    const uint64_t span = (uint64_t)hm[1] - hm[0] + 1;
    if (nrange_of(span, kRangeShiftWindow) > 256) return 1;  // too wide: the error stands
    syzcov_corpus_cfg cfg{};
    cfg.n_max = c.n;
    cfg.p_max = ends[1];  // the CANON buffer is indexed by the step's absolute offsets
    cfg.max_seg_len = c.cfg.max_seg_len;
    cfg.pc_lo = hm[0];
    cfg.pc_span = span;
    cfg.order_by = c.cfg.order_by;
    syzcov_corpus h = 0;
    rc = syzcov_corpus_create(&cfg, nullptr, 0, &h);
    if (rc) return rc;
    Corpus &w = *get(h);
    w.allow_fallback = false;
    syzcov_corpus_res rw{};
    {
        std::lock_guard<std::mutex> g(w.mu);  // same device as c
        rc = ph_canon(w, c.off, const_cast<uint32_t *>(c.raw_in), c.n, s);
        if (!rc) rc = order ? ph_order_given(w, order, c.n, s) : ph_order(w, nullptr, c.n, s);
        if (!rc) rc = ph_minimize(w, 1, s);
        if (!rc) rc = ph_finish(w, s);
        if (!rc) rc = ph_result(w, &rw, s);
        // PCs outside the universe can make the union larger than the key
        // space the UNION buffer is sized for: then it goes to a side buffer
        uint32_t *un = c.buf<uint32_t>(SYZCOV_CORPUS_UNION);
        if (!rc && rw.n_union > c.sizes[SYZCOV_CORPUS_UNION] / 4) {
            if (rw.n_union > c.fb_union_cap) {
                if (c.fb_union) hipFree(c.fb_union);
                c.fb_union = nullptr;
                c.fb_union_cap = 0;
                if (hipMalloc(&c.fb_union, align_up((size_t)rw.n_union * 4, 256)) != hipSuccess)
                    rc = SYZCOV_ENOMEM;
                else c.fb_union_cap = rw.n_union;
            }
            un = c.fb_union;
            c.fb_union_used = true;
        }
        if (!rc && rw.n_kept)
            rc = hipMemcpyAsync(c.buf<int32_t>(SYZCOV_CORPUS_KEPT_IDX), rw.kept_idx,
                                (size_t)rw.n_kept * 4, hipMemcpyDeviceToDevice, s) == hipSuccess
                     ? 0 : SYZCOV_EHIP;
        if (!rc && rw.n_union)
            rc = hipMemcpyAsync(un, rw.union_pcs, (size_t)rw.n_union * 4, hipMemcpyDeviceToDevice,
                                s) == hipSuccess ? 0 : SYZCOV_EHIP;
        if (!rc) {  // maxCover |= the union's representable PCs
            uint64_t *sc = scal(c);
            uint32_t *maxc = c.buf<uint32_t>(SYZCOV_CORPUS_MAX_COVER);
            SYZ_HIP(hipMemsetAsync(sc + SC_MISSED, 0, 8, s));
            if (rw.n_union)
                hipLaunchKernelGGL(corpus_merge_pcs_kernel, dim3(grid_for(rw.n_union, 256, 1024)),
                                   dim3(256), 0, s, (const uint32_t *)un, rw.n_union,
                                   c.key_mode ? c.buf<uint32_t>(SYZCOV_CORPUS_PC_OF_KEY) : nullptr,
                                   c.kshift, c.kbase, c.pc_lo, c.span, maxc,
                                   (unsigned long long *)(sc + SC_MISSED));
            SYZ_HIP(hipMemsetAsync(sc + SC_MAXCOV, 0, 8, s));
            hipLaunchKernelGGL(corpus_popcount_kernel, dim3(grid_for(c.nwords, 256, 1024)),
                               dim3(256), 0, s, (const uint32_t *)maxc, (uint64_t)c.nwords,
                               (unsigned long long *)(sc + SC_MAXCOV));
            SYZ_LAUNCH_CHECK();
            uint64_t mc = 0, missed = 0;
            SYZ_HIP(hipMemcpyAsync(&mc, sc + SC_MAXCOV, 8, hipMemcpyDeviceToHost, s));
            SYZ_HIP(hipMemcpyAsync(&missed, sc + SC_MISSED, 8, hipMemcpyDeviceToHost, s));
            SYZ_HIP(hipStreamSynchronize(s));
            r->max_cover_missed = (uint32_t)std::min<uint64_t>(missed, 0xFFFFFFFFu);
            r->n_ids = rw.n_ids;
            r->n_kept = rw.n_kept;
            r->n_union = rw.n_union;
            r->records = rw.records;
            r->max_cover = mc;
            r->fallback = 1;
            r->union_pcs = un;
            // the step's scalars now describe the recomputed results (a second
            // result call returns them without recomputing)
            uint64_t hs[8];
            SYZ_HIP(hipMemcpyAsync(hs, sc, sizeof hs, hipMemcpyDeviceToHost, s));
            SYZ_HIP(hipStreamSynchronize(s));
            hs[SC_ERR] |= kErrRecomputed;
            hs[SC_NIDS] = rw.n_ids;
            hs[SC_NKEPT] = rw.n_kept;
            hs[SC_NUNION] = rw.n_union;
            hs[SC_MAXCOV] = mc;
            hs[SC_REC] = rw.records;
            SYZ_HIP(hipMemcpyAsync(sc, hs, sizeof hs, hipMemcpyHostToDevice, s));
        }
        hipStreamSynchronize(s);
    }
    syzcov_corpus_destroy(h);
    return rc;
}

static int ph_result(Corpus &c, syzcov_corpus_res *r, hipStream_t s) {
    uint64_t h[16];
    SYZ_HIP(hipMemcpyAsync(h, scal(c), sizeof h, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    const uint32_t err = (uint32_t)h[SC_ERR];
    r->err_flags = err;
    r->n_ids = (uint32_t)h[SC_NIDS];
    r->n_kept = (uint32_t)h[SC_NKEPT];
    r->n_union = (uint32_t)h[SC_NUNION];
    r->max_cover = h[SC_MAXCOV];
    r->records = h[SC_REC];
    r->kept_idx = c.buf<int32_t>(SYZCOV_CORPUS_KEPT_IDX);
    r->union_pcs = c.buf<uint32_t>(SYZCOV_CORPUS_UNION);
    r->fallback = 0;
    r->max_cover_missed = 0;
    if (err & kErrRecomputed) {  // corpus_fallback already ran for this step
        r->err_flags = err & ~kErrRecomputed;
        r->fallback = 1;
        r->max_cover_missed = (uint32_t)std::min<uint64_t>(h[SC_MISSED], 0xFFFFFFFFu);
        if (c.fb_union_used) r->union_pcs = c.fb_union;
        return 0;
    }
    if ((err & (SYZCOV_ERR_WINDOW | SYZCOV_ERR_UNIVERSE)) &&
        !(err & (SYZCOV_ERR_SEGLEN | SYZCOV_ERR_ORDER))) {
        const int rc = corpus_fallback(c, r, s);
        if (rc <= 0) return rc;  // recomputed (0) or failed (< 0); 1: not possible here
    }
    if (err & SYZCOV_ERR_SEGLEN) {
        set_error("an input is longer than max_seg_len=%zu", c.cfg.max_seg_len);
        return SYZCOV_ETOOLONG;
    }
    if (err & SYZCOV_ERR_WINDOW) {
        set_error("a PC fell outside the engine's PC window");
        return SYZCOV_ERANGE;
    }
    if (err & SYZCOV_ERR_UNIVERSE) {
        set_error("a PC is not in the registered PC universe");
        return SYZCOV_ERANGE;
    }
    if (err & SYZCOV_ERR_ORDER) {
        set_error("the processing order holds an entry outside [0, %zu)", c.N);
        return SYZCOV_EINVAL;
    }
    if (err) {
        set_error("engine error flags %#x", err);
        return SYZCOV_EHIP;
    }
    return 0;
}

// RAII: the handle's device current, the handle locked.
class Use {
  public:
    explicit Use(Corpus *c) : c_(c), g_(c->mu) {
        hipGetDevice(&prev_);
        if (prev_ != c->dev) hipSetDevice(c->dev);
    }
    ~Use() {
        if (prev_ != c_->dev) hipSetDevice(prev_);
    }

  private:
    Corpus *c_;
    std::lock_guard<std::mutex> g_;
    int prev_ = 0;
};

// cover.Minimize through an engine handle on host buffers (the drop-in
// call): stage, step, read back.
// Go's order must be a permutation of the inputs (host check, O(n)).
static bool is_permutation(const int32_t *order, size_t n) {
    std::vector<uint8_t> seen(n, 0);
    for (size_t i = 0; i < n; i++) {
        const uint32_t v = (uint32_t)order[i];
        if (v >= n || seen[v]) return false;
        seen[v] = 1;
    }
    return true;
}

static int64_t minimize_host(Corpus &c, const uint64_t *offsets, const uint32_t *pcs, size_t n,
                             const int32_t *order, int32_t *out_idx, uint32_t *union_out,
                             size_t union_out_cap, uint64_t *n_union_out, hipStream_t s) {
    const uint64_t base = offsets[0], P = offsets[n] - base;
    if (P > c.cfg.p_max) return SYZCOV_EINVAL;
    if (order && !is_permutation(order, n)) {
        set_error("the processing order is not a permutation of the %zu inputs", n);
        return SYZCOV_EINVAL;
    }
    std::vector<uint64_t> hoff(n + 1);
    for (size_t i = 0; i <= n; i++) {
        hoff[i] = offsets[i] - base;
        if (i && hoff[i] < hoff[i - 1]) return SYZCOV_EINVAL;
        if (i && hoff[i] - hoff[i - 1] > c.cfg.max_seg_len) {
            set_error("an input is longer than max_seg_len=%zu", c.cfg.max_seg_len);
            return SYZCOV_ETOOLONG;
        }
    }
    const size_t need = align_up((n + 1) * 8, 256) + align_up((P + 1) * 4, 256) + n * 4;
    if (need > c.stage_cap) {
        if (c.stage) {
            SYZ_HIP(hipStreamSynchronize(s));
            hipFree(c.stage);
            c.stage = nullptr;
            c.stage_cap = 0;
        }
        if (hipMalloc(&c.stage, need) != hipSuccess) {
            set_error("hipMalloc(%zu) failed", need);
            return SYZCOV_ENOMEM;
        }
        c.stage_cap = need;
    }
    uint64_t *d_off = (uint64_t *)c.stage;
    uint32_t *d_pcs = (uint32_t *)((uint8_t *)c.stage + align_up((n + 1) * 8, 256));
    int32_t *d_ord = (int32_t *)((uint8_t *)d_pcs + align_up((P + 1) * 4, 256));
    SYZ_HIP(hipMemcpyAsync(d_off, hoff.data(), (n + 1) * 8, hipMemcpyHostToDevice, s));
    if (P) SYZ_HIP(hipMemcpyAsync(d_pcs, pcs + base, P * 4, hipMemcpyHostToDevice, s));
    if (order) SYZ_HIP(hipMemcpyAsync(d_ord, order, n * 4, hipMemcpyHostToDevice, s));
    int rc = ph_canon(c, d_off, d_pcs, n, s);
    if (!rc) rc = order ? ph_order_given(c, d_ord, n, s) : ph_order(c, nullptr, n, s);
    if (!rc) rc = ph_minimize(c, 1, s);
    if (!rc) rc = ph_finish(c, s);
    syzcov_corpus_res r{};
    if (!rc) rc = ph_result(c, &r, s);
    if (rc == SYZCOV_ERANGE && !c.raw_in && (r.err_flags & (SYZCOV_ERR_WINDOW | SYZCOV_ERR_UNIVERSE)) &&
        !(r.err_flags & (SYZCOV_ERR_SEGLEN | SYZCOV_ERR_ORDER)) && P) {
        // canonicalized in place: restage the raw PCs for the window-mode recompute
        if (hipMemcpyAsync(d_pcs, pcs + base, P * 4, hipMemcpyHostToDevice, s) == hipSuccess) {
            c.raw_in = d_pcs;
            const int fr = corpus_fallback(c, &r, s);
            c.raw_in = nullptr;
            if (fr <= 0) rc = fr;
        }
    }
    if (rc) {
        hipStreamSynchronize(s);
        return rc;
    }
    if (r.n_kept)
        SYZ_HIP(hipMemcpyAsync(out_idx, r.kept_idx, (size_t)r.n_kept * 4, hipMemcpyDeviceToHost, s));
    if (n_union_out) *n_union_out = r.n_union;
    if (union_out && r.n_union) {
        if (union_out_cap < r.n_union) {
            hipStreamSynchronize(s);
            set_error("union capacity %zu < %u", union_out_cap, r.n_union);
            return SYZCOV_ERANGE;
        }
        SYZ_HIP(hipMemcpyAsync(union_out, r.union_pcs, (size_t)r.n_union * 4,
                               hipMemcpyDeviceToHost, s));
    }
    SYZ_HIP(hipStreamSynchronize(s));
    return r.n_kept;
}

}  // namespace syz

using namespace syz;

extern "C" {

int64_t syzcov_corpus_mem_size(const syzcov_corpus_cfg *cfg) {
    Corpus c;
    int rc = setup(c, cfg);
    if (rc) return rc;
    return plan(c);
}

int syzcov_corpus_create(const syzcov_corpus_cfg *cfg, void *mem, size_t mem_size,
                         syzcov_corpus *out) {
    if (!out) return SYZCOV_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        set_error("no HIP device (libsyzcov has no CPU path)");
        return SYZCOV_ENODEV;
    }
    Corpus *c = new (std::nothrow) Corpus();
    if (!c) return SYZCOV_ENOMEM;
    int rc = setup(*c, cfg);
    const int64_t need = rc ? rc : plan(*c);
    if (need < 0) {
        delete c;
        return (int)need;
    }
    hipGetDevice(&c->dev);
    c->cfg.universe = nullptr;  // host memory is not retained past the call
    if (mem) {
        if (mem_size < (size_t)need || ((uintptr_t)mem & 255)) {
            delete c;
            set_error("caller memory: %zu bytes at %p, need %lld 256-byte aligned", mem_size, mem,
                      (long long)need);
            return SYZCOV_EINVAL;
        }
        c->mem = (uint8_t *)mem;
    } else {
        if (hipMalloc(&c->mem, (size_t)need) != hipSuccess) {
            delete c;
            set_error("hipMalloc(%lld) failed", (long long)need);
            return SYZCOV_ENOMEM;
        }
        c->own_mem = true;
    }
    c->mem_size = (size_t)need;
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
        rc = SYZCOV_EHIP;
    } else {
        c->cfg.universe = cfg->universe;
        rc = init_device(*c, s);
        c->cfg.universe = nullptr;
        if (!rc && hipStreamSynchronize(s) != hipSuccess) rc = SYZCOV_EHIP;
        hipStreamDestroy(s);
    }
    if (rc) {
        if (c->own_mem) hipFree(c->mem);
        delete c;
        return rc;
    }
    *out = reinterpret_cast<syzcov_corpus>(c);
    return 0;
}

int syzcov_corpus_destroy(syzcov_corpus h) {
    Corpus *c = get(h);
    if (!c) return 0;
    {
        // no device-wide sync: hipFree waits for the work on the memory it
        // frees, and caller-provided memory stays the caller's to retire
        Use u(c);
        if (c->own_mem) hipFree(c->mem);
        if (c->stage) hipFree(c->stage);
        if (c->fb_union) hipFree(c->fb_union);
    }
    delete c;
    return 0;
}

int syzcov_corpus_info(syzcov_corpus h, syzcov_corpus_info_t *out) {
    Corpus *c = get(h);
    if (!c || !out) return SYZCOV_EINVAL;
    out->key_mode = c->key_mode;
    out->kshift = c->kshift;
    out->kbase = c->kbase;
    out->pc_lo = c->pc_lo;
    out->span = c->span;
    out->win_lo = c->win_lo;
    out->win_span = c->win_span;
    out->nrange = c->nrange;
    out->nwords = c->nwords;
    out->n_global = c->n_global;
    out->union_cap = c->union_cap;
    out->rec_cap = c->cfg.rec_cap;
    out->sent_key = c->sent_key;
    out->mem = c->mem;
    out->mem_size = c->mem_size;
    out->canon_align_k = c->ak;
    return 0;
}

// The step's canonical lists in the raw lists' CSR slots (out[off[i] ..
// off[i] + new_len[i])), from whichever layout CANON holds: one wave per
// input copies its sub-runs range by range.
__global__ __launch_bounds__(256) void corpus_unalign_kernel(const uint64_t *__restrict__ off,
                                                             const uint32_t *__restrict__ canon,
                                                             const uint32_t *__restrict__ split,
                                                             const uint32_t *__restrict__ nl,
                                                             uint64_t n, uint32_t nrange,
                                                             uint32_t ak,
                                                             uint32_t *__restrict__ out) {
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / 64);
    for (uint64_t i = (uint64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; i < n; i += nw) {
        const uint64_t ib = aligned_base(off[i], i, ak);
        uint32_t s0 = 0;
        for (uint32_t j = 0; j < nrange; j++) {
            const uint32_t s1 = (split && nrange > 1) ? split[i * nrange + j] : nl[i];
            const uint64_t a = ib + aligned_sub(s0, j, ak);
            for (uint32_t q = __lane_id(); q < s1 - s0; q += 64) out[off[i] + s0 + q] = canon[a + q];
            s0 = s1;
        }
    }
}

int syzcov_corpus_canonical(syzcov_corpus h, uint32_t *out, void *stream) {
    Corpus *c = get(h);
    if (!c || !out || !c->canon || !c->off || !c->n) return SYZCOV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(corpus_unalign_kernel, dim3(grid_for(c->n, 4, 8192)), dim3(256), 0, s, c->off,
                       (const uint32_t *)c->canon, c->buf<uint32_t>(SYZCOV_CORPUS_SPLIT),
                       c->buf<uint32_t>(SYZCOV_CORPUS_NEW_LEN), (uint64_t)c->n, c->nrange, c->ak,
                       out);
    SYZ_LAUNCH_CHECK();
    return 0;
}

int syzcov_corpus_buffer(syzcov_corpus h, int which, uint64_t *offset, uint64_t *bytes) {
    Corpus *c = get(h);
    if (!c || which < 0 || which >= SYZCOV_CORPUS_NBUF) return SYZCOV_EINVAL;
    if (offset) *offset = c->offs[which];
    if (bytes) *bytes = c->sizes[which];
    return 0;
}

int syzcov_corpus_canon(syzcov_corpus h, const uint64_t *off, uint32_t *raw, size_t n,
                        void *stream) {
    Corpus *c = get(h);
    if (!c) return SYZCOV_EINVAL;
    Use u(c);
    return ph_canon(*c, off, raw, n, (hipStream_t)stream);
}

int syzcov_corpus_order(syzcov_corpus h, const int32_t *lens, size_t N, void *stream) {
    Corpus *c = get(h);
    if (!c) return SYZCOV_EINVAL;
    Use u(c);
    return ph_order(*c, lens, N, (hipStream_t)stream);
}

int syzcov_corpus_minimize(syzcov_corpus h, int do_pass2, void *stream) {
    Corpus *c = get(h);
    if (!c) return SYZCOV_EINVAL;
    Use u(c);
    return ph_minimize(*c, do_pass2, (hipStream_t)stream);
}

int64_t syzcov_corpus_dense_first(syzcov_corpus h, void *stream) {
    Corpus *c = get(h);
    if (!c) return SYZCOV_EINVAL;
    Use u(c);
    return ph_dense_first(*c, (hipStream_t)stream);
}

int syzcov_corpus_pass2(syzcov_corpus h, void *stream) {
    Corpus *c = get(h);
    if (!c) return SYZCOV_EINVAL;
    Use u(c);
    return ph_pass2(*c, (hipStream_t)stream);
}

int syzcov_corpus_finish(syzcov_corpus h, void *stream) {
    Corpus *c = get(h);
    if (!c) return SYZCOV_EINVAL;
    Use u(c);
    return ph_finish(*c, (hipStream_t)stream);
}

int syzcov_corpus_step(syzcov_corpus h, const uint64_t *off, uint32_t *raw, size_t n,
                       void *stream) {
    Corpus *c = get(h);
    if (!c) return SYZCOV_EINVAL;
    Use u(c);
    hipStream_t s = (hipStream_t)stream;
    int rc = ph_canon(*c, off, raw, n, s);
    if (!rc) rc = ph_order(*c, nullptr, n, s);
    if (!rc) rc = ph_minimize(*c, 1, s);
    if (!rc) rc = ph_finish(*c, s);
    return rc;
}

int syzcov_corpus_result(syzcov_corpus h, syzcov_corpus_res *res, void *stream) {
    Corpus *c = get(h);
    if (!c || !res) return SYZCOV_EINVAL;
    Use u(c);
    return ph_result(*c, res, (hipStream_t)stream);
}

int64_t syzcov_corpus_minimize_host(syzcov_corpus h, const uint64_t *offsets, const uint32_t *pcs,
                                    size_t n, int32_t *out_idx, uint32_t *union_out,
                                    size_t union_cap, uint64_t *n_union) {
    Corpus *c = get(h);
    if (!c || !offsets || !out_idx || n == 0 || n > c->cfg.n_max) return SYZCOV_EINVAL;
    if (offsets[n] > offsets[0] && !pcs) return SYZCOV_EINVAL;
    Use u(c);
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return SYZCOV_EHIP;
    const int64_t rc =
        minimize_host(*c, offsets, pcs, n, nullptr, out_idx, union_out, union_cap, n_union, s);
    hipStreamDestroy(s);
    return rc;
}

int64_t syzcov_corpus_minimize_host_order(syzcov_corpus h, const uint64_t *offsets,
                                          const uint32_t *pcs, size_t n, const int32_t *order,
                                          int32_t *out_idx, uint32_t *union_out, size_t union_cap,
                                          uint64_t *n_union) {
    Corpus *c = get(h);
    if (!c || !offsets || !order || !out_idx || n == 0 || n > c->cfg.n_max) return SYZCOV_EINVAL;
    if (offsets[n] > offsets[0] && !pcs) return SYZCOV_EINVAL;
    Use u(c);
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return SYZCOV_EHIP;
    const int64_t rc =
        minimize_host(*c, offsets, pcs, n, order, out_idx, union_out, union_cap, n_union, s);
    hipStreamDestroy(s);
    return rc;
}

int syzcov_corpus_order_part(syzcov_corpus h, const int32_t *lens, size_t N, void *stream) {
    Corpus *c = get(h);
    if (!c || !c->shard || !lens) return SYZCOV_EINVAL;
    Use u(c);
    return ph_order(*c, lens, N, (hipStream_t)stream, (uint32_t)c->cfg.rank, (uint32_t)c->world);
}

int syzcov_corpus_order_given(syzcov_corpus h, const int32_t *order, size_t N, void *stream) {
    Corpus *c = get(h);
    if (!c) return SYZCOV_EINVAL;
    Use u(c);
    return ph_order_given(*c, order, N, (hipStream_t)stream);
}

}  // extern "C"

// cover.Minimize (syzcov_minimize, api.cc) on large corpora: a window-mode
// engine over the corpus' own PC extent, CACHED per device across calls (a
// manager minimizes corpora of similar size over the same kernel text, so the
// handle is created once and reused while the corpus fits its capacity and
// window; syzcov_pool_trim releases it).  The corpus is staged once into the
// cache's device buffer, its PC extent taken there (one min/max pass, no host
// scan), and the order is the caller's (Go's own sort.Sort, the shim) or the
// restated sort over the raw lengths (Go sorts by len(cov), duplicates
// included).  Returns 1 with the count in *out_n, 0 if the corpus does not
// suit the engine or the device is short of memory or the cache is busy (the
// caller takes the dictionary path), < 0 on error.
namespace syz {
int minmax_pcs(const uint32_t *pcs, size_t n, uint32_t *mm, hipStream_t s);

struct DropinCache {
    std::mutex mu;
    syzcov_corpus h = 0;
    size_t n_cap = 0, seg_cap = 0;
    uint64_t p_cap = 0;
    uint32_t lo = 0;
    uint64_t span = 0;
    void *stage = nullptr;  // off u64[n+1] | pcs u32[P+1] | order i32[n] | min/max
    size_t stage_cap = 0;
    void *gscratch = nullptr;  // groups_lds: lengths, split points, kept, workspace
    size_t gscratch_cap = 0;
};
// the calling thread's last syzcov_minimize_corpus (syzcov_minimize_corpus_stats)
thread_local syzcov_groups_stats g_gstats{};
// HIP events around a corpus-size minimizeCorpus call: upload | device | download
struct GroupTimer {
    hipEvent_t e[4] = {};
    bool ok = true;
    GroupTimer() {
        for (auto &x : e) ok = ok && hipEventCreate(&x) == hipSuccess;
    }
    ~GroupTimer() {
        for (auto &x : e)
            if (x) hipEventDestroy(x);
    }
    void mark(int i, hipStream_t s) {
        if (ok) ok = hipEventRecord(e[i], s) == hipSuccess;
    }
    void finish(int path) {
        g_gstats = {};
        g_gstats.path = path;
        if (!ok || hipEventSynchronize(e[3]) != hipSuccess) return;
        hipEventElapsedTime(&g_gstats.upload_ms, e[0], e[1]);
        hipEventElapsedTime(&g_gstats.device_ms, e[1], e[2]);
        hipEventElapsedTime(&g_gstats.download_ms, e[2], e[3]);
    }
};
constexpr int kMaxDev = 16;
static DropinCache g_dropin[kMaxDev];

static void dropin_release(DropinCache &dc) {
    if (dc.h) syzcov_corpus_destroy(dc.h);
    if (dc.stage) hipFree(dc.stage);
    if (dc.gscratch) hipFree(dc.gscratch);
    dc.h = 0;
    dc.stage = dc.gscratch = nullptr;
    dc.stage_cap = dc.gscratch_cap = dc.n_cap = dc.seg_cap = dc.p_cap = dc.span = 0;
}

void dropin_trim() {
    int cur = 0;
    hipGetDevice(&cur);
    for (int d = 0; d < kMaxDev; d++) {
        std::lock_guard<std::mutex> g(g_dropin[d].mu);
        if (!g_dropin[d].h && !g_dropin[d].stage) continue;
        hipSetDevice(d);
        dropin_release(g_dropin[d]);
    }
    hipSetDevice(cur);
}

// the handle for a corpus of n inputs / P PCs / longest max_len over [lo, hi]
// (out_of_place: the caller needs the staged raw PCs after the step)
static int dropin_handle(DropinCache &dc, size_t n, uint64_t P, size_t max_len, uint32_t lo,
                         uint32_t hi, bool out_of_place = false) {
    if (dc.h && n <= dc.n_cap && P <= dc.p_cap && max_len <= dc.seg_cap && lo >= dc.lo &&
        (uint64_t)hi - dc.lo < dc.span && (!out_of_place || !get(dc.h)->cfg.canon_in_place))
        return 1;
    // grow: capacities only rise, the window widens to cover both corpora
    // (whole 2^20-PC ranges) while it stays within the engine's 256 ranges
    uint64_t nlo = lo, nhi = hi;
    if (dc.h) {
        nlo = std::min<uint64_t>(lo, dc.lo);
        nhi = std::max<uint64_t>(hi, dc.lo + dc.span - 1);
    }
    nlo &= ~((1ull << kRangeShiftWindow) - 1);
    if (nrange_of(nhi - nlo + 1, kRangeShiftWindow) > 256) {
        nlo = lo & ~((1ull << kRangeShiftWindow) - 1);
        nhi = hi;
        // aligning lo down can add a 257th range to an extent just under
        // 2^28 PCs: then the exact extent (which the caller checked fits)
        if (nrange_of(nhi - nlo + 1, kRangeShiftWindow) > 256) nlo = lo;
    }
    nhi = std::min<uint64_t>(0xFFFFFFFFull, nhi);
    syzcov_corpus_cfg cfg{};
    cfg.n_max = std::max(n, dc.n_cap);
    cfg.p_max = std::max<uint64_t>(P, dc.p_cap);
    cfg.max_seg_len = std::max(max_len, dc.seg_cap);
    cfg.pc_lo = (uint32_t)nlo;
    cfg.pc_span = nhi - nlo + 1;
    cfg.order_by = 1;  // Go sorts by len(cov), duplicates included
    // the staged copy is the cache's own; out of place once a caller asked
    cfg.canon_in_place = cfg.max_seg_len <= 16384 && !out_of_place &&
                         !(dc.h && !get(dc.h)->cfg.canon_in_place);
    if (dc.h) syzcov_corpus_destroy(dc.h);
    dc.h = 0;
    int rc = syzcov_corpus_create(&cfg, nullptr, 0, &dc.h);
    if (rc == SYZCOV_ENOMEM && (cfg.n_max > n || cfg.p_max > P)) {  // retry at this corpus' size
        cfg.n_max = n;
        cfg.p_max = P;
        rc = syzcov_corpus_create(&cfg, nullptr, 0, &dc.h);
    }
    if (rc) {  // short of memory or a window the engine cannot take: the dictionary path
        dc.h = 0;
        return rc == SYZCOV_ENOMEM || rc == SYZCOV_ERANGE ? 0 : rc;
    }
    dc.n_cap = cfg.n_max;
    dc.p_cap = cfg.p_max;
    dc.seg_cap = cfg.max_seg_len;
    dc.lo = cfg.pc_lo;
    dc.span = cfg.pc_span;
    return 1;
}

static int64_t dropin_run(DropinCache &dc, const uint64_t *offsets, const uint32_t *pcs, size_t n,
                          const int32_t *order, int32_t *out_idx, hipStream_t s) {
    const uint64_t base = offsets[0], P = offsets[n] - base;
    size_t max_len = 1;
    std::vector<uint64_t> hoff(n + 1);
    for (size_t i = 0; i <= n; i++) {
        hoff[i] = offsets[i] - base;
        if (i && hoff[i] < hoff[i - 1]) return SYZCOV_EINVAL;
        if (i) max_len = std::max<size_t>(max_len, hoff[i] - hoff[i - 1]);
    }
    if (order && !is_permutation(order, n)) {
        set_error("the processing order is not a permutation of the %zu inputs", n);
        return SYZCOV_EINVAL;
    }
    const size_t o_pcs = align_up((n + 1) * 8, 256), o_ord = o_pcs + align_up((P + 1) * 4, 256),
                 o_mm = o_ord + align_up(n * 4, 256), need = o_mm + 256;
    if (need > dc.stage_cap) {
        if (dc.stage) hipFree(dc.stage);
        dc.stage = nullptr;
        dc.stage_cap = 0;
        if (hipMalloc(&dc.stage, need) != hipSuccess) return 0;  // short of memory: dictionary path
        dc.stage_cap = need;
    }
    uint8_t *st = (uint8_t *)dc.stage;
    uint64_t *d_off = (uint64_t *)st;
    uint32_t *d_pcs = (uint32_t *)(st + o_pcs), *d_mm = (uint32_t *)(st + o_mm);
    int32_t *d_ord = (int32_t *)(st + o_ord);
    SYZ_HIP(hipMemcpyAsync(d_off, hoff.data(), (n + 1) * 8, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(d_pcs, pcs + base, P * 4, hipMemcpyHostToDevice, s));
    if (order) SYZ_HIP(hipMemcpyAsync(d_ord, order, n * 4, hipMemcpyHostToDevice, s));
    int rc = minmax_pcs(d_pcs, P, d_mm, s);
    if (rc) return rc;
    uint32_t mm[2];
    SYZ_HIP(hipMemcpyAsync(mm, d_mm, 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    if (nrange_of((uint64_t)mm[1] - mm[0] + 1, kRangeShiftWindow) > 256) return 0;
    rc = dropin_handle(dc, n, P, max_len, mm[0], mm[1]);
    if (rc <= 0) return rc;
    Corpus &c = *get(dc.h);
    Use u(&c);
    rc = ph_canon(c, d_off, d_pcs, n, s);
    if (!rc) rc = order ? ph_order_given(c, d_ord, n, s) : ph_order(c, nullptr, n, s);
    if (!rc) rc = ph_minimize(c, 1, s);
    if (!rc) rc = ph_finish(c, s);
    syzcov_corpus_res r{};
    if (!rc) rc = ph_result(c, &r, s);
    if (!rc && r.n_kept)
        rc = hipMemcpyAsync(out_idx, r.kept_idx, (size_t)r.n_kept * 4, hipMemcpyDeviceToHost, s) ==
                     hipSuccess
                 ? 0
                 : SYZCOV_EHIP;
    if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = SYZCOV_EHIP;
    return rc ? rc : (int64_t)r.n_kept + 1;  // + 1: 0 means "not taken"
}

int minimize_groups_order(const int32_t *ord_g, const int32_t *perm, const uint64_t *goff_dev,
                          uint32_t ngroups, uint32_t n, int32_t *order_c, uint32_t *rank_grp,
                          hipStream_t s);
static int64_t groups_lds(DropinCache &dc, size_t n, uint64_t P, size_t max_len, uint32_t G,
                          const uint64_t *d_off, uint32_t *d_pcs, const int32_t *d_ordc,
                          const uint64_t *d_goff, uint32_t lo, uint32_t hi, int32_t *out_idx,
                          GroupTimer &tm, hipStream_t s);

// Manager.minimizeCorpus (manager.go:504-524) on the cached engine: the
// corpus is staged as it is; the groups (inputs of one RpcInput.Call, corpus
// order inside, :511-516) exist only in the processing order, which
// concatenates every group's Go sort.Sort order (the segmented restatement,
// gosort.hip) — so the engine canonicalizes once and runs one Minimize per
// group over its rank interval (minimize_range_groups).  Kept corpus indices
// come out grouped by ascending call value, each group in its Minimize order.
int universe_shift_dev(const uint32_t *u, uint32_t n, uint32_t *d_ks, hipStream_t s);
size_t minimize_groups_lds_ws_size(size_t n_items, uint64_t nkeys, uint32_t range_shift);
int minimize_groups_lds(const uint64_t *off, const uint32_t *words, const uint32_t *split,
                        const int32_t *order, size_t n_items, uint64_t nkeys, uint32_t range_shift,
                        const uint64_t *goff_dev, uint32_t ngroups, uint8_t *kept, void *ws,
                        hipStream_t s);
constexpr uint32_t kGroupLdsMaxItems = 1u << 16;  // minimize_range.hip GM_MAX_ITEMS
constexpr uint32_t kGroupLdsShift = 15;           // keys per LDS piece: 2^15 ranks

static int64_t dropin_run_groups(DropinCache &dc, const int32_t *call, const uint64_t *offsets,
                                 const uint32_t *pcs, size_t n, int32_t *out_idx,
                                 GroupTimer &tm, hipStream_t s) {
    const uint64_t base = offsets[0], P = offsets[n] - base;
    std::vector<uint64_t> hoff(n + 1);
    size_t max_len = 1;
    for (size_t i = 0; i <= n; i++) {
        hoff[i] = offsets[i] - base;
        if (i && hoff[i] < hoff[i - 1]) return SYZCOV_EINVAL;
        if (i) max_len = std::max<size_t>(max_len, hoff[i] - hoff[i - 1]);
    }
    // groups: stable by call value (the reference's append order); a counting
    // sort over the calls' value range (sys.CallCount values in practice), a
    // stable comparison sort only for a sparse one
    std::vector<int32_t> perm(n);
    {
        int32_t cmin = INT32_MAX, cmax = INT32_MIN;
        for (size_t i = 0; i < n; i++) {
            cmin = std::min(cmin, call[i]);
            cmax = std::max(cmax, call[i]);
        }
        const uint64_t span = (uint64_t)((int64_t)cmax - cmin) + 1;
        if (span <= std::max<uint64_t>(1u << 16, 4 * (uint64_t)n)) {
            std::vector<uint32_t> cnt(span + 1, 0);
            for (size_t i = 0; i < n; i++) cnt[(uint64_t)((int64_t)call[i] - cmin) + 1]++;
            for (uint64_t v = 0; v < span; v++) cnt[v + 1] += cnt[v];
            for (size_t i = 0; i < n; i++) perm[cnt[(uint64_t)((int64_t)call[i] - cmin)]++] = (int32_t)i;
        } else {
            for (size_t i = 0; i < n; i++) perm[i] = (int32_t)i;
            std::stable_sort(perm.begin(), perm.end(),
                             [&](int32_t a, int32_t b) { return call[a] < call[b]; });
        }
    }
    std::vector<uint64_t> goff;
    std::vector<int64_t> lens(n);
    for (size_t i = 0; i < n; i++) {
        if (i == 0 || call[perm[i]] != call[perm[i - 1]]) goff.push_back(i);
        lens[i] = (int64_t)(hoff[perm[i] + 1] - hoff[perm[i]]);  // len(cov), duplicates included
    }
    goff.push_back(n);
    const uint32_t G = (uint32_t)goff.size() - 1;
    const size_t wseg = syzcov_dev_sort_seg_ws_size(n, G);
    const size_t o_pcs = align_up((n + 1) * 8, 256), o_perm = o_pcs + align_up((P + 1) * 4, 256),
                 o_goff = o_perm + align_up(n * 4, 256), o_lens = o_goff + align_up((G + 1) * 8, 256),
                 o_ordg = o_lens + align_up(n * 8, 256), o_ordc = o_ordg + align_up(n * 4, 256),
                 o_rg = o_ordc + align_up(n * 4, 256), o_mm = o_rg + align_up(n * 4, 256),
                 o_ws = o_mm + 256, need = o_ws + align_up(wseg, 256);
    if (need > dc.stage_cap) {
        if (dc.stage) hipFree(dc.stage);
        dc.stage = nullptr;
        dc.stage_cap = 0;
        if (hipMalloc(&dc.stage, need) != hipSuccess) return 0;
        dc.stage_cap = need;
    }
    uint8_t *st = (uint8_t *)dc.stage;
    uint64_t *d_off = (uint64_t *)st, *d_goff = (uint64_t *)(st + o_goff);
    uint32_t *d_pcs = (uint32_t *)(st + o_pcs), *d_mm = (uint32_t *)(st + o_mm);
    int32_t *d_perm = (int32_t *)(st + o_perm), *d_ordg = (int32_t *)(st + o_ordg),
            *d_ordc = (int32_t *)(st + o_ordc);
    tm.mark(0, s);
    SYZ_HIP(hipMemcpyAsync(d_off, hoff.data(), (n + 1) * 8, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(d_pcs, pcs + base, P * 4, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(d_perm, perm.data(), n * 4, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(d_goff, goff.data(), (G + 1) * 8, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(st + o_lens, lens.data(), n * 8, hipMemcpyHostToDevice, s));
    tm.mark(1, s);
    int rc = minmax_pcs(d_pcs, P, d_mm, s);
    if (rc) return rc;
    uint32_t mm[2];
    SYZ_HIP(hipMemcpyAsync(mm, d_mm, 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    if (nrange_of((uint64_t)mm[1] - mm[0] + 1, kRangeShiftWindow) > 256) return 0;
    rc = syzcov_dev_sort_order_segmented((const int64_t *)(st + o_lens), d_goff, G, n, 0, d_ordg,
                                         st + o_ws, wseg, s);
    if (!rc)
        rc = minimize_groups_order(d_ordg, d_perm, d_goff, G, (uint32_t)n, d_ordc,
                                   (uint32_t *)(st + o_rg), s);
    if (rc) return rc;
    uint64_t gmax = 0;
    for (uint32_t g = 0; g < G; g++) gmax = std::max<uint64_t>(gmax, goff[g + 1] - goff[g]);
    if (gmax <= kGroupLdsMaxItems && !(force_flags() & FORCE_GROUP_CHUNKS)) {
        const int64_t k = groups_lds(dc, n, P, max_len, G, d_off, d_pcs, d_ordc, d_goff, mm[0],
                                     mm[1], out_idx, tm, s);
        if (k != 0) {  // taken (or failed); 0: the per-group engine below
            if (k > 0) tm.finish(SYZCOV_GROUPS_PATH_LDS);
            return k;
        }
        SYZ_HIP(hipMemcpyAsync(d_pcs, pcs + base, P * 4, hipMemcpyHostToDevice, s));
    }
    rc = dropin_handle(dc, n, P, max_len, mm[0], mm[1]);
    if (rc <= 0) return rc;
    Corpus &c = *get(dc.h);
    Use u(&c);
    rc = ph_canon(c, d_off, d_pcs, n, s);
    if (!rc) rc = ph_order_given(c, d_ordc, n, s);
    if (!rc) rc = ph_minimize_groups(c, goff.data(), G, s);
    if (!rc) rc = ph_finish(c, s);
    syzcov_corpus_res r{};
    if (!rc) rc = ph_result(c, &r, s);
    tm.mark(2, s);
    if (!rc && r.n_kept)
        rc = hipMemcpyAsync(out_idx, r.kept_idx, (size_t)r.n_kept * 4, hipMemcpyDeviceToHost, s) ==
                     hipSuccess
                 ? 0
                 : SYZCOV_EHIP;
    tm.mark(3, s);
    if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = SYZCOV_EHIP;
    if (!rc) tm.finish(SYZCOV_GROUPS_PATH_ENGINE);
    return rc ? rc : (int64_t)r.n_kept + 1;
}


// Manager.minimizeCorpus with every group small (<= 2^16 inputs, as a
// corpus of ~10^5-10^6 inputs over a few thousand syscalls has): the corpus
// is staged (d_off, d_pcs raw), grouped and ordered (d_ordc: rank -> input,
// d_goff: the groups' rank intervals).  The union of the corpus (a window-
// mode step on a transient handle, canon out of place) is its own PC
// universe: its kshift makes the keys (pc >> kshift) - kbase collision-free
// on every corpus PC, so key words need no membership check.  The raw lists
// are canonicalized into key words over ranges of 2^15 keys and every (group,
// range) piece takes its first covers in LDS (group_min_kernel): no chunks,
// no records, no per-group launches.  Returns kept + 1 (0: not taken).
static int64_t groups_lds(DropinCache &dc, size_t n, uint64_t P, size_t max_len, uint32_t G,
                          const uint64_t *d_off, uint32_t *d_pcs, const int32_t *d_ordc,
                          const uint64_t *d_goff, uint32_t lo, uint32_t hi, int32_t *out_idx,
                          GroupTimer &tm, hipStream_t s) {
    // the union step runs on the drop-in cache's window-mode engine (no second
    // corpus-sized engine per call), out of place: (2) below canonicalizes the
    // staged raw PCs again, into key words
    int rc = dropin_handle(dc, n, P, max_len, lo, hi, true);
    if (rc <= 0) return rc;
    Corpus &c = *get(dc.h);
    Use u(&c);
    int64_t ret = 0;
    // a HIP error inside the block ends it with rc set (the cleanup below runs)
#define GL_HIP(x)                   \
    if ((x) != hipSuccess) {        \
        rc = SYZCOV_EHIP;           \
        break;                      \
    }
    do {
        // (1) the corpus union: one window-mode Minimize (its own order)
        rc = ph_canon(c, d_off, d_pcs, n, s);
        if (!rc) rc = ph_order(c, nullptr, n, s);
        if (!rc) rc = ph_minimize(c, 1, s);
        if (!rc) rc = ph_finish(c, s);
        syzcov_corpus_res r{};
        if (!rc) rc = ph_result(c, &r, s);
        if (rc) break;
        // the union drops PC 0xFFFFFFFF (cover.go:97); the universe keeps it
        const uint32_t nu = r.n_union + (hi == 0xFFFFFFFFu ? 1u : 0u);
        if (nu == 0) { rc = SYZCOV_EHIP; break; }
        uint32_t *univ = c.buf<uint32_t>(SYZCOV_CORPUS_UNION);  // sized span + 1 >= nu
        if (r.union_pcs != univ) break;  // (no side buffer in window mode: not taken)
        if (hi == 0xFFFFFFFFu) {
            const uint32_t sent = 0xFFFFFFFFu;
            GL_HIP(hipMemcpyAsync(univ + r.n_union, &sent, 4, hipMemcpyHostToDevice, s));
        }
        uint32_t *d_ks = (uint32_t *)(scal(c) + SC_MM);
        if ((rc = universe_shift_dev(univ, nu, d_ks, s))) break;
        uint32_t ks = 0, ends[2];
        GL_HIP(hipMemcpyAsync(&ks, d_ks, 4, hipMemcpyDeviceToHost, s));
        GL_HIP(hipMemcpyAsync(&ends[0], univ, 4, hipMemcpyDeviceToHost, s));
        GL_HIP(hipMemcpyAsync(&ends[1], univ + nu - 1, 4, hipMemcpyDeviceToHost, s));
        GL_HIP(hipStreamSynchronize(s));
        ks = std::min<uint32_t>(ks, SYZCOV_KSHIFT_MAX);
        const uint32_t kbase = ends[0] >> ks;
        const uint64_t nkeys = (uint64_t)(ends[1] >> ks) - kbase + 1;
        if (nkeys > (1ull << 25)) break;  // key words: keys < 2^25
        // (2) key words over ranges of 2^15 keys (out of place: CANON)
        const uint64_t R = (nkeys + (1ull << kGroupLdsShift) - 1) >> kGroupLdsShift;
        if (R > 256) break;  // minimize_range.hip MAX_R: not taken
        const size_t o_nl = 0, o_split = align_up((n + 1) * 4, 256),
                     o_rt = o_split + align_up(n * R * 4, 256), o_err = o_rt + align_up(R * 8, 256),
                     o_kept = o_err + 256, o_out = o_kept + align_up(n, 256),
                     o_cnt = o_out + align_up(n * 4, 256), o_ws = o_cnt + 256,
                     ws_sz = std::max({syzcov_dev_canon_split_ws_size(n),
                                       minimize_groups_lds_ws_size(n, nkeys, kGroupLdsShift),
                                       syzcov_dev_compact_ws_size(n)}),
                     need = o_ws + align_up(ws_sz, 256);
        if (need > dc.gscratch_cap) {  // grow-only, kept in the drop-in cache
            if (dc.gscratch) hipFree(dc.gscratch);
            dc.gscratch = nullptr;
            dc.gscratch_cap = 0;
            if (hipMalloc(&dc.gscratch, need) != hipSuccess) {
                dc.gscratch = nullptr;
                break;  // short of memory: not taken
            }
            dc.gscratch_cap = need;
        }
        uint8_t *sc8 = (uint8_t *)dc.gscratch;
        uint32_t *nl = (uint32_t *)(sc8 + o_nl), *split = (uint32_t *)(sc8 + o_split);
        uint32_t *err = (uint32_t *)(sc8 + o_err);
        uint8_t *kept = sc8 + o_kept;
        int32_t *d_out = (int32_t *)(sc8 + o_out);
        uint32_t *d_cnt = (uint32_t *)(sc8 + o_cnt);
        GL_HIP(hipMemsetAsync(sc8 + o_rt, 0, R * 8 + 256, s));  // range totals, err
        uint32_t *words = c.buf<uint32_t>(SYZCOV_CORPUS_CANON);  // key words, out of place
        rc = syzcov_dev_canon_split_keys(d_off, d_pcs, words, nl, n, max_len, ends[0],
                                         (uint64_t)ends[1] - ends[0] + 1, ks, kbase, nkeys,
                                         kGroupLdsShift, split, (uint64_t *)(sc8 + o_rt), err,
                                         sc8 + o_ws, ws_sz, s);
        // (3) first covers per (group, range) in LDS; kept by rank
        if (!rc)
            rc = minimize_groups_lds(d_off, words, split, d_ordc, n, nkeys, kGroupLdsShift, d_goff,
                                     G, kept, sc8 + o_ws, s);
        if (!rc) rc = syzcov_dev_compact_kept(kept, d_ordc, n, d_out, d_cnt, sc8 + o_ws, s);
        if (rc) break;
        uint32_t hk[2];
        GL_HIP(hipMemcpyAsync(&hk[0], d_cnt, 4, hipMemcpyDeviceToHost, s));
        GL_HIP(hipMemcpyAsync(&hk[1], err, 4, hipMemcpyDeviceToHost, s));
        GL_HIP(hipStreamSynchronize(s));
        if (hk[1]) {  // every corpus PC is in its own union: cannot happen
            set_error("grouped minimize: canonicalize flags %#x", hk[1]);
            rc = SYZCOV_EHIP;
            break;
        }
        tm.mark(2, s);
        if (hk[0]) GL_HIP(hipMemcpyAsync(out_idx, d_out, (size_t)hk[0] * 4, hipMemcpyDeviceToHost, s));
        tm.mark(3, s);
        GL_HIP(hipStreamSynchronize(s));
        ret = (int64_t)hk[0] + 1;
    } while (0);
#undef GL_HIP
    hipStreamSynchronize(s);
    return rc ? rc : ret;
}

int minimize_corpus_via_engine(const int32_t *call, const uint64_t *offsets, const uint32_t *pcs,
                               size_t n, int32_t *out_idx, int64_t *out_n) {
    if (offsets[n] == offsets[0]) return 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return 0;
    DropinCache &dc = g_dropin[dev];
    std::unique_lock<std::mutex> lk(dc.mu, std::try_to_lock);
    if (!lk.owns_lock()) return 0;
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return SYZCOV_EHIP;
    int64_t k;
    {
        GroupTimer tm;
        k = dropin_run_groups(dc, call, offsets, pcs, n, out_idx, tm, s);
    }
    hipStreamDestroy(s);
    if (k <= 0) return (int)k;
    *out_n = k - 1;
    return 1;
}

// the slab path's record (api.cc), and the query
void groups_stats_slabs() {
    g_gstats = {};
    g_gstats.path = SYZCOV_GROUPS_PATH_SLABS;
}
void groups_stats_reset() { g_gstats = {}; }
int groups_stats(syzcov_groups_stats *out) {
    if (!out) return SYZCOV_EINVAL;
    *out = g_gstats;
    return 0;
}

int minimize_via_engine(const uint64_t *offsets, const uint32_t *pcs, size_t n,
                        const int32_t *order, int32_t *out_idx, int64_t *out_n) {
    if (offsets[n] == offsets[0]) return 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return 0;
    DropinCache &dc = g_dropin[dev];
    std::unique_lock<std::mutex> lk(dc.mu, std::try_to_lock);
    if (!lk.owns_lock()) return 0;  // another caller holds the cached engine
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return SYZCOV_EHIP;
    const int64_t k = dropin_run(dc, offsets, pcs, n, order, out_idx, s);
    hipStreamDestroy(s);
    if (k <= 0) return (int)k;
    *out_n = k - 1;
    return 1;
}
}  // namespace syz
