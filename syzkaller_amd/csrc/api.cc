// api.cc — drop-in host API of libsyzcov (include/syzcov.h tier 1).
//
// Each host thread owns a HIP stream and a grow-only device arena, so calls
// are reentrant (the fuzzer's goroutines call cover ops concurrently under
// coverMu.RLock: syz-fuzzer/fuzzer.go:383-386,458-478).  Every call stages its
// host operands into the arena, runs the device kernels and copies the result
// back; there is no host compute path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <memory>
#include <mutex>
#include <new>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/syzcov.h"
#include "force.h"

namespace syz {

static thread_local char g_err[512];

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}

// The library's one run-time override (tests of the exact fallbacks and of
// both candidate passes; every tuning choice is a compile-time default):
// SYZCOV_FORCE, a comma-separated list of "canon3" (key mode canonicalizes
// with the 3-pass window-offset sort instead of the 2-pass key sort), "redo"
// (every wave-canonicalized segment takes the order-check-failure path, the
// workgroup sort of canon.hip), "nc_lds" / "nc_probe" (newcov's LDS-staged or
// global-probe candidate pass instead of the one the batch's shape picks).
// Read at every call, so a test can set and clear it.
uint32_t force_flags() {
    const char *e = getenv("SYZCOV_FORCE");
    if (!e || !*e) return 0;
    uint32_t f = 0;
    if (strstr(e, "canon3")) f |= FORCE_CANON3;
    if (strstr(e, "redo")) f |= FORCE_REDO;
    if (strstr(e, "nc_lds")) f |= FORCE_NC_LDS;
    if (strstr(e, "nc_probe")) f |= FORCE_NC_PROBE;
    if (strstr(e, "group_chunks")) f |= FORCE_GROUP_CHUNKS;
    if (strstr(e, "nc_sep")) f |= FORCE_NC_SEP;
    if (strstr(e, "mr_bytes")) f |= FORCE_MR_BYTES;
    if (strstr(e, "nc_hash64")) f |= FORCE_NC_HASH64;
    if (strstr(e, "min_atomics")) f |= FORCE_MIN_ATOMICS;
    if (strstr(e, "no_init_block")) f |= FORCE_NO_INIT_BLOCK;
    if (strstr(e, "small_init")) f |= FORCE_SMALL_INIT;
    return f;
}

size_t setop_ws_size(size_t ntot);
int dev_setop(int op, const uint32_t *a, size_t na, const uint32_t *b, size_t nb, uint32_t *out,
              uint32_t *n_out, uint32_t *err, void *ws, hipStream_t s);

static inline size_t al(size_t x) { return (x + 255) / 256 * 256; }

// A grow-only device arena.  Growth frees the old block after the stream has
// drained; a block larger than kKeepBytes is released at the end of the call
// that needed it (corpus-level calls), so an idle thread pins at most that.
struct Arena {
    void *p = nullptr;
    size_t cap = 0;
};
constexpr size_t kKeepBytes = 32ull << 20;

// A device context: a stream and three arenas (staged corpus, its
// dictionary, the call's work buffers).  Contexts live in a process-wide pool
// per device: a call leases one for its duration and returns it, so the
// number of contexts is the peak number of CONCURRENT callers (the fuzzer's
// <= 32 goroutines), not the number of OS threads that ever called in (cgo
// moves goroutines across many threads, and thread-exit destructors cannot be
// relied on to run before the HIP runtime is torn down).
struct Ctx {
    int dev = -1;
    hipStream_t s = nullptr;
    Arena a[3];
};
enum { A_STAGE = 0, A_DICT = 1, A_WORK = 2 };

static int device_count() {
    static std::once_flag once;
    static int n = 0;
    std::call_once(once, [] {
        if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    });
    return n;
}

struct CtxPool {
    std::mutex mu;
    std::vector<Ctx *> idle[16];
    size_t created[16] = {};
};
static CtxPool &pool() {
    static CtxPool *p = new CtxPool();  // never destroyed: outlives every caller
    return *p;
}

// RAII lease of the current device's context; get() == nullptr + error if none.
class CtxLease {
  public:
    CtxLease() {
        if (device_count() == 0) {
            set_error("no HIP device (libsyzcov has no CPU path)");
            return;
        }
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return;
        CtxPool &P = pool();
        {
            std::lock_guard<std::mutex> g(P.mu);
            if (!P.idle[dev].empty()) {
                c_ = P.idle[dev].back();
                P.idle[dev].pop_back();
                return;
            }
        }
        Ctx *n = new (std::nothrow) Ctx();
        if (!n) return;
        n->dev = dev;
        if (hipStreamCreateWithFlags(&n->s, hipStreamNonBlocking) != hipSuccess) {
            set_error("hipStreamCreate failed");
            delete n;
            return;
        }
        std::lock_guard<std::mutex> g(P.mu);
        P.created[dev]++;
        c_ = n;
    }
    ~CtxLease() {
        if (!c_) return;
        hipStreamSynchronize(c_->s);
        CtxPool &P = pool();
        std::lock_guard<std::mutex> g(P.mu);
        P.idle[c_->dev].push_back(c_);
    }
    Ctx *get() const { return c_; }
    CtxLease(const CtxLease &) = delete;
    CtxLease &operator=(const CtxLease &) = delete;

  private:
    Ctx *c_ = nullptr;
};

// Bump allocator over an arena: plan sizes first, then reserve once.
struct Plan {
    std::vector<size_t> sizes;
    size_t add(size_t bytes) {
        sizes.push_back(al(bytes ? bytes : 1));
        return sizes.size() - 1;
    }
    size_t total() const {
        size_t t = 0;
        for (size_t s : sizes) t += s;
        return t;
    }
};

static int reserve(Ctx *c, int which, const Plan &p, std::vector<uint8_t *> &ptrs) {
    Arena &A = c->a[which];
    const size_t need = p.total();
    if (need > A.cap) {
        if (A.p) {
            hipStreamSynchronize(c->s);
            hipFree(A.p);
        }
        A.p = nullptr;
        A.cap = 0;
        size_t cap = need + need / 4;
        if (hipMalloc(&A.p, cap) != hipSuccess) {
            set_error("hipMalloc(%zu) failed", cap);
            return SYZCOV_ENOMEM;
        }
        A.cap = cap;
    }
    ptrs.clear();
    uint8_t *b = (uint8_t *)A.p;
    for (size_t s : p.sizes) {
        ptrs.push_back(b);
        b += s;
    }
    return 0;
}
static int reserve(Ctx *c, const Plan &p, std::vector<uint8_t *> &ptrs) {
    return reserve(c, A_WORK, p, ptrs);
}

// End of a corpus-level call: drain, and give back arenas above kKeepBytes.
static void release_large(Ctx *c) {
    hipStreamSynchronize(c->s);
    for (Arena &x : c->a)
        if (x.cap > kKeepBytes) {
            hipFree(x.p);
            x.p = nullptr;
            x.cap = 0;
        }
}

#define CK(expr)                                                                         \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess) {                                                          \
            set_error("%s:%d %s: %s", __FILE__, __LINE__, #expr, hipGetErrorString(e_)); \
            return SYZCOV_EHIP;                                                          \
        }                                                                                \
    } while (0)
#define RC(expr)                  \
    do {                          \
        int r_ = (expr);          \
        if (r_ < 0) return r_;    \
    } while (0)

}  // namespace syz

using namespace syz;
namespace syz {
void dropin_trim();
}

extern "C" {

const char *syzcov_version(void) { return "syzcov 0.2 gfx950"; }

int syzcov_pool_trim(void) {
    dropin_trim();  // the cached cover.Minimize engine (corpus.hip)
    CtxPool &P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    int cur = 0;
    hipGetDevice(&cur);
    // idle contexts are destroyed whole: arenas AND streams (each HIP stream
    // pins runtime memory of its own, ~25 MB measured); leased ones are untouched
    for (int d = 0; d < 16; d++) {
        for (Ctx *c : P.idle[d]) {
            hipSetDevice(d);
            hipStreamSynchronize(c->s);
            for (Arena &x : c->a)
                if (x.p) hipFree(x.p);
            hipStreamDestroy(c->s);
            delete c;
        }
        P.created[d] -= P.idle[d].size();
        P.idle[d].clear();
    }
    hipSetDevice(cur);
    return 0;
}

int64_t syzcov_pool_contexts(int device) {
    if (device < 0 || device >= 16) return SYZCOV_EINVAL;
    CtxPool &P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    return (int64_t)P.created[device];
}
const char *syzcov_last_error(void) { return g_err; }

uint64_t syzcov_restore_pc(uint32_t pc, uint32_t base) {
    return ((uint64_t)base << 32) + (uint64_t)pc;  // cover.go:23-25
}

int64_t syzcov_canonicalize(uint32_t *cov, size_t n) {
    if (n == 0) return 0;
    if (!cov) return SYZCOV_EINVAL;
    CtxLease lease;
    Ctx *c = lease.get();
    if (!c) return SYZCOV_ENODEV;
    Plan p;
    size_t i_off = p.add(2 * 8), i_pcs = p.add(n * 4), i_len = p.add(4),
           i_ws = p.add(syzcov_dev_canon_ws_size(1, n));
    std::vector<uint8_t *> b;
    RC(reserve(c, p, b));
    uint64_t hoff[2] = {0, n};
    CK(hipMemcpyAsync(b[i_off], hoff, 16, hipMemcpyHostToDevice, c->s));
    CK(hipMemcpyAsync(b[i_pcs], cov, n * 4, hipMemcpyHostToDevice, c->s));
    RC(syzcov_dev_canonicalize((uint64_t *)b[i_off], (uint32_t *)b[i_pcs], (uint32_t *)b[i_pcs],
                               (uint32_t *)b[i_len], 1, n, nullptr, 0, 0, nullptr, b[i_ws],
                               p.sizes[i_ws], c->s));
    uint32_t nl = 0;
    CK(hipMemcpyAsync(&nl, b[i_len], 4, hipMemcpyDeviceToHost, c->s));
    CK(hipStreamSynchronize(c->s));
    if (nl) {
        CK(hipMemcpyAsync(cov, b[i_pcs], (size_t)nl * 4, hipMemcpyDeviceToHost, c->s));
        CK(hipStreamSynchronize(c->s));
    }
    return nl;
}

int64_t syzcov_cover_dedup64(uint64_t *cov, size_t n) {
    if (n == 0) return 0;
    if (!cov) return SYZCOV_EINVAL;
    if (n > ((size_t)1 << 31)) return SYZCOV_ETOOLONG;
    CtxLease lease;
    Ctx *c = lease.get();
    if (!c) return SYZCOV_ENODEV;
    Plan p;
    size_t i_off = p.add(2 * 8), i_pcs = p.add(n * 8), i_len = p.add(4);
    std::vector<uint8_t *> b;
    RC(reserve(c, p, b));
    uint64_t hoff[2] = {0, n};
    CK(hipMemcpyAsync(b[i_off], hoff, 16, hipMemcpyHostToDevice, c->s));
    CK(hipMemcpyAsync(b[i_pcs], cov, n * 8, hipMemcpyHostToDevice, c->s));
    RC(syzcov_dev_cover_dedup64((uint64_t *)b[i_pcs], (uint64_t *)b[i_off], 1,
                                (uint32_t *)b[i_len], nullptr, c->s));
    uint32_t nl = 0;
    CK(hipMemcpyAsync(&nl, b[i_len], 4, hipMemcpyDeviceToHost, c->s));
    CK(hipStreamSynchronize(c->s));
    if (nl) {
        CK(hipMemcpyAsync(cov, b[i_pcs], (size_t)nl * 8, hipMemcpyDeviceToHost, c->s));
        CK(hipStreamSynchronize(c->s));
    }
    return nl;
}

static int64_t setop(int op, const uint32_t *a, size_t na, const uint32_t *b_, size_t nb,
                     uint32_t *out) {
    if ((na && !a) || (nb && !b_) || !out) return SYZCOV_EINVAL;
    if (na + nb == 0) return 0;
    CtxLease lease;
    Ctx *c = lease.get();
    if (!c) return SYZCOV_ENODEV;
    Plan p;
    size_t i_a = p.add(na * 4), i_b = p.add(nb * 4), i_o = p.add((na + nb) * 4), i_n = p.add(8),
           i_ws = p.add(setop_ws_size(na + nb));
    std::vector<uint8_t *> b;
    RC(reserve(c, p, b));
    uint32_t *dn = (uint32_t *)b[i_n], *derr = dn + 1;
    CK(hipMemsetAsync(dn, 0, 8, c->s));
    if (na) CK(hipMemcpyAsync(b[i_a], a, na * 4, hipMemcpyHostToDevice, c->s));
    if (nb) CK(hipMemcpyAsync(b[i_b], b_, nb * 4, hipMemcpyHostToDevice, c->s));
    RC(dev_setop(op, (uint32_t *)b[i_a], na, (uint32_t *)b[i_b], nb, (uint32_t *)b[i_o], dn, derr,
                 b[i_ws], c->s));
    uint32_t h[2];
    CK(hipMemcpyAsync(h, dn, 8, hipMemcpyDeviceToHost, c->s));
    CK(hipStreamSynchronize(c->s));
    if (h[1]) {
        set_error("set-op operand is not sorted");
        return SYZCOV_ENOTSORTED;
    }
    if (h[0]) {
        CK(hipMemcpyAsync(out, b[i_o], (size_t)h[0] * 4, hipMemcpyDeviceToHost, c->s));
        CK(hipStreamSynchronize(c->s));
    }
    return h[0];
}

int64_t syzcov_difference(const uint32_t *a, size_t na, const uint32_t *b, size_t nb,
                          uint32_t *out) {
    return setop(0, a, na, b, nb, out);
}
int64_t syzcov_symmetric_difference(const uint32_t *a, size_t na, const uint32_t *b, size_t nb,
                                    uint32_t *out) {
    return setop(1, a, na, b, nb, out);
}
int64_t syzcov_union(const uint32_t *a, size_t na, const uint32_t *b, size_t nb, uint32_t *out) {
    return setop(2, a, na, b, nb, out);
}
int64_t syzcov_intersection(const uint32_t *a, size_t na, const uint32_t *b, size_t nb,
                            uint32_t *out) {
    return setop(3, a, na, b, nb, out);
}

}  // extern "C"

// ------------------------------------------------------------------ corpus
namespace syz {
// cover.Minimize calls with at least this many inputs run on the corpus
// engine (corpus.hip); smaller ones on the dictionary path below
constexpr size_t kEngineMinInputs = 1024;
int minimize_via_engine(const uint64_t *offsets, const uint32_t *pcs, size_t n,
                        const int32_t *order, int32_t *out_idx, int64_t *out_n);
// Manager.minimizeCorpus with at least this many inputs runs on the corpus
// engine (per-group Minimize over one rank space, corpus.hip); below it the
// per-group launches cost more than the dictionary path's batched slabs
constexpr size_t kGroupEngineMinInputs = 65536;
void groups_stats_slabs();
void groups_stats_reset();
int groups_stats(syzcov_groups_stats *out);
int minimize_corpus_via_engine(const int32_t *call, const uint64_t *offsets, const uint32_t *pcs,
                               size_t n, int32_t *out_idx, int64_t *out_n);
int minmax_pcs(const uint32_t *pcs, size_t n, uint32_t *out2, hipStream_t s);
int ui_stats_launch(const uint64_t *off, const uint32_t *pcs, uint32_t n, const int32_t *call,
                    uint32_t ncalls, const uint64_t *tab, uint32_t pc_lo, uint32_t nids,
                    uint32_t sent_id, uint32_t *cnt_all, int32_t *own_all, uint32_t *cnt_call,
                    int32_t *own_call, uint8_t *flag_all, uint32_t *slab, uint64_t slab_words,
                    uint32_t *cover, uint32_t *ucov, uint32_t *in_unique, hipStream_t s);
int unique_cover_launch(const uint64_t *off, const uint32_t *pcs, uint32_t n, const int32_t *call,
                        const uint64_t *tab, uint64_t span, uint32_t pc_lo, uint32_t nids,
                        uint32_t *cnt, int32_t *owner, uint8_t *flag, int32_t *pc_of,
                        hipStream_t s);
int minimize_groups_order(const int32_t *ord_g, const int32_t *perm, const uint64_t *goff_dev,
                          uint32_t ngroups, uint32_t n, int32_t *order_c, uint32_t *rank_grp,
                          hipStream_t s);
int minimize_groups_batch(const uint64_t *off, const uint32_t *pcs, const int32_t *order_c,
                          const uint32_t *rank_grp, uint32_t r0, uint32_t r1, uint32_t g0,
                          uint32_t nids, const uint64_t *tab, uint32_t pc_lo, int32_t *first,
                          size_t first_n, uint8_t *cand, uint8_t *kept, hipStream_t s);

// Stage a CSR corpus and build its dense dictionary.  Fills device pointers.
struct CorpusDev {
    uint64_t *off;
    uint32_t *pcs;
    uint8_t *pres;
    uint64_t *tab;
    uint32_t pc_lo;
    uint64_t span;
    uint32_t n_ids;
};

static int stage_corpus(Ctx *c, const uint64_t *offsets, const uint32_t *pcs, size_t n,
                        CorpusDev &cd) {
    const uint64_t base = offsets[0];
    const uint64_t P = offsets[n] - base;
    std::vector<uint64_t> hoff(n + 1);
    for (size_t i = 0; i <= n; i++) hoff[i] = offsets[i] - base;
    Plan p0;
    const size_t i_off = p0.add((n + 1) * 8), i_pcs = p0.add(P * 4 + 4), i_mm = p0.add(256);
    std::vector<uint8_t *> b0;
    RC(reserve(c, A_STAGE, p0, b0));
    CK(hipMemcpyAsync(b0[i_off], hoff.data(), (n + 1) * 8, hipMemcpyHostToDevice, c->s));
    if (P) CK(hipMemcpyAsync(b0[i_pcs], pcs + base, P * 4, hipMemcpyHostToDevice, c->s));
    cd.off = (uint64_t *)b0[i_off];
    cd.pcs = (uint32_t *)b0[i_pcs];
    // PC window from a device min/max reduction
    uint32_t *d_mm = (uint32_t *)b0[i_mm];
    uint32_t mm[2] = {0, 0};
    if (P) {
        RC(minmax_pcs(cd.pcs, P, d_mm, c->s));
        CK(hipMemcpyAsync(mm, d_mm, 8, hipMemcpyDeviceToHost, c->s));
        CK(hipStreamSynchronize(c->s));
    }
    cd.pc_lo = mm[0];
    cd.span = (uint64_t)mm[1] - mm[0] + 1;
    const uint64_t nwords = (cd.span + 31) / 32;
    Plan p1;
    const size_t i_pres = p1.add(al(cd.span)), i_tab = p1.add(nwords * 8),
                 i_ws = p1.add(syzcov_dev_dict_ws_size(cd.span) + 256);
    std::vector<uint8_t *> b1;
    RC(reserve(c, A_DICT, p1, b1));
    cd.pres = b1[i_pres];
    cd.tab = (uint64_t *)b1[i_tab];
    uint32_t *d_err = d_mm + 4, *d_nids = d_mm + 8;
    CK(hipMemsetAsync(cd.pres, 0, al(cd.span), c->s));
    CK(hipMemsetAsync(d_err, 0, 4, c->s));
    RC(syzcov_dev_mark(cd.off, nullptr, cd.pcs, n, cd.pres, cd.pc_lo, cd.span, d_err, c->s));
    RC(syzcov_dev_dict_build(cd.pres, cd.span, cd.tab, d_nids, b1[i_ws], c->s));
    uint32_t h[2];
    CK(hipMemcpyAsync(h, d_err, 4, hipMemcpyDeviceToHost, c->s));
    CK(hipMemcpyAsync(h + 1, d_nids, 4, hipMemcpyDeviceToHost, c->s));
    CK(hipStreamSynchronize(c->s));
    if (h[0]) {
        set_error("internal: PC outside its own min/max window");
        return SYZCOV_EHIP;
    }
    cd.n_ids = h[1];
    return 0;
}
}  // namespace syz

extern "C" {

int syzcov_sort_order(const int64_t *lens, size_t n, int sort_variant, int32_t *order) {
    if (n == 0) return 0;
    if (!lens || !order) return SYZCOV_EINVAL;
    CtxLease lease;
    Ctx *c = lease.get();
    if (!c) return SYZCOV_ENODEV;
    Plan p;
    size_t i_l = p.add(n * 8), i_o = p.add(n * 4), i_ws = p.add(syzcov_dev_sort_ws_size(n));
    std::vector<uint8_t *> b;
    RC(reserve(c, p, b));
    CK(hipMemcpyAsync(b[i_l], lens, n * 8, hipMemcpyHostToDevice, c->s));
    RC(syzcov_dev_sort_order((int64_t *)b[i_l], n, sort_variant, (int32_t *)b[i_o], b[i_ws],
                             p.sizes[i_ws], c->s));
    CK(hipMemcpyAsync(order, b[i_o], n * 4, hipMemcpyDeviceToHost, c->s));
    CK(hipStreamSynchronize(c->s));
    return 0;
}

int64_t syzcov_minimize(const uint64_t *offsets, const uint32_t *pcs, size_t n,
                        const int32_t *order, int sort_variant, int32_t *out_idx) {
    if (n == 0) return 0;
    if (!offsets || !out_idx || n > 0x7FFFFFFF) return SYZCOV_EINVAL;
    if (offsets[n] > offsets[0] && !pcs) return SYZCOV_EINVAL;
    // corpus-sized calls take the benchmarked engine (corpus.hip: a cached
    // window-mode handle over the corpus' own PC extent; the caller's order,
    // or the restated sort over the raw lengths Go sorts on)
    if ((order || sort_variant == 0) && n >= kEngineMinInputs && device_count() > 0) {
        int64_t k = 0;
        const int rc = minimize_via_engine(offsets, pcs, n, order, out_idx, &k);
        if (rc < 0) return rc;
        if (rc == 1) return k;
    }
    CtxLease lease;
    Ctx *c = lease.get();
    if (!c) return SYZCOV_ENODEV;
    CorpusDev cd;
    int rc = stage_corpus(c, offsets, pcs, n, cd);
    if (rc) {
        release_large(c);
        return rc;
    }
    Plan p;
    size_t i_ord = p.add(n * 4), i_len = p.add(n * 8), i_first = p.add((size_t)cd.n_ids * 4 + 4),
           i_cand = p.add(n), i_kept = p.add(n), i_out = p.add(n * 4), i_cnt = p.add(4),
           i_ws = p.add(std::max(syzcov_dev_compact_ws_size(n), syzcov_dev_sort_ws_size(n)));
    std::vector<uint8_t *> b;
    rc = reserve(c, p, b);
    if (rc) {
        release_large(c);
        return rc;
    }
    int32_t *d_ord = (int32_t *)b[i_ord];
    do {
        if (order) {
            for (size_t i = 0; i < n; i++)
                if (order[i] < 0 || (size_t)order[i] >= n) {
                    rc = SYZCOV_EINVAL;
                    break;
                }
            if (rc) break;
            if (hipMemcpyAsync(d_ord, order, n * 4, hipMemcpyHostToDevice, c->s) != hipSuccess) {
                rc = SYZCOV_EHIP;
                break;
            }
        } else {
            std::vector<int64_t> lens(n);
            for (size_t i = 0; i < n; i++) lens[i] = (int64_t)(offsets[i + 1] - offsets[i]);
            if (hipMemcpyAsync(b[i_len], lens.data(), n * 8, hipMemcpyHostToDevice, c->s) !=
                hipSuccess) {
                rc = SYZCOV_EHIP;
                break;
            }
            rc = syzcov_dev_sort_order((int64_t *)b[i_len], n, sort_variant, d_ord, b[i_ws],
                                       p.sizes[i_ws], c->s);
            if (rc) break;
        }
        hipMemsetD32Async((hipDeviceptr_t)b[i_first], 0x7FFFFFFF, cd.n_ids + 1, c->s);
        hipMemsetAsync(b[i_kept], 0, n, c->s);
        rc = syzcov_dev_minimize_pass1(cd.off, nullptr, cd.pcs, d_ord, nullptr, n, cd.tab, cd.pc_lo,
                                       (int32_t *)b[i_first], b[i_cand], c->s);
        if (rc) break;
        rc = syzcov_dev_minimize_pass2(cd.off, nullptr, cd.pcs, d_ord, nullptr, n, cd.tab, cd.pc_lo,
                                       (int32_t *)b[i_first], b[i_cand], b[i_kept], c->s);
        if (rc) break;
        rc = syzcov_dev_compact_kept(b[i_kept], d_ord, n, (int32_t *)b[i_out], (uint32_t *)b[i_cnt],
                                     b[i_ws], c->s);
        if (rc) break;
        uint32_t k = 0;
        if (hipMemcpyAsync(&k, b[i_cnt], 4, hipMemcpyDeviceToHost, c->s) != hipSuccess ||
            hipStreamSynchronize(c->s) != hipSuccess) {
            rc = SYZCOV_EHIP;
            break;
        }
        if (k && (hipMemcpyAsync(out_idx, b[i_out], (size_t)k * 4, hipMemcpyDeviceToHost, c->s) !=
                      hipSuccess ||
                  hipStreamSynchronize(c->s) != hipSuccess)) {
            rc = SYZCOV_EHIP;
            break;
        }
        rc = (int)k;
    } while (0);
    hipStreamSynchronize(c->s);
    release_large(c);
    return rc;
}

// Manager.minimizeCorpus (syz-manager/manager.go:504-524): group the corpus by
// call (corpus order inside a group, :511-516), cover.Minimize each group
// (:519-523).  The kept corpus indices come out grouped by ascending call
// value; the reference walks its groups in Go map order, which is random, so
// every group order is one the reference can produce.
static int64_t minimize_corpus_impl(Ctx *c, const int32_t *call, const uint64_t *offsets,
                                    const uint32_t *pcs, size_t n, int sort_variant,
                                    int32_t *out_idx) {
    // host grouping: stable by call value (the reference's append order)
    std::vector<int32_t> perm(n);
    for (size_t i = 0; i < n; i++) perm[i] = (int32_t)i;
    std::stable_sort(perm.begin(), perm.end(),
                     [&](int32_t a, int32_t b) { return call[a] < call[b]; });
    std::vector<uint64_t> goff;
    std::vector<int64_t> lens(n);
    for (size_t i = 0; i < n; i++) {
        if (i == 0 || call[perm[i]] != call[perm[i - 1]]) goff.push_back(i);
        lens[i] = (int64_t)(offsets[perm[i] + 1] - offsets[perm[i]]);
        if (lens[i] >= 0xFFFFFFFFll) return SYZCOV_ERANGE;
    }
    goff.push_back(n);
    const size_t G = goff.size() - 1;
    CorpusDev cd;
    RC(stage_corpus(c, offsets, pcs, n, cd));
    const uint32_t nids = std::max<uint32_t>(cd.n_ids, 1);
    // first-cover slabs for as many groups as fit 1 GiB (at least one)
    const size_t per = (size_t)nids * 4;
    size_t gb = std::max<size_t>(1, std::min<size_t>(G, (1ull << 30) / per));
    Plan p;
    size_t i_len = p.add(n * 8), i_goff = p.add((G + 1) * 8), i_perm = p.add(n * 4),
           i_ordg = p.add(n * 4), i_ordc = p.add(n * 4), i_rg = p.add(n * 4),
           i_first = p.add(gb * per), i_cand = p.add(n), i_kept = p.add(n), i_out = p.add(n * 4),
           i_cnt = p.add(4),
           i_ws = p.add(std::max(syzcov_dev_compact_ws_size(n), syzcov_dev_sort_seg_ws_size(n, G)));
    std::vector<uint8_t *> b;
    RC(reserve(c, p, b));
    CK(hipMemcpyAsync(b[i_len], lens.data(), n * 8, hipMemcpyHostToDevice, c->s));
    CK(hipMemcpyAsync(b[i_goff], goff.data(), (G + 1) * 8, hipMemcpyHostToDevice, c->s));
    CK(hipMemcpyAsync(b[i_perm], perm.data(), n * 4, hipMemcpyHostToDevice, c->s));
    RC(syzcov_dev_sort_order_segmented((int64_t *)b[i_len], (uint64_t *)b[i_goff], G, n,
                                       sort_variant, (int32_t *)b[i_ordg], b[i_ws], p.sizes[i_ws],
                                       c->s));
    RC(minimize_groups_order((int32_t *)b[i_ordg], (int32_t *)b[i_perm], (uint64_t *)b[i_goff],
                             (uint32_t)G, (uint32_t)n, (int32_t *)b[i_ordc], (uint32_t *)b[i_rg],
                             c->s));
    CK(hipMemsetAsync(b[i_kept], 0, n, c->s));
    for (size_t g0 = 0; g0 < G; g0 += gb) {
        const size_t g1 = std::min(G, g0 + gb);
        RC(minimize_groups_batch(cd.off, cd.pcs, (int32_t *)b[i_ordc], (uint32_t *)b[i_rg],
                                 (uint32_t)goff[g0], (uint32_t)goff[g1], (uint32_t)g0, nids, cd.tab,
                                 cd.pc_lo, (int32_t *)b[i_first], (g1 - g0) * nids, b[i_cand],
                                 b[i_kept], c->s));
    }
    RC(syzcov_dev_compact_kept(b[i_kept], (int32_t *)b[i_ordc], n, (int32_t *)b[i_out],
                               (uint32_t *)b[i_cnt], b[i_ws], c->s));
    uint32_t k = 0;
    CK(hipMemcpyAsync(&k, b[i_cnt], 4, hipMemcpyDeviceToHost, c->s));
    CK(hipStreamSynchronize(c->s));
    if (k) {
        CK(hipMemcpyAsync(out_idx, b[i_out], (size_t)k * 4, hipMemcpyDeviceToHost, c->s));
        CK(hipStreamSynchronize(c->s));
    }
    return (int64_t)k;
}

int64_t syzcov_minimize_corpus(const int32_t *call, const uint64_t *offsets, const uint32_t *pcs,
                               size_t n, int sort_variant, int32_t *out_idx) {
    groups_stats_reset();
    if (n == 0) return 0;
    if (!call || !offsets || !out_idx || n > 0x7FFFFFFF || sort_variant != 0)
        return SYZCOV_EINVAL;
    if (offsets[n] > offsets[0] && !pcs) return SYZCOV_EINVAL;
    if (n >= kGroupEngineMinInputs && device_count() > 0) {
        int64_t k = 0;
        const int rc = minimize_corpus_via_engine(call, offsets, pcs, n, out_idx, &k);
        if (rc < 0) return rc;
        if (rc == 1) return k;
    }
    CtxLease lease;
    Ctx *c = lease.get();
    if (!c) return SYZCOV_ENODEV;
    const int64_t rc = minimize_corpus_impl(c, call, offsets, pcs, n, sort_variant, out_idx);
    hipStreamSynchronize(c->s);
    release_large(c);
    if (rc >= 0) groups_stats_slabs();
    return rc;
}

int syzcov_minimize_corpus_stats(syzcov_groups_stats *out) { return groups_stats(out); }

// Manager.uniqueCover (syz-manager/html.go:213-238).
static int64_t unique_cover_impl(Ctx *c, const int32_t *call, const uint64_t *offsets,
                                 const uint32_t *pcs, size_t n, uint32_t *out) {
    for (size_t i = 0; call && i < n; i++)
        if (call[i] == INT32_MIN) {
            set_error("call key INT32_MIN is reserved");
            return SYZCOV_EINVAL;
        }
    CorpusDev cd;
    RC(stage_corpus(c, offsets, pcs, n, cd));
    const uint32_t nids = cd.n_ids;
    if (nids == 0) return 0;
    Plan p;
    size_t i_call = p.add(call ? n * 4 : 4), i_cnt = p.add((size_t)nids * 4 + 4),
           i_own = p.add((size_t)nids * 4 + 4), i_flag = p.add(nids), i_pc = p.add((size_t)nids * 4),
           i_out = p.add((size_t)nids * 4), i_n = p.add(4),
           i_ws = p.add(syzcov_dev_compact_ws_size(nids));
    std::vector<uint8_t *> b;
    RC(reserve(c, p, b));
    if (call) CK(hipMemcpyAsync(b[i_call], call, n * 4, hipMemcpyHostToDevice, c->s));
    RC(unique_cover_launch(cd.off, cd.pcs, (uint32_t)n, call ? (const int32_t *)b[i_call] : nullptr,
                           cd.tab, cd.span, cd.pc_lo, nids, (uint32_t *)b[i_cnt],
                           (int32_t *)b[i_own], b[i_flag], (int32_t *)b[i_pc], c->s));
    RC(syzcov_dev_compact_kept(b[i_flag], (const int32_t *)b[i_pc], nids, (int32_t *)b[i_out],
                               (uint32_t *)b[i_n], b[i_ws], c->s));
    uint32_t k = 0;
    CK(hipMemcpyAsync(&k, b[i_n], 4, hipMemcpyDeviceToHost, c->s));
    CK(hipStreamSynchronize(c->s));
    if (k) {
        CK(hipMemcpyAsync(out, b[i_out], (size_t)k * 4, hipMemcpyDeviceToHost, c->s));
        CK(hipStreamSynchronize(c->s));
    }
    // html.go:236 calls cover.Canonicalize(cov) but returns cov itself: the
    // sorted slice in full, so a lone 0xFFFFFFFF is kept
    return (int64_t)k;
}

// Manager UI statistics (html.go:67-99 httpSummary, :157-175 httpCorpus).
static int64_t ui_stats_impl(Ctx *c, const int32_t *call, const uint64_t *offsets,
                             const uint32_t *pcs, size_t n, uint32_t ncalls, uint32_t *inputs,
                             uint32_t *cover, uint32_t *ucov, uint32_t *in_unique) {
    for (size_t i = 0; i < n; i++) {
        if (offsets[i + 1] < offsets[i]) return SYZCOV_EINVAL;
        if (call && (call[i] < 0 || (uint32_t)call[i] >= ncalls)) {
            set_error("call group %d of input %zu outside [0, %u)", call[i], i, ncalls);
            return SYZCOV_EINVAL;
        }
        for (uint64_t k = offsets[i] + 1; k < offsets[i + 1]; k++)
            if (pcs[k] <= pcs[k - 1]) {
                set_error("cover of input %zu is not canonical", i);
                return SYZCOV_ENOTSORTED;
            }
    }
    if (inputs) {
        std::fill(inputs, inputs + ncalls, 0u);
        for (size_t i = 0; i < n; i++) inputs[call[i]]++;
    }
    const bool empty = offsets[n] == offsets[0];
    CorpusDev cd{};
    if (!empty) RC(stage_corpus(c, offsets, pcs, n, cd));
    const uint32_t nids = empty ? 0 : cd.n_ids;
    if (nids == 0) {
        if (cover) std::fill(cover, cover + ncalls, 0u);
        if (ucov) std::fill(ucov, ucov + ncalls, 0u);
        if (in_unique) std::fill(in_unique, in_unique + n, 0u);
        return 0;
    }
    // 0xFFFFFFFF is the largest PC: if present, it is the last dense id
    const bool has_sent = cd.pc_lo + (cd.span - 1) == 0xFFFFFFFFull;
    const uint32_t sent_id = has_sent ? nids - 1 : 0xFFFFFFFFu;
    const uint64_t wpg = ((uint64_t)nids + 31) / 32;
    const uint64_t slab_words = call ? std::min<uint64_t>((uint64_t)ncalls * wpg, 64ull << 20) : 1;
    Plan p;
    size_t i_call = p.add(call ? n * 4 : 4), i_ca = p.add((size_t)nids * 4 + 4),
           i_oa = p.add((size_t)nids * 4 + 4), i_cc = p.add((size_t)nids * 4 + 4),
           i_oc = p.add((size_t)nids * 4 + 4), i_fl = p.add(nids),
           i_slab = p.add(std::max<uint64_t>(slab_words, wpg) * 4), i_cov = p.add((size_t)ncalls * 4),
           i_uc = p.add((size_t)ncalls * 4), i_in = p.add(n * 4);
    std::vector<uint8_t *> b;
    RC(reserve(c, p, b));
    if (call) CK(hipMemcpyAsync(b[i_call], call, n * 4, hipMemcpyHostToDevice, c->s));
    RC(ui_stats_launch(cd.off, cd.pcs, (uint32_t)n, call ? (const int32_t *)b[i_call] : nullptr,
                       ncalls, cd.tab, cd.pc_lo, nids, sent_id, (uint32_t *)b[i_ca],
                       (int32_t *)b[i_oa], (uint32_t *)b[i_cc], (int32_t *)b[i_oc], b[i_fl],
                       (uint32_t *)b[i_slab], std::max<uint64_t>(slab_words, wpg),
                       (uint32_t *)b[i_cov], (uint32_t *)b[i_uc], (uint32_t *)b[i_in], c->s));
    if (call && cover) CK(hipMemcpyAsync(cover, b[i_cov], (size_t)ncalls * 4, hipMemcpyDeviceToHost, c->s));
    if (call && ucov) CK(hipMemcpyAsync(ucov, b[i_uc], (size_t)ncalls * 4, hipMemcpyDeviceToHost, c->s));
    if (in_unique) CK(hipMemcpyAsync(in_unique, b[i_in], n * 4, hipMemcpyDeviceToHost, c->s));
    CK(hipStreamSynchronize(c->s));
    return (int64_t)nids - (has_sent ? 1 : 0);
}

int64_t syzcov_ui_stats(const int32_t *call, const uint64_t *offsets, const uint32_t *pcs,
                        size_t n, uint32_t ncalls, uint32_t *inputs, uint32_t *cover,
                        uint32_t *unique_cover, uint32_t *input_unique) {
    if (!offsets || n > 0x7FFFFFFF || (n && offsets[n] != offsets[0] && !pcs)) return SYZCOV_EINVAL;
    if ((inputs || cover || unique_cover) && (!call || ncalls == 0)) return SYZCOV_EINVAL;
    if (!call) ncalls = 0;
    if (n == 0) {
        if (inputs) std::fill(inputs, inputs + ncalls, 0u);
        if (cover) std::fill(cover, cover + ncalls, 0u);
        if (unique_cover) std::fill(unique_cover, unique_cover + ncalls, 0u);
        return 0;
    }
    CtxLease lease;
    Ctx *c = lease.get();
    if (!c) return SYZCOV_ENODEV;
    const int64_t rc = ui_stats_impl(c, call, offsets, pcs, n, ncalls, inputs, cover, unique_cover,
                                     input_unique);
    hipStreamSynchronize(c->s);
    release_large(c);
    return rc;
}

int64_t syzcov_unique_cover(const int32_t *call, const uint64_t *offsets, const uint32_t *pcs,
                            size_t n, uint32_t *out) {
    if (n == 0) return 0;
    if (!offsets || !out || n > 0x7FFFFFFF) return SYZCOV_EINVAL;
    if (offsets[n] == offsets[0]) return 0;
    if (!pcs) return SYZCOV_EINVAL;
    CtxLease lease;
    Ctx *c = lease.get();
    if (!c) return SYZCOV_ENODEV;
    const int64_t rc = unique_cover_impl(c, call, offsets, pcs, n, out);
    hipStreamSynchronize(c->s);
    release_large(c);
    return rc;
}

int64_t syzcov_union_all(const uint64_t *offsets, const uint32_t *pcs, size_t n, uint32_t *out) {
    if (n == 0) return 0;
    if (!offsets || !out) return SYZCOV_EINVAL;
    if (offsets[n] == offsets[0]) return 0;
    if (!pcs) return SYZCOV_EINVAL;
    CtxLease lease;
    Ctx *c = lease.get();
    if (!c) return SYZCOV_ENODEV;
    CorpusDev cd;
    int64_t rc = stage_corpus(c, offsets, pcs, n, cd);
    if (!rc) {
        Plan p;
        const size_t i_out = p.add((size_t)cd.n_ids * 4 + 4), i_n = p.add(256);
        std::vector<uint8_t *> b;
        rc = reserve(c, p, b);
        if (!rc) {
            uint32_t *d_out = (uint32_t *)b[i_out], *d_n = (uint32_t *)b[i_n];
            rc = syzcov_dev_dict_to_list(cd.tab, cd.span, cd.pc_lo, d_out, d_n, c->s);
            uint32_t k = 0;
            if (!rc && (hipMemcpyAsync(&k, d_n, 4, hipMemcpyDeviceToHost, c->s) != hipSuccess ||
                        hipStreamSynchronize(c->s) != hipSuccess))
                rc = SYZCOV_EHIP;
            if (!rc && k &&
                (hipMemcpyAsync(out, d_out, (size_t)k * 4, hipMemcpyDeviceToHost, c->s) !=
                     hipSuccess ||
                 hipStreamSynchronize(c->s) != hipSuccess))
                rc = SYZCOV_EHIP;
            if (!rc) rc = k;
        }
    }
    hipStreamSynchronize(c->s);
    release_large(c);
    return rc;
}

// ------------------------------------------------------------ priorities
int syzcov_calculate_priorities(const uint64_t *prog_off, const uint16_t *call_ids, size_t nprog,
                                int C, int key_mode, const float *static_prios, float *out,
                                uint32_t *raw_counts) {
    if (C <= 0 || !out || (nprog && !prog_off) || (key_mode != 0 && key_mode != 1))
        return SYZCOV_EINVAL;
    const uint64_t base = nprog ? prog_off[0] : 0;
    const uint64_t ncalls = nprog ? prog_off[nprog] - base : 0;
    if (key_mode == 1 && ncalls && !call_ids) return SYZCOV_EINVAL;
    std::vector<int32_t> lens(nprog ? nprog : 1);
    std::vector<uint64_t> hoff(nprog + 1);
    for (size_t p = 0; p < nprog; p++) {
        const uint64_t l = prog_off[p + 1] - prog_off[p];
        if (key_mode == 0 && l > (uint64_t)C) {
            set_error("program %zu has %llu calls > %d (prio.go:148 would panic)", p,
                      (unsigned long long)l, C);
            return SYZCOV_ETOOLONG;
        }
        if (l > 0x7FFFFFFF) return SYZCOV_EINVAL;
        lens[p] = (int32_t)l;
    }
    for (size_t p = 0; p <= nprog; p++) hoff[p] = nprog ? prog_off[p] - base : 0;
    CtxLease lease;
    Ctx *c = lease.get();
    if (!c) return SYZCOV_ENODEV;
    const size_t rows = syzcov_dev_prio_rows(C), ldp = syzcov_dev_prio_ldp(nprog ? nprog : 1);
    int max_len = 0;
    for (size_t q = 0; q < nprog; q++) max_len = std::max(max_len, lens[q]);
    if (key_mode == 0) {  // positional: the active keys only (prio.hip)
        Plan p;
        size_t i_len = p.add(lens.size() * 4), i_cnt = p.add(rows * rows * 4),
               i_st = p.add((size_t)C * C * 4), i_out = p.add((size_t)C * C * 4),
               i_raw = p.add(raw_counts ? (size_t)C * C * 4 : 0),
               i_ws = p.add(syzcov_dev_prio_pos_ws_size(nprog ? nprog : 1, C, max_len));
        std::vector<uint8_t *> b;
        RC(reserve(c, p, b));
        CK(hipMemcpyAsync(b[i_len], lens.data(), lens.size() * 4, hipMemcpyHostToDevice, c->s));
        if (static_prios)
            CK(hipMemcpyAsync(b[i_st], static_prios, (size_t)C * C * 4, hipMemcpyHostToDevice,
                              c->s));
        CK(hipMemsetAsync(b[i_cnt], 0, rows * rows * 4, c->s));
        RC(syzcov_dev_prio_counts_pos((int32_t *)b[i_len], nprog, C, max_len, (int32_t *)b[i_cnt],
                                      b[i_ws], p.sizes[i_ws], c->s));
        RC(syzcov_dev_prio_finish((int32_t *)b[i_cnt], C,
                                  static_prios ? (float *)b[i_st] : nullptr, (float *)b[i_out],
                                  raw_counts ? (uint32_t *)b[i_raw] : nullptr, c->s));
        CK(hipMemcpyAsync(out, b[i_out], (size_t)C * C * 4, hipMemcpyDeviceToHost, c->s));
        if (raw_counts)
            CK(hipMemcpyAsync(raw_counts, b[i_raw], (size_t)C * C * 4, hipMemcpyDeviceToHost,
                              c->s));
        CK(hipStreamSynchronize(c->s));
        return 0;
    }
    Plan p;
    size_t i_len = p.add(lens.size() * 4), i_off = p.add((nprog + 1) * 8),
           i_ids = p.add(key_mode ? ncalls * 2 : 0), i_at = p.add(rows * ldp),
           i_cnt = p.add(rows * rows * 4), i_st = p.add((size_t)C * C * 4),
           i_out = p.add((size_t)C * C * 4), i_raw = p.add(raw_counts ? (size_t)C * C * 4 : 0),
           i_err = p.add(4), i_dws = p.add(syzcov_dev_prio_counts_ws_size(nprog, C));
    std::vector<uint8_t *> b;
    RC(reserve(c, p, b));
    CK(hipMemsetAsync(b[i_err], 0, 4, c->s));
    CK(hipMemcpyAsync(b[i_len], lens.data(), lens.size() * 4, hipMemcpyHostToDevice, c->s));
    CK(hipMemcpyAsync(b[i_off], hoff.data(), (nprog + 1) * 8, hipMemcpyHostToDevice, c->s));
    if (key_mode && ncalls)
        CK(hipMemcpyAsync(b[i_ids], call_ids + base, ncalls * 2, hipMemcpyHostToDevice, c->s));
    if (static_prios)
        CK(hipMemcpyAsync(b[i_st], static_prios, (size_t)C * C * 4, hipMemcpyHostToDevice, c->s));
    RC(syzcov_dev_prio_build_at(key_mode, (int32_t *)b[i_len], (uint64_t *)b[i_off],
                                (uint16_t *)b[i_ids], nprog, C, (int8_t *)b[i_at], ldp,
                                (uint32_t *)b[i_err], c->s));
    CK(hipMemsetAsync(b[i_cnt], 0, rows * rows * 4, c->s));
    RC(syzcov_dev_prio_counts_ws((int8_t *)b[i_at], ldp, nprog, C, (int32_t *)b[i_cnt], b[i_dws],
                                 p.sizes[i_dws], c->s));
    RC(syzcov_dev_prio_finish((int32_t *)b[i_cnt], C, static_prios ? (float *)b[i_st] : nullptr,
                              (float *)b[i_out], raw_counts ? (uint32_t *)b[i_raw] : nullptr,
                              c->s));
    uint32_t herr = 0;
    CK(hipMemcpyAsync(&herr, b[i_err], 4, hipMemcpyDeviceToHost, c->s));
    CK(hipMemcpyAsync(out, b[i_out], (size_t)C * C * 4, hipMemcpyDeviceToHost, c->s));
    if (raw_counts)
        CK(hipMemcpyAsync(raw_counts, b[i_raw], (size_t)C * C * 4, hipMemcpyDeviceToHost, c->s));
    CK(hipStreamSynchronize(c->s));
    if (herr) {
        set_error("call id >= C");
        return SYZCOV_EINVAL;
    }
    return 0;
}

int syzcov_static_priorities(const uint32_t *id_off, const uint16_t *id_calls, const float *id_w,
                             size_t nids, const uint32_t *call_off, const uint32_t *call_ids,
                             const float *call_w, int C, float *out) {
    if (C <= 0 || !id_off || !call_off || !out) return SYZCOV_EINVAL;
    const size_t nm = id_off[nids], nc = call_off[C];
    if ((nm && (!id_calls || !id_w)) || (nc && (!call_ids || !call_w))) return SYZCOV_EINVAL;
    CtxLease lease;
    Ctx *c = lease.get();
    if (!c) return SYZCOV_ENODEV;
    Plan p;
    size_t i_io = p.add((nids + 1) * 4), i_ic = p.add(nm * 2), i_iw = p.add(nm * 4),
           i_co = p.add(((size_t)C + 1) * 4), i_ci = p.add(nc * 4), i_cw = p.add(nc * 4),
           i_o = p.add((size_t)C * C * 4);
    std::vector<uint8_t *> b;
    RC(reserve(c, p, b));
    CK(hipMemcpyAsync(b[i_io], id_off, (nids + 1) * 4, hipMemcpyHostToDevice, c->s));
    if (nm) CK(hipMemcpyAsync(b[i_ic], id_calls, nm * 2, hipMemcpyHostToDevice, c->s));
    if (nm) CK(hipMemcpyAsync(b[i_iw], id_w, nm * 4, hipMemcpyHostToDevice, c->s));
    CK(hipMemcpyAsync(b[i_co], call_off, ((size_t)C + 1) * 4, hipMemcpyHostToDevice, c->s));
    if (nc) CK(hipMemcpyAsync(b[i_ci], call_ids, nc * 4, hipMemcpyHostToDevice, c->s));
    if (nc) CK(hipMemcpyAsync(b[i_cw], call_w, nc * 4, hipMemcpyHostToDevice, c->s));
    RC(syzcov_dev_static_prio((uint32_t *)b[i_io], (uint16_t *)b[i_ic], (float *)b[i_iw],
                              (uint32_t *)b[i_co], (uint32_t *)b[i_ci], (float *)b[i_cw], C,
                              (float *)b[i_o], c->s));
    CK(hipMemcpyAsync(out, b[i_o], (size_t)C * C * 4, hipMemcpyDeviceToHost, c->s));
    CK(hipStreamSynchronize(c->s));
    return 0;
}

int syzcov_normalize_prio(float *prios, int C) {
    if (C <= 0 || !prios) return SYZCOV_EINVAL;
    CtxLease lease;
    Ctx *c = lease.get();
    if (!c) return SYZCOV_ENODEV;
    Plan p;
    size_t i_p = p.add((size_t)C * C * 4);
    std::vector<uint8_t *> b;
    RC(reserve(c, p, b));
    CK(hipMemcpyAsync(b[i_p], prios, (size_t)C * C * 4, hipMemcpyHostToDevice, c->s));
    RC(syzcov_dev_normalize_prio((float *)b[i_p], C, c->s));
    CK(hipMemcpyAsync(prios, b[i_p], (size_t)C * C * 4, hipMemcpyDeviceToHost, c->s));
    CK(hipStreamSynchronize(c->s));
    return 0;
}

int syzcov_build_choice_table(const float *prios, const uint8_t *enabled, int C, int64_t *run) {
    if (C <= 0 || !prios || !run) return SYZCOV_EINVAL;
    CtxLease lease;
    Ctx *c = lease.get();
    if (!c) return SYZCOV_ENODEV;
    Plan p;
    size_t i_p = p.add((size_t)C * C * 4), i_e = p.add(C), i_r = p.add((size_t)C * C * 8);
    std::vector<uint8_t *> b;
    RC(reserve(c, p, b));
    CK(hipMemcpyAsync(b[i_p], prios, (size_t)C * C * 4, hipMemcpyHostToDevice, c->s));
    if (enabled) CK(hipMemcpyAsync(b[i_e], enabled, C, hipMemcpyHostToDevice, c->s));
    // disabled rows keep the caller's contents (nil rows in Go)
    CK(hipMemcpyAsync(b[i_r], run, (size_t)C * C * 8, hipMemcpyHostToDevice, c->s));
    RC(syzcov_dev_choice_table((float *)b[i_p], enabled ? b[i_e] : nullptr, C, (int64_t *)b[i_r],
                               c->s));
    CK(hipMemcpyAsync(run, b[i_r], (size_t)C * C * 8, hipMemcpyDeviceToHost, c->s));
    CK(hipStreamSynchronize(c->s));
    return 0;
}

int syzcov_choose_batch(const int64_t *run, const uint8_t *enabled, int C, const int32_t *calls,
                        const int64_t *x, size_t nq, int32_t *out) {
    if (nq == 0) return 0;
    if (C <= 0 || !run || !calls || !x || !out) return SYZCOV_EINVAL;
    CtxLease lease;
    Ctx *c = lease.get();
    if (!c) return SYZCOV_ENODEV;
    Plan p;
    size_t i_r = p.add((size_t)C * C * 8), i_e = p.add(C), i_c = p.add(nq * 4), i_x = p.add(nq * 8),
           i_o = p.add(nq * 4), i_f = p.add(4);
    std::vector<uint8_t *> b;
    RC(reserve(c, p, b));
    CK(hipMemcpyAsync(b[i_r], run, (size_t)C * C * 8, hipMemcpyHostToDevice, c->s));
    if (enabled) CK(hipMemcpyAsync(b[i_e], enabled, C, hipMemcpyHostToDevice, c->s));
    CK(hipMemcpyAsync(b[i_c], calls, nq * 4, hipMemcpyHostToDevice, c->s));
    CK(hipMemcpyAsync(b[i_x], x, nq * 8, hipMemcpyHostToDevice, c->s));
    CK(hipMemsetAsync(b[i_f], 0, 4, c->s));
    RC(syzcov_dev_choose((const int64_t *)b[i_r], enabled ? b[i_e] : nullptr, C,
                         (const int32_t *)b[i_c], (const int64_t *)b[i_x], nq, (int32_t *)b[i_o],
                         (uint32_t *)b[i_f], c->s));
    uint32_t err = 0;
    CK(hipMemcpyAsync(out, b[i_o], nq * 4, hipMemcpyDeviceToHost, c->s));
    CK(hipMemcpyAsync(&err, b[i_f], 4, hipMemcpyDeviceToHost, c->s));
    CK(hipStreamSynchronize(c->s));
    if (err) {
        set_error("Choose: call id >= C or draw outside [0, run[call][C-1])");
        return SYZCOV_ERANGE;
    }
    return 0;
}

}  // extern "C"
