/*
 * cover_oracle.c — literal sequential restatement of cover/cover.go.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Compiled with -ffp-contract=off.
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

#define SENT 0xFFFFFFFFu /* cover/cover.go:17 `const sent = ^uint32(0)` */

static int cmp_u32(const void *a, const void *b) {
    uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
    return x < y ? -1 : x > y;
}

/* cover/cover.go:28-40.  The sort algorithm is irrelevant for the result:
 * uint32 values with equal keys are indistinguishable. */
size_t orc_canonicalize(uint32_t *cov, size_t n) {
    qsort(cov, n, sizeof(uint32_t), cmp_u32);
    size_t i = 0;
    uint32_t last = SENT; /* :30 `last := sent` */
    for (size_t k = 0; k < n; k++) {
        uint32_t pc = cov[k];
        if (pc != last) {
            last = pc;
            cov[i++] = pc;
        }
    }
    return i;
}

static int cmp_u64(const void *a, const void *b) {
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

/* executor/executor.cc:574-587: std::sort, then skip pc == last with
 * last = 0 at the start (:578), so zero PCs are dropped too.  (The network
 * used to sort is irrelevant: equal u64 values are indistinguishable.) */
size_t orc_cover_dedup64(uint64_t *cov, size_t n) {
    qsort(cov, n, sizeof(uint64_t), cmp_u64);
    size_t w = 0;
    uint64_t last = 0;
    for (size_t i = 0; i < n; i++) {
        uint64_t pc = cov[i];
        if (pc == last) continue;
        cov[w++] = last = pc;
    }
    return w;
}

/* The four closures passed to foreach (cover/cover.go:42-79). */
static uint32_t f_apply(int op, uint32_t v0, uint32_t v1) {
    switch (op) {
    case 0: /* Difference :43-48 */
        return v0 < v1 ? v0 : SENT;
    case 1: /* SymmetricDifference :52-60 */
        if (v0 < v1) return v0;
        if (v1 < v0) return v1;
        return SENT;
    case 2: /* Union :64-69 */
        return v0 <= v1 ? v0 : v1;
    default: /* Intersection :73-78 */
        return v0 == v1 ? v0 : SENT;
    }
}

/* cover/cover.go:81-102 */
size_t orc_setop(int op, const uint32_t *a, size_t na, const uint32_t *b, size_t nb,
                 uint32_t *out) {
    size_t r = 0;
    for (size_t i0 = 0, i1 = 0; i0 < na || i1 < nb;) {
        uint32_t v0 = SENT, v1 = SENT;
        if (i0 < na) v0 = a[i0];
        if (i1 < nb) v1 = b[i1];
        if (v0 <= v1) i0++;
        if (v1 <= v0) i1++;
        uint32_t v = f_apply(op, v0, v1);
        if (v != SENT) out[r++] = v;
    }
    return r;
}

/* ---- map[uint32]struct{} stand-in: open addressing, occupancy bytes so
 * that 0xFFFFFFFF is an ordinary key (Minimize treats it as a PC). ---- */
typedef struct {
    uint32_t *keys;
    uint8_t *used;
    size_t cap, size;
} u32set;

static uint64_t mix(uint32_t x) {
    uint64_t z = (uint64_t)x * 0x9E3779B97F4A7C15ull;
    return z ^ (z >> 29);
}

static void set_init(u32set *s, size_t cap) {
    s->cap = 16;
    while (s->cap < cap) s->cap <<= 1;
    s->keys = (uint32_t *)malloc(s->cap * sizeof(uint32_t));
    s->used = (uint8_t *)calloc(s->cap, 1);
    s->size = 0;
}

static void set_free(u32set *s) {
    free(s->keys);
    free(s->used);
}

static int set_has(const u32set *s, uint32_t k) {
    size_t m = s->cap - 1, h = (size_t)mix(k) & m;
    while (s->used[h]) {
        if (s->keys[h] == k) return 1;
        h = (h + 1) & m;
    }
    return 0;
}

static void set_add(u32set *s, uint32_t k);

static void set_grow(u32set *s) {
    u32set t;
    set_init(&t, s->cap * 2);
    for (size_t i = 0; i < s->cap; i++)
        if (s->used[i]) set_add(&t, s->keys[i]);
    set_free(s);
    *s = t;
}

static void set_add(u32set *s, uint32_t k) {
    if ((s->size + 1) * 2 > s->cap) set_grow(s);
    size_t m = s->cap - 1, h = (size_t)mix(k) & m;
    while (s->used[h]) {
        if (s->keys[h] == k) return;
        h = (h + 1) & m;
    }
    s->used[h] = 1;
    s->keys[h] = k;
    s->size++;
}

/* cover/cover.go:104-131 */
size_t orc_minimize(const uint64_t *offsets, const uint32_t *pcs, size_t n, int variant,
                    int32_t *out_idx) {
    int32_t *order = (int32_t *)malloc((n ? n : 1) * sizeof(int32_t));
    int64_t *len = (int64_t *)calloc(n ? n : 1, sizeof(int64_t));
    for (size_t i = 0; i < n; i++) {
        order[i] = (int32_t)i; /* inputs[i] = &minInput{idx: i, cov: cov} :106-112 */
        len[i] = (int64_t)(offsets[i + 1] - offsets[i]);
    }
    orc_sort_min_inputs(order, len, n, variant); /* :113 sort.Sort(minInputArray(inputs)) */
    size_t kept = 0;
    u32set covered;                              /* :115 covered := make(map[uint32]struct{}) */
    set_init(&covered, 1024);
    for (size_t r = 0; r < n; r++) {             /* :116 for _, inp := range inputs */
        int32_t idx = order[r];
        int hit = 0;
        for (uint64_t p = offsets[idx]; p < offsets[idx + 1]; p++) {
            uint32_t pc = pcs[p];
            if (!hit) {
                if (!set_has(&covered, pc)) {
                    hit = 1;
                    out_idx[kept++] = idx; /* min = append(min, inp.idx) */
                }
            }
            if (hit) set_add(&covered, pc);
        }
    }
    set_free(&covered);
    free(order);
    free(len);
    return kept;
}

size_t orc_union_fold(const uint64_t *offsets, const uint32_t *pcs, size_t n, uint32_t *out) {
    size_t cap = (size_t)offsets[n] + 1;
    uint32_t *total = (uint32_t *)malloc(cap * sizeof(uint32_t));
    uint32_t *tmp = (uint32_t *)malloc(cap * sizeof(uint32_t));
    size_t nt = 0;
    for (size_t i = 0; i < n; i++) { /* total = Union(total, c) */
        size_t m = orc_setop(2, total, nt, pcs + offsets[i], (size_t)(offsets[i + 1] - offsets[i]),
                             tmp);
        uint32_t *s = total;
        total = tmp;
        tmp = s;
        nt = m;
    }
    memcpy(out, total, nt * sizeof(uint32_t));
    free(total);
    free(tmp);
    return nt;
}

/* syz-fuzzer/fuzzer.go:456-480, one record at a time, in batch order. */
void orc_newcov_batch(const uint64_t *mc_off, const uint32_t *mc_pcs, int ncalls,
                      const uint32_t *flakes, size_t nflakes, const int32_t *callid,
                      const uint64_t *rec_off, const uint32_t *rec_pcs, size_t nrec,
                      uint8_t *is_new, uint64_t *new_off, uint32_t *new_pcs) {
    size_t maxrec = 0, total = (size_t)mc_off[ncalls];
    for (size_t k = 0; k < nrec; k++) {
        size_t l = (size_t)(rec_off[k + 1] - rec_off[k]);
        if (l > maxrec) maxrec = l;
        total += l;
    }
    /* per-call working lists */
    uint32_t **mc = (uint32_t **)calloc((size_t)ncalls, sizeof(uint32_t *));
    size_t *mcn = (size_t *)calloc((size_t)ncalls, sizeof(size_t));
    for (int c = 0; c < ncalls; c++) {
        mcn[c] = (size_t)(mc_off[c + 1] - mc_off[c]);
        mc[c] = (uint32_t *)malloc((mcn[c] + 1) * sizeof(uint32_t));
        memcpy(mc[c], mc_pcs + mc_off[c], mcn[c] * sizeof(uint32_t));
    }
    uint32_t *d1 = (uint32_t *)malloc((maxrec + 1) * sizeof(uint32_t));
    uint32_t *d2 = (uint32_t *)malloc((maxrec + 1) * sizeof(uint32_t));
    for (size_t k = 0; k < nrec; k++) {
        const uint32_t *cov = rec_pcs + rec_off[k];
        size_t l = (size_t)(rec_off[k + 1] - rec_off[k]);
        is_new[k] = 0;
        if (l == 0) continue; /* :460 if len(cov) == 0 { continue } */
        int c = callid[k];
        size_t n1 = orc_setop(0, cov, l, mc[c], mcn[c], d1); /* :465 */
        size_t n2 = orc_setop(0, d1, n1, flakes, nflakes, d2); /* :466 */
        if (n2 != 0) {
            uint32_t *u = (uint32_t *)malloc((mcn[c] + n2 + 1) * sizeof(uint32_t));
            size_t nu = orc_setop(2, mc[c], mcn[c], d2, n2, u); /* :470 */
            free(mc[c]);
            mc[c] = u;
            mcn[c] = nu;
            is_new[k] = 1; /* :474-477 triage append */
        }
    }
    size_t o = 0;
    for (int c = 0; c < ncalls; c++) {
        new_off[c] = o;
        memcpy(new_pcs + o, mc[c], mcn[c] * sizeof(uint32_t));
        o += mcn[c];
        free(mc[c]);
    }
    new_off[ncalls] = o;
    (void)total;
    free(mc);
    free(mcn);
    free(d1);
    free(d2);
}
