/*
 * fullsize.c — full-size CPU oracle run over a synthetic corpus that does not
 * fit host memory (config C3: 10M inputs, 20.5 G raw PCs = 82 GB).
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h): run once in the build container by
 * tools/gen_golden_fullsize.py to write the digests in tests/golden/; the GPU
 * tests compare the engine's results against those digests.
 *
 * The computation is cover.Minimize (cover/cover.go:104-131) and the Union
 * fold `total = Union(total, cov)` (manager.go:606-610) over the canonical
 * covers (cover.go:27-40) of the synthetic inputs, restated so that the corpus
 * is never held in memory:
 *   pass 1  regenerate + canonicalize every input (threads), keep its length
 *   order   Go sort.Sort(minInputArray) over the lengths (orc_sort_min_inputs)
 *   pass 2  walk the ranks in order; blocks of ranks are regenerated and
 *           canonicalized by the threads, then scanned sequentially with the
 *           reference's loop (`hit` / covered set), the set being a bitmap over
 *           the whole uint32 space (512 MB) instead of a Go map
 *   union   the covered set after the last input = the Union fold's result,
 *           minus 0xFFFFFFFF (Union drops the sentinel, cover.go:97)
 * Canonicalize uses an LSD radix sort instead of qsort; the result of sort +
 * unique does not depend on the sort algorithm, and the tool checks its
 * canonical lists against orc_canonicalize on the first inputs of every run.
 *
 * Usage: fullsize SEED N MEAN SIGMA LOG2 THREADS OUTDIR
 * Writes OUTDIR/{lens.u32,order.i32,kept.i32,union.u32} and prints a summary.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define SENT 0xFFFFFFFFu

/* sort + unique with cover.go:30's `last := sent` start */
static size_t canon_radix(uint32_t *a, uint32_t *tmp, size_t n) {
    uint32_t cnt[2048];
    uint32_t *src = a, *dst = tmp;
    for (int pass = 0; pass < 3; pass++) {
        const int sh = pass * 11;
        memset(cnt, 0, sizeof cnt);
        for (size_t i = 0; i < n; i++) cnt[(src[i] >> sh) & 2047]++;
        uint32_t s = 0;
        for (int d = 0; d < 2048; d++) {
            uint32_t c = cnt[d];
            cnt[d] = s;
            s += c;
        }
        for (size_t i = 0; i < n; i++) dst[cnt[(src[i] >> sh) & 2047]++] = src[i];
        uint32_t *t = src;
        src = dst;
        dst = t;
    }
    /* after 3 passes the sorted keys are in tmp (odd pass count) */
    size_t k = 0;
    uint32_t last = SENT;
    for (size_t i = 0; i < n; i++)
        if (src[i] != last) {
            last = src[i];
            a[k++] = last;
        }
    return k;
}

typedef struct {
    uint64_t seed;
    uint32_t mean, sigma, log2;
    int mode; /* synth mode: bit 1 = the x86-like universe */
} cfg_t;

/* canonical cover of synthetic input `i` into out (capacity 65535); returns length */
static size_t gen_canon(const cfg_t *c, uint64_t i, uint32_t *out, uint32_t *tmp) {
    uint32_t L = orc_synth_len(c->seed, i, c->mean, c->sigma);
    orc_synth_input(c->seed, i, L, c->log2, c->mode, out);
    return canon_radix(out, tmp, L);
}

/* ---------------------------------------------------------------- pass 1 */
typedef struct {
    const cfg_t *c;
    uint64_t lo, hi;
    uint32_t *lens;
    uint64_t raw, canon;
} p1_t;

static void *pass1(void *arg) {
    p1_t *p = (p1_t *)arg;
    uint32_t *buf = malloc(65536 * 4), *tmp = malloc(65536 * 4);
    for (uint64_t i = p->lo; i < p->hi; i++) {
        p->raw += orc_synth_len(p->c->seed, i, p->c->mean, p->c->sigma);
        size_t k = gen_canon(p->c, i, buf, tmp);
        p->lens[i] = (uint32_t)k;
        p->canon += k;
    }
    free(buf);
    free(tmp);
    return NULL;
}

/* ---------------------------------------------------------------- pass 2 */
typedef struct {
    const cfg_t *c;
    const int32_t *order;
    const uint64_t *boff; /* block-local offsets of ranks [r0, r1) */
    uint32_t *bpcs;
    uint64_t r0, r1, t, nt;
} p2_t;

static void *pass2_gen(void *arg) {
    p2_t *p = (p2_t *)arg;
    /* the raw list is longer than its canonical slot: generate into scratch */
    uint32_t *buf = malloc(65536 * 4), *tmp = malloc(65536 * 4);
    for (uint64_t r = p->r0 + p->t; r < p->r1; r += p->nt) {
        uint64_t o = p->boff[r - p->r0];
        size_t k = gen_canon(p->c, (uint64_t)p->order[r], buf, tmp);
        if (o + k != p->boff[r - p->r0 + 1]) abort();
        memcpy(p->bpcs + o, buf, k * 4);
    }
    free(buf);
    free(tmp);
    return NULL;
}

static int write_file(const char *dir, const char *name, const void *data, size_t bytes) {
    char path[4096];
    snprintf(path, sizeof path, "%s/%s", dir, name);
    FILE *f = fopen(path, "wb");
    if (!f) return -1;
    size_t w = bytes ? fwrite(data, 1, bytes, f) : 0;
    fclose(f);
    return w == bytes ? 0 : -1;
}

int main(int argc, char **argv) {
    if (argc != 8 && argc != 9) {
        fprintf(stderr, "usage: %s SEED N MEAN SIGMA LOG2 THREADS OUTDIR [MODE]\n", argv[0]);
        return 2;
    }
    cfg_t c = {strtoull(argv[1], 0, 0), 0, 0, 0, argc == 9 ? atoi(argv[8]) : 0};
    const uint64_t n = strtoull(argv[2], 0, 0);
    c.mean = (uint32_t)strtoul(argv[3], 0, 0);
    c.sigma = (uint32_t)strtoul(argv[4], 0, 0);
    c.log2 = (uint32_t)strtoul(argv[5], 0, 0);
    const int nt = atoi(argv[6]);
    const char *dir = argv[7];

    /* self-check: the radix canonical list equals orc_canonicalize (qsort) */
    {
        uint32_t *a = malloc(65536 * 4), *b = malloc(65536 * 4), *t = malloc(65536 * 4);
        for (uint64_t i = 0; i < 64 && i < n; i++) {
            uint32_t L = orc_synth_len(c.seed, i, c.mean, c.sigma);
            orc_synth_input(c.seed, i, L, c.log2, c.mode, a);
            memcpy(b, a, (size_t)L * 4);
            size_t k1 = canon_radix(a, t, L), k2 = orc_canonicalize(b, L);
            if (k1 != k2 || memcmp(a, b, k1 * 4)) {
                fprintf(stderr, "radix canonicalize disagrees with orc_canonicalize at %llu\n",
                        (unsigned long long)i);
                return 1;
            }
        }
        free(a);
        free(b);
        free(t);
    }

    uint32_t *lens = malloc(n * 4);
    pthread_t th[256];
    p1_t p1[256];
    for (int t = 0; t < nt; t++) {
        p1[t] = (p1_t){&c, n * t / nt, n * (t + 1) / nt, lens, 0, 0};
        pthread_create(&th[t], NULL, pass1, &p1[t]);
    }
    uint64_t raw = 0, canon = 0;
    for (int t = 0; t < nt; t++) {
        pthread_join(th[t], NULL);
        raw += p1[t].raw;
        canon += p1[t].canon;
    }
    fprintf(stderr, "pass 1 done: %llu raw, %llu canonical PCs\n", (unsigned long long)raw,
            (unsigned long long)canon);

    /* cover.go:113 sort.Sort(minInputArray(inputs)), Go >= 1.19 pdqsort */
    int64_t *len64 = malloc(n * 8);
    int32_t *order = malloc(n * 4);
    for (uint64_t i = 0; i < n; i++) {
        len64[i] = lens[i];
        order[i] = (int32_t)i;
    }
    orc_sort_min_inputs(order, len64, n, 0);
    free(len64);
    fprintf(stderr, "order done\n");

    /* pass 2: the reference's scan (cover.go:115-129) over a bitmap set */
    uint64_t *covered = calloc((1ull << 32) / 64, 8);
    int32_t *kept = malloc(n * 4);
    uint64_t nkept = 0;
    const uint64_t B = 32768;
    uint64_t *boff = malloc((B + 1) * 8);
    uint32_t *bpcs = malloc(B * 65536ull * 4 > (1ull << 31) ? (1ull << 31) : B * 65536ull * 4);
    for (uint64_t r0 = 0; r0 < n; r0 += B) {
        uint64_t r1 = r0 + B < n ? r0 + B : n;
        boff[0] = 0;
        for (uint64_t r = r0; r < r1; r++) boff[r - r0 + 1] = boff[r - r0] + lens[order[r]];
        if (boff[r1 - r0] * 4 > (1ull << 31)) {
            fprintf(stderr, "block too large\n");
            return 1;
        }
        p2_t p2[256];
        for (int t = 0; t < nt; t++) {
            p2[t] = (p2_t){&c, order, boff, bpcs, r0, r1, (uint64_t)t, (uint64_t)nt};
            pthread_create(&th[t], NULL, pass2_gen, &p2[t]);
        }
        for (int t = 0; t < nt; t++) pthread_join(th[t], NULL);
        for (uint64_t r = r0; r < r1; r++) {
            int hit = 0;
            for (uint64_t q = boff[r - r0]; q < boff[r - r0 + 1]; q++) {
                uint32_t pc = bpcs[q];
                uint64_t m = 1ull << (pc & 63);
                uint64_t *w = &covered[pc >> 6];
                if (!hit && !(*w & m)) {
                    hit = 1;
                    kept[nkept++] = order[r];
                }
                if (hit) *w |= m;
            }
        }
        if ((r0 / B) % 32 == 0)
            fprintf(stderr, "pass 2: %llu / %llu ranks\n", (unsigned long long)r1,
                    (unsigned long long)n);
    }
    /* the covered set in ascending order; Union drops the sentinel */
    uint64_t nunion = 0;
    for (uint64_t w = 0; w < (1ull << 32) / 64; w++) nunion += __builtin_popcountll(covered[w]);
    uint32_t *uni = malloc((nunion ? nunion : 1) * 4);
    uint64_t k = 0;
    for (uint64_t w = 0; w < (1ull << 32) / 64; w++)
        for (uint64_t x = covered[w]; x; x &= x - 1)
            uni[k++] = (uint32_t)(w * 64 + __builtin_ctzll(x));
    if (k && uni[k - 1] == SENT) k--;

    if (write_file(dir, "lens.u32", lens, n * 4) || write_file(dir, "order.i32", order, n * 4) ||
        write_file(dir, "kept.i32", kept, nkept * 4) || write_file(dir, "union.u32", uni, k * 4)) {
        fprintf(stderr, "write failed\n");
        return 1;
    }
    printf("{\"n\": %llu, \"raw_pcs\": %llu, \"canonical_pcs\": %llu, \"n_kept\": %llu, "
           "\"n_union\": %llu}\n",
           (unsigned long long)n, (unsigned long long)raw, (unsigned long long)canon,
           (unsigned long long)nkept, (unsigned long long)k);
    return 0;
}
