/*
 * newcov_full.c — full-size CPU oracle of config C5: the fuzzer's streaming
 * new-coverage check (syz-fuzzer/fuzzer.go:456-480) over a stream of batches
 * of 65,536 synthetic call records against per-CallID maxCover and the
 * global flakes set.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h): run by tools/gen_golden_fullsize.py
 * C5 in the build container; the GPU test compares the engine's per-batch
 * is_new flags and final maxCover against the digests it writes.
 *
 * Restatement: for every record in stream order (batch b, record k = synthetic
 * input b * NREC + k, canonical cover = sort + unique of its raw KCOV list,
 * CallID orc_synth_callid):
 *     diff := Difference(Difference(cov, maxCover[c]), flakes)     (:465-466)
 *     if len(diff) != 0 { maxCover[c] = Union(maxCover[c], diff); new }  (:467-477)
 * Each set is a bitmap over the PC window [0x81000000, +16 << LOG2) instead of
 * a sorted list: the same set, and Difference / Union reduce to bit tests and
 * sets (0xFFFFFFFF never occurs in the synthetic PCs).  Records of one call
 * touch only that call's maxCover, so calls are processed by different
 * threads, each walking the stream in order; generation is threaded by
 * record.
 *
 * Flakes: the unique PCs of synthetic input 2^40 of length 2^(LOG2-7).
 *
 * Usage: newcov_full SEED NREC NBATCH NCALLS MEAN SIGMA LOG2 THREADS OUTDIR
 * Writes OUTDIR/is_new.u8 (NBATCH * NREC flags), OUTDIR/maxcover_n.u32 (per
 * call) and OUTDIR/maxcover.u32 (the calls' sorted PCs, concatenated).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define PC_LO 0x81000000u
#define FLAKE_INPUT (1ull << 40)

typedef struct {
    uint64_t seed, first;
    uint32_t nrec, mean, sigma, log2;
    const uint64_t *off; /* raw slot starts (prefix of the raw lengths) */
    uint32_t *pcs;
    uint32_t *clen;      /* canonical lengths */
    uint32_t t, nt;
} gen_t;

static void *gen_recs(void *arg) {
    gen_t *g = (gen_t *)arg;
    for (uint32_t k = g->t; k < g->nrec; k += g->nt) {
        uint32_t *p = g->pcs + g->off[k];
        uint32_t L = (uint32_t)(g->off[k + 1] - g->off[k]);
        orc_synth_input(g->seed, g->first + k, L, g->log2, 0, p);
        /* Canonicalize (cover.go:27-40) in the record's own slot */
        g->clen[k] = (uint32_t)orc_canonicalize(p, L);
    }
    return NULL;
}

typedef struct {
    const uint64_t *roff;
    const uint32_t *clen;
    const uint32_t *pcs;
    const int32_t *cid;
    uint32_t nrec;
    uint64_t **mc;        /* per call bitmap */
    const uint64_t *fl;   /* flakes bitmap */
    uint8_t *is_new;
    uint32_t t, nt;
} chk_t;

static inline int btest(const uint64_t *b, uint32_t o) { return (b[o >> 6] >> (o & 63)) & 1; }

static void *check(void *arg) {
    chk_t *c = (chk_t *)arg;
    for (uint32_t k = 0; k < c->nrec; k++) {
        int32_t call = c->cid[k];
        if ((uint32_t)call % c->nt != c->t) continue;
        uint64_t *m = c->mc[call];
        const uint32_t *p = c->pcs + c->roff[k];
        size_t n = c->clen[k];
        int any = 0;
        for (size_t i = 0; i < n; i++) {
            uint32_t o = p[i] - PC_LO;
            if (!btest(m, o) && !btest(c->fl, o)) { any = 1; break; }
        }
        c->is_new[k] = (uint8_t)any;
        if (!any) continue;
        for (size_t i = 0; i < n; i++) { /* Union(maxCover, diff) */
            uint32_t o = p[i] - PC_LO;
            if (!btest(c->fl, o)) m[o >> 6] |= 1ull << (o & 63);
        }
    }
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
    if (argc != 10) {
        fprintf(stderr, "usage: %s SEED NREC NBATCH NCALLS MEAN SIGMA LOG2 THREADS OUTDIR\n",
                argv[0]);
        return 2;
    }
    const uint64_t seed = strtoull(argv[1], NULL, 0);
    const uint32_t nrec = (uint32_t)strtoul(argv[2], NULL, 0);
    const uint32_t nb = (uint32_t)strtoul(argv[3], NULL, 0);
    const uint32_t ncalls = (uint32_t)strtoul(argv[4], NULL, 0);
    const uint32_t mean = (uint32_t)strtoul(argv[5], NULL, 0);
    const uint32_t sigma = (uint32_t)strtoul(argv[6], NULL, 0);
    const uint32_t log2 = (uint32_t)strtoul(argv[7], NULL, 0);
    uint32_t nt = (uint32_t)strtoul(argv[8], NULL, 0);
    const char *dir = argv[9];
    if (nt < 1) nt = 1;
    if (nt > 64) nt = 64;
    const uint64_t span = 16ull << log2, words = (span + 63) / 64;
    uint64_t **mc = calloc(ncalls, sizeof *mc);
    for (uint32_t c = 0; c < ncalls; c++) mc[c] = calloc(words, 8);
    uint64_t *fl = calloc(words, 8);
    { /* flakes */
        uint32_t L = orc_synth_len(seed, FLAKE_INPUT, 1u << (log2 - 7), 1);
        uint32_t *f = malloc((size_t)L * 4);
        orc_synth_input(seed, FLAKE_INPUT, L, log2, 0, f);
        for (uint32_t i = 0; i < L; i++) fl[(f[i] - PC_LO) >> 6] |= 1ull << ((f[i] - PC_LO) & 63);
        free(f);
    }
    uint8_t *is_new = malloc((size_t)nb * nrec);
    uint64_t *off = malloc(((size_t)nrec + 1) * 8);
    uint32_t *clen = malloc((size_t)nrec * 4);
    int32_t *cid = malloc((size_t)nrec * 4);
    pthread_t th[64];
    gen_t g[64];
    chk_t ck[64];
    uint64_t total_pcs = 0;
    uint32_t *pcs = NULL;
    size_t pcap = 0;
    for (uint32_t b = 0; b < nb; b++) {
        const uint64_t first = (uint64_t)b * nrec;
        off[0] = 0;
        for (uint32_t k = 0; k < nrec; k++)
            off[k + 1] = off[k] + orc_synth_len(seed, first + k, mean, sigma);
        if (off[nrec] > pcap) {
            pcap = off[nrec];
            free(pcs);
            pcs = malloc(pcap * 4);
        }
        for (uint32_t t = 0; t < nt; t++) {
            g[t] = (gen_t){seed, first, nrec, mean, sigma, log2, off, pcs, clen, t, nt};
            pthread_create(&th[t], NULL, gen_recs, &g[t]);
        }
        for (uint32_t t = 0; t < nt; t++) pthread_join(th[t], NULL);
        for (uint32_t k = 0; k < nrec; k++) cid[k] = orc_synth_callid(seed, first + k, ncalls);
        for (uint32_t t = 0; t < nt; t++) {
            ck[t] = (chk_t){off, clen, pcs, cid, nrec, mc, fl, is_new + (size_t)b * nrec, t, nt};
            pthread_create(&th[t], NULL, check, &ck[t]);
        }
        for (uint32_t t = 0; t < nt; t++) pthread_join(th[t], NULL);
        for (uint32_t k = 0; k < nrec; k++) total_pcs += clen[k];
    }
    /* maxCover read back as sorted PC lists */
    uint32_t *mn = calloc(ncalls, 4);
    FILE *f;
    char path[4096];
    snprintf(path, sizeof path, "%s/maxcover.u32", dir);
    f = fopen(path, "wb");
    if (!f) return 1;
    uint64_t mtot = 0, nnew = 0;
    uint32_t *row = malloc(64 * 4);
    for (uint32_t c = 0; c < ncalls; c++) {
        for (uint64_t w = 0; w < words; w++) {
            uint64_t x = mc[c][w];
            uint32_t r = 0;
            while (x) {
                int bi = __builtin_ctzll(x);
                row[r++] = PC_LO + (uint32_t)(w * 64 + bi);
                x &= x - 1;
            }
            if (r) fwrite(row, 4, r, f);
            mn[c] += r;
        }
        mtot += mn[c];
    }
    fclose(f);
    for (size_t i = 0; i < (size_t)nb * nrec; i++) nnew += is_new[i];
    if (write_file(dir, "is_new.u8", is_new, (size_t)nb * nrec) ||
        write_file(dir, "maxcover_n.u32", mn, (size_t)ncalls * 4))
        return 1;
    printf("{\"record_pcs\": %llu, \"new_records\": %llu, \"max_cover_total\": %llu}\n",
           (unsigned long long)total_pcs, (unsigned long long)nnew, (unsigned long long)mtot);
    return 0;
}
