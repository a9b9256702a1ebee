/*
 * grouped_full.c — full-size CPU oracle of Manager.minimizeCorpus
 * (syz-manager/manager.go:504-524) over a synthetic corpus of RAW covers (as a
 * manager holds them; duplicates count in len(cov), cover.go:142).
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h): run once in the build container by
 * tools/gen_golden_fullsize.py; the GPU tests and the bench compare
 * syzcov_minimize_corpus against its digests.
 *
 *   groups  the inputs grouped by call (synthetic call ids, orc_synth_callid),
 *           corpus order inside a group (manager.go:511-516); the groups are
 *           emitted in ascending call id (the reference's Go map order is
 *           random, so every group order is one it can produce)
 *   order   per group, Go sort.Sort(minInputArray) over the raw lengths
 *           (cover.go:113; orc_sort_min_inputs, pdqsort)
 *   scan    per group, the reference's loop (cover.go:115-129) over a
 *           covered bitmap of the corpus' PC window, cleared per group
 * The raw covers are regenerated per input (the corpus is never held).
 *
 * Usage: grouped_full SEED N MEAN SIGMA LOG2 NCALLS OUTFILE
 * Writes the kept corpus indices (int32) to OUTFILE and prints a summary.
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define PC_LO 0x81000000u /* the synthetic universe's window (synth_oracle.c) */

int main(int argc, char **argv) {
    if (argc != 8) {
        fprintf(stderr, "usage: %s SEED N MEAN SIGMA LOG2 NCALLS OUTFILE\n", argv[0]);
        return 2;
    }
    const uint64_t seed = strtoull(argv[1], 0, 0), n = strtoull(argv[2], 0, 0);
    const uint32_t mean = (uint32_t)strtoul(argv[3], 0, 0), sigma = (uint32_t)strtoul(argv[4], 0, 0);
    const uint32_t log2 = (uint32_t)strtoul(argv[5], 0, 0), ncalls = (uint32_t)strtoul(argv[6], 0, 0);
    const uint64_t span = 16ull << log2; /* U[k] = PC_LO + 16k + (h & 15) */
    /* groups by call id, corpus order inside (a counting sort is stable) */
    uint64_t *cnt = calloc(ncalls + 1, 8);
    int32_t *call = malloc(n * 4);
    for (uint64_t i = 0; i < n; i++) {
        call[i] = orc_synth_callid(seed, i, ncalls);
        cnt[call[i] + 1]++;
    }
    for (uint32_t g = 0; g < ncalls; g++) cnt[g + 1] += cnt[g];
    int32_t *grp = malloc(n * 4);
    uint64_t *cur = malloc(ncalls * 8);
    memcpy(cur, cnt, ncalls * 8);
    for (uint64_t i = 0; i < n; i++) grp[cur[call[i]]++] = (int32_t)i;
    uint64_t *covered = malloc(span / 8);
    uint32_t *buf = malloc(65536 * 4);
    int32_t *kept = malloc(n * 4), *ord = malloc(n * 4);
    int64_t *len = malloc(n * 8);
    uint64_t nkept = 0, raw = 0;
    for (uint32_t g = 0; g < ncalls; g++) {
        const uint64_t a = cnt[g], m = cnt[g + 1] - a;
        if (!m) continue;
        for (uint64_t j = 0; j < m; j++) {
            ord[j] = (int32_t)j;
            len[j] = orc_synth_len(seed, (uint64_t)grp[a + j], mean, sigma);
        }
        orc_sort_min_inputs(ord, len, m, 0);
        memset(covered, 0, span / 8);
        for (uint64_t r = 0; r < m; r++) {
            const int32_t idx = grp[a + ord[r]];
            const uint32_t L = (uint32_t)len[ord[r]];
            orc_synth_input(seed, (uint64_t)idx, L, log2, 0, buf);
            raw += L;
            int hit = 0;
            for (uint32_t q = 0; q < L; q++) {
                const uint64_t o = (uint64_t)(buf[q] - PC_LO);
                if (o >= span) {
                    fprintf(stderr, "PC %#x outside the window\n", buf[q]);
                    return 1;
                }
                const uint64_t bit = 1ull << (o & 63);
                uint64_t *w = &covered[o >> 6];
                if (!hit && !(*w & bit)) {
                    hit = 1;
                    kept[nkept++] = idx;
                }
                if (hit) *w |= bit;
            }
        }
    }
    FILE *f = fopen(argv[7], "wb");
    if (!f || (nkept && fwrite(kept, 4, nkept, f) != nkept)) {
        fprintf(stderr, "write failed\n");
        return 1;
    }
    fclose(f);
    printf("{\"n\": %llu, \"raw_pcs\": %llu, \"groups\": %u, \"n_kept\": %llu}\n",
           (unsigned long long)n, (unsigned long long)raw, ncalls, (unsigned long long)nkept);
    return 0;
}
