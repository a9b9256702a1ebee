/*
 * prio_oracle.c — literal restatement of prog/prio.go (dynamic part,
 * normalisation, combine, choice table).  float32 arithmetic, one rounding
 * per Go operation: compiled with -ffp-contract=off and float literals.
 * Parity UNPINNED: the reference has no test covering prio.go.
 * TEST INFRASTRUCTURE ONLY.
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

/* prog/prio.go:137-151 (before the normalizePrio call at :152). */
int orc_dynamic_raw(const int32_t *prog_len, size_t nprog, int C, float *prios) {
    memset(prios, 0, (size_t)C * (size_t)C * sizeof(float));
    for (size_t p = 0; p < nprog; p++) {
        int n = prog_len[p];
        if (n > C) return -1; /* prios[i0] index out of range: Go panics */
        for (int i0 = 0; i0 < n; i0++)
            for (int i1 = 0; i1 < n; i1++) {
                if (i0 == i1) continue;
                prios[(size_t)i0 * C + i1] += 1.0f;
            }
    }
    return 0;
}

/* prog/prio.go:158-192 */
void orc_normalize_prio(float *prios, int C) {
    for (int r = 0; r < C; r++) {
        float *prio = prios + (size_t)r * C;
        float max = 0.0f;
        float min = 1e10f;
        int nzero = 0;
        for (int i = 0; i < C; i++) {
            float p = prio[i];
            if (max < p) max = p;
            if (p != 0 && min > p) min = p;
            if (p == 0) nzero++;
        }
        if (nzero != 0) min /= 2.0f * (float)nzero;
        for (int i = 0; i < C; i++) {
            float p = prio[i];
            if (max == 0) {
                prio[i] = 1.0f;
                continue;
            }
            if (p == 0) p = min;
            float num = p - min;
            float den = max - min;
            float q = num / den;
            q = q * 0.9f;
            p = q + 0.1f;
            if (p > 1) p = 1.0f;
            prio[i] = p;
        }
    }
}

/* prog/prio.go:29-38 with the static matrix supplied by the caller. */
int orc_calculate_priorities(const int32_t *prog_len, size_t nprog, int C,
                             const float *static_prios, float *out) {
    if (orc_dynamic_raw(prog_len, nprog, C, out) != 0) return -1;
    orc_normalize_prio(out, C);
    for (size_t i = 0; i < (size_t)C * C; i++) out[i] *= static_prios[i];
    return 0;
}

/* prog/prio.go:106-133 over a usage table (id -> (call, weight) pairs, ids in
 * the order given; Go walks its `uses` map in random order, this restatement
 * fixes ascending id order). */
void orc_static_prio(const uint32_t *id_off, const uint16_t *id_calls, const float *id_w,
                     size_t nids, int C, float *prios) {
    memset(prios, 0, (size_t)C * (size_t)C * sizeof(float));
    for (size_t k = 0; k < nids; k++) /* for _, calls := range uses */
        for (uint32_t a = id_off[k]; a < id_off[k + 1]; a++)     /* c0, w0 */
            for (uint32_t b = id_off[k]; b < id_off[k + 1]; b++) { /* c1, w1 */
                int c0 = id_calls[a], c1 = id_calls[b];
                if (c0 == c1) continue;
                float prod = id_w[a] * id_w[b];
                prios[(size_t)c0 * C + c1] += prod;
            }
    for (int c0 = 0; c0 < C; c0++) { /* :124-132 */
        float max = 0;
        for (int j = 0; j < C; j++)
            if (max < prios[(size_t)c0 * C + j]) max = prios[(size_t)c0 * C + j];
        prios[(size_t)c0 * C + c0] = max;
    }
    orc_normalize_prio(prios, C); /* :133 */
}

/* prog/prio.go:202-228 */
void orc_build_choice_table(const float *prios, const uint8_t *enabled, int C, int64_t *run) {
    for (int i = 0; i < C; i++) {
        if (!enabled[i]) continue;
        int64_t sum = 0;
        for (int j = 0; j < C; j++) {
            if (enabled[j]) {
                float x = prios[(size_t)i * C + j] * 1000.0f;
                sum += (int64_t)x; /* Go int(): truncation toward zero */
            }
            run[(size_t)i * C + j] = sum;
        }
    }
}
