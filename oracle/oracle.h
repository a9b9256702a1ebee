/*
 * oracle.h — CPU restatement of the reference coverage hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in syzkaller_amd/ may include, link or
 * call this code; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker / CPU baseline.
 *
 * Every function restates, literally and sequentially, the Go code it cites:
 *   cover/cover.go          (Canonicalize, foreach-based set ops, Minimize)
 *   Go stdlib sort.Sort     (pdqsort, Go >= 1.19; legacy quickSort, Go 1.8-1.18)
 *   prog/prio.go            (calcDynamicPrio, normalizePrio, CalculatePriorities
 *                            combine step, BuildChoiceTable)
 *
 * Parity pinning: the cover functions are pinned by every known-answer table in
 * cover/cover_test.go:60-168 (transcribed in tests/golden/cover_kat.json).
 * Priorities are "parity unpinned": the reference has no test for prio.go.
 */
#ifndef SYZCOV_ORACLE_H
#define SYZCOV_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* cover/cover.go:28-40 — in place; returns the new length. */
size_t orc_canonicalize(uint32_t *cov, size_t n);

/* executor/executor.cc:574-587 cover_dedup — in place; returns the new
 * length (sorted, distinct, nonzero: `last` starts at 0). */
size_t orc_cover_dedup64(uint64_t *cov, size_t n);

/* cover/cover.go:42-102.  op: 0 Difference, 1 SymmetricDifference, 2 Union,
 * 3 Intersection.  out must hold na+nb.  Returns result length. */
size_t orc_setop(int op, const uint32_t *a, size_t na, const uint32_t *b, size_t nb,
                 uint32_t *out);

/* Go sort.Sort over minInputArray (cover/cover.go:133-143): sorts idx[] by
 * len[idx] descending.  variant 0 = pdqsort (Go >= 1.19), 1 = legacy. */
void orc_sort_min_inputs(int32_t *idx, const int64_t *len, size_t n, int variant);

/* cover/cover.go:104-131.  Corpus in CSR form (offsets[n+1], pcs).
 * out_idx must hold n entries; returns the number kept. */
size_t orc_minimize(const uint64_t *offsets, const uint32_t *pcs, size_t n, int variant,
                    int32_t *out_idx);

/* Union fold `total = Union(total, cov_i)` over a CSR corpus (the caller
 * pattern of manager.go:610, html.go:72-79, cover_test.go:182-185).
 * out must hold the total PC count; returns |union|. */
size_t orc_union_fold(const uint64_t *offsets, const uint32_t *pcs, size_t n, uint32_t *out);

/* syz-fuzzer/fuzzer.go:456-480 executed sequentially over a batch of call
 * records.  maxcover is a CSR of ncalls sorted lists (input), flakes a sorted
 * list.  is_new[k] = 1 iff record k produced a non-empty diff.  The updated
 * maxCover is returned in CSR form through new_off/new_pcs (caller sizes
 * new_pcs to |maxcover| + total record PCs). */
void orc_newcov_batch(const uint64_t *mc_off, const uint32_t *mc_pcs, int ncalls,
                      const uint32_t *flakes, size_t nflakes,
                      const int32_t *callid, const uint64_t *rec_off,
                      const uint32_t *rec_pcs, size_t nrec, uint8_t *is_new,
                      uint64_t *new_off, uint32_t *new_pcs);

/* prog/prio.go:137-154 raw counts (before normalizePrio), positional: for
 * every program p, prios[i0][i1] += 1 for i0 != i1 < len(p).  Row-major C*C
 * float32.  Returns -1 if some program is longer than C (Go would panic). */
int orc_dynamic_raw(const int32_t *prog_len, size_t nprog, int C, float *prios);

/* prog/prio.go:158-192, in place, row-major C*C float32. */
void orc_normalize_prio(float *prios, int C);

/* prog/prio.go:29-38 given a static matrix: dynamic = normalize(raw dynamic);
 * dynamic[i][j] *= static[i][j]. */
int orc_calculate_priorities(const int32_t *prog_len, size_t nprog, int C,
                             const float *static_prios, float *out);

/* prog/prio.go:106-133 (calcStaticPriorities' accumulation, diagonal and
 * normalisation) over a usage table in CSR form, ids in ascending order. */
void orc_static_prio(const uint32_t *id_off, const uint16_t *id_calls, const float *id_w,
                     size_t nids, int C, float *prios);

/* prog/prio.go:202-228.  enabled[C] (0/1); run must hold C*C int64; rows of
 * disabled calls are left untouched (nil in Go) — the caller pre-fills them. */
void orc_build_choice_table(const float *prios, const uint8_t *enabled, int C, int64_t *run);

/* Synthetic corpus generator (integer-exact variant; see
 * syzkaller_amd/csrc/synth.hip for the device twin). */
uint32_t orc_synth_len(uint64_t seed, uint64_t input, uint32_t mean, uint32_t sigma);
/* mode bit 0: uniform key draws; bit 1: the x86-like universe (5..14-byte gaps) */
void orc_synth_input(uint64_t seed, uint64_t input, uint32_t len, uint32_t log2_space,
                     int mode, uint32_t *out);
uint32_t orc_synth_universe(uint64_t seed, uint32_t k);
uint32_t orc_synth_universe_mode(uint64_t seed, uint32_t k, int mode);
int32_t orc_synth_callid(uint64_t seed, uint64_t input, uint32_t ncalls);

#ifdef __cplusplus
}
#endif
#endif
