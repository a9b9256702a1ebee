/*
 * syzcov.h — C-ABI of the MI355X coverage-analysis engine (libsyzcov.so).
 *
 * Plain pointers and sizes only; no torch or HIP types in any signature
 * (streams and device pointers travel as void* / uint64_t).  Two tiers:
 *
 *  1. Drop-in host API.  Exactly what syzkaller's Go packages would bind over
 *     cgo to replace the pure-Go hot path (INTEGRATION.md shows the shim).
 *     Host buffers in, host buffers out; every call computes on the GPU
 *     (no CPU fallback: with no usable HIP device a call returns
 *     SYZCOV_ENODEV).  Reentrant: each host thread gets its own HIP stream
 *     and scratch, so the fuzzer's <=32 goroutines may call concurrently
 *     (syz-fuzzer/fuzzer.go:166, config/config.go:150).
 *
 *  2. Device-resident launch API (syzcov_dev_*).  Device pointers plus a HIP
 *     stream; no host synchronisation, no allocation (caller-provided
 *     workspace), so the calls can be captured into a hipGraph.  This is what
 *     the corpus engine, bench.py and the multi-GPU path drive.
 *
 * Semantics follow the Go reference bit-for-bit (cover/cover.go, prog/prio.go)
 * for the input domain the reference's callers produce.  Where the reference
 * has undefined-looking behaviour the engine is explicit:
 *   - set ops require each operand sorted non-decreasing (duplicates allowed:
 *     they get foreach's multiset behaviour); unsorted operands -> SYZCOV_ENOTSORTED
 *     (no reference caller passes one: SURVEY §7(d));
 *   - 0xFFFFFFFF is dropped from set-op results (cover.go:17,97) and is an
 *     ordinary PC for Minimize (cover.go:116-129);
 *   - Canonicalize drops a 0xFFFFFFFF only when it is the sole distinct value
 *     (cover.go:30 `last := sent`).
 *
 * Return codes: >= 0 success (a count where documented), < 0 error.
 */
#ifndef SYZCOV_H
#define SYZCOV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SYZCOV_OK 0
#define SYZCOV_EINVAL -1      /* bad arguments */
#define SYZCOV_ENOTSORTED -2  /* set-op operand not sorted */
#define SYZCOV_ENODEV -3      /* no HIP device */
#define SYZCOV_EHIP -4        /* HIP runtime error */
#define SYZCOV_ERANGE -5      /* a PC outside the configured PC window */
#define SYZCOV_ENOMEM -6      /* device allocation failed */
#define SYZCOV_ETOOLONG -7    /* program longer than the call table (Go would panic) */

/* bits of a device err_flag word (engine kernels) */
#define SYZCOV_ERR_WINDOW 1u  /* a PC outside the configured PC window */
#define SYZCOV_ERR_SEGLEN 2u  /* a segment longer than the declared max_seg_len */
#define SYZCOV_ERR_UNIVERSE 4u /* key mode: a PC that is not in the registered universe */
#define SYZCOV_ERR_ORDER 8u   /* a caller order entry outside [0, N) */
/* Key mode: the key shift is capped so a universe PC's low kshift bits fit
 * one byte of the membership table with bit 7 free and 0x7F left for "no
 * universe PC", and a canonical key word (key | low << 26) fits 32 bits. */
#define SYZCOV_KSHIFT_MAX 6u

/* Version / build identification: "syzcov <ver> gfx950". */
const char *syzcov_version(void);
/* Human-readable text for the last error on this thread. */
const char *syzcov_last_error(void);
/* Device contexts (stream + arenas) the pool holds on `device`: calls lease
 * one for their duration, so this is the peak number of concurrent callers
 * since the last trim, independent of how many OS threads ever called in. */
int64_t syzcov_pool_contexts(int device);
/* Destroy every idle pooled context: its arenas (a call keeps up to 3 x 32 MB
 * between calls; larger ones are freed as it returns) and its stream.  Later
 * calls create contexts again as needed. */
int syzcov_pool_trim(void);

/* ======================= 1. drop-in host API ========================= */

/* cover.RestorePC (cover/cover.go:23-25). */
uint64_t syzcov_restore_pc(uint32_t pc, uint32_t base);

/* cover.Canonicalize (cover/cover.go:27-40): sorts and de-duplicates cov IN
 * PLACE and returns the new length n' (the Go shim returns cov[:n'], keeping
 * the reference's aliasing, html.go:236). */
int64_t syzcov_canonicalize(uint32_t *cov, size_t n);

/* The executor's cover_dedup (executor/executor.cc:574-587) of one raw u64
 * KCOV buffer: sorts cov IN PLACE, keeps the distinct nonzero PCs (the
 * reference's `last` starts at 0) at the front and returns their count.
 * n <= 2^31, else SYZCOV_ETOOLONG. */
int64_t syzcov_cover_dedup64(uint64_t *cov, size_t n);

/* cover.Difference / SymmetricDifference / Union / Intersection
 * (cover/cover.go:42-79, merge core foreach :81-102).  `out` must hold
 * na (Difference), na+nb (SymmetricDifference, Union), min(na,nb)
 * (Intersection) entries.  Returns the result length (the shim returns nil
 * for 0, matching foreach's nil result). */
int64_t syzcov_difference(const uint32_t *a, size_t na, const uint32_t *b, size_t nb,
                          uint32_t *out);
int64_t syzcov_symmetric_difference(const uint32_t *a, size_t na, const uint32_t *b, size_t nb,
                                    uint32_t *out);
int64_t syzcov_union(const uint32_t *a, size_t na, const uint32_t *b, size_t nb, uint32_t *out);
int64_t syzcov_intersection(const uint32_t *a, size_t na, const uint32_t *b, size_t nb,
                            uint32_t *out);

/* cover.Minimize (cover/cover.go:104-131).  The corpus is CSR:
 * cover i = pcs[offsets[i] .. offsets[i+1]).  `order` (nullable) is the
 * processing order — order[r] = index of the r-th input after Go's
 * sort.Sort(minInputArray) (cover.go:113).  The Go shim passes the order its
 * own sort.Sort produced (exact by construction); NULL makes the engine
 * compute it on the GPU with its restatement of Go >= 1.19 pdqsort
 * (sort_variant must be 0; for Go 1.8-1.18's quickSort order the caller passes
 * `order`: the library has no host sort).  Writes the kept input indices
 * in processing order to out_idx (capacity n) and returns their count. */
int64_t syzcov_minimize(const uint64_t *offsets, const uint32_t *pcs, size_t n,
                        const int32_t *order, int sort_variant, int32_t *out_idx);

/* Manager.minimizeCorpus (syz-manager/manager.go:504-524): the corpus is
 * grouped by call (call[i] = any int32 key of RpcInput.Call; corpus order is
 * kept inside a group, :511-516) and cover.Minimize runs on every group
 * (:519-523), each with its own Go sort.Sort order (Go >= 1.19 pdqsort;
 * sort_variant must be 0).  out_idx (capacity n)
 * receives the kept CORPUS indices, groups in ascending call value, each
 * group in its Minimize output order; returns their count.  The reference
 * concatenates groups in Go map order (random), so the shim may reorder
 * whole groups freely. */
int64_t syzcov_minimize_corpus(const int32_t *call, const uint64_t *offsets, const uint32_t *pcs,
                               size_t n, int sort_variant, int32_t *out_idx);

/* What the calling thread's last syzcov_minimize_corpus did: the path it took
 * and, on the two corpus-size paths, where its time went (HIP events on its
 * stream): host -> device staging, the device work between the last upload
 * and the kept list's download (two canonicalizations, the Go orders and the
 * grouped Minimize, host syncs included), and the download. */
#define SYZCOV_GROUPS_PATH_NONE 0   /* no call yet, or it failed */
#define SYZCOV_GROUPS_PATH_LDS 1    /* every group <= 2^16 inputs: one LDS pass (group_min) */
#define SYZCOV_GROUPS_PATH_ENGINE 2 /* the per-group engine on the cached handle */
#define SYZCOV_GROUPS_PATH_SLABS 3  /* < 65,536 inputs (or no engine): per-group slabs */
typedef struct syzcov_groups_stats {
    int32_t path;        /* SYZCOV_GROUPS_PATH_* */
    float upload_ms;     /* corpus paths: offsets, PCs, grouping, lengths to the device */
    float device_ms;     /* corpus paths: the device part of the call */
    float download_ms;   /* corpus paths: the kept indices back */
} syzcov_groups_stats;
int syzcov_minimize_corpus_stats(syzcov_groups_stats *out);

/* Go sort.Sort(minInputArray) restatement: order[r] for inputs of the given
 * lengths (len(cov) including duplicates).  Computed on the GPU. */
int syzcov_sort_order(const int64_t *lens, size_t n, int sort_variant, int32_t *order);

/* Union of a whole corpus (the `total = Union(total, cov)` fold of
 * manager.go:610 / html.go:72-79 / cover_test.go:182-185) in one pass.
 * out must hold the total PC count; returns |union|. */
int64_t syzcov_union_all(const uint64_t *offsets, const uint32_t *pcs, size_t n, uint32_t *out);

/* Manager.uniqueCover (syz-manager/html.go:213-238): the sorted PCs counted
 * exactly once over the corpus.  call == NULL is uniqueCover(false): every
 * occurrence counts, duplicates inside a cover included.  call != NULL
 * (one int32 key per input, INT32_MIN reserved) is uniqueCover(true): a PC
 * counts once per call group, so it is unique iff one group holds it.
 * out capacity: the corpus' distinct PC count (<= total PCs).  Returns the
 * count.  UI callers: httpSummary (:86-95), httpCorpus (:155-169), httpCover
 * (:203-205) intersect per-call or per-input covers with it. */
int64_t syzcov_unique_cover(const int32_t *call, const uint64_t *offsets, const uint32_t *pcs,
                            size_t n, uint32_t *out);

/* Manager UI statistics over a corpus of CANONICAL covers (the manager's
 * corpus holds canonical covers; anything else -> SYZCOV_ENOTSORTED).
 * Replaces the Union fold and Intersection calls of httpSummary
 * (syz-manager/html.go:67-99) and httpCorpus (:157-175).  call[i] is input
 * i's call group in [0, ncalls) (RpcInput.Call numbered by the caller).
 * Per group g (each output nullable, all need call):
 *   inputs[g]       = CallCov.count                              (:74-75)
 *   cover[g]        = len(CallCov.cov), the Union fold            (:76)
 *   unique_cover[g] = len(Intersection(cov, uniqueCover(true)))  (:86-90)
 * Per input i (nullable; call may be NULL):
 *   input_unique[i] = len(Intersection(inp.Cover, uniqueCover(false))) (:160-168)
 * Returns len(Union of all covers), the "cover" stat (:92-97); the sentinel
 * 0xFFFFFFFF is never counted, as Union/Intersection drop it. */
int64_t syzcov_ui_stats(const int32_t *call, const uint64_t *offsets, const uint32_t *pcs,
                        size_t n, uint32_t ncalls, uint32_t *inputs, uint32_t *cover,
                        uint32_t *unique_cover, uint32_t *input_unique);

/* prog.CalculatePriorities (prog/prio.go:29-38) given the static matrix
 * (calcStaticPriorities, :40-135, stays with the caller: it depends only on
 * sys.Calls).  key_mode 0 = positional, exactly the reference's
 * calcDynamicPrio (:137-154, which indexes by call position); key_mode 1 =
 * by syscall id.  prog_off/call_ids describe programs in CSR form (ids are
 * only read in key_mode 1; in mode 0 only the lengths matter).  static_prios
 * and out are row-major C*C float32.  raw_counts (nullable, C*C uint32)
 * receives the exact co-occurrence counts before normalisation. */
int syzcov_calculate_priorities(const uint64_t *prog_off, const uint16_t *call_ids,
                                size_t nprog, int C, int key_mode, const float *static_prios,
                                float *out, uint32_t *raw_counts);

/* prog.calcStaticPriorities (prog/prio.go:40-135) from the syscall usage
 * table (usage id -> (call, weight) pairs, as noteUsage builds it, :42-104),
 * in two CSR views: by id (id_off[nids+1], id_calls, id_w) and by call
 * (call_off[C+1], call_ids = usage-id indices ascending, call_w = the call's
 * weight in that id).  out: C*C float32, normalised (:133).  The reference
 * sums in Go map order; the engine uses ascending id order. */
int syzcov_static_priorities(const uint32_t *id_off, const uint16_t *id_calls, const float *id_w,
                             size_t nids, const uint32_t *call_off, const uint32_t *call_ids,
                             const float *call_w, int C, float *out);
int syzcov_dev_static_prio(const uint32_t *id_off, const uint16_t *id_calls, const float *id_w,
                           const uint32_t *call_off, const uint32_t *call_ids,
                           const float *call_w, int C, float *out, void *stream);

/* prog.normalizePrio (prog/prio.go:158-192), in place, C*C float32. */
int syzcov_normalize_prio(float *prios, int C);

/* prog.BuildChoiceTable (prog/prio.go:202-228): run[i][j] for enabled rows
 * (int64, C*C); rows of disabled calls are left untouched (nil in Go).
 * enabled == NULL enables every call (prio.go:203-208). */
int syzcov_build_choice_table(const float *prios, const uint8_t *enabled, int C, int64_t *run);

/* ChoiceTable.Choose (prog/prio.go:230-249) for nq (call, x) pairs, where
 * x[k] is the caller's r.Intn(run[call][C-1]) draw (math/rand stays with the
 * caller).  out[k] = sort.SearchInts(run[call], x) if that call is enabled;
 * -1 if not (Choose draws again); -2 for call < 0 or a disabled call's nil
 * row (Choose picks uniformly from enabledCalls).  run/enabled as produced
 * for syzcov_build_choice_table (enabled == NULL: all).  A call >= C or an x
 * outside [0, run[call][C-1]) -> SYZCOV_ERANGE. */
int syzcov_choose_batch(const int64_t *run, const uint8_t *enabled, int C, const int32_t *calls,
                        const int64_t *x, size_t nq, int32_t *out);

/* Streaming new-coverage check of syz-fuzzer execute() (fuzzer.go:456-480)
 * against resident state.  A handle holds per-CallID maxCover and the global
 * flakes set as device bitmaps over a PC window [pc_lo, pc_lo + pc_span). */
typedef uint64_t syzcov_cover_state;
int syzcov_state_create(int ncalls, uint32_t pc_lo, uint64_t pc_span, syzcov_cover_state *out);
int syzcov_state_destroy(syzcov_cover_state st);
/* maxCover[call] = Union(maxCover[call], pcs) (sorted list). */
int syzcov_state_add(syzcov_cover_state st, int call, const uint32_t *pcs, size_t n);
int syzcov_state_set_flakes(syzcov_cover_state st, const uint32_t *pcs, size_t n);
/* Optional, before the first add/newcov: the PC universe = every PC KCOV can
 * report, i.e. the RETURN address of each `call __sanitizer_cov_trace_pc`
 * (the call sites of allCoverPCs, syz-manager/cover.go:274-306, plus the
 * call's length: KCOV records return addresses, which is why cover.go:82
 * subtracts 1), truncated to u32.  maxCover, corpusCover and flakes are then
 * kept over the universe's dense keys (keys.hip).  Every PC passed in from
 * then on is checked against the universe: one that is not in it fails the
 * call (SYZCOV_ERANGE; a newcov/triage batch is rejected whole) instead of
 * sharing a key with a universe PC, so results are the reference's or an
 * error, never different ones. */
int syzcov_state_set_universe(syzcov_cover_state st, const uint32_t *pcs, size_t n);
/* Reads maxCover[call] back as a sorted list (out capacity: pc_span or the
 * count from a NULL-out call); returns its length. */
int64_t syzcov_state_get(syzcov_cover_state st, int call, uint32_t *out, size_t cap);
/* One batch of executed call records in batch order (record k: call id
 * callid[k], sorted cover rec_pcs[rec_off[k] .. rec_off[k+1])).  Sets
 * is_new[k] exactly as the sequential reference loop would, and updates
 * maxCover as it would.  Returns the number of new records. */
int64_t syzcov_newcov_batch(syzcov_cover_state st, const int32_t *callid, const uint64_t *rec_off,
                            const uint32_t *rec_pcs, size_t nrec, uint8_t *is_new);

/* Device-resident form of syzcov_newcov_batch for batches already in HBM
 * (callid, rec_off, pcs, is_new are device pointers; rec_off[0] == 0 and
 * rec_off[nrec] == npc, the host-side total that sizes the workspace).  Launches
 * asynchronously on `stream`; stats (device u32[2], nullable) receives
 * [0] error (1 PC outside the window, 2 call id out of range, 3 unsorted
 * record: the batch then changes nothing) and [1] the candidates left after
 * the maxCover/flakes bitmap filter. */
size_t syzcov_state_newcov_ws_size(size_t nrec, uint64_t npc);
int syzcov_state_newcov_dev(syzcov_cover_state st, const int32_t *callid, const uint64_t *rec_off,
                            const uint32_t *pcs, size_t nrec, uint64_t npc, uint8_t *is_new,
                            uint32_t *stats, void *ws, size_t ws_size, void *stream);

/* corpusCover (syz-fuzzer/fuzzer.go:62-89), held by the same handle over the
 * same index space as maxCover and flakes.  corpus_add: corpusCover[call] =
 * Union(corpusCover[call], pcs) (fuzzer.go:451, after the caller's
 * prog.Minimize); corpus_get reads it back like syzcov_state_get. */
int syzcov_state_corpus_add(syzcov_cover_state st, int call, const uint32_t *pcs, size_t n);
int64_t syzcov_state_corpus_get(syzcov_cover_state st, int call, uint32_t *out, size_t cap);
/* Reads the flakes set back (sorted), like syzcov_state_get. */
int64_t syzcov_state_flakes_get(syzcov_cover_state st, uint32_t *out, size_t cap);
/* addInput (fuzzer.go:344-375) for a batch of manager-pushed inputs in
 * order (record k: call id, sorted cover as in syzcov_newcov_batch; the
 * caller has run Canonicalize, :365, and the corpusHashes check, :361-364):
 * accepted[k] iff Difference(Difference(cov, maxCover), flakes) != ∅ at its
 * turn; an accepted input's whole cover joins corpusCover and maxCover
 * (:372-373).  Returns the number accepted. */
int64_t syzcov_state_add_inputs(syzcov_cover_state st, const int32_t *callid,
                                const uint64_t *rec_off, const uint32_t *rec_pcs, size_t nrec,
                                uint8_t *accepted);
/* triageInput (fuzzer.go:377-417) for ntri inputs.  Input t: call id
 * callid[t], sorted cover cov_pcs[cov_off[t] .. cov_off[t+1]); its three
 * re-executions are runs 3t, 3t+1, 3t+2 of run_off/run_pcs (sorted; an empty
 * run is a call that did not execute, :401-404).  Schedule: every input's
 * newCover = Difference(Difference(cov, corpusCover[call]), flakes) (:384-385)
 * is taken before any flakes update (one interleaving of the reference's
 * concurrent triage goroutines); then each input with a non-empty newCover
 * runs its loop: minCover = Intersection(minCover, run), flakes =
 * Union(flakes, SymmetricDifference(cov, run)) (:405-415).  Outputs
 * new_cnt[t] = len(newCover) and stableNewCover = Intersection(newCover,
 * minCover) (:417) at stable_pcs[cov_off[t] ..] (stable_cnt[t] PCs; capacity
 * = the cover CSR).  flakes is updated in the handle.  Returns the number
 * of inputs with a non-empty stableNewCover (those go on to prog.Minimize). */
int64_t syzcov_state_triage(syzcov_cover_state st, size_t ntri, const int32_t *callid,
                            const uint64_t *cov_off, const uint32_t *cov_pcs,
                            const uint64_t *run_off, const uint32_t *run_pcs, uint32_t *new_cnt,
                            uint32_t *stable_cnt, uint32_t *stable_pcs);

/* Executor output of one program (writer executor/executor.cc:455-466,
 * reader ipc/ipc.go:225-291: u32 ncmd, then per completed call u32
 * call_index, call_num, errno, cover_size, pcs[cover_size], little-endian)
 * -> the records syz-fuzzer execute() checks (fuzzer.go:456-460): calls in
 * index order, empty covers skipped.  call_num[i] = p.Calls[i].Meta.ID (the
 * reader's consistency check), callid_of_num[num] = sys.Calls[num].CallID.
 * Writes errnos[ncalls] (int64: -1 = not executed, else the u32 value) and, per record, rec_callid,
 * rec_call_index and CSR rec_off[nrec+1] / rec_pcs (capacity pcs_cap).
 * Returns nrec; a malformed buffer (the reader's error cases) returns < 0.
 * Host only: append programs and hand the batch to syzcov_newcov_batch. */
int64_t syzcov_parse_exec_output(const uint8_t *out, size_t out_len, size_t ncalls,
                                 const uint32_t *call_num, const int32_t *callid_of_num,
                                 size_t nnum, int64_t *errnos, int32_t *rec_callid,
                                 uint32_t *rec_call_index, uint64_t *rec_off, uint32_t *rec_pcs,
                                 size_t pcs_cap);

/* ================ resident corpus engine (corpus.hip) ==================
 * The manager-side corpus path the benchmark measures (BASELINE configs C2 /
 * C3), one handle per GPU: Canonicalize every input (cover/cover.go:27-40),
 * Go's sort.Sort(minInputArray) order (cover.go:113), first-cover Minimize
 * (cover.go:104-131), the kept list, the sorted union (the `Union(total, cov)`
 * fold, syz-manager/manager.go:606-610) and the resident maxCover |= union.
 * Replaces cover.Minimize + the union fold for Manager.minimizeCorpus-sized
 * corpora (manager.go:504-550); syzcov_minimize routes large corpora here.
 *
 * Modes: with `universe` (the sorted, unique PCs KCOV can report: the return
 * addresses of the __sanitizer_cov_trace_pc calls, syz-manager/cover.go:82,
 * 274-306, truncated to u32) every phase works on dense keys (keys.hip) and a
 * PC outside the universe fails the step (SYZCOV_ERANGE), never aliases;
 * without it, on PC offsets of [pc_lo, pc_lo + pc_span) (<= 2^28 PCs).
 *
 * Memory: one device block of syzcov_corpus_mem_size(cfg) bytes, laid out
 * as syzcov_corpus_buffer reports; the caller may pass its own (256-byte
 * aligned) or let the handle allocate.  Phase calls are asynchronous on the
 * caller's stream; a handle serves one step at a time (calls on one handle
 * are serialized by its lock, but two streams must not interleave steps).
 *
 * Sharded by input over `world` GPUs (n_global > n_max; rank r holds global
 * inputs [r * n_max, r * n_max + n)), the caller runs the collectives
 * between the phases (syzkaller_amd/dist.py does it over RCCL):
 *   canon -> all-gather NEW_LEN[:n] into GLENS -> order(GLENS, N), or
 *   order_part(GLENS, N) + MAX all-reduce ORDER[:N] (the order split over the
 *   ranks) -> minimize(do_pass2 = 0)
 *   key mode:    MIN all-reduce FIRST (int32 x span) -> pass2
 *   window mode: all-gather + OR COVERED (bitmap_op) -> n_ids = dense_first
 *                -> MIN all-reduce FIRST_DENSE[:n_ids] -> pass2
 *   -> MAX all-reduce KEPT[:N + 4] (u8): pass2 puts this shard's SYZCOV_ERR_*
 *      flags in KEPT[N..N+3], one byte per flag bit (so the MAX is the OR of
 *      each bit), and finish ORs them into the step's flags, so every rank
 *      fails a step any shard flagged, with the same flags (its aliased first
 *      covers went into the MIN merge)
 *   -> finish -> result.
 * A step abandoned between minimize(do_pass2 = 0) and pass2 is cleaned up by
 * the next canon (FIRST refilled).  canon_in_place: the canonical key words
 * replace the raw PCs, so every step must be fed raw PCs again. */
typedef uint64_t syzcov_corpus;
typedef struct syzcov_corpus_cfg {
    size_t n_max;        /* inputs per step on this GPU */
    size_t n_global;     /* 0: one GPU; else the sharded protocol over n_global inputs */
    size_t rank;         /* this shard (sharded runs) */
    uint64_t p_max;      /* raw PCs per step on this GPU */
    size_t max_seg_len;  /* longest input (a longer one fails the step) */
    uint32_t pc_lo;      /* window mode: the PC window */
    uint64_t pc_span;
    const uint32_t *universe; /* key mode (host; read during create only) */
    size_t universe_n;
    int canon_in_place;  /* canonical lists overwrite the raw ones (max_seg_len <= 16384) */
    int order_by;        /* 0: canonical lengths; 1: raw lengths (Minimize of covers as given) */
    uint64_t rec_cap;    /* first-cover records (0 = default) */
    int canon_layout;    /* 0: the canonical lists in the raw lists' CSR slots; 1 (out of
                            place over > 1 range): line-aligned, every input's range
                            sub-run on its own 128-B lines, so Minimize reads each line
                            once (CANON holds p_max + 31 (nrange + 1) n_max + 32 words) */
} syzcov_corpus_cfg;
typedef struct syzcov_corpus_info_t {
    uint32_t key_mode, kshift, kbase, pc_lo; /* key(pc) = (pc >> kshift) - kbase */
    uint64_t span;       /* keys (key mode) or window PCs */
    uint32_t win_lo, sent_key;  /* canonicalize's window; index of 0xFFFFFFFF (or ~0) */
    uint64_t win_span, nrange, nwords, n_global, union_cap, rec_cap;
    void *mem;
    uint64_t mem_size;
    uint64_t canon_align_k; /* 0: CANON in CSR slots; else the line-aligned layout's
                               ak = 31 (nrange + 1): input i at align32(off[i] + ak i),
                               range j's sub-run at + align32(split[i][j-1] + 31 j) */
} syzcov_corpus_info_t;
typedef struct syzcov_corpus_res {
    uint32_t err_flags;  /* SYZCOV_ERR_* bits of the step */
    uint32_t n_ids;      /* distinct keys of the corpus (sentinel included) */
    uint32_t n_kept, n_union;
    uint64_t max_cover;  /* |maxCover| after the merge */
    uint64_t records;    /* first-cover records of the step */
    const int32_t *kept_idx;   /* device: kept input indices, processing order */
    const uint32_t *union_pcs; /* device: the sorted union */
    uint32_t fallback;   /* 1: the step saw a PC outside the key space (err_flags says
                            which) and was recomputed in window mode; kept list and
                            union exact */
    uint32_t max_cover_missed; /* fallback: union PCs the resident maxCover cannot
                            represent (key mode: not the universe PC of their key;
                            window mode: outside the window) and so did not take; the
                            reference's maxCover would hold them (0: maxCover exact) */
} syzcov_corpus_res;
/* buffers of the layout (syzcov_corpus_buffer: byte offset in the block, size) */
enum {
    SYZCOV_CORPUS_CANON = 0,   /* u32 [p_max + 1] canonical lists (not in place) */
    SYZCOV_CORPUS_NEW_LEN,     /* u32 [n_max + 1] canonical lengths */
    SYZCOV_CORPUS_SPLIT,       /* u32 [n_max][nrange] range split points */
    SYZCOV_CORPUS_RANGE_TOT,   /* u64 [nrange] */
    SYZCOV_CORPUS_COVERED,     /* u32 bitmap: the step's union */
    SYZCOV_CORPUS_MAX_COVER,   /* u32 [nwords] resident maxCover */
    SYZCOV_CORPUS_TAB,         /* u64 [nwords] dictionary of the union */
    SYZCOV_CORPUS_FIRST,       /* i32 [span] first-cover ranks (INT32_MAX between steps) */
    SYZCOV_CORPUS_REC,         /* u64 [rec_cap] first-cover records (key mode: 2 rec_cap, the
                                  second half their copy sorted by key bucket) */
    SYZCOV_CORPUS_CAND,        /* u8  [n_max + 1] */
    SYZCOV_CORPUS_KEPT,        /* u8  [n_global + 4] kept flag per global rank, + 4 error-flag bytes */
    SYZCOV_CORPUS_LENS,        /* i64 [n_global + 1] */
    SYZCOV_CORPUS_ORDER,       /* i32 [n_global + 1] Go's processing order */
    SYZCOV_CORPUS_KEPT_IDX,    /* i32 [n_global + 1] kept inputs, processing order */
    SYZCOV_CORPUS_UNION,       /* u32 [union_cap] sorted union */
    SYZCOV_CORPUS_SCAL,        /* u64 [16] step scalars */
    SYZCOV_CORPUS_PC_OF_KEY,   /* u32 [span] key mode */
    SYZCOV_CORPUS_LOW_OF_KEY,  /* u8  [span] key mode: membership table */
    SYZCOV_CORPUS_GLENS,       /* i32 [n_global] sharded: gathered lengths */
    SYZCOV_CORPUS_SEL,         /* unused (0 bytes): kept so the ids below stay */
    SYZCOV_CORPUS_IOTA,        /* unused (0 bytes) */
    SYZCOV_CORPUS_ITEMS,       /* i32 [n_max + 1] sharded: local inputs in order */
    SYZCOV_CORPUS_RANKS,       /* i32 [n_max + 1] sharded: their global ranks */
    SYZCOV_CORPUS_FIRST_DENSE, /* i32 [union_cap] sharded window mode */
    SYZCOV_CORPUS_WS,          /* scratch */
    SYZCOV_CORPUS_WS2,         /* sharded scratch */
    SYZCOV_CORPUS_NBUF
};
int64_t syzcov_corpus_mem_size(const syzcov_corpus_cfg *cfg);
int syzcov_corpus_create(const syzcov_corpus_cfg *cfg, void *mem, size_t mem_size,
                         syzcov_corpus *out);
int syzcov_corpus_destroy(syzcov_corpus h);
int syzcov_corpus_info(syzcov_corpus h, syzcov_corpus_info_t *out);
int syzcov_corpus_buffer(syzcov_corpus h, int which, uint64_t *offset, uint64_t *bytes);
/* The step's canonical lists (key words in key mode) copied into the raw
 * lists' CSR slots: out[off[i] .. off[i] + new_len[i]) (device, p_max words),
 * whichever layout CANON holds (info.canon_align_k). */
int syzcov_corpus_canonical(syzcov_corpus h, uint32_t *out, void *stream);
/* Phases (device pointers, asynchronous on `stream`).  raw is written when
 * canon_in_place. */
int syzcov_corpus_canon(syzcov_corpus h, const uint64_t *off, uint32_t *raw, size_t n,
                        void *stream);
/* lens: device int32[N] (sharded: the gathered lengths), NULL = this step's */
int syzcov_corpus_order(syzcov_corpus h, const int32_t *lens, size_t N, void *stream);
/* Sharded: this rank's PART of the order over the gathered lengths (the ranks
 * split the late pdqsort rounds and the finisher, syzcov_dev_sort_order_part);
 * the caller then MAX all-reduces ORDER[:N] (int32), which gives every rank
 * the full order, before minimize. */
int syzcov_corpus_order_part(syzcov_corpus h, const int32_t *lens, size_t N, void *stream);
/* The caller's processing order instead (device int32[N]: order[r] = the
 * input of rank r, e.g. the Go shim's own sort.Sort(minInputArray),
 * cover.go:113; sharded: the global order, identical on every rank).  An
 * entry outside [0, N) is replaced by 0 and fails the step (SYZCOV_ERR_ORDER);
 * a permutation is the caller's contract (the host form checks it). */
int syzcov_corpus_order_given(syzcov_corpus h, const int32_t *order, size_t N, void *stream);
int syzcov_corpus_minimize(syzcov_corpus h, int do_pass2, void *stream);
/* window mode, sharded: returns n_ids (synchronizes the stream) */
int64_t syzcov_corpus_dense_first(syzcov_corpus h, void *stream);
int syzcov_corpus_pass2(syzcov_corpus h, void *stream);
int syzcov_corpus_finish(syzcov_corpus h, void *stream);
/* canon + order + minimize + finish on one GPU */
int syzcov_corpus_step(syzcov_corpus h, const uint64_t *off, uint32_t *raw, size_t n,
                       void *stream);
/* Synchronizes the stream; the step's counts and device result pointers.
 * A PC outside the key space (key mode: not in the universe; either mode:
 * outside the window) does not fail the step: like cover.Minimize on any u32
 * input, it is recomputed by a window-mode engine over the step's own PC
 * extent (res.fallback = 1; maxCover takes the union's PCs it can represent).
 * That needs the raw PCs, so a step canonicalized in place (on device) or
 * sharded returns SYZCOV_ERANGE instead, as does a corpus wider than 2^28 PCs;
 * SYZCOV_ETOOLONG: an input longer than max_seg_len. */
int syzcov_corpus_result(syzcov_corpus h, syzcov_corpus_res *res, void *stream);
/* The drop-in form: cover.Minimize + the union fold of a host CSR corpus
 * (offsets[n + 1], pcs) through the handle; out_idx (capacity n) receives the
 * kept indices in processing order, union_out (nullable, capacity union_cap)
 * the sorted union, *n_union (nullable) its size.  Returns the kept count. */
int64_t syzcov_corpus_minimize_host(syzcov_corpus h, const uint64_t *offsets, const uint32_t *pcs,
                                    size_t n, int32_t *out_idx, uint32_t *union_out,
                                    size_t union_cap, uint64_t *n_union);
/* The same with the caller's processing order (host int32[n], a permutation
 * of [0, n); SYZCOV_EINVAL otherwise): what the cover.Minimize shim passes. */
int64_t syzcov_corpus_minimize_host_order(syzcov_corpus h, const uint64_t *offsets,
                                          const uint32_t *pcs, size_t n, const int32_t *order,
                                          int32_t *out_idx, uint32_t *union_out, size_t union_cap,
                                          uint64_t *n_union);

/* =================== 2. device-resident launch API ==================== */
/* All pointers below are device pointers; `stream` is a hipStream_t.
 * `ws` is caller-provided device workspace of at least the returned size.  */

/* Segmented Canonicalize of a CSR corpus, out of place (out may equal in).
 * Segment i's canonical list goes to out[off[i] .. off[i] + new_len[i]).
 * If pres != NULL, also marks pres[pc - pc_lo] = 1 (uint8 presence map over
 * the PC window of pc_span bytes) and sets *err_flag (device u32) to nonzero
 * when a PC falls outside the window. */
size_t syzcov_dev_canon_ws_size(size_t nseg, size_t max_seg_len);
int syzcov_dev_canonicalize(const uint64_t *off, const uint32_t *in, uint32_t *out,
                            uint32_t *new_len, size_t nseg, size_t max_seg_len, uint8_t *pres,
                            uint32_t pc_lo, uint64_t pc_span, uint32_t *err_flag, void *ws,
                            size_t ws_size, void *stream);

/* Presence marking of a CSR corpus with explicit lengths (len == NULL:
 * lengths from offsets). */
int syzcov_dev_mark(const uint64_t *off, const uint32_t *len, const uint32_t *pcs, size_t nseg,
                    uint8_t *pres, uint32_t pc_lo, uint64_t pc_span, uint32_t *err_flag,
                    void *stream);

/* Bitmap set algebra on u32 words (ops as syzcov_dev_bytemap_op) + popcount. */
int syzcov_dev_bitmap_op(int op, uint32_t *dst, const uint32_t *src, uint64_t nwords,
                         uint64_t *popcount_out, void *stream);
/* Dictionary from a presence bitmap (see syzcov_dev_dict_build). */
int syzcov_dev_dict_build_bits(const uint32_t *bits, uint64_t pc_span, uint64_t *tab,
                               uint32_t *n_ids, void *ws, void *stream);

/* Dense PC-id dictionary from a presence map: tab[w] = {prefix:32 | bits:32}
 * for 32-PC word w (prefix = set bits before w).  *n_ids receives the total
 * (device u32).  ws: syzcov_dev_dict_ws_size(pc_span). */
size_t syzcov_dev_dict_ws_size(uint64_t pc_span);
int syzcov_dev_dict_build(const uint8_t *pres, uint64_t pc_span, uint64_t *tab, uint32_t *n_ids,
                          void *ws, void *stream);

/* Sorted list of the PCs present in the dictionary, minus 0xFFFFFFFF
 * (Union drops the sentinel).  *n_out (device u32) receives the count. */
int syzcov_dev_dict_to_list(const uint64_t *tab, uint64_t pc_span, uint32_t pc_lo,
                            uint32_t *out, uint32_t *n_out, void *stream);
/* The same with the dropped value given: in key mode the KEY of 0xFFFFFFFF
 * (the largest key, the key map being monotone); 0xFFFFFFFF otherwise. */
int syzcov_dev_dict_to_list_drop(const uint64_t *tab, uint64_t pc_span, uint32_t pc_lo,
                                 uint32_t drop, uint32_t *out, uint32_t *n_out, void *stream);

/* Minimize pass 1 over n work items in rank order: item j is input
 * order[j] with rank ranks[j] (ranks == NULL: rank j).  first[id] (pre-set to
 * INT32_MAX) receives the minimum rank covering dense id `id`; cand[j] = 1
 * iff item j lowered some first[] entry (a necessary condition for being
 * kept).  Sharded runs pass each shard's items with their GLOBAL ranks and
 * then MIN-all-reduce first[]. */
int syzcov_dev_minimize_pass1(const uint64_t *off, const uint32_t *len, const uint32_t *pcs,
                              const int32_t *order, const int32_t *ranks, size_t n,
                              const uint64_t *tab, uint32_t pc_lo, int32_t *first, uint8_t *cand,
                              void *stream);
/* Minimize pass 2: kept[rank] = 1 for every candidate item j holding a PC
 * with first[id(pc)] == rank (kept[] pre-zeroed, indexed by rank, so shards
 * can MAX-all-reduce it). */
int syzcov_dev_minimize_pass2(const uint64_t *off, const uint32_t *len, const uint32_t *pcs,
                              const int32_t *order, const int32_t *ranks, size_t n,
                              const uint64_t *tab, uint32_t pc_lo, const int32_t *first,
                              const uint8_t *cand, uint8_t *kept, void *stream);
/* Sharded runs: window-indexed first_w <-> dense-id first (one int32 per
 * present PC of the dictionary `tab`) so the RCCL MIN moves n_ids, not
 * pc_span, entries.  to_dense = 1 gathers, 0 scatters back. */
int syzcov_dev_first_dense(const uint64_t *tab, uint64_t pc_span, int32_t *first_w,
                           int32_t *dense, int to_dense, void *stream);

/* ---- engine default path: wavefront canonicalize + range-partitioned Minimize ----
 * Canonicalize (cover.go:27-40) with ONE wavefront per segment (LDS radix
 * sort over window offsets, unique, PCs written to out[off[i] ..), in place
 * allowed when max_seg_len <= 16384).  PCs outside [pc_lo, pc_lo + pc_span)
 * set SYZCOV_ERR_WINDOW in *err_flag, a segment longer than max_seg_len sets
 * SYZCOV_ERR_SEGLEN (it is not canonicalized).  If split != NULL (nrange = ceil(pc_span / 2^range_shift)
 * <= 256 columns per segment), split[i * nrange + j] = number of canonical
 * PCs of segment i below pc_lo + ((j + 1) << range_shift) and range_tot[j]
 * (u64, pre-zeroed) accumulates the canonical PCs of range j.
 * ws: syzcov_dev_canon_split_ws_size(nseg). */
size_t syzcov_dev_canon_split_ws_size(size_t nseg);
int syzcov_dev_canon_split(const uint64_t *off, const uint32_t *raw, uint32_t *out,
                           uint32_t *new_len, size_t nseg, size_t max_seg_len, uint32_t pc_lo,
                           uint64_t pc_span, uint32_t range_shift, uint32_t *split,
                           uint64_t *range_tot, uint32_t *err_flag, void *ws, size_t ws_size,
                           void *stream);
/* Key mode (keys.hip): key(pc) = (pc >> kshift) - kbase over a registered PC
 * universe (the PCs KCOV reports: return addresses of the
 * __sanitizer_cov_trace_pc calls) with kshift = the largest collision-free
 * shift, at most SYZCOV_KSHIFT_MAX, nkeys <= 2^25.  Canonicalize runs on the
 * PCs of [pc_lo, pc_lo + pc_span) exactly as syzcov_dev_canon_split; every
 * canonical PC is written as its KEY WORD key | (pc & (2^kshift - 1)) << 26
 * (so two PCs sharing a key stay two entries), and split[] / range_tot[]
 * count ranges of 2^range_shift keys.  The window must map into [0, nkeys).
 * Membership in the universe is checked where the words are consumed
 * (syzcov_dev_minimize_range_keys). */
int syzcov_dev_canon_split_keys(const uint64_t *off, const uint32_t *raw, uint32_t *out,
                                uint32_t *new_len, size_t nseg, size_t max_seg_len, uint32_t pc_lo,
                                uint64_t pc_span, uint32_t kshift, uint32_t kbase, uint64_t nkeys,
                                uint32_t range_shift, uint32_t *split, uint64_t *range_tot,
                                uint32_t *err_flag, void *ws, size_t ws_size, void *stream);
/* Either of the two above (key mode iff key_out) writing the LINE-ALIGNED
 * layout: every (input, range) sub-run starts on its own 128-byte line, so a
 * Minimize pass that reads range j of an input in one workgroup and range j + 1
 * in another never fetches a line twice.  With ak = 31 (nrange + 1), input i's
 * words start at align32(off[i] + ak i) and range j's sub-run at
 * + align32(split[i][j-1] + 31 j) (split[i][-1] = 0); out holds
 * syzcov_dev_canon_aligned_words(p, nseg, nrange) words.  split is required;
 * out must not alias raw.  Read it back with syzcov_dev_minimize_range_aligned. */
int syzcov_dev_canon_split_aligned(const uint64_t *off, const uint32_t *raw, uint32_t *out,
                                   uint32_t *new_len, size_t nseg, size_t max_seg_len,
                                   uint32_t pc_lo, uint64_t pc_span, uint32_t kshift,
                                   uint32_t kbase, uint64_t nkeys, int key_out,
                                   uint32_t range_shift, uint32_t *split, uint64_t *range_tot,
                                   uint32_t *err_flag, void *ws, size_t ws_size, void *stream);
uint64_t syzcov_dev_canon_aligned_words(uint64_t p_max, uint64_t nseg, uint64_t nrange);
/* cover_dedup (executor/executor.cc:574-587) of nseg raw u64 KCOV buffers
 * [off[s], off[s+1]) of pcs, IN PLACE: buffer s becomes its sorted distinct
 * nonzero PCs, new_len[s] of them (UINT32_MAX for a buffer longer than 2^31
 * or with off[s+1] < off[s], left untouched).  out32 (nullable, sized like
 * pcs) receives at the same positions each kept PC truncated to u32, as
 * executor.cc:459-463 writes them.  No workspace. */
int syzcov_dev_cover_dedup64(uint64_t *pcs, const uint64_t *off, size_t nseg, uint32_t *new_len,
                             uint32_t *out32, void *stream);
/* Executor KCOV buffers straight into the new-coverage check:
 * syzcov_dev_cover_dedup64 of the nbuf buffers [off[b], off[b+1]) of pcs64
 * (in place; off[0] = 0, off[nbuf] = total), then each buffer's kept PCs
 * truncated to u32 (executor.cc:459-463) packed into a CSR of records:
 * rec_off[0..nbuf] (u64, rec_off[0] = 0) and rec_pcs (room for `total`
 * words) -- what syzcov_state_newcov_dev takes, with no host round trip.  A
 * malformed buffer contributes an empty record and sets *err |= 1 (device
 * u32, nullable).  (Records are sorted when a buffer's PCs share their high
 * 32 bits, as a kernel's do; newcov rejects an unsorted one.)
 * ws: syzcov_dev_cover_ingest64_ws_size(nbuf, total). */
size_t syzcov_dev_cover_ingest64_ws_size(size_t nbuf, uint64_t total);
int syzcov_dev_cover_ingest64(uint64_t *pcs64, const uint64_t *off, size_t nbuf, uint64_t total,
                              uint64_t *rec_off, uint32_t *rec_pcs, uint32_t *err, void *ws,
                              size_t ws_size, void *stream);
/* out[i] = the PC of key word words[i] (exact, no table); in place allowed. */
int syzcov_dev_words_to_pcs(const uint32_t *words, size_t n, uint32_t kshift, uint32_t kbase,
                            uint32_t *out, void *stream);
/* Key tables of a universe (univ sorted, collision-free under kshift <=
 * SYZCOV_KSHIFT_MAX, else *err_flag |= 1): pc_of_key[key(univ[i])] = univ[i]
 * (0 for keys without a universe PC) and low_of_key[key(univ[i])] =
 * univ[i] & (2^kshift - 1) (0x7F without one).  Either table may be NULL. */
int syzcov_dev_universe_keymap(const uint32_t *univ, size_t n, uint32_t kshift, uint32_t kbase,
                               uint64_t nkeys, uint32_t *pc_of_key, uint8_t *low_of_key,
                               uint32_t *err_flag, void *stream);
/* out[i] = pc_of_key[keys[i]] for i < min(*n_dev, n_max) (n_dev: device count,
 * nullable); keys >= nkeys give 0xFFFFFFFF; in place allowed. */
int syzcov_dev_keys_to_pcs(const uint32_t *pc_of_key, uint64_t nkeys, const uint32_t *keys,
                           uint32_t *out, const uint32_t *n_dev, size_t n_max, void *stream);

/* covered[w] = bits of first[] < INT32_MAX over [0, span) (the union of a
 * sharded step from its MIN all-reduced first-cover array). */
int syzcov_dev_first_to_bits(const int32_t *first, uint64_t span, uint32_t *covered, void *stream);

/* Minimize (cover.go:104-131) over canonical covers with split[] from
 * syzcov_dev_canon_split.  Item j (processing order) is input order[j] with
 * rank ranks[j] (NULL: j).  covered: window bitmap of nrange << range_shift
 * bits (pre-zeroed, or a shard's covered set); on return it holds the union
 * of the items' covers.  first_w: int32 per window PC, all INT32_MAX on entry
 * and on return.  rec: capacity rec_cap of (rank << 32 | offset) records;
 * *rec_cnt (device u64) receives the record count (> rec_cap: overflow,
 * handled exactly by fallback kernels).  cand: u8 per item (pre-zeroed).
 * kept: u8 per rank (pre-zeroed) receives kept[rank] = 1 (do_pass2).  first_chunk /
 * growth / pcs_per_wg_hint tune the chunk schedule (0 = defaults: 64, 4,
 * 2^19); any values give the same result.
 * ws: syzcov_dev_minimize_range_ws_size(n_items, pc_span, range_shift). */
size_t syzcov_dev_minimize_range_ws_size(size_t n_items, uint64_t pc_span, uint32_t range_shift);
int syzcov_dev_minimize_range(const uint64_t *off, const uint32_t *len, const uint32_t *pcs,
                              const uint32_t *split, const int32_t *order, const int32_t *ranks,
                              size_t n_items, uint32_t pc_lo, uint64_t pc_span,
                              uint32_t range_shift, const uint64_t *range_tot, uint32_t *covered,
                              int32_t *first_w, uint64_t *rec, uint64_t rec_cap, uint64_t *rec_cnt,
                              uint8_t *cand, uint8_t *kept, int do_pass2, size_t first_chunk,
                              uint32_t growth, uint64_t pcs_per_wg_hint, void *ws, void *stream);
/* Key mode (keys.hip): the same over KEY WORDS (syzcov_dev_canon_split_keys)
 * of nkeys <= 2^25 keys in ranges of 2^range_shift <= 2^17 keys.  Every word
 * is checked against the membership table low_of_key (syzcov_dev_universe_keymap,
 * padded with 0x7F to nrange << range_shift bytes): a word whose PC is not in
 * the universe sets SYZCOV_ERR_UNIVERSE in *err_flag and the step's results
 * must not be used.  first_w / covered / records are over keys.  Sharded runs
 * MIN all-reduce first_w and call syzcov_dev_minimize_range_keys_pass2. */
int syzcov_dev_minimize_range_keys(const uint64_t *off, const uint32_t *len,
                                   const uint32_t *words, const uint32_t *split,
                                   const int32_t *order, const int32_t *ranks, size_t n_items,
                                   uint64_t nkeys, uint32_t range_shift,
                                   const uint64_t *range_tot, const uint8_t *low_of_key,
                                   uint32_t *covered, int32_t *first_w, uint64_t *rec,
                                   uint64_t rec_cap, uint64_t *rec_cnt, uint8_t *cand,
                                   uint8_t *kept, int do_pass2, uint32_t *err_flag, void *ws,
                                   void *stream);
int syzcov_dev_minimize_range_keys_pass2(const uint64_t *off, const uint32_t *len,
                                         const uint32_t *words, const uint32_t *split,
                                         const int32_t *order, const int32_t *ranks,
                                         size_t n_items, uint64_t nkeys, uint32_t range_shift,
                                         const uint64_t *range_tot, uint32_t *covered,
                                         int32_t *first_w, uint64_t *rec, uint64_t rec_cap,
                                         uint64_t *rec_cnt, uint8_t *cand, uint8_t *kept,
                                         void *ws, void *stream);
/* syzcov_dev_minimize_range(_keys) over canonical lists in the line-aligned
 * layout of syzcov_dev_canon_split_aligned (key mode iff low_of_key: pc_lo = 0,
 * pc_span = the key count, err_flag as in _keys); default chunking. */
int syzcov_dev_minimize_range_aligned(const uint64_t *off, const uint32_t *pcs,
                                      const uint32_t *split, const int32_t *order,
                                      const int32_t *ranks, size_t n_items, uint32_t pc_lo,
                                      uint64_t pc_span, uint32_t range_shift,
                                      const uint64_t *range_tot, const uint8_t *low_of_key,
                                      uint32_t *covered, int32_t *first_w, uint64_t *rec,
                                      uint64_t rec_cap, uint64_t *rec_cnt, uint8_t *cand,
                                      uint8_t *kept, int do_pass2, uint32_t *err_flag, void *ws,
                                      void *stream);
/* Its sharded pass 2 (key_mode: tab and first_dense NULL, as _keys_pass2;
 * window mode: as syzcov_dev_minimize_range_pass2). */
int syzcov_dev_minimize_range_aligned_pass2(const uint64_t *off, const uint32_t *pcs,
                                            const uint32_t *split, const int32_t *order,
                                            const int32_t *ranks, size_t n_items, uint32_t pc_lo,
                                            uint64_t pc_span, uint32_t range_shift,
                                            const uint64_t *range_tot, int key_mode,
                                            uint32_t *covered, int32_t *first_w, uint64_t *rec,
                                            uint64_t rec_cap, uint64_t *rec_cnt, uint8_t *cand,
                                            const uint64_t *tab, const int32_t *first_dense,
                                            uint8_t *kept, void *ws, void *stream);
/* Sharded runs: call syzcov_dev_minimize_range with do_pass2 = 0 (first_w then
 * holds this shard's first ranks and covered its union), merge the shards'
 * covered bitmaps (OR) into the dictionary `tab` (syzcov_dev_dict_build_bits),
 * MIN-merge first_dense (syzcov_dev_first_dense to_dense = 1 over tab), then
 * call this with the same arguments and ws: kept[rank] = 1 iff the merged
 * first rank of one of the item's PCs equals its rank; first_w is reset.
 * tab == NULL: single-GPU pass 2 from first_w. */
int syzcov_dev_minimize_range_pass2(const uint64_t *off, const uint32_t *len, const uint32_t *pcs,
                                    const uint32_t *split, const int32_t *order,
                                    const int32_t *ranks, size_t n_items, uint32_t pc_lo,
                                    uint64_t pc_span, uint32_t range_shift,
                                    const uint64_t *range_tot, uint32_t *covered, int32_t *first_w,
                                    uint64_t *rec, uint64_t rec_cap, uint64_t *rec_cnt,
                                    uint8_t *cand, const uint64_t *tab, const int32_t *first_dense,
                                    uint8_t *kept, void *ws, void *stream);

/* Ordered compaction: out_idx = [order[r] for r if kept[r]]; *n_out (device u32). */
size_t syzcov_dev_compact_ws_size(size_t n);
int syzcov_dev_compact_kept(const uint8_t *kept, const int32_t *order, size_t n, int32_t *out_idx,
                            uint32_t *n_out, void *ws, void *stream);

/* Exact Go sort.Sort(minInputArray) order on the device from int64 lengths. */
size_t syzcov_dev_sort_ws_size(size_t n);
int syzcov_dev_sort_order(const int64_t *lens, size_t n, int sort_variant, int32_t *order,
                          void *ws, size_t ws_size, void *stream);
/* One part of the order for a corpus sharded over `nparts` ranks: the parts
 * run the same level-synchronous rounds until the order holds >= 4 * nparts
 * segments, then each finishes only the segments starting in its block of
 * positions and leaves -1 in the others'; an int32 MAX all-reduce of the
 * parts' `order` arrays is the full order (cover.go:113).  Same workspace as
 * syzcov_dev_sort_order. */
int syzcov_dev_sort_order_part(const int64_t *lens, size_t n, uint32_t part, uint32_t nparts,
                               int32_t *order, void *ws, size_t ws_size, void *stream);
/* Segmented form: an independent Go sort.Sort per group, group g = lens
 * [goff[g], goff[g+1]) (device u64, ngroups >= 1, every group non-empty,
 * lengths < 0xFFFFFFFF).  order[i] for i in group g is a grouped index inside
 * group g, exactly the order Go gives that group as its own slice. */
size_t syzcov_dev_sort_seg_ws_size(size_t n, size_t ngroups);
int syzcov_dev_sort_order_segmented(const int64_t *lens, const uint64_t *goff, size_t ngroups,
                                    size_t n, int sort_variant, int32_t *order, void *ws,
                                    size_t ws_size, void *stream);

/* Bitmap/byte-map set algebra over a PC window (coalesced, ballot-packed):
 * op 0: dst |= src  (Union)      op 1: dst &= src  (Intersection)
 * op 2: dst &= ~src (Difference) op 3: dst ^= src  (SymmetricDifference)
 * Maps are uint8 per PC; *popcount_out (device u64, nullable) receives the
 * number of nonzero bytes of the result. */
/* A bitmap of nwords u32 words <-> its byte map (32 bytes per word, byte b of
 * word w = bit b of w, 0 or 1; any nonzero byte reads back as a set bit): the
 * form the shard bitmaps take for their uint8 MAX all-reduce (north_star;
 * syzkaller_amd/dist.py merge_bitmap_u8).  bytes: 16-byte aligned, 32 nwords. */
int syzcov_dev_bits_to_bytes(const uint32_t *bits, uint64_t nwords, uint8_t *bytes, void *stream);
int syzcov_dev_bytes_to_bits(const uint8_t *bytes, uint64_t nwords, uint32_t *bits, void *stream);
int syzcov_dev_bytemap_op(int op, uint8_t *dst, const uint8_t *src, uint64_t nbytes,
                          uint64_t *popcount_out, void *stream);

/* Synthetic corpus (integer-exact): lengths for inputs
 * [first, first+n), then PCs into CSR.  mode bit 0: uniform key draws (else
 * k = 2^S u^3); bit 1: the x86-like universe (neighbouring PCs 5..14 bytes
 * apart: pairs per 16-byte block, U[2m] = 0x81000000 + 16m + a, U[2m+1] = U[2m] + 5 + b,
 * kshift 2), else one PC per
 * 16-byte slot (U[k] = 0x81000000 + 16k + (h(k) & 15), kshift 4). */
int syzcov_dev_synth_lens(uint64_t seed, uint64_t first, size_t n, uint32_t mean, uint32_t sigma,
                          uint32_t *lens, void *stream);
int syzcov_dev_synth_pcs(uint64_t seed, uint64_t first, size_t n, const uint64_t *off,
                         uint32_t log2_space, int mode, uint32_t *pcs, void *stream);
/* C5's synthetic call records: out[i] = CallID of record first + i, uniform
 * over [0, ncalls) (counter-based: oracle/synth_oracle.c regenerates it). */
int syzcov_dev_synth_callids(uint64_t seed, uint64_t first, size_t n, uint32_t ncalls,
                             int32_t *out, void *stream);
/* The synthetic PC universe U[k], k < 2^log2_space (sorted);
 * _mode: bit 1 of syzcov_dev_synth_pcs's mode selects the x86-like one. */
int syzcov_dev_synth_universe(uint64_t seed, uint32_t log2_space, uint32_t *out, void *stream);
int syzcov_dev_synth_universe_mode(uint64_t seed, uint32_t log2_space, int mode, uint32_t *out,
                                   void *stream);
/* dst <- src, 16-byte aligned, nbytes % 16 == 0: the streaming-copy kernel
 * whose rate the bench reports as the measured HBM peak. */
int syzcov_dev_stream_copy(const void *src, void *dst, size_t nbytes, void *stream);
/* HBM copy-rate probes for the bench's measured peak: form 0 = the streaming
 * copy above, 1 = one 16-byte element per thread, one pass (<= 2^36 bytes). */
int syzcov_dev_copy_peak(const void *src, void *dst, size_t nbytes, int form, void *stream);

/* Dynamic priority counts as a dense contraction on i8 MFMA with i32
 * accumulation: counts = AᵀA over the matrix AT (rows = syzcov_dev_prio_rows(C)
 * keys x ldp = syzcov_dev_prio_ldp(nprog) programs, zero padded), stored
 * K-blocked: (key r, program p) at byte (p / 64) * rows * 64 + r * 64 + p % 64.  Row C of AT is all ones, so
 * counts[i][C] = colsum(A)[i] feeds the diagonal correction.
 * key_mode 0 (positional, reference-exact: prio.go:142-150 indexes by call
 * position): AT[k][p] = [k < lens[p]]; key_mode 1: AT[c][p] = number of calls
 * of syscall id c in program p (CSR prog_off/call_ids, <= 127 per program).
 * counts is rows x rows int32, zeroed by the caller; shards accumulate into
 * it and may be summed with an RCCL int32 sum all-reduce. */
size_t syzcov_dev_prio_rows(int C);
size_t syzcov_dev_prio_ldp(size_t nprog);
int syzcov_dev_prio_build_at(int key_mode, const int32_t *lens, const uint64_t *prog_off,
                             const uint16_t *call_ids, size_t nprog, int C, int8_t *at,
                             size_t ldp, uint32_t *err_flag, void *stream);
int syzcov_dev_prio_counts(const int8_t *at, size_t ldp, size_t nprog, int C, int32_t *counts,
                           void *stream);
/* The same contraction on 256 x 256 tiles (a 128 x 128 sub-tile per wave, one
 * workgroup per CU, K split over the workgroups with partial tiles in ws and
 * one reduction): LDS traffic under the MFMA time instead of over it.  ws:
 * syzcov_dev_prio_counts_ws_size(nprog, C) bytes (0: the rows are not a
 * multiple of 256; then, or with a smaller ws, syzcov_dev_prio_counts runs).
 * Accumulates into counts like syzcov_dev_prio_counts. */
size_t syzcov_dev_prio_counts_ws_size(size_t nprog, int C);
int syzcov_dev_prio_counts_ws(const int8_t *at, size_t ldp, size_t nprog, int C, int32_t *counts,
                              void *ws, size_t ws_size, void *stream);
/* Positional counts (key_mode 0) over the ACTIVE keys only: A[p][k] is zero
 * for k >= max_len, so AT is built for the first roundup(max_len, 128) keys,
 * the MFMA tiles are K-split with partial tiles + a reduction, and the
 * colsum column counts[i][C] comes from a length histogram.  counts
 * (prio_rows(C)^2 int32) must be zeroed by the caller; max_len = max(lens)
 * (<= C).  ws: syzcov_dev_prio_pos_ws_size(nprog, C, max_len). */
size_t syzcov_dev_prio_pos_ws_size(size_t nprog, int C, int max_len);
int syzcov_dev_prio_counts_pos(const int32_t *lens, size_t nprog, int C, int max_len,
                               int32_t *counts, void *ws, size_t ws_size, void *stream);
/* counts -> D = AᵀA - diag(colsum) -> float32 exactly as Go's repeated
 * `+= 1.0` would hold it (min(n, 2^24)) -> normalizePrio -> * static
 * (nullable).  raw_out (nullable, C*C uint32) receives D. */
int syzcov_dev_prio_finish(const int32_t *counts, int C, const float *static_prios, float *out,
                           uint32_t *raw_out, void *stream);
int syzcov_dev_normalize_prio(float *prios, int C, void *stream);
int syzcov_dev_choice_table(const float *prios, const uint8_t *enabled, int C, int64_t *run,
                            void *stream);
int syzcov_dev_choose(const int64_t *run, const uint8_t *enabled, int C, const int32_t *calls,
                      const int64_t *x, size_t nq, int32_t *out, uint32_t *err_flag, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* SYZCOV_H */
