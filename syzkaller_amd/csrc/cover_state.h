// cover_state.h — the fuzzer's resident coverage state (syz-fuzzer/fuzzer.go:
// 62-89: maxCover, corpusCover, flakes under coverMu) shared by newcov.hip
// (execute's new-coverage check, addInput) and triage.hip (triageInput).
#pragma once
#include "common.h"

#include <mutex>

namespace syz {

__device__ __forceinline__ bool bit_test(const uint32_t *__restrict__ bm, uint64_t o) {
    return (bm[o >> 5] >> (o & 31)) & 1u;
}

// Where a PC lives in the bitmaps: its window offset, or its dense key.
struct Index {
    int key_mode;
    uint32_t pc_lo, kshift, kbase;
    uint64_t span;                 // window span, or nkeys
    const uint8_t *low_of_key;     // key mode: universe membership (keys.hip)
};

// Bitmap index of pc; false only if it is outside the window / key range (no
// membership test: for positions, e.g. range boundaries, where the PC itself
// is checked elsewhere).
__device__ __forceinline__ bool pc_index_range(const Index &X, uint32_t pc, uint32_t *idx) {
    const uint32_t k = X.key_mode ? (pc >> X.kshift) - X.kbase : pc - X.pc_lo;
    *idx = k;
    return k < X.span;
}

// Bitmap index of pc; false if pc is outside the window / key range, or, in
// key mode, not a universe PC (its key belongs to another PC or to none: the
// caller rejects it instead of aliasing it, keys.hip).
__device__ __forceinline__ bool pc_index(const Index &X, uint32_t pc, uint32_t *idx) {
    if (X.key_mode) {
        const uint32_t k = (pc >> X.kshift) - X.kbase;  // wraps past span below kbase
        *idx = k;
        return k < X.span && X.low_of_key[k] == (pc & ((1u << X.kshift) - 1u));
    }
    const uint32_t o = pc - X.pc_lo;
    *idx = o;
    return pc >= X.pc_lo && (uint64_t)o < X.span;
}

struct CoverState {
    int dev = 0;
    int ncalls = 0;
    uint32_t pc_lo = 0;
    uint64_t pc_span = 0;
    // bitmap index space: window offsets, or dense keys of the registered
    // universe (key mode); words = 32-bit words per bitmap
    Index X{};
    uint64_t words = 0;
    uint32_t *maxcov = nullptr;  // ncalls x words
    uint32_t *corpus = nullptr;  // corpusCover: ncalls x words, allocated on first use
    uint32_t *flakes = nullptr;  // words
    // maxCover[c] | flakes per call, the LDS-staged candidate pass's one test
    // per PC; allocated on first use, rebuilt when marked stale (flakes or
    // maxCover changed outside the newcov kernels, which keep it in step)
    uint32_t *mfl = nullptr;
    bool mfl_stale = true;
    // the device may leave mfl stale (newcov.hip, the fused pass's mfl mode:
    // two words past mfl's bitmaps); a non-fused batch then rebuilds it
    bool mfl_dev_mode = false;
    uint32_t *pc_of_key = nullptr;  // key mode: key -> PC (reads of maxCover)
    uint8_t *low_of_key = nullptr;  // key mode: membership table (pc_index)
    // key mode with kshift <= 4: the same table as nibbles over whole ranges
    // of 2^RSH keys (8 keys per word), staged half a range at a time in LDS by
    // the candidate pass's separate membership pass (newcov.hip)
    uint32_t *nib = nullptr;
    // LDS-staged candidate pass: per-call record counts | offsets | cursors |
    // work-item prefix over (call, range) | work-item descriptors; one batch
    // at a time per state
    uint32_t *grp = nullptr;
    bool dirty = false;          // maxCover touched: the universe can no longer change
    hipStream_t s = nullptr;
    // device-tier batches run on the caller's stream: ordered after the
    // handle's stream (ev_state) and the handle's stream after them (ev_dev)
    hipEvent_t ev_state = nullptr, ev_dev = nullptr;
    std::mutex mu;  // the reference's coverMu
    // grow-only scratch
    void *scratch = nullptr;
    size_t scap = 0;
};

int bitmap_to_list(const uint32_t *bm, uint64_t pc_span, uint32_t pc_lo, uint32_t *out,
                   size_t cap, int64_t *count, hipStream_t s, const uint32_t *pc_of_key);

// shared host helpers (newcov.hip)
int state_grow(CoverState *st, size_t need);
int state_ensure_corpus(CoverState *st);
int state_bitmap_get(CoverState *st, const uint32_t *bm, uint32_t *out, size_t cap, int64_t *count);
int state_set_bits(CoverState *st, uint32_t *bm, const uint32_t *pcs, size_t n);

}  // namespace syz
