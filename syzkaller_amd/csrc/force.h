// force.h — SYZCOV_FORCE, the library's one run-time override (api.cc), for
// tests of the exact fallback paths.
#pragma once
#include <stdint.h>

namespace syz {
enum : uint32_t {
    FORCE_CANON3 = 1u,
    FORCE_REDO = 2u,
    FORCE_NC_LDS = 4u,
    FORCE_NC_PROBE = 8u,
    FORCE_GROUP_CHUNKS = 16u,  // minimizeCorpus: the per-group chunked engine for small groups too
    FORCE_NC_SEP = 32u,        // newcov key mode: candidate pass + separate membership pass
    FORCE_MR_BYTES = 64u,      // corpus key mode, kshift <= 2: byte tables, not nibbles
    FORCE_NC_HASH64 = 128u,    // newcov ownership: u64 keys + separate values, not packed slots
    FORCE_MIN_ATOMICS = 256u,  // corpus key mode: min_records' atomics, not bucketed first covers
    FORCE_NO_INIT_BLOCK = 512u,  // corpus key mode: chunks from item 0, no initial LDS block
    FORCE_SMALL_INIT = 1024u,    // corpus key mode: an initial block of one first chunk (tests)
};
uint32_t force_flags();
}  // namespace syz
