// ingest.cc — executor output → new-coverage records (host side, no GPU).
//
// The executor writes, after a u32 record count, one record per completed call
// (executor/executor.cc:455-466):
//     u32 call_index, u32 call_num, u32 errno, u32 cover_size, u32 pcs[cover_size]
// little-endian; the PCs are already sorted and de-duplicated there
// (cover_dedup, executor.cc:574-587).  ipc.Env.Exec reads it back into
// cov[call_index] / errnos[call_index] (ipc/ipc.go:225-291), and
// syz-fuzzer execute() walks the calls in index order, skipping empty covers
// (syz-fuzzer/fuzzer.go:456-460).  This parser does both steps and emits the
// records syzcov_newcov_batch consumes, in that order, so a fuzzer can append
// many programs to one batch.
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/syzcov.h"

namespace syz {
void set_error(const char *fmt, ...);
}

extern "C" int64_t syzcov_parse_exec_output(const uint8_t *out, size_t out_len, size_t ncalls,
                                            const uint32_t *call_num, const int32_t *callid_of_num,
                                            size_t nnum, int64_t *errnos, int32_t *rec_callid,
                                            uint32_t *rec_call_index, uint64_t *rec_off,
                                            uint32_t *rec_pcs, size_t pcs_cap) {
    using syz::set_error;
    if (!out || (ncalls && (!call_num || !errnos || !rec_callid || !rec_call_index || !rec_off)) ||
        (nnum && !callid_of_num))
        return SYZCOV_EINVAL;
    size_t pos = 0;
    auto rd = [&](uint32_t *v) {
        if (pos > out_len || out_len - pos < 4) return false;
        uint32_t x;
        memcpy(&x, out + pos, 4);  // little-endian host (x86-64 / arm64)
        *v = x;
        pos += 4;
        return true;
    };
    uint32_t ncmd = 0;
    if (!rd(&ncmd)) {
        set_error("failed to read output coverage: short buffer");
        return SYZCOV_EINVAL;
    }
    for (size_t i = 0; i < ncalls; i++) errnos[i] = -1;  // not executed (ipc.go:233-235)
    // cover of call i = [beg[i], beg[i] + len[i]) in `out`, in arrival order
    std::vector<size_t> beg(ncalls, 0);
    std::vector<uint32_t> len(ncalls, 0);
    std::vector<uint8_t> seen(ncalls, 0);
    for (uint32_t r = 0; r < ncmd; r++) {
        uint32_t ci, num, err, sz;
        if (!rd(&ci) || !rd(&num) || !rd(&err) || !rd(&sz)) {
            set_error("failed to read output coverage: record %u", r);
            return SYZCOV_EINVAL;
        }
        // the reference tests callIndex > len(cov) and then indexes p.Calls,
        // so callIndex == len(cov) panics there; it is an error here
        if (ci >= ncalls) {
            set_error("record %u: call %u, total calls %zu", r, ci, ncalls);
            return SYZCOV_ERANGE;
        }
        if (seen[ci]) {
            set_error("double coverage for call %u", ci);
            return SYZCOV_EINVAL;
        }
        if (call_num[ci] != num) {
            set_error("call %u: expect syscall %u, got %u", ci, call_num[ci], num);
            return SYZCOV_EINVAL;
        }
        if ((uint64_t)sz * 4 > out_len - pos) {
            set_error("record %u, call %u, coversize=%u: short buffer", r, ci, sz);
            return SYZCOV_EINVAL;
        }
        seen[ci] = 1;
        beg[ci] = pos;
        len[ci] = sz;
        errnos[ci] = (int64_t)err;  // Go: int(uint32)
        pos += (size_t)sz * 4;
    }
    // execute(): calls in index order, empty covers skipped
    int64_t nrec = 0;
    uint64_t npc = 0;
    rec_off[0] = 0;
    for (size_t ci = 0; ci < ncalls; ci++) {
        if (!len[ci]) continue;
        const uint32_t num = call_num[ci];
        if (num >= nnum) {
            set_error("call %zu: syscall %u outside the CallID table", ci, num);
            return SYZCOV_ERANGE;
        }
        if (npc + len[ci] > pcs_cap || !rec_pcs) {
            set_error("record PCs exceed capacity %zu", pcs_cap);
            return SYZCOV_ERANGE;
        }
        memcpy(rec_pcs + npc, out + beg[ci], (size_t)len[ci] * 4);
        rec_callid[nrec] = callid_of_num[num];
        rec_call_index[nrec] = (uint32_t)ci;
        npc += len[ci];
        rec_off[++nrec] = npc;
    }
    return nrec;
}
