// ingest_fuzz.cc — ASan/UBSan harness for libsyzcov's executor-output parser
// (syzkaller_amd/csrc/ingest.cc, the reader of ipc/ipc.go:225-291).  The
// buffer lives in the fuzzer's shared memory and is written by the executor
// in the VM, so the parser must survive any bytes: truncated headers and
// records, cover sizes past the end, call indices out of range, duplicates,
// syscall mismatches, numbers outside the CallID table, capacity overflow.
// Built by tests/test_sanitize.py with -fsanitize=address,undefined and
// -fno-sanitize-recover; any report aborts.  Invariants on success: records
// in call-index order, offsets monotone, PCs within capacity and equal to the
// input's cover.
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/syzcov.h"

namespace syz {
void set_error(const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
}
}  // namespace syz

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint64_t rnd() {
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return rng_state;
}
static uint32_t rnd_u(uint32_t n) { return n ? (uint32_t)(rnd() % n) : 0; }

static void put(std::vector<uint8_t> &b, uint32_t v) {
    uint8_t x[4];
    memcpy(x, &v, 4);
    b.insert(b.end(), x, x + 4);
}

#define CHECK(c)                                                  \
    do {                                                          \
        if (!(c)) {                                               \
            fprintf(stderr, "check failed line %d: %s\n", __LINE__, #c); \
            abort();                                              \
        }                                                         \
    } while (0)

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20000;
    int ok = 0, rejected = 0;
    for (int it = 0; it < iters; it++) {
        const size_t ncalls = rnd_u(10);
        const size_t nnum = 1 + rnd_u(50);
        std::vector<uint32_t> call_num(ncalls);
        for (auto &x : call_num) x = rnd_u((uint32_t)nnum + (rnd_u(8) == 0 ? 5 : 0));
        std::vector<int32_t> callid(nnum);
        for (auto &x : callid) x = (int32_t)rnd_u(293);
        // a well-formed output, then damage it
        std::vector<uint8_t> out;
        std::vector<std::vector<uint32_t>> cov(ncalls);
        std::vector<size_t> done;
        for (size_t i = 0; i < ncalls; i++)
            if (rnd_u(4)) done.push_back(i);
        for (size_t k = done.size(); k > 1; k--) std::swap(done[k - 1], done[rnd_u((uint32_t)k)]);
        put(out, (uint32_t)done.size());
        for (size_t ci : done) {
            const uint32_t n = rnd_u(6) == 0 ? 0 : rnd_u(40);
            uint32_t pc = rnd_u(1000);
            for (uint32_t j = 0; j < n; j++) cov[ci].push_back(pc += 1 + rnd_u(100));
            put(out, (uint32_t)ci);
            put(out, call_num[ci]);
            put(out, (uint32_t)rnd());
            put(out, n);
            for (uint32_t v : cov[ci]) put(out, v);
        }
        const int damage = rnd_u(8);
        if (damage == 1 && !out.empty()) out.resize(rnd_u((uint32_t)out.size()));  // truncate
        if (damage == 2 && out.size() > 4) {  // random bytes anywhere
            for (int k = 0; k < 3; k++) out[rnd_u((uint32_t)out.size())] = (uint8_t)rnd();
        }
        if (damage == 3 && out.size() >= 4) {  // record count too large
            const uint32_t v = 0xFFFFFFFFu - rnd_u(3);
            memcpy(out.data(), &v, 4);
        }
        if (damage == 4 && out.size() >= 20) {  // cover size past the end
            const uint32_t v = 0x40000000u + rnd_u(100);
            memcpy(out.data() + 16, &v, 4);
        }
        if (damage == 5) {  // pure noise
            out.resize(rnd_u(200));
            for (auto &x : out) x = (uint8_t)rnd();
        }
        // the parser reads exactly out.size() bytes: a heap copy of that size
        // lets ASan catch any read past the end
        uint8_t *buf = (uint8_t *)malloc(out.size() ? out.size() : 1);
        if (!out.empty()) memcpy(buf, out.data(), out.size());
        size_t cap = rnd_u(3) == 0 ? rnd_u(60) : out.size() / 4 + 1;
        std::vector<int64_t> errnos(ncalls + 1);
        std::vector<int32_t> rcid(ncalls + 1);
        std::vector<uint32_t> rci(ncalls + 1);
        std::vector<uint64_t> roff(ncalls + 1);
        uint32_t *pcs = (uint32_t *)malloc((cap ? cap : 1) * 4);
        const int64_t r = syzcov_parse_exec_output(
            buf, out.size(), ncalls, ncalls ? call_num.data() : nullptr, callid.data(), nnum,
            errnos.data(), rcid.data(), rci.data(), roff.data(), pcs, cap);
        if (r >= 0) {
            ok++;
            CHECK((size_t)r <= ncalls);
            CHECK(roff[0] == 0);
            for (int64_t k = 0; k < r; k++) {
                CHECK(roff[k + 1] > roff[k]);
                CHECK(roff[k + 1] <= cap);
                CHECK(k == 0 || rci[k] > rci[k - 1]);
                CHECK(rci[k] < ncalls);
                if (damage == 0) {
                    const auto &c = cov[rci[k]];
                    CHECK(roff[k + 1] - roff[k] == c.size());
                    CHECK(!memcmp(pcs + roff[k], c.data(), c.size() * 4));
                    CHECK(rcid[k] == callid[call_num[rci[k]]]);
                }
            }
        } else {
            rejected++;
            CHECK(r == SYZCOV_EINVAL || r == SYZCOV_ERANGE);
        }
        free(buf);
        free(pcs);
    }
    printf("ok %d rejected %d\n", ok, rejected);
    return 0;
}
