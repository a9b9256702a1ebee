// abi_stress.cc — the drop-in C-ABI under concurrent callers (the fuzzer
// calls the cover ops from up to 32 goroutines, syz-fuzzer/fuzzer.go:166,
// 383-386, config.go:150), built with host-side ASan + UBSan
// (tools/build_asan.sh; device code is not instrumented).
//
// usage: abi_stress THREADS ITERS
// Each thread runs ITERS rounds of mixed ops on random inputs and checks every
// result against the CPU oracle (oracle/cover_oracle.c, the checker):
//   Union / Difference / Intersection / SymmetricDifference, Canonicalize,
//   Minimize (small corpora) and, every 4th round, a larger Minimize whose
//   staging exceeds the arena keep threshold.
// Two rounds of fresh OS threads: the pooled contexts (api.cc) number at most
// THREADS and the second round reuses them; idle contexts hold at most their
// 3 x 32 MB arenas, and syzcov_pool_trim() gives those back (what remains is
// the HIP runtime's own, < 512 MB; the "hip" probe mode measures it).
// Prints OK on success.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <unistd.h>
#include <vector>

#include "../../include/syzcov.h"
#include "../../oracle/oracle.h"

static std::atomic<int> failures{0};

struct Rng {
    uint64_t s;
    uint64_t next() {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        return s;
    }
    uint32_t below(uint32_t n) { return n ? (uint32_t)(next() % n) : 0; }
};

static std::vector<uint32_t> canon_set(Rng &r, uint32_t n, uint32_t span) {
    std::vector<uint32_t> v(n);
    for (auto &x : v) x = 0x81000000u + r.below(span);
    if (r.below(9) == 0) v.push_back(0xFFFFFFFFu);
    v.resize(orc_canonicalize(v.data(), v.size()));
    return v;
}

static void fail(const char *what, int t, int it) {
    fprintf(stderr, "thread %d iter %d: %s (%s)\n", t, it, what, syzcov_last_error());
    failures++;
}

static void worker(int t, int iters) {
    Rng r{0x9E3779B97F4A7C15ull * (uint64_t)(t + 1)};
    for (int it = 0; it < iters && !failures; it++) {
        const uint32_t span = r.below(3) ? 4096 : 1u << 24;
        auto a = canon_set(r, r.below(3000), span), b = canon_set(r, r.below(3000), span);
        std::vector<uint32_t> got(a.size() + b.size() + 1), exp(a.size() + b.size() + 1);
        for (int op = 0; op < 4; op++) {
            int64_t n = op == 0   ? syzcov_difference(a.data(), a.size(), b.data(), b.size(), got.data())
                        : op == 1 ? syzcov_symmetric_difference(a.data(), a.size(), b.data(),
                                                                b.size(), got.data())
                        : op == 2 ? syzcov_union(a.data(), a.size(), b.data(), b.size(), got.data())
                                  : syzcov_intersection(a.data(), a.size(), b.data(), b.size(),
                                                        got.data());
            size_t m = orc_setop(op, a.data(), a.size(), b.data(), b.size(), exp.data());
            if (n < 0 || (size_t)n != m || memcmp(got.data(), exp.data(), m * 4)) {
                fail("set op", t, it);
                return;
            }
        }
        // Canonicalize (in place) on a raw list with duplicates
        std::vector<uint32_t> raw(r.below(5000));
        for (auto &x : raw) x = 0x81000000u + r.below(span);
        std::vector<uint32_t> raw2 = raw;
        int64_t n = syzcov_canonicalize(raw.data(), raw.size());
        size_t m = orc_canonicalize(raw2.data(), raw2.size());
        if (n < 0 || (size_t)n != m || memcmp(raw.data(), raw2.data(), m * 4)) {
            fail("canonicalize", t, it);
            return;
        }
        // Minimize: small corpora each round, a 40 MB one every 4th round
        const uint32_t ninp = it % 4 == 3 ? 5000 : 50 + r.below(200);
        const uint32_t mean = it % 4 == 3 ? 2048 : 100;
        std::vector<uint64_t> off(ninp + 1, 0);
        std::vector<uint32_t> pcs;
        for (uint32_t i = 0; i < ninp; i++) {
            auto c = canon_set(r, r.below(2 * mean), span);
            pcs.insert(pcs.end(), c.begin(), c.end());
            off[i + 1] = pcs.size();
        }
        if (pcs.empty()) pcs.push_back(0);
        std::vector<int32_t> kg(ninp), ke(ninp);
        n = syzcov_minimize(off.data(), pcs.data(), ninp, nullptr, 0, kg.data());
        m = orc_minimize(off.data(), pcs.data(), ninp, 0, ke.data());
        if (n < 0 || (size_t)n != m || memcmp(kg.data(), ke.data(), m * 4)) {
            fail("minimize", t, it);
            return;
        }
    }
}

// probe: what the HIP runtime alone keeps after a thread that made a stream
// and a 20 MB allocation has exited (argv[3] == "hip")
static void hip_only(int, int) {
    hipStream_t s;
    void *p = nullptr;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipMalloc(&p, 20 << 20);
    hipMemsetAsync(p, 0, 20 << 20, s);
    hipStreamSynchronize(s);
    hipFree(p);
    hipStreamDestroy(s);
}

int main(int argc, char **argv) {
    const int nt = argc > 1 ? atoi(argv[1]) : 32, iters = argc > 2 ? atoi(argv[2]) : 20;
    const bool hip_probe = argc > 3 && !strcmp(argv[3], "hip");
    if (hipSetDevice(0) != hipSuccess) {
        fprintf(stderr, "no device\n");
        return 1;
    }
    hipFree(nullptr);
    size_t free0 = 0, total = 0;
    hipMemGetInfo(&free0, &total);
    int64_t ctx_r0 = 0;
    for (int round = 0; round < 2; round++) {
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> th;
        for (int t = 0; t < nt; t++) th.emplace_back(hip_probe ? hip_only : worker, t + round * nt, iters);
        for (auto &x : th) x.join();
        if (failures) { fflush(stdout); _exit(1); }
        hipDeviceSynchronize();
        size_t free1 = 0;
        hipMemGetInfo(&free1, &total);
        const long long lost = (long long)free0 - (long long)free1;
        const double sec =
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        const int64_t nctx = syzcov_pool_contexts(0);
        printf("round %d: %d threads x %d iters in %.1f s, device memory held after the "
               "threads exited: %lld MB, pooled contexts %lld\n",
               round, nt, iters, sec, lost >> 20, (long long)nctx);
        fflush(stdout);
        if (hip_probe) continue;
        if (nctx > nt) {
            fprintf(stderr, "%lld contexts for %d concurrent callers\n", (long long)nctx, nt);
            { fflush(stdout); _exit(1); }
        }
        // idle contexts keep at most 3 arenas of 32 MB (+ 25% growth slack) each
        if (lost > nctx * 3 * (40ll << 20) + (512ll << 20)) {
            fprintf(stderr, "%lld MB held by %lld idle contexts\n", lost >> 20, (long long)nctx);
            { fflush(stdout); _exit(1); }
        }
        if (round == 0) {
            ctx_r0 = nctx;
        } else if (nctx != ctx_r0) {
            // a new set of OS threads reuses the pooled contexts
            fprintf(stderr, "contexts grew across thread churn: %lld -> %lld\n",
                    (long long)ctx_r0, (long long)nctx);
            { fflush(stdout); _exit(1); }
        }
    }
    if (!hip_probe) {  // trimming gives the arenas back
        syzcov_pool_trim();
        size_t free2 = 0;
        hipMemGetInfo(&free2, &total);
        const long long held = (long long)free0 - (long long)free2;
        printf("after syzcov_pool_trim: %lld MB held, pooled contexts %lld\n", held >> 20,
               (long long)syzcov_pool_contexts(0));
        fflush(stdout);
        // what the HIP runtime alone keeps after as many threads (the "hip"
        // probe mode, passed in by the test) plus 256 MB
        long long base = 256;
        if (const char *e = getenv("SYZCOV_STRESS_RUNTIME_MB")) base = atoll(e);
        if (held > ((base + 256) << 20)) { fflush(stdout); _exit(1); }
    }
    printf("OK\n");
    // no static teardown: the HIP runtime's exit-time frees trip the ASan
    // device allocator's own check (its runtime is marked unloaded by then)
    fflush(stdout);
    _exit(0);
}
