// gosort.hip — the processing order of cover.Minimize: Go's
// sort.Sort(minInputArray) (cover/cover.go:113; Less = len desc, :141-143).
//
// sort.Sort is not stable, so equal-length inputs are ordered by the exact
// swap sequence of Go's algorithm (pdqsort in Go >= 1.19, quickSort + gap-6
// ShellSort in Go 1.8-1.18).  This file restates both over (idx, len) pairs.
//
// Stage 1 of the port: the restatement runs on the host over the D2H'd
// lengths and the order is uploaded (one 12 B/input round trip).  The
// level-synchronous device version (parallel Hoare partition by prefix sums,
// see DESIGN.md) replaces it behind the same entry point.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "common.h"

namespace syz {
namespace gosort {

struct Arr {
    int32_t *idx;
    const int64_t *len;
    bool less(long i, long j) const { return len[idx[i]] > len[idx[j]]; }
    void swap(long i, long j) const {
        int32_t t = idx[i];
        idx[i] = idx[j];
        idx[j] = t;
    }
};

static int blen(unsigned long x) { return x ? 64 - __builtin_clzl(x) : 0; }

static void insertion(const Arr &d, long a, long b) {
    for (long i = a + 1; i < b; i++)
        for (long j = i; j > a && d.less(j, j - 1); j--) d.swap(j, j - 1);
}

static void sift(const Arr &d, long lo, long hi, long first) {
    for (long root = lo;;) {
        long child = 2 * root + 1;
        if (child >= hi) return;
        if (child + 1 < hi && d.less(first + child, first + child + 1)) child++;
        if (!d.less(first + root, first + child)) return;
        d.swap(first + root, first + child);
        root = child;
    }
}

static void heap(const Arr &d, long a, long b) {
    long hi = b - a;
    for (long i = (hi - 1) / 2; i >= 0; i--) sift(d, i, hi, a);
    for (long i = hi - 1; i >= 0; i--) {
        d.swap(a, a + i);
        sift(d, 0, i, a);
    }
}

// ---- Go >= 1.19 pdqsort
struct Pivot {
    long pos;
    int hint;  // 0 unknown, 1 increasing, 2 decreasing
};

static Pivot choose_pivot(const Arr &d, long a, long b) {
    long l = b - a;
    int swaps = 0;
    long i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
    auto order2 = [&](long &x, long &y) {
        if (d.less(y, x)) {
            swaps++;
            long t = x;
            x = y;
            y = t;
        }
    };
    auto median = [&](long x, long y, long z) {
        order2(x, y);
        order2(y, z);
        order2(x, y);
        return y;
    };
    if (l >= 8) {
        if (l >= 50) {
            i = median(i - 1, i, i + 1);
            j = median(j - 1, j, j + 1);
            k = median(k - 1, k, k + 1);
        }
        j = median(i, j, k);
    }
    return {j, swaps == 0 ? 1 : (swaps == 12 ? 2 : 0)};
}

static bool partial_insertion(const Arr &d, long a, long b) {
    long i = a + 1;
    for (int step = 0; step < 5; step++) {
        while (i < b && !d.less(i, i - 1)) i++;
        if (i == b) return true;
        if (b - a < 50) return false;
        d.swap(i, i - 1);
        if (i - a >= 2)
            for (long j = i - 1; j >= 1 && d.less(j, j - 1); j--) d.swap(j, j - 1);
        if (b - i >= 2)
            for (long j = i + 1; j < b && d.less(j, j - 1); j++) d.swap(j, j - 1);
    }
    return false;
}

static void break_patterns(const Arr &d, long a, long b) {
    long n = b - a;
    if (n < 8) return;
    uint64_t r = (uint64_t)n;
    unsigned long mod = 1ul << blen((unsigned long)n);
    long idx = a + (n / 4) * 2 - 1;
    for (int i = 0; i < 3; i++) {
        r ^= r << 13;
        r ^= r >> 7;
        r ^= r << 17;
        long other = (long)((unsigned long)r & (mod - 1));
        if (other >= n) other -= n;
        d.swap(idx - 1 + i, a + other);
    }
}

static long partition_equal(const Arr &d, long a, long b, long pivot) {
    d.swap(a, pivot);
    long i = a + 1, j = b - 1;
    for (;;) {
        while (i <= j && !d.less(a, i)) i++;
        while (i <= j && d.less(a, j)) j--;
        if (i > j) return i;
        d.swap(i, j);
        i++;
        j--;
    }
}

static long partition(const Arr &d, long a, long b, long pivot, bool &already) {
    d.swap(a, pivot);
    long i = a + 1, j = b - 1;
    while (i <= j && d.less(i, a)) i++;
    while (i <= j && !d.less(j, a)) j--;
    if (i > j) {
        d.swap(j, a);
        already = true;
        return j;
    }
    d.swap(i, j);
    i++;
    j--;
    for (;;) {
        while (i <= j && d.less(i, a)) i++;
        while (i <= j && !d.less(j, a)) j--;
        if (i > j) break;
        d.swap(i, j);
        i++;
        j--;
    }
    d.swap(j, a);
    already = false;
    return j;
}

static void pdq(const Arr &d, long a, long b, int limit) {
    bool balanced = true, partitioned = true;
    for (;;) {
        long n = b - a;
        if (n <= 12) {
            insertion(d, a, b);
            return;
        }
        if (limit == 0) {
            heap(d, a, b);
            return;
        }
        if (!balanced) {
            break_patterns(d, a, b);
            limit--;
        }
        Pivot pv = choose_pivot(d, a, b);
        if (pv.hint == 2) {
            for (long i = a, j = b - 1; i < j; i++, j--) d.swap(i, j);
            pv.pos = (b - 1) - (pv.pos - a);
            pv.hint = 1;
        }
        if (balanced && partitioned && pv.hint == 1 && partial_insertion(d, a, b)) return;
        if (a > 0 && !d.less(a - 1, pv.pos)) {
            a = partition_equal(d, a, b, pv.pos);
            continue;
        }
        bool already;
        long mid = partition(d, a, b, pv.pos, already);
        partitioned = already;
        long ln = mid - a, rn = b - mid, thr = n / 8;
        if (ln < rn) {
            balanced = ln >= thr;
            pdq(d, a, mid, limit);
            a = mid + 1;
        } else {
            balanced = rn >= thr;
            pdq(d, mid + 1, b, limit);
            b = mid;
        }
    }
}

// ---- Go 1.8-1.18 quickSort
static void median3(const Arr &d, long m1, long m0, long m2) {
    if (d.less(m1, m0)) d.swap(m1, m0);
    if (d.less(m2, m1)) {
        d.swap(m2, m1);
        if (d.less(m1, m0)) d.swap(m1, m0);
    }
}

static void do_pivot(const Arr &d, long lo, long hi, long &midlo, long &midhi) {
    long m = (long)((unsigned long)(lo + hi) >> 1);
    if (hi - lo > 40) {
        long s = (hi - lo) / 8;
        median3(d, lo, lo + s, lo + 2 * s);
        median3(d, m, m - s, m + s);
        median3(d, hi - 1, hi - 1 - s, hi - 1 - 2 * s);
    }
    median3(d, lo, m, hi - 1);
    long pivot = lo, a = lo + 1, c = hi - 1;
    while (a < c && d.less(a, pivot)) a++;
    long b = a;
    for (;;) {
        while (b < c && !d.less(pivot, b)) b++;
        while (b < c && d.less(pivot, c - 1)) c--;
        if (b >= c) break;
        d.swap(b, c - 1);
        b++;
        c--;
    }
    bool protect = hi - c < 5;
    if (!protect && hi - c < (hi - lo) / 4) {
        int dups = 0;
        if (!d.less(pivot, hi - 1)) {
            d.swap(c, hi - 1);
            c++;
            dups++;
        }
        if (!d.less(b - 1, pivot)) {
            b--;
            dups++;
        }
        if (!d.less(m, pivot)) {
            d.swap(m, b - 1);
            b--;
            dups++;
        }
        protect = dups > 1;
    }
    if (protect) {
        for (;;) {
            while (a < b && !d.less(b - 1, pivot)) b--;
            while (a < b && d.less(a, pivot)) a++;
            if (a >= b) break;
            d.swap(a, b - 1);
            a++;
            b--;
        }
    }
    d.swap(pivot, b - 1);
    midlo = b - 1;
    midhi = c;
}

static void quick(const Arr &d, long a, long b, int depth) {
    while (b - a > 12) {
        if (depth == 0) {
            heap(d, a, b);
            return;
        }
        depth--;
        long mlo, mhi;
        do_pivot(d, a, b, mlo, mhi);
        if (mlo - a < b - mhi) {
            quick(d, a, mlo, depth);
            a = mhi;
        } else {
            quick(d, mhi, b, depth);
            b = mlo;
        }
    }
    if (b - a > 1) {
        for (long i = a + 6; i < b; i++)
            if (d.less(i, i - 6)) d.swap(i, i - 6);
        insertion(d, a, b);
    }
}

static void sort_host(int32_t *idx, const int64_t *len, size_t n, int variant) {
    for (size_t i = 0; i < n; i++) idx[i] = (int32_t)i;
    Arr d{idx, len};
    if (variant == 1) {
        int depth = 0;
        for (long i = (long)n; i > 0; i >>= 1) depth++;
        quick(d, 0, (long)n, 2 * depth);
    } else if (n > 1) {
        pdq(d, 0, (long)n, blen(n));
    }
}

}  // namespace gosort
}  // namespace syz

using namespace syz;

extern "C" size_t syzcov_dev_sort_ws_size(size_t n) { return 256 + n * 0; }

extern "C" int syzcov_dev_sort_order(const int64_t *lens, size_t n, int sort_variant,
                                     int32_t *order, void *ws, size_t ws_size, void *stream) {
    (void)ws;
    (void)ws_size;
    if (n == 0) return 0;
    if (!lens || !order || (sort_variant != 0 && sort_variant != 1) || n > 0x7FFFFFFF)
        return SYZCOV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    std::vector<int64_t> hl(n);
    std::vector<int32_t> ho(n);
    SYZ_HIP(hipMemcpyAsync(hl.data(), lens, n * 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    gosort::sort_host(ho.data(), hl.data(), n, sort_variant);
    SYZ_HIP(hipMemcpyAsync(order, ho.data(), n * 4, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipStreamSynchronize(s));
    return 0;
}
