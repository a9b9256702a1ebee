/*
 * gosort_oracle.c — restatement of Go's sort.Sort (standard library), which
 * cover.Minimize uses to order its inputs (cover/cover.go:113 with
 * minInputArray.Less = len(a[i].cov) > len(a[j].cov), cover.go:141-143).
 *
 * The standard library is a third-party dependency absent from
 * /root/reference (no Go toolchain, no go.mod: README.md:67 requires Go >= 1.7).
 * Restated here from the published algorithm:
 *   variant 0: pdqsort, src/sort/zsortinterface.go, Go >= 1.19 (default);
 *   variant 1: quickSort + gap-6 ShellSort pass, src/sort/sort.go, Go 1.8-1.18.
 * Inputs with n <= 6 (and ties-free inputs) sort identically in both variants;
 * all TestMinimize corpora (cover_test.go:104-168) have n <= 4.
 *
 * TEST INFRASTRUCTURE ONLY.
 */
#include "oracle.h"

typedef struct {
    int32_t *idx;
    const int64_t *len;
} minarr;

/* minInputArray.Less / Swap (cover/cover.go:141-143) */
static int Less(const minarr *d, long i, long j) { return d->len[d->idx[i]] > d->len[d->idx[j]]; }
static void Swap(minarr *d, long i, long j) {
    int32_t t = d->idx[i];
    d->idx[i] = d->idx[j];
    d->idx[j] = t;
}

static int bits_len(unsigned long x) {
    int n = 0;
    while (x) {
        n++;
        x >>= 1;
    }
    return n;
}

static void insertionSort(minarr *d, long a, long b) {
    for (long i = a + 1; i < b; i++)
        for (long j = i; j > a && Less(d, j, j - 1); j--) Swap(d, j, j - 1);
}

static void siftDown(minarr *d, long lo, long hi, long first) {
    long root = lo;
    for (;;) {
        long child = 2 * root + 1;
        if (child >= hi) return;
        if (child + 1 < hi && Less(d, first + child, first + child + 1)) child++;
        if (!Less(d, first + root, first + child)) return;
        Swap(d, first + root, first + child);
        root = child;
    }
}

static void heapSort(minarr *d, long a, long b) {
    long first = a, lo = 0, hi = b - a;
    for (long i = (hi - 1) / 2; i >= 0; i--) siftDown(d, i, hi, first);
    for (long i = hi - 1; i >= 0; i--) {
        Swap(d, first, first + i);
        siftDown(d, lo, i, first);
    }
}

/* ------------------------------ pdqsort ------------------------------ */
enum { unknownHint = 0, increasingHint = 1, decreasingHint = 2 };

static void order2(const minarr *d, long *a, long *b, int *swaps) {
    if (Less(d, *b, *a)) {
        (*swaps)++;
        long t = *a;
        *a = *b;
        *b = t;
    }
}

static long median(const minarr *d, long a, long b, long c, int *swaps) {
    order2(d, &a, &b, swaps);
    order2(d, &b, &c, swaps);
    order2(d, &a, &b, swaps);
    return b;
}

static long medianAdjacent(const minarr *d, long a, int *swaps) {
    return median(d, a - 1, a, a + 1, swaps);
}

static long choosePivot(const minarr *d, long a, long b, int *hint) {
    const long shortestNinther = 50;
    const int maxSwaps = 4 * 3;
    long l = b - a;
    int swaps = 0;
    long i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
    if (l >= 8) {
        if (l >= shortestNinther) {
            i = medianAdjacent(d, i, &swaps);
            j = medianAdjacent(d, j, &swaps);
            k = medianAdjacent(d, k, &swaps);
        }
        j = median(d, i, j, k, &swaps);
    }
    if (swaps == 0)
        *hint = increasingHint;
    else if (swaps == maxSwaps)
        *hint = decreasingHint;
    else
        *hint = unknownHint;
    return j;
}

static void reverseRange(minarr *d, long a, long b) {
    long i = a, j = b - 1;
    while (i < j) {
        Swap(d, i, j);
        i++;
        j--;
    }
}

static int partialInsertionSort(minarr *d, long a, long b) {
    const int maxSteps = 5;
    const long shortestShifting = 50;
    long i = a + 1;
    for (int step = 0; step < maxSteps; step++) {
        while (i < b && !Less(d, i, i - 1)) i++;
        if (i == b) return 1;
        if (b - a < shortestShifting) return 0;
        Swap(d, i, i - 1);
        if (i - a >= 2) {
            for (long j = i - 1; j >= 1; j--) { /* sic: j >= 1, as in Go */
                if (!Less(d, j, j - 1)) break;
                Swap(d, j, j - 1);
            }
        }
        if (b - i >= 2) {
            for (long j = i + 1; j < b; j++) {
                if (!Less(d, j, j - 1)) break;
                Swap(d, j, j - 1);
            }
        }
    }
    return 0;
}

static void breakPatterns(minarr *d, long a, long b) {
    long length = b - a;
    if (length >= 8) {
        uint64_t r = (uint64_t)length; /* xorshift(length) */
        unsigned long modulus = 1ul << bits_len((unsigned long)length); /* nextPowerOfTwo */
        long idx = a + (length / 4) * 2 - 1;
        for (int i = 0; i < 3; i++) {
            r ^= r << 13;
            r ^= r >> 7;
            r ^= r << 17;
            long other = (long)((unsigned long)r & (modulus - 1));
            if (other >= length) other -= length;
            Swap(d, idx - 1 + i, a + other);
        }
    }
}

static long partitionEqual(minarr *d, long a, long b, long pivot) {
    Swap(d, a, pivot);
    long i = a + 1, j = b - 1;
    for (;;) {
        while (i <= j && !Less(d, a, i)) i++;
        while (i <= j && Less(d, a, j)) j--;
        if (i > j) break;
        Swap(d, i, j);
        i++;
        j--;
    }
    return i;
}

static long partition(minarr *d, long a, long b, long pivot, int *already) {
    Swap(d, a, pivot);
    long i = a + 1, j = b - 1;
    while (i <= j && Less(d, i, a)) i++;
    while (i <= j && !Less(d, j, a)) j--;
    if (i > j) {
        Swap(d, j, a);
        *already = 1;
        return j;
    }
    Swap(d, i, j);
    i++;
    j--;
    for (;;) {
        while (i <= j && Less(d, i, a)) i++;
        while (i <= j && !Less(d, j, a)) j--;
        if (i > j) break;
        Swap(d, i, j);
        i++;
        j--;
    }
    Swap(d, j, a);
    *already = 0;
    return j;
}

static void pdqsort(minarr *d, long a, long b, int limit) {
    const long maxInsertion = 12;
    int wasBalanced = 1, wasPartitioned = 1;
    for (;;) {
        long length = b - a;
        if (length <= maxInsertion) {
            insertionSort(d, a, b);
            return;
        }
        if (limit == 0) {
            heapSort(d, a, b);
            return;
        }
        if (!wasBalanced) {
            breakPatterns(d, a, b);
            limit--;
        }
        int hint;
        long pivot = choosePivot(d, a, b, &hint);
        if (hint == decreasingHint) {
            reverseRange(d, a, b);
            pivot = (b - 1) - (pivot - a);
            hint = increasingHint;
        }
        if (wasBalanced && wasPartitioned && hint == increasingHint) {
            if (partialInsertionSort(d, a, b)) return;
        }
        if (a > 0 && !Less(d, a - 1, pivot)) {
            long mid = partitionEqual(d, a, b, pivot);
            a = mid;
            continue;
        }
        int already;
        long mid = partition(d, a, b, pivot, &already);
        wasPartitioned = already;
        long leftLen = mid - a, rightLen = b - mid;
        long balanceThreshold = length / 8;
        if (leftLen < rightLen) {
            wasBalanced = leftLen >= balanceThreshold;
            pdqsort(d, a, mid, limit);
            a = mid + 1;
        } else {
            wasBalanced = rightLen >= balanceThreshold;
            pdqsort(d, mid + 1, b, limit);
            b = mid;
        }
    }
}

/* --------------------------- legacy quickSort --------------------------- */
static void medianOfThree(minarr *d, long m1, long m0, long m2) {
    if (Less(d, m1, m0)) Swap(d, m1, m0);
    if (Less(d, m2, m1)) {
        Swap(d, m2, m1);
        if (Less(d, m1, m0)) Swap(d, m1, m0);
    }
}

static void doPivot(minarr *d, long lo, long hi, long *midlo, long *midhi) {
    long m = (long)((unsigned long)(lo + hi) >> 1);
    if (hi - lo > 40) {
        long s = (hi - lo) / 8;
        medianOfThree(d, lo, lo + s, lo + 2 * s);
        medianOfThree(d, m, m - s, m + s);
        medianOfThree(d, hi - 1, hi - 1 - s, hi - 1 - 2 * s);
    }
    medianOfThree(d, lo, m, hi - 1);
    long pivot = lo;
    long a = lo + 1, c = hi - 1;
    for (; a < c && Less(d, a, pivot); a++) {
    }
    long b = a;
    for (;;) {
        for (; b < c && !Less(d, pivot, b); b++) {
        }
        for (; b < c && Less(d, pivot, c - 1); c--) {
        }
        if (b >= c) break;
        Swap(d, b, c - 1);
        b++;
        c--;
    }
    int protect = hi - c < 5;
    if (!protect && hi - c < (hi - lo) / 4) {
        int dups = 0;
        if (!Less(d, pivot, hi - 1)) {
            Swap(d, c, hi - 1);
            c++;
            dups++;
        }
        if (!Less(d, b - 1, pivot)) {
            b--;
            dups++;
        }
        if (!Less(d, m, pivot)) {
            Swap(d, m, b - 1);
            b--;
            dups++;
        }
        protect = dups > 1;
    }
    if (protect) {
        for (;;) {
            for (; a < b && !Less(d, b - 1, pivot); b--) {
            }
            for (; a < b && Less(d, a, pivot); a++) {
            }
            if (a >= b) break;
            Swap(d, a, b - 1);
            a++;
            b--;
        }
    }
    Swap(d, pivot, b - 1);
    *midlo = b - 1;
    *midhi = c;
}

static void quickSort(minarr *d, long a, long b, int maxDepth) {
    while (b - a > 12) {
        if (maxDepth == 0) {
            heapSort(d, a, b);
            return;
        }
        maxDepth--;
        long mlo, mhi;
        doPivot(d, a, b, &mlo, &mhi);
        if (mlo - a < b - mhi) {
            quickSort(d, a, mlo, maxDepth);
            a = mhi;
        } else {
            quickSort(d, mhi, b, maxDepth);
            b = mlo;
        }
    }
    if (b - a > 1) {
        for (long i = a + 6; i < b; i++)
            if (Less(d, i, i - 6)) Swap(d, i, i - 6);
        insertionSort(d, a, b);
    }
}

void orc_sort_min_inputs(int32_t *idx, const int64_t *len, size_t n, int variant) {
    minarr d = {idx, len};
    if (variant == 1) {
        int depth = 0;
        for (long i = (long)n; i > 0; i >>= 1) depth++;
        quickSort(&d, 0, (long)n, depth * 2);
        return;
    }
    if (n <= 1) return;
    pdqsort(&d, 0, (long)n, bits_len((unsigned long)n));
}
