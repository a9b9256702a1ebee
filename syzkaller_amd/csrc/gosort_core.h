// gosort_core.h — Go >= 1.19 sort.Sort (pdqsort, src/sort/zsortinterface.go)
// restated for the minInputArray of cover.Minimize (cover/cover.go:113,
// Less = len desc, :141-143), as __host__ __device__ building blocks over an
// accessor D { bool less(i, j); void swap(i, j); }.
//
// The device sort (gosort.hip) runs the SAME per-segment control steps
// (breakPatterns, choosePivot, partialInsertionSort, partition,
// partitionEqual) level-synchronously over disjoint segments; segments small
// enough run this file's sequential loop in one thread.  Segments never read
// or write outside [a, b) except `a-1` (a finished pivot), so processing them
// in any order reproduces Go's depth-first result exactly.
#pragma once

#include <stdint.h>

namespace syz {
namespace gocore {

enum { kUnknown = 0, kIncreasing = 1, kDecreasing = 2 };

__host__ __device__ inline int bits_len(uint64_t x) {
    int n = 0;
    while (x) {
        n++;
        x >>= 1;
    }
    return n;
}

template <class D>
__host__ __device__ inline void insertion_sort(D &d, int a, int b) {
    for (int i = a + 1; i < b; i++)
        for (int j = i; j > a && d.less(j, j - 1); j--) d.swap(j, j - 1);
}

template <class D>
__host__ __device__ inline void sift_down(D &d, int lo, int hi, int first) {
    int root = lo;
    for (;;) {
        int child = 2 * root + 1;
        if (child >= hi) return;
        if (child + 1 < hi && d.less(first + child, first + child + 1)) child++;
        if (!d.less(first + root, first + child)) return;
        d.swap(first + root, first + child);
        root = child;
    }
}

template <class D>
__host__ __device__ inline void heap_sort(D &d, int a, int b) {
    int hi = b - a;
    for (int i = (hi - 1) / 2; i >= 0; i--) sift_down(d, i, hi, a);
    for (int i = hi - 1; i >= 0; i--) {
        d.swap(a, a + i);
        sift_down(d, 0, i, a);
    }
}

template <class D>
__host__ __device__ inline void break_patterns(D &d, int a, int b) {
    const int n = b - a;
    if (n < 8) return;
    uint64_t r = (uint64_t)n;  // xorshift(length)
    const uint64_t mod = 1ull << bits_len((uint64_t)n);
    const int idx = a + (n / 4) * 2 - 1;
    for (int i = 0; i < 3; i++) {
        r ^= r << 13;
        r ^= r >> 7;
        r ^= r << 17;
        int other = (int)(r & (mod - 1));
        if (other >= n) other -= n;
        d.swap(idx - 1 + i, a + other);
    }
}

template <class D>
__host__ __device__ inline int choose_pivot(D &d, int a, int b, int *hint) {
    const int l = b - a;
    int swaps = 0;
    int i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
    auto order2 = [&](int &x, int &y) {
        if (d.less(y, x)) {
            swaps++;
            int t = x;
            x = y;
            y = t;
        }
    };
    auto median = [&](int x, int y, int z) {
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
    *hint = swaps == 0 ? kIncreasing : (swaps == 12 ? kDecreasing : kUnknown);
    return j;
}

template <class D>
__host__ __device__ inline void reverse_range(D &d, int a, int b) {
    for (int i = a, j = b - 1; i < j; i++, j--) d.swap(i, j);
}

template <class D>
__host__ __device__ inline bool partial_insertion_sort(D &d, int a, int b) {
    int i = a + 1;
    for (int step = 0; step < 5; step++) {
        while (i < b && !d.less(i, i - 1)) i++;
        if (i == b) return true;
        if (b - a < 50) return false;
        d.swap(i, i - 1);
        if (i - a >= 2)
            for (int j = i - 1; j >= 1 && d.less(j, j - 1); j--) d.swap(j, j - 1);
        if (b - i >= 2)
            for (int j = i + 1; j < b && d.less(j, j - 1); j++) d.swap(j, j - 1);
    }
    return false;
}

template <class D>
__host__ __device__ inline int partition_equal(D &d, int a, int b, int pivot) {
    d.swap(a, pivot);
    int i = a + 1, j = b - 1;
    for (;;) {
        while (i <= j && !d.less(a, i)) i++;
        while (i <= j && d.less(a, j)) j--;
        if (i > j) return i;
        d.swap(i, j);
        i++;
        j--;
    }
}

template <class D>
__host__ __device__ inline int partition(D &d, int a, int b, int pivot, bool *already) {
    d.swap(a, pivot);
    int i = a + 1, j = b - 1;
    while (i <= j && d.less(i, a)) i++;
    while (i <= j && !d.less(j, a)) j--;
    if (i > j) {
        d.swap(j, a);
        *already = true;
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
    *already = false;
    return j;
}

// The pdqsort loop entered with explicit state (the recursion of the smaller
// side is an explicit stack: depth <= bits_len(n)).
struct Task {
    int a, b, limit;
    bool wb, wp;
};

// Task stacks: an array (host), or registers (device leaves: an array indexed
// by the stack pointer would live in scratch memory, which the HIP runtime
// then keeps allocated per queue, ~100 MB each).  The parked side is the
// larger one and the loop continues on the smaller (<= half), so the depth is
// at most log2(n) (<= 5 for the 32-element leaves).
template <int N>
struct ArrayStack {
    Task e[N];
    int sp = 0;
    __host__ __device__ void push(const Task &t) { e[sp++] = t; }
    __host__ __device__ Task pop() { return e[--sp]; }
};
// Leaf stack in ONE 64-bit register: up to 3 parked tasks of 21 bits each
// (a and b relative to the leaf start, 7 bits each; limit 5 bits; the two
// flags).  A leaf of n <= 64 parks at most 3 (64 -> 31 -> 15 -> 7).  An
// array (even of named members) indexed by the stack pointer is compiled to
// scratch memory, which the HIP runtime then keeps allocated per queue.
struct BitStack {
    uint64_t bits = 0;
    int sp = 0, base = 0;
    __host__ __device__ explicit BitStack(int leaf_start) : base(leaf_start) {}
    __host__ __device__ void push(const Task &t) {
        const uint64_t e = (uint64_t)(t.a - base) | (uint64_t)(t.b - base) << 7 |
                           (uint64_t)t.limit << 14 | (uint64_t)t.wb << 19 | (uint64_t)t.wp << 20;
        bits = bits << 21 | e;
        sp++;
    }
    __host__ __device__ Task pop() {
        const uint64_t e = bits & 0x1FFFFFull;
        bits >>= 21;
        sp--;
        return Task{base + (int)(e & 127), base + (int)((e >> 7) & 127), (int)((e >> 14) & 31),
                    (bool)((e >> 19) & 1), (bool)((e >> 20) & 1)};
    }
};
template <int N>
struct ArrayStackAt : ArrayStack<N> {
    __host__ __device__ explicit ArrayStackAt(int) {}
};

template <class D, int STACK = 40, class Stack = ArrayStackAt<STACK>>
__host__ __device__ inline void pdq_loop(D &d, Task t0) {
    Stack st(t0.a);
    st.push(t0);
    while (st.sp) {
        Task t = st.pop();
        int a = t.a, b = t.b, limit = t.limit;
        bool wb = t.wb, wp = t.wp;
        for (;;) {
            const int n = b - a;
            if (n <= 12) {
                insertion_sort(d, a, b);
                break;
            }
            if (limit == 0) {
                heap_sort(d, a, b);
                break;
            }
            if (!wb) {
                break_patterns(d, a, b);
                limit--;
            }
            int hint;
            int pivot = choose_pivot(d, a, b, &hint);
            if (hint == kDecreasing) {
                reverse_range(d, a, b);
                pivot = (b - 1) - (pivot - a);
                hint = kIncreasing;
            }
            if (wb && wp && hint == kIncreasing && partial_insertion_sort(d, a, b)) break;
            if (a > 0 && !d.less(a - 1, pivot)) {
                a = partition_equal(d, a, b, pivot);
                continue;
            }
            bool already;
            const int mid = partition(d, a, b, pivot, &already);
            const int ln = mid - a, rn = b - mid, thr = n / 8;
            // Go recurses into the smaller side (fresh flags) and then loops
            // on the larger one.  The larger side's loop state is parked on
            // the stack while the smaller side runs (depth <= log2 n).
            if (ln < rn) {
                st.push(Task{mid + 1, b, limit, ln >= thr, already});
                b = mid;
            } else {
                st.push(Task{a, mid, limit, rn >= thr, already});
                a = mid + 1;
            }
            wb = true;
            wp = true;
        }
    }
}

}  // namespace gocore
}  // namespace syz
