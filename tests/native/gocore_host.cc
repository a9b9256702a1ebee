// Host build of syzkaller_amd/csrc/gosort_core.h for the CPU test suite:
// the sequential pdqsort loop that the device sort runs on its leaves.
#define __host__
#define __device__
#include "../../syzkaller_amd/csrc/gosort_core.h"

struct Acc {
    int *idx;
    const long long *len;
    bool less(int i, int j) const { return len[idx[i]] > len[idx[j]]; }
    void swap(int i, int j) const {
        int t = idx[i];
        idx[i] = idx[j];
        idx[j] = t;
    }
};

extern "C" void gocore_sort(const long long *len, int n, int *idx) {
    for (int i = 0; i < n; i++) idx[i] = i;
    if (n <= 1) return;
    Acc d{idx, len};
    const syz::gocore::Task t{0, n, syz::gocore::bits_len(n), true, true};
    if (n <= 64)  // the device leaves' register stack
        syz::gocore::pdq_loop<Acc, 3, syz::gocore::BitStack>(d, t);
    else
        syz::gocore::pdq_loop<Acc, 64>(d, t);
}
