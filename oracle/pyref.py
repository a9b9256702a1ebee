"""Pure-Python literal restatement of cover/cover.go, Go's sort.Sort and the
manager's uniqueCover (syz-manager/html.go:213-238) and the executor's
cover_dedup (executor/executor.cc:574-587), used
only to cross-check the C oracle on small cases (two independent
transcriptions of the same published algorithms).  TEST INFRASTRUCTURE ONLY.
"""
from __future__ import annotations

SENT = 0xFFFFFFFF  # cover/cover.go:17


def canonicalize(cov):  # cover.go:28-40
    cov = sorted(int(x) for x in cov)
    out, last = [], SENT
    for pc in cov:
        if pc != last:
            last = pc
            out.append(pc)
    return out


def _foreach(c0, c1, f):  # cover.go:81-102
    res = []
    i0 = i1 = 0
    while i0 < len(c0) or i1 < len(c1):
        v0 = c0[i0] if i0 < len(c0) else SENT
        v1 = c1[i1] if i1 < len(c1) else SENT
        if v0 <= v1:
            i0 += 1
        if v1 <= v0:
            i1 += 1
        v = f(v0, v1)
        if v != SENT:
            res.append(v)
    return res


def difference(a, b):
    return _foreach(list(a), list(b), lambda v0, v1: v0 if v0 < v1 else SENT)


def symmetric_difference(a, b):
    return _foreach(list(a), list(b),
                    lambda v0, v1: v0 if v0 < v1 else (v1 if v1 < v0 else SENT))


def union(a, b):
    return _foreach(list(a), list(b), lambda v0, v1: v0 if v0 <= v1 else v1)


def intersection(a, b):
    return _foreach(list(a), list(b), lambda v0, v1: v0 if v0 == v1 else SENT)


class _MinArr:
    """minInputArray (cover.go:133-143) over (idx, len) pairs."""

    def __init__(self, lens):
        self.a = [(i, l) for i, l in enumerate(lens)]

    def less(self, i, j):
        return self.a[i][1] > self.a[j][1]

    def swap(self, i, j):
        self.a[i], self.a[j] = self.a[j], self.a[i]


def _insertion(d, a, b):
    for i in range(a + 1, b):
        j = i
        while j > a and d.less(j, j - 1):
            d.swap(j, j - 1)
            j -= 1


def _sift(d, lo, hi, first):
    root = lo
    while True:
        child = 2 * root + 1
        if child >= hi:
            return
        if child + 1 < hi and d.less(first + child, first + child + 1):
            child += 1
        if not d.less(first + root, first + child):
            return
        d.swap(first + root, first + child)
        root = child


def _heap(d, a, b):
    first, lo, hi = a, 0, b - a
    for i in range((hi - 1) // 2, -1, -1):
        _sift(d, i, hi, first)
    for i in range(hi - 1, -1, -1):
        d.swap(first, first + i)
        _sift(d, lo, i, first)


def _pdq(d, a, b, limit):
    was_bal, was_part = True, True
    while True:
        length = b - a
        if length <= 12:
            _insertion(d, a, b)
            return
        if limit == 0:
            _heap(d, a, b)
            return
        if not was_bal:
            if length >= 8:  # breakPatterns
                r = length
                modulus = 1 << length.bit_length()
                idx = a + (length // 4) * 2 - 1
                for i in range(3):
                    r ^= (r << 13) & 0xFFFFFFFFFFFFFFFF
                    r ^= r >> 7
                    r ^= (r << 17) & 0xFFFFFFFFFFFFFFFF
                    other = r & (modulus - 1)
                    if other >= length:
                        other -= length
                    d.swap(idx - 1 + i, a + other)
            limit -= 1
        # choosePivot
        swaps = [0]

        def order2(x, y):
            if d.less(y, x):
                swaps[0] += 1
                return y, x
            return x, y

        def median(x, y, z):
            x, y = order2(x, y)
            y, z = order2(y, z)
            x, y = order2(x, y)
            return y

        l = length
        i, j, k = a + l // 4, a + l // 4 * 2, a + l // 4 * 3
        if l >= 8:
            if l >= 50:
                i = median(i - 1, i, i + 1)
                j = median(j - 1, j, j + 1)
                k = median(k - 1, k, k + 1)
            j = median(i, j, k)
        pivot = j
        hint = 1 if swaps[0] == 0 else (2 if swaps[0] == 12 else 0)
        if hint == 2:
            x, y = a, b - 1
            while x < y:
                d.swap(x, y)
                x += 1
                y -= 1
            pivot = (b - 1) - (pivot - a)
            hint = 1
        if was_bal and was_part and hint == 1:
            if _partial_insertion(d, a, b):
                return
        if a > 0 and not d.less(a - 1, pivot):
            d.swap(a, pivot)
            x, y = a + 1, b - 1
            while True:
                while x <= y and not d.less(a, x):
                    x += 1
                while x <= y and d.less(a, y):
                    y -= 1
                if x > y:
                    break
                d.swap(x, y)
                x += 1
                y -= 1
            a = x
            continue
        mid, already = _partition(d, a, b, pivot)
        was_part = already
        left, right = mid - a, b - mid
        thr = length // 8
        if left < right:
            was_bal = left >= thr
            _pdq(d, a, mid, limit)
            a = mid + 1
        else:
            was_bal = right >= thr
            _pdq(d, mid + 1, b, limit)
            b = mid


def _partial_insertion(d, a, b):
    i = a + 1
    for _ in range(5):
        while i < b and not d.less(i, i - 1):
            i += 1
        if i == b:
            return True
        if b - a < 50:
            return False
        d.swap(i, i - 1)
        if i - a >= 2:
            j = i - 1
            while j >= 1:
                if not d.less(j, j - 1):
                    break
                d.swap(j, j - 1)
                j -= 1
        if b - i >= 2:
            j = i + 1
            while j < b:
                if not d.less(j, j - 1):
                    break
                d.swap(j, j - 1)
                j += 1
    return False


def _partition(d, a, b, pivot):
    d.swap(a, pivot)
    i, j = a + 1, b - 1
    while i <= j and d.less(i, a):
        i += 1
    while i <= j and not d.less(j, a):
        j -= 1
    if i > j:
        d.swap(j, a)
        return j, True
    d.swap(i, j)
    i += 1
    j -= 1
    while True:
        while i <= j and d.less(i, a):
            i += 1
        while i <= j and not d.less(j, a):
            j -= 1
        if i > j:
            break
        d.swap(i, j)
        i += 1
        j -= 1
    d.swap(j, a)
    return j, False


def go_sort_order(lens):
    """Go >= 1.19 sort.Sort(minInputArray): processing order of input indices."""
    d = _MinArr(lens)
    n = len(lens)
    if n > 1:
        _pdq(d, 0, n, n.bit_length())
    return [i for i, _ in d.a]


def minimize(covers):  # cover.go:104-131
    order = go_sort_order([len(c) for c in covers])
    covered, out = set(), []
    for idx in order:
        hit = False
        for pc in covers[idx]:
            if not hit and pc not in covered:
                hit = True
                out.append(idx)
            if hit:
                covered.add(pc)
    return out


def unique_cover(calls, covers, per_call):  # syz-manager/html.go:213-238
    total = {}
    call_cover = {}
    for c, cov in zip(calls, covers):
        if per_call and c not in call_cover:
            call_cover[c] = set()
        for pc in cov:
            pc = int(pc)
            if per_call:
                if pc in call_cover[c]:
                    continue
                call_cover[c].add(pc)
            total[pc] = total.get(pc, 0) + 1
    cov = sorted(pc for pc, n in total.items() if n == 1)
    canonicalize(list(cov))  # :236 `cover.Canonicalize(cov)`, return value ignored:
    return cov               # the full sorted slice (a lone 0xFFFFFFFF survives)


def summary_stats(calls, covers):  # syz-manager/html.go:67-99, literally
    cc = {}
    for c, cov in zip(calls, covers):
        e = cc.setdefault(c, [0, []])
        e[0] += 1
        e[1] = union(e[1], [int(x) for x in cov])
    total_unique = unique_cover(calls, covers, True)
    cov_all, rows = [], []
    for c, (count, ccov) in cc.items():
        cov_all = union(cov_all, ccov)
        rows.append((c, count, len(ccov), len(intersection(ccov, total_unique))))
    return sorted(rows), len(cov_all)


def corpus_stats(calls, covers, call):  # syz-manager/html.go:157-175 (before the sort)
    total_unique = unique_cover(calls, covers, False)
    return [(i, len(cov), len(intersection([int(x) for x in cov], total_unique)))
            for i, (c, cov) in enumerate(zip(calls, covers)) if c == call]


def cover_dedup64(cov):  # executor/executor.cc:574-587
    cov = sorted(int(x) for x in cov)
    out, last = [], 0
    for pc in cov:
        if pc == last:
            continue
        out.append(pc)
        last = pc
    return out


def parse_exec_output(out, call_num, callid_of_num):
    """ipc/ipc.go:225-291 + the fuzzer.go:456-460 walk, literally.  Raises on
    the reader's error cases (ValueError; IndexError where Go panics)."""
    import struct
    pos = 0

    def rd():
        nonlocal pos
        if len(out) - pos < 4:
            raise ValueError("short read")
        v = struct.unpack_from("<I", out, pos)[0]
        pos += 4
        return v
    ncmd = rd()
    cov = [None] * len(call_num)
    errnos = [-1] * len(call_num)
    for _ in range(ncmd):
        ci, num, err, sz = rd(), rd(), rd(), rd()
        if ci > len(cov):
            raise ValueError("call index")
        if cov[ci] is not None:  # IndexError for ci == len(cov), as Go panics
            raise ValueError("double coverage")
        if call_num[ci] != num:
            raise ValueError("call num")
        cov[ci] = [rd() for _ in range(sz)]
        errnos[ci] = err  # int(uint32) in Go
    recs = [(callid_of_num[call_num[i]], i, c) for i, c in enumerate(cov) if c]
    return errnos, recs
