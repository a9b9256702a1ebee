"""Python mirror of syzkaller's `cover` package (cover/cover.go), backed by
libsyzcov's HIP kernels.  Same names, argument meaning and results as the Go
API the cgo shim keeps:

    Cover, Copy, RestorePC, Canonicalize, Difference, SymmetricDifference,
    Union, Intersection, Minimize

plus corpus-level batch entry points (UnionAll, SortOrder) used by the
manager-side callers.  Empty results are empty uint32 arrays (Go's nil).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, lib

SENT = 0xFFFFFFFF
Cover = np.ndarray  # canonical: sorted, unique uint32


def _u32(x) -> np.ndarray:
    a = np.asarray(x)
    if a.dtype != np.uint32:
        a = a.astype(np.uint32)
    return np.ascontiguousarray(a)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def Copy(cov) -> np.ndarray:  # cover.go:19-21
    return _u32(cov).copy()


def RestorePC(pc: int, base: int) -> int:  # cover.go:23-25
    return int(lib().syzcov_restore_pc(pc & 0xFFFFFFFF, base & 0xFFFFFFFF))


def Canonicalize(cov) -> np.ndarray:
    """cover.go:27-40.  If `cov` is a contiguous uint32 numpy array it is
    sorted/de-duplicated IN PLACE and the returned array is a view of its
    prefix (the reference's aliasing, relied on by html.go:236)."""
    a = cov if (isinstance(cov, np.ndarray) and cov.dtype == np.uint32
                and cov.flags.c_contiguous and cov.flags.writeable) else _u32(cov).copy()
    if a.size == 0:
        return a[:0]
    n = check(lib().syzcov_canonicalize(_ptr(a), a.size), "Canonicalize")
    return a[:n]


def _setop(fn, name, a, b, cap):
    a, b = _u32(a), _u32(b)
    out = np.empty(max(cap(a.size, b.size), 1), dtype=np.uint32)
    n = check(fn(_ptr(a), a.size, _ptr(b), b.size, _ptr(out)), name)
    return out[:n]


def Difference(cov0, cov1) -> np.ndarray:  # cover.go:42-49
    return _setop(lib().syzcov_difference, "Difference", cov0, cov1, lambda x, y: x)


def SymmetricDifference(cov0, cov1) -> np.ndarray:  # cover.go:51-61
    return _setop(lib().syzcov_symmetric_difference, "SymmetricDifference", cov0, cov1,
                  lambda x, y: x + y)


def Union(cov0, cov1) -> np.ndarray:  # cover.go:63-70
    return _setop(lib().syzcov_union, "Union", cov0, cov1, lambda x, y: x + y)


def Intersection(cov0, cov1) -> np.ndarray:  # cover.go:72-79
    return _setop(lib().syzcov_intersection, "Intersection", cov0, cov1, lambda x, y: min(x, y))


def to_csr(corpus):
    lens = np.fromiter((len(c) for c in corpus), dtype=np.uint64, count=len(corpus))
    off = np.zeros(len(corpus) + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    if len(corpus) and off[-1] > 0:
        pcs = np.concatenate([_u32(c) for c in corpus])
    else:
        pcs = np.zeros(1, dtype=np.uint32)
    return off, _u32(pcs)


def SortOrder(lens, variant: int = 0) -> np.ndarray:
    """Go sort.Sort(minInputArray) processing order (cover.go:113)."""
    lens = np.ascontiguousarray(np.asarray(lens, dtype=np.int64))
    order = np.empty(max(lens.size, 1), dtype=np.int32)
    if lens.size:
        check(lib().syzcov_sort_order(_ptr(lens), lens.size, variant, _ptr(order)), "SortOrder")
    return order[:lens.size]


def MinimizeCSR(off, pcs, order=None, variant: int = 0) -> list:
    off = np.ascontiguousarray(off, dtype=np.uint64)
    pcs = _u32(pcs)
    n = off.size - 1
    if n <= 0:
        return []
    out = np.empty(n, dtype=np.int32)
    op = None
    if order is not None:
        order = np.ascontiguousarray(order, dtype=np.int32)
        op = _ptr(order)
    k = check(lib().syzcov_minimize(_ptr(off), _ptr(pcs), n, op, variant, _ptr(out)), "Minimize")
    return out[:k].tolist()


def Minimize(corpus, order=None, variant: int = 0) -> list:
    """cover.go:104-131: indices of the kept inputs in processing order."""
    off, pcs = to_csr(corpus)
    return MinimizeCSR(off, pcs, order, variant)


def UnionAllCSR(off, pcs) -> np.ndarray:
    off = np.ascontiguousarray(off, dtype=np.uint64)
    pcs = _u32(pcs)
    n = off.size - 1
    out = np.empty(max(int(off[-1] - off[0]) if n > 0 else 0, 1), dtype=np.uint32)
    if n <= 0:
        return out[:0]
    k = check(lib().syzcov_union_all(_ptr(off), _ptr(pcs), n, _ptr(out)), "UnionAll")
    return out[:k]


def UnionAll(corpus) -> np.ndarray:
    """The `total = Union(total, cov)` fold over a corpus, in one pass."""
    return UnionAllCSR(*to_csr(corpus))


def MinimizeCorpus(calls, corpus, variant: int = 0) -> list:
    """Manager.minimizeCorpus's grouping + per-call cover.Minimize
    (syz-manager/manager.go:504-524) in one engine call: kept corpus indices,
    groups in ascending call value (the reference's group order is Go map
    order, i.e. random), each group in its Minimize output order."""
    off, pcs = to_csr(corpus)
    n = off.size - 1
    if n <= 0:
        return []
    cid = np.ascontiguousarray(np.asarray(calls, dtype=np.int32))
    if cid.size != n:
        raise ValueError("one call id per corpus input")
    out = np.empty(n, dtype=np.int32)
    k = check(lib().syzcov_minimize_corpus(_ptr(cid), _ptr(off), _ptr(pcs), n, variant,
                                           _ptr(out)), "MinimizeCorpus")
    return out[:k].tolist()


def UniqueCover(corpus, calls=None) -> np.ndarray:
    """Manager.uniqueCover (syz-manager/html.go:213-238): PCs counted exactly
    once; calls=None is uniqueCover(false) (every occurrence counts), a call
    key per input is uniqueCover(true) (once per call group)."""
    off, pcs = to_csr(corpus)
    n = off.size - 1
    out = np.empty(max(int(off[-1]) if n > 0 else 0, 1), dtype=np.uint32)
    if n <= 0:
        return out[:0]
    cp = None
    if calls is not None:
        cid = np.ascontiguousarray(np.asarray(calls, dtype=np.int32))
        if cid.size != n:
            raise ValueError("one call key per corpus input")
        cp = _ptr(cid)
    k = check(lib().syzcov_unique_cover(cp, _ptr(off), _ptr(pcs), n, _ptr(out)), "UniqueCover")
    return out[:k]


def UIStats(corpus, calls, ncalls: int):
    """The manager UI's coverage numbers (syz-manager/html.go) in one device
    call over canonical covers: per call group g (calls[i] in [0, ncalls)) the
    input count, len(Union of its covers) and len(Intersection(that union,
    uniqueCover(true))) of httpSummary (:67-99); per input
    len(Intersection(cover, uniqueCover(false))) of httpCorpus (:157-175);
    and the total cover.  Returns (inputs, cover, unique_cover,
    input_unique, total)."""
    off, pcs = to_csr(corpus)
    n = off.size - 1
    cid = np.ascontiguousarray(np.asarray(calls, dtype=np.int32))
    if cid.size != max(n, 0):
        raise ValueError("one call group per corpus input")
    inputs, cov, ucov = (np.zeros(max(ncalls, 1), dtype=np.uint32) for _ in range(3))
    inu = np.zeros(max(n, 1), dtype=np.uint32)
    if n <= 0:
        return inputs[:ncalls], cov[:ncalls], ucov[:ncalls], inu[:0], 0
    total = check(lib().syzcov_ui_stats(_ptr(cid), _ptr(off), _ptr(pcs), n, ncalls, _ptr(inputs),
                                        _ptr(cov), _ptr(ucov), _ptr(inu)), "UIStats")
    return inputs[:ncalls], cov[:ncalls], ucov[:ncalls], inu[:n], int(total)
