"""GPU parity: libsyzcov's HIP kernels vs the CPU oracle (restatement of
cover/cover.go + Go sort.Sort), on the reference's KATs, quirks, seeded random
cases and synthetic corpora.  Bit-exact everywhere (integer/index work)."""
import numpy as np
import pytest

from oracle import oracle as orc
from tests.conftest import augment

pytestmark = pytest.mark.gpu

SENT = 0xFFFFFFFF


@pytest.fixture(scope="module")
def cover():
    from syzkaller_amd import cover as c
    return c


def _ops(cover):
    return {
        "difference": (cover.Difference, orc.difference),
        "symmetric_difference": (cover.SymmetricDifference, orc.symmetric_difference),
        "union": (cover.Union, orc.union),
        "intersection": (cover.Intersection, orc.intersection),
    }


@pytest.mark.parametrize("name", ["difference", "symmetric_difference", "union", "intersection"])
def test_setop_kat(cover, kat, name):
    t = kat[name]
    gpu, _ = _ops(cover)[name]
    for a, b, r in augment(t["cases"], t["symmetric"]):
        assert list(gpu(a, b)) == r, (name, a, b)


def test_canonicalize_kat(cover, kat):
    for a, _, r in augment(kat["canonicalize"]["cases"], False):
        assert list(cover.Canonicalize(a)) == r
    for a, r in kat["quirks"]["canonicalize"]:
        assert list(cover.Canonicalize(a)) == r


def test_quirk_setops(cover, kat):
    ops = _ops(cover)
    for name, a, b, r in kat["quirks"]["setops"]:
        assert list(ops[name][0](a, b)) == r, (name, a, b)


def test_minimize_kat(cover, kat):
    for case in kat["minimize"]["cases"]:
        assert cover.Minimize(case["inp"]) == case["out"], case["name"]
    for case in kat["quirks"]["minimize"]:
        assert cover.Minimize(case["inp"]) == case["out"]


def test_canonicalize_in_place_aliasing(cover):
    a = np.array([6, 1, 2, 6, 3, 3, 4, 5, 1], dtype=np.uint32)
    r = cover.Canonicalize(a)
    assert list(r) == [1, 2, 3, 4, 5, 6]
    assert np.shares_memory(r, a) and list(a[:6]) == [1, 2, 3, 4, 5, 6]


@pytest.mark.parametrize("n", [0, 1, 7, 64, 255, 256, 257, 1000, 2048, 4097, 8192, 16384, 16385,
                               40000, 65535, 100000, 300001])
def test_canonicalize_sizes(cover, n):
    rng = np.random.default_rng(n)
    for hi in (50, 1 << 20, 1 << 32):
        a = rng.integers(0, hi, size=n, dtype=np.uint64).astype(np.uint32)
        if n > 3:
            a[rng.integers(0, n, size=3)] = SENT
        assert np.array_equal(cover.Canonicalize(a.copy()), orc.canonicalize(a)), (n, hi)


def test_canonicalize_all_sentinel(cover):
    assert cover.Canonicalize(np.full(5000, SENT, np.uint32)).size == 0
    assert cover.Canonicalize(np.full(20000, SENT, np.uint32)).size == 0


def _rand_sorted(rng, n, hi, dups):
    a = np.sort(rng.integers(0, hi, size=n, dtype=np.uint64)).astype(np.uint32)
    return a if dups else np.unique(a)


@pytest.mark.parametrize("dups", [False, True])
def test_setops_random(cover, dups):
    rng = np.random.default_rng(7 + dups)
    ops = _ops(cover)
    for trial in range(60):
        na, nb = (int(x) for x in rng.integers(0, 3000, size=2))
        hi = int(rng.choice([10, 1000, 1 << 32]))
        a, b = _rand_sorted(rng, na, hi, dups), _rand_sorted(rng, nb, hi, dups)
        if trial % 5 == 0 and a.size:
            a[-1] = SENT
        for name, (g, o) in ops.items():
            assert np.array_equal(g(a, b), o(a, b)), (name, trial)


def test_setop_unsorted_rejected(cover):
    from syzkaller_amd import SyzcovError
    with pytest.raises(SyzcovError):
        cover.Union([3, 1], [2])


def test_sort_order_matches_go(cover):
    rng = np.random.default_rng(11)
    for trial in range(40):
        n = int(rng.integers(0, 20000))
        kind = trial % 4
        lens = (rng.integers(0, 8, size=n) if kind == 0 else
                rng.integers(0, 1 << 16, size=n) if kind == 1 else
                np.sort(rng.integers(0, 100, size=n)) if kind == 2 else
                rng.normal(2048, 512, size=n).astype(np.int64).clip(1, 65535))
        assert np.array_equal(cover.SortOrder(lens), orc.sort_order(lens)), trial
    # the legacy Go <= 1.18 order is the caller's to pass (no host path in the library)
    from syzkaller_amd import SyzcovError
    with pytest.raises(SyzcovError):
        cover.SortOrder(lens, orc.LEGACY)
    # C2-sized: 1M canonical lengths ~ N(2048, 512) (deep global rounds + LDS finisher)
    lens = rng.normal(2048, 512, size=1_000_000).astype(np.int64).clip(1, 65535)
    assert np.array_equal(cover.SortOrder(lens), orc.sort_order(lens))
    # nearly sorted / reversed / all-equal at scale (partialInsertionSort, reverse, partitionEqual)
    for lens in (np.sort(lens)[::-1].copy(), np.sort(lens), np.full(300_000, 7)):
        assert np.array_equal(cover.SortOrder(lens), orc.sort_order(lens))


def test_minimize_random_vs_oracle(cover):
    rng = np.random.default_rng(5)
    for trial in range(60):
        n = int(rng.integers(0, 400))
        hi = int(rng.choice([30, 500, 1 << 32]))
        covs = [orc.canonicalize(rng.integers(0, hi, size=int(rng.integers(0, 40)),
                                              dtype=np.uint64).astype(np.uint32))
                for _ in range(n)]
        assert cover.Minimize(covs) == list(orc.minimize(covs)), trial
        # Go 1.8-1.18: the caller's legacy sort.Sort order, Minimize on the GPU
        legacy = orc.sort_order([len(c) for c in covs], orc.LEGACY)
        assert cover.Minimize(covs, order=legacy) == list(orc.minimize(covs, orc.LEGACY)), trial


def test_minimize_non_canonical_covers(cover):
    """Minimize accepts raw covers (duplicates count in len, cover.go:142)."""
    rng = np.random.default_rng(9)
    for _ in range(30):
        covs = [rng.integers(0, 60, size=int(rng.integers(0, 25))).astype(np.uint32)
                for _ in range(int(rng.integers(1, 150)))]
        assert cover.Minimize(covs) == list(orc.minimize(covs))


def test_minimize_explicit_order(cover):
    covs = [[1, 2], [2, 3], [3, 4], [1, 4]]
    order = [3, 2, 1, 0]
    # processing order given by the caller's own sort.Sort
    exp = []
    seen = set()
    for i in order:
        if any(p not in seen for p in covs[i]):
            exp.append(i)
        seen.update(covs[i])
    assert cover.Minimize(covs, order=order) == exp


def test_minimize_synthetic_corpus(cover):
    off, pcs = orc.synth_corpus(0x5EED0001, 3000, mean=512, sigma=128, log2_space=16)
    coff, cpcs = orc.canonicalize_csr(off, pcs)
    exp = orc.minimize_csr(coff, cpcs)
    got = cover.MinimizeCSR(coff, cpcs)
    assert got == list(exp)
    assert np.array_equal(cover.UnionAllCSR(coff, cpcs), orc.union_fold_csr(coff, cpcs))


def test_union_all_vs_fold(cover):
    rng = np.random.default_rng(3)
    covs = [orc.canonicalize(rng.integers(0, 5000, size=int(rng.integers(0, 300))))
            for _ in range(200)]
    covs.append(np.array([7, SENT], np.uint32))
    off, p = orc.to_csr(covs)
    assert np.array_equal(cover.UnionAll(covs), orc.union_fold_csr(off, p))


def test_concurrent_callers(cover):
    """The fuzzer calls cover ops from many goroutines: per-thread streams."""
    import threading
    rng = np.random.default_rng(1)
    cases = [(_rand_sorted(rng, 500, 2000, False), _rand_sorted(rng, 700, 2000, False))
             for _ in range(32)]
    errors = []

    def run(i):
        a, b = cases[i]
        for _ in range(5):
            if not np.array_equal(cover.Union(a, b), orc.union(a, b)):
                errors.append(i)

    ts = [threading.Thread(target=run, args=(i,)) for i in range(len(cases))]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errors


@pytest.mark.parametrize("op", [0, 1, 2, 3])
def test_bitmap_and_bytemap_ops(op):
    """The bitmap / byte-map set algebra of the north star (OR = Union, AND =
    Intersection, ANDNOT = Difference, XOR = SymmetricDifference over a PC
    window, cover.go:42-79 on set operands) + popcount, against numpy and
    against the oracle's list set ops on the same sets."""
    import ctypes as C
    import torch
    from syzkaller_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(50 + op)
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    npf = [np.bitwise_or, np.bitwise_and, lambda a, b: a & ~b, np.bitwise_xor][op]
    for nwords in (1, 3, 17, 4097, (1 << 20) + 5):
        dens = rng.choice([0.01, 0.5])
        a = (rng.random(nwords * 32) < dens)
        b = (rng.random(nwords * 32) < 0.3)
        aw = np.packbits(a, bitorder="little").view(np.uint32)
        bw = np.packbits(b, bitorder="little").view(np.uint32)
        d = torch.from_numpy(aw.view(np.int32).copy()).cuda()
        src = torch.from_numpy(bw.view(np.int32).copy()).cuda()
        pop = torch.zeros(1, dtype=torch.int64, device="cuda")
        _lib.check(L.syzcov_dev_bitmap_op(op, P(d), P(src), nwords, P(pop), s), "bitmap_op")
        exp = npf(aw, bw)
        got = d.cpu().numpy().view(np.uint32)
        assert np.array_equal(got, exp), (op, nwords)
        assert int(pop.item()) == int(np.unpackbits(exp.view(np.uint8)).sum())
        if nwords == 17:  # the same sets as sorted PC lists through the oracle
            la = np.nonzero(a)[0].astype(np.uint32)
            lb = np.nonzero(b)[0].astype(np.uint32)
            ref = orc.setop({0: orc.UNION, 1: orc.INTERSECTION, 2: orc.DIFFERENCE,
                            3: orc.SYMDIFF}[op], la, lb)
            assert np.array_equal(np.nonzero(np.unpackbits(got.view(np.uint8),
                                                           bitorder="little"))[0], ref)
    for nbytes in (1, 15, 16, 33, 4099, (1 << 22) + 7):
        a = (rng.random(nbytes) < 0.4) * rng.integers(1, 256, size=nbytes)
        b = (rng.random(nbytes) < 0.4) * rng.integers(1, 256, size=nbytes)
        d = torch.from_numpy(a.astype(np.uint8)).cuda()
        src = torch.from_numpy(b.astype(np.uint8)).cuda()
        pop = torch.zeros(1, dtype=torch.int64, device="cuda")
        _lib.check(L.syzcov_dev_bytemap_op(op, P(d), P(src), nbytes, P(pop), s), "bytemap_op")
        exp = npf((a != 0).astype(np.uint8), (b != 0).astype(np.uint8)) & 1
        assert np.array_equal(d.cpu().numpy(), exp.astype(np.uint8)), (op, nbytes)
        assert int(pop.item()) == int(exp.sum())


def _minimize_in_order(covs, order):
    """cover.go:114-129 over a given processing order (Python restatement)."""
    seen, out = set(), []
    for i in order:
        c = covs[i]
        if any(int(p) not in seen for p in c):
            out.append(int(i))
        seen.update(int(p) for p in c)
    return out


def test_minimize_engine_with_caller_order(cover):
    """cover.Minimize as the Go shim calls it (its own sort.Sort order, raw
    covers with duplicates) at engine size (>= 1024 inputs): the cached
    window-mode engine takes the caller's order.  Three corpora in a row: the
    cache is reused, then grows (a wider PC window, more inputs)."""
    from syzkaller_amd import SyzcovError, _lib
    rng = np.random.default_rng(21)
    for trial, (n, hi) in enumerate(((3000, 1 << 16), (2500, 1 << 16), (5000, 1 << 21))):
        base = 0x81000000 + trial * 4096
        covs = [(base + rng.integers(0, hi, size=int(rng.integers(0, 300)))).astype(np.uint32)
                for _ in range(n)]
        legacy = orc.sort_order([len(c) for c in covs], orc.LEGACY)
        assert cover.Minimize(covs, order=legacy) == list(orc.minimize(covs, orc.LEGACY)), trial
        perm = rng.permutation(n).astype(np.int32)
        assert cover.Minimize(covs, order=perm) == _minimize_in_order(covs, perm), trial
        assert cover.Minimize(covs) == list(orc.minimize(covs)), trial
    bad = np.zeros(n, np.int32)  # not a permutation
    with pytest.raises(SyzcovError):
        cover.Minimize(covs, order=bad)
    assert _lib.lib().syzcov_pool_trim() == 0  # releases the cached engine too
    assert cover.Minimize(covs, order=perm) == _minimize_in_order(covs, perm)


@pytest.mark.parametrize("nparts", [2, 3, 8])
def test_sort_order_parts_merge_to_go_order(cover, nparts):
    """The order split over ranks (syzcov_dev_sort_order_part): every part's
    array MAX-merged is Go's order (cover.go:113), for tie-heavy lengths at
    small and C2 scale (the split happens mid-rounds at 1M, at the finisher
    for a single small segment)."""
    import ctypes as C
    import torch
    from syzkaller_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(41 + nparts)
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for n in (1, 5, 3000, 1_000_000):
        lens = rng.normal(2048, 512, size=n).astype(np.int64).clip(1, 65535)
        exp = orc.sort_order(lens)
        d_lens = torch.from_numpy(lens).cuda()
        ws = torch.empty(L.syzcov_dev_sort_ws_size(n), dtype=torch.uint8, device="cuda")
        merged = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        seen = torch.zeros(n, dtype=torch.int32, device="cuda")
        for part in range(nparts):
            out = torch.empty(n, dtype=torch.int32, device="cuda")
            _lib.check(L.syzcov_dev_sort_order_part(C.c_void_p(d_lens.data_ptr()), n, part, nparts,
                                                    C.c_void_p(out.data_ptr()),
                                                    C.c_void_p(ws.data_ptr()), ws.numel(), s),
                       "sort_order_part")
            torch.maximum(merged, out, out=merged)
            seen += (out >= 0).to(torch.int32)
        assert np.array_equal(merged.cpu().numpy(), exp), (n, nparts)
        assert int(seen.min().item()) >= 1  # every position final on some part
        if n == 1_000_000:  # the late rounds were split: most positions on one part only
            assert float((seen == 1).float().mean().item()) > 0.5


def test_bits_bytes_roundtrip():
    """The byte-map form of a bitmap (the key-mode union's uint8 MAX
    all-reduce, dist.merge_bitmap_u8): bit b of word w <-> byte 32 w + b, and
    the MAX of byte maps is the OR of the bitmaps."""
    import ctypes as C
    import torch
    from syzkaller_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(61)
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    for nwords in (1, 5, 4099, 131072):
        a = rng.random(nwords * 32) < 0.3
        b = rng.random(nwords * 32) < 0.3
        aw = torch.from_numpy(np.packbits(a, bitorder="little").view(np.int32).copy()).cuda()
        bw = torch.from_numpy(np.packbits(b, bitorder="little").view(np.int32).copy()).cuda()
        au = torch.empty(nwords * 32, dtype=torch.uint8, device="cuda")
        bu = torch.empty_like(au)
        _lib.check(L.syzcov_dev_bits_to_bytes(P(aw), nwords, P(au), s), "bits_to_bytes")
        _lib.check(L.syzcov_dev_bits_to_bytes(P(bw), nwords, P(bu), s), "bits_to_bytes")
        assert np.array_equal(au.cpu().numpy(), a.astype(np.uint8))
        m = torch.maximum(au, bu * 7)  # any nonzero byte reads back as a set bit
        out = torch.empty_like(aw)
        _lib.check(L.syzcov_dev_bytes_to_bits(P(m), nwords, P(out), s), "bytes_to_bits")
        exp = np.packbits(a | b, bitorder="little").view(np.int32)
        assert np.array_equal(out.cpu().numpy(), exp), nwords
