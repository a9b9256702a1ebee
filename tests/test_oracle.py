"""The CPU oracle against the reference's own known-answer tables
(cover/cover_test.go:60-168) and against an independent pure-Python
transcription.  CPU only."""
import numpy as np
import pytest

from oracle import oracle as orc
from oracle import pyref
from tests.conftest import augment

OPS = {
    "difference": (orc.difference, pyref.difference),
    "symmetric_difference": (orc.symmetric_difference, pyref.symmetric_difference),
    "union": (orc.union, pyref.union),
    "intersection": (orc.intersection, pyref.intersection),
}


def _is_sorted(a):
    a = list(a)
    return all(a[i] <= a[i + 1] for i in range(len(a) - 1))


@pytest.mark.parametrize("name", list(OPS))
def test_setop_kat(kat, name):
    t = kat[name]
    c_fn, py_fn = OPS[name]
    for a, b, r in augment(t["cases"], t["symmetric"]):
        assert _is_sorted(a) and _is_sorted(b) and _is_sorted(r)
        assert list(c_fn(a, b)) == r, (name, a, b)
        assert py_fn(a, b) == r


def test_canonicalize_kat(kat):
    for a, _, r in augment(kat["canonicalize"]["cases"], False):
        assert list(orc.canonicalize(a)) == r
        assert pyref.canonicalize(a) == r


def test_minimize_kat(kat):
    for case in kat["minimize"]["cases"]:
        for variant in (orc.PDQSORT, orc.LEGACY):
            assert list(orc.minimize(case["inp"], variant)) == case["out"], case["name"]
        assert pyref.minimize(case["inp"]) == case["out"]


def test_quirks(kat):
    q = kat["quirks"]
    for a, r in q["canonicalize"]:
        assert list(orc.canonicalize(a)) == r
        assert pyref.canonicalize(a) == r
    for name, a, b, r in q["setops"]:
        assert list(OPS[name][0](a, b)) == r
        assert OPS[name][1](a, b) == r
    for case in q["minimize"]:
        assert list(orc.minimize(case["inp"])) == case["out"]
        assert pyref.minimize(case["inp"]) == case["out"]


def test_minimize_random_property():
    """TestMinimizeRandom (cover_test.go:170-205) with fixed seeds instead of
    time.Now(): Union of the kept inputs == Union of all inputs."""
    rng = np.random.default_rng(0x5EED)
    for _ in range(300):
        n = int(rng.integers(0, 20))
        covs = [list(orc.canonicalize(rng.integers(0, 100, size=int(rng.integers(0, 10)))))
                for _ in range(n)]
        total = []
        for c in covs:
            total = pyref.union(total, c)
        mini = orc.minimize(covs)
        m = []
        for idx in mini:
            m = pyref.union(m, covs[idx])
        assert m == total


def test_sort_c_vs_python():
    """Two independent transcriptions of Go's pdqsort agree, including
    tie-heavy inputs large enough to reach partition/partitionEqual,
    breakPatterns and partialInsertionSort."""
    rng = np.random.default_rng(1)
    for trial in range(200):
        n = int(rng.integers(0, 3000))
        kind = trial % 5
        if kind == 0:
            lens = rng.integers(0, 10, size=n)
        elif kind == 1:
            lens = rng.integers(0, 1 << 16, size=n)
        elif kind == 2:
            lens = np.sort(rng.integers(0, 50, size=n))  # ascending = reverse of desired
        elif kind == 3:
            lens = np.sort(rng.integers(0, 50, size=n))[::-1].copy()
            if n > 3:
                lens[rng.integers(0, n)] = 1000  # nearly sorted
        else:
            lens = np.full(n, 7)
        c = orc.sort_order(lens)
        p = pyref.go_sort_order([int(x) for x in lens])
        assert list(c) == p, (trial, n, kind)
        # it must be a valid descending order
        assert all(lens[c[i]] >= lens[c[i + 1]] for i in range(n - 1))


def test_minimize_c_vs_python():
    rng = np.random.default_rng(2)
    for _ in range(100):
        n = int(rng.integers(0, 200))
        covs = [list(orc.canonicalize(rng.integers(0, 300, size=int(rng.integers(0, 12)))))
                for _ in range(n)]
        assert list(orc.minimize(covs)) == pyref.minimize(covs)


def test_legacy_sort_is_a_sort():
    rng = np.random.default_rng(3)
    for _ in range(100):
        n = int(rng.integers(0, 2000))
        lens = rng.integers(0, 20, size=n)
        c = orc.sort_order(lens, orc.LEGACY)
        assert sorted(c) == list(range(n))
        assert all(lens[c[i]] >= lens[c[i + 1]] for i in range(n - 1))
    # n <= 6: both variants are the same stable insertion sort
    for _ in range(100):
        lens = rng.integers(0, 3, size=int(rng.integers(0, 7)))
        assert list(orc.sort_order(lens, orc.LEGACY)) == list(orc.sort_order(lens))


def test_newcov_batch_small():
    """Sequential fuzzer.go:456-480 semantics on a hand-checked batch."""
    mc = [[1, 2], [], [5]]
    flakes = [9]
    recs = [[1, 2], [2, 3], [3, 9], [9], [5, 6], [4]]
    cids = [0, 0, 0, 1, 2, 0]
    is_new, new_mc = orc.newcov_batch(mc, flakes, cids, recs)
    assert list(is_new) == [0, 1, 0, 0, 1, 1]
    assert [list(x) for x in new_mc] == [[1, 2, 3, 4], [], [5, 6]]


def test_prio_small():
    C = 5
    lens = [3, 2, 0, 5, 1]
    raw = orc.dynamic_raw(lens, C)
    exp = np.zeros((C, C), np.float32)
    for n in lens:
        for i in range(n):
            for j in range(n):
                if i != j:
                    exp[i, j] += 1
    assert np.array_equal(raw, exp)
    with pytest.raises(IndexError):
        orc.dynamic_raw([6], C)
    static = np.full((C, C), 0.5, np.float32)
    pr = orc.calculate_priorities(lens, static)
    assert pr.shape == (C, C) and np.all(pr > 0) and np.all(pr <= 0.5)
    run = orc.build_choice_table(pr, [1, 0, 1, 1, 1])
    assert np.all(run[1] == -1)  # disabled row stays nil
    assert np.all(np.diff(run[0]) >= 0)


def test_synth_deterministic():
    off, pcs = orc.synth_corpus(0x5EED0001, 50)
    off2, pcs2 = orc.synth_corpus(0x5EED0001, 50)
    assert np.array_equal(pcs, pcs2)
    lens = np.diff(off)
    assert 1000 < lens.mean() < 3000
    assert pcs.min() >= 0x81000000 and pcs.max() <= 0x84FFFFFF


def test_minimize_corpus_groups_vs_python():
    """manager.go:504-524: per-call Minimize in corpus order, restated twice."""
    rng = np.random.default_rng(21)
    for _ in range(40):
        n = int(rng.integers(0, 300))
        calls = rng.integers(0, 7, size=n)
        covs = [list(orc.canonicalize(rng.integers(0, 200, size=int(rng.integers(0, 10)))))
                for _ in range(n)]
        exp = []
        for c in sorted(set(calls.tolist())):
            members = [i for i in range(n) if calls[i] == c]
            exp += [members[k] for k in pyref.minimize([covs[i] for i in members])]
        assert orc.minimize_corpus(calls, covs) == exp


def test_new_input_is_newcov_without_flakes():
    """Manager.NewInput (manager.go:605-610) == the fuzzer's batched
    new-coverage check (fuzzer.go:456-480) with an empty flakes set, applied
    in arrival order; the sentinel-only cover is dropped by both."""
    rng = np.random.default_rng(22)
    ncalls = 5
    for _ in range(20):
        calls = rng.integers(0, ncalls, size=200)
        covs = [orc.canonicalize(rng.integers(0, 400, size=int(rng.integers(0, 8))))
                for _ in range(200)]
        covs[3] = np.array([0xFFFFFFFF], dtype=np.uint32)
        cc = {}
        acc = orc.new_inputs(cc, calls, covs)
        is_new, mc = orc.newcov_batch([[] for _ in range(ncalls)], [], calls, covs)
        assert acc == [bool(x) for x in is_new]
        for c in range(ncalls):
            assert list(mc[c]) == list(cc.get(c, []))


def test_unique_cover_restatement():
    """html.go:213-238 by hand: per input vs per call group."""
    covs = [[1, 2, 3], [3, 4], [4, 5, 5], [6]]
    calls = ["a", "a", "b", "b"]
    # per input: 3 twice, 4 twice, 5 twice (duplicate inside one cover counts)
    assert pyref.unique_cover(calls, covs, False) == [1, 2, 6]
    # per call: a = {1,2,3,4}, b = {4,5,6}: 4 is in both
    assert pyref.unique_cover(calls, covs, True) == [1, 2, 3, 5, 6]
    # html.go:236 ignores Canonicalize's return value: a lone 0xFFFFFFFF stays
    assert pyref.unique_cover(["a"], [[0xFFFFFFFF]], False) == [0xFFFFFFFF]
    assert pyref.unique_cover(["a", "b"], [[7, 0xFFFFFFFF], [7]], False) == [0xFFFFFFFF]



def test_ui_stats_restatement():
    """httpSummary / httpCorpus (html.go:67-99, :157-175) by hand."""
    covs = [[1, 2, 3], [3, 4], [4, 5], [6, 0xFFFFFFFF]]
    calls = ["a", "a", "b", "c"]
    rows, total = pyref.summary_stats(calls, covs)
    # a = {1,2,3,4}, b = {4,5}, c = {6} (Union drops the sentinel); unique per
    # call group: 1,2,3 (a), 5 (b), 6 (c) -- 4 is shared
    assert rows == [("a", 2, 4, 3), ("b", 1, 2, 1), ("c", 1, 1, 1)]
    assert total == 6
    # per input: PCs held by exactly one input (3 and 4 are held twice)
    assert pyref.corpus_stats(calls, covs, "a") == [(0, 3, 2), (1, 2, 0)]
    assert pyref.corpus_stats(calls, covs, "c") == [(3, 2, 1)]


def test_triage_oracle_kat():
    """triageInput (fuzzer.go:377-417) worked by hand: newCover [2,3,4];
    run 1 drops 4 and adds 5, run 2 drops 1, run 3 did not execute."""
    from oracle import oracle as o
    corpus = [np.zeros(0, np.uint32), np.array([1], np.uint32)]
    new, stable, fl = o.triage_batch(corpus, [9], [1], [[1, 2, 3, 4]],
                                     [[[1, 2, 3, 5], [2, 3, 4], []]])
    assert new == [3] and stable[0].tolist() == [2, 3] and fl.tolist() == [1, 4, 5, 9]
    # addInput: accepted iff something outside maxCover and flakes
    mc = [np.zeros(0, np.uint32)]
    cc = [np.zeros(0, np.uint32)]
    assert o.add_inputs(mc, cc, [5], [0, 0, 0], [[5], [1, 5], [1]]) == [False, True, False]
    assert mc[0].tolist() == [1, 5] and cc[0].tolist() == [1, 5]


def test_newcov_full_vs_list_oracle(tmp_path):
    """oracle/newcov_full.c (the bitmap restatement of fuzzer.go:456-480 that
    pins config C5 at full size) == the sorted-list restatement
    (orc_newcov_batch) on a small stream: 3 batches, flakes, 17 calls."""
    import subprocess
    import os
    seed, nrec, nb, ncalls, mean, sigma, log2 = 0x5EED0005, 1500, 3, 17, 300, 200, 12
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["make", "-s", "-C", os.path.join(root, "oracle")], check=True)
    subprocess.run([os.path.join(root, "oracle", "build", "newcov_full"), hex(seed), str(nrec),
                    str(nb), str(ncalls), str(mean), str(sigma), str(log2), "3", str(tmp_path)],
                   check=True, capture_output=True)
    is_new = np.fromfile(tmp_path / "is_new.u8", dtype=np.uint8)
    mn = np.fromfile(tmp_path / "maxcover_n.u32", dtype=np.uint32)
    mcp = np.fromfile(tmp_path / "maxcover.u32", dtype=np.uint32)
    fo, fp = orc.synth_corpus(seed, 1, 1 << (log2 - 7), 1, log2, first=1 << 40)
    flakes = orc.canonicalize(fp[:int(fo[1])])
    mc = [[] for _ in range(ncalls)]
    for b in range(nb):
        off, pcs = orc.synth_corpus(seed, nrec, mean, sigma, log2, first=b * nrec)
        c_off, c_pcs = orc.canonicalize_csr(off, pcs)
        recs = [c_pcs[c_off[i]:c_off[i + 1]] for i in range(nrec)]
        cids = orc.synth_callids(seed, nrec, ncalls, first=b * nrec)
        exp, mc = orc.newcov_batch(mc, flakes, cids, recs)
        assert np.array_equal(is_new[b * nrec:(b + 1) * nrec], exp), b
        assert 0 < exp.sum() < nrec
    assert mn.tolist() == [len(m) for m in mc]
    assert np.array_equal(mcp, np.concatenate([np.asarray(m, np.uint32) for m in mc]))


def test_cover_dedup_restatement():
    """executor.cc:574-587 (no reference test covers cover_dedup, and
    executor.cc does not build on its own: parity unpinned; the two
    restatements and numpy's unique agree, including its zero rule)."""
    kat = [([], []), ([0], []), ([0, 0], []), ([7], [7]), ([0, 0, 5, 3, 5], [3, 5]),
           ([2**64 - 1, 0, 1, 2**64 - 1], [1, 2**64 - 1]),
           ([0xffffffff81000010, 0xffffffff81000000, 0xffffffff81000010],
            [0xffffffff81000000, 0xffffffff81000010])]
    for buf, want in kat:
        assert orc.cover_dedup64(buf).tolist() == want
        assert pyref.cover_dedup64(buf) == want
    rng = np.random.default_rng(11)
    for n in (1, 2, 17, 300, 5000):
        for hi in (4, 1 << 20, None):
            buf = (rng.integers(0, 2**63, n, dtype=np.uint64) * 2 + 1 if hi is None
                   else rng.integers(0, hi, n).astype(np.uint64))
            got = orc.cover_dedup64(buf)
            u = np.unique(buf)
            assert np.array_equal(got, u[u != 0])
            assert got.tolist() == pyref.cover_dedup64(buf.tolist())
