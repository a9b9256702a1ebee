"""GPU parity of the fuzzer's addInput (syz-fuzzer/fuzzer.go:344-375) and
triageInput coverage steps (:377-417, incl. the flakes update :405-415)
against the sequential oracle (oracle.add_inputs / oracle.triage_batch).
Bit-exact (integer set work)."""
import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu
S = 0xFFFFFFFF


def _state(ncalls, lo, span, universe=None):
    from syzkaller_amd.fuzzer import CoverState
    st = CoverState(ncalls, lo, span)
    if universe is not None:
        st.set_universe(universe)
    return st


def test_triage_kat():
    st = _state(2, 0, 1 << 16)
    st.corpus_add(1, [1])
    st.set_flakes([9])
    new, stable = st.triage([1], [[1, 2, 3, 4]], [[[1, 2, 3, 5], [2, 3, 4], []]])
    assert new.tolist() == [3] and stable[0].tolist() == [2, 3]
    assert st.flakes().tolist() == [1, 4, 5, 9]
    # nothing new against corpusCover + flakes: no re-executions, flakes unchanged
    new, stable = st.triage([1], [[1, 9]], [[[7], [8], [9]]])
    assert new.tolist() == [0] and stable[0].size == 0
    assert st.flakes().tolist() == [1, 4, 5, 9]
    st.close()


def _rand_cover(rng, pool, n):
    return np.unique(rng.choice(pool, size=n)).astype(np.uint32)


@pytest.mark.parametrize("mode", ["window", "keys"])
def test_triage_random_vs_oracle(mode):
    rng = np.random.default_rng(51)
    ncalls, lo, span = 11, 0x81000000, 1 << 20
    pool = np.unique(rng.integers(lo, lo + span, size=30000)).astype(np.uint32)
    st = _state(ncalls, lo, span, pool if mode == "keys" else None)
    corpus = [_rand_cover(rng, pool, int(rng.integers(0, 3000))) for _ in range(ncalls)]
    for c in range(ncalls):
        st.corpus_add(c, corpus[c])
    flakes = _rand_cover(rng, pool, 500)
    st.set_flakes(flakes)
    for batch in range(3):
        n = 300
        cids = rng.integers(0, ncalls, size=n)
        covers, runs = [], []
        for t in range(n):
            cov = _rand_cover(rng, pool[: int(rng.choice([200, pool.size]))],
                              int(rng.integers(0, 2500)))
            if rng.random() < 0.1:
                cov = np.append(cov, np.uint32(S))
            rr = []
            for _ in range(3):
                u = rng.random()
                if u < 0.15:
                    r = np.zeros(0, np.uint32)  # not executed
                elif u < 0.2:
                    r = np.array([S], np.uint32)  # executed, only the sentinel
                elif u < 0.5:
                    r = cov.copy()  # stable
                else:  # flaky: drop some, add some
                    keep = cov[(cov != S) & (rng.random(cov.size) < 0.9)]
                    r = np.union1d(keep, _rand_cover(rng, pool, 20)).astype(np.uint32)
                rr.append(r)
            covers.append(cov)
            runs.append(rr)
        exp_new, exp_stable, flakes = orc.triage_batch(corpus, flakes, cids, covers, runs)
        got_new, got_stable = st.triage(cids, covers, runs)
        assert got_new.tolist() == exp_new, batch
        for t in range(n):
            assert np.array_equal(got_stable[t], exp_stable[t]), (batch, t)
        assert np.array_equal(st.flakes(), flakes), batch
        # the caller minimizes, then corpusCover[call] |= minCover (:451)
        for t in range(n):
            if exp_stable[t].size:
                c = int(cids[t])
                corpus[c] = orc.union(corpus[c], exp_stable[t])
                st.corpus_add(c, exp_stable[t])
    for c in range(ncalls):
        assert np.array_equal(st.corpus_cover(c), corpus[c])
    st.close()


def test_triage_rejects_bad_batches():
    from syzkaller_amd import SyzcovError
    lo, span = 0x81000000, 1 << 16
    st = _state(3, lo, span)
    st.set_flakes([lo + 1])
    cov = [lo + 2, lo + 3]
    for runs in ([[lo + 3, lo + 2], [], []],        # unsorted run
                 [[lo + span + 5], [], []]):       # run PC outside the window
        with pytest.raises(SyzcovError):
            st.triage([0], [cov], [runs])
        assert st.flakes().tolist() == [lo + 1]  # rejected batch: flakes unchanged
    with pytest.raises(SyzcovError):
        st.triage([3], [cov], [[[], [], []]])  # call id out of range
    st.close()


@pytest.mark.parametrize("mode", ["window", "keys"])
def test_add_inputs_vs_oracle(mode):
    rng = np.random.default_rng(52)
    ncalls, lo, span = 9, 0x81000000, 1 << 20
    pool = np.unique(rng.integers(lo, lo + span, size=20000)).astype(np.uint32)
    st = _state(ncalls, lo, span, pool if mode == "keys" else None)
    maxc = [np.zeros(0, np.uint32) for _ in range(ncalls)]
    corp = [np.zeros(0, np.uint32) for _ in range(ncalls)]
    flakes = _rand_cover(rng, pool, 800)
    st.set_flakes(flakes)
    for batch in range(3):
        n = 2000
        cids = rng.integers(0, ncalls, size=n)
        covers = []
        for _ in range(n):
            cov = _rand_cover(rng, pool[: int(rng.choice([100, pool.size]))],
                              int(rng.integers(0, 200)))
            if rng.random() < 0.05:
                cov = np.append(cov, np.uint32(S))
            covers.append(cov)
        exp = orc.add_inputs(maxc, corp, flakes, cids, covers)
        got = st.add_inputs(cids, covers)
        assert got.astype(bool).tolist() == exp, batch
        for c in range(ncalls):
            assert np.array_equal(st.max_cover(c), maxc[c]), (batch, c)
            assert np.array_equal(st.corpus_cover(c), corp[c]), (batch, c)
    st.close()
