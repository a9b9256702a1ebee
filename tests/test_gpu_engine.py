"""GPU parity of the device-resident corpus pipeline (engine.CorpusEngine) and
of the synthetic generator, the priorities path and the fuzzer new-coverage
check, against the CPU oracle."""
import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available()
    return t


def _to_np_u32(t):
    return t.cpu().numpy().view(np.uint32)


def test_synth_matches_cpu_twin(torch):
    from syzkaller_amd.engine import synth_corpus, synth_universe
    for uniform, x86 in ((False, False), (True, False), (False, True), (True, True)):
        off, pcs, lens, total = synth_corpus(300, 0x5EED0001, first=1000, uniform=uniform,
                                             x86=x86)
        o_off, o_pcs = orc.synth_corpus(0x5EED0001, 300, first=1000, uniform=uniform, x86=x86)
        assert np.array_equal(off.cpu().numpy().astype(np.uint64), o_off)
        assert np.array_equal(_to_np_u32(pcs)[:total], o_pcs[:total])
    for x86 in (False, True):
        assert np.array_equal(_to_np_u32(synth_universe(14, 0x5EED0001, x86=x86)),
                              orc.synth_universe(0x5EED0001, 14, x86=x86))


@pytest.mark.parametrize("layout", [0, 1], ids=["csr", "aligned"])
@pytest.mark.parametrize("n,mean,sigma,log2", [(4000, 2048, 512, 22), (3000, 300, 200, 12),
                                               (500, 9000, 6000, 20)])
def test_engine_step_vs_oracle(torch, n, mean, sigma, log2, layout):
    """Window mode against the oracle, canonical lists in CSR slots or in the
    line-aligned layout (every (input, range) sub-run on its own lines); the
    500-input case holds inputs past the wave kernels (> 8189 and > 16384
    PCs: the workgroup paths, whose output is spread to the aligned starts)."""
    from syzkaller_amd.engine import CorpusEngine, synth_corpus, synth_window
    seed = 0x5EED0002
    off, raw, lens, total = synth_corpus(n, seed, mean=mean, sigma=sigma, log2_space=log2)
    lo, span = synth_window(log2)
    eng = CorpusEngine(n, total, int(lens.max().item()), lo, span, canon_layout=layout)
    assert bool(eng.canon_align_k) == (layout == 1 and eng.nrange > 1)
    res = eng.step(off, raw, n)
    # oracle
    o_off, o_pcs = orc.synth_corpus(seed, n, mean=mean, sigma=sigma, log2_space=log2)
    c_off, c_pcs = orc.canonicalize_csr(o_off, o_pcs)
    # canonical covers, per input, in their CSR slots
    canon = _to_np_u32(eng.canonical_pcs(off, n))
    new_len = eng.new_len[:n].cpu().numpy()
    offs = off.cpu().numpy()
    assert np.array_equal(new_len, np.diff(c_off).astype(np.int32))
    for i in range(0, n, max(1, n // 50)):
        assert np.array_equal(canon[offs[i]:offs[i] + new_len[i]], c_pcs[c_off[i]:c_off[i + 1]])
    exp_kept = orc.minimize_csr(c_off, c_pcs)
    assert res.n_kept == len(exp_kept)
    assert res.kept_idx.cpu().numpy().tolist() == list(exp_kept)
    exp_union = orc.union_fold_csr(c_off, c_pcs)
    assert res.n_union == exp_union.size
    assert np.array_equal(_to_np_u32(res.union), exp_union)
    assert res.max_cover == exp_union.size
    # second step: maxCover is already saturated by the same corpus
    res2 = eng.step(off, raw, n)
    assert res2.kept_idx.cpu().numpy().tolist() == list(exp_kept)
    assert res2.max_cover == exp_union.size


@pytest.mark.parametrize("rec_cap", [64, 64 * 300, 64 * 5000])
def test_engine_record_overflow(torch, rec_cap):
    """Records overflowing their region (all regions at 64, some at 64 * 300)
    take the exact fallbacks: same kept list and union, and first_w is left
    all INT32_MAX (a second step gives the same result)."""
    from syzkaller_amd.engine import INT32_MAX, CorpusEngine, synth_corpus, synth_window
    n, seed, log2 = 3000, 0x5EED0007, 14
    off, raw, lens, total = synth_corpus(n, seed, mean=400, sigma=150, log2_space=log2)
    lo, span = synth_window(log2)
    eng = CorpusEngine(n, total, int(lens.max().item()), lo, span, rec_cap=rec_cap)
    o_off, o_pcs = orc.synth_corpus(seed, n, mean=400, sigma=150, log2_space=log2)
    c_off, c_pcs = orc.canonicalize_csr(o_off, o_pcs)
    exp_kept = list(orc.minimize_csr(c_off, c_pcs))
    exp_union = orc.union_fold_csr(c_off, c_pcs)
    for _ in range(2):
        res = eng.step(off, raw, n)
        assert res.kept_idx.cpu().numpy().tolist() == exp_kept
        assert np.array_equal(_to_np_u32(res.union), exp_union)
        assert bool((eng.first == INT32_MAX).all().item())
    if rec_cap == 64:
        assert int(eng.rec_cnt.item()) > rec_cap  # the fallback path ran


def test_engine_sentinel_window(torch):
    """Window touching 0xFFFFFFFF: inputs made only of the sentinel canonicalize
    to empty, otherwise it is an ordinary PC (cover.go:36-52, 104-131)."""
    from syzkaller_amd.engine import CorpusEngine
    rng = np.random.default_rng(21)
    lo, span = 0xFFFF0000, 1 << 16
    covers = []
    for i in range(700):
        l = int(rng.integers(0, 400))
        c = rng.integers(0, 1 << 16, size=l, dtype=np.uint64) | np.uint64(0xFFFF0000)
        if i % 7 == 0:
            c = np.full(int(rng.integers(1, 5)), 0xFFFFFFFF, np.uint64)
        elif i % 5 == 0:
            c = np.concatenate([c, [0xFFFFFFFF] * 3])
        covers.append(c.astype(np.uint32))
    lens = np.array([len(c) for c in covers], np.int64)
    o_off = np.zeros(len(covers) + 1, np.uint64)
    o_off[1:] = np.cumsum(lens)
    o_pcs = np.concatenate(covers + [np.zeros(1, np.uint32)])
    n = len(covers)
    off = torch.from_numpy(o_off.astype(np.int64)).cuda()
    raw = torch.from_numpy(o_pcs.view(np.int32)).cuda()
    eng = CorpusEngine(n, int(lens.sum()), int(lens.max()), lo, span)
    res = eng.step(off, raw, n)
    c_off, c_pcs = orc.canonicalize_csr(o_off, o_pcs[:int(lens.sum())])
    assert np.array_equal(eng.new_len[:n].cpu().numpy(), np.diff(c_off).astype(np.int32))
    assert res.kept_idx.cpu().numpy().tolist() == list(orc.minimize_csr(c_off, c_pcs))
    assert np.array_equal(_to_np_u32(res.union), orc.union_fold_csr(c_off, c_pcs))


def test_sharded_engine_world1(torch):
    """The RCCL path (bits->bytes MAX all-reduce, all-gather of lengths, MIN
    all-reduce of first[], MAX of kept) at world size 1, in a subprocess."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "gpu_dist_check.py")],
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr


def test_sharded_engine_two_ranks(torch):
    """Two ranks of the sharded range engine on one GPU (gloo collectives
    staged through the host): covered OR merge, first MIN merge over the
    merged dictionary, kept MAX merge, against the single-GPU engine."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "gpu_dist_multi.py"), "2"],
                       capture_output=True, text=True, timeout=115)
    assert r.returncode == 0 and r.stdout.count("OK") == 2, r.stdout + r.stderr


def test_sharded_error_reaches_every_rank(torch):
    """Key mode, two ranks on one GPU: a non-universe PC on ONE shard fails
    the step on EVERY rank (its aliased first covers went into the MIN merge);
    a step abandoned after pass 1 does not poison the next one."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "gpu_dist_err.py"), "2"],
                       capture_output=True, text=True, timeout=160)
    assert r.returncode == 0 and r.stdout.count("OK") == 2, r.stdout + r.stderr


def test_engine_properties_large(torch):
    """Size-independent properties at 200k inputs: union(kept) == union(all),
    kept order follows non-increasing canonical length, first kept = rank 0."""
    from syzkaller_amd import cover
    from syzkaller_amd.engine import CorpusEngine, synth_corpus, synth_window
    n = 200_000
    off, raw, lens, total = synth_corpus(n, 0x5EED0003, mean=256, sigma=64, log2_space=20)
    lo, span = synth_window(20)
    eng = CorpusEngine(n, total, int(lens.max().item()), lo, span)
    res = eng.step(off, raw, n)
    kept = res.kept_idx.cpu().numpy()
    new_len = eng.new_len[:n].cpu().numpy()
    assert np.all(np.diff(new_len[kept].astype(np.int64)) <= 0)
    order = eng.order[:n].cpu().numpy()
    assert kept[0] == order[0]
    canon = _to_np_u32(eng.canonical_pcs(off, n))
    offs = off.cpu().numpy()
    kept_union = np.unique(np.concatenate([canon[offs[i]:offs[i] + new_len[i]] for i in kept]))
    assert np.array_equal(kept_union, _to_np_u32(res.union))
    # order equals Go's sort over the canonical lengths
    assert np.array_equal(order, orc.sort_order(new_len.astype(np.int64)))
    assert np.array_equal(cover.SortOrder(new_len), order)


def test_prio_positional_vs_oracle(torch):
    from syzkaller_amd import prio
    rng = np.random.default_rng(4)
    for C, nprog in ((40, 500), (300, 2000), (1170, 3000)):
        lens = rng.integers(0, min(C, 60) + 1, size=nprog)
        corpus = [rng.integers(0, C, size=int(l)).tolist() for l in lens]
        static = rng.uniform(0.1, 1.0, size=(C, C)).astype(np.float32)
        got, raw = prio.CalculatePriorities(corpus, static, return_raw=True)
        exp_raw = orc.dynamic_raw(lens, C)
        assert np.array_equal(raw.astype(np.float32), exp_raw)
        exp = orc.calculate_priorities(lens, static)
        np.testing.assert_allclose(got, exp, rtol=1e-6, atol=0)  # north-star tolerance
        assert np.array_equal(got, exp)  # and in fact bit-exact


@pytest.mark.parametrize("C,nprog,maxlen", [(300, 700, 300), (1170, 300, 1170), (129, 5000, 128),
                                             (200, 1, 0)])
def test_prio_positional_active_rows(torch, C, nprog, maxlen):
    """Positional counts over the active keys only (roundup(max len, 128)
    rows, partial tiles + reduction, colsum from the length histogram) at
    the edges: max len = C (active block past C), 128/129, empty programs."""
    from syzkaller_amd import prio
    rng = np.random.default_rng(C + nprog)
    lens = rng.integers(0, maxlen + 1, size=nprog)
    lens[0] = maxlen
    corpus = [[0] * int(l) for l in lens]
    static = rng.uniform(0.1, 1.0, size=(C, C)).astype(np.float32)
    got, raw = prio.CalculatePriorities(corpus, static, return_raw=True)
    assert np.array_equal(raw.astype(np.float32), orc.dynamic_raw(lens, C))
    assert np.array_equal(got, orc.calculate_priorities(lens, static))


def test_static_prio_vs_oracle(torch):
    """calcStaticPriorities over all sys/*.txt calls (1170) on the GPU vs the
    float32 restatement (same ascending-id summation order): bit-exact."""
    from syzkaller_amd import prio
    st = prio.StaticPriorities()
    exp = orc.static_prio(prio.sys_table())
    assert st.shape == (1170, 1170)
    np.testing.assert_allclose(st, exp, rtol=1e-6, atol=0)
    assert np.array_equal(st, exp)
    # and the default CalculatePriorities path multiplies it in (prio.go:32-36)
    rng = np.random.default_rng(2)
    lens = rng.integers(1, 40, size=500)
    corpus = [[0] * int(l) for l in lens]
    got = prio.CalculatePriorities(corpus)
    assert np.array_equal(got, orc.calculate_priorities(lens, exp))


def test_prio_by_id_vs_numpy(torch):
    from syzkaller_amd import prio
    rng = np.random.default_rng(8)
    C, nprog = 200, 1500
    corpus = [rng.integers(0, C, size=int(rng.integers(0, 40))).tolist() for _ in range(nprog)]
    A = np.zeros((nprog, C), np.int64)
    for p, calls in enumerate(corpus):
        for c in calls:
            A[p, c] += 1
    D = A.T @ A - np.diag(A.sum(0))
    _, raw = prio.CalculatePriorities(corpus, None, ncalls=C, key_mode=1, return_raw=True)
    assert np.array_equal(raw.astype(np.int64), D)


def test_prio_too_long_program(torch):
    from syzkaller_amd import SyzcovError, prio
    with pytest.raises(SyzcovError):
        prio.CalculatePriorities([[0] * 11], None, ncalls=10)


def test_normalize_and_choice_table(torch):
    from syzkaller_amd import prio
    rng = np.random.default_rng(6)
    C = 257
    p = rng.integers(0, 50, size=(C, C)).astype(np.float32)
    p[3] = 0  # all-zero row -> 1
    assert np.array_equal(prio.normalizePrio(p), orc.normalize_prio(p))
    pr = orc.normalize_prio(p)
    en = (rng.random(C) < 0.7).astype(np.uint8)
    ct = prio.BuildChoiceTable(pr, en)
    exp = orc.build_choice_table(pr, en)
    for i in range(C):
        if en[i]:
            assert np.array_equal(ct.run[i], exp[i])
        else:
            assert ct.run[i] is None
    import random
    r = random.Random(0)
    i = next(i for i in range(C) if en[i])
    for _ in range(100):
        assert ct.enabled[ct.Choose(r, i)]


def test_choose_batch(torch):
    """Batched ChoiceTable.Choose (prio.go:230-249): for given draws x the
    device search equals sort.SearchInts on the row (bisect_left), with the
    reference's reject (-1) and uniform-fallback (-2) cases."""
    import random
    from syzkaller_amd import SyzcovError, prio
    rng = np.random.default_rng(8)
    C = 1170
    p = rng.integers(0, 50, size=(C, C)).astype(np.float32)
    pr = orc.normalize_prio(p)
    en = (rng.random(C) < 0.6).astype(np.uint8)
    ct = prio.BuildChoiceTable(pr, en)
    exp_run = orc.build_choice_table(pr, en)
    nq = 200_000
    calls = rng.integers(-1, C, size=nq).astype(np.int32)
    x = np.zeros(nq, dtype=np.int64)
    exp = np.full(nq, -2, dtype=np.int32)
    for k in range(nq):
        c = calls[k]
        if c >= 0 and en[c]:
            row = exp_run[c]
            x[k] = rng.integers(0, row[-1])
            # exact hits on a run value pick its first index (SearchInts)
            if k % 97 == 0 and row[0] < row[-1]:
                v = row[rng.integers(0, C - 1)]
                x[k] = v if v < row[-1] else row[0]
            i = int(np.searchsorted(row, x[k], side="left"))
            exp[k] = i if en[i] else -1
    got = ct.choose_draws(calls, x)
    assert np.array_equal(got, exp)
    assert (got == -1).any() and (got >= 0).any() and (got == -2).any()
    c0 = next(c for c in range(C) if en[c])
    with pytest.raises(SyzcovError):  # outside r.Intn's range
        ct.choose_draws([c0], [exp_run[c0][-1]])
    with pytest.raises(SyzcovError):
        ct.choose_draws([C], [0])
    picks = ct.choose_batch(random.Random(1), [c0] * 500 + [-1] * 20)
    assert all(ct.enabled[i] for i in picks)


def test_newcov_batch_vs_sequential(torch):
    from syzkaller_amd.fuzzer import CoverState
    rng = np.random.default_rng(12)
    ncalls, lo, span = 30, 0x81000000, 1 << 16
    st = CoverState(ncalls, lo, span)
    mc = [[] for _ in range(ncalls)]
    for c in range(0, ncalls, 3):
        init = np.unique(rng.integers(lo, lo + span, size=200)).astype(np.uint32)
        st.add(c, init)
        mc[c] = init
    flakes = np.unique(rng.integers(lo, lo + span, size=300)).astype(np.uint32)
    st.set_flakes(flakes)
    for batch in range(4):
        nrec = 3000
        cids = rng.integers(0, ncalls, size=nrec)
        recs = [np.unique(rng.integers(lo, lo + int(rng.choice([512, span])),
                                       size=int(rng.integers(0, 60)))).astype(np.uint32)
                for _ in range(nrec)]
        exp_new, mc = orc.newcov_batch(mc, flakes, cids, recs)
        got = st.new_coverage(cids, recs)
        assert np.array_equal(got, exp_new), batch
        for c in range(ncalls):
            assert np.array_equal(st.max_cover(c), mc[c]), (batch, c)
    st.close()


def test_newcov_key_mode_membership(torch):
    """Key mode at kshift 4 (the fused candidate + membership pass of
    newcov.hip) over a universe with gap keys (blocks of 16 PCs holding none)
    and many PCs whose low bits are 15 — the value the staged nibble table
    also holds for a gap key, so both the nibble test and the exact byte test
    decide candidates.  Universe-only batches match the sequential reference
    (syz-fuzzer/fuzzer.go:456-480); a batch holding a stray PC (a universe
    PC's key, other low bits), a gap-key PC with low bits 15, or one with
    other low bits is rejected and leaves maxCover as it was."""
    from syzkaller_amd import SyzcovError
    from syzkaller_amd.fuzzer import CoverState
    rng = np.random.default_rng(5)
    base, nblk, ncalls = 0x81000000, 1 << 15, 8
    lows = rng.integers(0, 16, nblk)
    lows[::7] = 15
    gap = np.arange(nblk) % 3 == 0
    univ = (base + 16 * np.arange(nblk, dtype=np.int64) + lows)[~gap].astype(np.uint32)
    st = CoverState(ncalls, base, 16 * nblk)
    st.set_universe(univ)
    mc = [np.zeros(0, np.uint32) for _ in range(ncalls)]
    flakes = np.zeros(0, np.uint32)
    for batch in range(3):
        nrec = 2000
        cids = rng.integers(0, ncalls, size=nrec)
        recs = [np.unique(rng.choice(univ, size=int(rng.integers(1, 300)))).astype(np.uint32)
                for _ in range(nrec)]
        exp_new, mc = orc.newcov_batch(mc, flakes, cids, recs)
        assert np.array_equal(st.new_coverage(cids, recs), exp_new), batch
    gk = np.flatnonzero(gap)
    mk = np.flatnonzero(~gap)[123]
    bad = [base + 16 * int(gk[5]) + 15, base + 16 * int(gk[9]) + 3,
           base + 16 * int(mk) + (int(lows[mk]) + 1) % 16]
    for pc in bad:
        cids = rng.integers(0, ncalls, size=400)
        recs = [np.unique(rng.choice(univ, size=60)).astype(np.uint32) for _ in range(400)]
        recs[200] = np.unique(np.append(recs[200], np.uint32(pc))).astype(np.uint32)
        with pytest.raises(SyzcovError):
            st.new_coverage(cids, recs)
        for c in range(ncalls):
            assert np.array_equal(st.max_cover(c), mc[c]), (hex(pc), c)
    st.close()
