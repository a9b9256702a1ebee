"""Key mode (keys.hip): the engine over dense keys (pc >> kshift) - kbase of
a registered PC universe, against the CPU oracle, which works on PCs."""
import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available()
    return t


def test_keymap_roundtrip(torch):
    from syzkaller_amd.engine import synth_universe, universe_keymap, _p, _stream
    from syzkaller_amd import _lib
    u = synth_universe(16, 0x5EED0002)
    uh = u.cpu().numpy().view(np.uint32)
    assert np.array_equal(uh, [orc.lib().orc_synth_universe(0x5EED0002, k) for k in range(1 << 16)])
    ks, kbase, nkeys, pok, lok, ulo, uhi = universe_keymap(u, "cuda")
    assert (ulo, uhi) == (int(uh[0]), int(uh[-1]))
    assert ks == 4 and nkeys == 1 << 16
    # membership table: the low kshift bits of each key's universe PC
    assert np.array_equal(lok.cpu().numpy(), (uh & 15).astype(np.uint8))
    keep = np.arange(uh.size) % 3 != 2  # every third key without a universe PC
    ks2, _, n2, _, lok2, _, _ = universe_keymap(uh[keep].copy(), "cuda")
    assert ks2 == 4 and n2 == int(np.nonzero(keep)[0][-1]) + 1  # keys up to the last kept PC
    l2 = lok2.cpu().numpy()
    assert np.array_equal(l2[keep[:n2]], (uh[keep] & 15).astype(np.uint8)[:int(keep[:n2].sum())])
    assert np.all(l2[~keep[:n2]] == 0x7F)  # keys without a universe PC
    keys = torch.from_numpy(((uh >> ks) - kbase).astype(np.int32)).cuda()
    out = torch.empty_like(keys)
    L = _lib.lib()
    _lib.check(L.syzcov_dev_keys_to_pcs(_p(pok), nkeys, _p(keys), _p(out), None, keys.numel(),
                                        _stream()), "keys_to_pcs")
    assert np.array_equal(out.cpu().numpy().view(np.uint32), uh)
    with pytest.raises(ValueError):  # unsorted universe
        universe_keymap(np.array([5, 3], np.uint32), "cuda")


@pytest.mark.parametrize("force", ["", "small_init", "no_init_block"],
                         ids=["init-block", "init-64", "chunks-only"])
@pytest.mark.parametrize("layout", [0, 1], ids=["csr", "aligned"])
@pytest.mark.parametrize("n,mean,sigma,log2", [(4000, 2048, 512, 22), (3000, 300, 200, 12),
                                               (500, 9000, 6000, 20), (2000, 600, 300, 17),
                                               (3000, 1500, 900, 19)])
def test_engine_key_mode_vs_oracle(torch, n, mean, sigma, log2, layout, force, monkeypatch):
    """Key-mode steps against the oracle (cover.go:28-40, 104-131).  Minimize's
    first items go through the initial LDS block (every item at these sizes),
    a one-chunk block followed by geometric chunks (small_init), or chunks
    only (no_init_block)."""
    monkeypatch.setenv("SYZCOV_FORCE", force)
    from syzkaller_amd.engine import CorpusEngine, synth_corpus, synth_universe, synth_window
    seed = 0x5EED0002
    off, raw, lens, total = synth_corpus(n, seed, mean=mean, sigma=sigma, log2_space=log2)
    lo, span = synth_window(log2)
    eng = CorpusEngine(n, total, int(lens.max().item()), lo, span,
                       universe=synth_universe(log2, seed), canon_layout=layout)
    assert bool(eng.canon_align_k) == (layout == 1 and eng.nrange > 1)
    assert eng.key_mode and eng.span == 1 << log2 and eng.kshift == 4
    res = eng.step(off, raw, n)
    o_off, o_pcs = orc.synth_corpus(seed, n, mean=mean, sigma=sigma, log2_space=log2)
    c_off, c_pcs = orc.canonicalize_csr(o_off, o_pcs)
    new_len = eng.new_len[:n].cpu().numpy()
    assert np.array_equal(new_len, np.diff(c_off).astype(np.int32))
    canon = eng.canonical_pcs(off, n).cpu().numpy().view(np.uint32)
    offs = off.cpu().numpy()
    for i in range(0, n, max(1, n // 40)):
        assert np.array_equal(canon[offs[i]:offs[i] + new_len[i]], c_pcs[c_off[i]:c_off[i + 1]])
    exp_kept = orc.minimize_csr(c_off, c_pcs)
    assert res.kept_idx.cpu().numpy().tolist() == list(exp_kept)
    exp_union = orc.union_fold_csr(c_off, c_pcs)
    assert np.array_equal(res.union.cpu().numpy().view(np.uint32), exp_union)
    assert res.max_cover == exp_union.size
    res2 = eng.step(off, raw, n)
    assert res2.kept_idx.cpu().numpy().tolist() == list(exp_kept)
    assert np.array_equal(res2.union.cpu().numpy().view(np.uint32), exp_union)


@pytest.mark.parametrize("force", ["", "mr_bytes", "small_init", "mr_bytes,small_init"],
                         ids=["nibbles", "bytes", "nibbles-init-64", "bytes-init-64"])
def test_engine_key_mode_x86_vs_oracle(torch, force, monkeypatch):
    """The x86-like universe (PC pairs per 16-byte block, kshift 2): Minimize's
    tables are nibbles over 2^18 keys (every low value fits 2 bits) or, with
    SYZCOV_FORCE=mr_bytes, bytes over 2^17; both against the oracle, then a
    non-universe PC (a universe PC + 1: same key, other low bits) in early,
    middle and last inputs is never aliased (the step recomputes in window
    mode and returns the reference's results)."""
    monkeypatch.setenv("SYZCOV_FORCE", force)
    from syzkaller_amd.engine import CorpusEngine, synth_corpus, synth_universe, synth_window
    n, log2, seed = 3000, 19, 0x5EED0002
    u = synth_universe(log2, seed, x86=True)
    uh = u.cpu().numpy().view(np.uint32)
    lo, span = synth_window(log2, x86=True)
    off, raw, lens, total = synth_corpus(n, seed, mean=1200, sigma=500, log2_space=log2, x86=True)
    eng = CorpusEngine(n, total, int(lens.max().item()), lo, span, universe=u)
    assert eng.kshift == 2 and eng.nrange == (8 if "mr_bytes" in force else 4)
    exp_kept, exp_union = _oracle_of(off, raw, n)
    res = eng.step(off, raw, n)
    assert not res.fallback
    assert res.kept_idx.cpu().numpy().tolist() == exp_kept
    assert np.array_equal(res.union.cpu().numpy().view(np.uint32), exp_union)
    for where in (0, 1500, 2999):
        off, raw, lens, total = synth_corpus(n, seed, mean=1200, sigma=500, log2_space=log2,
                                             x86=True)
        j = int(off[where].item()) + int(lens[where].item()) // 2
        k = int(raw[j].item()) & 0xFFFFFFFF
        raw[j] = np.int32(np.uint32(_stray(uh, int(np.searchsorted(uh, k)))))
        exp_kept, exp_union = _oracle_of(off, raw, n)
        res = eng.step(off, raw, n)
        assert res.fallback and res.err_flags & 4, where
        assert res.kept_idx.cpu().numpy().tolist() == exp_kept, where
        assert np.array_equal(res.union.cpu().numpy().view(np.uint32), exp_union), where


def test_engine_key_mode_window_error(torch):
    """A PC far below the universe's first key: out of the key range, and the
    corpus' PC extent (2^31 PCs) is too wide for the window-mode recompute, so
    the step raises instead of returning a wrong result."""
    from syzkaller_amd.engine import CorpusEngine, synth_corpus, synth_universe, synth_window
    n, log2 = 300, 14
    off, raw, lens, total = synth_corpus(n, 0x5EED0002, mean=200, sigma=50, log2_space=log2)
    raw[5] = 0x10  # far below the universe
    lo, span = synth_window(log2)
    eng = CorpusEngine(n, total, int(lens.max().item()), lo, span,
                       universe=synth_universe(log2, 0x5EED0002))
    with pytest.raises(RuntimeError):
        eng.step(off, raw, n)


@pytest.mark.parametrize("keys", [True, False], ids=["key-mode", "window-mode"])
def test_engine_offsets_past_2_32(torch, keys):
    """Inputs stored past element 2^32 + 2^31 of the PC array (as in C3's
    82 GB corpus): 64-bit CSR offsets whose low halves are >= 2^31 reach every
    kernel (the whole-wave minimize path once read them sign-extended).  Long
    inputs take the whole-wave path; canonicalized in place."""
    from syzkaller_amd.engine import CorpusEngine, synth_corpus, synth_universe, synth_window
    n, seed, log2, base = 3000, 0x5EED0002, 20, (1 << 32) + (1 << 31) + 3
    off, raw, lens, total = synth_corpus(n, seed, mean=2048, sigma=512, log2_space=log2)
    big = torch.empty(base + total + 1, dtype=torch.int32, device="cuda")
    big[base:base + total + 1].copy_(raw)
    offb = off + base
    del raw
    lo, span = synth_window(log2)
    eng = CorpusEngine(n, base + total, int(lens.max().item()), lo, span, canon_in_place=True,
                       universe=synth_universe(log2, seed) if keys else None)
    res = eng.step(offb, big, n)
    o_off, o_pcs = orc.synth_corpus(seed, n, mean=2048, sigma=512, log2_space=log2)
    c_off, c_pcs = orc.canonicalize_csr(o_off, o_pcs)
    assert np.array_equal(eng.new_len[:n].cpu().numpy(), np.diff(c_off).astype(np.int32))
    assert res.kept_idx.cpu().numpy().tolist() == list(orc.minimize_csr(c_off, c_pcs))
    assert np.array_equal(res.union.cpu().numpy().view(np.uint32), orc.union_fold_csr(c_off, c_pcs))
    del big
    torch.cuda.empty_cache()


@pytest.mark.parametrize("force", ["", "canon3", "redo"])
def test_engine_key_mode_sentinel(torch, force, monkeypatch):
    """Key mode with a universe whose last PC is 0xFFFFFFFF: inputs made only of
    the sentinel canonicalize to empty, otherwise it is an ordinary key
    (cover.go:28-40, 104-131).  force (SYZCOV_FORCE) selects the
    canonicalization: the 2-pass key sort (default), the 3-pass window-offset
    sort, or the workgroup sort every segment whose wave order check fails
    takes."""
    monkeypatch.setenv("SYZCOV_FORCE", force)
    from syzkaller_amd.engine import CorpusEngine
    rng = np.random.default_rng(33)
    univ = (np.uint64(0xFFFF0000) + 4 * np.arange(1 << 14, dtype=np.uint64) + 3).astype(np.uint32)
    covers = []
    for i in range(900):
        ln = int(rng.integers(0, 3000)) if i % 3 else int(rng.integers(0, 300))
        c = univ[rng.integers(0, univ.size, size=ln)]
        if i % 7 == 0:
            c = np.full(int(rng.integers(1, 5)), 0xFFFFFFFF, np.uint32)
        elif i % 5 == 0:
            c = np.concatenate([c, np.full(3, 0xFFFFFFFF, np.uint32)])
        covers.append(c.astype(np.uint32))
    lens = np.array([len(c) for c in covers], np.int64)
    o_off = np.zeros(len(covers) + 1, np.uint64)
    o_off[1:] = np.cumsum(lens)
    o_pcs = np.concatenate(covers + [np.zeros(1, np.uint32)])
    n = len(covers)
    off = torch.from_numpy(o_off.astype(np.int64)).cuda()
    raw = torch.from_numpy(o_pcs.view(np.int32)).cuda()
    eng = CorpusEngine(n, int(lens.sum()), int(lens.max()), 0xFFFF0000, 1 << 16,
                       universe=univ)
    assert eng.key_mode and eng.kshift == 2 and eng.span == 1 << 14
    res = eng.step(off, raw, n)
    c_off, c_pcs = orc.canonicalize_csr(o_off, o_pcs[:int(lens.sum())])
    assert np.array_equal(eng.new_len[:n].cpu().numpy(), np.diff(c_off).astype(np.int32))
    canon = eng.canonical_pcs(off, n).cpu().numpy().view(np.uint32)
    for i in range(n):
        a, b = int(o_off[i]), int(o_off[i]) + int(c_off[i + 1] - c_off[i])
        assert np.array_equal(canon[a:b], c_pcs[c_off[i]:c_off[i + 1]]), i
    assert res.kept_idx.cpu().numpy().tolist() == list(orc.minimize_csr(c_off, c_pcs))
    assert np.array_equal(res.union.cpu().numpy().view(np.uint32), orc.union_fold_csr(c_off, c_pcs))


@pytest.mark.parametrize("force", ["", "canon3"])
def test_engine_key_mode_clustered(torch, force, monkeypatch):
    """Covers as real kernels produce them: runs of neighbouring PCs (a few
    functions), repeated PCs, a few far-away PCs, in execution order: the
    digits of a sort pass concentrate on a few histogram bins (same-address
    LDS atomics in every wave instruction).  The key sort and the 3-pass
    window-offset sort must give the oracle's canonical covers and Minimize
    result (cover.go:28-40, 104-131)."""
    monkeypatch.setenv("SYZCOV_FORCE", force)
    from syzkaller_amd.engine import CorpusEngine
    rng = np.random.default_rng(91)
    univ = (np.uint64(0x81000000) + 16 * np.arange(1 << 18, dtype=np.uint64)
            + rng.integers(0, 16, 1 << 18).astype(np.uint64)).astype(np.uint32)
    covers = []
    for i in range(1500):
        kind = i % 4
        if kind == 0:  # one dense run of neighbouring PCs
            a = int(rng.integers(0, univ.size - 4000))
            c = univ[a:a + int(rng.integers(1, 3500))]
        elif kind == 1:  # a dense run plus far-away PCs: coarse buckets, a full one
            a = int(rng.integers(0, univ.size - 2000))
            c = np.concatenate([univ[a:a + int(rng.integers(200, 1800))],
                                univ[rng.integers(0, univ.size, size=int(rng.integers(1, 300)))]])
        elif kind == 2:  # few distinct PCs, each repeated (loops)
            c = np.repeat(univ[rng.integers(0, univ.size, size=int(rng.integers(1, 60)))],
                          int(rng.integers(1, 50)))
        else:  # several runs
            runs = [univ[a:a + int(rng.integers(5, 400))]
                    for a in rng.integers(0, univ.size - 400, size=int(rng.integers(1, 8)))]
            c = np.concatenate(runs)
        c = c[rng.permutation(c.size)][:8000]
        covers.append(c.astype(np.uint32))
    lens = np.array([c.size for c in covers], np.int64)
    o_off = np.zeros(len(covers) + 1, np.uint64)
    o_off[1:] = np.cumsum(lens)
    o_pcs = np.concatenate(covers + [np.zeros(1, np.uint32)])
    n = len(covers)
    off = torch.from_numpy(o_off.astype(np.int64)).cuda()
    raw = torch.from_numpy(o_pcs.view(np.int32)).cuda()
    eng = CorpusEngine(n, int(lens.sum()), int(lens.max()), int(univ[0]),
                       int(univ[-1]) - int(univ[0]) + 1, universe=univ)
    assert eng.key_mode
    res = eng.step(off, raw, n)
    c_off, c_pcs = orc.canonicalize_csr(o_off, o_pcs[:int(lens.sum())])
    assert np.array_equal(eng.new_len[:n].cpu().numpy(), np.diff(c_off).astype(np.int32))
    canon = eng.canonical_pcs(off, n).cpu().numpy().view(np.uint32)
    for i in range(n):
        a, b = int(o_off[i]), int(o_off[i]) + int(c_off[i + 1] - c_off[i])
        assert np.array_equal(canon[a:b], c_pcs[c_off[i]:c_off[i + 1]]), i
    assert res.kept_idx.cpu().numpy().tolist() == list(orc.minimize_csr(c_off, c_pcs))
    assert np.array_equal(res.union.cpu().numpy().view(np.uint32), orc.union_fold_csr(c_off, c_pcs))


@pytest.mark.parametrize("in_place", [False, True], ids=["out-of-place", "in-place"])
def test_engine_key_mode_tiny_segments(torch, in_place):
    """Covers of 0..9 PCs at every alignment of their first PC (the wave
    kernel loads 4-PC chunks of a segment: fewer than 4 PCs take the
    workgroup path, the first and last chunks of longer ones start at the
    segment's first PC / end at its last), between long covers, with repeats
    (cover.go:28-40, 104-131)."""
    from syzkaller_amd.engine import CorpusEngine
    rng = np.random.default_rng(17)
    univ = (np.uint64(0x81000000) + 16 * np.arange(1 << 16, dtype=np.uint64)
            + rng.integers(0, 16, 1 << 16).astype(np.uint64)).astype(np.uint32)
    covers = []
    for i in range(400):
        ln = int(rng.integers(1200, 2600)) if i % 7 == 3 else i % 10
        c = univ[rng.integers(0, univ.size, size=ln)]
        if ln > 2 and i % 3 == 0:
            c[-1] = c[0]  # a repeat
        covers.append(c.astype(np.uint32))
    lens = np.array([c.size for c in covers], np.int64)
    o_off = np.zeros(len(covers) + 1, np.uint64)
    o_off[1:] = np.cumsum(lens)
    o_pcs = np.concatenate(covers + [np.zeros(1, np.uint32)])
    n = len(covers)
    off = torch.from_numpy(o_off.astype(np.int64)).cuda()
    raw = torch.from_numpy(o_pcs.view(np.int32)).cuda()
    eng = CorpusEngine(n, int(lens.sum()) + 1, int(lens.max()), int(univ[0]),
                       int(univ[-1]) - int(univ[0]) + 1, universe=univ, canon_in_place=in_place)
    exp_kept, exp_union = _oracle_of(off, raw, n)
    c_off, c_pcs = orc.canonicalize_csr(o_off, o_pcs[:int(lens.sum())])
    res = eng.step(off, raw, n)
    assert np.array_equal(eng.new_len[:n].cpu().numpy(), np.diff(c_off).astype(np.int32))
    if not in_place:
        canon = eng.canonical_pcs(off, n).cpu().numpy().view(np.uint32)
        for i in range(n):
            a, b = int(o_off[i]), int(o_off[i]) + int(c_off[i + 1] - c_off[i])
            assert np.array_equal(canon[a:b], c_pcs[c_off[i]:c_off[i + 1]]), i
    assert res.kept_idx.cpu().numpy().tolist() == exp_kept
    assert np.array_equal(res.union.cpu().numpy().view(np.uint32), exp_union)


def _stray(u: np.ndarray, i: int) -> int:
    """A PC next to universe PC u[i] that is not in the universe."""
    us = set(u.tolist())
    return next(int(u[j]) + d for j in range(i, u.size) for d in (1, 2, 3, 5)
                if int(u[j]) + d not in us and int(u[j]) + d <= int(u[-1]))


def _oracle_of(off, raw, n):
    o_off = off[:n + 1].cpu().numpy().astype(np.uint64)
    o_pcs = raw[:int(o_off[-1])].cpu().numpy().view(np.uint32)
    c_off, c_pcs = orc.canonicalize_csr(o_off, o_pcs)
    return list(orc.minimize_csr(c_off, c_pcs)), orc.union_fold_csr(c_off, c_pcs)


@pytest.mark.parametrize("force", ["", "canon3", "redo"])
@pytest.mark.parametrize("in_place", [False, True], ids=["out-of-place", "in-place"])
def test_engine_key_mode_nonuniverse(torch, force, in_place, monkeypatch):
    """A PC inside the universe's key range that is not a universe PC (it
    shares its key with a universe PC, cover.go would treat them as two PCs)
    is never aliased.  Out of place the step is recomputed in window mode over
    the corpus' PC extent and returns the reference's results (cover.Minimize
    never fails, cover.go:104-131); in place the raw PCs are gone and the step
    raises.  Every canonicalization path checks membership (keys.hip)."""
    monkeypatch.setenv("SYZCOV_FORCE", force)
    from syzkaller_amd.engine import CorpusEngine, synth_corpus, synth_universe, synth_window
    n, log2, seed = 2000, 16, 0x5EED0002
    u = synth_universe(log2, seed)
    uh = u.cpu().numpy().view(np.uint32)
    lo, span = synth_window(log2)
    for where in (0, 777, 1999):
        off, raw, lens, total = synth_corpus(n, seed, mean=1500, sigma=600, log2_space=log2)
        eng = CorpusEngine(n, total, int(lens.max().item()), lo, span, universe=u,
                           canon_in_place=in_place)
        res = eng.step(off, raw, n)  # clean corpus: fine
        assert res.n_kept > 0 and not res.fallback
        mc0 = res.max_cover
        off, raw, lens, total = synth_corpus(n, seed, mean=1500, sigma=600, log2_space=log2)
        j = int(off[where].item()) + int(lens[where].item()) // 2
        k = int(raw[j].item()) & 0xFFFFFFFF
        raw[j] = np.int32(np.uint32(_stray(uh, int(np.searchsorted(uh, k)))))
        if in_place:
            with pytest.raises(RuntimeError, match="universe"):
                eng.step(off, raw, n)
            continue
        exp_kept, exp_union = _oracle_of(off, raw, n)
        res = eng.step(off, raw, n)
        assert res.fallback and res.err_flags & 4, where
        assert res.kept_idx.cpu().numpy().tolist() == exp_kept, where
        assert np.array_equal(res.union.cpu().numpy().view(np.uint32), exp_union), where
        assert res.max_cover == mc0  # the stray PC has no key of its own
        assert res.max_cover_missed == 1  # ... and maxCover says it did not take it
        res2 = eng.result()  # a second read returns the recomputed step
        assert res2.fallback and res2.n_kept == res.n_kept
        res3 = eng.step(off, raw, n)  # and the next step recomputes again
        assert res3.kept_idx.cpu().numpy().tolist() == exp_kept


def test_engine_key_mode_fallback_outside_extent(torch):
    """PCs above the universe's last PC (outside the key range, SYZCOV_ERR_WINDOW)
    and a caller order: the window-mode recompute keeps the caller's order,
    the host drop-in form restages its in-place PCs, maxCover takes only the
    union's universe PCs."""
    import ctypes as C
    from syzkaller_amd import _lib
    from syzkaller_amd.engine import CorpusEngine, synth_corpus, synth_universe, synth_window
    n, log2, seed = 1500, 15, 0x5EED0002
    u = synth_universe(log2, seed)
    uh = u.cpu().numpy().view(np.uint32)
    lo, span = synth_window(log2)
    off, raw, lens, total = synth_corpus(n, seed, mean=900, sigma=300, log2_space=log2)
    for i in (3, 700, 1499):  # a few PCs past the universe's extent
        raw[int(off[i].item())] = np.int32(np.uint32(int(uh[-1]) + 1000 + i))
    exp_kept, exp_union = _oracle_of(off, raw, n)
    eng = CorpusEngine(n, total, int(lens.max().item()), lo, span, universe=u)
    res = eng.step(off, raw, n)
    assert res.fallback and res.err_flags & 1
    assert res.kept_idx.cpu().numpy().tolist() == exp_kept
    assert np.array_equal(res.union.cpu().numpy().view(np.uint32), exp_union)
    univ_in_union = np.intersect1d(exp_union, uh).size
    assert res.max_cover == univ_in_union
    assert res.max_cover_missed == exp_union.size - univ_in_union == 3
    # host form, canon in place inside the handle, with a caller order
    L = _lib.lib()
    h_off = off.cpu().numpy().astype(np.uint64)
    h_pcs = raw[:total].cpu().numpy().view(np.uint32).copy()
    covs = [h_pcs[h_off[i]:h_off[i + 1]] for i in range(n)]
    perm = np.random.default_rng(4).permutation(n).astype(np.int32)
    seen, exp_p = set(), []
    for i in perm:
        if any(int(p) not in seen for p in covs[i]):
            exp_p.append(int(i))
        seen.update(int(p) for p in covs[i])
    cfg = _lib.CorpusCfg(n_max=n, p_max=total, max_seg_len=int(lens.max().item()),
                         universe=uh.ctypes.data, universe_n=uh.size, canon_in_place=1)
    h = C.c_uint64(0)
    _lib.check(L.syzcov_corpus_create(C.byref(cfg), None, 0, C.byref(h)), "corpus_create")
    out = np.empty(n, np.int32)
    un = np.empty(total, np.uint32)
    nu = C.c_uint64(0)
    k = _lib.check(L.syzcov_corpus_minimize_host_order(h.value, h_off.ctypes.data, h_pcs.ctypes.data,
                                                       n, perm.ctypes.data, out.ctypes.data,
                                                       un.ctypes.data, un.size, C.byref(nu)),
                   "corpus_minimize_host_order")
    L.syzcov_corpus_destroy(h.value)
    assert out[:k].tolist() == exp_p
    assert np.array_equal(un[:nu.value], exp_union)


def test_engine_key_mode_fallback_keeps_caller_lens_order(torch):
    """A step ordered by CALLER lengths (syzcov_corpus_order with lens) whose
    corpus holds a non-universe PC: the window-mode recompute must process the
    inputs in the order sorted over those lengths, not the handle's own."""
    from syzkaller_amd.engine import CorpusEngine, synth_corpus, synth_universe, synth_window
    n, log2, seed = 1200, 15, 0x5EED0002
    u = synth_universe(log2, seed)
    uh = u.cpu().numpy().view(np.uint32)
    lo, span = synth_window(log2)
    off, raw, lens, total = synth_corpus(n, seed, mean=700, sigma=300, log2_space=log2)
    j = int(off[500].item()) + 2
    raw[j] = np.int32(np.uint32(_stray(uh, int(np.searchsorted(uh, int(raw[j].item()) & 0xFFFFFFFF)))))
    # caller lengths unrelated to the covers: Go's sort over them decides the order
    clens = np.random.default_rng(11).integers(1, 50, n).astype(np.int32)
    order = orc.sort_order(clens.astype(np.int64))
    o_off = off.cpu().numpy().astype(np.uint64)
    o_pcs = raw[:total].cpu().numpy().view(np.uint32)
    c_off, c_pcs = orc.canonicalize_csr(o_off, o_pcs)
    seen, exp = set(), []
    for i in order:
        cov = c_pcs[c_off[i]:c_off[i + 1]]
        if any(int(p) not in seen for p in cov):
            exp.append(int(i))
        seen.update(int(p) for p in cov)
    eng = CorpusEngine(n, total, int(lens.max().item()), lo, span, universe=u)
    eng.canonicalize(off, raw, n)
    eng.sort_order(torch.from_numpy(clens).cuda(), n)
    eng.minimize(True)
    eng.finish()
    res = eng.result()
    assert res.fallback and res.err_flags & 4
    assert res.kept_idx.cpu().numpy().tolist() == exp


def test_engine_key_mode_gap_key(torch):
    """A universe with keys that hold no PC (every other synthetic PC): the
    universe's own PCs give the oracle's results; a PC on such a key is never
    aliased (the step is recomputed in window mode)."""
    from syzkaller_amd.engine import CorpusEngine
    rng = np.random.default_rng(7)
    full = np.array([orc.lib().orc_synth_universe(0x5EED0002, k) for k in range(1 << 14)],
                    np.uint32)
    univ = full[::2].copy()
    covers = [np.sort(rng.choice(univ, size=int(rng.integers(1, 900)))) for _ in range(600)]
    lens = np.array([c.size for c in covers], np.int64)
    o_off = np.zeros(len(covers) + 1, np.uint64)
    o_off[1:] = np.cumsum(lens)
    o_pcs = np.concatenate(covers).astype(np.uint32)
    off = torch.from_numpy(o_off.astype(np.int64)).cuda()
    raw = torch.from_numpy(o_pcs.view(np.int32)).cuda()
    eng = CorpusEngine(len(covers), int(lens.sum()), int(lens.max()), int(univ[0]),
                       int(univ[-1]) - int(univ[0]) + 1, universe=univ)
    res = eng.step(off, raw, len(covers))
    c_off, c_pcs = orc.canonicalize_csr(o_off, o_pcs)
    assert res.kept_idx.cpu().numpy().tolist() == list(orc.minimize_csr(c_off, c_pcs))
    assert np.array_equal(res.union.cpu().numpy().view(np.uint32), orc.union_fold_csr(c_off, c_pcs))
    raw[int(o_off[300]) + 0] = np.int32(full[101].view(np.int32))  # a removed PC: a gap key
    exp_kept, exp_union = _oracle_of(off, raw, len(covers))
    res = eng.step(off, raw, len(covers))  # recomputed in window mode, exact
    assert res.fallback
    assert res.kept_idx.cpu().numpy().tolist() == exp_kept
    assert np.array_equal(res.union.cpu().numpy().view(np.uint32), exp_union)


@pytest.mark.parametrize("force", ["redo", "canon3"])
@pytest.mark.parametrize("layout", [0, 1], ids=["csr", "aligned"])
@pytest.mark.parametrize("keys", [True, False], ids=["key-mode", "window-mode"])
def test_engine_forced_redo_vs_oracle(torch, keys, layout, force, monkeypatch):
    """The canon wave sort checks its own order and sends a failing segment to
    the workgroup sort (canon.hip).  Forcing every segment down that path
    (SYZCOV_FORCE=redo; in the line-aligned layout its contiguous output is
    then spread to the sub-runs' aligned starts), or key mode down the 3-pass
    wave sort (canon3), must give the oracle's results."""
    monkeypatch.setenv("SYZCOV_FORCE", force)
    from syzkaller_amd.engine import CorpusEngine, synth_corpus, synth_universe, synth_window
    n, log2, seed = 3000, 18, 0x5EED0002
    off, raw, lens, total = synth_corpus(n, seed, mean=2048, sigma=900, log2_space=log2)
    lo, span = synth_window(log2)
    eng = CorpusEngine(n, total, int(lens.max().item()), lo, span,
                       universe=synth_universe(log2, seed) if keys else None,
                       canon_layout=layout)
    res = eng.step(off, raw, n)
    o_off, o_pcs = orc.synth_corpus(seed, n, mean=2048, sigma=900, log2_space=log2)
    c_off, c_pcs = orc.canonicalize_csr(o_off, o_pcs)
    assert np.array_equal(eng.new_len[:n].cpu().numpy(), np.diff(c_off).astype(np.int32))
    canon = eng.canonical_pcs(off, n).cpu().numpy().view(np.uint32)
    offs = off.cpu().numpy()
    for i in range(0, n, 37):
        assert np.array_equal(canon[offs[i]:offs[i] + int(c_off[i + 1] - c_off[i])],
                              c_pcs[c_off[i]:c_off[i + 1]])
    assert res.kept_idx.cpu().numpy().tolist() == list(orc.minimize_csr(c_off, c_pcs))
    assert np.array_equal(res.union.cpu().numpy().view(np.uint32), orc.union_fold_csr(c_off, c_pcs))


@pytest.mark.parametrize("keys", [True, False], ids=["key-mode", "window-mode"])
def test_engine_segment_longer_than_declared(torch, keys):
    """An input longer than the engine's declared max_seg_len is not
    canonicalized silently: SYZCOV_ERR_SEGLEN, and the step raises."""
    from syzkaller_amd.engine import CorpusEngine, synth_corpus, synth_universe, synth_window
    n, log2, seed = 500, 16, 0x5EED0002
    off, raw, lens, total = synth_corpus(n, seed, mean=2048, sigma=512, log2_space=log2)
    lo, span = synth_window(log2)
    ml = int(lens.max().item())
    eng = CorpusEngine(n, total, ml - 1, lo, span,
                       universe=synth_universe(log2, seed) if keys else None)
    with pytest.raises(RuntimeError, match="max_seg_len"):
        eng.step(off, raw, n)


def test_engine_key_mode_top_key_not_sentinel(torch):
    """A universe whose last PC shares the sentinel's key (0xFFFFFFC0 at
    kshift 6) but does not hold 0xFFFFFFFF: that PC is an ordinary PC and
    stays in the union (only 0xFFFFFFFF itself is dropped, cover.go:97)."""
    from syzkaller_amd.engine import CorpusEngine
    univ = (0xFFFF0000 + 64 * np.arange(1024, dtype=np.uint64)).astype(np.uint32)
    assert univ[-1] == 0xFFFFFFC0
    rng = np.random.default_rng(11)
    covers = [np.sort(rng.choice(univ, size=int(rng.integers(1, 200)), replace=False))
              for _ in range(300)]
    covers[17] = np.array([0xFFFFFFC0], np.uint32)  # the top key alone in one input
    lens = np.array([c.size for c in covers], np.int64)
    o_off = np.zeros(len(covers) + 1, np.uint64)
    o_off[1:] = np.cumsum(lens)
    o_pcs = np.concatenate(covers).astype(np.uint32)
    off = torch.from_numpy(o_off.astype(np.int64)).cuda()
    raw = torch.from_numpy(o_pcs.view(np.int32).copy()).cuda()
    eng = CorpusEngine(len(covers), int(lens.sum()), int(lens.max()), int(univ[0]),
                       int(univ[-1]) - int(univ[0]) + 1, universe=univ)
    assert eng.kshift == 6 and eng.sent_key is None
    res = eng.step(off, raw, len(covers))
    c_off, c_pcs = orc.canonicalize_csr(o_off, o_pcs)
    assert res.kept_idx.cpu().numpy().tolist() == list(orc.minimize_csr(c_off, c_pcs))
    un = res.union.cpu().numpy().view(np.uint32)
    assert np.array_equal(un, orc.union_fold_csr(c_off, c_pcs)) and un[-1] == 0xFFFFFFC0
