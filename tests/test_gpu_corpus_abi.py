"""The resident corpus engine through its C-ABI handle (include/syzcov.h,
"resident corpus engine"; corpus.hip), driven over ctypes the way the Go host
would over cgo: no torch buffers, the handle allocates its own memory.

  C2 on device pointers: syzcov_corpus_step / _result against the oracle's
     full-size digests (tests/golden/fullsize_digests.json)
  C1 from host pointers: syzcov_corpus_minimize_host and the drop-in
     syzcov_minimize (which routes corpus-sized calls to the engine) against
     the C1 digests
  covers as cover.Minimize receives them (unsorted, duplicates) against the
     oracle's literal restatement of cover.go:104-131; errors: a PC outside
     the window / universe fails the call, never returns an aliased result
"""
import ctypes as C
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def golden(name):
    with open(os.path.join(HERE, "golden", "fullsize_digests.json")) as f:
        return json.load(f)[name]


def sha_np(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).astype("<i4").tobytes()).hexdigest()


@pytest.fixture(scope="module")
def L():
    import torch
    assert torch.cuda.is_available()
    from syzkaller_amd import _lib
    return _lib.lib()


def _cfg(**kw):
    from syzkaller_amd._lib import CorpusCfg
    return CorpusCfg(**kw)


def _create(L, cfg):
    from syzkaller_amd._lib import check
    h = C.c_uint64(0)
    check(L.syzcov_corpus_create(C.byref(cfg), None, 0, C.byref(h)), "corpus_create")
    return h.value


def _minimize_host(L, h, off, pcs, n, union_cap):
    out = np.empty(n, np.int32)
    un = np.empty(union_cap, np.uint32)
    nu = C.c_uint64(0)
    k = L.syzcov_corpus_minimize_host(h, off.ctypes.data, pcs.ctypes.data, n, out.ctypes.data,
                                      un.ctypes.data, union_cap, C.byref(nu))
    return k, out[:max(k, 0)], un[:nu.value]


def _d2h(L, ptr, n, s):
    """n 32-bit words at a result pointer of the handle, through the library's
    own copy kernel (16-byte multiples: every buffer of the layout is padded
    to 256 bytes)."""
    import torch
    from syzkaller_amd._lib import check
    t = torch.empty((n + 3) // 4 * 4, dtype=torch.int32, device="cuda")
    if n:
        check(L.syzcov_dev_stream_copy(C.c_void_p(ptr), C.c_void_p(t.data_ptr()), t.numel() * 4, s),
              "stream_copy")
    torch.cuda.synchronize()
    return t[:n].cpu().numpy()


def test_corpus_handle_c2_digest(L):
    """C2 (1M inputs, key mode) through the handle on device pointers."""
    import torch
    from syzkaller_amd._lib import CorpusRes, check
    from syzkaller_amd.engine import synth_corpus, synth_universe
    g = golden("C2")
    n = g["n"]
    off, raw, lens, total = synth_corpus(n, g["seed"], mean=g["mean"], sigma=g["sigma"],
                                         log2_space=g["log2_space"])
    univ = synth_universe(g["log2_space"], g["seed"]).cpu().numpy().view(np.uint32).copy()
    cfg = _cfg(n_max=n, p_max=total, max_seg_len=int(lens.max().item()),
               universe=univ.ctypes.data, universe_n=univ.size)
    h = _create(L, cfg)
    try:
        s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        for step in range(2):  # the second step finds the handle's state clean
            check(L.syzcov_corpus_step(h, C.c_void_p(off.data_ptr()), C.c_void_p(raw.data_ptr()),
                                       n, s), "corpus_step")
            r = CorpusRes()
            check(L.syzcov_corpus_result(h, C.byref(r), s), "corpus_result")
            assert (r.n_kept, r.n_union, r.max_cover) == (g["n_kept"], g["n_union"], g["n_union"])
            kept = _d2h(L, r.kept_idx, r.n_kept, s)
            union = _d2h(L, r.union_pcs, r.n_union, s)
            assert sha_np(kept) == g["kept_sha256"]
            assert sha_np(union) == g["union_sha256"]
    finally:
        L.syzcov_corpus_destroy(h)


def test_corpus_minimize_host_c1_digest(L):
    """C1 (10k inputs) from host buffers: syzcov_corpus_minimize_host (window
    mode) and the drop-in syzcov_minimize (corpus-sized: the engine route)."""
    g = golden("C1")
    n = g["n"]
    off, pcs = orc.synth_corpus(g["seed"], n, g["mean"], g["sigma"], g["log2_space"])
    off = np.ascontiguousarray(off, np.uint64)
    pcs = np.ascontiguousarray(pcs, np.uint32)
    lens = np.diff(off)
    lo, hi = int(pcs[:int(off[-1])].min()), int(pcs[:int(off[-1])].max())
    # the oracle's order sorts canonical lengths (its corpus is canonicalized
    # first); Minimize of canonical covers is the reference call
    c_off, c_pcs = orc.canonicalize_csr(off, pcs)
    c_off = np.ascontiguousarray(c_off, np.uint64)
    c_pcs = np.ascontiguousarray(c_pcs, np.uint32)
    cfg = _cfg(n_max=n, p_max=int(c_off[-1]), max_seg_len=int(np.diff(c_off).max()), pc_lo=lo,
               pc_span=hi - lo + 1)
    h = _create(L, cfg)
    try:
        k, kept, union = _minimize_host(L, h, c_off, c_pcs, n, 1 << 23)
        assert k == g["n_kept"] and sha_np(kept) == g["kept_sha256"]
        assert union.size == g["n_union"] and sha_np(union) == g["union_sha256"]
    finally:
        L.syzcov_corpus_destroy(h)
    out = np.empty(n, np.int32)
    k2 = L.syzcov_minimize(c_off.ctypes.data, c_pcs.ctypes.data, n, None, 0, out.ctypes.data)
    assert k2 == g["n_kept"] and sha_np(out[:k2]) == g["kept_sha256"]
    assert int(lens.max()) > 0


def _random_covers(rng, n, universe, raw):
    covers = []
    for i in range(n):
        ln = int(rng.integers(0, 700)) if i % 5 else int(rng.integers(0, 40))
        c = universe[rng.integers(0, universe.size, size=ln)]
        if not raw:
            c = np.unique(c)
        covers.append(c.astype(np.uint32))
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum([c.size for c in covers])
    pcs = np.concatenate(covers + [np.zeros(1, np.uint32)])
    return off, pcs


@pytest.mark.parametrize("raw", [False, True], ids=["canonical", "raw-covers"])
@pytest.mark.parametrize("keys", [False, True], ids=["window", "keys"])
def test_corpus_minimize_host_vs_oracle(L, raw, keys):
    """cover.Minimize + the union fold on covers as given: canonical, or
    unsorted with duplicates (Go sorts by len(cov) with the duplicates,
    order_by = 1), against the oracle's cover.go restatement."""
    rng = np.random.default_rng(11 + raw + 2 * keys)
    univ = np.unique((0x81000000 + 5 * np.arange(60000) + rng.integers(0, 3, 60000))
                     .astype(np.uint32))
    n = 3000
    off, pcs = _random_covers(rng, n, univ, raw)
    lens = np.diff(off)
    cfg = _cfg(n_max=n, p_max=int(off[-1]) + 1, max_seg_len=max(1, int(lens.max())),
               pc_lo=int(univ[0]), pc_span=int(univ[-1]) - int(univ[0]) + 1,
               universe=univ.ctypes.data if keys else None, universe_n=univ.size if keys else 0,
               order_by=1)
    h = _create(L, cfg)
    try:
        k, kept, union = _minimize_host(L, h, off, pcs, n, univ.size + 1)
    finally:
        L.syzcov_corpus_destroy(h)
    assert k >= 0, L.syzcov_last_error()
    assert kept.tolist() == list(orc.minimize_csr(off, pcs))
    c_off, c_pcs = orc.canonicalize_csr(off, pcs)
    assert np.array_equal(union, orc.union_fold_csr(c_off, c_pcs))
    if raw:  # the drop-in call (>= 1024 inputs: the engine route) agrees
        out = np.empty(n, np.int32)
        k2 = L.syzcov_minimize(off.ctypes.data, pcs.ctypes.data, n, None, 0, out.ctypes.data)
        assert out[:k2].tolist() == kept.tolist()


def test_corpus_handle_errors(L):
    """A PC far outside the window (a PC extent too wide for the window-mode
    recompute) fails the call with SYZCOV_ERANGE.  Key mode, a PC next to a
    universe PC but not in the universe is never aliased: the step is
    recomputed in window mode and returns the reference's result.  The handle
    then serves the clean corpus again."""
    rng = np.random.default_rng(5)
    univ = (0x90000000 + 16 * np.arange(1 << 15) + rng.integers(0, 16, 1 << 15)).astype(np.uint32)
    n = 1500
    off, pcs = _random_covers(rng, n, univ, False)
    lens = np.diff(off)
    for keys in (False, True):
        cfg = _cfg(n_max=n, p_max=int(off[-1]) + 1, max_seg_len=int(lens.max()),
                   pc_lo=int(univ[0]), pc_span=int(univ[-1]) - int(univ[0]) + 1,
                   universe=univ.ctypes.data if keys else None,
                   universe_n=univ.size if keys else 0)
        h = _create(L, cfg)
        try:
            k0, kept0, _ = _minimize_host(L, h, off, pcs, n, univ.size + 1)
            assert k0 > 0
            bad = pcs.copy()
            j = int(off[700]) + 3
            bad[j] = 0x10  # below the window
            assert _minimize_host(L, h, off, bad, n, univ.size + 1)[0] == -5  # SYZCOV_ERANGE
            if keys:  # inside the key range, not a universe PC
                bad = pcs.copy()
                u = int(bad[j])
                stray = u + 1 if (u + 1) not in set(univ.tolist()) else u - 1
                bad[j] = stray
                bad[int(off[700]):int(off[701])].sort()
                c_off, c_pcs = orc.canonicalize_csr(off, bad)
                kb, keptb, unb = _minimize_host(L, h, off, bad, n, univ.size + 1)
                assert keptb.tolist() == list(orc.minimize_csr(c_off, c_pcs))
                assert np.array_equal(unb, orc.union_fold_csr(c_off, c_pcs))
            k1, kept1, _ = _minimize_host(L, h, off, pcs, n, univ.size + 1)
            assert k1 == k0 and kept1.tolist() == kept0.tolist()
        finally:
            L.syzcov_corpus_destroy(h)


def test_dropin_minimize_unaligned_wide_extent(L):
    """cover.Minimize through the drop-in on >= 1024 inputs (the cached-engine
    route) whose PC extent is just under 2^28 PCs and starts off a 2^20-PC
    boundary: aligning the window down would need 257 ranges, so the engine
    takes the exact extent (or the dictionary path) and the call never fails."""
    rng = np.random.default_rng(9)
    lo = 0x10000000 + (1 << 19) + 5
    hi = lo + (1 << 28) - (1 << 19) - 1
    n = 1100
    lens = rng.integers(1, 300, n)
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    pcs = rng.integers(lo, hi + 1, int(off[-1]), dtype=np.uint64).astype(np.uint32)
    pcs[0], pcs[-1] = lo, hi  # the extent's two ends
    out = np.empty(n, np.int32)
    k = L.syzcov_minimize(off.ctypes.data, pcs.ctypes.data, n, None, 0, out.ctypes.data)
    assert k >= 0, L.syzcov_last_error()
    assert out[:k].tolist() == list(orc.minimize_csr(off, pcs))
