"""Full-size parity: the engine at BASELINE.json's own sizes against the CPU
oracle's digests (tests/golden/fullsize_digests.json, written by
tools/gen_golden_fullsize.py from oracle/fullsize.c).

  C2  1M inputs, one GPU                      kept / union / order / lens digests
  C2X C2 over the x86-like universe (kshift 2, 2^23 keys), both canon layouts
  C3  10M inputs (82 GB raw), one GPU         kept / union / order / lens digests
  C3  canonical lengths in 1M chunks + the 10M Go sort order on the device
  C2  world-8 sharded rehearsal on one GPU    kept / union / order digests
  C3  world-8 sharded rehearsal on one GPU    kept / union / order digests (in place)
  C4  1M programs: raw co-occurrence counts against the closed form
      D[i][j] = #{p : len(p) > max(i, j)}, D[i][i] = 0 (prio.go:137-154)
  C5  the bench's new-coverage stream: 32 history batches + 2 more of 65,536
      call records over 293 calls (key and window mode), per-batch is_new
      and the final per-call maxCover against oracle/newcov_full.c
"""
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


def sha(t) -> str:
    return hashlib.sha256(t.cpu().numpy().astype("<i4").tobytes()).hexdigest()


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available()
    return t


def _engine_vs_digest(torch, name, inplace, keys=True, layout=0):
    from syzkaller_amd.engine import CorpusEngine, synth_corpus, synth_universe, synth_window
    g = golden(name)
    n = g["n"]
    x86 = bool(g.get("synth_mode", 0) & 2)
    off, raw, lens, total = synth_corpus(n, g["seed"], mean=g["mean"], sigma=g["sigma"],
                                         log2_space=g["log2_space"], x86=x86)
    assert total == g["raw_pcs"]
    lo, span = synth_window(g["log2_space"], x86=x86)
    univ = synth_universe(g["log2_space"], g["seed"], x86=x86) if keys else None
    eng = CorpusEngine(n, total, int(lens.max().item()), lo, span, canon_in_place=inplace,
                       universe=univ, canon_layout=layout)
    assert eng.key_mode == keys
    res = eng.step(off, raw, n)
    assert int(eng.new_len[:n].to(torch.int64).sum().item()) == g["canonical_pcs"]
    assert sha(eng.new_len[:n]) == g["lens_sha256"]
    assert sha(eng.order[:n]) == g["order_sha256"]
    assert res.n_kept == g["n_kept"]
    assert res.kept_idx[:16].cpu().tolist() == g["kept_head"]
    assert sha(res.kept_idx) == g["kept_sha256"]
    assert res.n_union == g["n_union"] and res.max_cover == g["n_union"]
    assert sha(res.union) == g["union_sha256"]
    return eng, off, raw


@pytest.mark.parametrize("keys", [True, False], ids=["key-mode", "window-mode"])
def test_c2_fullsize_digest(torch, keys):
    """Config C2 (1M inputs, 2.05 G raw PCs) on one GPU, dense universe keys
    and window offsets: bit-exact kept list, union, canonical lengths and Go
    sort order; a second step (engine state reused, maxCover saturated) gives
    the same."""
    eng, off, raw = _engine_vs_digest(torch, "C2", inplace=False, keys=keys)
    g = golden("C2")
    res = eng.step(off, raw, g["n"])
    assert sha(res.kept_idx) == g["kept_sha256"] and sha(res.union) == g["union_sha256"]


@pytest.mark.parametrize("layout", [0, 1], ids=["csr", "aligned"])
def test_c2x_fullsize_digest(torch, layout):
    """C2 over the x86-like universe (PCs 5..14 bytes apart): kshift 2, 2^23
    dense keys (the 3-pass canon sort) against the oracle's C2X digests,
    canonical lists in both layouts: CSR with Minimize's nibble tables (32
    ranges of 2^18 keys), line-aligned with byte tables (64 of 2^17)."""
    eng, off, raw = _engine_vs_digest(torch, "C2X", inplace=False, layout=layout)
    assert eng.kshift == 2 and eng.span == (1 << 23) - 1
    assert eng.nrange == (32 if layout == 0 else 64)


def test_c3_fullsize_digest(torch):
    """Config C3 (10M inputs, 20.5 G raw PCs = 82 GB) on ONE 288 GB GPU,
    canonicalized in place: bit-exact against the oracle's digests."""
    free, _ = torch.cuda.mem_get_info()
    if free < 120 << 30:
        pytest.skip(f"C3 needs ~100 GB of HBM, {free >> 30} GB free")
    eng, off, raw = _engine_vs_digest(torch, "C3", inplace=True)
    del eng, off, raw
    torch.cuda.empty_cache()


def test_c3_order_chunked(torch):
    """C3's 10M canonical lengths, canonicalized 1M inputs at a time, and the
    device restatement of Go's sort.Sort over all 10M of them."""
    from syzkaller_amd.engine import CorpusEngine, synth_corpus, synth_universe, synth_window
    g = golden("C3")
    n, chunk = g["n"], 1_000_000
    lo, span = synth_window(g["log2_space"])
    lens = torch.empty(n, dtype=torch.int32, device="cuda")
    eng = None
    for c0 in range(0, n, chunk):
        off, raw, l_, total = synth_corpus(chunk, g["seed"], first=c0, mean=g["mean"],
                                           sigma=g["sigma"], log2_space=g["log2_space"])
        if eng is None:
            eng = CorpusEngine(chunk, int(total * 1.01), 16384, lo, span, n_global=n,
                               universe=synth_universe(g["log2_space"], g["seed"]))
        eng.canonicalize(off, raw, chunk)
        lens[c0:c0 + chunk].copy_(eng.new_len[:chunk])
        del off, raw
    assert sha(lens) == g["lens_sha256"]
    eng.sort_order(lens, n)
    assert sha(eng.order[:n]) == g["order_sha256"]


@pytest.mark.parametrize("keys", ["keys", "window"])
def test_world8_rehearsal_c2(torch, keys):
    """Eight ranks of the sharded engine on one GPU (gloo collectives) over C2,
    checked against the ORACLE's digests (not against the single-GPU engine).
    Key mode exchanges the first-cover array (MIN) and kept flags (MAX);
    window mode the covered bitmaps, first ranks over the merged dictionary
    and kept flags."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(HERE, "gpu_dist_rehearse.py"), "8", "C2",
                        keys], capture_output=True, text=True, timeout=280)
    assert r.returncode == 0 and r.stdout.count("OK") == 8, r.stdout[-3000:] + r.stderr[-3000:]


def test_world4_rehearsal_c2x(torch):
    """Four ranks over C2X (the x86-like universe: kshift 2, Minimize's nibble
    tables) on one GPU against the oracle's C2X digests."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(HERE, "gpu_dist_rehearse.py"), "4", "C2X",
                        "keys"], capture_output=True, text=True, timeout=280)
    assert r.returncode == 0 and r.stdout.count("OK") == 4, r.stdout[-3000:] + r.stderr[-3000:]


def test_world8_rehearsal_c3(torch):
    """Eight ranks over C3 (10M inputs, 82 GB of raw PCs, 1.25M per rank,
    canonicalized in place) on one GPU: the 8-GPU bench's workload and data
    path, rehearsed against the ORACLE's C3 digests (kept list, union, Go
    order over all 10M canonical lengths)."""
    import subprocess
    import sys
    free, _ = torch.cuda.mem_get_info()
    if free < 140 << 30:
        pytest.skip(f"the C3 rehearsal needs ~110 GB of HBM, {free >> 30} GB free")
    r = subprocess.run([sys.executable, os.path.join(HERE, "gpu_dist_rehearse.py"), "8", "C3",
                        "keys"], capture_output=True, text=True, timeout=560)
    assert r.returncode == 0 and r.stdout.count("OK") == 8, r.stdout[-3000:] + r.stderr[-3000:]


def test_c4_closed_form_1m(torch):
    """C4: 1M programs with lengths ~ N(30, 8) (the bench's own generator):
    the raw co-occurrence counts of the i8-MFMA AᵀA are exactly
    D[i][j] = #{p : len(p) > max(i, j)} (i != j), D[i][i] = 0; the normalised
    priorities equal the oracle's normalizePrio of that matrix."""
    import ctypes as C
    from syzkaller_amd import _lib
    from syzkaller_amd.engine import PrioEngine, _stream
    L = _lib.lib()
    nprog, seed = 1_000_000, 0x5EED0004
    eng = PrioEngine(nprog)
    lens = torch.empty(nprog, dtype=torch.int32, device="cuda")
    _lib.check(L.syzcov_dev_synth_lens(seed, 0, nprog, 30, 8, C.c_void_p(lens.data_ptr()),
                                       _stream()), "synth_lens")
    out = eng.step(lens)
    Cn = eng.C
    raw = torch.empty(Cn * Cn, dtype=torch.int32, device="cuda")
    _lib.check(L.syzcov_dev_prio_finish(C.c_void_p(eng.counts.data_ptr()), Cn, None,
                                        C.c_void_p(eng.out.data_ptr()), C.c_void_p(raw.data_ptr()),
                                        _stream()), "prio_finish")
    hl = lens.cpu().numpy()
    assert np.array_equal(hl[:2000], orc.synth_lens(seed, 2000, 30, 8).astype(np.int32))
    gt = np.zeros(Cn + 1, np.int64)  # gt[m] = #{p : len(p) > m}
    h = np.bincount(hl, minlength=Cn + 1)
    gt[:Cn + 1] = nprog - np.cumsum(h)[:Cn + 1]
    idx = np.arange(Cn)
    D = gt[np.maximum(idx[:, None], idx[None, :])]
    np.fill_diagonal(D, 0)
    got = raw.cpu().numpy().astype(np.int64).reshape(Cn, Cn)
    assert np.array_equal(got, D)
    # normalised (no static factor) == normalizePrio of the exact float32 counts
    exp = orc.normalize_prio(D.astype(np.float32))
    assert np.array_equal(eng.out.cpu().numpy().reshape(Cn, Cn), exp)
    assert out is eng.out


def test_c4_dense_closed_form(torch):
    """The dense contraction (all C keys, AT in HBM: the bench's --prio-dense
    line, 256 x 256 MFMA tiles with partial tiles and one reduction) gives the
    same exact counts as the closed form D[i][j] = #{p : len(p) > max(i, j)}."""
    import ctypes as C
    from syzkaller_amd import _lib
    from syzkaller_amd.engine import PrioEngine, _stream
    L = _lib.lib()
    nprog, seed = 300_000, 0x5EED0004
    eng = PrioEngine(nprog, active_rows=False)
    assert eng.tile == 256  # C = 1170: 1280 rows, five 256-row tile rows
    lens = torch.empty(nprog, dtype=torch.int32, device="cuda")
    _lib.check(L.syzcov_dev_synth_lens(seed, 0, nprog, 30, 8, C.c_void_p(lens.data_ptr()),
                                       _stream()), "synth_lens")
    eng.step(lens)
    Cn = eng.C
    raw = torch.empty(Cn * Cn, dtype=torch.int32, device="cuda")
    _lib.check(L.syzcov_dev_prio_finish(C.c_void_p(eng.counts.data_ptr()), Cn, None,
                                        C.c_void_p(eng.out.data_ptr()), C.c_void_p(raw.data_ptr()),
                                        _stream()), "prio_finish")
    hl = lens.cpu().numpy()
    h = np.bincount(hl, minlength=Cn + 1)
    gt = nprog - np.cumsum(h)[:Cn + 1].astype(np.int64)
    idx = np.arange(Cn)
    D = gt[np.maximum(idx[:, None], idx[None, :])]
    np.fill_diagonal(D, 0)
    assert np.array_equal(raw.cpu().numpy().astype(np.int64).reshape(Cn, Cn), D)


@pytest.mark.parametrize("name,keys", [("C5", True), ("C5", False), ("C5S", True)],
                         ids=["early-key-mode", "early-window-mode", "steady-key-mode"])
def test_c5_newcov_stream_fullsize(torch, name, keys):
    """Config C5 at its own size (syz-fuzzer/fuzzer.go:456-480): the stream
    bench.py --workload newcov times (seed 0x5EED0005, batch b = records
    b * 65536 ..), every batch through syzcov_state_newcov_dev, is_new of each
    batch and every call's maxCover at the end bit-identical to the oracle.
    C5: 32 history batches + the 2 timed ones (every record still new);
    C5S: 512 + 2, the steady state the bench reports (maxCover near
    saturation; new counts of every batch, digests of the last two)."""
    import ctypes as C
    from syzkaller_amd import _lib
    from syzkaller_amd.engine import synth_corpus, synth_records, synth_universe, synth_window
    from syzkaller_amd.fuzzer import CoverState
    g = golden(name)
    first_digest = g.get("is_new_sha256_first_batch", 0)
    L = _lib.lib()
    P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    s = lambda: C.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
    lo, span = synth_window(g["log2_space"])
    st = CoverState(g["ncalls"], lo, span)
    if keys:
        u = synth_universe(g["log2_space"], g["seed"])
        st.set_universe(u.cpu().numpy().view(np.uint32))
        del u
    fo, fp, _, _ = synth_corpus(1, g["seed"], first=1 << 40, mean=1 << (g["log2_space"] - 7),
                                sigma=1, log2_space=g["log2_space"])
    st.set_flakes(np.unique(fp[:int(fo[1].item())].cpu().numpy().view(np.uint32)))
    nrec = g["records"]
    is_new = torch.empty(nrec, dtype=torch.uint8, device="cuda")
    stats = torch.zeros(2, dtype=torch.int32, device="cuda")
    total = 0
    for b in range(g["batches"]):
        cid, roff, pcs, npc = synth_records(nrec, g["seed"], b * nrec, g["ncalls"],
                                            mean=g["mean"], sigma=g["sigma"],
                                            log2_space=g["log2_space"])
        total += npc
        wsz = L.syzcov_state_newcov_ws_size(nrec, npc)
        ws = torch.empty(wsz, dtype=torch.uint8, device="cuda")
        _lib.check(L.syzcov_state_newcov_dev(st.h, P(cid), P(roff), P(pcs), nrec, npc, P(is_new),
                                             P(stats), P(ws), wsz, s()), "state_newcov_dev")
        assert int(stats[0].item()) == 0, b
        assert int(is_new.sum().item()) == g["new_per_batch"][b], b
        if b >= first_digest:
            h = hashlib.sha256(is_new.cpu().numpy().tobytes()).hexdigest()
            assert h == g["is_new_sha256"][b - first_digest], b
        del ws, pcs
    assert total == g["record_pcs"]
    mn = np.array([st.max_cover(c).size for c in range(g["ncalls"])], np.uint32)
    assert int(mn.sum()) == g["max_cover_total"]
    assert hashlib.sha256(mn.tobytes()).hexdigest() == g["max_cover_n_sha256"]
    hh = hashlib.sha256()
    for c in range(g["ncalls"]):
        hh.update(st.max_cover(c).astype("<u4").tobytes())
    assert hh.hexdigest() == g["max_cover_sha256"]
    st.close()


def _c2_host(torch, g):
    from syzkaller_amd.engine import synth_corpus
    off, raw, lens, total = synth_corpus(g["n"], g["seed"], mean=g["mean"], sigma=g["sigma"],
                                         log2_space=g["log2_space"])
    assert total == g["raw_pcs"]
    h_off = off.cpu().numpy().astype(np.uint64)
    h_pcs = raw[:total].cpu().numpy().view(np.uint32).copy()
    del off, raw
    torch.cuda.empty_cache()
    return h_off, h_pcs


def test_c2_dropin_raw_covers_digest(torch):
    """cover.Minimize through the drop-in C-ABI (host buffers) on C2's RAW
    covers, as the cgo shim calls it: with the caller's own sort.Sort order
    over len(cov) (here the library's restated order over the raw lengths
    stands in for Go's) and without an order: the oracle's kept list (C2R,
    oracle/grouped_full.c with one group)."""
    from syzkaller_amd import _lib
    L = _lib.lib()
    g = golden("C2R")
    h_off, h_pcs = _c2_host(torch, g)
    n = g["n"]
    out = np.empty(n, np.int32)
    rl = np.diff(h_off).astype(np.int64)
    order = np.empty(n, np.int32)
    _lib.check(L.syzcov_sort_order(rl.ctypes.data, n, 0, order.ctypes.data), "sort_order")
    for op in (order, None):
        k = _lib.check(L.syzcov_minimize(h_off.ctypes.data, h_pcs.ctypes.data, n,
                                         None if op is None else op.ctypes.data, 0,
                                         out.ctypes.data), "minimize")
        assert k == g["n_kept"]
        assert out[:16].tolist() == g["kept_head"]
        assert hashlib.sha256(out[:k].astype("<i4").tobytes()).hexdigest() == g["kept_sha256"]
    L.syzcov_pool_trim()


def test_c2_minimize_corpus_293_groups_digest(torch):
    """Manager.minimizeCorpus (manager.go:504-524) on C2's raw covers in 293
    call groups (synthetic call ids) through syzcov_minimize_corpus (the
    engine's per-group Minimize over one rank space): the oracle's kept
    corpus indices, groups in ascending call id (C2G, oracle/grouped_full.c)."""
    import ctypes as C
    from syzkaller_amd import _lib
    L = _lib.lib()
    g = golden("C2G")
    h_off, h_pcs = _c2_host(torch, g)
    n = g["n"]
    cid = torch.empty(n, dtype=torch.int32, device="cuda")
    _lib.check(L.syzcov_dev_synth_callids(g["seed"], 0, n, g["ncalls"], C.c_void_p(cid.data_ptr()),
                                          C.c_void_p(torch.cuda.current_stream().cuda_stream)),
               "synth_callids")
    calls = cid.cpu().numpy().astype(np.int32)
    out = np.empty(n, np.int32)
    k = _lib.check(L.syzcov_minimize_corpus(calls.ctypes.data, h_off.ctypes.data,
                                            h_pcs.ctypes.data, n, 0, out.ctypes.data),
                   "minimize_corpus")
    assert k == g["n_kept"]
    assert out[:16].tolist() == g["kept_head"]
    assert hashlib.sha256(out[:k].astype("<i4").tobytes()).hexdigest() == g["kept_sha256"]
    L.syzcov_pool_trim()
