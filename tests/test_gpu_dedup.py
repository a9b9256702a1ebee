"""GPU parity: the executor's cover_dedup (executor/executor.cc:574-587) of
raw u64 KCOV buffers (dedup.hip, syzcov_dev_cover_dedup64 and the host
syzcov_cover_dedup64) against the C oracle.  Bit-exact.  The oracle is
parity unpinned by reference fixtures (test_oracle.py)."""
import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu

# every branch: one tile of 16 .. 4096 values, and the in-HBM merges of
# 2 .. 16 tiles with ragged last tiles (kCoverSize = 64K, executor.cc:50)
LENS = [0, 1, 2, 3, 15, 16, 17, 31, 100, 255, 256, 257, 1000, 1023, 1024, 1025, 2048,
        4095, 4096, 4097, 5000, 8191, 8192, 8193, 12288, 16385, 40000, 65535]


def _buf(rng, n, kind):
    if kind == "kernel":  # x86-64 kernel text, loops repeat PCs
        return np.uint64(0xffffffff81000000) + rng.integers(0, 1 << 16, n).astype(np.uint64)
    if kind == "dense":  # many zeros and duplicates
        return rng.integers(0, 64, n).astype(np.uint64)
    if kind == "wide":  # any u64, including 0 and ~0
        b = rng.integers(0, 2**64, n, dtype=np.uint64)
        if n > 4:
            b[rng.integers(0, n, 3)] = np.uint64(2**64 - 1)
            b[rng.integers(0, n, 2)] = 0
        return b
    if kind == "cross":  # u32 keys across a 2^32 boundary; spans up to 2^32 - 1
        b = np.uint64(0xFFFFFF00) + rng.integers(0, 512, n).astype(np.uint64)
        if n > 4 and n % 2:
            b[0] = np.uint64(0x1_0000_0000 - 7)
            b[1] = np.uint64(0x1_0000_0000 - 7 + 0xFFFFFFFF)  # span exactly 2^32 - 1
        return b
    if kind == "sorted":
        return np.sort(rng.integers(1, 1 << 40, n).astype(np.uint64))
    return np.sort(rng.integers(1, 1 << 40, n).astype(np.uint64))[::-1].copy()  # reversed


def _run(lens, bufs, out32=True):
    import torch
    from syzkaller_amd._lib import check, lib
    from syzkaller_amd.engine import _p, _stream
    off = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(np.asarray(lens, np.uint64), out=off[1:])
    flat = np.concatenate(bufs + [np.zeros(1, np.uint64)])
    d_pcs = torch.from_numpy(flat.view(np.int64).copy()).cuda()
    d_off = torch.from_numpy(off.view(np.int64)).cuda()
    d_len = torch.full((len(lens),), 7, dtype=torch.int32, device="cuda")
    d_o32 = torch.zeros(flat.size, dtype=torch.int32, device="cuda") if out32 else None
    check(lib().syzcov_dev_cover_dedup64(_p(d_pcs), _p(d_off), len(lens), _p(d_len),
                                         _p(d_o32) if out32 else None, _stream()),
          "dev_cover_dedup64")
    torch.cuda.synchronize()
    pcs = d_pcs.cpu().numpy().view(np.uint64)
    nl = d_len.cpu().numpy().view(np.uint32)
    o32 = d_o32.cpu().numpy().view(np.uint32) if out32 else None
    return off, pcs, nl, o32


@pytest.mark.parametrize("kind", ["kernel", "dense", "wide", "sorted", "reversed", "cross"])
def test_dedup_batch_vs_oracle(kind):
    rng = np.random.default_rng(["kernel", "dense", "wide", "sorted", "reversed", "cross"].index(kind))
    lens = list(LENS) + list(rng.integers(0, 3000, 40))
    rng.shuffle(lens)
    bufs = [_buf(rng, int(n), kind) for n in lens]
    off, pcs, nl, o32 = _run(lens, bufs)
    for s, b in enumerate(bufs):
        want = orc.cover_dedup64(b)
        k = int(off[s])
        assert nl[s] == want.size, (kind, s, len(b))
        assert np.array_equal(pcs[k:k + want.size], want), (kind, s, len(b))
        # executor.cc:459-463 writes (uint32_t)cover_data[i]
        assert np.array_equal(o32[k:k + want.size], (want & np.uint64(0xFFFFFFFF)).astype(np.uint32))


def test_dedup_without_out32_and_repeat():
    rng = np.random.default_rng(5)
    lens = [65535, 3, 4097, 0, 9000]
    bufs = [_buf(rng, n, "kernel") for n in lens]
    off, pcs, nl, _ = _run(lens, bufs, out32=False)
    for s, b in enumerate(bufs):
        want = orc.cover_dedup64(b)
        assert nl[s] == want.size and np.array_equal(pcs[int(off[s]):int(off[s]) + want.size], want)


def test_dedup_many_small_buffers():
    # more buffers than the grid (2^20 workgroups): the grid-stride loop
    rng = np.random.default_rng(9)
    n = (1 << 20) + 37
    lens = rng.integers(0, 4, n)
    flat = rng.integers(0, 3, int(lens.sum())).astype(np.uint64)
    off0 = np.zeros(n + 1, np.uint64)
    np.cumsum(lens.astype(np.uint64), out=off0[1:])
    bufs = [flat[int(off0[i]):int(off0[i + 1])] for i in range(n)]
    off, pcs, nl, o32 = _run(list(lens), bufs)
    for s in list(range(0, n, 997)) + [n - 1]:
        want = orc.cover_dedup64(bufs[s])
        assert nl[s] == want.size and np.array_equal(pcs[int(off[s]):int(off[s]) + want.size], want)
    # the whole batch at once: every kept count and the compacted prefixes
    exp_len = np.array([np.count_nonzero(np.unique(b)) for b in bufs[:20000]], np.uint32)
    assert np.array_equal(nl[:20000], exp_len)


def test_dedup_malformed_offsets_flagged():
    import torch
    from syzkaller_amd._lib import check, lib
    from syzkaller_amd.engine import _p, _stream
    off = np.array([0, 6, 2], np.uint64)  # segment 1 runs backwards
    pcs = np.arange(8, 0, -1).astype(np.uint64)
    d_pcs = torch.from_numpy(pcs.view(np.int64).copy()).cuda()
    d_off = torch.from_numpy(off.view(np.int64)).cuda()
    d_len = torch.zeros(2, dtype=torch.int32, device="cuda")
    check(lib().syzcov_dev_cover_dedup64(_p(d_pcs), _p(d_off), 2, _p(d_len), None, _stream()),
          "dev_cover_dedup64")
    nl = d_len.cpu().numpy().view(np.uint32)
    assert nl[0] == 6 and nl[1] == 0xFFFFFFFF
    got = d_pcs.cpu().numpy().view(np.uint64)
    assert got.tolist() == [3, 4, 5, 6, 7, 8, 2, 1]


def test_host_cover_dedup():
    from syzkaller_amd.fuzzer import cover_dedup
    rng = np.random.default_rng(3)
    for n in (0, 1, 5, 4096, 4097, 65535):
        for kind in ("kernel", "wide", "dense"):
            b = _buf(rng, n, kind)
            assert np.array_equal(cover_dedup(b), orc.cover_dedup64(b)), (n, kind)


def test_ingest_into_newcov():
    """raw u64 KCOV buffers -> cover_dedup -> u32 words packed as
    records (syzcov_dev_cover_ingest64) -> the fuzzer's new-coverage check
    (syzcov_state_newcov_dev), all on the device, against the oracle's
    cover_dedup + newcov_batch (fuzzer.go:456-480) over the same buffers."""
    import torch
    from syzkaller_amd._lib import check, lib
    from syzkaller_amd.engine import _p, _stream
    from syzkaller_amd.fuzzer import CoverState
    rng = np.random.default_rng(21)
    ncalls, lo, span = 17, 0x81000000, 1 << 16
    lens = [int(x) for x in rng.integers(0, 3000, 600)] + [0, 1, 5000, 9000, 4096]
    bufs = [np.uint64(0xffffffff00000000 + lo) + rng.integers(0, span, n).astype(np.uint64)
            for n in lens]
    for b in bufs[::7]:  # a few zero PCs (dropped by cover_dedup)
        if b.size:
            b[0] = 0
    callids = rng.integers(0, ncalls, len(lens)).astype(np.int32)
    off = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(np.asarray(lens, np.uint64), out=off[1:])
    total = int(off[-1])
    L = lib()
    d_pcs = torch.from_numpy(np.concatenate(bufs).view(np.int64).copy()).cuda()
    d_off = torch.from_numpy(off.view(np.int64)).cuda()
    d_roff = torch.zeros(len(lens) + 1, dtype=torch.int64, device="cuda")
    d_rpcs = torch.zeros(total, dtype=torch.int32, device="cuda")
    d_err = torch.zeros(1, dtype=torch.int32, device="cuda")
    wsz = L.syzcov_dev_cover_ingest64_ws_size(len(lens), total)
    ws = torch.empty(wsz, dtype=torch.uint8, device="cuda")
    check(L.syzcov_dev_cover_ingest64(_p(d_pcs), _p(d_off), len(lens), total, _p(d_roff),
                                      _p(d_rpcs), _p(d_err), _p(ws), wsz, _stream()),
          "dev_cover_ingest64")
    recs = [(orc.cover_dedup64(b) & np.uint64(0xFFFFFFFF)).astype(np.uint32) for b in bufs]
    roff = d_roff.cpu().numpy().view(np.uint64)
    rpcs = d_rpcs.cpu().numpy().view(np.uint32)
    assert int(d_err.item()) == 0
    assert roff.tolist() == np.concatenate([[0], np.cumsum([r.size for r in recs])]).tolist()
    for k, r in enumerate(recs):
        assert np.array_equal(rpcs[int(roff[k]):int(roff[k + 1])], r), k
    # the same records through the device new-coverage check, twice (the
    # second batch sees the first's maxCover)
    st = CoverState(ncalls, lo, span)
    exp_mc = [[] for _ in range(ncalls)]
    d_cid = torch.from_numpy(callids).cuda()
    npc = int(roff[-1])
    nwsz = L.syzcov_state_newcov_ws_size(len(lens), npc)
    nws = torch.empty(nwsz, dtype=torch.uint8, device="cuda")
    for rep in range(2):
        flags = torch.zeros(len(lens), dtype=torch.uint8, device="cuda")
        stats = torch.zeros(2, dtype=torch.int32, device="cuda")
        check(L.syzcov_state_newcov_dev(st.h, _p(d_cid), _p(d_roff), _p(d_rpcs), len(lens), npc,
                                        _p(flags), _p(stats), _p(nws), nwsz, _stream()),
              "state_newcov_dev")
        exp, exp_mc = orc.newcov_batch(exp_mc, [], callids, recs)
        assert int(stats[0].item()) == 0
        assert np.array_equal(flags.cpu().numpy(), exp), rep
        assert (rep == 0) == bool(exp.any())
    for c in range(ncalls):
        assert np.array_equal(st.max_cover(c), exp_mc[c]), c
    st.close()


def test_ingest_flags_malformed_buffer():
    import torch
    from syzkaller_amd._lib import check, lib
    from syzkaller_amd.engine import _p, _stream
    # buffer 0 = [0, 6), buffer 1 runs backwards (6 -> 2), buffer 2 is empty
    off = np.array([0, 6, 2, 2], np.uint64)
    pcs = np.array([9, 3, 3, 7, 1, 2, 5, 5], np.uint64)
    L = lib()
    d_pcs = torch.from_numpy(pcs.view(np.int64).copy()).cuda()
    d_off = torch.from_numpy(off.view(np.int64)).cuda()
    d_roff = torch.full((4,), -1, dtype=torch.int64, device="cuda")
    d_rpcs = torch.zeros(8, dtype=torch.int32, device="cuda")
    d_err = torch.zeros(1, dtype=torch.int32, device="cuda")
    wsz = L.syzcov_dev_cover_ingest64_ws_size(3, 8)
    ws = torch.empty(wsz, dtype=torch.uint8, device="cuda")
    check(L.syzcov_dev_cover_ingest64(_p(d_pcs), _p(d_off), 3, 8, _p(d_roff), _p(d_rpcs),
                                      _p(d_err), _p(ws), wsz, _stream()), "dev_cover_ingest64")
    assert int(d_err.item()) == 1
    assert d_roff.cpu().tolist() == [0, 5, 5, 5]
    assert d_rpcs.cpu().numpy()[:5].tolist() == [1, 2, 3, 7, 9]
