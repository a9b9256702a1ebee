"""libsyzcov's host-side logic (no GPU): the executor output parser against
the literal ipc.go reader restatement."""
import numpy as np
import pytest

from oracle import pyref


def _exec_output(rng, ncalls, call_num, done_frac=0.8, lo=0, span=1 << 32):
    """A well-formed executor output (executor.cc:455-466) for one program:
    a random subset of calls completes, in random order."""
    import struct
    done = [i for i in range(ncalls) if rng.random() < done_frac]
    rng.shuffle(done)
    body = b""
    for ci in done:
        cov = sorted(set(lo + int(x) for x in rng.integers(0, span, size=int(rng.integers(0, 40)),
                                                            dtype=np.uint64)))
        err = int(rng.choice([0, 0, 14, 0xFFFFFFF0]))
        body += struct.pack("<4I", ci, call_num[ci], err, len(cov))
        body += struct.pack(f"<{len(cov)}I", *cov)
    return struct.pack("<I", len(done)) + body


def test_parse_exec_output_vs_restatement():
    """libsyzcov's host parser (no GPU) against the literal ipc.go reader."""
    import struct
    from syzkaller_amd.fuzzer import parse_exec_output
    from syzkaller_amd import SyzcovError
    rng = np.random.default_rng(41)
    callid_of_num = rng.integers(0, 293, size=1170).tolist()
    for _ in range(200):
        ncalls = int(rng.integers(0, 12))
        call_num = rng.integers(0, 1170, size=ncalls).tolist()
        out = _exec_output(rng, ncalls, call_num)
        exp_err, exp_recs = pyref.parse_exec_output(out, call_num, callid_of_num)
        errnos, (cid, ci, off, pcs) = parse_exec_output(out, call_num, callid_of_num)
        assert errnos.tolist() == exp_err
        got = [(int(cid[k]), int(ci[k]), pcs[off[k]:off[k + 1]].tolist()) for k in range(cid.size)]
        assert got == exp_recs
    # the reader's error cases
    cn = [5, 6]
    bad = [struct.pack("<I", 1),                                   # short
           struct.pack("<5I", 1, 2, 5, 0, 0),                      # call index out of range
           struct.pack("<9I", 2, 0, 5, 0, 0, 0, 5, 0, 0),          # double coverage
           struct.pack("<5I", 1, 1, 5, 0, 0),                      # wrong syscall number
           struct.pack("<5I", 1, 0, 5, 0, 3)]                      # cover past the end
    for b in bad:
        with pytest.raises((ValueError, IndexError)):
            pyref.parse_exec_output(b, cn, callid_of_num)
        with pytest.raises(SyzcovError):
            parse_exec_output(b, cn, callid_of_num)


def _chunk_items_by_marks(nch, ug_windows):
    """Host emulation of pass1_stream_kernel's item lookup (minimize_range.hip):
    64 items with chunk counts nch (empty sub-runs allowed); per 64-chunk window,
    items starting inside it mark (index + 1) at their start offset (max on
    collision), a prefix max over the 64 lanes carries each mark forward, and
    the item covering the previous window's last chunk fills the lanes before
    the first mark.  Returns the item of every chunk of the stream."""
    ex = np.concatenate([[0], np.cumsum(nch)[:-1]]).astype(np.int64)
    tot = int(np.sum(nch))
    sj, out = 0, []
    for cb in range(0, max(tot, 1) + 64 * ug_windows, 64):
        own = np.zeros(64, np.int64)
        for j in range(64):
            if 0 <= ex[j] - cb < 64:
                own[ex[j] - cb] = max(own[ex[j] - cb], j + 1)
        pm = np.maximum.accumulate(own)
        jl = np.where(pm > 0, np.maximum(sj, pm - 1), sj)
        sj = int(jl[63])
        out.extend(int(jl[l]) for l in range(64) if cb + l < tot)
    return np.array(out, np.int64), ex


@pytest.mark.parametrize("seed", range(6))
def test_pass1_item_marks_match_searchsorted(seed):
    """The mark + prefix-max lookup gives every chunk the last item starting
    at or before it (np.searchsorted), including empty sub-runs (items with no
    chunks share their start with the next item) and long runs spanning many
    windows."""
    rng = np.random.default_rng(seed)
    for _ in range(50):
        kind = rng.integers(0, 3)
        if kind == 0:
            nch = rng.integers(0, 40, 64)          # short runs, many starts per window
        elif kind == 1:
            nch = rng.integers(0, 300, 64)         # long runs
        else:
            nch = rng.integers(0, 3, 64) * rng.integers(0, 2, 64)  # mostly empty
        got, ex = _chunk_items_by_marks(nch, 2)
        tot = int(nch.sum())
        want = np.searchsorted(ex, np.arange(tot), side="right") - 1
        assert np.array_equal(got, want)
        # a chunk's item really holds it
        assert all(ex[j] <= c < ex[j] + nch[j] for c, j in enumerate(got))
