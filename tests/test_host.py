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
