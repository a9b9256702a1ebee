"""Resident fuzzer-side coverage state: per-CallID maxCover, corpusCover and
flakes on the GPU; the batched new-coverage check of syz-fuzzer execute()
(syz-fuzzer/fuzzer.go:456-480), addInput (:344-375) and triageInput's
coverage steps (:377-417)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, lib


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def _csr(lists):
    """list of PC lists -> (off u64[n+1], pcs u32[max(total, 1)])."""
    lens = np.fromiter((len(r) for r in lists), dtype=np.uint64, count=len(lists))
    off = np.zeros(len(lists) + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    pcs = (np.concatenate([np.asarray(r, dtype=np.uint32) for r in lists])
           if len(lists) and off[-1] else np.zeros(1, dtype=np.uint32))
    return off, np.ascontiguousarray(pcs, dtype=np.uint32)


class CoverState:
    def __init__(self, ncalls: int, pc_lo: int = 0, pc_span: int = 1 << 32):
        h = C.c_uint64(0)
        check(lib().syzcov_state_create(ncalls, pc_lo, pc_span, C.byref(h)), "state_create")
        self.h = h.value
        self.ncalls = ncalls

    def close(self):
        if self.h:
            lib().syzcov_state_destroy(self.h)
            self.h = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add(self, call: int, pcs):
        a = np.ascontiguousarray(pcs, dtype=np.uint32)
        check(lib().syzcov_state_add(self.h, call, _ptr(a), a.size), "state_add")

    def set_universe(self, pcs):
        """Known PC universe (allCoverPCs, syz-manager/cover.go:57-69) before
        the first add/check: maxCover of those PCs is kept over dense ids."""
        a = np.ascontiguousarray(pcs, dtype=np.uint32)
        check(lib().syzcov_state_set_universe(self.h, _ptr(a), a.size), "state_set_universe")

    def set_flakes(self, pcs):
        a = np.ascontiguousarray(pcs, dtype=np.uint32)
        check(lib().syzcov_state_set_flakes(self.h, _ptr(a), a.size), "state_set_flakes")

    def max_cover(self, call: int) -> np.ndarray:
        n = check(lib().syzcov_state_get(self.h, call, None, 0), "state_get")
        out = np.empty(max(n, 1), dtype=np.uint32)
        n = check(lib().syzcov_state_get(self.h, call, _ptr(out), out.size), "state_get")
        return out[:n]

    def corpus_add(self, call: int, pcs):
        """corpusCover[call] = Union(corpusCover[call], pcs) (fuzzer.go:451)."""
        a = np.ascontiguousarray(pcs, dtype=np.uint32)
        check(lib().syzcov_state_corpus_add(self.h, call, _ptr(a), a.size), "state_corpus_add")

    def corpus_cover(self, call: int) -> np.ndarray:
        n = check(lib().syzcov_state_corpus_get(self.h, call, None, 0), "state_corpus_get")
        out = np.empty(max(n, 1), dtype=np.uint32)
        n = check(lib().syzcov_state_corpus_get(self.h, call, _ptr(out), out.size),
                  "state_corpus_get")
        return out[:n]

    def flakes(self) -> np.ndarray:
        n = check(lib().syzcov_state_flakes_get(self.h, None, 0), "state_flakes_get")
        out = np.empty(max(n, 1), dtype=np.uint32)
        n = check(lib().syzcov_state_flakes_get(self.h, _ptr(out), out.size), "state_flakes_get")
        return out[:n]

    def add_inputs(self, callids, covers) -> np.ndarray:
        """addInput (fuzzer.go:344-375) for manager-pushed inputs in order
        (covers already canonical): accepted[k]; accepted covers join
        corpusCover and maxCover."""
        cid = np.ascontiguousarray(callids, dtype=np.int32)
        off, pcs = _csr(covers)
        acc = np.zeros(max(len(covers), 1), dtype=np.uint8)
        check(lib().syzcov_state_add_inputs(self.h, _ptr(cid), _ptr(off), _ptr(pcs), len(covers),
                                            _ptr(acc)), "state_add_inputs")
        return acc[:len(covers)]

    def triage(self, callids, covers, runs):
        """triageInput's coverage steps (fuzzer.go:377-417) for a batch:
        covers[t] the input's cover, runs[t] its three re-execution covers
        (empty = not executed).  Returns (len(newCover) per input,
        stableNewCover per input); flakes grows by the runs' symmetric
        differences (see syzcov_state_triage for the schedule)."""
        n = len(covers)
        assert len(runs) == n and all(len(r) == 3 for r in runs)
        cid = np.ascontiguousarray(callids, dtype=np.int32)
        coff, cpcs = _csr(covers)
        roff, rpcs = _csr([r for rr in runs for r in rr])
        new_cnt = np.zeros(max(n, 1), dtype=np.uint32)
        st_cnt = np.zeros(max(n, 1), dtype=np.uint32)
        st_pcs = np.zeros(max(cpcs.size, 1), dtype=np.uint32)
        check(lib().syzcov_state_triage(self.h, n, _ptr(cid), _ptr(coff), _ptr(cpcs), _ptr(roff),
                                        _ptr(rpcs), _ptr(new_cnt), _ptr(st_cnt), _ptr(st_pcs)),
              "state_triage")
        stable = [st_pcs[int(coff[t]):int(coff[t]) + int(st_cnt[t])].copy() for t in range(n)]
        return new_cnt[:n], stable

    def new_coverage(self, callids, records) -> np.ndarray:
        """is_new[k] for a batch of executed call records, in batch order,
        updating maxCover exactly like the sequential reference loop."""
        lens = np.fromiter((len(r) for r in records), dtype=np.uint64, count=len(records))
        off = np.zeros(len(records) + 1, dtype=np.uint64)
        np.cumsum(lens, out=off[1:])
        pcs = (np.concatenate([np.asarray(r, dtype=np.uint32) for r in records])
               if len(records) and off[-1] else np.zeros(1, dtype=np.uint32))
        return self.new_coverage_csr(callids, off, pcs)

    def new_coverage_csr(self, callids, off, pcs) -> np.ndarray:
        cid = np.ascontiguousarray(callids, dtype=np.int32)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        pcs = np.ascontiguousarray(pcs, dtype=np.uint32)
        nrec = off.size - 1
        is_new = np.zeros(max(nrec, 1), dtype=np.uint8)
        check(lib().syzcov_newcov_batch(self.h, _ptr(cid), _ptr(off), _ptr(pcs), nrec,
                                        _ptr(is_new)), "newcov_batch")
        return is_new[:nrec]


def cover_dedup(cov) -> np.ndarray:
    """The executor's cover_dedup (executor/executor.cc:574-587) of one raw
    u64 KCOV buffer on the GPU: the sorted distinct nonzero PCs.  Batches of
    device-resident buffers: syzcov_dev_cover_dedup64."""
    a = np.ascontiguousarray(np.asarray(cov, dtype=np.uint64)).copy()
    n = check(lib().syzcov_cover_dedup64(_ptr(a), a.size), "cover_dedup") if a.size else 0
    return a[:n]


def parse_exec_output(out: bytes, call_num, callid_of_num):
    """Executor output of one program (ipc/ipc.go:225-291) -> (errnos,
    records) where records = (callid[], call_index[], off[], pcs[]) are the
    calls execute() checks (fuzzer.go:456-460), in call order, empty covers
    skipped.  Host-side parser of libsyzcov (no GPU needed)."""
    buf = np.frombuffer(out, dtype=np.uint8)
    buf = np.ascontiguousarray(buf) if buf.size else np.zeros(1, np.uint8)
    cn = np.ascontiguousarray(call_num, dtype=np.uint32)
    cmap = np.ascontiguousarray(callid_of_num, dtype=np.int32)
    nc = cn.size
    errnos = np.empty(max(nc, 1), np.int64)
    rcid = np.empty(max(nc, 1), np.int32)
    rci = np.empty(max(nc, 1), np.uint32)
    roff = np.zeros(nc + 1, np.uint64)
    cap = max(len(out) // 4, 1)
    pcs = np.empty(cap, np.uint32)
    n = check(lib().syzcov_parse_exec_output(_ptr(buf), len(out), nc, _ptr(cn) if nc else None,
                                             _ptr(cmap) if cmap.size else None, cmap.size,
                                             _ptr(errnos), _ptr(rcid), _ptr(rci), _ptr(roff),
                                             _ptr(pcs), cap), "parse_exec_output")
    return errnos[:nc], (rcid[:n], rci[:n], roff[:n + 1], pcs[:int(roff[n])])
