"""Python mirror of prog/prio.go's public surface, backed by libsyzcov:

    CalculatePriorities(corpus, static) -> C x C float32   (prio.go:29-38)
    normalizePrio(prios)                                   (prio.go:158-192)
    BuildChoiceTable(prios, enabled) -> ChoiceTable        (prio.go:202-228)
    ChoiceTable.Choose(rnd, call)                          (prio.go:230-249)

`corpus` is a list of programs, each the list of its calls' syscall ids
(the reference's p.Calls[i].Meta.ID).  key_mode=0 reproduces the reference's
calcDynamicPrio exactly — it counts call POSITIONS, not ids (prio.go:142-150)
— key_mode=1 counts by syscall id.  The static matrix (calcStaticPriorities,
prio.go:40-135) depends only on sys.Calls and is supplied by the caller.
"""
from __future__ import annotations

import bisect
import ctypes as C

import numpy as np

from ._lib import check, lib


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def _csr(corpus):
    lens = np.fromiter((len(p) for p in corpus), dtype=np.uint64, count=len(corpus))
    off = np.zeros(len(corpus) + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    ids = (np.concatenate([np.asarray(p, dtype=np.uint16) for p in corpus])
           if len(corpus) and off[-1] else np.zeros(1, dtype=np.uint16))
    return off, np.ascontiguousarray(ids, dtype=np.uint16)


_TABLE = None


def sys_table():
    """The syscall usage table (sys/*.txt restated by tools/gen_sys_table.py):
    1170 calls in Call.ID order, CallID per call, usage id -> [(call, weight)]."""
    global _TABLE
    if _TABLE is None:
        import json
        import os
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "sys_table.json")
        with open(path) as f:
            _TABLE = json.load(f)
    return _TABLE


def usage_csr(table=None):
    """Both CSR views of the usage table (see syzcov_static_priorities)."""
    t = table or sys_table()
    C_ = t["ncalls"]
    ids = sorted(t["uses"])
    id_off = np.zeros(len(ids) + 1, np.uint32)
    calls, ws = [], []
    by_call = [[] for _ in range(C_)]
    for k, ident in enumerate(ids):
        members = sorted(t["uses"][ident])
        for c, w in members:
            calls.append(c)
            ws.append(w)
            by_call[c].append((k, w))
        id_off[k + 1] = len(calls)
    call_off = np.zeros(C_ + 1, np.uint32)
    cids, cws = [], []
    for c in range(C_):
        for k, w in by_call[c]:
            cids.append(k)
            cws.append(w)
        call_off[c + 1] = len(cids)
    return (id_off, np.asarray(calls, np.uint16), np.asarray(ws, np.float32), call_off,
            np.asarray(cids, np.uint32), np.asarray(cws, np.float32), C_)


def StaticPriorities(table=None) -> np.ndarray:
    """calcStaticPriorities (prio.go:40-135) on the GPU."""
    id_off, calls, ws, call_off, cids, cws, C_ = usage_csr(table)
    out = np.empty((C_, C_), dtype=np.float32)
    check(lib().syzcov_static_priorities(
        _ptr(id_off), _ptr(calls), _ptr(ws), id_off.size - 1, _ptr(call_off), _ptr(cids),
        _ptr(cws), C_, _ptr(out)), "StaticPriorities")
    return out


def CalculatePriorities(corpus, static=None, ncalls: int | None = None, key_mode: int = 0,
                        return_raw: bool = False):
    """prio.go:29-38.  static=None with ncalls=None uses the sys/*.txt table
    (calcStaticPriorities on the GPU) like the reference does."""
    if static is None and ncalls is None:
        static = StaticPriorities()
    if static is not None:
        static = np.ascontiguousarray(static, dtype=np.float32)
        C_ = static.shape[0]
    else:
        if ncalls is None:
            raise ValueError("need the static matrix or ncalls")
        C_ = ncalls
    off, ids = _csr(corpus)
    out = np.empty((C_, C_), dtype=np.float32)
    raw = np.empty((C_, C_), dtype=np.uint32) if return_raw else None
    check(lib().syzcov_calculate_priorities(
        _ptr(off), _ptr(ids), len(corpus), C_, key_mode,
        _ptr(static) if static is not None else None, _ptr(out),
        _ptr(raw) if raw is not None else None), "CalculatePriorities")
    return (out, raw) if return_raw else out


def normalizePrio(prios) -> np.ndarray:
    p = np.ascontiguousarray(prios, dtype=np.float32).copy()
    check(lib().syzcov_normalize_prio(_ptr(p), p.shape[0]), "normalizePrio")
    return p


class ChoiceTable:
    """prio.go:196-200.  run[i] is None for disabled calls (nil in Go)."""

    def __init__(self, run, enabled_calls, enabled):
        self.run = run
        self.enabledCalls = enabled_calls
        self.enabled = enabled

    def choose_draws(self, calls, x) -> np.ndarray:
        """One device pass of Choose's search for given draws x[k] =
        r.Intn(run[call][-1]): the chosen call, -1 (rejected, Choose draws
        again) or -2 (uniform over enabledCalls).  syzcov_choose_batch."""
        calls = np.ascontiguousarray(np.asarray(calls, dtype=np.int32))
        x = np.ascontiguousarray(np.asarray(x, dtype=np.int64))
        if calls.size != x.size:
            raise ValueError("one draw per call")
        out = np.empty(max(calls.size, 1), dtype=np.int32)
        if calls.size:
            check(lib().syzcov_choose_batch(_ptr(self._run), _ptr(self._en), self._run.shape[0],
                                            _ptr(calls), _ptr(x), calls.size, _ptr(out)),
                  "ChooseBatch")
        return out[:calls.size]

    def choose_batch(self, rnd, calls) -> list:
        """Choose (prio.go:230-249) for many calls at once: every call's pick
        follows Choose exactly (draw, search, redraw on a disabled hit), but
        the draws are taken round by round over the batch, so for one seed
        the picks differ from a sequential loop of Choose calls."""
        calls = [int(c) for c in calls]
        res = [None] * len(calls)
        todo = list(range(len(calls)))
        while todo:
            xs = []
            for k in todo:
                run = self.run[calls[k]] if calls[k] >= 0 else None
                xs.append(rnd.randrange(int(run[-1])) if run is not None else 0)
            got = self.choose_draws([calls[k] for k in todo], xs)
            nxt = []
            for k, g in zip(todo, got):
                if g == -2:
                    res[k] = self.enabledCalls[rnd.randrange(len(self.enabledCalls))]
                elif g == -1:
                    nxt.append(k)
                else:
                    res[k] = int(g)
            todo = nxt
        return res

    def Choose(self, rnd, call: int) -> int:  # prio.go:230-249
        if call < 0:
            return self.enabledCalls[rnd.randrange(len(self.enabledCalls))]
        run = self.run[call]
        if run is None:
            return self.enabledCalls[rnd.randrange(len(self.enabledCalls))]
        while True:
            x = rnd.randrange(int(run[-1]))
            i = bisect.bisect_left(run, x)  # sort.SearchInts
            if not self.enabled[i]:
                continue
            return i


def BuildChoiceTable(prios, enabled=None) -> ChoiceTable:
    prios = np.ascontiguousarray(prios, dtype=np.float32)
    C_ = prios.shape[0]
    en = (np.ones(C_, dtype=np.uint8) if enabled is None
          else np.ascontiguousarray(np.asarray(enabled, dtype=np.uint8)))
    run = np.zeros((C_, C_), dtype=np.int64)
    check(lib().syzcov_build_choice_table(_ptr(prios), _ptr(en), C_, _ptr(run)),
          "BuildChoiceTable")
    rows = [run[i] if en[i] else None for i in range(C_)]
    ct = ChoiceTable(rows, [i for i in range(C_) if en[i]], en.astype(bool))
    ct._run, ct._en = run, en  # device layout for choose_draws
    return ct
