"""Device-resident corpus engine: the manager-side hot path of syzkaller on
one MI355X (or one shard of a multi-GPU node).

One `step()` is the C2 workload of BASELINE.json on a raw corpus already in
HBM (CSR: offsets u64[n+1], raw KCOV PCs u32):

    canon     Canonicalize every input (cover.go:27-40): one wavefront per
              segment, LDS radix sort + unique, plus per-range split points
    order     Go sort.Sort(minInputArray) over canonical lengths (pdqsort restated)
    minimize  first-cover Minimize (cover.go:104-131): geometric rank chunks,
              LDS-resident covered bitmaps per 2^20-PC range, records of first
              covers, pass 2 over the records; leaves the corpus union in `covered`
    compact   kept inputs in processing order (the []int Minimize returns)
    union     sorted union list (the `Union(total, cov)` fold, manager.go:606-610)
    merge     resident maxCover |= union (manager.go:606-610 / fuzzer.go:470)

torch supplies device memory, the stream and torch.distributed (RCCL);
every computation is a libsyzcov HIP kernel launched on torch's current
stream (syzkaller_amd.dist.ShardedEngine adds the RCCL merges).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np
import torch

from ._lib import CORPUS_BUFS, CorpusCfg, CorpusInfo, CorpusRes, check, lib

INT32_MAX = 0x7FFFFFFF
SYZCOV_ERR_WINDOW, SYZCOV_ERR_SEGLEN, SYZCOV_ERR_UNIVERSE = 1, 2, 4  # err_flag bits (syzcov.h)
KSHIFT_MAX = 6  # SYZCOV_KSHIFT_MAX: a universe PC's low bits fit the membership byte


def _p(t: torch.Tensor | None):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _u32(n, dev):
    return torch.empty(n, dtype=torch.int32, device=dev)  # reinterpreted as uint32 by kernels


@dataclass
class StepResult:
    kept_idx: torch.Tensor      # int32 [n_kept] original input indices, processing order
    n_kept: int
    union: torch.Tensor         # int32-viewed uint32 [n_union] sorted PCs
    n_union: int
    n_ids: int                  # distinct PCs in the corpus (incl. a 0xFFFFFFFF sentinel)
    max_cover: int              # |maxCover| after the merge
    fallback: bool = False      # a PC outside the key space: recomputed in window mode
    err_flags: int = 0          # SYZCOV_ERR_* bits the step saw (with fallback: why)
    max_cover_missed: int = 0   # fallback: union PCs maxCover cannot represent (not taken)


_DT = {"CANON": torch.int32, "NEW_LEN": torch.int32, "SPLIT": torch.int32,
       "RANGE_TOT": torch.int64, "COVERED": torch.int32, "MAX_COVER": torch.int32,
       "TAB": torch.int64, "FIRST": torch.int32, "REC": torch.int64, "CAND": torch.uint8,
       "KEPT": torch.uint8, "LENS": torch.int64, "ORDER": torch.int32, "KEPT_IDX": torch.int32,
       "UNION": torch.int32, "SCAL": torch.int64, "PC_OF_KEY": torch.int32,
       "LOW_OF_KEY": torch.uint8, "GLENS": torch.int32, "SEL": torch.uint8,
       "IOTA": torch.int32, "ITEMS": torch.int32, "RANKS": torch.int32,
       "FIRST_DENSE": torch.int32, "WS": torch.uint8, "WS2": torch.uint8}


class CorpusEngine:
    """The resident corpus engine of libsyzcov (corpus.hip, include/syzcov.h
    "resident corpus engine") behind one handle: the device memory is one
    torch allocation laid out by the library, every phase a C-ABI call on
    torch's current stream, so bench.py measures exactly what a Go host would
    call over cgo.  Sized for up to `n_max` inputs / `p_max` raw PCs (longest
    input `max_seg_len`) over the PC window [pc_lo, pc_lo + pc_span), or over
    the dense keys of a registered PC `universe` (key mode).  `n_global` >
    n_max: shard `rank` of a larger corpus (dist.ShardedEngine)."""

    PHASES = ("canon", "order", "minimize", "finish")

    def __init__(self, n_max: int, p_max: int, max_seg_len: int, pc_lo: int, pc_span: int,
                 device="cuda", n_global: int | None = None, rank: int = 0, rec_cap: int = 0,
                 canon_in_place: bool = False, universe=None, order_by: int = 0,
                 canon_layout: int = 0):
        L = lib()
        dev = torch.device(device)
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.dev, self.L, self.h = dev, L, None
        self.n_max, self.p_max, self.max_seg = n_max, p_max, max_seg_len
        self.n_global = n_global or n_max
        self.canon_in_place = canon_in_place
        self._univ = None
        if universe is not None:  # host copy (read by create only)
            if isinstance(universe, torch.Tensor):
                universe = universe.cpu().numpy().view(np.uint32)
            self._univ = np.ascontiguousarray(universe, dtype=np.uint32)
        cfg = CorpusCfg(n_max=n_max, n_global=n_global or 0, rank=rank, p_max=p_max,
                        max_seg_len=max_seg_len, pc_lo=pc_lo, pc_span=pc_span,
                        universe=None if self._univ is None else self._univ.ctypes.data,
                        universe_n=0 if self._univ is None else self._univ.size,
                        canon_in_place=int(canon_in_place), order_by=order_by, rec_cap=rec_cap,
                        canon_layout=canon_layout)
        size = check(L.syzcov_corpus_mem_size(C.byref(cfg)), "corpus_mem_size")
        with torch.cuda.device(dev):
            self.mem = torch.empty(size, dtype=torch.uint8, device=dev)
            h = C.c_uint64(0)
            check(L.syzcov_corpus_create(C.byref(cfg), _p(self.mem), size, C.byref(h)),
                  "corpus_create")
        self.h = h.value
        self._univ = None
        info = CorpusInfo()
        check(L.syzcov_corpus_info(self.h, C.byref(info)), "corpus_info")
        self.key_mode = bool(info.key_mode)
        self.kshift, self.kbase = info.kshift, info.kbase
        self.pc_lo, self.span = info.pc_lo, info.span
        self.win_lo, self.win_span = info.win_lo, info.win_span
        self.nrange, self.nwords = info.nrange, info.nwords
        self.rec_cap = info.rec_cap
        self.canon_align_k = info.canon_align_k  # 0: CANON in CSR slots
        self.sent_key = None if info.sent_key == 0xFFFFFFFF else info.sent_key
        for name in CORPUS_BUFS:
            setattr(self, name.lower(), self._view(name))
        self.canon_buf = self.canon           # the CANON buffer (None when in place)
        self.canon = None                     # the step's canonical lists
        self.union = self.union               # noqa: PLW0127 (named for callers)
        self.scal = self.scal
        self.rec_cnt = self.scal[7:8]
        self.out_idx = self.kept_idx

    def _view(self, name: str):
        off, nb = C.c_uint64(0), C.c_uint64(0)
        check(self.L.syzcov_corpus_buffer(self.h, CORPUS_BUFS.index(name), C.byref(off),
                                          C.byref(nb)), "corpus_buffer")
        if nb.value == 0:
            return None
        return self.mem[off.value:off.value + nb.value].view(_DT[name])

    def close(self):
        if self.h:
            self.L.syzcov_corpus_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass

    def alg_bytes(self, raw_pcs: int, canon_pcs: int) -> dict:
        """Algorithmic HBM bytes per launch of the streaming phases (DESIGN.md
        §4): canon reads every raw PC and writes every canonical PC once;
        Minimize pass 1 reads every canonical PC once."""
        return {"canon": 4 * raw_pcs + 4 * canon_pcs, "minimize": 4 * canon_pcs}

    # ---------------------------------------------------------------- phases
    def canonicalize(self, off: torch.Tensor, raw: torch.Tensor, n: int):
        """Wavefront canonicalize + per-range split points and range totals
        (key mode: key words, common.h)."""
        check(self.L.syzcov_corpus_canon(self.h, _p(off), _p(raw), n, _stream()), "corpus_canon")
        self.canon = raw if self.canon_in_place else self.canon_buf
        self._canon_step = (off.data_ptr(), n)  # the offsets/n the handle holds

    def sort_order(self, lens32: torch.Tensor | None = None, n: int | None = None):
        """Go sort.Sort order over int32 lengths (None: this step's own);
        clears Minimize's inputs."""
        own = lens32 is None or lens32.data_ptr() == self.new_len.data_ptr()
        check(self.L.syzcov_corpus_order(self.h, None if own else _p(lens32), n, _stream()),
              "corpus_order")

    def minimize(self, do_pass2: bool = True):
        """First-cover Minimize over this step's items (sharded: this shard's,
        with global ranks; pass 2 after the exchange)."""
        check(self.L.syzcov_corpus_minimize(self.h, int(do_pass2), _stream()), "corpus_minimize")

    def finish(self):
        """Kept list, sorted union, maxCover |= union."""
        check(self.L.syzcov_corpus_finish(self.h, _stream()), "corpus_finish")

    # ------------------------------------------------------------------ step
    def step(self, off: torch.Tensor, raw: torch.Tensor, n: int, sync: bool = True, ev=None):
        k = [0]

        def mark_ev():
            if ev is not None:
                ev[k[0]].record()
            k[0] += 1
        mark_ev()
        self.canonicalize(off, raw, n)
        mark_ev()
        self.sort_order(None, n)
        mark_ev()
        self.minimize(True)
        mark_ev()
        self.finish()
        mark_ev()
        return self.result() if sync else None

    def result(self) -> StepResult:
        r = CorpusRes()
        rc = self.L.syzcov_corpus_result(self.h, C.byref(r), _stream())
        if rc < 0:
            msg = self.L.syzcov_last_error().decode(errors="replace")
            msg += f" [err_flags {r.err_flags:#x}]"
            if r.err_flags & SYZCOV_ERR_UNIVERSE:
                msg += (" (key mode would alias it with a universe PC; keys.hip; the window-mode "
                        "recompute needs the raw PCs: canon in place or sharded cannot)")
            raise RuntimeError(msg)
        union = self.union[:r.n_union]
        if r.n_union and r.union_pcs != self.union.data_ptr():
            # a window-mode recompute whose union outgrew the key space's buffer
            # (PCs outside the universe): the handle's side buffer, copied out
            union = torch.empty(-(-r.n_union // 4) * 4, dtype=torch.int32, device=self.dev)
            check(self.L.syzcov_dev_stream_copy(C.c_void_p(r.union_pcs), _p(union), union.numel() * 4,
                                                _stream()), "dev_stream_copy")
            union = union[:r.n_union]
        return StepResult(self.kept_idx[:r.n_kept], r.n_kept, union, r.n_union,
                          r.n_ids, r.max_cover, bool(r.fallback), r.err_flags,
                          r.max_cover_missed)

    def canonical_pcs(self, off: torch.Tensor, n: int) -> torch.Tensor:
        """The canonical covers as PCs, in the CSR slots of `off` (key mode:
        decoded from the key words canon wrote there)."""
        lists = self.canon
        if self.canon_align_k:  # line-aligned layout: back into the CSR slots
            # syzcov_corpus_canonical unpacks by the handle's own offsets and n
            # (the last canon step's): another off or n would size the output
            # below what the kernel writes
            if getattr(self, "_canon_step", None) != (off.data_ptr(), n):
                raise ValueError("canonical_pcs: off / n differ from the last canonicalize step")
            lists = torch.zeros(int(off[n].item()) + 1, dtype=torch.int32, device=self.dev)
            check(self.L.syzcov_corpus_canonical(self.h, _p(lists), _stream()),
                  "corpus_canonical")
        if not self.key_mode:
            return lists
        out = torch.empty_like(lists)
        check(self.L.syzcov_dev_words_to_pcs(_p(lists), int(off[n].item()), self.kshift,
                                             self.kbase, _p(out), _stream()), "dev_words_to_pcs")
        return out


class PrioEngine:
    """Device-resident prog.CalculatePriorities (prio.go:29-38) for a corpus of
    `nprog` programs given by their lengths (positional key mode, exactly the
    reference's calcDynamicPrio) over the C = 1170 calls of sys/*.txt."""

    PHASES = ("static", "build", "gemm", "finish")

    def __init__(self, nprog: int, device="cuda", table=None, active_rows: bool = True):
        from . import prio as P
        L = lib()
        self.L, self.dev = L, torch.device(device)
        id_off, calls, ws, call_off, cids, cws, C_ = P.usage_csr(table)
        def dev_copy(a):  # unsigned arrays travel as same-width signed views
            return torch.from_numpy(np.ascontiguousarray(a)).to(self.dev)
        self.id_off = dev_copy(id_off.view(np.int32))
        self.calls = dev_copy(calls.view(np.int16))
        self.ws = dev_copy(ws)
        self.call_off = dev_copy(call_off.view(np.int32))
        self.cids = dev_copy(cids.view(np.int32))
        self.cws = dev_copy(cws)
        self.C = C_
        self.nprog = nprog
        self.rows = L.syzcov_dev_prio_rows(C_)
        self.ldp = L.syzcov_dev_prio_ldp(nprog)
        self.at = (None if active_rows else
                   torch.empty(self.rows * self.ldp, dtype=torch.int8, device=self.dev))
        self.counts = torch.empty(self.rows * self.rows, dtype=torch.int32, device=self.dev)
        self.static = torch.empty(C_ * C_, dtype=torch.float32, device=self.dev)
        self.out = torch.empty(C_ * C_, dtype=torch.float32, device=self.dev)
        self.err = torch.zeros(4, dtype=torch.int32, device=self.dev)
        # positional counts over the active keys only (prio.hip): the AT of
        # roundup(max len, 128) keys lives in the workspace instead of self.at
        self.active_rows = active_rows
        self.max_len = None
        self.pos_ws = None
        # dense mode: 256 x 256 tiles with a partial-tile workspace (prio.hip
        # prio_gemm256_kernel); 0 bytes: 128 x 128 tiles with atomics
        self.tile = 128
        self.dense_ws = None
        if not active_rows:
            wsz = L.syzcov_dev_prio_counts_ws_size(nprog, C_)
            if wsz:
                self.dense_ws = torch.empty(wsz, dtype=torch.uint8, device=self.dev)
                self.tile = 256

    def gemm_ops(self) -> int:
        """MFMA ops one counts launch executes (upper-triangle 128x128 tiles)."""
        nt = self.rows // self.tile
        if not self.active_rows:
            return nt * (nt + 1) // 2 * self.tile * self.tile * 2 * self.ldp
        if self.active_rows and self.max_len is not None:
            # the active block holds the ones row too: roundup(min(max_len, C) + 1, 128)
            # rows, as pos_plan sizes it (prio.hip)
            nt = max(1, -(-(min(self.max_len, self.C) + 1) // 128))
        return nt * (nt + 1) // 2 * 128 * 128 * 2 * self.ldp

    def step(self, lens: torch.Tensor, ev=None, reduce=None):
        """`reduce(counts)` (sharded by program: dist.merge_counts) runs
        between the contraction and the normalisation."""
        L, s = self.L, _stream()

        def mark_ev(i):
            if ev is not None:
                ev[i].record()
        mark_ev(0)
        check(L.syzcov_dev_static_prio(_p(self.id_off), _p(self.calls), _p(self.ws),
                                       _p(self.call_off), _p(self.cids), _p(self.cws), self.C,
                                       _p(self.static), s), "dev_static_prio")
        mark_ev(1)
        if self.active_rows:
            # max len sizes the active key block (one host read of a device max)
            ml = int(lens[:self.nprog].max().item()) if self.nprog else 0
            if ml > self.C:
                raise ValueError(f"program of {ml} calls > {self.C} (prio.go:148 would panic)")
            wsz = L.syzcov_dev_prio_pos_ws_size(self.nprog, self.C, ml)
            if self.pos_ws is None or self.pos_ws.numel() < wsz:
                self.pos_ws = torch.empty(wsz, dtype=torch.uint8, device=self.dev)
            self.max_len = ml
            self.counts.zero_()
            mark_ev(2)
            check(L.syzcov_dev_prio_counts_pos(_p(lens), self.nprog, self.C, ml, _p(self.counts),
                                               _p(self.pos_ws), self.pos_ws.numel(), s),
                  "dev_prio_counts_pos")
        else:
            check(L.syzcov_dev_prio_build_at(0, _p(lens), None, None, self.nprog, self.C,
                                             _p(self.at), self.ldp, _p(self.err), s),
                  "dev_prio_build_at")
            self.counts.zero_()
            mark_ev(2)
            if self.dense_ws is not None:
                check(L.syzcov_dev_prio_counts_ws(_p(self.at), self.ldp, self.nprog, self.C,
                                                  _p(self.counts), _p(self.dense_ws),
                                                  self.dense_ws.numel(), s), "dev_prio_counts_ws")
            else:
                check(L.syzcov_dev_prio_counts(_p(self.at), self.ldp, self.nprog, self.C,
                                               _p(self.counts), s), "dev_prio_counts")
        if reduce is not None:
            reduce(self.counts)
        mark_ev(3)
        check(L.syzcov_dev_prio_finish(_p(self.counts), self.C, _p(self.static), _p(self.out),
                                       None, s), "dev_prio_finish")
        mark_ev(4)
        return self.out


def synth_corpus(n: int, seed: int, first: int = 0, mean: int = 2048, sigma: int = 512,
                 log2_space: int = 22, uniform: bool = False, device="cuda", x86: bool = False):
    """Generate a raw synthetic corpus directly in HBM (counter-based, so the
    CPU twin in oracle/ reproduces it bit-for-bit).  x86: PCs of the x86-like
    universe (neighbours 5..14 bytes apart, kshift 2), else one per 16-byte
    slot."""
    L = lib()
    dev = torch.device(device)
    lens = torch.empty(n, dtype=torch.int32, device=dev)
    s = _stream()
    check(L.syzcov_dev_synth_lens(seed, first, n, mean, sigma, _p(lens), s), "synth_lens")
    off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens.to(torch.int64), 0, out=off[1:])
    total = int(off[-1].item())
    pcs = torch.empty(total + 1, dtype=torch.int32, device=dev)
    check(L.syzcov_dev_synth_pcs(seed, first, n, _p(off), log2_space,
                                 int(uniform) | (2 if x86 else 0), _p(pcs), s), "synth_pcs")
    return off, pcs, lens, total


def synth_records(nrec: int, seed: int, first: int, ncalls: int, mean: int = 2048,
                  sigma: int = 512, log2_space: int = 22, device="cuda"):
    """Config C5's call records first .. first + nrec - 1 in HBM: the
    canonical cover of synthetic input `first + k` (Canonicalize on the GPU,
    then compacted into a record CSR) and its CallID.  Returns (callid i32,
    rec_off i64[nrec + 1], pcs i32-viewed u32, number of PCs); the CPU twin is
    oracle/newcov_full.c."""
    L = lib()
    dev = torch.device(device)
    off, raw, lens, total = synth_corpus(nrec, seed, first=first, mean=mean, sigma=sigma,
                                         log2_space=log2_space, device=dev)
    lo, span = synth_window(log2_space)
    new_len = torch.empty(nrec + 1, dtype=torch.int32, device=dev)
    err = torch.zeros(4, dtype=torch.int32, device=dev)
    wsz = L.syzcov_dev_canon_split_ws_size(nrec)
    ws = torch.empty(wsz, dtype=torch.uint8, device=dev)
    s = _stream()
    check(L.syzcov_dev_canon_split(_p(off), _p(raw), _p(raw), _p(new_len), nrec,
                                   int(lens.max().item()), lo, span, 20, None, None, _p(err),
                                   _p(ws), wsz, s), "canon_split")
    if int(err[0].item()):
        raise RuntimeError(f"canonicalize flags {int(err[0].item()):#x}")
    nl = new_len[:nrec].to(torch.int64)
    roff = torch.zeros(nrec + 1, dtype=torch.int64, device=dev)
    torch.cumsum(nl, 0, out=roff[1:])
    npc = int(roff[-1].item())
    seg = torch.repeat_interleave(torch.arange(nrec, device=dev), nl)
    src = off[:-1][seg] + (torch.arange(npc, device=dev) - roff[:-1][seg])
    pcs = raw[src].contiguous()
    cid = torch.empty(nrec, dtype=torch.int32, device=dev)
    check(L.syzcov_dev_synth_callids(seed, first, nrec, ncalls, _p(cid), s), "synth_callids")
    return cid, roff, pcs, npc


SYNTH_PC_LO = 0x81000000


def universe_shift(u: np.ndarray) -> int:
    """Largest kshift <= KSHIFT_MAX with no two neighbouring (sorted, unique)
    universe PCs sharing pc >> kshift: (a >> s) != (b >> s) iff a ^ b has a
    bit >= s, so the bound is the min over neighbours of the highest differing
    bit."""
    u = np.asarray(u, dtype=np.uint32)
    if u.size < 2:
        return 0
    if not np.all(u[1:] > u[:-1]):
        raise ValueError("the PC universe must be sorted and unique")
    return min(KSHIFT_MAX, int((u[1:] ^ u[:-1]).min()).bit_length() - 1)


def universe_keymap(universe, dev):
    """(kshift, kbase, nkeys, pc_of_key, low_of_key, lowest PC, highest PC) of a
    registered PC universe: the sorted unique u32 PCs KCOV can report, i.e. the
    return addresses of the __sanitizer_cov_trace_pc calls (the call sites
    syz-manager/cover.go:274-306 lists, plus the call's length; cover.go:82
    subtracts the 1 back).  low_of_key is the membership table every key-mode
    kernel checks (keys.hip)."""
    if isinstance(universe, torch.Tensor):
        uh = universe.cpu().numpy().view(np.uint32)
        ud = universe.to(dev)
    else:
        uh = np.ascontiguousarray(universe, dtype=np.uint32)
        ud = torch.from_numpy(uh.view(np.int32)).to(dev)
    ks = universe_shift(uh)
    kbase = int(uh[0]) >> ks
    nkeys = (int(uh[-1]) >> ks) - kbase + 1
    pc_of_key = torch.empty(nkeys, dtype=torch.int32, device=dev)
    low_of_key = torch.empty(nkeys, dtype=torch.uint8, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    L = lib()
    check(L.syzcov_dev_universe_keymap(_p(ud), uh.size, ks, kbase, nkeys, _p(pc_of_key),
                                       _p(low_of_key), _p(err), _stream()), "dev_universe_keymap")
    if int(err.item()):
        raise ValueError("universe keymap failed (unsorted or colliding universe)")
    return ks, kbase, nkeys, pc_of_key, low_of_key, int(uh[0]), int(uh[-1])


def synth_universe(log2_space: int = 22, seed: int = 0x5EED0002, device="cuda",
                   x86: bool = False) -> torch.Tensor:
    """The synthetic generator's PC universe U[k], k < 2^log2_space (sorted;
    it depends on the corpus seed; x86: the 5..14-byte-gap universe)."""
    u = torch.empty(1 << log2_space, dtype=torch.int32, device=device)
    check(lib().syzcov_dev_synth_universe_mode(seed, log2_space, 2 if x86 else 0, _p(u),
                                               _stream()), "synth_universe")
    return u


def synth_window(log2_space: int = 22, x86: bool = False):
    return SYNTH_PC_LO, (8 if x86 else 16) << log2_space
