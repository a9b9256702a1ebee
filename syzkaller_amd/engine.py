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

from ._lib import check, lib

INT32_MAX = 0x7FFFFFFF
SYZCOV_ERR_WINDOW, SYZCOV_ERR_SEGLEN, SYZCOV_ERR_UNIVERSE = 1, 2, 4  # err_flag bits (syzcov.h)
KSHIFT_MAX = 7  # SYZCOV_KSHIFT_MAX: a universe PC's low bits fit the membership byte
RANGE_SHIFT = 20  # 2^20 PCs per LDS-resident range (128 KB covered bitmap)


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


class CorpusEngine:
    """Buffers sized for up to `n_max` inputs / `p_max` raw PCs (longest input
    `max_seg_len`) over the PC window [pc_lo, pc_lo + pc_span), at most 256
    ranges of 2^20 PCs.  `n_global` > n_max: a shard of a larger corpus
    (ranks, kept flags and the order span the whole corpus)."""

    PHASES = ("canon", "order", "minimize", "compact", "union", "merge")

    def __init__(self, n_max: int, p_max: int, max_seg_len: int, pc_lo: int, pc_span: int,
                 device="cuda", n_global: int | None = None, sort_variant: int = 0,
                 rec_cap: int = 0, canon_in_place: bool = False, universe=None):
        L = lib()
        dev = torch.device(device)
        self.dev, self.L = dev, L
        self.n_max, self.p_max, self.max_seg = n_max, p_max, max_seg_len
        # Key mode (keys.hip): with the PC universe registered, every phase works
        # on dense keys (pc >> kshift) - kbase instead of window offsets
        self.key_mode = universe is not None
        self.kshift, self.kbase = 0, pc_lo
        self.win_lo, self.win_span = pc_lo, pc_span  # Canonicalize's sort window
        if self.key_mode:
            (self.kshift, self.kbase, nkeys, self.pc_of_key, self.low_of_key, ulo,
             uhi) = universe_keymap(universe, dev)
            self.win_lo, self.win_span = ulo, uhi - ulo + 1  # the universe's extent
            pc_lo, pc_span = 0, nkeys  # minimize / union / maxCover window = the key range
        self.pc_lo, self.span = pc_lo, pc_span
        so = (0xFFFFFFFF >> self.kshift) - self.kbase  # key of the 0xFFFFFFFF sentinel
        self.sent_key = so if 0 <= so < pc_span else None
        self.sort_variant = sort_variant
        self.n_global = n_global or n_max
        self.rshift = RANGE_SHIFT
        self.nrange = (pc_span + (1 << RANGE_SHIFT) - 1) >> RANGE_SHIFT
        if self.nrange > 256:
            raise ValueError("PC window too wide for the range engine (> 256 ranges of 2^20)")
        nwords = (pc_span + 31) // 32
        self.nwords = nwords
        # canonical covers: their own buffer, or the raw CSR slots themselves
        # (canon_in_place: halves the corpus footprint; the raw lists are consumed)
        self.canon_in_place = canon_in_place
        if canon_in_place and max_seg_len > 16384:
            raise ValueError("in-place canonicalization needs max_seg_len <= 16384")
        self.canon = None if canon_in_place else _u32(p_max + 1, dev)
        self.new_len = _u32(n_max + 1, dev)
        # split points (columns per segment) and PCs per range, from canon
        self.split = (torch.empty(n_max * self.nrange, dtype=torch.int32, device=dev)
                      if self.nrange > 1 else None)
        self.range_tot = torch.zeros(self.nrange, dtype=torch.int64, device=dev)
        # covered set (one bit per window PC; ends up as the corpus union) and
        # the resident maxCover
        self.covered = torch.zeros((self.nrange << RANGE_SHIFT) // 32, dtype=torch.int32,
                                   device=dev)
        self.max_cover = torch.zeros(nwords, dtype=torch.int32, device=dev)
        self.tab = torch.empty(nwords, dtype=torch.int64, device=dev)
        # first-cover rank per window PC: INT32_MAX outside a step's records
        self.first = torch.full((pc_span,), INT32_MAX, dtype=torch.int32, device=dev)
        self.rec_cap = rec_cap or max(1 << 22, min(p_max, 1 << 26))
        self.rec = torch.empty(self.rec_cap, dtype=torch.int64, device=dev)
        self.rec_cnt = torch.zeros(1, dtype=torch.int64, device=dev)
        self.cand = torch.empty(n_max + 1, dtype=torch.uint8, device=dev)
        self.kept = torch.zeros(self.n_global + 1, dtype=torch.uint8, device=dev)
        self.lens64 = torch.empty(self.n_global + 1, dtype=torch.int64, device=dev)
        self.order = torch.empty(self.n_global + 1, dtype=torch.int32, device=dev)
        self.out_idx = torch.empty(self.n_global + 1, dtype=torch.int32, device=dev)
        self.union = _u32(min(pc_span, p_max) + 1, dev)
        self.scal = torch.zeros(16, dtype=torch.int64, device=dev)  # err, n_ids, n_kept, ...
        ws = max(L.syzcov_dev_canon_split_ws_size(n_max),
                 L.syzcov_dev_dict_ws_size(pc_span),
                 L.syzcov_dev_compact_ws_size(self.n_global),
                 L.syzcov_dev_sort_ws_size(self.n_global),
                 L.syzcov_dev_minimize_range_ws_size(self.n_global, pc_span, RANGE_SHIFT))
        self.ws = torch.empty(ws, dtype=torch.uint8, device=dev)
        self.ws_size = ws

    def alg_bytes(self, raw_pcs: int, canon_pcs: int) -> dict:
        """Algorithmic HBM bytes per launch of the streaming phases (DESIGN.md
        §4): canon reads every raw PC and writes every canonical PC once;
        Minimize pass 1 reads every canonical PC once."""
        return {"canon": 4 * raw_pcs + 4 * canon_pcs, "minimize": 4 * canon_pcs}

    # ---------------------------------------------------------------- phases
    def canonicalize(self, off: torch.Tensor, raw: torch.Tensor, n: int):
        """Wavefront canonicalize + per-range split points and range totals."""
        self.scal.zero_()
        self.range_tot.zero_()
        if self.canon_in_place:
            self.canon = raw
        if self.key_mode:
            check(self.L.syzcov_dev_canon_split_keys(
                _p(off), _p(raw), _p(self.canon), _p(self.new_len), n, self.max_seg, self.win_lo,
                self.win_span, self.kshift, self.kbase, self.span, _p(self.low_of_key),
                self.rshift, _p(self.split),
                _p(self.range_tot), _p(self.scal), _p(self.ws), self.ws_size, _stream()),
                "dev_canon_split_keys")
            return
        check(self.L.syzcov_dev_canon_split(_p(off), _p(raw), _p(self.canon), _p(self.new_len), n,
                                            self.max_seg, self.pc_lo, self.span, self.rshift,
                                            _p(self.split), _p(self.range_tot), _p(self.scal),
                                            _p(self.ws), self.ws_size, _stream()),
              "dev_canon_split")

    def sort_order(self, lens32: torch.Tensor, n: int):
        """Go sort.Sort order over canonical lengths (lens32: int32 [n])."""
        self.lens64[:n].copy_(lens32[:n])  # int32 -> int64 in the copy kernel
        check(self.L.syzcov_dev_sort_order(_p(self.lens64), n, self.sort_variant, _p(self.order),
                                           _p(self.ws), self.ws_size, _stream()), "dev_sort_order")

    def minimize_clear(self, n_items):
        """Zero minimize's inputs (covered, cand, kept)."""
        self.covered.zero_()
        self.cand[:n_items].zero_()
        self.kept.zero_()

    def minimize(self, off, order, ranks, n_items, do_pass2=True, cleared=False):
        """Range-partitioned first-cover Minimize; leaves the union in covered.
        cleared: minimize_clear() already ran on this stream."""
        if not cleared:
            self.minimize_clear(n_items)
        check(self.L.syzcov_dev_minimize_range(
            _p(off), _p(self.new_len), _p(self.canon), _p(self.split), _p(order), _p(ranks),
            n_items, self.pc_lo, self.span, self.rshift, _p(self.range_tot), _p(self.covered),
            _p(self.first), _p(self.rec), self.rec_cap, _p(self.rec_cnt), _p(self.cand),
            _p(self.kept), int(do_pass2), 0, 0, 0, _p(self.ws), _stream()), "dev_minimize_range")

    def minimize_pass2(self, off, order, ranks, n_items, tab=None, first_dense=None):
        """Pass 2 over the records (sharded: against the MIN-merged dense table)."""
        check(self.L.syzcov_dev_minimize_range_pass2(
            _p(off), _p(self.new_len), _p(self.canon), _p(self.split), _p(order), _p(ranks),
            n_items, self.pc_lo, self.span, self.rshift, _p(self.range_tot), _p(self.covered),
            _p(self.first), _p(self.rec), self.rec_cap, _p(self.rec_cnt), _p(self.cand), _p(tab),
            _p(first_dense), _p(self.kept), _p(self.ws), _stream()), "dev_minimize_range_pass2")

    def compact(self, n_ranks: int, ws=None):
        check(self.L.syzcov_dev_compact_kept(_p(self.kept), _p(self.order), n_ranks,
                                             _p(self.out_idx), _p(self.scal[2:3]),
                                             _p(self.ws if ws is None else ws), _stream()),
              "dev_compact_kept")

    def build_dict(self, ws=None):
        """Dense-id dictionary of the covered set; *n_ids -> scal[1]."""
        check(self.L.syzcov_dev_dict_build_bits(_p(self.covered), self.span, _p(self.tab),
                                                _p(self.scal[1:2]),
                                                _p(self.ws if ws is None else ws), _stream()),
              "dev_dict_build_bits")

    def union_list(self):
        # Union drops 0xFFFFFFFF (cover.go:97): in key mode, its key
        drop = 0xFFFFFFFF
        if self.key_mode:
            drop = self.sent_key if self.sent_key is not None else 0xFFFFFFFF
        check(self.L.syzcov_dev_dict_to_list_drop(_p(self.tab), self.span, self.pc_lo, drop,
                                                  _p(self.union), _p(self.scal[3:4]), _stream()),
              "dev_dict_to_list_drop")
        if self.key_mode:  # sorted keys -> sorted PCs (the key map is monotone)
            check(self.L.syzcov_dev_keys_to_pcs(_p(self.pc_of_key), self.span, _p(self.union),
                                                _p(self.union),
                                                _p(self.scal[3:4]), self.union.numel(), _stream()),
                  "dev_keys_to_pcs")

    def merge_max_cover(self):
        """maxCover |= union.  The union (Union fold) drops 0xFFFFFFFF
        (cover.go:97): if the window holds it, its covered bit goes first."""
        so = self.sent_key
        if so is not None:
            self.covered[so >> 5] &= ~(1 << (so & 31)) if (so & 31) != 31 else 0x7FFFFFFF
        check(self.L.syzcov_dev_bitmap_op(0, _p(self.max_cover), _p(self.covered), self.nwords,
                                          _p(self.scal[4:5]), _stream()), "dev_bitmap_op")

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
        # queued ahead of the sort, whose final read-back leaves the GPU idle
        # while the host issues the next launches
        self.minimize_clear(n)
        self.sort_order(self.new_len, n)
        mark_ev()
        self.minimize(off, self.order, None, n, cleared=True)
        mark_ev()
        self.compact(n)
        mark_ev()
        self.build_dict()
        self.union_list()
        mark_ev()
        self.merge_max_cover()
        mark_ev()
        return self.result() if sync else None

    def result(self) -> StepResult:
        sc = self.scal.cpu().tolist()
        if sc[0] & SYZCOV_ERR_WINDOW:
            raise RuntimeError("a PC fell outside the engine's PC window")
        if sc[0] & SYZCOV_ERR_SEGLEN:
            raise RuntimeError(f"an input is longer than max_seg_len={self.max_seg}")
        if sc[0] & SYZCOV_ERR_UNIVERSE:
            raise RuntimeError("a PC is not in the registered PC universe (key mode would alias "
                               "it with a universe PC; keys.hip)")
        if sc[0] & 0xFFFFFFFF:
            raise RuntimeError(f"engine error flags {sc[0] & 0xFFFFFFFF:#x}")
        n_ids, n_kept, n_union = (int(x) & 0xFFFFFFFF for x in sc[1:4])
        return StepResult(self.out_idx[:n_kept], n_kept, self.union[:n_union], n_union, n_ids,
                          int(sc[4]))

    def canonical_pcs(self, off: torch.Tensor, n: int) -> torch.Tensor:
        """The canonical covers as PCs, in the CSR slots of `off` (key mode:
        mapped back from the keys canon wrote there)."""
        if not self.key_mode:
            return self.canon
        out = torch.empty_like(self.canon)
        check(self.L.syzcov_dev_keys_to_pcs(_p(self.pc_of_key), self.span, _p(self.canon), _p(out),
                                            None, int(off[n].item()), _stream()),
              "dev_keys_to_pcs")
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

    def gemm_ops(self) -> int:
        """MFMA ops one counts launch executes (upper-triangle 128x128 tiles)."""
        nt = self.rows // 128
        if self.active_rows and self.max_len is not None:
            nt = max(1, -(-min(self.max_len, self.C) // 128))
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
                 log2_space: int = 22, uniform: bool = False, device="cuda"):
    """Generate a raw synthetic corpus directly in HBM (counter-based, so the
    CPU twin in oracle/ reproduces it bit-for-bit)."""
    L = lib()
    dev = torch.device(device)
    lens = torch.empty(n, dtype=torch.int32, device=dev)
    s = _stream()
    check(L.syzcov_dev_synth_lens(seed, first, n, mean, sigma, _p(lens), s), "synth_lens")
    off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens.to(torch.int64), 0, out=off[1:])
    total = int(off[-1].item())
    pcs = torch.empty(total + 1, dtype=torch.int32, device=dev)
    check(L.syzcov_dev_synth_pcs(seed, first, n, _p(off), log2_space, int(uniform), _p(pcs), s),
          "synth_pcs")
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


def synth_universe(log2_space: int = 22, seed: int = 0x5EED0002, device="cuda") -> torch.Tensor:
    """The synthetic generator's PC universe U[k], k < 2^log2_space (sorted;
    it depends on the corpus seed)."""
    u = torch.empty(1 << log2_space, dtype=torch.int32, device=device)
    check(lib().syzcov_dev_synth_universe(seed, log2_space, _p(u), _stream()), "synth_universe")
    return u


def synth_window(log2_space: int = 22):
    return SYNTH_PC_LO, 16 << log2_space
