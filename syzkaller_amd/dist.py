"""The corpus engine sharded by input over the GPUs of one node: each rank
holds a contiguous slice of a global corpus of fixed size (C3's 10M inputs
at every N, so the bench's curve is strong scaling).

One process per GPU, torch.distributed over RCCL ("nccl" backend on ROCm).
The only exchanges are the reductions the first-cover formulation needs
(SURVEY §8e):

    canonical lens all-gather              -> the Go sort.Sort order's rounds
    order          int32 MAX all-reduce    -> each rank finished its part of it
    first[]        int32 MIN all-reduce    -> global first-cover rank per key
                                              (key mode: the union = keys with one)
    covered bitmap uint8 MAX all-reduce    -> key mode: the union (north_star's shard
                                              bitmap merge; one byte per key)
    covered bitmap all-gather + OR          -> window mode: the union = identical
                                              dictionary, first[] MIN over its ids
    kept flags     uint8 MAX all-reduce    -> identical kept list on every rank

The collective glue below is device-agnostic (it runs under gloo on CPU
tensors in tests/test_dist_gloo.py); the per-shard compute is libsyzcov's
corpus handle (corpus.hip) via engine.CorpusEngine.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .engine import CorpusEngine, _p, _stream
from ._lib import check


# ------------------------------------------------------------------ glue
def _staged(t: torch.Tensor):
    """gloo moves host tensors only: device tensors go through a host copy
    (multi-rank tests on one GPU); with RCCL the tensor is used in place."""
    return t.is_cuda and dist.get_backend() == "gloo"


def _all_reduce(t: torch.Tensor, op) -> None:
    if _staged(t):
        h = t.cpu()
        dist.all_reduce(h, op=op)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op)


def _all_gather(out: torch.Tensor, t: torch.Tensor) -> None:
    if _staged(t):
        h = out.cpu()
        dist.all_gather_into_tensor(h, t.cpu())
        out.copy_(h)
    else:
        dist.all_gather_into_tensor(out, t)


def merge_first(first: torch.Tensor) -> None:
    """Global first-cover rank per dense PC id."""
    _all_reduce(first, dist.ReduceOp.MIN)


def merge_order(order: torch.Tensor) -> None:
    """The Go order split over the ranks (syzcov_corpus_order_part): each
    rank holds its segments' positions and -1 in the others'; every position
    is final on some rank with the same value wherever it is, so MAX."""
    _all_reduce(order, dist.ReduceOp.MAX)


def merge_counts(counts: torch.Tensor) -> None:
    """CalculatePriorities sharded by program: each rank's
    int32 co-occurrence counts AᵀA of its own programs; the global counts are
    their SUM (exact: the contraction is linear in the programs)."""
    _all_reduce(counts, dist.ReduceOp.SUM)


def merge_kept(kept: torch.Tensor) -> None:
    """kept[] is indexed by global rank; each rank set only its own items."""
    _all_reduce(kept, dist.ReduceOp.MAX)


def merge_covered(covered: torch.Tensor, world: int, or_into) -> None:
    """Union of the shards' covered bitmaps (u32 words).  RCCL has no bitwise
    OR, so the bitmaps are all-gathered (world x |bitmap|, 8 MB each at C3)
    and OR-ed locally with `or_into(dst, src)` (the HIP bitmap kernel on GPU,
    torch.bitwise_or under gloo)."""
    if world == 1:
        return
    out = torch.empty(world * covered.numel(), dtype=covered.dtype, device=covered.device)
    _all_gather(out, covered.contiguous())
    parts = out.view(world, -1)
    covered.copy_(parts[0])
    for r in range(1, world):
        or_into(covered, parts[r])


def merge_bitmap_u8(covered: torch.Tensor, u8: torch.Tensor, to_bytes, to_bits) -> None:
    """Union of the shards' covered bitmaps (u32 words) as north_star names it:
    each bitmap as a byte map (one byte per key, 0 or 1: `to_bytes(words,
    u8)`), a uint8 MAX all-reduce over RCCL, and back into `covered`
    (`to_bits(u8, words)`).  The HIP converters on the GPU
    (syzcov_dev_bits_to_bytes / _bytes_to_bits), numpy ones under gloo."""
    to_bytes(covered, u8)
    _all_reduce(u8, dist.ReduceOp.MAX)
    to_bits(u8, covered)


def gather_lens(local_lens: torch.Tensor, world: int) -> torch.Tensor:
    """Canonical lengths of every shard, in global input order."""
    out = torch.empty(local_lens.numel() * world, dtype=local_lens.dtype,
                      device=local_lens.device)
    _all_gather(out, local_lens.contiguous())
    return out


def local_items(order: torch.Tensor, rank: int, n_local: int):
    """Work items of this shard in global processing order: (local input
    index, global rank) for every global rank whose input lives here.  (Host
    reference form; the device engine uses ShardedEngine._local_items, which
    has no host sync.)"""
    base = rank * n_local
    sel = (order >= base) & (order < base + n_local)
    ranks = torch.nonzero(sel, as_tuple=False).flatten().to(torch.int32)
    return (order[ranks.long()] - base).to(torch.int32), ranks


# ---------------------------------------------------------------- engine
class ShardedEngine(CorpusEngine):
    """Rank `rank` of `world`: n local inputs of a global corpus of n*world
    (global input i lives on rank i // n).  The per-shard compute is the
    library's corpus handle (corpus.hip); the collectives run between its
    phase calls, on the buffers of its layout (include/syzcov.h)."""

    # "exchange": the MIN merge of first ranks (key mode: the first-cover array
    # itself; window mode: over the dictionary of the OR-merged covered sets),
    # pass 2 and the MAX merge of kept flags
    PHASES = ("canon", "order", "minimize", "exchange", "finish")

    def __init__(self, n: int, p_max: int, max_seg_len: int, pc_lo: int, pc_span: int,
                 rank: int, world: int, device="cuda", universe=None, canon_in_place=False,
                 split_order: bool = True, canon_layout: int = 0, bitmap_union: bool = True):
        super().__init__(n, p_max, max_seg_len, pc_lo, pc_span, device=device,
                         n_global=n * world, rank=rank, universe=universe,
                         canon_in_place=canon_in_place, canon_layout=canon_layout)
        self.rank, self.world, self.n_local = rank, world, n
        # the ranks split the Go order's late rounds and finisher (each finishes
        # the segments starting in its block), merged by an int32 MAX all-reduce
        self.split_order = split_order and world > 1
        # key mode: the union is the uint8 MAX all-reduce of the shards' covered
        # byte maps (north_star); False derives it from the MIN-merged first
        # ranks alone (pass 2's first_to_bits), 4 MB less per rank at 2^22 keys
        self.bitmap_union = bitmap_union and self.key_mode
        self.cov_u8 = (torch.empty(self.covered.numel() * 32, dtype=torch.uint8, device=self.dev)
                       if self.bitmap_union else None)

    def _to_bytes(self, words, u8):
        check(self.L.syzcov_dev_bits_to_bytes(_p(words), words.numel(), _p(u8), _stream()),
              "dev_bits_to_bytes")

    def _to_bits(self, u8, words):
        check(self.L.syzcov_dev_bytes_to_bits(_p(u8), words.numel(), _p(words), _stream()),
              "dev_bytes_to_bits")

    def _or_into(self, dst, src):
        check(self.L.syzcov_dev_bitmap_op(0, _p(dst), _p(src), dst.numel(), None, _stream()),
              "dev_bitmap_op")

    def step(self, off, raw, n, sync: bool = True, ev=None):
        """One rank's step.  Exchanges: canonical lengths (all-gather), first
        ranks (int32 MIN; window mode after an all-gather + OR of the covered
        bitmaps and over their dictionary), kept flags by global rank (u8 MAX)."""
        k = [0]

        def mark_ev():
            if ev is not None:
                ev[k[0]].record()
            k[0] += 1
        assert n == self.n_local
        N = n * self.world
        L, h, s = self.L, self.h, _stream()
        mark_ev()
        self.canonicalize(off, raw, n)
        mark_ev()
        _all_gather(self.glens[:N], self.new_len[:n].contiguous())  # RCCL all-gather
        if self.split_order:
            check(L.syzcov_corpus_order_part(h, _p(self.glens), N, s), "corpus_order_part")
            merge_order(self.order[:N])                             # RCCL int32 MAX
        else:
            self.sort_order(self.glens, N)                          # identical on every rank
        mark_ev()
        self.minimize(do_pass2=False)
        mark_ev()
        if self.key_mode:
            # dense key space: the first-cover array itself is the exchange
            # (nkeys int32, 16 MB at 2^22 keys; no dictionary, no host sync)
            merge_first(self.first[:self.span])                      # RCCL int32 MIN
            if self.bitmap_union:  # the shard bitmaps as byte maps, RCCL uint8 MAX
                self._to_bytes(self.covered, self.cov_u8)
                _all_reduce(self.cov_u8, dist.ReduceOp.MAX)
        else:
            merge_covered(self.covered[:self.nwords], self.world, self._or_into)
            n_ids = check(L.syzcov_corpus_dense_first(h, s), "corpus_dense_first")
            merge_first(self.first_dense[:n_ids])                   # RCCL int32 MIN
        check(L.syzcov_corpus_pass2(h, s), "corpus_pass2")          # kept against the global first
        if self.bitmap_union:
            # the union finish publishes: the MAX-merged shard bitmaps (the same
            # set pass 2 rebuilt from the global first ranks)
            self._to_bits(self.cov_u8, self.covered)
        # RCCL uint8 MAX of kept flags by global rank; kept[N..N+3] carry the
        # shard's error flags, one byte per flag bit (pass 2 wrote them, finish
        # ORs the merged bytes back: a shard that saw a non-universe PC fed its
        # aliased first covers into the MIN merge, so every rank fails the step
        # with the same flags)
        merge_kept(self.kept[:N + 4])
        mark_ev()
        self.finish()
        mark_ev()
        return self.result() if sync else None
