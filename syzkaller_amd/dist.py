"""The corpus engine sharded by input over the GPUs of one node (weak
scaling: each rank holds a contiguous slice of the global corpus).

One process per GPU, torch.distributed over RCCL ("nccl" backend on ROCm).
The only exchanges are the reductions the first-cover formulation needs
(SURVEY §8e):

    canonical lens all-gather              -> identical Go sort.Sort order
    covered bitmap all-gather + OR          -> the corpus union = identical dictionary
    first[]        int32 MIN all-reduce    -> global first-cover rank per dense PC id
    kept flags     uint8 MAX all-reduce    -> identical kept list on every rank

The collective glue below is device-agnostic (it runs under gloo on CPU
tensors in tests/test_dist_gloo.py); the per-shard compute is libsyzcov's
HIP kernels via engine.CorpusEngine.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .engine import INT32_MAX, CorpusEngine, _p, _stream
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
    (global input i lives on rank i // n)."""

    def __init__(self, n: int, p_max: int, max_seg_len: int, pc_lo: int, pc_span: int,
                 rank: int, world: int, device="cuda", sort_variant: int = 0, universe=None):
        super().__init__(n, p_max, max_seg_len, pc_lo, pc_span, device=device,
                         n_global=n * world, sort_variant=sort_variant, universe=universe)
        self.rank, self.world, self.n_local = rank, world, n
        self.glens = torch.empty(n * world, dtype=torch.int32, device=self.dev)
        # the merged union can be larger than this shard's PC count
        gcap = min(pc_span, p_max * world) + 1
        self.union = torch.empty(gcap, dtype=torch.int32, device=self.dev)
        # compact first-cover exchange: one int32 per PC of the merged union
        self.first_dense = torch.empty(gcap, dtype=torch.int32, device=self.dev)
        # dictionary/compaction scratch apart from ws, which carries minimize's
        # rank-ordered descriptors from pass 1 to pass 2
        self.ws2 = torch.empty(max(self.L.syzcov_dev_dict_ws_size(pc_span),
                                   self.L.syzcov_dev_compact_ws_size(n * world)),
                               dtype=torch.uint8, device=self.dev)
        # local work items: global ranks of this shard's inputs and the inputs
        # themselves, by two ordered compactions (exactly n of them: the order
        # is a permutation of the N global inputs)
        self.iota = torch.arange(n * world, dtype=torch.int32, device=self.dev)
        self.sel = torch.empty(n * world, dtype=torch.uint8, device=self.dev)
        self.ranks_l = torch.empty(n + 1, dtype=torch.int32, device=self.dev)
        self.items_l = torch.empty(n + 1, dtype=torch.int32, device=self.dev)
        self.cnt_l = torch.zeros(2, dtype=torch.int32, device=self.dev)

    # "exchange": the covered OR, the dictionary, the first-rank MIN merge,
    # pass 2 and the kept merge (the only phase with collectives besides order)
    PHASES = ("canon", "order", "minimize", "exchange", "compact", "union", "merge")

    def _local_items(self, N: int):
        """(local input index, global rank) of this shard's items in global
        processing order, on the device with no host sync."""
        n, base, s = self.n_local, self.rank * self.n_local, _stream()
        order = self.order[:N]
        torch.logical_and(order >= base, order < base + n, out=self.sel.view(torch.bool))
        check(self.L.syzcov_dev_compact_kept(_p(self.sel), _p(self.iota), N, _p(self.ranks_l),
                                             _p(self.cnt_l[0:1]), _p(self.ws2), s),
              "dev_compact_kept")
        check(self.L.syzcov_dev_compact_kept(_p(self.sel), _p(order), N, _p(self.items_l),
                                             _p(self.cnt_l[1:2]), _p(self.ws2), s),
              "dev_compact_kept")
        self.items_l[:n].sub_(base)
        return self.items_l[:n], self.ranks_l[:n]

    def _or_into(self, dst, src):
        check(self.L.syzcov_dev_bitmap_op(0, _p(dst), _p(src), dst.numel(), None, _stream()),
              "dev_bitmap_op")

    def step(self, off, raw, n, sync: bool = True, ev=None):
        """One rank's step.  Exchanges: canonical lengths (all-gather), covered
        bitmaps (all-gather + OR), first ranks over the merged dictionary (int32
        MIN), kept flags by global rank (uint8 MAX)."""
        k = [0]

        def mark_ev():
            if ev is not None:
                ev[k[0]].record()
            k[0] += 1
        assert n == self.n_local
        N = n * self.world
        L, s = self.L, _stream()
        mark_ev()
        self.canonicalize(off, raw, n)
        mark_ev()
        self.glens = gather_lens(self.new_len[:n], self.world)   # RCCL all-gather
        self.sort_order(self.glens, N)                          # identical on every rank
        mark_ev()
        items, ranks = self._local_items(N)
        m = n
        self.minimize(off, items, ranks, m, do_pass2=False)
        mark_ev()
        if self.key_mode:
            # dense key space: the first-cover array itself is the exchange
            # (nkeys int32, 16 MB at 2^22 keys; no dictionary, no host sync)
            merge_first(self.first[:self.span])                  # RCCL int32 MIN
            check(L.syzcov_dev_first_to_bits(_p(self.first), self.span, _p(self.covered), s),
                  "dev_first_to_bits")                          # union = keys with a first cover
            self.minimize_pass2(off, items, ranks, m)            # kept against the global first
            self.first[:self.span].fill_(INT32_MAX)              # other ranks' entries too
            merge_kept(self.kept[:N])                            # RCCL uint8 MAX
            self.build_dict(self.ws2)
            mark_ev()
            self.compact(N, self.ws2)
            mark_ev()
            self.union_list()
            mark_ev()
            self.merge_max_cover()
            mark_ev()
            return self.result() if sync else None
        merge_covered(self.covered[:self.nwords], self.world, self._or_into)
        self.build_dict(self.ws2)
        n_ids = int(self.scal[1].item()) & 0xFFFFFFFF
        check(L.syzcov_dev_first_dense(_p(self.tab), self.span, _p(self.first),
                                       _p(self.first_dense), 1, s), "dev_first_dense")
        merge_first(self.first_dense[:n_ids])                    # RCCL int32 MIN
        self.minimize_pass2(off, items, ranks, m, tab=self.tab, first_dense=self.first_dense)
        merge_kept(self.kept[:N])                                 # RCCL uint8 MAX
        mark_ev()
        self.compact(N, self.ws2)
        mark_ev()
        self.union_list()
        mark_ev()
        self.merge_max_cover()
        mark_ev()
        return self.result() if sync else None
