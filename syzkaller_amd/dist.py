"""The corpus engine sharded by input over the GPUs of one node (weak
scaling: each rank holds a contiguous slice of the global corpus).

One process per GPU, torch.distributed over RCCL ("nccl" backend on ROCm).
The only exchanges are the reductions the first-cover formulation needs
(SURVEY §8e):

    presence map   uint8 MAX all-reduce   -> identical dense-id dictionary
    canonical lens all-gather             -> identical Go sort.Sort order
    first[]        int32 MIN all-reduce   -> global first-cover rank per PC id
    kept flags     uint8 MAX all-reduce   -> identical kept list on every rank

The collective glue below is device-agnostic (it runs under gloo on CPU
tensors in tests/test_dist_gloo.py); the per-shard compute is libsyzcov's
HIP kernels via engine.CorpusEngine.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .engine import CorpusEngine, StepResult, _p, _stream
from ._lib import check


# ------------------------------------------------------------------ glue
def merge_presence(pres: torch.Tensor) -> None:
    """Union of the shards' presence maps (RCCL has no OR: uint8 MAX)."""
    dist.all_reduce(pres, op=dist.ReduceOp.MAX)


def merge_first(first: torch.Tensor) -> None:
    """Global first-cover rank per dense PC id."""
    dist.all_reduce(first, op=dist.ReduceOp.MIN)


def merge_kept(kept: torch.Tensor) -> None:
    """kept[] is indexed by global rank; each rank set only its own items."""
    dist.all_reduce(kept, op=dist.ReduceOp.MAX)


def gather_lens(local_lens: torch.Tensor, world: int) -> torch.Tensor:
    """Canonical lengths of every shard, in global input order."""
    out = torch.empty(local_lens.numel() * world, dtype=local_lens.dtype,
                      device=local_lens.device)
    dist.all_gather_into_tensor(out, local_lens.contiguous())
    return out


def local_items(order: torch.Tensor, rank: int, n_local: int):
    """Work items of this shard in global processing order: (local input
    index, global rank) for every global rank whose input lives here."""
    base = rank * n_local
    sel = (order >= base) & (order < base + n_local)
    ranks = torch.nonzero(sel, as_tuple=False).flatten().to(torch.int32)
    return (order[ranks.long()] - base).to(torch.int32), ranks


# ---------------------------------------------------------------- engine
class ShardedEngine(CorpusEngine):
    """Rank `rank` of `world`: n local inputs of a global corpus of n*world."""

    def __init__(self, n: int, p_max: int, max_seg_len: int, pc_lo: int, pc_span: int,
                 rank: int, world: int, device="cuda", sort_variant: int = 0, mode: str = "pc"):
        super().__init__(n, p_max, max_seg_len, pc_lo, pc_span, device=device,
                         n_global=n * world, sort_variant=sort_variant, mode=mode)
        self.rank, self.world, self.n_local = rank, world, n
        self.glens = torch.empty(n * world, dtype=torch.int32, device=self.dev)
        self.pres_bytes = torch.empty(self.nwords * 32, dtype=torch.uint8, device=self.dev)
        # the global dictionary can be larger than this shard's PC count
        gcap = min(pc_span, p_max * world) + 1
        self.union = torch.empty(gcap, dtype=torch.int32, device=self.dev)
        if mode == "pc":
            # compact first-cover exchange: one int32 per present PC, not per window slot
            self.first_dense = torch.empty(gcap, dtype=torch.int32, device=self.dev)
        else:
            self.ids_cap = gcap
            self.first = torch.empty(gcap, dtype=torch.int32, device=self.dev)
            self.ws = torch.empty(max(self.ws_size, self.L.syzcov_dev_minimize_ws_size(gcap)),
                                  dtype=torch.uint8, device=self.dev)
            self.ws_size = self.ws.numel()

    def merge_first_window(self):
        """first_w (window-indexed) -> dense ids -> RCCL MIN -> back."""
        L, s = self.L, _stream()
        n_ids = int(self.scal[1].item()) & 0xFFFFFFFF
        check(L.syzcov_dev_first_dense(_p(self.tab), self.span, _p(self.first),
                                       _p(self.first_dense), 1, s), "dev_first_dense")
        merge_first(self.first_dense[:n_ids])
        check(L.syzcov_dev_first_dense(_p(self.tab), self.span, _p(self.first),
                                       _p(self.first_dense), 0, s), "dev_first_dense")

    def merge_presence_bits(self):
        """bits -> uint8 per PC -> RCCL MAX -> bits (exact OR of the shards)."""
        L, s = self.L, _stream()
        check(L.syzcov_dev_bits_to_bytes(_p(self.pres), self.span, _p(self.pres_bytes), s),
              "dev_bits_to_bytes")
        merge_presence(self.pres_bytes)
        check(L.syzcov_dev_bytes_to_bits(_p(self.pres_bytes), self.span, _p(self.pres), s),
              "dev_bytes_to_bits")

    def step(self, off, raw, n, sync: bool = True, ev=None):
        k = [0]

        def mark_ev():
            if ev is not None:
                ev[k[0]].record()
            k[0] += 1
        assert n == self.n_local
        N = n * self.world
        pc = self.mode == "pc"
        mark_ev()
        if pc:
            self.canonicalize_pcs(off, raw, n)          # local presence marked in-kernel
            mark_ev()
            self.merge_presence_bits()                  # RCCL uint8 MAX
            self.build_dict()
            mark_ev()
        else:
            self.mark(off, raw, n)
            self.merge_presence_bits()                  # RCCL uint8 MAX
            mark_ev()
            self.build_dict()
            mark_ev()
            self.canonicalize(off, raw, n)
            mark_ev()
        self.glens = gather_lens(self.new_len[:n], self.world)  # RCCL all-gather
        self.sort_order(self.glens, N)                  # identical on every rank
        mark_ev()
        items, ranks = local_items(self.order[:N], self.rank, n)
        if pc:
            self.minimize_win(off, items, ranks, items.numel(), do_pass2=False)
            self.merge_first_window()                   # RCCL int32 MIN over dense ids
            self.minimize_win_pass2(off, items, ranks, items.numel())
        else:
            self.minimize(off, items, ranks, items.numel(), do_pass2=False)
            merge_first(self.first)                     # RCCL int32 MIN
            self.minimize_pass2(off, items, ranks, items.numel())
        merge_kept(self.kept[:N])                       # RCCL uint8 MAX
        mark_ev()
        self.compact(N)
        mark_ev()
        self.union_list()
        mark_ev()
        self.merge_max_cover()
        mark_ev()
        return self.result() if sync else None
