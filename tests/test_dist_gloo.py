"""World-size-2 (and 3) test of the sharded path's collective layer on CPU
(gloo): the product's gather_lens / local_items / merge_covered /
merge_first / merge_kept glue, with each shard's kernels emulated by the
oracle, must reproduce cover.Minimize + Union over the whole corpus."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as orc


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


SEED, N_LOCAL, LOG2 = 0x5EED0003, 300, 12


def _worker_range(rank, world, port, q):
    """The range engine's exchange (engine.dist.ShardedEngine.step_range) with
    each shard's kernels emulated by the oracle: local first-cover ranks and
    local union -> covered OR merge -> dictionary -> first MIN merge over dense
    ids -> pass 2 -> kept MAX merge."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from syzkaller_amd import dist as sdist
        lo, span = 0x81000000, 16 << LOG2
        off, pcs = orc.synth_corpus(SEED, N_LOCAL, 256, 96, LOG2, first=rank * N_LOCAL)
        c_off, c_pcs = orc.canonicalize_csr(off, pcs)
        lens = torch.from_numpy(np.diff(c_off).astype(np.int32))
        glens = sdist.gather_lens(lens, world).numpy()
        order = torch.from_numpy(orc.sort_order(glens.astype(np.int64)))
        items, ranks = sdist.local_items(order, rank, N_LOCAL)
        # pass 1 (emulated): window-indexed local first ranks + local covered bitmap
        first_w = np.full(span, 0x7FFFFFFF, np.int64)
        for i, r in zip(items.tolist(), ranks.tolist()):
            w = c_pcs[c_off[i]:c_off[i + 1]] - lo
            first_w[w] = np.minimum(first_w[w], r)
        bits = np.packbits((first_w != 0x7FFFFFFF).astype(np.uint8), bitorder="little")
        covered = torch.from_numpy(bits.view(np.int32).copy())
        # key mode's form of the same union: the shard bitmaps as byte maps,
        # uint8 MAX all-reduce (north_star), back to bits
        cov_u8 = covered.clone()
        u8 = torch.empty(cov_u8.numel() * 32, dtype=torch.uint8)

        def to_bytes(words, out):
            out.copy_(torch.from_numpy(np.unpackbits(words.numpy().view(np.uint8),
                                                     bitorder="little")))

        def to_bits(b, words):
            words.copy_(torch.from_numpy(np.packbits(b.numpy() != 0, bitorder="little")
                                         .view(np.int32).copy()))
        sdist.merge_bitmap_u8(cov_u8, u8, to_bytes, to_bits)
        sdist.merge_covered(covered, world, lambda d, s_: d.bitwise_or_(s_))
        assert torch.equal(cov_u8, covered), "u8 MAX merge != OR merge"
        gbits = np.unpackbits(covered.numpy().view(np.uint8), bitorder="little")[:span]
        present = np.nonzero(gbits)[0]
        # dictionary (dense id = rank of the PC in the merged union) and MIN merge
        first_d = torch.from_numpy(first_w[present].astype(np.int32))
        sdist.merge_first(first_d)
        gfirst = np.full(span, 0x7FFFFFFF, np.int64)
        gfirst[present] = first_d.numpy()
        kept = torch.zeros(N_LOCAL * world, dtype=torch.uint8)
        for i, r in zip(items.tolist(), ranks.tolist()):
            if np.any(gfirst[c_pcs[c_off[i]:c_off[i + 1]] - lo] == r):
                kept[r] = 1
        sdist.merge_kept(kept)
        q.put((rank, order[kept.bool()].tolist(), (present + lo).astype(np.uint32).tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_range_exchange_matches_oracle(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_range, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    off, pcs = orc.synth_corpus(SEED, N_LOCAL * world, 256, 96, LOG2)
    c_off, c_pcs = orc.canonicalize_csr(off, pcs)
    exp_kept = list(orc.minimize_csr(c_off, c_pcs))
    exp_union = orc.union_fold_csr(c_off, c_pcs).tolist()
    for rank, kept_idx, union in res:
        assert kept_idx == exp_kept, rank
        assert union == exp_union, rank


def _worker_prio(rank, world, port, q):
    """CalculatePriorities sharded by program: each rank's raw co-occurrence
    counts (emulated by the oracle) merged with the product's merge_counts."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from syzkaller_amd import dist as sdist
        lens = orc.synth_lens(0x5EED0004, 500, 30, 8, first=rank * 500).astype(np.int32)
        counts = torch.from_numpy(orc.dynamic_raw(lens, 64).astype(np.int32))
        sdist.merge_counts(counts)
        q.put((rank, counts.numpy()))
    finally:
        dist.destroy_process_group()


def test_sharded_prio_counts_sum():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_prio, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    lens = orc.synth_lens(0x5EED0004, 500 * world, 30, 8).astype(np.int32)
    exp = orc.dynamic_raw(lens, 64).astype(np.int32)
    for rank, c in res:
        assert np.array_equal(c, exp), rank

