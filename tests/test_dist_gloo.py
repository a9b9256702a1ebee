"""World-size-2 (and 3) test of the sharded path's collective layer on CPU
(gloo): the product's merge_presence / gather_lens / local_items /
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


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from syzkaller_amd import dist as sdist
        lo, span = 0x81000000, 16 << LOG2
        off, pcs = orc.synth_corpus(SEED, N_LOCAL, 256, 96, LOG2, first=rank * N_LOCAL)
        # mark (emulated kernel) + RCCL/gloo MAX merge (product glue)
        pres = np.zeros(span, np.uint8)
        pres[pcs[:off[-1]] - lo] = 1
        pres_t = torch.from_numpy(pres)
        sdist.merge_presence(pres_t)
        gp = pres_t.numpy()
        ids_of = np.cumsum(gp, dtype=np.int64) - 1  # dense id = rank in PC order
        # canonicalize (emulated) -> canonical lengths -> all-gather (glue)
        c_off, c_pcs = orc.canonicalize_csr(off, pcs)
        lens = torch.from_numpy(np.diff(c_off).astype(np.int32))
        glens = sdist.gather_lens(lens, world).numpy()
        order = torch.from_numpy(orc.sort_order(glens.astype(np.int64)))
        items, ranks = sdist.local_items(order, rank, N_LOCAL)
        # pass 1 (emulated): first[id] = min global rank over local items
        n_ids = int(gp.sum())
        first = np.full(n_ids, 0x7FFFFFFF, np.int32)
        for i, r in zip(items.tolist(), ranks.tolist()):
            ids = ids_of[c_pcs[c_off[i]:c_off[i + 1]] - lo]
            first[ids] = np.minimum(first[ids], r)
        first_t = torch.from_numpy(first)
        sdist.merge_first(first_t)
        gfirst = first_t.numpy()
        # pass 2 (emulated) into kept[global rank], then MAX merge (glue)
        kept = torch.zeros(N_LOCAL * world, dtype=torch.uint8)
        for i, r in zip(items.tolist(), ranks.tolist()):
            ids = ids_of[c_pcs[c_off[i]:c_off[i + 1]] - lo]
            if np.any(gfirst[ids] == r):
                kept[r] = 1
        sdist.merge_kept(kept)
        kept_idx = order[kept.bool()].tolist()
        union = (np.nonzero(gp)[0] + lo).astype(np.uint32)
        q.put((rank, kept_idx, union.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_minimize_union_matches_oracle(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # whole-corpus oracle
    off, pcs = orc.synth_corpus(SEED, N_LOCAL * world, 256, 96, LOG2)
    c_off, c_pcs = orc.canonicalize_csr(off, pcs)
    exp_kept = list(orc.minimize_csr(c_off, c_pcs))
    exp_union = orc.union_fold_csr(c_off, c_pcs).tolist()
    for rank, kept_idx, union in res:
        assert kept_idx == exp_kept, rank
        assert union == exp_union, rank
