"""Subprocess body for tests/test_gpu_engine.py::test_sharded_error_reaches_every_rank:
two key-mode ranks share cuda:0 (gloo collectives staged through the host).
(1) Rank 1's shard holds one PC that is not in the universe: its aliased
first covers go into the MIN merge, so EVERY rank's step must fail, not only
rank 1's (the error bits ride in KEPT[N..N+3] through the kept MAX merge,
one byte per bit); rank 0's out-of-extent PC adds SYZCOV_ERR_WINDOW, and every
rank must report both flags.
(2) A step abandoned after pass 1 (no exchange, no pass 2) leaves its first
ranks in FIRST: the next step must still give the clean results.
Each rank prints OK."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, world, port):
    import numpy as np
    import torch
    import torch.distributed as dist
    from syzkaller_amd.dist import ShardedEngine
    from syzkaller_amd.engine import synth_corpus, synth_universe, synth_window
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    n, seed, log2 = 1500, 0x5EED0002, 16
    lo, span = synth_window(log2)
    u = synth_universe(log2, seed)
    uh = u.cpu().numpy().view(np.uint32)

    def corpus():
        return synth_corpus(n, seed, first=rank * n, mean=1200, sigma=500, log2_space=log2)
    off, raw, lens, total = corpus()
    eng = ShardedEngine(n, total, int(lens.max().item()), lo, span, rank, world, universe=u)
    clean = eng.step(off, raw, n)
    kept0, union0 = clean.kept_idx.cpu().clone(), clean.union.cpu().clone()
    # (1) a stray PC (next to a universe PC, sharing its key) on the last rank only
    if rank == world - 1:
        j = int(off[n // 2].item()) + 3
        k = int(raw[j].item()) & 0xFFFFFFFF
        i = int(np.searchsorted(uh, k))
        us = set(uh.tolist())
        stray = next(int(uh[t]) + d for t in range(i, uh.size) for d in (1, 2, 3, 5)
                     if int(uh[t]) + d not in us)
        raw[j] = np.int32(np.uint32(stray))
    # ... and a PC outside the universe's extent on rank 0 (SYZCOV_ERR_WINDOW):
    # every rank must see both flags, OR-merged (one kept byte per flag bit)
    if rank == 0:
        raw[int(off[n // 3].item()) + 1] = np.int32(np.uint32(int(uh[-1]) + (1 << 12)))
    try:
        eng.step(off, raw, n)
        raise AssertionError(f"rank {rank}: a shard's non-universe PC did not fail the step")
    except RuntimeError as e:
        assert "[err_flags 0x5]" in str(e), (rank, str(e))  # WINDOW | UNIVERSE on every rank
    # (2) abandon a step after pass 1, then a full step on the clean corpus
    off, raw, lens, total = corpus()
    eng.canonicalize(off, raw, n)
    N = n * world
    from syzkaller_amd.dist import _all_gather
    _all_gather(eng.glens[:N], eng.new_len[:n].contiguous())
    eng.sort_order(eng.glens, N)
    eng.minimize(do_pass2=False)
    res = eng.step(off, raw, n)
    assert torch.equal(res.kept_idx.cpu(), kept0), rank
    assert torch.equal(res.union.cpu(), union0), rank
    dist.destroy_process_group()
    print("OK", rank, res.n_kept, res.n_union, flush=True)


def main():
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=worker, args=(r, world, port)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=150)
    codes = [p.exitcode for p in ps]
    for p in ps:
        if p.exitcode is None:
            p.kill()
    print("exit codes", codes, flush=True)
    sys.exit(0 if all(c == 0 for c in codes) else 1)


if __name__ == "__main__":
    main()
