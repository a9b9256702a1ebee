"""Subprocess body for tests/test_gpu_engine.py::test_sharded_engine_two_ranks:
two ranks of the sharded range engine share cuda:0 (collectives over gloo,
staged through the host), so the covered OR merge, the MIN merge of first
ranks over the merged dictionary and the kept MAX merge all run with real
HIP kernels.  Each rank checks its results against the single-GPU engine on
the whole corpus and prints OK."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, world, port, n, seed, log2):
    import numpy as np
    import torch
    import torch.distributed as dist
    from syzkaller_amd.dist import ShardedEngine
    from syzkaller_amd.engine import CorpusEngine, synth_corpus, synth_window
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    lo, span = synth_window(log2)
    off, raw, lens, total = synth_corpus(n, seed, first=rank * n, mean=600, sigma=300,
                                         log2_space=log2)
    eng = ShardedEngine(n, total, int(lens.max().item()), lo, span, rank, world)
    for _ in range(2):  # second step: engine state (first_w, records) must be clean
        res = eng.step(off, raw, n)
    # reference: the whole corpus on one engine
    goff, graw, glens, gtotal = synth_corpus(n * world, seed, mean=600, sigma=300,
                                             log2_space=log2)
    ref = CorpusEngine(n * world, gtotal, int(glens.max().item()), lo, span).step(goff, graw,
                                                                                n * world)
    assert res.n_kept == ref.n_kept, (res.n_kept, ref.n_kept)
    assert torch.equal(res.kept_idx.cpu(), ref.kept_idx.cpu())
    assert res.n_union == ref.n_union
    assert np.array_equal(res.union.cpu().numpy(), ref.union.cpu().numpy())
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
    ps = [ctx.Process(target=worker, args=(r, world, port, 3000, 0x5EED0013, 18))
          for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=100)
    codes = [p.exitcode for p in ps]
    print("exit codes", codes)
    sys.exit(0 if all(c == 0 for c in codes) else 1)


if __name__ == "__main__":
    main()
