"""Subprocess body for tests/test_gpu_engine.py::test_sharded_engine_world1:
the sharded engine (RCCL collectives, world_size 1) must give exactly the
single-GPU engine's results.  Prints OK on success."""
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    from syzkaller_amd.dist import ShardedEngine
    from syzkaller_amd.engine import CorpusEngine, synth_corpus, synth_window

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    n = 5000
    off, raw, lens, total = synth_corpus(n, 0x5EED0009, mean=700, sigma=300, log2_space=18)
    lo, span = synth_window(18)
    a = CorpusEngine(n, total, int(lens.max().item()), lo, span).step(off, raw, n)
    eng = ShardedEngine(n, total, int(lens.max().item()), lo, span, 0, 1)
    for _ in range(2):
        b = eng.step(off, raw, n)
        assert a.n_kept == b.n_kept and a.n_union == b.n_union and a.max_cover == b.max_cover
        assert torch.equal(a.kept_idx.cpu(), b.kept_idx.cpu())
        assert np.array_equal(a.union.cpu().numpy(), b.union.cpu().numpy())
    dist.destroy_process_group()
    print("OK", a.n_kept, a.n_union)


if __name__ == "__main__":
    main()
