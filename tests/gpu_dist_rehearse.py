"""Subprocess body for tests/test_gpu_fullsize.py::test_world8_rehearsal_*:
WORLD ranks of the sharded engine share cuda:0 (collectives over gloo, staged
through the host) and process config C2's 1M-input corpus (or C3's 10M,
canonicalized in place: 82 GB of raw PCs on the one GPU) split by input
(rank r holds global inputs [r*n, (r+1)*n)).  Rank 0 compares the kept list
and the union with the CPU oracle's full-size digests
(tests/golden/fullsize_digests.json) and prints OK.

usage: gpu_dist_rehearse.py WORLD [CONFIG] [keys|window]"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, world, port, cfg, keys):
    import torch
    import torch.distributed as dist
    from syzkaller_amd.dist import ShardedEngine
    from syzkaller_amd.engine import synth_corpus, synth_universe, synth_window
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    n = cfg["n"] // world
    x86 = cfg.get("synth_mode", 0) == 2  # C2X: the x86-like universe
    lo, span = synth_window(cfg["log2_space"], x86=x86)
    off, raw, lens, total = synth_corpus(n, cfg["seed"], first=rank * n, mean=cfg["mean"],
                                         sigma=cfg["sigma"], log2_space=cfg["log2_space"],
                                         x86=x86)
    univ = synth_universe(cfg["log2_space"], cfg["seed"], x86=x86) if keys else None
    inplace = cfg["n"] > 1_000_000
    eng = ShardedEngine(n, total, int(lens.max().item()), lo, span, rank, world, universe=univ,
                        canon_in_place=inplace)
    # the second step must find the engine state clean.  In place, the first
    # step's canonical key words replaced the raw PCs, so the second step is fed
    # raw PCs again, as a host re-feeds KCOV lists each step (syzcov.h)
    for step in range(2):
        if step and inplace:
            del off, raw
            off, raw, lens, total = synth_corpus(n, cfg["seed"], first=rank * n,
                                                 mean=cfg["mean"], sigma=cfg["sigma"],
                                                 log2_space=cfg["log2_space"], x86=x86)
        res = eng.step(off, raw, n)
        kept = res.kept_idx.cpu().numpy().astype("<i4").tobytes()
        union = res.union.cpu().numpy().astype("<i4").tobytes()
        got = (res.n_kept, hashlib.sha256(kept).hexdigest(), res.n_union,
               hashlib.sha256(union).hexdigest())
        exp = (cfg["n_kept"], cfg["kept_sha256"], cfg["n_union"], cfg["union_sha256"])
        assert got == exp, (rank, step, got, exp)
        # every rank computed the same Go order over the gathered lengths
        order = eng.order[:cfg["n"]].cpu().numpy().astype("<i4").tobytes()
        assert hashlib.sha256(order).hexdigest() == cfg["order_sha256"], (rank, step)
    dist.destroy_process_group()
    print("OK", rank, res.n_kept, res.n_union, flush=True)


def main():
    import socket
    import torch.multiprocessing as mp
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    name = sys.argv[2] if len(sys.argv) > 2 else "C2"
    keys = (sys.argv[3] if len(sys.argv) > 3 else "keys") == "keys"
    with open(os.path.join(ROOT, "tests", "golden", "fullsize_digests.json")) as f:
        cfg = json.load(f)[name]
    assert cfg["n"] % world == 0
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=worker, args=(r, world, port, cfg, keys)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=240 if cfg["n"] <= 1_000_000 else 520)
    codes = [p.exitcode for p in ps]
    for p in ps:
        if p.exitcode is None:
            p.kill()
    print("exit codes", codes, flush=True)
    sys.exit(0 if all(c == 0 for c in codes) else 1)


if __name__ == "__main__":
    main()
