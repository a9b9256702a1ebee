# one-GPU diagnosis of the C3 rehearsal: a ShardedEngine of world 1 (gloo) and
# of world 2 (two processes) over C3-sized shards, in place
import json, os, sys
import torch
sys.path.insert(0, '.')


def run(rank, world, port, n):
    import torch.distributed as dist
    from syzkaller_amd.dist import ShardedEngine
    from syzkaller_amd.engine import synth_corpus, synth_universe, synth_window
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    g = json.load(open('tests/golden/fullsize_digests.json'))['C3']
    lo, span = synth_window(g['log2_space'])
    univ = synth_universe(g['log2_space'], g['seed'])
    off, raw, lens, total = synth_corpus(n, g['seed'], first=rank * n, mean=g['mean'], sigma=g['sigma'], log2_space=g['log2_space'])
    r32 = raw[:int(total)].to(torch.int64) & 0xFFFFFFFF
    print('rank', rank, 'min %#x max %#x' % (int(r32.min()), int(r32.max())), 'lensmax', int(lens.max()), 'total', total, 'off_end', int(off[n]), flush=True)
    del r32
    torch.cuda.synchronize()
    eng = ShardedEngine(n, total, int(lens.max().item()), lo, span, rank, world, universe=univ, canon_in_place=True)
    print('rank', rank, 'free GB', torch.cuda.mem_get_info()[0] >> 30, flush=True)
    try:
        res = eng.step(off, raw, n)
        print('rank', rank, 'world', world, 'ok', res.n_kept, res.n_union, flush=True)
    except RuntimeError as e:
        print('rank', rank, 'world', world, 'ERR', e, flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    import socket
    import torch.multiprocessing as mp
    for world in (8,):
        s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
        ctx = mp.get_context("spawn")
        ps = [ctx.Process(target=run, args=(r, world, port, 1_250_000)) for r in range(world)]
        for p in ps: p.start()
        for p in ps: p.join(timeout=200)
        print('world', world, 'exit', [p.exitcode for p in ps], flush=True)
