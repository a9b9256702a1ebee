#!/usr/bin/env python3
"""Benchmarks of the syzkaller coverage hot path on MI355X.

Default (the driver's headline line): input-PCs processed/sec for
Canonicalize + Minimize + maxCover Union (BASELINE.json metric) over config C3
(10M inputs, the config the target is quoted on) at EVERY N: the whole corpus
on one GPU at N=1, sharded by input over the ranks at N>1 (RCCL merges; total
work fixed, so "strong" scaling and one config.workload string for the whole
1 -> 8 curve); --global-inputs overrides the corpus size.  N=1 adds config C2
(1M inputs, one GPU) as the `c2` sub-record.

One step = one pass of the hot path over one synthetic corpus already
resident in HBM (raw KCOV lists, CSR):
  Canonicalize (one wavefront per input: LDS radix sort + unique, range
  split points) -> Go sort.Sort order -> Minimize (first-cover pass 1 with
  LDS-resident covered ranges, pass 2 over the records) -> ordered
  compaction -> sorted Union list -> maxCover merge.
Prints ONE JSON line (rank 0).  Per-phase device times come from HIP events
on the stream the kernels run on; the dominant kernel's roofline uses its
ALGORITHMIC bytes.

--workload prio: config C4 (CalculatePriorities, 1M programs x 1170 calls,
i8 MFMA AᵀA) — a separate line with an MFMA roofline.
--workload newcov: config C5 (the fuzzer's streaming new-coverage check).
--workload dedup: the executor's cover_dedup (executor.cc:574-587) of raw u64
KCOV buffers (--records buffers per batch, the C2 length distribution).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# per-phase HBM bytes per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes over
# this same bench command (tools/profile.sh -> tools/traffic.py), committed per round:
# {"C3": {phase: ...}, "C2": ..., "newcov": ..., "dedup": ...}
TRAFFIC_JSON = os.path.join(ROOT, "profiles", "r06_traffic.json")


def traffic_of(workload: str, phase: str):
    """(bytes per launch, source) of a phase of a workload, or (None, None)."""
    if not os.path.exists(TRAFFIC_JSON):
        return None, None
    with open(TRAFFIC_JSON) as f:
        b = json.load(f).get(workload, {}).get(phase, {}).get("bytes")
    return b, (f"{os.path.relpath(TRAFFIC_JSON, ROOT)}[{workload}][{phase}]" if b else None)
I8_PEAK_TOPS = 5000.0      # dense i8 MFMA = 2x bf16 (~2.5 PF dense): MI355X_MICROARCH.md
SEED_C1 = 0x5EED0001  # BASELINE.json configs[0]: the CPU (reference) config
SEED = 0x5EED0002     # configs[1]: 1M inputs, one GPU
SEED_C3 = 0x5EED0003  # configs[2]: 10M inputs over the GPUs of one node
C3_INPUTS = 10_000_000
C2_INPUTS = 1_000_000
SEED_PRIO = 0x5EED0004
SEED_NEWCOV = 0x5EED0005
SEED_DEDUP = 0x5EED0006
FLAKE_INPUT = 1 << 40  # synthetic input index the C5 flakes set is drawn as


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=["corpus", "prio", "newcov", "dedup"], default="corpus")
    ap.add_argument("--records", type=int, default=65536, help="newcov: call records per batch")
    ap.add_argument("--no-early", action="store_true",
                    help="newcov: skip the early-regime sub-record (32 history batches)")
    ap.add_argument("--ncalls", type=int, default=293, help="newcov: CallIDs (sys.CallID)")
    ap.add_argument("--history", type=int, default=512,
                    help="newcov: batches streamed through the check before the bench (512: "
                         "maxCover near saturation, a long-running fuzzer; 32: the early, "
                         "candidate-heavy regime)")
    ap.add_argument("--inputs", type=int, default=1_000_000,
                    help="prio: programs per GPU; dedup/newcov: see --records")
    ap.add_argument("--global-inputs", type=int, default=None,
                    help="corpus inputs over all ranks, sharded by input (default: config "
                         "C3's 10M inputs, seed 0x5EED0003, at every N)")
    ap.add_argument("--seed", type=lambda x: int(x, 0), default=None)
    ap.add_argument("--mean", type=int, default=2048)
    ap.add_argument("--sigma", type=int, default=512)
    ap.add_argument("--log2-space", type=int, default=22)
    ap.add_argument("--cpu-sample", type=int, default=10_000,
                    help="inputs of config C1 timed on the CPU baseline (0 = skip)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--prio-dense", action="store_true",
                    help="prio: contract over all C keys instead of the active positional keys")
    ap.add_argument("--no-c2", action="store_true",
                    help="N=1: skip the C2 sub-record (1M inputs, BASELINE configs[1])")
    ap.add_argument("--no-dropin", action="store_true",
                    help="N=1: skip the drop-in legs (cover.Minimize from host buffers)")
    ap.add_argument("--no-universe", action="store_true",
                    help="window offsets instead of the dense keys of the registered PC "
                         "universe (keys.hip), for the corpus engine and newcov's maxCover")
    ap.add_argument("--x86", action="store_true",
                    help="corpus: the x86-like PC universe (neighbours 5..14 bytes apart, kshift 2) "
                         "instead of one PC per 16-byte slot; config name gets an X")
    ap.add_argument("--canon-layout", type=int, default=0, choices=[0, 1],
                    help="canonical lists: 0 CSR slots, 1 line-aligned sub-runs "
                         "(syzcov_corpus_cfg.canon_layout)")
    ap.add_argument("--no-rank-share", action="store_true",
                    help="N=1: skip the c3_rank_of_8 sub-record (rank 0's share of C3 over 8 GPUs)")
    ap.add_argument("--rank-share-only", action="store_true",
                    help="run only the c3_rank_of_8 leg and print it (a probe)")
    ap.add_argument("--no-order-parts", action="store_true",
                    help="c3_rank_of_8 without the per-rank order parts timed after its steps "
                         "(profiles: the counters then cover the step alone)")
    ap.add_argument("--dry-run", action="store_true",
                    help="start the ranks and the process group, run no workload (a check of "
                         "the --gpus N launcher; runs on a host without a GPU)")
    return ap.parse_args()


def launch_ranks(args) -> int:
    """`--gpus N` (N > 1) without a torch.distributed launcher: start N rank
    processes of this script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set,
    rank r on GPU r), relay rank 0's JSON line (everything else on stderr) and return the first failing
    exit code.  This process never touches the GPU (no torch import): every
    rank is a fresh child, never an exec of a GPU-initialised process."""
    import socket
    import subprocess
    n = args.gpus
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env, stdout=subprocess.PIPE if r == 0 else sys.stderr,
                                      text=True))
    import threading
    out0 = []  # rank 0 prints one line; read on a thread so a failing rank is seen at once
    reader = threading.Thread(target=lambda: out0.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    rc = 0
    while rc == 0 and any(p.poll() is None for p in procs):
        time.sleep(0.2)
        rc = next((p.returncode for p in procs if p.returncode not in (None, 0)), 0)
    if rc != 0:  # one rank failed: the others would wait in a collective forever
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p in procs:
        c = p.wait()
        if rc == 0 and c != 0:
            rc = c
    reader.join(timeout=10)
    # only the JSON line goes to stdout: what the ranks' libraries print there
    # (gloo's "[Gloo] Rank r is connected ..." notes) is relayed to stderr
    for line in "".join(out0).splitlines(keepends=True):
        (sys.stdout if line.startswith("{") else sys.stderr).write(line)
    sys.stdout.flush()
    return rc


def bench_dry(args):
    """The launcher and the process group without a workload: one line with
    the world the ranks actually formed."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
        t = __import__("torch").ones(1)
        dist.all_reduce(t)
        assert int(t.item()) == world
    glob = args.global_inputs or C3_INPUTS
    out = {"metric": "dry run (no workload)", "value": None, "n_gpus": world,
           "config": {"workload": corpus_workload(glob)[2], "global_inputs": glob,
                      "parallelism": f"shard-by-input x{world}"},
           "rccl_ranks": dist.get_world_size() if world > 1 else 1,
           "backend": dist.get_backend() if world > 1 else None}
    return rank, world, out


def cpu_baseline(args):
    """Oracle (literal C restatement of cover.go; Go toolchain absent) on the
    host, on BASELINE.json configs[0] = C1: the 10k-input synthetic corpus
    (seed 0x5EED0001), Canonicalize + Minimize + the Union fold, timed
    separately."""
    from oracle import oracle as orc
    orc.lib()
    n = args.cpu_sample
    off, pcs = orc.synth_corpus(SEED_C1, n, args.mean, args.sigma, args.log2_space)
    raw_pcs = int(off[-1])
    t0 = time.perf_counter()
    c_off, c_pcs = orc.canonicalize_csr(off, pcs)
    t1 = time.perf_counter()
    kept = orc.minimize_csr(c_off, c_pcs)
    t2 = time.perf_counter()
    union = orc.union_fold_csr(c_off, c_pcs)
    t3 = time.perf_counter()
    canon_pcs = int(c_off[-1])
    return {
        "value": raw_pcs / (t3 - t0), "unit": "input-PCs/s", "cores": 1, "kind": "port",
        "sample": (f"config C1: {n} inputs of the seed-{SEED_C1:#x} synthetic corpus "
                   f"({raw_pcs} raw PCs): Canonicalize {t1 - t0:.2f}s + Minimize {t2 - t1:.2f}s "
                   f"+ Union fold {t3 - t2:.2f}s, 1 thread, oracle/ C restatement of "
                   f"cover/cover.go (Go toolchain absent)"),
        "phases_s": {"canonicalize": t1 - t0, "minimize": t2 - t1, "union_fold": t3 - t2},
        # cover.Minimize (its sort.Sort included, cover.go:113) + the Union fold
        "minimize_canonical_pcs_per_s": canon_pcs / (t2 - t1),
        "minimize_union_canonical_pcs_per_s": canon_pcs / (t3 - t1),
        "union_fold_canonical_pcs_per_s": canon_pcs / (t3 - t2),
        "results": {"kept": int(len(kept)), "union": int(union.size)},
        "host": platform.processor() or platform.machine(),
        "nproc": os.cpu_count(),
    }


def stream_peak(dev, nbytes: int = 4 << 30, reps: int = 10) -> dict:
    """Measured HBM copy rate (GB/s, read + write bytes), next to the 8 TB/s
    vendor figure: the better of the library's two copy forms (the streaming
    copy, and the one-element-per-thread float4 shape of the guide's 6.29 TB/s
    measurement)."""
    import ctypes as C
    import torch
    from syzkaller_amd import _lib
    L = _lib.lib()
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    a.fill_(1)
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)

    rates = {}
    for form, name in ((0, "streaming"), (1, "flat_float4")):
        def copy():
            _lib.check(L.syzcov_dev_copy_peak(C.c_void_p(a.data_ptr()), C.c_void_p(b.data_ptr()),
                                              nbytes, form, s), "copy_peak")
        copy()
        copy()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            copy()
        e1.record()
        torch.cuda.synchronize()
        rates[name] = 2 * nbytes / (e0.elapsed_time(e1) / reps * 1e-3) / 1e9
    del a, b
    torch.cuda.empty_cache()
    return rates


def cpu_baseline_prio(nprog: int, C: int):
    from oracle import oracle as orc
    import numpy as np
    orc.lib()
    lens = orc.synth_lens(SEED_PRIO, nprog, 30, 8)
    static = np.ones((C, C), np.float32)
    t0 = time.perf_counter()
    orc.calculate_priorities(lens.astype(np.int32), static)
    dt = time.perf_counter() - t0
    return {"value": nprog / dt, "unit": "programs/s", "cores": 1, "kind": "port",
            "sample": f"{nprog} programs, calcDynamicPrio + normalizePrio + combine, "
                      f"oracle/ C restatement of prog/prio.go, 1 thread"}


def init_dist():
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev_idx = local if world > 1 else 0
    backend = "nccl"  # RCCL over xGMI
    ngpu = torch.cuda.device_count()
    if world > ngpu:
        # rehearsal of the N-rank path on fewer GPUs (e.g. 2 ranks on the 1-GPU
        # test box): ranks share devices and the collectives go through gloo
        dev_idx, backend = local % ngpu, "gloo"
    dev = torch.device("cuda", dev_idx)
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group(backend)
    return world, rank, dev


def timed(run_step, nphase, args, world, dev):
    """W warmup steps, then K timed steps bracketed by barrier + sync; per-phase
    HIP-event times; returns (seconds (max over ranks), per-phase ms)."""
    import torch
    import torch.distributed as dist
    for _ in range(args.warmup):
        run_step(None)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    evs = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(nphase + 1)]
        run_step(ev)
        evs.append(ev)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ph = [0.0] * nphase
    for ev in evs:
        for i in range(nphase):
            ph[i] += ev[i].elapsed_time(ev[i + 1]) / len(evs)
    return dt, ph


def corpus_workload(glob: int) -> tuple[str, int, str]:
    """(config name, seed, config.workload) of a corpus of `glob` inputs over
    all ranks: the same string at every N, so the driver's 1 -> 8 curve joins
    like with like (the sharding is in config.parallelism)."""
    if glob == C3_INPUTS:
        cname, seed = "C3", SEED_C3
    elif glob == C2_INPUTS:
        cname, seed = "C2", SEED
    else:
        cname, seed = "custom", SEED
    return cname, seed, f"{cname}: Canonicalize + Minimize + maxCover union, {glob} inputs"


def corpus_run(args, world, rank, dev, glob, seed, steps, warmup, traffic_key, x86=False):
    """K timed steps of the corpus pipeline over `glob` inputs (rank r holds
    [r*n, (r+1)*n)), generated into HBM, canonicalized out of place; returns
    the measured part of a line (phases, roofline of the dominant phase and of
    Minimize, results).  x86: the x86-like PC universe (kshift 2)."""
    import torch
    from syzkaller_amd.engine import CorpusEngine, synth_corpus, synth_universe, synth_window
    n = -(-glob // world)
    lo, span = synth_window(args.log2_space, x86=x86)
    off, raw, lens, total = synth_corpus(n, seed, first=rank * n, mean=args.mean,
                                         sigma=args.sigma, log2_space=args.log2_space, device=dev,
                                         x86=x86)
    max_len = int(lens.max().item())
    del lens
    # the PC universe (allCoverPCs, syz-manager/cover.go:57-69) is registered once,
    # outside the timed steps, like the resident maxCover
    univ = None if args.no_universe else synth_universe(args.log2_space, seed, device=dev, x86=x86)
    if world > 1:
        from syzkaller_amd.dist import ShardedEngine
        eng = ShardedEngine(n, total, max_len, lo, span, rank, world, device=dev, universe=univ,
                            canon_layout=args.canon_layout)
    else:
        eng = CorpusEngine(n, total, max_len, lo, span, device=dev, universe=univ,
                           canon_layout=args.canon_layout)
    del univ
    torch.cuda.synchronize()
    phases = list(eng.PHASES)
    a = argparse.Namespace(steps=steps, warmup=warmup)
    dt, phl = timed(lambda ev: eng.step(off, raw, n, sync=False, ev=ev), len(phases), a, world,
                    dev)
    ph = dict(zip(phases, phl))
    res = eng.result()
    canon_pcs = int(eng.new_len[:n].to(torch.int64).sum().item())
    # algorithmic bytes per launch: canon reads raw + writes the
    # canonical list; minimize reads the canonical list once
    alg = eng.alg_bytes(total, canon_pcs)
    dom = max(alg, key=lambda p: ph[p])
    achieved = alg[dom] / (ph[dom] * 1e-3) / 1e9
    traffic, tsrc = traffic_of(traffic_key, dom) if world == 1 else (None, None)
    mz = alg["minimize"] / (ph["minimize"] * 1e-3) / 1e9
    out = {
        "value": total * world * steps / dt, "ms_per_step": dt / steps * 1e3,
        "inputs_per_gpu": n, "raw_pcs_per_gpu": total, "canonical_pcs_per_gpu": canon_pcs,
        "aligned": bool(eng.canon_align_k),
        "keys": (f"dense keys of the registered PC universe: (pc >> {eng.kshift}) - "
                 f"{eng.kbase:#x}, {eng.span} keys" if eng.key_mode
                 else f"window offsets pc - {lo:#x}, {span} keys"),
        "phases_ms": {k: round(v, 4) for k, v in ph.items()},
        "results": {"kept": res.n_kept, "union": res.n_union, "max_cover": res.max_cover,
                    "n_ids": res.n_ids},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": tsrc,
                     "alg_bytes_per_launch": alg[dom]},
        # the Minimize phase's own roofline (the metric's Minimize + Union part)
        "minimize_roofline": {
            "achieved": mz, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": mz / HBM_PEAK_GBS,
            "traffic": traffic_of(traffic_key, "minimize")[0] if world == 1 else None,
            "alg_bytes_per_launch": alg["minimize"]},
        # cover.Minimize's own work (cover.go:104-131): Go's sort.Sort order, the
        # first-cover passes, the kept list; + the union (maxCover merge)
        "minimize_union_pcs_per_s": canon_pcs * world / ((ph["order"] + ph["minimize"]
                                                          + ph.get("exchange", 0.0)
                                                          + ph["finish"]) * 1e-3),
    }
    eng.close()
    del eng, off, raw
    torch.cuda.empty_cache()
    return out


def rank_share_run(args, dev, world: int = 8, rank: int = 0, glob: int = C3_INPUTS,
                   seed: int = SEED_C3, steps: int = 10, warmup: int = 2) -> dict:
    """Rank `rank`'s exact share of the `world`-GPU step over C3, on this one
    GPU: its n = glob / world inputs canonicalized (out of place), its part of
    Go's order over ALL glob canonical lengths (syzcov_corpus_order_part: the
    replicated early rounds plus the late rounds of the segments starting in
    its block), Minimize pass 1 over its own items at GLOBAL ranks, pass 2 and
    finish — every kernel the rank runs in `dist.ShardedEngine.step`.  The
    collectives cannot run on one GPU; each is replaced by what it leaves in the
    buffer: the other ranks' canonical lengths are computed before the timed
    steps (the all-gather's result) and the merged order is copied in (the MAX
    all-reduce's result, a 40 MB device copy inside the timed order phase);
    the MIN merge of first ranks and the MAX merge of kept flags are skipped
    (pass 2 reads this rank's own first ranks: the same kernels and bytes).
    Their bytes are reported apart (`collectives`)."""
    import ctypes as C
    import torch
    from syzkaller_amd import _lib
    from syzkaller_amd.dist import ShardedEngine
    from syzkaller_amd.engine import synth_corpus, synth_universe, synth_window
    L = _lib.lib()
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    n = glob // world
    N = n * world
    lo, span = synth_window(args.log2_space)
    totals, max_len = [], 0
    lens = torch.empty(n, dtype=torch.int32, device=dev)
    for r in range(world):  # every rank's raw size (synth_lens is the generator's own)
        _lib.check(L.syzcov_dev_synth_lens(seed, r * n, n, args.mean, args.sigma,
                                           C.c_void_p(lens.data_ptr()), s), "synth_lens")
        totals.append(int(lens.to(torch.int64).sum().item()))
        max_len = max(max_len, int(lens.max().item()))
    del lens
    univ = None if args.no_universe else synth_universe(args.log2_space, seed, device=dev)
    eng = ShardedEngine(n, max(totals), max_len, lo, span, rank, world, device=dev, universe=univ,
                        canon_layout=args.canon_layout)
    del univ
    # the all-gather's result: every other rank's canonical lengths (its canon
    # on this GPU, outside the timed steps)
    glens = eng.glens[:N]
    for r in range(world):
        if r == rank:
            continue
        off_r, raw_r, _, _ = synth_corpus(n, seed, first=r * n, mean=args.mean, sigma=args.sigma,
                                          log2_space=args.log2_space, device=dev)
        eng.canonicalize(off_r, raw_r, n)
        glens[r * n:(r + 1) * n].copy_(eng.new_len[:n])
        del off_r, raw_r
        torch.cuda.empty_cache()
    off, raw, _, total = synth_corpus(n, seed, first=rank * n, mean=args.mean, sigma=args.sigma,
                                      log2_space=args.log2_space, device=dev)
    eng.canonicalize(off, raw, n)
    glens[rank * n:(rank + 1) * n].copy_(eng.new_len[:n])
    # the MAX all-reduce's result: Go's order over all N lengths
    _lib.check(L.syzcov_corpus_order(eng.h, C.c_void_p(glens.data_ptr()), N, s), "corpus_order")
    full_order = eng.order[:N].clone()
    torch.cuda.synchronize()
    phases = ("canon", "order", "minimize", "exchange", "finish")

    def step(ev):
        k = [0]

        def mark():
            if ev is not None:
                ev[k[0]].record()
            k[0] += 1
        mark()
        eng.canonicalize(off, raw, n)
        mark()
        glens[rank * n:(rank + 1) * n].copy_(eng.new_len[:n])  # this rank's part of the gather
        _lib.check(L.syzcov_corpus_order_part(eng.h, C.c_void_p(glens.data_ptr()), N, s),
                   "corpus_order_part")
        eng.order[:N].copy_(full_order)                         # stands in for the MAX merge
        mark()
        eng.minimize(do_pass2=False)
        mark()
        if eng.bitmap_union:  # the shard bitmap as a byte map (its MAX all-reduce not run)
            eng._to_bytes(eng.covered, eng.cov_u8)
        _lib.check(L.syzcov_corpus_pass2(eng.h, s), "corpus_pass2")
        if eng.bitmap_union:
            eng._to_bits(eng.cov_u8, eng.covered)
        mark()
        eng.finish()
        mark()
    a = argparse.Namespace(steps=steps, warmup=warmup)
    dt, phl = timed(step, len(phases), a, 1, dev)
    ph = dict(zip(phases, phl))
    res = eng.result()
    # every rank's part of the order (the phase's critical path is the slowest
    # part): syzcov_dev_sort_order_part over the same lengths, part r of world
    lens64 = glens.to(torch.int64)
    wsz = L.syzcov_dev_sort_ws_size(N)
    ws = torch.empty(wsz, dtype=torch.uint8, device=dev)
    po = torch.empty(N, dtype=torch.int32, device=dev)
    part_ms = []
    for r in range(0 if getattr(args, "no_order_parts", False) else world):
        for rep in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            _lib.check(L.syzcov_dev_sort_order_part(C.c_void_p(lens64.data_ptr()), N, r, world,
                                                    C.c_void_p(po.data_ptr()),
                                                    C.c_void_p(ws.data_ptr()), wsz, s),
                       "dev_sort_order_part")
            e1.record()
            torch.cuda.synchronize()
            if rep:
                part_ms.append((r, e0.elapsed_time(e1)))
    order_parts = [round(min(t for q, t in part_ms if q == r), 4)
                   for r in range(world)] if part_ms else None
    del lens64, ws, po
    canon_pcs = int(eng.new_len[:n].to(torch.int64).sum().item())
    alg = eng.alg_bytes(total, canon_pcs)
    cf = alg["canon"] / (ph["canon"] * 1e-3) / 1e9
    mf = alg["minimize"] / (ph["minimize"] * 1e-3) / 1e9
    # what the rank's collectives move (ring algorithms: an all-gather receives
    # (w-1)/w of the result, an all-reduce sends and receives 2(w-1)/w of it)
    f_ag, f_ar = (world - 1) / world, 2 * (world - 1) / world
    coll = {"lens_allgather_int32": N * 4, "order_max_allreduce_int32": N * 4,
            "first_min_allreduce_int32": eng.span * 4, "kept_max_allreduce_u8": N + 4,
            "covered_max_allreduce_u8": eng.cov_u8.numel() if eng.bitmap_union else 0}
    ring = (f_ag * coll["lens_allgather_int32"] + f_ar * (coll["order_max_allreduce_int32"]
            + coll["first_min_allreduce_int32"] + coll["kept_max_allreduce_u8"]
            + coll["covered_max_allreduce_u8"]))
    out = {
        "workload": (f"rank {rank} of {world} over C3 ({glob} inputs, seed {seed:#x}): its {n} "
                     f"inputs, Go's order over all {N} lengths, pass 1 at global ranks"),
        "ms_per_step": dt / steps * 1e3,
        "rank_input_pcs_per_s": total * steps / dt,
        "raw_pcs": total, "canonical_pcs": canon_pcs,
        "phases_ms": {k: round(v, 4) for k, v in ph.items()},
        "canon_roofline": {"achieved": cf, "frac": cf / HBM_PEAK_GBS,
                           "alg_bytes_per_launch": alg["canon"],
                           "traffic": traffic_of("C3R8", "canon")[0]},
        "minimize_roofline": {"achieved": mf, "frac": mf / HBM_PEAK_GBS,
                              "alg_bytes_per_launch": alg["minimize"],
                              "traffic": traffic_of("C3R8", "minimize")[0]},
        # Minimize + union as the metric counts it: order + minimize + the
        # exchange phase's pass 2 + finish
        "minimize_union_ms": ph["order"] + ph["minimize"] + ph["exchange"] + ph["finish"],
        # each rank's order part alone (device tier, this GPU): the slowest is
        # the 8-GPU order phase's critical path
        "order_part_ms_by_rank": order_parts,
        "collectives": {"bytes": coll, "ring_bytes_per_rank": int(ring),
                        "note": "not run on one GPU; the 8-GPU step adds their time"},
        "results": {"kept_local_first": res.n_kept, "union_local": res.n_union},
        "stand_ins": "other ranks' lengths precomputed; merged order copied in; own first ranks "
                     "for the MIN merge; own byte map for the covered MAX merge (converted both "
                     "ways); kept MAX skipped",
    }
    eng.close()
    del eng, off, raw, full_order
    torch.cuda.empty_cache()
    return out


def bench_corpus(args):
    """The headline: config C3 (10M inputs, seed 0x5EED0003) at EVERY N — the
    whole corpus on one GPU at N=1, sharded by input over the ranks at N>1
    (total work fixed: strong scaling).  N=1 adds config C2 (1M inputs, the
    one-GPU config of BASELINE.json) as the `c2` sub-record, the drop-in legs
    and the CPU baseline."""
    world, rank, dev = init_dist()
    if args.rank_share_only:
        return rank, world, {"c3_rank_of_8": rank_share_run(args, dev, steps=args.steps,
                                                            warmup=args.warmup)}
    glob = args.global_inputs or C3_INPUTS
    cname, seed, workload = corpus_workload(glob)
    if args.x86:
        cname += "X"
        workload = workload.replace(":", "X (x86-like PC universe):", 1)
    if args.seed is not None:
        seed = args.seed
    m = corpus_run(args, world, rank, dev, glob, seed, args.steps, args.warmup, cname,
                   x86=args.x86)
    out = {
        "metric": "input-PCs processed/sec for Canonicalize+Minimize+Union (maxCover merge)",
        "value": m.pop("value"), "unit": "input-PCs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": m.pop("ms_per_step"),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "u32", "data": "synthetic (counter-based generator, SURVEY §8d)",
        "config": {"workload": workload, "seed": seed, "global_inputs": glob,
                   "inputs_per_gpu": m.pop("inputs_per_gpu"),
                   "raw_pcs_per_gpu": m.pop("raw_pcs_per_gpu"),
                   "canonical_pcs_per_gpu": m.pop("canonical_pcs_per_gpu"),
                   "pc_space": 1 << args.log2_space, "len_mean": args.mean,
                   "len_sigma": args.sigma, "keys": m.pop("keys"),
                   "canon": "out of place" + (", line-aligned sub-runs" if m.pop("aligned")
                                              else ", CSR slots"),
                   "parallelism": f"shard-by-input x{world}"},
    }
    out.update(m)
    if world == 1:
        rates = stream_peak(dev)
        pk = max(rates.values())
        out["roofline"]["peak_measured"] = pk
        out["roofline"]["peak_measured_forms"] = rates
        out["roofline"]["peak_guide_float4_copy"] = 6290.0  # MI355X_MICROARCH.md:36
        out["roofline"]["frac_of_measured"] = out["roofline"]["achieved"] / pk
        if not args.no_c2 and (glob != C2_INPUTS or args.x86):
            c2 = corpus_run(args, 1, 0, dev, C2_INPUTS, SEED, max(args.steps, 10), args.warmup,
                            "C2")
            c2["workload"] = corpus_workload(C2_INPUTS)[2] + " (one GPU, BASELINE configs[1])"
            c2["seed"] = SEED
            out["c2"] = c2
        if not args.no_c2 and not (glob == C2_INPUTS and args.x86):
            # C2 over an x86-like universe (PCs 5..14 bytes apart, kshift 2,
            # 2^23 keys): the canon's 3-pass sort and 64 Minimize ranges
            cx = corpus_run(args, 1, 0, dev, C2_INPUTS, SEED, max(args.steps, 10), args.warmup,
                            "C2X", x86=True)
            cx["workload"] = ("C2X: C2 over the x86-like PC universe (neighbours 5..14 bytes "
                              "apart, kshift 2)")
            cx["seed"] = SEED
            out["c2x"] = cx
        if not args.no_rank_share and glob == C3_INPUTS and not args.x86:
            # the 8-GPU step's per-rank work, measured on this GPU
            out["c3_rank_of_8"] = rank_share_run(args, dev, steps=max(args.steps, 10),
                                                 warmup=args.warmup)
        if not args.no_c2:
            out["c4"] = c4_subrecord(args, dev)
        if not args.no_dropin:
            out["dropin"] = dropin_legs(args, dev)
            out["dropin"]["pairwise"] = pairwise_leg()
    if rank == 0 and world == 1 and not args.no_cpu and args.cpu_sample > 0:
        cb = out["cpu_baseline"] = cpu_baseline(args)
        out["vs_cpu"] = out["value"] / cb["value"]
        # like with like: both rates count Go's sort.Sort order, the Minimize
        # passes and the union over canonical PCs
        out["vs_cpu_minimize_union"] = (out["minimize_union_pcs_per_s"]
                                        / cb["minimize_union_canonical_pcs_per_s"])
    return rank, world, out


def dropin_legs(args, dev):
    """cover.Minimize through the drop-in C-ABI from HOST buffers, PCIe
    included, on the C1 / C2 synthetic corpora (raw covers, as a manager
    holds them):
      shim       syzcov_minimize with the order Go's own sort.Sort produced (what
                 the cgo shim of INTEGRATION.md passes; here the library's restated
                 sort over the raw lengths stands in for it, timed apart): the
                 cached window-mode engine, one call after a warm-up call
      handle     syzcov_corpus_minimize_host on a persistent key-mode handle
                 (the manager's resident form; its own order over canonical lengths)
      groups     syzcov_minimize_corpus (Manager.minimizeCorpus, manager.go:504-524)
                 over the same corpus split into 293 call groups (sys.CallCount)."""
    import ctypes as C
    import numpy as np
    import torch
    from syzkaller_amd import _lib
    from syzkaller_amd.engine import synth_corpus, synth_universe
    L = _lib.lib()
    legs = {}
    for name, n, seed in (("C1", 10_000, SEED_C1), ("C2", C2_INPUTS, SEED)):
        off, raw, lens, total = synth_corpus(n, seed, mean=args.mean, sigma=args.sigma,
                                             log2_space=args.log2_space, device=dev)
        h_off = off.cpu().numpy().astype(np.uint64)
        h_pcs = raw[:total].cpu().numpy().view(np.uint32)
        max_len = int(lens.max().item())
        canon_pcs = canonical_total(off, raw, n, max_len, args.log2_space, dev)  # (in place)
        del off, raw, lens
        torch.cuda.empty_cache()
        out = np.empty(n, np.int32)
        # the shim's order: Go sort.Sort(minInputArray) over len(cov) (cover.go:113)
        rl = np.diff(h_off).astype(np.int64)
        order = np.empty(n, np.int32)
        _lib.check(L.syzcov_sort_order(rl.ctypes.data, n, 0, order.ctypes.data), "sort_order")
        ts = []
        for _ in range(2):  # the first call creates the cached engine
            t0 = time.perf_counter()
            k = _lib.check(L.syzcov_minimize(h_off.ctypes.data, h_pcs.ctypes.data, n,
                                             order.ctypes.data, 0, out.ctypes.data), "minimize")
            ts.append(time.perf_counter() - t0)
        kept_shim = out[:k].copy()
        t0 = time.perf_counter()
        k0 = _lib.check(L.syzcov_minimize(h_off.ctypes.data, h_pcs.ctypes.data, n, None, 0,
                                          out.ctypes.data), "minimize")
        t_noorder = time.perf_counter() - t0
        assert k0 == k and np.array_equal(out[:k0], kept_shim)
        L.syzcov_pool_trim()
        univ = synth_universe(args.log2_space, seed, device=dev).cpu().numpy().view(np.uint32)
        cfg = _lib.CorpusCfg(n_max=n, p_max=total, max_seg_len=max_len,
                             universe=univ.ctypes.data, universe_n=univ.size)
        h = C.c_uint64(0)
        _lib.check(L.syzcov_corpus_create(C.byref(cfg), None, 0, C.byref(h)), "corpus_create")
        un = np.empty(1 << args.log2_space, np.uint32)
        nu = C.c_uint64(0)
        reps, tk = 2, []
        for _ in range(reps + 1):
            ta = time.perf_counter()
            k2 = _lib.check(L.syzcov_corpus_minimize_host(h.value, h_off.ctypes.data,
                                                          h_pcs.ctypes.data, n, out.ctypes.data,
                                                          un.ctypes.data, un.size, C.byref(nu)),
                            "corpus_minimize_host")
            tk.append(time.perf_counter() - ta)
        L.syzcov_corpus_destroy(h.value)
        leg = {
            "inputs": n, "raw_pcs": total,
            "shim_ms": round(ts[1] * 1e3, 2), "shim_first_call_ms": round(ts[0] * 1e3, 2),
            "shim_kept": k, "shim_input_pcs_per_s": total / ts[1],
            "restated_order_in_library_ms": round(t_noorder * 1e3, 2),
            "handle_minimize_host_ms": round(min(tk[1:]) * 1e3, 2),
            "handle_minimize_host_kept": k2, "handle_union": nu.value,
            "handle_minimize_host_input_pcs_per_s": total / min(tk[1:]),
            "shim_vs_handle": ts[1] / min(tk[1:]),
            "note": "host buffers in and out, PCIe transfers included; the shim orders by the "
                    "raw lengths (Minimize of covers as given), the handle by canonical lengths"}
        # Manager.minimizeCorpus: the corpus in 293 call groups (synthetic call ids)
        calls = np.empty(n, np.int32)
        s_ = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        cid = torch.empty(n, dtype=torch.int32, device=dev)
        _lib.check(L.syzcov_dev_synth_callids(seed, 0, n, 293, C.c_void_p(cid.data_ptr()), s_),
                   "synth_callids")
        calls[:] = cid.cpu().numpy()
        tgs = []
        for _ in range(2):  # the first call allocates the staging buffers
            t0 = time.perf_counter()
            kg = _lib.check(L.syzcov_minimize_corpus(calls.ctypes.data, h_off.ctypes.data,
                                                     h_pcs.ctypes.data, n, 0, out.ctypes.data),
                            "minimize_corpus")
            tgs.append(time.perf_counter() - t0)
        tg = tgs[1]
        gs = _lib.GroupsStats()
        _lib.check(L.syzcov_minimize_corpus_stats(C.byref(gs)), "minimize_corpus_stats")
        # device part: one canonicalization (4 B read per raw PC, 4 B written per
        # canonical PC) and one grouped Minimize pass (4 B per canonical PC); the
        # path's extra union step is not counted
        g_alg = 4 * total + 8 * canon_pcs
        leg.update({"groups": 293, "minimize_corpus_ms": round(tg * 1e3, 2),
                    "minimize_corpus_first_call_ms": round(tgs[0] * 1e3, 2),
                    "minimize_corpus_kept": kg, "minimize_corpus_input_pcs_per_s": total / tg,
                    "minimize_corpus_vs_handle": tg / min(tk[1:]),
                    "minimize_corpus_path": _lib.GROUPS_PATHS.get(gs.path, gs.path),
                    "minimize_corpus_upload_ms": round(gs.upload_ms, 3),
                    "minimize_corpus_device_ms": round(gs.device_ms, 3),
                    "minimize_corpus_download_ms": round(gs.download_ms, 3),
                    "minimize_corpus_device_roofline": (
                        {"achieved": g_alg / (gs.device_ms * 1e-3) / 1e9,
                         "frac": g_alg / (gs.device_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "unit": "GB/s", "alg_bytes": g_alg, "canonical_pcs": canon_pcs,
                         "note": "device_ms includes the path's union step and its host "
                                 "read-backs; alg bytes count one canon + one Minimize pass"}
                        if gs.device_ms > 0 else None)})
        L.syzcov_pool_trim()
        legs[name] = leg
        del h_pcs, h_off
    return legs


def canonical_total(off, raw, n: int, max_len: int, log2_space: int, dev) -> int:
    """Canonical PCs of a synthetic corpus (its raw lists canonicalized IN PLACE
    on the device, syzcov_dev_canon_split): the algorithmic-bytes count of a
    leg that only sees host buffers."""
    import ctypes as C
    import torch
    from syzkaller_amd import _lib
    from syzkaller_amd.engine import synth_window
    L = _lib.lib()
    lo, span = synth_window(log2_space)
    nl = torch.empty(n + 1, dtype=torch.int32, device=dev)
    err = torch.zeros(4, dtype=torch.int32, device=dev)
    wsz = L.syzcov_dev_canon_split_ws_size(n)
    ws = torch.empty(wsz, dtype=torch.uint8, device=dev)
    P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    _lib.check(L.syzcov_dev_canon_split(P(off), P(raw), P(raw), P(nl), n, max_len, lo, span, 20,
                                        None, None, P(err), P(ws), wsz,
                                        C.c_void_p(torch.cuda.current_stream().cuda_stream)),
               "canon_split")
    if int(err[0].item()):
        raise RuntimeError(f"canonicalize flags {int(err[0].item()):#x}")
    return int(nl[:n].to(torch.int64).sum().item())


def pairwise_leg(reps: int = 2000, nthreads: int = 32) -> dict:
    """The drop-in per-call set ops on the fuzzer's list sizes: cover.Difference
    and cover.Union (cover/cover.go:42-79) of two ~2k-PC canonical lists, as
    syz-fuzzer calls Difference twice per executed call (fuzzer.go:465-466),
    through syzcov_difference / syzcov_union (one device round trip each) from
    1 thread and from `nthreads` concurrent threads, beside the oracle's merge
    (C, 1 thread: Go's foreach loop)."""
    import ctypes as C
    import threading
    import numpy as np
    from oracle import oracle as orc
    from syzkaller_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(17)
    pool = 0x81000000 + 16 * np.arange(1 << 16, dtype=np.uint32)
    a = np.sort(rng.choice(pool, 2048, replace=False)).astype(np.uint32)
    b = np.sort(np.concatenate([a[rng.random(a.size) < 0.95],
                                rng.choice(pool, 100, replace=False)])).astype(np.uint32)
    b = np.unique(b)
    out = {}
    for name, fn in (("difference", L.syzcov_difference), ("union", L.syzcov_union)):
        def calls(k, o):
            for _ in range(k):
                fn(a.ctypes.data, a.size, b.ctypes.data, b.size, o.ctypes.data)
        o = np.empty(a.size + b.size, np.uint32)
        calls(50, o)  # the first call creates the context pool
        t0 = time.perf_counter()
        calls(reps, o)
        t1 = time.perf_counter()
        per = max(1, reps // nthreads)
        outs = [np.empty(a.size + b.size, np.uint32) for _ in range(nthreads)]
        th = [threading.Thread(target=calls, args=(per, outs[i])) for i in range(nthreads)]
        t2 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        t3 = time.perf_counter()
        # the oracle's merge (C: Go's foreach loop) on the same buffers, called
        # like the library (pointers, preallocated output)
        op = orc.DIFFERENCE if name == "difference" else orc.UNION
        ol, co = orc.lib(), np.empty(a.size + b.size + 1, np.uint32)
        ol.orc_setop(op, a.ctypes.data, a.size, b.ctypes.data, b.size, co.ctypes.data)
        t4 = time.perf_counter()
        for _ in range(reps):
            ol.orc_setop(op, a.ctypes.data, a.size, b.ctypes.data, b.size, co.ctypes.data)
        t5 = time.perf_counter()
        out[name] = {"us_per_call_1_thread": round((t1 - t0) / reps * 1e6, 2),
                     f"us_per_call_{nthreads}_threads": round((t3 - t2) / (per * nthreads) * 1e6, 2),
                     "calls_per_s_1_thread": reps / (t1 - t0),
                     f"calls_per_s_{nthreads}_threads": per * nthreads / (t3 - t2),
                     "cpu_oracle_us_per_call": round((t5 - t4) / reps * 1e6, 2)}
    L.syzcov_pool_trim()
    out["lists"] = f"|a| = {a.size}, |b| = {b.size} canonical PCs (95% of a plus 100 others)"
    out["note"] = ("one GPU round trip per call (2 H2D copies, a kernel, a D2H copy, a sync); "
                   "both timings include the ctypes call (~1 us). The "
                   "fuzzer's per-call checks belong on syzcov_newcov_batch / syzcov_state_triage "
                   "(INTEGRATION.md)")
    return out


def prio_run(args, world, rank, dev, dense: bool, steps: int, warmup: int):
    """K timed steps of CalculatePriorities over `args.inputs` synthetic
    programs per GPU: positional counts over the active keys (reference-exact,
    prio.go:142-150), or the dense contraction over all C keys (the MFMA GEMM
    over an AT in HBM).  Returns (seconds, phase ms, engine)."""
    import ctypes as C
    import torch
    from syzkaller_amd import _lib
    from syzkaller_amd.engine import PrioEngine
    L = _lib.lib()
    nprog = args.inputs
    eng = PrioEngine(nprog, device=dev, active_rows=not dense)
    lens = torch.empty(nprog, dtype=torch.int32, device=dev)
    _lib.check(L.syzcov_dev_synth_lens(SEED_PRIO, rank * nprog, nprog, 30, 8,
                                       C.c_void_p(lens.data_ptr()),
                                       C.c_void_p(torch.cuda.current_stream().cuda_stream)),
               "synth_lens")
    torch.cuda.synchronize()
    phases = list(eng.PHASES)
    reduce = None
    if world > 1:  # sharded by program: int32 SUM all-reduce of the counts
        from syzkaller_amd.dist import merge_counts
        reduce = merge_counts
    a = argparse.Namespace(steps=steps, warmup=warmup)
    dt, phl = timed(lambda ev: eng.step(lens, ev, reduce), len(phases), a, world, dev)
    return dt, dict(zip(phases, phl)), eng


def c4_subrecord(args, dev) -> dict:
    """Config C4 beside the corpus headline (N=1): CalculatePriorities over 1M
    programs, positional (the reference's semantics) and dense (all 1170 keys
    on i8 MFMA, the contraction north_star names), each with its MFMA roofline."""
    out = {"programs": args.inputs}
    for name, dense in (("positional", False), ("dense", True)):
        dt, ph, eng = prio_run(args, 1, 0, dev, dense, 10, 3)
        ops = eng.gemm_ops()
        ach = ops / (ph["gemm"] * 1e-3) / 1e12
        out[name] = {"ms_per_step": dt / 10 * 1e3, "phases_ms": {k: round(v, 4) for k, v in ph.items()},
                     "programs_per_s": args.inputs * 10 / dt,
                     "mfma_roofline": {"achieved": ach, "peak": I8_PEAK_TOPS, "unit": "TOPS",
                                       "frac": ach / I8_PEAK_TOPS, "mfma_ops_per_launch": ops,
                                       "tile": eng.tile if dense else 128}}
        del eng
    return out


def bench_prio(args):
    world, rank, dev = init_dist()
    nprog = args.inputs
    # default: positional counts over the active keys (reference-exact, prio.go:142-150);
    # --prio-dense: the full 1170-key contraction (the dense MFMA GEMM)
    dt, ph, eng = prio_run(args, world, rank, dev, args.prio_dense, args.steps, args.warmup)
    ops = eng.gemm_ops()
    achieved = ops / (ph["gemm"] * 1e-3) / 1e12
    out = {
        "metric": "programs/sec for CalculatePriorities (static + i8-MFMA AᵀA dynamic + normalize)",
        "value": nprog * world * args.steps / dt, "unit": "programs/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "i8",
        "data": "synthetic program lengths ~ N(30, 8) (SURVEY §8d C4)",
        "config": {"workload": "C4: CalculatePriorities, positional (reference-exact) keys"
                               + (", all C keys contracted" if args.prio_dense
                                  else f", active keys 0..{eng.max_len - 1}"),
                   "programs_per_gpu": nprog, "calls": eng.C,
                   "at_rows": eng.rows if args.prio_dense else -(-(eng.max_len + 1) // 128) * 128,
                   "at_cols": eng.ldp,
                   "parallelism": f"shard-by-program x{world}"
                                  + (", int32 SUM all-reduce of counts" if world > 1 else "")},
        "phases_ms": {k: round(v, 4) for k, v in ph.items()},
        "roofline": {"bound": "mfma", "kernel": "prio_gemm", "achieved": achieved,
                     "peak": I8_PEAK_TOPS, "unit": "TOPS", "frac": achieved / I8_PEAK_TOPS,
                     "traffic": None, "mfma_ops_per_launch": ops,
                     "algorithmic_ops_2NC2": 2 * nprog * eng.C * eng.C},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline_prio(min(nprog, 200_000), eng.C)
    return rank, world, out


def cpu_baseline_newcov(args, nrec: int, nhist: int = 16384):
    """Oracle (sequential fuzzer.go:456-480 loop: Difference x2 + Union per
    record, C restatement): `nhist` history records bring maxCover up
    (untimed), then the next `nrec` records are timed."""
    from oracle import oracle as orc
    import numpy as np
    orc.lib()
    off, pcs = orc.synth_corpus(SEED_NEWCOV, nhist + nrec, args.mean, args.sigma,
                                args.log2_space)
    c_off, c_pcs = orc.canonicalize_csr(off, pcs)
    recs = [c_pcs[c_off[i]:c_off[i + 1]] for i in range(nhist + nrec)]
    cids = orc.synth_callids(SEED_NEWCOV, nhist + nrec, args.ncalls)  # the GPU stream's first records
    fo, fp = orc.synth_corpus(SEED_NEWCOV, 1, 1 << (args.log2_space - 7), 1, args.log2_space,
                              first=FLAKE_INPUT)
    flakes = orc.canonicalize(fp[:int(fo[1])])
    _, mc = orc.newcov_batch([[] for _ in range(args.ncalls)], flakes, cids[:nhist],
                             recs[:nhist])
    t0 = time.perf_counter()
    orc.newcov_batch(mc, flakes, cids[nhist:], recs[nhist:])
    dt = time.perf_counter() - t0
    npc = int(c_off[-1] - c_off[nhist])
    return {"value": npc / dt, "unit": "record-PCs/s", "cores": 1, "kind": "port",
            "sample": f"{nrec} records ({npc} PCs) after {nhist} history records (untimed), "
                      f"sequential Difference/Difference/Union per record against per-call "
                      f"maxCover lists, oracle/ C restatement of syz-fuzzer/fuzzer.go:456-480, "
                      f"1 thread"}


def newcov_run(args, history, world, rank, dev):
    """One C5 measurement: `history` batches streamed through the check, then
    W + K fresh timed batches.  Returns (seconds, phase ms, timed PCs, candidates
    per batch, new records per batch, new records during the history)."""
    import ctypes as C
    import numpy as np
    import torch
    from syzkaller_amd import _lib
    from syzkaller_amd.engine import synth_corpus, synth_records, synth_window
    from syzkaller_amd.fuzzer import CoverState
    L = _lib.lib()
    s = lambda: C.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
    P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    lo, span = synth_window(args.log2_space)
    nrec, nb = args.records, args.warmup + args.steps

    def make_batch(b):
        # batch b of rank r's stream: records (r * (history + nb) + b) * nrec + k
        # (history batches first): the stream oracle/newcov_full.c restates
        first = (rank * (history + nb) + b) * nrec
        return synth_records(nrec, SEED_NEWCOV, first, args.ncalls, mean=args.mean,
                             sigma=args.sigma, log2_space=args.log2_space, device=dev)

    st = CoverState(args.ncalls, lo, span)
    if not args.no_universe:  # per-call bitmaps over the 2^22 dense keys
        univ = torch.empty(1 << args.log2_space, dtype=torch.int32, device=dev)
        _lib.check(L.syzcov_dev_synth_universe(SEED_NEWCOV, args.log2_space, P(univ), s()),
                   "synth_universe")
        st.set_universe(univ.cpu().numpy().view(np.uint32))
        del univ
    # flakes: one synthetic draw from the same universe (input index 2^40)
    fo, fp, _, _ = synth_corpus(1, SEED_NEWCOV, first=FLAKE_INPUT, mean=1 << (args.log2_space - 7),
                                sigma=1, log2_space=args.log2_space, device=dev)
    st.set_flakes(np.unique(fp[:int(fo[1].item())].cpu().numpy().view(np.uint32)))
    # a fuzzer that has been running: `history` batches streamed through the
    # same check before the bench (maxCover near saturation after 512)
    hist_new = 0
    for h in range(history):
        cid, roff, pcs, npc = make_batch(h)
        wsz = L.syzcov_state_newcov_ws_size(nrec, npc)
        ws = torch.empty(wsz, dtype=torch.uint8, device=dev)
        flags = torch.zeros(nrec, dtype=torch.uint8, device=dev)
        _lib.check(L.syzcov_state_newcov_dev(st.h, P(cid), P(roff), P(pcs), nrec, npc, P(flags),
                                             None, P(ws), wsz, s()), "state_newcov_dev")
        hist_new += int(flags.sum().item())
        del ws, pcs
    batches = [make_batch(history + b) for b in range(nb)]
    max_npc = max(b[3] for b in batches)
    wsz = L.syzcov_state_newcov_ws_size(nrec, max_npc)
    ws = torch.empty(wsz, dtype=torch.uint8, device=dev)
    is_new = torch.zeros(nb, nrec, dtype=torch.uint8, device=dev)  # counted after the timing
    stats = torch.zeros(nb, 2, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    it = [0]

    def run_step(ev):
        b = it[0]
        cid, roff, pcs, npc = batches[b]
        if ev is not None:
            ev[0].record()
        _lib.check(L.syzcov_state_newcov_dev(st.h, P(cid), P(roff), P(pcs), nrec, npc,
                                             P(is_new[b]), P(stats[b]), P(ws), wsz, s()),
                   "state_newcov_dev")
        if ev is not None:
            ev[1].record()
        it[0] += 1
    dt, phl = timed(run_step, 1, args, world, dev)
    sc = stats.cpu().tolist()
    if any(x[0] for x in sc):
        raise RuntimeError(f"newcov batch rejected: {sc}")
    nnew = is_new.sum(dim=1).cpu().tolist()
    timed_pcs = sum(b[3] for b in batches[args.warmup:])
    st.close()
    return dt, phl, timed_pcs, [x[1] for x in sc[args.warmup:]], nnew[args.warmup:], hist_new


def bench_newcov(args):
    """C5: streaming new-coverage check (syz-fuzzer execute, fuzzer.go:456-480)
    of batches of call records against the resident per-CallID maxCover and
    the global flakes set.  Every step is a FRESH batch (W + K distinct batches
    are generated into HBM up front), so maxCover evolves as in a fuzzer.  At
    N=1 with the default 512 history batches (the steady state, maxCover near
    saturation) the line also carries the early regime (32 history batches:
    every record still brings new PCs) as the `early` sub-record."""
    world, rank, dev = init_dist()
    nrec = args.records
    dt, phl, timed_pcs, cands, nnew, hist_new = newcov_run(args, args.history, world, rank, dev)
    value = timed_pcs * world / dt
    achieved = timed_pcs / args.steps * 4 / (phl[0] * 1e-3) / 1e9
    out = {
        "metric": "record-PCs checked/sec, streaming new-coverage check (fuzzer.go:456-480)",
        "value": value, "unit": "record-PCs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic canonical call records (SURVEY §8d C5), fresh batch every step",
        "config": {"workload": f"C5: {nrec} call records per batch vs resident maxCover",
                   "records_per_batch": nrec, "calls": args.ncalls,
                   "pcs_per_batch": timed_pcs // args.steps, "pc_space": 1 << args.log2_space,
                   "flakes": f"unique PCs of one synthetic {1 << (args.log2_space - 7)}-PC draw",
                   "maxcover": ("bitmaps over the dense keys of the synthetic 2^%d-PC "
                                "universe" % args.log2_space if not args.no_universe
                                else "window bitmaps (1 bit per PC offset)"),
                   "maxcover_bytes": args.ncalls * ((1 << args.log2_space) if not args.no_universe
                                                    else (16 << args.log2_space)) // 8,
                   "history_batches": args.history, "history_new_records": hist_new},
        "phases_ms": {"newcov": round(phl[0], 4)},
        "results": {"candidates_per_batch": cands, "new_records_per_batch": nnew,
                    "records_per_s": nrec * args.steps * world / dt},
        "roofline": {"bound": "hbm", "kernel": "newcov (split + fused check + hash)",
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "alg_bytes_per_launch": timed_pcs // args.steps * 4},
    }
    if world == 1 and args.history == 512:  # per timed batch of this command's shape
        out["roofline"]["traffic"], out["roofline"]["traffic_source"] = traffic_of("newcov",
                                                                                   "newcov")
    if world == 1 and args.history == 512 and not args.no_early:
        # the early regime (the fuzzer's first minutes), same batch shape
        e_dt, e_phl, e_pcs, e_cands, e_new, e_hist = newcov_run(args, 32, world, rank, dev)
        e_ach = e_pcs / args.steps * 4 / (e_phl[0] * 1e-3) / 1e9
        out["early"] = {
            "history_batches": 32, "history_new_records": e_hist,
            "value": e_pcs / e_dt, "ms_per_step": e_dt / args.steps * 1e3,
            "phases_ms": {"newcov": round(e_phl[0], 4)},
            "results": {"candidates_per_batch": e_cands, "new_records_per_batch": e_new},
            "roofline": {"achieved": e_ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": e_ach / HBM_PEAK_GBS,
                         "traffic": traffic_of("newcov_early", "newcov")[0],
                         "alg_bytes_per_launch": e_pcs // args.steps * 4}}
    if rank == 0 and world == 1 and not args.no_cpu and args.cpu_sample > 0:
        out["cpu_baseline"] = cpu_baseline_newcov(args, min(args.cpu_sample, 2000, nrec))
    return rank, world, out


def cpu_baseline_dedup(bufs) -> dict:
    """Oracle cover_dedup (executor.cc:574-587 restated in C: qsort + the
    `last` loop) over a sample of the same buffers, 1 thread."""
    from oracle import oracle as orc
    orc.lib()
    t0 = time.perf_counter()
    npc = 0
    for b in bufs:
        orc.cover_dedup64(b)
        npc += b.size
    dt = time.perf_counter() - t0
    return {"value": npc / dt, "unit": "raw-PCs/s", "cores": 1, "kind": "port",
            "sample": f"{len(bufs)} buffers ({npc} raw u64 PCs) of the timed batch, "
                      f"oracle/ C restatement of executor/executor.cc:574-587 (qsort), 1 thread"}


def bench_dedup(args):
    """The executor's cover_dedup (executor/executor.cc:574-587) on the GPU:
    batches of raw u64 KCOV buffers (the C2 generator's raw PCs as x86-64
    kernel addresses 0xffffffff_xxxxxxxx, lengths ~ N(mean, sigma)) deduped in
    place, with the u32 words executor.cc:459-463 writes.  Every step is a
    FRESH batch (W + K batches generated into HBM up front)."""
    import ctypes as C
    import torch
    world, rank, dev = init_dist()
    from syzkaller_amd import _lib
    from syzkaller_amd.engine import synth_corpus
    L = _lib.lib()
    s = lambda: C.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
    P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    nbuf, nb = args.records, args.warmup + args.steps
    batches = []
    for b in range(nb):
        off, raw, _, total = synth_corpus(nbuf, SEED_DEDUP, first=(rank * nb + b) * nbuf,
                                          mean=args.mean, sigma=args.sigma,
                                          log2_space=args.log2_space, device=dev)
        pcs = raw[:total].to(torch.int64) | (-(1 << 32))
        del raw
        batches.append((off, pcs, total))
    o32 = torch.empty(max(b[2] for b in batches), dtype=torch.int32, device=dev)
    nl = torch.empty(nb, nbuf, dtype=torch.int32, device=dev)
    ns = min(nbuf, 20000)  # the CPU baseline's sample: the last batch's first buffers
    soff = batches[-1][0][:ns + 1].cpu().numpy()
    spcs = batches[-1][1][:int(soff[-1])].cpu().numpy().view("uint64")
    sample = [spcs[soff[i]:soff[i + 1]].copy() for i in range(ns)]
    torch.cuda.synchronize()
    it = [0]

    def run_step(ev):
        b = it[0]
        off, pcs, _ = batches[b]
        if ev is not None:
            ev[0].record()
        _lib.check(L.syzcov_dev_cover_dedup64(P(pcs), P(off), nbuf, P(nl[b]), P(o32), s()),
                   "dev_cover_dedup64")
        if ev is not None:
            ev[1].record()
        it[0] += 1
    dt, phl = timed(run_step, 1, args, world, dev)
    kept = nl[args.warmup:].to(torch.int64).sum(1).cpu().tolist()
    if nl[args.warmup:].min().item() < 0:  # a wide/malformed mark left behind
        raise RuntimeError("dedup: a buffer was left unprocessed")
    raw_t = sum(b[2] for b in batches[args.warmup:])
    alg = (8 * raw_t + 12 * sum(kept)) / args.steps  # read u64 + write u64 and the u32 word
    achieved = alg / (phl[0] * 1e-3) / 1e9
    out = {
        "metric": "raw KCOV PCs deduped/sec (executor cover_dedup, executor.cc:574-587)",
        "value": raw_t * world / dt, "unit": "raw-PCs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic raw KCOV buffers (C2 lengths, x86-64 kernel addresses), fresh batch "
                "every step",
        "config": {"workload": f"cover_dedup: {nbuf} raw u64 KCOV buffers per batch",
                   "buffers_per_batch": nbuf, "raw_pcs_per_batch": raw_t // args.steps,
                   "len_mean": args.mean, "len_sigma": args.sigma,
                   "parallelism": f"shard-by-buffer x{world}"},
        "phases_ms": {"dedup": round(phl[0], 4)},
        "results": {"kept_per_batch": kept},
        "roofline": {"bound": "hbm", "kernel": "dedup (narrow<4,8,16> + wide)",
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "alg_bytes_per_launch": alg},
    }
    if world == 1:  # per timed batch of this command's shape
        out["roofline"]["traffic"], out["roofline"]["traffic_source"] = traffic_of("dedup", "dedup")
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline_dedup(sample)
    return rank, world, out


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: running {world} ranks",
              file=sys.stderr)
    fn = {"prio": bench_prio, "newcov": bench_newcov, "dedup": bench_dedup}.get(args.workload,
                                                                             bench_corpus)
    rank, world, out = (bench_dry if args.dry_run else fn)(args)
    if world > 1:
        import torch.distributed as dist
        # the ranks the collectives actually ran over, and their backend
        out["rccl_ranks"] = dist.get_world_size()
        out["backend"] = dist.get_backend()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
