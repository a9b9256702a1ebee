#!/usr/bin/env python3
"""Kernel micro-bench on the C2 corpus: times one engine phase at a time.
    python tools/kbench.py canon|minimize|step|order|dedup|groups [--keys] [--inputs N] [--reps R]
groups: syzcov_minimize_corpus (293 call groups) and syzcov_minimize from host
buffers of the C2 corpus, wall time per call.
dedup: the executor's cover_dedup (executor.cc:574-587) over N raw u64 KCOV
buffers made of the C2 generator's raw PCs (high half 0xffffffff), in place,
with the u32 output words; the buffers are restored outside the events."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from syzkaller_amd.engine import (CorpusEngine, synth_corpus, synth_universe,  # noqa: E402
                                  synth_window)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", nargs="?", default="canon")
    ap.add_argument("--inputs", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--mean", type=int, default=2048)
    ap.add_argument("--sigma", type=int, default=512)
    ap.add_argument("--log2-space", type=int, default=22)
    ap.add_argument("--keys", action="store_true", help="key mode (the synthetic PC universe)")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    n = a.inputs
    if a.what == "order":  # Go sort.Sort order over n synthetic lengths only
        import ctypes as C
        from syzkaller_amd._lib import check, lib
        L = lib()
        lens = torch.empty(n, dtype=torch.int32, device="cuda")
        check(L.syzcov_dev_synth_lens(0x5EED0002, 0, n, a.mean, a.sigma, C.c_void_p(lens.data_ptr()),
                                      C.c_void_p(torch.cuda.current_stream().cuda_stream)), "synth")
        lo, span = synth_window(a.log2_space)
        eng = CorpusEngine(n, 1, 1, lo, span)
        for _ in range(a.reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            eng.sort_order(lens, n)
            e.record()
            torch.cuda.synchronize()
            print(f"order: {s.elapsed_time(e):.3f} ms  n={n}", flush=True)
        return
    if a.what == "groups":  # Manager.minimizeCorpus drop-in from host buffers (C2 + call ids)
        import ctypes as C
        import numpy as np
        from syzkaller_amd._lib import check, lib
        L = lib()
        off, raw, lens, total = synth_corpus(n, 0x5EED0002, mean=a.mean, sigma=a.sigma,
                                             log2_space=a.log2_space)
        h_off = off.cpu().numpy().astype(np.uint64)
        h_pcs = raw[:total].cpu().numpy().view(np.uint32)
        cid = torch.empty(n, dtype=torch.int32, device="cuda")
        check(L.syzcov_dev_synth_callids(0x5EED0002, 0, n, 293, C.c_void_p(cid.data_ptr()),
                                         C.c_void_p(torch.cuda.current_stream().cuda_stream)),
              "synth_callids")
        calls = cid.cpu().numpy()
        del off, raw, lens, cid
        torch.cuda.empty_cache()
        out = np.empty(n, np.int32)
        for r in range(a.reps + 1):
            t0 = time.perf_counter()
            k = check(L.syzcov_minimize_corpus(calls.ctypes.data, h_off.ctypes.data,
                                               h_pcs.ctypes.data, n, 0, out.ctypes.data),
                      "minimize_corpus")
            t1 = time.perf_counter()
            k1 = check(L.syzcov_minimize(h_off.ctypes.data, h_pcs.ctypes.data, n, None, 0,
                                         out.ctypes.data), "minimize")
            t2 = time.perf_counter()
            print(f"groups: minimize_corpus {1e3 * (t1 - t0):.1f} ms (kept {k}), "
                  f"minimize {1e3 * (t2 - t1):.1f} ms (kept {k1})", flush=True)
        return
    if a.what == "dedup":
        import ctypes as C
        from syzkaller_amd._lib import check, lib
        off, raw, lens, total = synth_corpus(n, 0x5EED0002, mean=a.mean, sigma=a.sigma,
                                             log2_space=a.log2_space)
        src = raw[:total].to(torch.int64) | (-(1 << 32))  # 0xffffffff_xxxxxxxx
        buf = torch.empty_like(src)
        o32 = torch.empty(total, dtype=torch.int32, device="cuda")
        nl = torch.empty(n, dtype=torch.int32, device="cuda")
        del raw
        st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
        for r in range(a.reps + 1):
            buf.copy_(src)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            check(lib().syzcov_dev_cover_dedup64(P(buf), P(off), n, P(nl), P(o32), st), "dedup")
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e)
            kept = int(nl.to(torch.int64).sum().item())
            if r:
                print(f"dedup: {ms:.3f} ms  raw {total} u64 PCs in {n} buffers, kept {kept}  "
                      f"{total / ms / 1e6:.2f} G PCs/s  {(8 * total + 12 * kept) / ms / 1e6:.1f} GB/s "
                      f"(8 B read per PC + 12 B written per kept PC)", flush=True)
        return
    lo, span = synth_window(a.log2_space)
    off, raw, lens, total = synth_corpus(n, 0x5EED0002, mean=a.mean, sigma=a.sigma,
                                         log2_space=a.log2_space)
    univ = synth_universe(a.log2_space, 0x5EED0002) if a.keys else None
    eng = CorpusEngine(n, total, int(lens.max().item()), lo, span, universe=univ)
    if a.what == "canon":  # canon alone (experimental builds may not order correctly)
        eng.canonicalize(off, raw, n)
    else:
        eng.step(off, raw, n)
    torch.cuda.synchronize()
    fns = {
        "canon": lambda: eng.canonicalize(off, raw, n),
        "minimize": lambda: (eng.sort_order(None, n), eng.minimize()),
        "step": lambda: eng.step(off, raw, n, sync=False),
    }
    f = fns[a.what]
    if a.what == "minimize":  # minimize alone (the order outside the events)
        canon_pcs = int(eng.new_len[:n].to(torch.int64).sum().item())
        for _ in range(a.reps):
            eng.sort_order(None, n)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            eng.minimize()
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e)
            print(f"minimize: {ms:.3f} ms  canonical {canon_pcs} PCs  nrange {eng.nrange}  "
                  f"{4 * canon_pcs / ms / 1e6:.1f} GB/s (4 B/PC)", flush=True)
        return
    for _ in range(a.reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        f()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e)
        print(f"{a.what}: {ms:.3f} ms  raw {total} PCs  {8 * total / ms / 1e6:.1f} GB/s (8 B/PC)",
              flush=True)


if __name__ == "__main__":
    main()
