#!/usr/bin/env python3
"""C3 (10M inputs, key mode, canonicalized in place) one phase at a time, with
a device synchronisation and consistency checks after each phase, so a fault
or a bad intermediate names its phase.  usage: tools/diag_c3.py [n] [window]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from syzkaller_amd.engine import CorpusEngine, synth_corpus, synth_universe, synth_window  # noqa

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
keys = not (len(sys.argv) > 2 and sys.argv[2] == "window")
seed = 0x5EED0003
t0 = time.time()


def log(*a):
    print(f"[{time.time() - t0:7.1f}s]", *a, flush=True)


off, raw, lens, total = synth_corpus(n, seed)
lo, span = synth_window(22)
univ = synth_universe(22, seed) if keys else None
eng = CorpusEngine(n, total, int(lens.max().item()), lo, span, canon_in_place=True, universe=univ)
log("corpus", n, "inputs", total, "raw PCs, max len", int(lens.max().item()), "key mode", keys)
eng.canonicalize(off, raw, n)
torch.cuda.synchronize()
log("canon ok, err flags", int(eng.scal[0].item()))
nl = eng.new_len[:n].to(torch.int64)
assert bool((nl <= lens.to(torch.int64)).all()) and bool((nl > 0).all())
# canonical keys: sorted, < span, per segment (chunks of 256k inputs)
bad = 0
CH = 1 << 17
for a in range(0, n, CH):
    b = min(n, a + CH)
    st = off[a:b]
    ln = nl[a:b]
    tot = int(ln.sum().item())
    seg = torch.repeat_interleave(torch.arange(b - a, device="cuda"), ln)
    pos = torch.arange(tot, device="cuda", dtype=torch.int64)
    cs = torch.zeros(b - a + 1, dtype=torch.int64, device="cuda")
    torch.cumsum(ln, 0, out=cs[1:])
    idx = st[seg] + (pos - cs[seg])
    v = raw[idx].to(torch.int64) & 0xFFFFFFFF
    oob = v >= eng.span
    first = pos == cs[seg]
    unsorted = torch.zeros_like(oob)
    unsorted[1:] = (v[1:] <= v[:-1]) & ~first[1:]
    if bool(oob.any()) or bool(unsorted.any()):
        bad += 1
        i = int(torch.nonzero(oob | unsorted)[0].item())
        log(f"BAD chunk {a}: oob {int(oob.sum())} unsorted {int(unsorted.sum())} first at seg "
            f"{a + int(seg[i])} value {int(v[i]):#x}")
        if bad > 3:
            sys.exit(1)
    if eng.split is not None:
        sp = eng.split.view(n, eng.nrange)[a:b].to(torch.int64)
        if not bool((sp[:, -1] == ln).all()) or not bool((sp[:, 1:] >= sp[:, :-1]).all()):
            log(f"BAD split columns in chunk {a}")
            sys.exit(1)
    del seg, pos, idx, v
log("canonical keys checked, bad chunks", bad)
if bad:
    sys.exit(1)
eng.minimize_clear(n)
eng.sort_order(eng.new_len, n)
torch.cuda.synchronize()
o = eng.order[:n].to(torch.int64)
assert bool((torch.sort(o).values == torch.arange(n, device="cuda")).all()), "order not a permutation"
log("order ok (permutation)")
log("range_tot", eng.range_tot.tolist())
eng.minimize(off, eng.order, None, n, cleared=True)
torch.cuda.synchronize()
log("minimize ok, records", int(eng.rec_cnt.item()), "cap", eng.rec_cap)
eng.compact(n)
eng.build_dict()
eng.union_list()
eng.merge_max_cover()
res = eng.result()
log("step ok: kept", res.n_kept, "union", res.n_union)
