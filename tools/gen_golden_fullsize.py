#!/usr/bin/env python3
"""Generate tests/golden/fullsize_digests.json: the CPU oracle's results on the
full-size synthetic corpora of BASELINE.json's configs, as
digests the GPU tests compare the engine against.

  C1  10k inputs   seed 0x5EED0001   (CPU-only config)
  C2  1M inputs    seed 0x5EED0002   (one MI355X; also the world-8 rehearsal)
  C3  10M inputs   seed 0x5EED0003   (the 8-GPU config; 82 GB of raw PCs)
  C2X C2 over the x86-like universe (PCs 5..14 bytes apart: kshift 2, 2^23 keys)
  C5S the same stream over 514 batches (512 history, steady state)
  C2G Manager.minimizeCorpus over C2's RAW covers in 293 call groups
      (synthetic call ids; oracle/grouped_full.c): the kept corpus indices
  C2R cover.Minimize over C2's RAW covers (one group: order by raw lengths,
      what the drop-in syzcov_minimize computes from host buffers)
  C5  34 batches of 65,536 call records, seed 0x5EED0005, 293 calls: the
      fuzzer's new-coverage check (oracle/newcov_full.c), per-batch is_new
      flags and the final per-call maxCover (the bench's stream: 32 history
      batches, then the batches it times)

Each run is oracle/build/fullsize (oracle/fullsize.c): the reference's
Canonicalize + sort.Sort + Minimize loop + Union fold, restated so the corpus
is regenerated instead of held in memory.  TEST INFRASTRUCTURE: run once in
the build container (C3 takes ~15 min on 8 threads); the digests are data.

usage: python tools/gen_golden_fullsize.py [C1 C2 C3 ...]
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "golden", "fullsize_digests.json")
CONFIGS = {
    "C1": dict(seed=0x5EED0001, n=10_000),
    "C2": dict(seed=0x5EED0002, n=1_000_000),
    "C3": dict(seed=0x5EED0003, n=10_000_000),
    # C2 over the x86-like universe: 2^22 PCs 5..14 bytes apart, so kshift 2
    # and 2^23 keys (synth mode bit 1)
    "C2X": dict(seed=0x5EED0002, n=1_000_000, mode=2),
}
MEAN, SIGMA, LOG2 = 2048, 512, 22
C5 = dict(seed=0x5EED0005, records=65536, batches=34, ncalls=293)
# C5 in steady state: 512 history batches (maxCover near saturation: new
# coverage is rare, as in a long-running fuzzer), then the bench's 2 batches;
# per-batch digests only for the last 2 (counts for all)
C5S = dict(C5, batches=514, digest_last=2)


def sha(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 24), b""):
            h.update(blk)
    return h.hexdigest()


def run(name: str, threads: int) -> dict:
    cfg = CONFIGS[name]
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    exe = os.path.join(ROOT, "oracle", "build", "fullsize")
    with tempfile.TemporaryDirectory() as d:
        t0 = time.time()
        r = subprocess.run([exe, hex(cfg["seed"]), str(cfg["n"]), str(MEAN), str(SIGMA), str(LOG2),
                            str(threads), d, str(cfg.get("mode", 0))], check=True,
                           capture_output=True, text=True)
        summary = json.loads(r.stdout)
        kept = np.fromfile(os.path.join(d, "kept.i32"), dtype=np.int32)
        union = np.fromfile(os.path.join(d, "union.u32"), dtype=np.uint32)
        out = dict(seed=cfg["seed"], n=cfg["n"], mean=MEAN, sigma=SIGMA, log2_space=LOG2,
                   synth_mode=cfg.get("mode", 0),
                   raw_pcs=summary["raw_pcs"], canonical_pcs=summary["canonical_pcs"],
                   n_kept=summary["n_kept"], kept_sha256=sha(os.path.join(d, "kept.i32")),
                   kept_head=kept[:16].tolist(), kept_tail=kept[-16:].tolist(),
                   n_union=summary["n_union"], union_sha256=sha(os.path.join(d, "union.u32")),
                   union_head=union[:4].tolist(), union_tail=union[-4:].tolist(),
                   order_sha256=sha(os.path.join(d, "order.i32")),
                   lens_sha256=sha(os.path.join(d, "lens.u32")),
                   sort="pdqsort (Go >= 1.19)", oracle_seconds=round(time.time() - t0, 1),
                   oracle_threads=threads)
    return out


GROUPED = {"C2G": dict(seed=0x5EED0002, n=1_000_000, ncalls=293),
           "C2R": dict(seed=0x5EED0002, n=1_000_000, ncalls=1)}


def run_grouped(name: str) -> dict:
    g = GROUPED[name]
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    exe = os.path.join(ROOT, "oracle", "build", "grouped_full")
    with tempfile.TemporaryDirectory() as d:
        t0 = time.time()
        out = os.path.join(d, "kept.i32")
        r = subprocess.run([exe, hex(g["seed"]), str(g["n"]), str(MEAN), str(SIGMA), str(LOG2),
                            str(g["ncalls"]), out], check=True, capture_output=True, text=True)
        summary = json.loads(r.stdout)
        kept = np.fromfile(out, dtype=np.int32)
        return dict(seed=g["seed"], n=g["n"], ncalls=g["ncalls"], mean=MEAN, sigma=SIGMA,
                    log2_space=LOG2, raw_pcs=summary["raw_pcs"], n_kept=summary["n_kept"],
                    kept_sha256=sha(out), kept_head=kept[:16].tolist(),
                    kept_tail=kept[-16:].tolist(), covers="raw (duplicates count in len)",
                    groups="orc_synth_callid(seed, i, ncalls), ascending call id",
                    sort="pdqsort (Go >= 1.19)", oracle_seconds=round(time.time() - t0, 1))


def run_c5(threads: int, c: dict = C5) -> dict:
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    exe = os.path.join(ROOT, "oracle", "build", "newcov_full")
    with tempfile.TemporaryDirectory() as d:
        t0 = time.time()
        r = subprocess.run([exe, hex(c["seed"]), str(c["records"]), str(c["batches"]),
                            str(c["ncalls"]), str(MEAN), str(SIGMA), str(LOG2), str(threads), d],
                           check=True, capture_output=True, text=True)
        summary = json.loads(r.stdout)
        is_new = np.fromfile(os.path.join(d, "is_new.u8"), dtype=np.uint8)
        is_new = is_new.reshape(c["batches"], c["records"])
        return dict(seed=c["seed"], records=c["records"], batches=c["batches"],
                    ncalls=c["ncalls"], mean=MEAN, sigma=SIGMA, log2_space=LOG2,
                    record_pcs=summary["record_pcs"],
                    new_per_batch=[int(x) for x in is_new.sum(axis=1)],
                    is_new_sha256=[hashlib.sha256(row.tobytes()).hexdigest()
                                   for row in is_new[-c.get("digest_last", c["batches"]):]],
                    is_new_sha256_first_batch=c["batches"] - c.get("digest_last", c["batches"]),
                    max_cover_total=summary["max_cover_total"],
                    max_cover_n_sha256=sha(os.path.join(d, "maxcover_n.u32")),
                    max_cover_sha256=sha(os.path.join(d, "maxcover.u32")),
                    flakes="unique PCs of synthetic input 2^40, length 2^(log2-7)",
                    oracle_seconds=round(time.time() - t0, 1), oracle_threads=threads)


def main():
    names = sys.argv[1:] or list(CONFIGS)
    data = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            data = json.load(f)
    data["_about"] = ("CPU oracle digests (oracle/fullsize.c via tools/gen_golden_fullsize.py) of "
                      "Canonicalize + Minimize + Union over the synthetic corpora of SURVEY §8d: "
                      "kept = original indices in processing order (int32 LE), union = sorted "
                      "PCs (uint32 LE), order = Go sort.Sort processing order over the canonical "
                      "lengths, lens = canonical lengths (uint32 LE)")
    for name in names:
        print(f"{name} ...", flush=True)
        nt = int(os.environ.get("ORACLE_THREADS", os.cpu_count() or 8))
        if name in ("C5", "C5S"):
            data[name] = run_c5(nt, C5 if name == "C5" else C5S)
        elif name in GROUPED:
            data[name] = run_grouped(name)
        else:
            data[name] = run(name, nt)
        print(json.dumps(data[name]), flush=True)
        with open(OUT, "w") as f:
            json.dump(data, f, indent=1)


if __name__ == "__main__":
    main()
