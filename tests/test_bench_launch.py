"""bench.py --gpus N starts its own N ranks when no torch.distributed
launcher did (the driver's `python bench.py --gpus 8`): one JSON line from
rank 0 carrying the world the ranks formed, and a failing rank ends the run
instead of leaving its peers in a collective."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_launcher_forms_world():
    for n in (2, 3):
        r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--dry-run"],
                           capture_output=True, text=True, timeout=120, env=_env())
        assert r.returncode == 0, r.stderr[-2000:]
        # stdout is the one JSON line and nothing else (gloo's connection
        # notes from every rank go to stderr)
        lines = r.stdout.splitlines()
        assert len(lines) == 1 and lines[0].startswith("{"), r.stdout
        d = json.loads(lines[0])
        assert d["n_gpus"] == n and d["rccl_ranks"] == n, d


def test_single_rank_unchanged():
    r = subprocess.run([sys.executable, BENCH, "--dry-run"], capture_output=True, text=True,
                       timeout=120, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 1 and d["rccl_ranks"] == 1 and d["backend"] is None


def test_failing_ranks_end_the_run():
    # without a GPU every rank of the real workload fails at device setup: the
    # launcher must return their error, not hang
    env = _env()
    env["HIP_VISIBLE_DEVICES"] = ""  # no device even on a GPU host
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_same_workload_at_every_n(monkeypatch):
    """The driver builds its 1 -> 8 curve from `value` at each N: the N=1 line
    must name the same workload (C3, 10M inputs) as the N>1 lines."""
    sys.path.insert(0, ROOT)
    import bench
    seen = {}

    def fake_run(args, world, rank, dev, glob, seed, steps, warmup, key, x86=False):
        seen.update(glob=glob, seed=seed, key=key)
        return {"value": 1.0, "ms_per_step": 1.0, "inputs_per_gpu": glob, "raw_pcs_per_gpu": 0,
                "aligned": True,
                "canonical_pcs_per_gpu": 0, "keys": "", "phases_ms": {},
                "roofline": {"achieved": 1.0}, "minimize_union_pcs_per_s": 1.0}
    monkeypatch.setattr(bench, "init_dist", lambda: (1, 0, None))
    monkeypatch.setattr(bench, "corpus_run", fake_run)
    monkeypatch.setattr(bench, "stream_peak", lambda dev: {"flat_float4": 1.0})
    monkeypatch.setattr(bench, "rank_share_run", lambda *a, **k: {"ms_per_step": 1.0})
    monkeypatch.setattr(sys, "argv", ["bench.py", "--no-c2", "--no-dropin", "--no-cpu"])
    _, _, one = bench.bench_corpus(bench.parse())
    assert seen == {"glob": bench.C3_INPUTS, "seed": bench.SEED_C3, "key": "C3"}
    lines = {}
    for n in (1, 2):
        r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--dry-run"],
                           capture_output=True, text=True, timeout=120, env=_env())
        assert r.returncode == 0, r.stderr[-2000:]
        lines[n] = json.loads(r.stdout.strip().splitlines()[-1])
    assert one["config"]["workload"] == lines[1]["config"]["workload"] \
        == lines[2]["config"]["workload"], (one["config"], lines)
    assert one["config"]["workload"].startswith("C3: ") and one["scaling"] == "strong"
    assert "c3_rank_of_8" in one  # the 8-GPU step's per-rank share, measured at N=1
