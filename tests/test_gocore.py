"""The sequential pdqsort core shared by the device sort (gosort_core.h),
built for the host with g++, against the oracle's Go sort.Sort restatement."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as orc

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def core(tmp_path_factory):
    out = tmp_path_factory.mktemp("gocore") / "libgocore.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", str(out),
                    os.path.join(HERE, "native", "gocore_host.cc")], check=True)
    lib = C.CDLL(str(out))
    lib.gocore_sort.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    return lib


def test_core_matches_go_sort(core):
    rng = np.random.default_rng(21)
    for trial in range(600):
        # every other trial a leaf-sized input (<= 64: the register BitStack)
        n = int(rng.integers(0, 5000)) if trial % 2 else int(rng.integers(0, 65))
        kind = trial % 5
        lens = (rng.integers(0, 6, size=n) if kind == 0 else
                rng.integers(0, 1 << 20, size=n) if kind == 1 else
                np.sort(rng.integers(0, 40, size=n)) if kind == 2 else
                np.sort(rng.integers(0, 40, size=n))[::-1].copy() if kind == 3 else
                rng.normal(2048, 512, size=n).astype(np.int64))
        lens = np.ascontiguousarray(lens, dtype=np.int64)
        idx = np.empty(max(n, 1), dtype=np.int32)
        core.gocore_sort(lens.ctypes.data, n, idx.ctypes.data)
        assert np.array_equal(idx[:n], orc.sort_order(lens)), (trial, n, kind)
