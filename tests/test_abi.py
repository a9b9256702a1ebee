"""C-ABI library checks that need no GPU: it builds, loads, and exports every
symbol include/syzcov.h declares (no compute calls here)."""
import ctypes
import os
import subprocess

import pytest

from syzkaller_amd import _lib


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    declared = _lib.header_symbols()
    assert len(declared) >= 40
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing


def test_ctypes_signatures_cover_the_header():
    assert sorted(_lib._SIGS) == _lib.header_symbols()


def test_version_and_pure_helpers():
    L = _lib.lib()
    assert L.syzcov_version().decode().endswith("gfx950")
    # RestorePC is pure host arithmetic (cover.go:23-25)
    assert L.syzcov_restore_pc(0x1234, 0xffffffff) == (0xffffffff << 32) + 0x1234
    assert L.syzcov_dev_prio_rows(1170) == 1280
    assert L.syzcov_dev_prio_ldp(1000) == 1024


def test_no_oracle_in_product():
    """The product package never imports or links the test oracle."""
    root = os.path.dirname(_lib._HERE)
    import re
    bad = re.compile(r"^\s*(import\s+oracle|from\s+oracle|#\s*include\s*[<\"].*oracle)", re.M)
    for dirpath, _, files in os.walk(_lib._HERE):
        for f in files:
            if f.endswith((".py", ".hip", ".cc", ".h", "Makefile")):
                txt = open(os.path.join(dirpath, f)).read()
                assert not bad.search(txt), f
                assert "liboracle" not in txt, f
    out = subprocess.run(["ldd", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "liboracle" not in out
    assert os.path.exists(os.path.join(root, "oracle", "oracle.h"))


def test_gfx950_code_object_present(tmp_path):
    # (--offloading writes the extracted code objects next to its input: a copy
    # in a scratch directory keeps them out of the package)
    import shutil
    lib = shutil.copy(_lib.LIB_PATH, tmp_path / "libsyzcov.so")
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib)],
                         capture_output=True, text=True, cwd=tmp_path)
    txt = out.stdout + out.stderr
    assert "gfx950" in txt
