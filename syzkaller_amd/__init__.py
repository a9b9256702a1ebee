"""syzkaller_amd — MI355X-native coverage-analysis engine for syzkaller.

The hot path of syzkaller's manager and fuzzer (the `cover` set algebra,
corpus Minimize, the maxCover/corpusCover merges and prog.CalculatePriorities)
as hand-written HIP kernels for gfx950 behind a C-ABI (include/syzcov.h,
libsyzcov.so).  Python modules mirror the reference's Go API:

    syzkaller_amd.cover   — cover/cover.go
    syzkaller_amd.prio    — prog/prio.go (CalculatePriorities, BuildChoiceTable)
    syzkaller_amd.fuzzer  — syz-fuzzer execute()'s new-coverage check
    syzkaller_amd.engine  — device-resident corpus pipeline (torch tensors)
    syzkaller_amd.dist    — the same pipeline sharded over GPUs (RCCL)
"""
from ._lib import LIB_PATH, SyzcovError, build, lib  # noqa: F401

__all__ = ["LIB_PATH", "SyzcovError", "build", "lib"]
