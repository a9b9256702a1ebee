"""ctypes binding of libsyzcov.so (include/syzcov.h).

The product path has no CPU implementation: if the library is missing this
module raises, and every compute entry point returns SYZCOV_ENODEV without a
HIP device (raised as SyzcovError here)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
# SYZCOV_LIB: a variant build for tuning sweeps (tools/); default is the in-tree library
LIB_PATH = os.environ.get("SYZCOV_LIB") or os.path.join(_HERE, "libsyzcov.so")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "syzcov.h")

OK, EINVAL, ENOTSORTED, ENODEV, EHIP, ERANGE, ENOMEM, ETOOLONG = 0, -1, -2, -3, -4, -5, -6, -7
_NAMES = {EINVAL: "EINVAL", ENOTSORTED: "ENOTSORTED", ENODEV: "ENODEV", EHIP: "EHIP",
          ERANGE: "ERANGE", ENOMEM: "ENOMEM", ETOOLONG: "ETOOLONG"}


class SyzcovError(RuntimeError):
    def __init__(self, code: int, fn: str, msg: str):
        self.code = code
        super().__init__(f"{fn}: {_NAMES.get(code, code)} {msg}")


def build(jobs: int = 8) -> str:
    """Compile every HIP source for gfx950 into syzkaller_amd/libsyzcov.so."""
    subprocess.run(["make", "-s", f"-j{jobs}", "-C", _HERE], check=True)
    return LIB_PATH


p_ = C.c_void_p
sz = C.c_size_t
u32, u64, i32, i64 = C.c_uint32, C.c_uint64, C.c_int32, C.c_int64

# name: (restype, argtypes)
_SIGS = {
    "syzcov_version": (C.c_char_p, []),
    "syzcov_last_error": (C.c_char_p, []),
    "syzcov_pool_contexts": (i64, [C.c_int]),
    "syzcov_pool_trim": (C.c_int, []),
    "syzcov_restore_pc": (u64, [u32, u32]),
    "syzcov_canonicalize": (i64, [p_, sz]),
    "syzcov_cover_dedup64": (i64, [p_, sz]),
    "syzcov_difference": (i64, [p_, sz, p_, sz, p_]),
    "syzcov_symmetric_difference": (i64, [p_, sz, p_, sz, p_]),
    "syzcov_union": (i64, [p_, sz, p_, sz, p_]),
    "syzcov_intersection": (i64, [p_, sz, p_, sz, p_]),
    "syzcov_minimize": (i64, [p_, p_, sz, p_, C.c_int, p_]),
    "syzcov_sort_order": (C.c_int, [p_, sz, C.c_int, p_]),
    "syzcov_minimize_corpus": (i64, [p_, p_, p_, sz, C.c_int, p_]),
    "syzcov_minimize_corpus_stats": (C.c_int, [p_]),
    "syzcov_union_all": (i64, [p_, p_, sz, p_]),
    "syzcov_unique_cover": (i64, [p_, p_, p_, sz, p_]),
    "syzcov_ui_stats": (i64, [p_, p_, p_, sz, u32, p_, p_, p_, p_]),
    "syzcov_calculate_priorities": (C.c_int, [p_, p_, sz, C.c_int, C.c_int, p_, p_, p_]),
    "syzcov_static_priorities": (C.c_int, [p_, p_, p_, sz, p_, p_, p_, C.c_int, p_]),
    "syzcov_dev_static_prio": (C.c_int, [p_, p_, p_, p_, p_, p_, C.c_int, p_, p_]),
    "syzcov_normalize_prio": (C.c_int, [p_, C.c_int]),
    "syzcov_build_choice_table": (C.c_int, [p_, p_, C.c_int, p_]),
    "syzcov_choose_batch": (C.c_int, [p_, p_, C.c_int, p_, p_, sz, p_]),
    "syzcov_state_create": (C.c_int, [C.c_int, u32, u64, p_]),
    "syzcov_state_destroy": (C.c_int, [u64]),
    "syzcov_state_add": (C.c_int, [u64, C.c_int, p_, sz]),
    "syzcov_state_set_flakes": (C.c_int, [u64, p_, sz]),
    "syzcov_state_get": (i64, [u64, C.c_int, p_, sz]),
    "syzcov_newcov_batch": (i64, [u64, p_, p_, p_, sz, p_]),
    "syzcov_parse_exec_output": (i64, [p_, sz, sz, p_, p_, sz, p_, p_, p_, p_, p_, sz]),
    "syzcov_state_set_universe": (C.c_int, [u64, p_, sz]),
    "syzcov_state_corpus_add": (C.c_int, [u64, C.c_int, p_, sz]),
    "syzcov_state_corpus_get": (i64, [u64, C.c_int, p_, sz]),
    "syzcov_state_flakes_get": (i64, [u64, p_, sz]),
    "syzcov_state_add_inputs": (i64, [u64, p_, p_, p_, sz, p_]),
    "syzcov_state_triage": (i64, [u64, sz, p_, p_, p_, p_, p_, p_, p_, p_]),
    "syzcov_state_newcov_ws_size": (sz, [sz, u64]),
    "syzcov_state_newcov_dev": (C.c_int, [u64, p_, p_, p_, sz, u64, p_, p_, p_, sz, p_]),
    # resident corpus engine (corpus.hip)
    "syzcov_corpus_mem_size": (i64, [p_]),
    "syzcov_corpus_create": (C.c_int, [p_, p_, sz, p_]),
    "syzcov_corpus_destroy": (C.c_int, [u64]),
    "syzcov_corpus_info": (C.c_int, [u64, p_]),
    "syzcov_corpus_buffer": (C.c_int, [u64, C.c_int, p_, p_]),
    "syzcov_corpus_canonical": (C.c_int, [u64, p_, p_]),
    "syzcov_dev_canon_split_aligned": (C.c_int, [p_, p_, p_, p_, sz, sz, u32, u64, u32, u32, u64,
                                                 C.c_int, u32, p_, p_, p_, p_, sz, p_]),
    "syzcov_dev_canon_aligned_words": (u64, [u64, u64, u64]),
    "syzcov_dev_minimize_range_aligned": (C.c_int, [p_, p_, p_, p_, p_, sz, u32, u64, u32, p_, p_,
                                                    p_, p_, p_, u64, p_, p_, p_, C.c_int, p_, p_,
                                                    p_]),
    "syzcov_dev_minimize_range_aligned_pass2": (C.c_int, [p_, p_, p_, p_, p_, sz, u32, u64, u32,
                                                          p_, C.c_int, p_, p_, p_, u64, p_, p_, p_,
                                                          p_, p_, p_, p_]),
    "syzcov_corpus_canon": (C.c_int, [u64, p_, p_, sz, p_]),
    "syzcov_corpus_order": (C.c_int, [u64, p_, sz, p_]),
    "syzcov_corpus_order_given": (C.c_int, [u64, p_, sz, p_]),
    "syzcov_corpus_order_part": (C.c_int, [u64, p_, sz, p_]),
    "syzcov_corpus_minimize": (C.c_int, [u64, C.c_int, p_]),
    "syzcov_corpus_dense_first": (i64, [u64, p_]),
    "syzcov_corpus_pass2": (C.c_int, [u64, p_]),
    "syzcov_corpus_finish": (C.c_int, [u64, p_]),
    "syzcov_corpus_step": (C.c_int, [u64, p_, p_, sz, p_]),
    "syzcov_corpus_result": (C.c_int, [u64, p_, p_]),
    "syzcov_corpus_minimize_host": (i64, [u64, p_, p_, sz, p_, p_, sz, p_]),
    "syzcov_corpus_minimize_host_order": (i64, [u64, p_, p_, sz, p_, p_, p_, sz, p_]),
    # device tier
    "syzcov_dev_canon_ws_size": (sz, [sz, sz]),
    "syzcov_dev_canonicalize": (C.c_int, [p_, p_, p_, p_, sz, sz, p_, u32, u64, p_, p_, sz, p_]),
    "syzcov_dev_mark": (C.c_int, [p_, p_, p_, sz, p_, u32, u64, p_, p_]),
    "syzcov_dev_bitmap_op": (C.c_int, [C.c_int, p_, p_, u64, p_, p_]),
    "syzcov_dev_dict_build_bits": (C.c_int, [p_, u64, p_, p_, p_, p_]),
    "syzcov_dev_dict_ws_size": (sz, [u64]),
    "syzcov_dev_dict_build": (C.c_int, [p_, u64, p_, p_, p_, p_]),
    "syzcov_dev_dict_to_list": (C.c_int, [p_, u64, u32, p_, p_, p_]),
    "syzcov_dev_dict_to_list_drop": (C.c_int, [p_, u64, u32, u32, p_, p_, p_]),
    "syzcov_dev_minimize_pass1": (C.c_int, [p_, p_, p_, p_, p_, sz, p_, u32, p_, p_, p_]),
    "syzcov_dev_minimize_pass2": (C.c_int, [p_, p_, p_, p_, p_, sz, p_, u32, p_, p_, p_, p_]),
    "syzcov_dev_canon_split_ws_size": (sz, [sz]),
    "syzcov_dev_canon_split": (C.c_int, [p_, p_, p_, p_, sz, sz, u32, u64, u32, p_, p_, p_, p_, sz,
                                         p_]),
    "syzcov_dev_canon_split_keys": (C.c_int, [p_, p_, p_, p_, sz, sz, u32, u64, u32, u32, u64,
                                              u32, p_, p_, p_, p_, sz, p_]),
    "syzcov_dev_words_to_pcs": (C.c_int, [p_, sz, u32, u32, p_, p_]),
    "syzcov_dev_cover_dedup64": (C.c_int, [p_, p_, sz, p_, p_, p_]),
    "syzcov_dev_cover_ingest64_ws_size": (sz, [sz, u64]),
    "syzcov_dev_cover_ingest64": (C.c_int, [p_, p_, sz, u64, p_, p_, p_, p_, sz, p_]),
    "syzcov_dev_minimize_range_keys": (C.c_int, [p_, p_, p_, p_, p_, p_, sz, u64, u32, p_, p_, p_,
                                                 p_, p_, u64, p_, p_, p_, C.c_int, p_, p_, p_]),
    "syzcov_dev_minimize_range_keys_pass2": (C.c_int, [p_, p_, p_, p_, p_, p_, sz, u64, u32, p_,
                                                       p_, p_, p_, u64, p_, p_, p_, p_, p_]),
    "syzcov_dev_universe_keymap": (C.c_int, [p_, sz, u32, u32, u64, p_, p_, p_, p_]),
    "syzcov_dev_keys_to_pcs": (C.c_int, [p_, u64, p_, p_, p_, sz, p_]),
    "syzcov_dev_first_to_bits": (C.c_int, [p_, u64, p_, p_]),
    "syzcov_dev_minimize_range_ws_size": (sz, [sz, u64, u32]),
    "syzcov_dev_minimize_range": (C.c_int, [p_, p_, p_, p_, p_, p_, sz, u32, u64, u32, p_, p_, p_,
                                            p_, u64, p_, p_, p_, C.c_int, sz, u32, u64, p_, p_]),
    "syzcov_dev_minimize_range_pass2": (C.c_int, [p_, p_, p_, p_, p_, p_, sz, u32, u64, u32, p_,
                                                  p_, p_, p_, u64, p_, p_, p_, p_, p_, p_, p_]),
    "syzcov_dev_first_dense": (C.c_int, [p_, u64, p_, p_, C.c_int, p_]),
    "syzcov_dev_compact_ws_size": (sz, [sz]),
    "syzcov_dev_compact_kept": (C.c_int, [p_, p_, sz, p_, p_, p_, p_]),
    "syzcov_dev_sort_ws_size": (sz, [sz]),
    "syzcov_dev_sort_order": (C.c_int, [p_, sz, C.c_int, p_, p_, sz, p_]),
    "syzcov_dev_sort_order_part": (C.c_int, [p_, sz, u32, u32, p_, p_, sz, p_]),
    "syzcov_dev_sort_seg_ws_size": (sz, [sz, sz]),
    "syzcov_dev_sort_order_segmented": (C.c_int, [p_, p_, sz, sz, C.c_int, p_, p_, sz, p_]),
    "syzcov_dev_bytemap_op": (C.c_int, [C.c_int, p_, p_, u64, p_, p_]),
    "syzcov_dev_synth_lens": (C.c_int, [u64, u64, sz, u32, u32, p_, p_]),
    "syzcov_dev_synth_pcs": (C.c_int, [u64, u64, sz, p_, u32, C.c_int, p_, p_]),
    "syzcov_dev_synth_universe": (C.c_int, [u64, u32, p_, p_]),
    "syzcov_dev_synth_universe_mode": (C.c_int, [u64, u32, C.c_int, p_, p_]),
    "syzcov_dev_synth_callids": (C.c_int, [u64, u64, sz, u32, p_, p_]),
    "syzcov_dev_stream_copy": (C.c_int, [p_, p_, sz, p_]),
    "syzcov_dev_copy_peak": (C.c_int, [p_, p_, sz, C.c_int, p_]),
    "syzcov_dev_prio_rows": (sz, [C.c_int]),
    "syzcov_dev_prio_ldp": (sz, [sz]),
    "syzcov_dev_prio_build_at": (C.c_int, [C.c_int, p_, p_, p_, sz, C.c_int, p_, sz, p_, p_]),
    "syzcov_dev_prio_counts": (C.c_int, [p_, sz, sz, C.c_int, p_, p_]),
    "syzcov_dev_prio_counts_ws_size": (sz, [sz, C.c_int]),
    "syzcov_dev_bits_to_bytes": (C.c_int, [p_, u64, p_, p_]),
    "syzcov_dev_bytes_to_bits": (C.c_int, [p_, u64, p_, p_]),
    "syzcov_dev_prio_counts_ws": (C.c_int, [p_, sz, sz, C.c_int, p_, p_, sz, p_]),
    "syzcov_dev_prio_pos_ws_size": (sz, [sz, C.c_int, C.c_int]),
    "syzcov_dev_prio_counts_pos": (C.c_int, [p_, sz, C.c_int, C.c_int, p_, p_, sz, p_]),
    "syzcov_dev_prio_finish": (C.c_int, [p_, C.c_int, p_, p_, p_, p_]),
    "syzcov_dev_normalize_prio": (C.c_int, [p_, C.c_int, p_]),
    "syzcov_dev_choose": (C.c_int, [p_, p_, C.c_int, p_, p_, sz, p_, p_, p_]),
    "syzcov_dev_choice_table": (C.c_int, [p_, p_, C.c_int, p_, p_]),
}

_lib = None


def lib():
    """Load libsyzcov.so (raises if it was not built: there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built; run `make -C syzkaller_amd` "
                              "(syzkaller_amd has no CPU fallback)")
        # torch (if used) must own the HIP runtime first so both share one copy
        try:
            import torch  # noqa: F401
        except Exception:  # pragma: no cover - torch is optional for the C-ABI
            pass
        L = C.CDLL(LIB_PATH)
        missing = []
        for name, (res, args) in _SIGS.items():
            try:
                f = getattr(L, name)
            except AttributeError:
                missing.append(name)
                continue
            f.restype = res
            f.argtypes = args
        # a tuning variant (SYZCOV_LIB) may predate an entry point; the product
        # library must export every one
        if missing and not os.environ.get("SYZCOV_LIB"):
            raise ImportError(f"{LIB_PATH} lacks {missing}: rebuild it")
        _lib = L
    return _lib


def check(rc: int, fn: str) -> int:
    if rc < 0:
        raise SyzcovError(rc, fn, lib().syzcov_last_error().decode(errors="replace"))
    return rc


def header_symbols() -> list[str]:
    import re
    with open(HEADER) as f:
        txt = f.read()
    return sorted(set(re.findall(r"\b(syzcov_[a-z0-9_]+)\(", txt)))


# ---------------------------------------------------------------- corpus ABI
class GroupsStats(C.Structure):
    """syzcov_groups_stats (syzcov.h): the calling thread's last minimizeCorpus."""
    _fields_ = [("path", C.c_int32), ("upload_ms", C.c_float), ("device_ms", C.c_float),
                ("download_ms", C.c_float)]


GROUPS_PATHS = {0: "none", 1: "lds", 2: "engine", 3: "slabs"}


class CorpusCfg(C.Structure):
    """syzcov_corpus_cfg (include/syzcov.h)."""
    _fields_ = [("n_max", sz), ("n_global", sz), ("rank", sz), ("p_max", u64),
                ("max_seg_len", sz), ("pc_lo", u32), ("pc_span", u64), ("universe", p_),
                ("universe_n", sz), ("canon_in_place", C.c_int), ("order_by", C.c_int),
                ("rec_cap", u64), ("canon_layout", C.c_int)]


class CorpusInfo(C.Structure):
    """syzcov_corpus_info_t."""
    _fields_ = [("key_mode", u32), ("kshift", u32), ("kbase", u32), ("pc_lo", u32),
                ("span", u64), ("win_lo", u32), ("sent_key", u32), ("win_span", u64),
                ("nrange", u64), ("nwords", u64), ("n_global", u64), ("union_cap", u64),
                ("rec_cap", u64), ("mem", p_), ("mem_size", u64), ("canon_align_k", u64)]


class CorpusRes(C.Structure):
    """syzcov_corpus_res."""
    _fields_ = [("err_flags", u32), ("n_ids", u32), ("n_kept", u32), ("n_union", u32),
                ("max_cover", u64), ("records", u64), ("kept_idx", p_), ("union_pcs", p_),
                ("fallback", u32), ("max_cover_missed", u32)]


# enum of syzcov_corpus_buffer (include/syzcov.h)
CORPUS_BUFS = ("CANON", "NEW_LEN", "SPLIT", "RANGE_TOT", "COVERED", "MAX_COVER", "TAB", "FIRST",
               "REC", "CAND", "KEPT", "LENS", "ORDER", "KEPT_IDX", "UNION", "SCAL", "PC_OF_KEY",
               "LOW_OF_KEY", "GLENS", "SEL", "IOTA", "ITEMS", "RANKS", "FIRST_DENSE", "WS", "WS2")
