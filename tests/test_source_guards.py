"""Source guards for fault classes that compile silently (CPU, no GPU).

Two GPU faults came from the readlane builtins, which move 32 bits and return
int: round 3's whole-wave minimize widened a readlane result to
64 bits (a low half >= 2^31 sign-extended into a wild offset), round 5's
segment descriptor passed a u64 CSR base through readfirstlane.  Every use now
goes through common.h's typed helpers (wave_readfirstlane / wave_readlane
reject a non-32-bit or pointer argument at compile time and keep the caller's
unsigned type; uniform_u64 / wave_readlane_u64 split 64-bit values), and this
test keeps the raw builtins (and the raw instructions in inline asm) out of
every other source."""
import os
import re

CSRC = os.path.join(os.path.dirname(__file__), "..", "syzkaller_amd", "csrc")
RAW = re.compile(r"__builtin_amdgcn_read(first)?lane\s*\(")
ASM = re.compile(r'\basm\s*(volatile\s*)?\(\s*"[^"]*\bv_read(first)?lane')


def _sources():
    for f in sorted(os.listdir(CSRC)):
        if f.endswith((".hip", ".h", ".cc")):
            with open(os.path.join(CSRC, f)) as fh:
                yield f, fh.read()


def test_readlane_only_through_common_h():
    bad = []
    for f, txt in _sources():
        for i, line in enumerate(txt.splitlines(), 1):
            if RAW.search(line) and not (f == "common.h" and "readlane-door" in line):
                bad.append(f"{f}:{i}: {line.strip()}")
        if ASM.search(txt):
            bad.append(f"{f}: v_readlane / v_readfirstlane in inline asm")
    assert not bad, "raw readlane builtins outside common.h's typed helpers:\n" + "\n".join(bad)


def test_readlane_helpers_reject_wide_types():
    """The helpers' compile-time check is in place (a 64-bit value or pointer
    passed to them fails to compile)."""
    txt = dict(_sources())["common.h"]
    doors = [m.start() for m in re.finditer(r"readlane-door", txt)]
    assert len(doors) == 2, "exactly two builtin call sites (readfirstlane, readlane)"
    for name in ("wave_readfirstlane", "wave_readlane"):
        body = txt[txt.index(f"T {name}("):]
        body = body[:body.index("}")]
        assert "static_assert(sizeof(T) == 4 && std::is_integral<T>::value" in body, name
    assert "uniform_u64" in txt and "wave_readlane_u64" in txt


def test_uniform_u64_splits_halves():
    txt = dict(_sources())["common.h"]
    body = txt[txt.index("uint64_t uniform_u64("):]
    body = body[:body.index("}")]
    assert "(uint32_t)(v >> 32)" in body and "(uint32_t)v" in body
