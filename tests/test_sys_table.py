"""The committed syscall usage table (syzkaller_amd/data/sys_table.json):
shape facts the reference fixes and, when the reference is
mounted (this container only), regeneration from sys/*.txt is byte-stable."""
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLE = os.path.join(ROOT, "syzkaller_amd", "data", "sys_table.json")


def _table():
    with open(TABLE) as f:
        return json.load(f)


def test_call_ids():
    t = _table()
    assert t["ncalls"] == 1170 and t["call_count"] == 293
    names = [c["name"] for c in t["calls"]]
    assert names == sorted(names, key=lambda s: s.encode())  # Go byte order (lexer.go:235)
    assert names[0] == "accept" and names[1] == "accept$alg"
    # CallID = first appearance of CallName in ID order (decl.go:545-551)
    seen = {}
    for c in t["calls"]:
        seen.setdefault(c["call_name"], len(seen))
        assert c["call_id"] == seen[c["call_name"]]


def test_usage_weights():
    t = _table()
    allowed = {0.1, 0.2, 0.5, 1.0}  # prio.go:59,66,73-79,86,89,94,99
    for ident, members in t["uses"].items():
        assert members, ident
        for c, w in members:
            assert 0 <= c < t["ncalls"] and w in allowed, (ident, w)
        if ident.startswith("res") and not ident.startswith("res-"):
            assert ident in ("respid", "resuid", "resgid")
    assert any(k == "ptrto-" for k in t["uses"])  # arrays of non-struct elements (Name() == "")


@pytest.mark.skipif(not os.path.isdir("/root/reference/sys"), reason="reference not mounted")
def test_regenerates_identically(tmp_path):
    import subprocess
    import sys
    out = tmp_path / "t.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_sys_table.py"),
                    "/root/reference/sys", str(out)], check=True, capture_output=True)
    assert json.loads(out.read_text()) == _table()
