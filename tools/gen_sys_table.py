#!/usr/bin/env python3
"""Build-time generator of the syscall usage table behind
calcStaticPriorities (prog/prio.go:40-135).

The reference derives it from its generated `sys` package
(sys/sys_<arch>.go, gitignored output of sysgen), which this image cannot
build (no Go).  This tool restates the pieces that the static priorities
depend on:

  sysparser.Parse      sysparser/lexer.go:48-246, parser.go (line grammar,
                       nested types -> unnamedN, const/array fake flags,
                       syscalls sorted by name)
  sysgen type mapping  sysgen/sysgen.go:196-253 (resource Kind chains),
                       :262-285 (struct instance names), :362-667 (generateArg)
  sys.ForeachType      sys/decl.go:487-525
  sys.init IDs         sys/decl.go:534-555 (Call.ID, CallID by CallName)
  noteUsage            prog/prio.go:42-104

and writes, per usage id, the (call ID, weight) pairs — data, not source.
The GPU computes the static matrix from it (syzcov_dev_static_prio).

Usage: tools/gen_sys_table.py /root/reference/sys syzkaller_amd/data/sys_table.json
"""
from __future__ import annotations

import glob
import json
import os
import sys


class ParseError(Exception):
    pass


class Parser:
    """sysparser/parser.go: one line at a time, Ident/Parse/SkipWs."""

    def __init__(self, line: str):
        self.s, self.i = line, 0

    def eof(self):
        return self.i == len(self.s)

    def char(self):
        if self.eof():
            raise ParseError("unexpected eof: " + self.s)
        return self.s[self.i]

    def skip_ws(self):
        while self.i < len(self.s) and self.s[self.i] in " \t":
            self.i += 1

    def parse(self, ch):
        if self.eof() or self.s[self.i] != ch:
            raise ParseError(f"want {ch!r}: {self.s}")
        self.i += 1
        self.skip_ws()

    def ident(self):
        start = self.i
        if self.char() == '"':
            self.parse('"')
            while self.char() != '"':
                self.i += 1
            end = self.i + 1
            self.parse('"')
        else:
            while self.i < len(self.s) and (self.s[self.i].isalnum() or self.s[self.i] in "_$-:"):
                self.i += 1
            if start == self.i:
                raise ParseError("identifier expected: " + self.s)
            end = self.i
        v = self.s[start:end]
        self.skip_ws()
        return v


class Desc:
    def __init__(self):
        self.syscalls = []      # (name, callname, args[[name, type, a...]], ret[type, a...])
        self.structs = {}       # name -> (is_union, fields[[name, type, a...]])
        self.unnamed = {}       # unnamedN -> [type, a...]
        self.strflags = {}
        self.flags = {}
        self.resources = {}     # name -> base
        self.unnamed_seq = 0
        self.const_seq = 0


def parse_type1(p: Parser, d: Desc, name: str):
    typ = [name]
    if not p.eof() and p.char() == "[":
        p.parse("[")
        while True:
            ident = p.ident()
            if p.char() == "[":
                inner = parse_type1(p, d, ident)
                ident = f"unnamed{d.unnamed_seq}"
                d.unnamed_seq += 1
                d.unnamed[ident] = inner
            typ.append(ident)
            if p.char() == "]":
                break
            p.parse(",")
        p.parse("]")
    if name == "const" and len(typ) > 1:
        d.flags[f"const_flag_{d.const_seq}"] = typ[1:2]
        d.const_seq += 1
    if name == "array" and len(typ) > 2:
        d.flags[f"const_flag_{d.const_seq}"] = typ[2:3]
        d.const_seq += 1
    return typ


def parse_type(p, d):
    return parse_type1(p, d, p.ident())


def parse_files(files) -> Desc:
    d = Desc()
    cur = None  # (name, is_union, fields)
    for fname in files:
        with open(fname) as f:
            for raw in f.read().split("\n"):
                p = Parser(raw)
                if p.eof() or p.char() == "#":
                    continue
                if cur is not None:
                    if p.char() in "}]":
                        p.parse(p.char())
                        parse_type1(p, d, "")  # attributes
                        d.structs[cur[0]] = (cur[1], cur[2])
                        cur = None
                    else:
                        p.skip_ws()
                        fld = [p.ident()]
                        fld += parse_type(p, d)
                        cur[2].append(fld)
                    continue
                name = p.ident()
                if name == "include":
                    continue
                if name == "define":
                    continue
                if name == "resource":
                    p.skip_ws()
                    rid = p.ident()
                    p.parse("[")
                    base = p.ident()
                    p.parse("]")
                    d.resources[rid] = base
                    continue
                ch = p.char()
                if ch == "(":
                    p.parse("(")
                    args = []
                    while p.char() != ")":
                        arg = [p.ident()]
                        arg += parse_type(p, d)
                        args.append(arg)
                        if p.char() != ")":
                            p.parse(",")
                    p.parse(")")
                    ret = parse_type(p, d) if not p.eof() else []
                    callname = name.split("$", 1)[0]
                    d.syscalls.append((name, callname, args, ret))
                elif ch == "=":
                    p.parse("=")
                    is_str = p.char() == '"'
                    vals = []
                    while True:
                        v = p.ident()
                        vals.append(v[1:-1] if is_str else v)
                        if p.eof():
                            break
                        p.parse(",")
                    (d.strflags if is_str else d.flags)[name] = vals
                elif ch in "{[":
                    p.parse(ch)
                    cur = (name, ch == "[", [])
                else:
                    raise ParseError("bad line: " + raw)
    d.syscalls.sort(key=lambda s: s[0].encode())  # Go string order = byte order
    return d


def resource_kind(d: Desc, name: str):
    """sysgen.go:196-253: Kind = [root ..., name]."""
    kind = [name]
    base = d.resources[name]
    while base not in ("int8", "int16", "int32", "int64", "intptr"):
        kind.insert(0, base)
        base = d.resources[base]
    return kind


def usages_of_call(d: Desc, args, ret):
    """ForeachType (decl.go:487-525) + noteUsage (prio.go:42-104) over the
    types sysgen would generate for one call.  Returns {id: max weight}."""
    uses = {}

    def note(w, ident):
        if w > uses.get(ident, 0.0):
            uses[ident] = w

    seen = set()

    # Each function returns the (kind, name) of the generated type and
    # visits its subtree.  kind in {struct, union, array, ptr, resource,
    # buffer, other}; name = TypeName (generateArg's `name`).
    def gen(typ, a, name):
        a = [x for x in a if x != "opt"][:] if "opt" in a else list(a)
        if typ == "buffer":
            visit_ptr(("buffer", ""))
            return ("ptr", name)
        if typ == "filename":
            note(1.0, "filename")  # BufferType{Filename} under the PtrType
            return ("ptr", name)
        if typ == "string":
            if len(a) >= 1 and a[0][0] != '"':
                note(0.2, f"str-{a[0]}")
            return ("buffer", name)
        if typ == "vma":
            note(0.5, "vma")
            return ("other", name)
        if typ == "signalno":
            note(1.0, "signalno")
            return ("other", name)
        if typ in ("fileoff", "len", "bytesize", "bytesize2", "bytesize4", "bytesize8", "flags",
                   "const", "proc", "int8", "int16", "int32", "int64", "intptr", "int16be",
                   "int32be", "int64be", "intptrbe", "text", "salg_type", "salg_name"):
            return ("other", name)
        if typ == "array":
            if a[0] == "int8":
                return ("buffer", name)
            elem = gen(a[0], [], "")
            return ("array", name, elem)
        if typ == "ptr":
            pointee = gen(a[1], [], "")
            visit_ptr(pointee)
            return ("ptr", name)
        if typ.startswith("unnamed"):
            inner = d.unnamed[typ]
            return gen(inner[0], inner[1:], "")
        if typ in d.structs:
            is_union, fields = d.structs[typ]
            if typ not in seen:  # ForeachType prunes re-visits; usages are a set
                seen.add(typ)
                for fld in fields:
                    gen(fld[1], fld[2:], fld[0])
            # TypeName = field name if the struct is a field, else the struct name
            return ("union" if is_union else "struct", name if name else typ)
        if typ in d.resources:
            if typ in ("pid", "uid", "gid"):
                note(0.1, f"res{typ}")
            else:
                kind = resource_kind(d, typ)
                s = "res"
                for i, k in enumerate(kind):
                    s += "-" + k
                    note(0.2 if i < len(kind) - 1 else 1.0, s)
            return ("resource", name)
        raise ParseError(f"unknown type {typ}")

    def visit_ptr(pointee):
        # prio.go:71-80: pointee struct/union -> its Name(); array -> elem Name()
        if pointee[0] in ("struct", "union"):
            note(1.0, f"ptrto-{pointee[1]}")
        elif pointee[0] == "array":
            note(1.0, f"ptrto-{pointee[2][1]}")

    for arg in args:
        gen(arg[1], arg[2:], arg[0])
    if ret:
        gen(ret[0], ret[1:], "ret")
    return uses


def build_table(sysdir: str):
    files = sorted(glob.glob(os.path.join(sysdir, "*.txt")))  # filepath.Glob order
    d = parse_files(files)
    calls, callid = [], {}
    uses = {}  # id -> {call: w}
    for cid, (name, callname, args, ret) in enumerate(d.syscalls):
        if callname not in callid:
            callid[callname] = len(callid)
        calls.append({"name": name, "call_name": callname, "call_id": callid[callname]})
        for ident, w in usages_of_call(d, args, ret).items():
            uses.setdefault(ident, {})[cid] = w
    return {
        "source": "restated from sys/*.txt by tools/gen_sys_table.py (sysparser + sysgen + "
                  "ForeachType + prio.go noteUsage); arch-independent",
        "ncalls": len(calls), "call_count": len(callid), "calls": calls,
        "uses": {k: sorted(v.items()) for k, v in sorted(uses.items())},
    }


if __name__ == "__main__":
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/sys"
    dst = sys.argv[2] if len(sys.argv) > 2 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "syzkaller_amd", "data",
        "sys_table.json")
    t = build_table(src)
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    with open(dst, "w") as f:
        json.dump(t, f, separators=(",", ":"))
    print(f"{t['ncalls']} calls, {t['call_count']} call names, {len(t['uses'])} usage ids -> {dst}")
