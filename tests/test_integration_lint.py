"""The Go cgo shim in INTEGRATION.md cannot be compiled here (no Go toolchain,
SURVEY.md §8c), so this lints it against the C headers it binds: every
`C.<name>` is a macro, function or type declared in include/*.h (or a cgo
builtin), every field in a `C.<struct>{...}` literal or a `v.field` access on
a C-struct variable exists in that struct, every `C.okv_*(...)` call passes as
many arguments as the prototype takes, and the block-status switch maps every
OKV_BLK_* status the header defines."""
from __future__ import annotations

import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CGO_BUILTINS = {"int", "uint", "char", "double", "float", "size_t", "int8_t", "int16_t", "int32_t",
                "int64_t", "uint8_t", "uint16_t", "uint32_t", "uint64_t", "GoString", "CString",
                "GoBytes", "free"}


def _strip_comments(src: str) -> str:
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    return re.sub(r"//[^\n]*", " ", src)


def header_symbols():
    defines, funcs, structs = set(), {}, {}
    for name in sorted(os.listdir(os.path.join(ROOT, "include"))):
        if not name.endswith(".h"):
            continue
        src = _strip_comments(open(os.path.join(ROOT, "include", name)).read())
        defines |= set(re.findall(r"#define\s+(\w+)", src))
        for m in re.finditer(r"typedef\s+struct\s+\w*\s*\{(.*?)\}\s*(\w+)\s*;", src, re.S):
            fields = set()
            for decl in m.group(1).split(";"):
                decl = decl.strip()
                if not decl:
                    continue
                for part in decl.split(","):  # "uint64_t row_cap, key_cap, val_cap"
                    fm = re.search(r"(\w+)\s*(\[[^\]]*\])?\s*$", part.strip())
                    if fm:
                        fields.add(fm.group(1))
            structs[m.group(2)] = fields
        structs.update({t: set() for t in re.findall(r"typedef\s+struct\s+\w+\s+(\w+)\s*;", src)
                        if t not in structs})
        for m in re.finditer(r"\b(okv_\w+)\s*\(([^;{]*?)\)\s*;", src, re.S):
            params = m.group(2).strip()
            funcs[m.group(1)] = 0 if params in ("", "void") else len(_split_args(params))
    return defines, funcs, structs


def _split_args(s: str):
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return out


def _balanced(text: str, i: int, open_ch: str, close_ch: str) -> str:
    """Text between text[i] == open_ch and its matching close_ch."""
    depth = 0
    for j in range(i, len(text)):
        if text[j] == open_ch:
            depth += 1
        elif text[j] == close_ch:
            depth -= 1
            if depth == 0:
                return text[i + 1:j]
    raise AssertionError(f"unbalanced {open_ch} at {i}")


def go_blocks():
    md = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    return re.findall(r"```go\n(.*?)```", md, re.S)


def test_go_blocks_present():
    assert len(go_blocks()) >= 3


def test_c_identifiers_declared():
    defines, funcs, structs = header_symbols()
    known = defines | set(funcs) | set(structs) | CGO_BUILTINS
    missing = set()
    for blk in go_blocks():
        code = re.sub(r"//[^\n]*", "", blk)
        missing |= {n for n in re.findall(r"\bC\.(\w+)", code) if n not in known}
    assert not missing, f"INTEGRATION.md uses C.{sorted(missing)} which include/*.h does not declare"


def test_c_struct_fields_exist():
    _, _, structs = header_symbols()
    bad = []
    for blk in go_blocks():
        code = re.sub(r"//[^\n]*", "", blk)
        # composite literals C.<struct>{key: value, ...}
        for m in re.finditer(r"\bC\.(\w+)\{", code):
            body = _balanced(code, m.end() - 1, "{", "}")
            for arg in _split_args(body):
                km = re.match(r"\s*(\w+)\s*:", arg)
                if km and km.group(1) not in structs.get(m.group(1), set()):
                    bad.append(f"C.{m.group(1)}{{{km.group(1)}: ...}}")
        # variables bound to a C struct, then v.field accesses (latest binding wins)
        binds = [(m.start(), m.group(1), m.group(2)) for m in
                 re.finditer(r"\b(\w+)\s*:=\s*C\.(\w+)\{", code)]
        binds += [(m.start(), m.group(1), m.group(2)) for m in
                  re.finditer(r"\bvar\s+(\w+)\s+C\.(\w+)\b", code)]
        binds.sort()
        for m in re.finditer(r"\b(\w+)\.(\w+)\b", code):
            var, field = m.group(1), m.group(2)
            typ = None
            for pos, v, t in binds:
                if pos < m.start() and v == var:
                    typ = t
            if typ in structs and field not in structs[typ]:
                bad.append(f"{var}.{field} ({typ})")
    assert not bad, f"fields not declared in include/*.h: {bad}"


def test_c_call_arity():
    _, funcs, _ = header_symbols()
    bad = []
    for blk in go_blocks():
        code = re.sub(r"//[^\n]*", "", blk)
        for m in re.finditer(r"\bC\.(okv_\w+)\(", code):
            args = _split_args(_balanced(code, m.end() - 1, "(", ")"))
            if m.group(1) in funcs and len(args) != funcs[m.group(1)]:
                bad.append(f"{m.group(1)}: {len(args)} args, prototype takes {funcs[m.group(1)]}")
    assert not bad, bad


def test_block_status_switch_is_complete():
    defines, _, _ = header_symbols()
    statuses = {d for d in defines if d.startswith("OKV_BLK_")}
    code = "".join(go_blocks())
    mapped = set(re.findall(r"\bC\.(OKV_BLK_\w+)", code))
    assert statuses <= mapped, f"statuses the shim does not map: {sorted(statuses - mapped)}"


def test_lint_catches_the_round2_bug():
    """The linter itself: the undefined constant the round-2 shim used is caught."""
    defines, funcs, structs = header_symbols()
    assert "OKV_BLK_ZSTD" not in defines and "OKV_BLK_ZSTD_ERROR" in defines
    assert "compressed_size" in structs["okv_block_desc"]
    assert funcs["okv_decode_blocks"] == 8 and funcs["okv_decode_plan"] == 10
