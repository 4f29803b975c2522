"""Every ctypes binding of the C-ABI agrees with the prototypes in include/*.h (no GPU needed).

Two bindings are checked argument by argument against the headers:
- the package's own (`zbot_amd/engine.py:load_library`), and
- every `lib.zb_*.argtypes = ...` line inside INTEGRATION.md's python code blocks, i.e. the binding
  a ksim maintainer would copy next to train.py (that snippet still declared ABI 1's
  8 pointers for zb_step after ABI 2 added `success`, so the documented call raised ArgumentError).

Each header parameter is classified by the ctypes type that passes it correctly: a pointer, or a
scalar of a given C type. A binding's argtypes list must have the same length and the same class
at every position.
"""

import ctypes as C
import os
import re

import pytest

from zbot_amd import cstructs as cs
from zbot_amd import engine as E

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = ("zbot.h", "zbot_ppo.h", "zbot_policy.h")

# C scalar type -> the ctypes types that pass it correctly
_SCALARS = {
    "float": {C.c_float},
    "double": {C.c_double},
    "int": {C.c_int, C.c_int32},
    "int32_t": {C.c_int, C.c_int32},
    "uint32_t": {C.c_uint32, C.c_uint},
    "uint64_t": {C.c_uint64, C.c_ulonglong},
    "size_t": {C.c_size_t},
    "long long": {C.c_longlong, C.c_int64},
}


def header_prototypes() -> dict:
    """{name: [kind, ...]} for every zb_* prototype; kind is 'ptr' or a C scalar type name."""
    protos = {}
    for h in HEADERS:
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", " ", txt, flags=re.S)
        for m in re.finditer(r"\b(zb_[a-z0-9_]+)\s*\(([^()]*)\)\s*;", txt):
            name, params = m.group(1), " ".join(m.group(2).split())
            kinds = []
            if params not in ("", "void"):
                for p in params.split(","):
                    p = p.strip()
                    if "*" in p:
                        kinds.append("ptr")
                        continue
                    ty = re.sub(r"\b(const|unsigned)\b", " ", p).split()
                    ty = " ".join(ty[:-1])  # drop the parameter name
                    assert ty in _SCALARS, f"{h}: {name}: unclassified parameter type {p!r}"
                    kinds.append(ty)
            protos[name] = kinds
    return protos


def _is_pointer_type(t) -> bool:
    return t in (C.c_void_p, C.c_char_p) or (isinstance(t, type) and issubclass(t, C._Pointer))


def mismatches(argtypes, kinds) -> list:
    if len(argtypes) != len(kinds):
        return [f"{len(argtypes)} argtypes for {len(kinds)} parameters"]
    bad = []
    for i, (t, k) in enumerate(zip(argtypes, kinds)):
        ok = _is_pointer_type(t) if k == "ptr" else t in _SCALARS[k]
        if not ok:
            bad.append(f"argument {i + 1}: {getattr(t, '__name__', t)} for C {k}")
    return bad


def integration_argtypes(path=os.path.join(ROOT, "INTEGRATION.md")) -> dict:
    """{name: argtypes} from every `lib.zb_*.argtypes = <expr>` line of INTEGRATION.md's python
    blocks, evaluated in the snippet's own namespace (C = ctypes, vp = c_void_p, cs)."""
    txt = open(path).read()
    out = {}
    ns = {"C": C, "vp": C.c_void_p, "cs": cs}
    for block in re.findall(r"```python\n(.*?)```", txt, flags=re.S):
        # join continuation lines of a bracketed expression
        stmt, depth, stmts = "", 0, []
        for line in block.splitlines():
            stmt += line.split("#")[0] + " "
            depth += line.count("[") + line.count("(") - line.count("]") - line.count(")")
            if depth <= 0:
                stmts.append(stmt)
                stmt, depth = "", 0
        for s in stmts:
            m = re.match(r"\s*\w+\.(zb_[a-z0-9_]+)\.argtypes\s*=\s*(.+)$", s.strip())
            if m:
                out[m.group(1)] = eval(m.group(2), ns)  # noqa: S307 - our own document's literal lists
    return out


def test_header_parse_sees_the_abi():
    p = header_prototypes()
    assert p["zb_step"] == ["ptr"] * 9 + ["float", "ptr"]
    assert p["zb_create"] == ["ptr", "ptr", "int", "int", "int", "uint64_t", "ptr"]
    assert p["zb_adv_normalize"][2] == "long long"
    assert len(p) >= 30


def test_engine_binding_matches_headers():
    """engine.py's argtypes for every declared function that takes arguments."""
    E.build_library()
    L = E.load_library()
    problems = {}
    checked = 0
    for name, kinds in header_prototypes().items():
        at = getattr(L, name).argtypes
        if at is None:
            assert not kinds, f"engine.py declares no argtypes for {name}({len(kinds)} parameters)"
            continue
        checked += 1
        bad = mismatches(at, kinds)
        if bad:
            problems[name] = bad
    assert not problems, problems
    assert checked >= 25


def test_integration_binding_matches_headers():
    """The documented reference-side binding declares each function it binds
    with the header's arity and argument classes."""
    decl = integration_argtypes()
    assert {"zb_create", "zb_reset", "zb_step"} <= set(decl)
    protos = header_prototypes()
    problems = {n: mismatches(at, protos[n]) for n, at in decl.items()}
    problems = {n: b for n, b in problems.items() if b}
    assert not problems, problems


def test_checker_catches_the_r03_binding(tmp_path):
    """The round-3 INTEGRATION line (ABI 1's zb_step arity) is reported."""
    p = tmp_path / "old.md"
    p.write_text("```python\nlib.zb_step.argtypes = [vp] * 8 + [C.c_float, vp]\n```\n")
    bad = mismatches(integration_argtypes(str(p))["zb_step"], header_prototypes()["zb_step"])
    assert bad == ["10 argtypes for 11 parameters"]


@pytest.mark.parametrize("name", ["zb_step", "zb_rollout", "zb_reset"])
def test_integration_calls_pass_header_arity(name):
    """Every call `lib.<name>(...)` in the documented binding passes as many arguments as the
    header declares (the r03 snippet passed 11 to a 10-argtype declaration)."""
    txt = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    want = len(header_prototypes()[name])
    calls = 0
    for block in re.findall(r"```python\n(.*?)```", txt, flags=re.S):
        for m in re.finditer(rf"\blib\.{name}\(", block):
            i, depth, args, cur = m.end(), 1, 0, ""
            while depth:
                ch = block[i]
                if ch in "([":
                    depth += 1
                elif ch in ")]":
                    depth -= 1
                if ch == "," and depth == 1:
                    args += 1
                i += 1
            calls += 1
            assert args + 1 == want, f"INTEGRATION.md calls {name} with {args + 1} arguments, header has {want}"
    if name != "zb_rollout":
        assert calls >= 1
