"""The C-ABI library: built, loadable, exporting exactly what include/dlrm_hip.h declares.
CPU only — no compute call is made (no GPU here); only pure host entry points are called."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib(pkg):
    return pkg._lib.load()


def test_library_is_built_in_tree(pkg):
    assert os.path.exists(pkg._lib.LIB_PATH), "run __graft_entry__.build()"
    assert pkg._lib.LIB_PATH.startswith(ROOT)


def test_every_header_symbol_is_exported_and_bound(pkg, lib):
    names = pkg._lib.header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), f"{n} declared in include/dlrm_hip.h but not exported"
        assert n in pkg._lib.SIGNATURES, f"{n} has no ctypes signature"
    assert set(pkg._lib.SIGNATURES) == set(names)


def test_ctypes_arity_matches_header(pkg):
    text = open(pkg._lib.HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    for name, (_, args) in pkg._lib.SIGNATURES.items():
        m = re.search(r"\b" + name + r"\s*\(([^)]*)\)", text)
        assert m, name
        params = [p for p in m.group(1).split(",") if p.strip() and p.strip() != "void"]
        assert len(params) == len(args), (name, params, args)


def test_abi_version(lib):
    hdr = open(os.path.join(ROOT, "include", "dlrm_hip.h")).read()
    v = int(re.search(r"#define DLRM_HIP_ABI_VERSION (\d+)", hdr).group(1))
    assert lib.dlrm_abi_version() == v


def test_null_arguments_are_rejected_without_touching_a_device(lib, pkg):
    # argument validation happens on the host before any HIP call
    assert lib.dlrm_ctx_create(0, None, None) == pkg._lib.E_ARG
    assert lib.dlrm_maplookup(None, None, None, 0, 0, 0, 1, 1, None, 0, 0) == pkg._lib.E_ARG
    assert lib.dlrm_interact_fwd(None, 0, 16, 2, 1, None, 16, None, 32, None, 17, 0) == pkg._lib.E_ARG
    assert lib.dlrm_sgd_update(None, None, None, 0, None, 0, 0, 0, 1, 1, None, 0, 0, 0, 0.1) == pkg._lib.E_ARG
    assert lib.dlrm_ctx_destroy(None) == 0
    assert lib.dlrm_tables_destroy(None) == 0
    assert lib.dlrm_indexer_destroy(None) == 0
    assert lib.dlrm_last_error(None) == b"null context"


def test_library_has_gfx950_code_object(pkg):
    data = open(pkg._lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_julia_shim_binds_only_declared_entry_points(pkg):
    """The Julia ccall shim (dlrm.jl_amd/julia/DLRMHip.jl, not executable here: no Julia) names
    only functions the C header declares, so every binding resolves against the library."""
    _lib = pkg._lib
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    text = open(os.path.join(root, "dlrm.jl_amd", "julia", "DLRMHip.jl")).read()
    called = set(re.findall(r"ccall\(\(:(dlrm_[a-z0-9_]+)", text))
    assert called, "no ccall found"
    missing = called - set(_lib.header_functions())
    assert not missing, missing


def _julia_ccalls(text):
    """(name, return type, [argument types], [arguments]) of every ccall((:dlrm_*, libdlrm), ...)."""
    out = []
    for m in re.finditer(r"ccall\(\(:(dlrm_[a-z0-9_]+),\s*libdlrm\),", text):
        # split the rest of the ccall at top-level commas
        i, depth, parts, cur = m.end(), 1, [], ""
        while depth > 0:
            ch = text[i]
            if ch in "({[":
                depth += 1
            elif ch in ")}]":
                depth -= 1
            if depth == 1 and ch == ",":
                parts.append(cur.strip())
                cur = ""
            elif depth > 0:
                cur += ch
            i += 1
        parts.append(cur.strip())
        ret, tys, args = parts[0], parts[1], parts[2:]
        assert tys.startswith("(") and tys.endswith(")"), (m.group(1), tys)
        inner, depth, cur, types = tys[1:-1], 0, "", []
        for ch in inner + ",":
            if ch in "{(":
                depth += 1
            elif ch in "})":
                depth -= 1
            if ch == "," and depth == 0:
                if cur.strip():
                    types.append(cur.strip())
                cur = ""
            else:
                cur += ch
        out.append((m.group(1), ret, types, args))
    return out


def _c_kind(param):
    p = re.sub(r"\b(const|struct)\b", "", param).strip()
    if "*" in p:
        return "ptr"
    base = p.rsplit(None, 1)[0] if len(p.split()) > 1 else p
    return {"int": "i32", "unsigned": "u32", "int64_t": "i64", "size_t": "usize", "float": "f32"}[base.strip()]


def _julia_kind(t):
    if t.startswith(("Ptr{", "Ref{")) or t in ("Cstring",):
        return "ptr"
    return {"Cint": "i32", "Cuint": "u32", "Int64": "i64", "Csize_t": "usize", "Cfloat": "f32"}[t]


def test_julia_shim_ccall_types_match_header(pkg):
    """Every ccall in the Julia shim passes as many arguments as the C prototype has, each with a
    Julia type of the same C kind (pointer / int / unsigned / int64 / size_t / float), and
    returns Cint (or Cstring for dlrm_last_error)."""
    text = open(os.path.join(ROOT, "dlrm.jl_amd", "julia", "DLRMHip.jl")).read()
    hdr = re.sub(r"/\*.*?\*/", "", open(pkg._lib.HEADER).read(), flags=re.S)
    calls = _julia_ccalls(text)
    assert len(calls) >= 20
    for name, ret, types, args in calls:
        m = re.search(r"\b(?:int|const char\*)\s+" + name + r"\s*\(([^)]*)\)", hdr)
        assert m, f"{name}: no prototype in the header"
        params = [q for q in m.group(1).split(",") if q.strip() and q.strip() != "void"]
        assert len(types) == len(params), (name, types, params)
        assert len(args) == len(types), (name, "argument count != type tuple", args)
        for jt, cp in zip(types, params):
            assert _julia_kind(jt) == _c_kind(cp), (name, jt, cp)
        assert ret == ("Cstring" if name == "dlrm_last_error" else "Cint"), (name, ret)
