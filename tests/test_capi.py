"""CPU checks of the C-ABI boundary: the library builds, loads, and exports exactly
what include/nfsp.h declares (no compute calls -- no GPU here)."""
import ctypes
import os
import re

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "nfsp.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(nfsp_[a-z0-9_]+)\s*\(", src)))


def test_build_and_load(pkg):
    import __graft_entry__
    __graft_entry__.build()
    L = pkg.native.load()
    assert L.nfsp_version() == 1


def test_every_declared_symbol_exported_and_bound(pkg):
    L = pkg.native.load()
    decl = declared_symbols()
    assert len(decl) >= 19
    for name in decl:
        assert hasattr(L, name), name
        assert name in pkg.native.SIGNATURES, f"{name} not bound in native.py"
    assert sorted(pkg.native.SIGNATURES) == decl


def test_exports_are_c_abi(pkg):
    # no C++ mangling on the boundary: every nfsp_* symbol resolves by its plain name
    so = ctypes.CDLL(pkg.native.LIB_PATH)
    for name in declared_symbols():
        getattr(so, name)


def test_errors_without_gpu_are_loud(pkg):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(pkg.native.NativeError):
        pkg.native.lib()
    # argument validation works without a device
    L = pkg.native.load()
    assert L.nfsp_create(None, 1, 0, 0, 0) == pkg.native.EINVAL
    assert b"null" in L.nfsp_last_error()
    assert L.nfsp_env_reset(None, None) == pkg.native.EINVAL
    assert L.nfsp_exploitability(None, None, None, 0, None) == pkg.native.EINVAL
    assert L.nfsp_exploitability_batch(None, None, None, 1, 0, None) == pkg.native.EINVAL
    assert L.nfsp_group_create(None, None, 1, 0, None) == pkg.native.EINVAL


def test_hand_struct_layout_matches_device_header(pkg):
    hdr = open(os.path.join(REPO, os.path.basename(pkg.native.HERE), "csrc",
                            "nfsp_device.h")).read()
    assert "struct alignas(16) Hand" in hdr
    # field order in HAND_DTYPE mirrors the struct
    fields = ["hist", "s", "warn", "la", "rew", "rank", "dealer", "rnd", "term", "raises0",
              "raises1", "slot", "ndone", "done0", "done1", "done2", "c0", "c1", "pad"]
    import importlib
    le = importlib.import_module("nfsp_amd.leduc")
    assert list(le.HAND_DTYPE.names) == fields
    assert le.HAND_DTYPE.itemsize == 64


def _header_structs():
    """`typedef struct name { ... } name;` bodies of include/nfsp.h -> [(field, kind, dims)]."""
    import re
    src = open(os.path.join(REPO, "include", "nfsp.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    kinds = {"int32_t": "i32", "uint32_t": "u32", "int64_t": "i64", "uint64_t": "u64",
             "float": "f32", "double": "f64", "uint8_t": "u8"}
    out = {}
    for m in re.finditer(r"typedef struct (\w+) \{(.*?)\} \1;", src, re.S):
        fields = []
        for decl in m.group(2).split(";"):
            decl = decl.strip()
            if not decl:
                continue
            t, rest = decl.split(None, 1)
            for v in rest.split(","):
                v = v.strip()
                ptr = v.startswith("*") or t.endswith("*")
                name = re.match(r"\**\s*(\w+)", v).group(1)
                dims = tuple(int(d) for d in re.findall(r"\[(\d+)\]", v))
                fields.append((name, "ptr" if ptr else kinds[t.rstrip("*")], dims))
        out[m.group(1)] = fields
    return out


def _ctypes_fields(struct):
    import ctypes as C
    kinds = {C.c_int32: "i32", C.c_uint32: "u32", C.c_int64: "i64", C.c_uint64: "u64",
             C.c_float: "f32", C.c_double: "f64", C.c_uint8: "u8", C.c_void_p: "ptr"}
    out = []
    for name, t in struct._fields_:
        dims = []
        while hasattr(t, "_length_"):
            dims.append(t._length_)
            t = t._type_
        out.append((name, kinds[t], tuple(dims)))
    return out


def test_abi_structs_match_their_ctypes_mirrors(pkg):
    """Every struct of include/nfsp.h that native.py mirrors (nfsp_records, nfsp_engine_cfg,
    nfsp_engine_stats, nfsp_group_sched) has the same fields in the same order with the same
    types and shapes -- a field added on one side only (round 6: cfg.sched, sched.br_persist)
    would shift every later field."""
    import ctypes as C
    hdr = _header_structs()
    mirrors = {"nfsp_records": pkg.native.Records, "nfsp_engine_cfg": pkg.native.EngineCfg,
               "nfsp_engine_stats": pkg.native.EngineStats, "nfsp_group_sched": pkg.native.GroupSched}
    for name, st in mirrors.items():
        assert _ctypes_fields(st) == hdr[name], name
    assert C.sizeof(pkg.native.GroupSched) == 5 * 4
