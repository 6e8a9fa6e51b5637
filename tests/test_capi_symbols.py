"""The drop-in boundary: libpt.so loads and exports every entry point include/pt.h declares, the
Python binding declares the same set, and the Node addon binds them (no device calls here)."""
import os
import re
import subprocess

import pytest

import helpers as H

HEADER = os.path.join(H.ROOT, "include", "pt.h")
PKG = os.path.join(H.ROOT, "babylon.js-pathtracing-renderer_amd")
LIB = os.path.join(PKG, "libpt.so")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pt_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_effect_api():
    names = declared()
    for must in ("pt_ctx_create", "pt_effect_create", "pt_set_float", "pt_set_int", "pt_set_texture",
                 "pt_texture_create_rgba32f", "pt_render_target_create", "pt_render", "pt_read_pixels"):
        assert must in names


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build libpt.so first (__graft_entry__.build())"
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], check=True, capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (pt_[a-z0-9_]+)$", out, flags=re.M))
    missing = [n for n in declared() if n not in exported]
    assert not missing, missing


def test_library_loads_and_python_binding_matches_header():
    import babylon_pt as bp
    L = bp.lib()                       # dlopen + argtypes only; no HIP call
    assert sorted(bp.SYMBOLS) == declared()
    for n in bp.SYMBOLS:
        assert hasattr(L, n)
    assert L.pt_version().decode().startswith("libpt")


def test_library_is_gfx950_code():
    """The .hip_fatbin carries a gfx950 code object and nothing for other targets."""
    blob = open(LIB, "rb").read()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in blob
    assert b"amdhsa--gfx942" not in blob and b"amdhsa--gfx90a" not in blob


def test_napi_addon_binds_every_symbol():
    src = open(os.path.join(PKG, "napi", "pt_napi.c")).read()
    for n in declared():
        if n in ("pt_math_probe", "pt_math_exhaustive"):
            continue
        assert n in src, n
