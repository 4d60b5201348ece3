"""libspx.so loads without a GPU and exports every entry point of include/spx.h."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "spx.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(spx_[a-z_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    fns = header_functions()
    for name in ("spx_create", "spx_load", "spx_solve", "spx_pivot", "spx_get_tableau",
                 "spx_get_basis", "spx_destroy", "spx_last_error", "spx_create_sharded",
                 "spx_comm_unique_id", "spx_load_rows", "spx_pivot_at", "spx_run_pivots"):
        assert name in fns


def test_library_exports_every_header_symbol():
    from simplex_amd import _lib
    lib = _lib.lib()
    for name in header_functions():
        assert hasattr(lib, name), name
        assert name in _lib.SIGNATURES, f"{name} not bound in _lib.SIGNATURES"
    assert lib.spx_abi_version() == 1
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (spx_\w+)", out))
    assert set(header_functions()) <= exported


def test_default_opts_host_only():
    from simplex_amd import _lib
    o = _lib.default_opts()
    assert (o.rule, o.skip_zero_cols, o.eps_opt, o.eps_piv, o.chunk, o.use_graph) == \
        (0, 1, 1e-9, 1e-12, 32, 1)


def test_lib_embeds_gfx950_code_object():
    from simplex_amd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_missing_library_fails_loudly(monkeypatch):
    from simplex_amd import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", "/nonexistent/libspx.so")
    with pytest.raises(_lib.SpxLibraryError):
        _lib.lib()
