"""The C-ABI library loads and exports exactly what include/sdnroute.h
declares; error paths that need no GPU behave as documented.  CPU only (no
compute call is made here)."""
import ctypes
import os
import re
import subprocess

import pytest

from sdnmpi_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sdnroute.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sdnr_[a-z_]+)\s*\(", text)))


def test_header_matches_binding_list():
    assert declared_functions() == sorted(_native.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    path = _native.library_path()
    assert os.path.exists(path), "build first: __graft_entry__.build()"
    out = subprocess.check_output(["nm", "-D", "--defined-only", path]).decode()
    exported = set(re.findall(r"\bT (sdnr_\w+)", out))
    missing = set(declared_functions()) - exported
    assert not missing, missing
    # nothing undeclared leaks into the C ABI
    assert exported - set(declared_functions()) == set()


def test_library_loads_and_reports_abi():
    L = _native.library()
    assert L.sdnr_abi_version() == _native.ABI_VERSION
    for name in declared_functions():
        assert hasattr(L, name)


def test_null_context_errors_without_gpu():
    L = _native.library()
    assert L.sdnr_synchronize(None) == -22
    assert b"null context" in L.sdnr_last_error()
    assert L.sdnr_graph_info(None, None, None, None) == -22
    assert L.sdnr_dfs_tables(None, None, 0, None, None, None, 0) == -22
    assert L.sdnr_destroy(None) == 0


def test_create_fails_loudly_without_device():
    if _native.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(_native.SdnrError) as ei:
        _native.Context(0)
    assert ei.value.code == -19


def test_built_for_gfx950_only():
    blob = open(_native.library_path(), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100", b"--gfx908"):
        assert other not in blob


def test_library_build_id_is_the_trees():
    """The loaded library was compiled from exactly these sources (the id is
    checked by the loader; here it is read both ways)."""
    from sdnmpi_amd import _buildinfo as B
    L = _native.library()
    want = B.tree_build_id()
    assert want is not None and len(want) == 64
    assert L.sdnr_build_id().decode() == want
    assert B.file_build_id(_native.library_path()) == want


def test_loader_refuses_stale_library(tmp_path):
    """Edit one hashed input (a copy of the tree's sources) and the loader's
    check refuses the library built from the unedited tree."""
    import shutil
    from sdnmpi_amd import _buildinfo as B
    L = _native.library()
    csrc, inc = tmp_path / "csrc", tmp_path / "include"
    shutil.copytree(B.CSRC, csrc)
    shutil.copytree(B.INCLUDE, inc)
    _native.verify_build(L, str(csrc), str(inc))          # identical copy: accepted
    for label, path in B.inputs(str(csrc), str(inc)):
        if label.endswith("dfs.hip"):
            with open(path, "a") as f:
                f.write("\n// edited\n")
    assert B.tree_build_id(str(csrc), str(inc)) != B.tree_build_id()
    with pytest.raises(_native.NativeUnavailable) as ei:
        _native.verify_build(L, str(csrc), str(inc))
    assert "stale" in str(ei.value)
