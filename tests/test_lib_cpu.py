"""CPU-side checks of the C-ABI library: it loads without a GPU and exports exactly what
include/pemp.h declares (no compute calls here)."""
import os
import re

from pemp_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "pemp.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"\b(pemp_[a-z0-9_]+)\s*\(", src))


def test_header_matches_binding_table():
    assert declared_functions() == set(_lib.SIGNATURES)


def test_library_loads_and_exports_every_symbol():
    L = _lib.load_cdll()
    for name in declared_functions():
        assert hasattr(L, name), name
    assert L.pemp_abi_version() == _lib.ABI_VERSION


def test_workspace_queries_are_host_only():
    L = _lib.load_cdll()
    assert L.pemp_detect_workspace_size(8, 17, 640, 640, 5) > 0
    assert L.pemp_detect_workspace_size(0, 17, 640, 640, 5) == 0
