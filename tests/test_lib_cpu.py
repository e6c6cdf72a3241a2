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


def test_knn_rows_layout_is_host_only():
    """pemp_knn_rows_layout (pemp_mpn_forward_knn's hand-over): the bit rows, row starts and edge counts lie
    inside the knn build's workspace without overlapping; an image over 512 nodes has no bit rows."""
    import ctypes
    import numpy as np
    L = _lib.load_cdll()
    for name in ("pemp_knn_workspace_size", "pemp_feature_knn_workspace_size"):
        getattr(L, name).restype = ctypes.c_size_t
    for feature in (0, 1):
        nh = np.array([0, 153, 153, 400, 912], np.int64)
        p = nh.ctypes.data_as(ctypes.c_void_p)
        offs = (ctypes.c_size_t * 3)()
        assert L.pemp_knn_rows_layout(p, 4, feature, offs) == 0
        size = (L.pemp_feature_knn_workspace_size if feature else L.pemp_knn_workspace_size)(p, 4)
        n = int(nh[-1])
        spans = sorted([(offs[0], 8 * 8 * n), (offs[1], 4 * n), (offs[2], 8 * 4)])
        assert all(a + la <= b for (a, la), (b, _) in zip(spans, spans[1:])) and spans[-1][0] + spans[-1][1] <= size
        assert offs[0] % 256 == 0 and offs[1] % 256 == 0 and offs[2] % 256 == 0
    nh = np.array([0, 513], np.int64)
    assert L.pemp_knn_rows_layout(nh.ctypes.data_as(ctypes.c_void_p), 1, 0, offs) != 0
