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


def test_edge_cu_reservation_is_a_bounded_share():
    """The edge passes' CU reservation (mpn.hip edge_cus): small graphs keep every CU; large ones leave at most a
    quarter of the device free (a multiple of 8), whatever is asked, so a small device or a compute partition keeps
    at least 3/4 of its CUs for the forward (a fixed 64 would take most of such a device)."""
    L = _lib.load_cdll()
    pol = L.pemp_edge_cus_policy
    assert pol(256, 186_048, 64) == 192          # MI355X, c3: 64 reserved (the measured default)
    assert pol(256, 22_350, 64) == 256           # batch 1: every CU
    assert pol(256, 186_048, 0) == 256
    assert pol(256, 186_048, 200) == 192         # capped at a quarter
    for cus in (8, 16, 38, 40, 64, 80, 120, 152, 228, 256, 304):
        for E in (0, 65_535, 65_536, 250_000, 10**8):
            for req in (0, 7, 8, 64, 96, 10**6):
                n = pol(cus, E, req)
                assert 0.75 * cus <= n <= cus and (cus - n) % 8 == 0, (cus, E, req, n)
                if E < 65_536:
                    assert n == cus
    assert pol(0, 1000, 64) < 0 and pol(256, -1, 64) < 0


def test_ctypes_struct_mirrors_match_the_library():
    """The ctypes mirrors of the ABI structs have the library's sizes (a field added on one side only would shift
    every later field of the struct the kernels read)."""
    import ctypes
    L = _lib.load_cdll()
    for which, cls in enumerate((_lib.PempMpnWeights, _lib.PempMpnDesc, _lib.PempMlp, _lib.PempProjMaps,
                                 _lib.PempStepPlan)):
        assert L.pemp_abi_struct_size(which) == ctypes.sizeof(cls), cls.__name__
    assert L.pemp_abi_struct_size(7) == 0


def test_step_layout_is_host_arithmetic():
    """pemp_step_layout (host only): every output of the batch-step entry at a 256-byte aligned offset, in order,
    without overlap; the logit arrays laid out as mpn/model.py's forward lays them (64-element boundaries)."""
    import ctypes
    L = _lib.load_cdll()
    desc = _lib.PempMpnDesc(17, 17, 3, 1, 3, 64, 19, 128, 2, 3, _lib.MPN_COUNTS_IN_OFFSETS)
    p = _lib.PempStepPlan(B=8, J=17, H=640, W=640, pool_kernel=5, use_threshold=1, topk=5, det_cap=512, threshold=0.1,
                          C=128, F=1, A=19, mode=0, norm_factor=640.0, n_cap=1546, e_cap=232_846)
    p.desc = ctypes.pointer(desc)
    n = L.pemp_step_layout(ctypes.byref(p))
    assert n == p.bytes and n % 256 == 0
    sizes = [8 * 512 * 3 * 8, 8 * 512 * 4, 8 * 4, 1546 * 128 * 4, 1546 * 24, 1546 * 4, 1546 * 8, 1546 * 4,
             2 * 232_846 * 8, 232_846 * 19 * 4, 12 * 8]
    for i, sz in enumerate(sizes):
        assert p.off[i] % 256 == 0 and p.off[i] + sz <= p.off[i + 1], i
    assert p.n_rec == 2                          # T = 3, AUX_LOSS_STEPS 1: iterations 1 and 2 recorded
    ne, nn = 2 * 232_846, 3 * 1546
    assert (p.elog_n, p.nlog_off) == (ne, (ne + 63) // 64 * 64)
    assert p.clog_off == p.nlog_off + (nn + 63) // 64 * 64
    assert p.off[_lib.STEP_LOGITS] + 4 * (p.clog_off + nn * 17) <= n
    p.B = 0
    assert L.pemp_step_layout(ctypes.byref(p)) == 0
