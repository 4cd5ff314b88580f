"""The C-ABI library loads and exports exactly the entry points include/mepol_amd.h declares
(no compute calls: this runs without a GPU)."""
import ctypes
import os
import re

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "mepol_amd.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mepol_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_hot_path():
    names = declared_functions()
    for required in ["mepol_knn", "mepol_iw_forward", "mepol_entropy_forward", "mepol_csr_build",
                     "mepol_entropy_gamma", "mepol_entropy_reverse_scan", "mepol_step_mountaincar",
                     "mepol_step_gridworld", "mepol_rollout_step", "mepol_last_error_string"]:
        assert required in names


def test_library_exports_every_declared_symbol():
    from mepol_amd import _lib

    lib = _lib.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
        assert name in _lib.SIGNATURES, f"{name} missing from the ctypes signature table"
    assert lib.mepol_abi_version() == 4


def test_nm_symbols_are_c_linkage():
    from mepol_amd import _lib

    out = os.popen(f"nm -D --defined-only {_lib.LIB_PATH}").read()
    exported = set(re.findall(r"\bT (mepol_[a-z0-9_]+)\b", out))
    assert set(declared_functions()) <= exported


def test_bad_arguments_fail_loudly_without_gpu():
    """Argument validation happens on the host before any launch."""
    from mepol_amd import _lib

    lib = _lib.load()
    n = ctypes.c_size_t()
    rc = lib.mepol_knn_workspace_size(10, 10, 3, 50, 0, ctypes.byref(n))  # k+1 > n
    assert rc == 1001
    assert b"n_neighbors" in lib.mepol_last_error_string()
    # any d and any k+1 <= n have a plan (the exhaustive one beyond the f16 screen's shapes)
    for nn, d, kp1 in [(1000, 200, 5), (1000, 29, 101), (1000, 3, 1000)]:
        rc = lib.mepol_knn_workspace_size(nn, nn, d, kp1, 0, ctypes.byref(n))
        assert rc == 0 and n.value >= nn * d * 4
        ks, lst, sp = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        assert lib.mepol_knn_plan_info(nn, nn, d, kp1, 0, ctypes.byref(ks), ctypes.byref(lst),
                                       ctypes.byref(sp)) == 0
        assert ks.value == 0 and lst.value >= kp1
    rc = lib.mepol_knn_workspace_size(2 ** 31, 10, 3, 5, 0, ctypes.byref(n))  # int32 indices
    assert rc == 1003
    rc = lib.mepol_knn_workspace_size(200000, 200000, 29, 31, 0, ctypes.byref(n))
    assert rc == 0 and n.value > 200000 * 31 * 8
