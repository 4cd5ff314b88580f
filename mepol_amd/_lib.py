"""ctypes binding of the C ABI declared in include/mepol_amd.h (libmepol_amd.so, gfx950).

There is no CPU fallback: if the library is missing or cannot be loaded, every op raises.
Build it with ``make`` (or ``__graft_entry__.build()``).
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MEPOL_AMD_LIB", os.path.join(_HERE, "libmepol_amd.so"))

_c_i64 = ctypes.c_int64
_c_int = ctypes.c_int
_c_dbl = ctypes.c_double
_c_sz = ctypes.c_size_t
_c_vp = ctypes.c_void_p

ABI_VERSION = 4  # include/mepol_amd.h MEPOL_ABI_VERSION

# name -> argtypes (restype is int unless listed in _RESTYPES)
SIGNATURES = {
    "mepol_last_error_string": [],
    "mepol_abi_version": [],
    "mepol_knn_workspace_size": [_c_i64, _c_i64, _c_int, _c_int, _c_int, ctypes.POINTER(_c_sz)],
    "mepol_knn_plan_info": [_c_i64, _c_i64, _c_int, _c_int, _c_int, ctypes.POINTER(_c_int),
                            ctypes.POINTER(_c_int), ctypes.POINTER(_c_int)],
    "mepol_knn": [_c_vp, _c_i64, _c_vp, _c_i64, _c_int, _c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp,
                  _c_vp, _c_sz, _c_vp],
    "mepol_knn_deferred": [_c_vp, _c_i64, _c_vp, _c_i64, _c_int, _c_int, _c_int, _c_vp, _c_vp,
                           _c_vp, _c_vp, _c_vp, _c_vp, _c_sz, _c_vp],
    "mepol_knn_exact": [_c_vp, _c_i64, _c_vp, _c_i64, _c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp,
                        _c_vp],
    "mepol_iw_forward": [_c_vp, _c_vp, _c_i64, _c_i64, _c_vp, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp,
                         _c_vp],
    "mepol_iw_normalize": [_c_vp, _c_vp, _c_i64, _c_vp, _c_vp],
    "mepol_entropy_partials_size": [_c_i64],
    "mepol_entropy_gamma_partials_size": [_c_i64],
    "mepol_entropy_forward": [_c_vp, _c_vp, _c_vp, _c_i64, _c_i64, _c_int, _c_int, _c_dbl, _c_dbl,
                              _c_dbl, _c_dbl, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp],
    "mepol_entropy_forward_emit": [_c_vp, _c_vp, _c_vp, _c_i64, _c_i64, _c_int, _c_int, _c_dbl, _c_dbl,
                              _c_dbl, _c_dbl, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp],
    "mepol_iw_normalize_gathered": [_c_vp, _c_int, _c_i64, _c_int, _c_vp, _c_vp],
    "mepol_sharded_emit": [_c_vp, _c_int, _c_i64, _c_i64, _c_dbl, _c_i64, _c_vp, _c_vp, _c_vp],
    "mepol_csr_workspace_size": [_c_i64, _c_int, _c_i64, ctypes.POINTER(_c_sz)],
    "mepol_csr_build": [_c_vp, _c_i64, _c_int, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_sz,
                        _c_vp],
    "mepol_entropy_gamma": [_c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_vp, _c_vp, _c_vp],
    "mepol_entropy_reverse_scan": [_c_vp, _c_vp, _c_vp, _c_i64, _c_vp, _c_vp, _c_i64, _c_i64,
                                   _c_vp, _c_vp, _c_vp],
    "mepol_head_forward": [_c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_vp,
                           _c_vp, _c_vp],
    "mepol_head_workspace_size": [_c_i64, _c_int, _c_int, ctypes.POINTER(_c_sz)],
    "mepol_head_backward": [_c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_int,
                            _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_sz, _c_vp],
    "mepol_head_backward_phase": [_c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp,
                                  _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_sz, _c_int,
                                  _c_vp],
    "mepol_weight_grad_workspace_size": [_c_i64, _c_int, _c_int, ctypes.POINTER(_c_sz)],
    "mepol_weight_grad": [_c_vp, _c_i64, _c_int, _c_vp, _c_int, _c_vp, _c_vp, _c_sz, _c_vp],
    "mepol_layer_forward": [_c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_int, _c_vp, _c_vp],
    "mepol_layer_workspace_size": [_c_i64, _c_int, _c_int, ctypes.POINTER(_c_sz)],
    "mepol_layer_backward": [_c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_sz,
                             _c_vp],
    "mepol_policy_forward": [_c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_int,
                             _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_vp, _c_vp,
                             _c_vp],
    "mepol_dh1_layer1_workspace_size": [_c_i64, _c_int, _c_int, ctypes.POINTER(_c_sz)],
    "mepol_dh1_layer1_backward": [_c_vp, _c_i64, _c_int, _c_vp, _c_int, _c_vp, _c_vp, _c_int,
                                  _c_vp, _c_vp, _c_vp, _c_sz, _c_vp],
    "mepol_dh1_layer1_backward_masked": [_c_vp, _c_i64, _c_int, _c_vp, _c_int, _c_vp, _c_vp,
                                         _c_int, _c_vp, _c_vp, _c_vp, _c_sz, _c_vp],
    "mepol_dh1_layer1_backward_w2": [_c_vp, _c_i64, _c_int, _c_vp, _c_int, _c_vp, _c_vp,
                                     _c_int, _c_vp, _c_vp, _c_vp, _c_sz, _c_vp],
    "mepol_policy_forward_masked": [_c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_int, _c_vp, _c_vp,
                                    _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_vp,
                                    _c_vp, _c_vp, _c_vp, _c_vp],
    "mepol_gemm_nt": [_c_vp, _c_i64, _c_int, _c_i64, _c_vp, _c_int, _c_i64, _c_vp, _c_int, _c_vp,
                      _c_i64, _c_int, _c_vp],
    "mepol_step_mountaincar": [_c_vp, _c_vp, _c_i64, _c_i64, _c_vp],
    "mepol_step_gridworld": [_c_vp, _c_vp, _c_i64, _c_vp],
    "mepol_rollout_step": [_c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_i64,
                           _c_i64, _c_vp, _c_vp, _c_vp, _c_vp],
    "mepol_rollout_mlp": [_c_int, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_vp,
                          _c_int, _c_vp, _c_vp, _c_vp, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp,
                          _c_vp, _c_sz, _c_vp],
    "mepol_rollout_mlp_workspace_size": [_c_i64, _c_i64, _c_int, _c_int, _c_int,
                                         ctypes.POINTER(_c_sz)],
    "mepol_rollout_mlp_plan_info": [_c_i64, _c_int, _c_int, _c_int, ctypes.POINTER(_c_int),
                                    ctypes.POINTER(_c_int)],
    "mepol_memcpy_async": [_c_vp, _c_vp, _c_sz, _c_vp],
    "mepol_optim_step": [_c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp],
    "mepol_optim_step_snapshot": [_c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp,
                                  _c_vp, _c_vp, _c_vp, _c_vp],
}
_RESTYPES = {"mepol_last_error_string": ctypes.c_char_p}

_lib = None
_lock = threading.Lock()


class MepolError(RuntimeError):
    pass


class MepolInputError(MepolError, ValueError):
    """MEPOL_ERR_BAD_ARG: invalid input (e.g. non-finite particles); a ValueError like the
    reference's sklearn check_array rejection."""


def load():
    """Load libmepol_amd.so (once) and bind every exported symbol; raise if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise MepolError(
                    f"{LIB_PATH} not found: the MI355X kernels are not built (run `make` or "
                    "__graft_entry__.build()); there is no CPU fallback")
            lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            for name, argtypes in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.argtypes = argtypes
                fn.restype = _RESTYPES.get(name, ctypes.c_int)
            got = lib.mepol_abi_version()
            if got != ABI_VERSION:
                raise MepolError(f"{LIB_PATH} has C ABI version {got}, this binding expects "
                                 f"{ABI_VERSION}: rebuild the library (make)")
            _lib = lib
    return _lib


def call(name, *args):
    """Invoke a C-ABI entry point; raise MepolError with the library's message on failure."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.mepol_last_error_string()
        cls = MepolInputError if rc == 1001 else MepolError
        raise cls(f"{name} failed (rc={rc}): {msg.decode() if msg else ''}")
    return rc


def ptr(t):
    """Device pointer of a tensor (or None) as a ctypes void pointer."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())
