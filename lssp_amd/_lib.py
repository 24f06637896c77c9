"""ctypes binding of lssp_amd/lib/liblssp_amd.so (declared in include/lssp_amd.h).

The HIP library is the product: there is no CPU fallback.  If the library is
missing or cannot be loaded, importing this module raises, loudly.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# LSSP_AMD_LIB: another build of the same library (tuning experiments, tools/build_variant.sh)
LIB_PATH = os.environ.get("LSSP_AMD_LIB") or os.path.join(HERE, "lib", "liblssp_amd.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "lssp_amd.h")

_vp, _ci, _cd, _cl = ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_long
_pvp = ctypes.POINTER(ctypes.c_void_p)


ALLGATHER_FN = ctypes.CFUNCTYPE(_ci, _vp, _vp, _vp, _cl)
SENDRECV_FN = ctypes.CFUNCTYPE(_ci, _vp, _ci, ctypes.POINTER(_ci), ctypes.POINTER(_vp), ctypes.POINTER(_cl),
                               _ci, ctypes.POINTER(_ci), ctypes.POINTER(_vp), ctypes.POINTER(_cl))


class HostTransport(ctypes.Structure):
    """lssp_amd_host_transport (include/lssp_amd.h)"""
    _fields_ = [("user", _vp), ("allgather", ALLGATHER_FN), ("sendrecv", SENDRECV_FN)]


class SolveParams(ctypes.Structure):
    _fields_ = [("solver", _ci), ("tol_rel", _cd), ("tol_abs", _cd), ("tol_rb", _cd),
                ("maxit", _ci), ("restart", _ci), ("verb", _ci), ("aug_k", _ci),
                ("bgsl", _ci), ("idrs", _ci)]


# name -> (restype, argtypes); every symbol declared in include/lssp_amd.h
SIGNATURES = {
    "lssp_amd_strerror": (ctypes.c_char_p, [_ci]),
    "lssp_amd_version": (_ci, []),
    "lssp_amd_set_print": (None, [_vp, _vp]),
    "lssp_amd_ctx_create": (_ci, [_ci, _pvp]),
    "lssp_amd_ctx_destroy": (_ci, [_vp]),
    "lssp_amd_ctx_set_reduction": (_ci, [_vp, _ci]),
    "lssp_amd_ctx_sync": (_ci, [_vp]),
    "lssp_amd_ctx_stream": (_vp, [_vp]),
    "lssp_amd_vec_alloc": (_ci, [_vp, _cl, _pvp]),
    "lssp_amd_vec_free": (_ci, [_vp, _vp]),
    "lssp_amd_vec_upload": (_ci, [_vp, _vp, _vp, _cl]),
    "lssp_amd_vec_download": (_ci, [_vp, _vp, _vp, _cl]),
    "lssp_amd_csr_sort_columns": (_ci, [_ci, _ci, _vp, _vp, _vp]),
    "lssp_amd_mat_upload": (_ci, [_vp, _ci, _ci, _ci, _vp, _vp, _vp, _pvp]),
    "lssp_amd_mat_destroy": (_ci, [_vp]),
    "lssp_amd_mat_info": (_ci, [_vp, _vp, _vp, _vp]),
    "lssp_amd_mat_layout": (_ci, [_vp, _vp, _vp]),
    "lssp_amd_mat_bytes": (_ci, [_vp, _vp, _vp]),
    "lssp_amd_ilu_sweep_layout": (_ci, [_vp, _vp, _vp, _vp]),
    "lssp_amd_mv_amxpby": (_ci, [_vp, _cd, _vp, _vp, _cd, _vp]),
    "lssp_amd_mv_amxpbyz": (_ci, [_vp, _cd, _vp, _vp, _cd, _vp, _vp]),
    "lssp_amd_mv_amxy": (_ci, [_vp, _cd, _vp, _vp, _vp]),
    "lssp_amd_mv_mxy": (_ci, [_vp, _vp, _vp, _vp]),
    "lssp_amd_vec_set_value": (_ci, [_vp, _vp, _cl, _cd]),
    "lssp_amd_vec_copy": (_ci, [_vp, _vp, _vp, _cl]),
    "lssp_amd_stream_read": (_ci, [_vp, _vp, _cl, _vp]),
    "lssp_amd_vec_axy": (_ci, [_vp, _cd, _vp, _vp, _cl]),
    "lssp_amd_vec_axpby": (_ci, [_vp, _cd, _vp, _cd, _vp, _cl]),
    "lssp_amd_vec_axpbyz": (_ci, [_vp, _cd, _vp, _cd, _vp, _vp, _cl]),
    "lssp_amd_vec_scale": (_ci, [_vp, _vp, _cl, _cd]),
    "lssp_amd_vec_dot": (_ci, [_vp, _vp, _vp, _cl, _vp]),
    "lssp_amd_vec_norm": (_ci, [_vp, _vp, _cl, _vp]),
    "lssp_amd_ilu_create": (_ci, [_vp, _ci, _ci, _vp, _vp, _vp, _ci, _cd, _ci, _ci, _pvp]),
    "lssp_amd_ilu_from_factors": (_ci, [_vp, _ci, _vp, _vp, _vp, _vp, _vp, _vp, _pvp]),
    "lssp_amd_ilu_destroy": (_ci, [_vp]),
    "lssp_amd_ilu_apply": (_ci, [_vp, _vp, _vp, _vp]),
    "lssp_amd_ilu_apply_async": (_ci, [_vp, _vp, _vp, _vp]),
    "lssp_amd_ilu_check": (_ci, [_vp, _vp]),
    "lssp_amd_ilu_trisolve": (_ci, [_vp, _vp, _ci, _vp, _vp]),
    "lssp_amd_ilu_info": (_ci, [_vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "lssp_amd_ilu_get_factors": (_ci, [_vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "lssp_amd_solve": (_ci, [_vp, _vp, _vp, ctypes.POINTER(SolveParams), _vp, _vp, _vp, _vp, _vp, _ci, _vp]),
    "lssp_amd_comm_unique_id_size": (_ci, []),
    "lssp_amd_comm_get_unique_id": (_ci, [_vp]),
    "lssp_amd_comm_init": (_ci, [_vp, _ci, _ci, _vp]),
    "lssp_amd_comm_barrier": (_ci, [_vp]),
    "lssp_amd_comm_selftest": (_ci, [_vp]),
    "lssp_amd_comm_nranks": (_ci, [_vp, _vp]),
    "lssp_amd_comm_init_host": (_ci, [_vp, _ci, _ci, _vp]),
    "lssp_amd_mat_upload_dist": (_ci, [_vp, _ci, _ci, _ci, _vp, _vp, _vp, _pvp]),
    "lssp_amd_mat_local_rows": (_ci, [_vp, _vp, _vp, _vp]),
    "lssp_amd_idx_alloc": (_ci, [_vp, _cl, _pvp]),
    "lssp_amd_idx_free": (_ci, [_vp, _vp]),
    "lssp_amd_idx_upload": (_ci, [_vp, _vp, _vp, _cl]),
    "lssp_amd_idx_download": (_ci, [_vp, _vp, _vp, _cl]),
    "lssp_amd_csr_to_coo": (_ci, [_vp, _ci, _ci, _vp, _vp, _vp, _vp, _vp, _vp]),
    "lssp_amd_coo_to_csr": (_ci, [_vp, _ci, _ci, _vp, _vp, _vp, _vp, _vp, _vp]),
    "lssp_amd_csr_transpose": (_ci, [_vp, _ci, _ci, _ci, _vp, _vp, _vp, _vp, _vp, _vp]),
    "lssp_amd_csr_to_bcsr": (_ci, [_vp, _ci, _ci, _ci, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "lssp_amd_bcsr_to_csr": (_ci, [_vp, _ci, _ci, _ci, _ci, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "lssp_amd_poisson_nnz": (_cl, [_ci, _ci]),
    "lssp_amd_poisson_rows": (_ci, [_ci, _ci, _cl, _cl, _vp, _vp, _vp]),
}

_lib = None


def load() -> ctypes.CDLL:
    """Load the HIP library (once).  Raises if it is absent: no fallback."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"lssp_amd: HIP library not built: {LIB_PATH} "
                          "(run `make -C lssp_amd/csrc` or __graft_entry__.build())")
    # torch (when present) owns the process's HIP runtime; load it first so the
    # library binds to the same libamdhip64 / librccl (identical sonames)
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is plumbing only
        pass
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib
