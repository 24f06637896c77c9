"""Sparse format conversions on the device (include/lssp_amd.h, matrix-utils.h:22-49).

Inputs and outputs are device arrays (DIdx for the int members, DVec for the
values); nothing leaves HBM except the output sizes.  Same names and argument
meaning as the reference's lssp_mat_csr_to_coo / lssp_mat_coo_to_csr /
lssp_mat_transpose / lssp_mat_csr_to_bcsr / lssp_mat_bcsr_to_csr
(matrix-utils.cxx:62-380, :700-765); a malformed input raises LsspError
(LSSP_AMD_EINVAL) where the reference asserts, exits or reads out of bounds.
"""
from __future__ import annotations

import ctypes

from .device import DIdx, DVec, Device, _ck


def csr_to_coo(dev: Device, nrows: int, nnz: int, Ap: DIdx, Aj: DIdx, Ax: DVec):
    """-> (Ci, Cj, Cx); Cj / Cx are device copies of Aj / Ax (matrix-utils.cxx:281-322)"""
    Ci, Cj, Cx = dev.idx(nnz), dev.idx(nnz), dev.vec(nnz)
    _ck(dev.L.lssp_amd_csr_to_coo(dev.h, nrows, nnz, Ap.ptr, Aj.ptr, Ax.ptr, Ci.ptr, Cj.ptr, Cx.ptr),
        "csr_to_coo")
    return Ci, Cj, Cx


def coo_to_csr(dev: Device, nrows: int, nnz: int, Ci: DIdx, Cj: DIdx, Cx: DVec):
    """-> (Ap, Aj, Ax): stable bucketing by row (matrix-utils.cxx:324-380)"""
    Ap, Aj, Ax = dev.idx(nrows + 1), dev.idx(nnz), dev.vec(nnz)
    _ck(dev.L.lssp_amd_coo_to_csr(dev.h, nrows, nnz, Ci.ptr, Cj.ptr, Cx.ptr, Ap.ptr, Aj.ptr, Ax.ptr),
        "coo_to_csr")
    return Ap, Aj, Ax


def transpose(dev: Device, nrows: int, ncols: int, nnz: int, Ap: DIdx, Aj: DIdx, Ax: DVec):
    """-> (Tp, Tj, Tx) of the ncols x nrows transpose (matrix-utils.cxx:700-765)"""
    Tp, Tj, Tx = dev.idx(ncols + 1), dev.idx(nnz), dev.vec(nnz)
    _ck(dev.L.lssp_amd_csr_transpose(dev.h, nrows, ncols, nnz, Ap.ptr, Aj.ptr, Ax.ptr, Tp.ptr, Tj.ptr,
                                     Tx.ptr), "csr_transpose")
    return Tp, Tj, Tx


def csr_to_bcsr(dev: Device, n: int, nnz: int, bs: int, Ap: DIdx, Aj: DIdx, Ax: DVec):
    """-> (bnnz, Bp, Bj, Bx): bs x bs column-major blocks (matrix-utils.cxx:62-162)"""
    m = ctypes.c_int()
    _ck(dev.L.lssp_amd_csr_to_bcsr(dev.h, n, nnz, bs, Ap.ptr, Aj.ptr, Ax.ptr, ctypes.byref(m), None, None,
                                   None), "csr_to_bcsr")
    Bp, Bj, Bx = dev.idx(n // bs + 1), dev.idx(m.value), dev.vec(m.value * bs * bs)
    _ck(dev.L.lssp_amd_csr_to_bcsr(dev.h, n, nnz, bs, Ap.ptr, Aj.ptr, Ax.ptr, ctypes.byref(m), Bp.ptr,
                                   Bj.ptr, Bx.ptr), "csr_to_bcsr")
    return m.value, Bp, Bj, Bx


def bcsr_to_csr(dev: Device, nbrows: int, nbcols: int, bs: int, bnnz: int, Bp: DIdx, Bj: DIdx, Bx: DVec):
    """-> (nnz, Ap, Aj, Ax): entries with fabs(v) > 0, columns sorted (matrix-utils.cxx:164-215)"""
    m = ctypes.c_int()
    Ap = dev.idx(nbrows * bs + 1)
    _ck(dev.L.lssp_amd_bcsr_to_csr(dev.h, nbrows, nbcols, bs, bnnz, Bp.ptr, Bj.ptr, Bx.ptr, ctypes.byref(m),
                                   Ap.ptr, None, None), "bcsr_to_csr")
    Aj, Ax = dev.idx(m.value), dev.vec(m.value)
    _ck(dev.L.lssp_amd_bcsr_to_csr(dev.h, nbrows, nbcols, bs, bnnz, Bp.ptr, Bj.ptr, Bx.ptr, ctypes.byref(m),
                                   Ap.ptr, Aj.ptr, Ax.ptr), "bcsr_to_csr")
    return m.value, Ap, Aj, Ax
