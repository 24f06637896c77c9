"""Thin Python handles over the C-ABI (device context, vectors, CSR, ILU, solve).

Everything computes in lssp_amd/lib/liblssp_amd.so on the GPU; this module
only moves numpy arrays across the boundary and turns status codes into
exceptions (the reference would lssp_error() -> exit(1), utils.cxx:114-135).
"""
from __future__ import annotations

import ctypes
import weakref
from dataclasses import dataclass

import numpy as np

from . import _lib

GMRES, LGMRES, RGMRES, BICGSTAB, CG = 0, 1, 2, 4, 7
BICGSAFE, CGS, GPBICG, CR, CRS, BICRSTAB, BICRSAFE, GPBICR, QMRCGSTAB, TFQMR, ORTHOMIN = (
    6, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17)  # LSSP_SOLVER_TYPE (type-defs.h:157-178)
BICGSTABL, IDRS = 5, 18
ILUK, ILUT = 1, 2                  # LSSP_PC_TYPE (type-defs.h:63-101)
SERIAL, TREE = 0, 1                # reduction order


class LsspError(RuntimeError):
    def __init__(self, status: int, what: str):
        msg = _lib.load().lssp_amd_strerror(status).decode()
        super().__init__(f"{what}: {msg} (status {status})")
        self.status = status


def _ck(status: int, what: str):
    if status != 0:
        raise LsspError(status, what)


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


class Device:
    """One GPU context (device + HIP stream + reduction scratch)."""

    def __init__(self, device: int = 0, reduction: int = TREE):
        self.L = _lib.load()
        h = ctypes.c_void_p()
        _ck(self.L.lssp_amd_ctx_create(device, ctypes.byref(h)), "ctx_create")
        self.h = h
        self._children = weakref.WeakSet()  # closed before the context goes away
        self.set_reduction(reduction)

    def _adopt(self, obj):
        self._children.add(obj)
        return obj

    def set_reduction(self, mode: int):
        _ck(self.L.lssp_amd_ctx_set_reduction(self.h, mode), "set_reduction")
        self.reduction = mode

    def sync(self):
        _ck(self.L.lssp_amd_ctx_sync(self.h), "sync")

    @property
    def stream(self) -> int:
        return self.L.lssp_amd_ctx_stream(self.h) or 0

    def close(self):
        if self.h:
            for child in list(self._children):
                child.close()
            self.L.lssp_amd_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- vectors ----------------------------------------------------------
    def vec(self, n: int, data=None) -> "DVec":
        v = DVec(self, n)
        if data is not None:
            v.upload(data)
        return v

    def idx(self, n: int, data=None) -> "DIdx":
        v = DIdx(self, n)
        if data is not None:
            v.upload(data)
        return v

    # ---- comm ------------------------------------------------------------------
    def comm_init(self, nranks: int, rank: int, uid: bytes):
        buf = ctypes.create_string_buffer(uid, len(uid))
        _ck(self.L.lssp_amd_comm_init(self.h, nranks, rank, buf), "comm_init")

    def comm_init_host(self, nranks: int, rank: int, transport):
        """multi-rank protocol over a host-staged transport (e.g. lssp_amd.dist.GlooTransport)"""
        self._transport = transport  # keeps the ctypes callbacks alive
        _ck(self.L.lssp_amd_comm_init_host(self.h, nranks, rank, ctypes.byref(transport.struct)),
            "comm_init_host")

    def barrier(self):
        _ck(self.L.lssp_amd_comm_barrier(self.h), "barrier")

    def comm_nranks(self) -> int:
        """the communicator's rank count (ncclCommCount on RCCL; the host transport's count)"""
        v = ctypes.c_int()
        _ck(self.L.lssp_amd_comm_nranks(self.h, ctypes.byref(v)), "comm_nranks")
        return v.value

    def comm_selftest(self):
        """all-gather + grouped send/recv ring through the configured transport, checked"""
        _ck(self.L.lssp_amd_comm_selftest(self.h), "comm_selftest")


def comm_unique_id() -> bytes:
    L = _lib.load()
    n = L.lssp_amd_comm_unique_id_size()
    buf = ctypes.create_string_buffer(n)
    _ck(L.lssp_amd_comm_get_unique_id(buf), "get_unique_id")
    return buf.raw


class DVec:
    """A device fp64 vector (lssp_vec with d in HBM)."""

    def __init__(self, dev: Device, n: int):
        self.dev, self.n = dev, int(n)
        p = ctypes.c_void_p()
        _ck(dev.L.lssp_amd_vec_alloc(dev.h, self.n, ctypes.byref(p)), "vec_alloc")
        self.ptr = p
        dev._adopt(self)

    def upload(self, a):
        a = _f64(a)
        assert a.size <= self.n
        _ck(self.dev.L.lssp_amd_vec_upload(self.dev.h, self.ptr, _p(a), a.size), "vec_upload")
        return self

    def download(self, n: int | None = None) -> np.ndarray:
        out = np.empty(self.n if n is None else n)
        _ck(self.dev.L.lssp_amd_vec_download(self.dev.h, _p(out), self.ptr, out.size), "vec_download")
        return out

    def free(self):
        if self.ptr:
            self.dev.L.lssp_amd_vec_free(self.dev.h, self.ptr)
            self.ptr = None

    close = free

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class DIdx(DVec):
    """A device int32 array (the Ap / Aj / Ai members of a matrix in HBM)."""

    def __init__(self, dev: Device, n: int):
        self.dev, self.n = dev, int(n)
        p = ctypes.c_void_p()
        _ck(dev.L.lssp_amd_idx_alloc(dev.h, self.n, ctypes.byref(p)), "idx_alloc")
        self.ptr = p
        dev._adopt(self)

    def upload(self, a):
        a = _i32(a)
        assert a.size <= self.n
        _ck(self.dev.L.lssp_amd_idx_upload(self.dev.h, self.ptr, _p(a), a.size), "idx_upload")
        return self

    def download(self, n: int | None = None) -> np.ndarray:
        out = np.empty(self.n if n is None else n, np.int32)
        _ck(self.dev.L.lssp_amd_idx_download(self.dev.h, _p(out), self.ptr, out.size), "idx_download")
        return out

    def free(self):
        if self.ptr:
            self.dev.L.lssp_amd_idx_free(self.dev.h, self.ptr)
            self.ptr = None

    close = free


class DMat:
    """A device CSR matrix (lssp_mat_csr in HBM), entry order as given."""

    def __init__(self, dev: Device, Ap, Aj, Ax, ncols: int | None = None, dist=None):
        self.dev = dev
        Ap, Aj, Ax = _i32(Ap), _i32(Aj), _f64(Ax)
        h = ctypes.c_void_p()
        if dist is None:
            n = Ap.size - 1
            ncols = n if ncols is None else ncols
            _ck(dev.L.lssp_amd_mat_upload(dev.h, n, ncols, int(Ap[-1]), _p(Ap), _p(Aj), _p(Ax),
                                          ctypes.byref(h)), "mat_upload")
        else:
            n_global, row0 = dist
            _ck(dev.L.lssp_amd_mat_upload_dist(dev.h, n_global, row0, Ap.size - 1, _p(Ap), _p(Aj), _p(Ax),
                                               ctypes.byref(h)), "mat_upload_dist")
        self.h = h
        dev._adopt(self)
        r0, nl, nh = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        dev.L.lssp_amd_mat_local_rows(h, ctypes.byref(r0), ctypes.byref(nl), ctypes.byref(nh))
        self.row0, self.nrows, self.nhalo = r0.value, nl.value, nh.value
        self.nnz = int(Ap[-1])

    @property
    def nx(self) -> int:
        """length a vector multiplied by this matrix must have (owned + halo)"""
        return self.nrows + self.nhalo

    @property
    def ndiag(self) -> int:
        """> 0: the SpMV reads 1-byte diagonal ids (that many offsets) instead of columns"""
        v, w = ctypes.c_int(), ctypes.c_int()
        _ck(self.dev.L.lssp_amd_mat_layout(self.h, ctypes.byref(v), ctypes.byref(w)), "mat_layout")
        return v.value

    @property
    def windowed(self) -> bool:
        """the SpMV stages each 1024-row block's x span in LDS (k_spmv_win)"""
        v, w = ctypes.c_int(), ctypes.c_int()
        _ck(self.dev.L.lssp_amd_mat_layout(self.h, ctypes.byref(v), ctypes.byref(w)), "mat_layout")
        return bool(w.value)

    @property
    def device_bytes(self) -> tuple[int, int]:
        """(resident CSR bytes, bytes of the SpMV layouts beside it)"""
        c, a = ctypes.c_longlong(), ctypes.c_longlong()
        _ck(self.dev.L.lssp_amd_mat_bytes(self.h, ctypes.byref(c), ctypes.byref(a)), "mat_bytes")
        return c.value, a.value

    def close(self):
        if self.h:
            self.dev.L.lssp_amd_mat_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # mvops.h:9-19
    def mv_amxpby(self, alpha, x: DVec, beta, y: DVec):
        _ck(self.dev.L.lssp_amd_mv_amxpby(self.dev.h, alpha, self.h, x.ptr, beta, y.ptr), "mv_amxpby")

    def mv_amxpbyz(self, alpha, x: DVec, beta, y: DVec, z: DVec):
        _ck(self.dev.L.lssp_amd_mv_amxpbyz(self.dev.h, alpha, self.h, x.ptr, beta, y.ptr, z.ptr), "mv_amxpbyz")

    def mv_amxy(self, a, x: DVec, y: DVec):
        _ck(self.dev.L.lssp_amd_mv_amxy(self.dev.h, a, self.h, x.ptr, y.ptr), "mv_amxy")

    def mv_mxy(self, x: DVec, y: DVec):
        _ck(self.dev.L.lssp_amd_mv_mxy(self.dev.h, self.h, x.ptr, y.ptr), "mv_mxy")


class DILU:
    """Device ILU factors + their sync-free trisolve schedules (LSSP_PC.L/.U)."""

    def __init__(self, dev: Device, handle):
        self.dev, self.h = dev, handle
        dev._adopt(self)
        n, nl, nu, ll, lu, ts = (ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int(),
                                 ctypes.c_int(), ctypes.c_double())
        dev.L.lssp_amd_ilu_info(handle, ctypes.byref(n), ctypes.byref(nl), ctypes.byref(nu),
                                ctypes.byref(ll), ctypes.byref(lu), ctypes.byref(ts))
        self.n, self.nnzL, self.nnzU = n.value, nl.value, nu.value
        self.levelsL, self.levelsU, self.setup_seconds = ll.value, lu.value, ts.value

    def sweep_layout(self):
        """(line sweeps: 0 none, 1 ILU(0) grid, 2 ILU(1) grid; tile lines, tile planes)
        -- lssp_amd_ilu_sweep_layout."""
        a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _ck(self.dev.L.lssp_amd_ilu_sweep_layout(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)),
            "ilu_sweep_layout")
        return a.value, b.value, c.value

    @classmethod
    def create(cls, dev: Device, Ap, Aj, Ax, kind=ILUK, level=0, tol=1e-3, p=-1, blk=0):
        Ap, Aj, Ax = _i32(Ap), _i32(Aj), _f64(Ax)
        h = ctypes.c_void_p()
        _ck(dev.L.lssp_amd_ilu_create(dev.h, kind, Ap.size - 1, _p(Ap), _p(Aj), _p(Ax), level, tol, p, blk,
                                      ctypes.byref(h)), "ilu_create")
        return cls(dev, h)

    @classmethod
    def from_factors(cls, dev: Device, L, U):
        Lp, Lj, Lx = _i32(L[0]), _i32(L[1]), _f64(L[2])
        Up, Uj, Ux = _i32(U[0]), _i32(U[1]), _f64(U[2])
        h = ctypes.c_void_p()
        _ck(dev.L.lssp_amd_ilu_from_factors(dev.h, Lp.size - 1, _p(Lp), _p(Lj), _p(Lx), _p(Up), _p(Uj), _p(Ux),
                                            ctypes.byref(h)), "ilu_from_factors")
        return cls(dev, h)

    def factors(self):
        n = self.n
        Lp, Lj, Lx = np.zeros(n + 1, np.int32), np.zeros(self.nnzL, np.int32), np.zeros(self.nnzL)
        Up, Uj, Ux = np.zeros(n + 1, np.int32), np.zeros(self.nnzU, np.int32), np.zeros(self.nnzU)
        _ck(self.dev.L.lssp_amd_ilu_get_factors(self.h, _p(Lp), _p(Lj), _p(Lx), _p(Up), _p(Uj), _p(Ux)),
            "ilu_get_factors")
        return (Lp, Lj, Lx), (Up, Uj, Ux)

    def apply(self, x: DVec, rhs: DVec):
        """x = U^-1 L^-1 rhs (lssp_pc_ilu_solve, solver-tri.cxx:57-60)"""
        _ck(self.dev.L.lssp_amd_ilu_apply(self.dev.h, self.h, x.ptr, rhs.ptr), "ilu_apply")

    def apply_async(self, x: DVec, rhs: DVec):
        """the apply enqueued without waiting (lssp_amd_ilu_apply_async); check() reports timeouts"""
        _ck(self.dev.L.lssp_amd_ilu_apply_async(self.dev.h, self.h, x.ptr, rhs.ptr), "ilu_apply_async")

    def check(self):
        _ck(self.dev.L.lssp_amd_ilu_check(self.dev.h, self.h), "ilu_check")

    def trisolve(self, which: int, x: DVec, rhs: DVec):
        _ck(self.dev.L.lssp_amd_ilu_trisolve(self.dev.h, self.h, which, x.ptr, rhs.ptr), "ilu_trisolve")

    def close(self):
        if self.h:
            self.dev.L.lssp_amd_ilu_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class Result:
    nits: int
    residual: float
    trace: np.ndarray


def solve(dev: Device, A: DMat, M: DILU | None, x: DVec, b: DVec, solver=BICGSTAB, tol_rel=1e-7,
          tol_abs=1e-7, tol_rb=1e-7, maxit=1000, restart=-1, verb=0, trace_cap=0, aug_k=3, bgsl=4,
          idrs=4) -> Result:
    prm = _lib.SolveParams(solver, tol_rel, tol_abs, tol_rb, maxit, restart, verb, aug_k, bgsl, idrs)
    it, res, tl = ctypes.c_int(), ctypes.c_double(), ctypes.c_int()
    tr = np.zeros(max(trace_cap, 1))
    _ck(dev.L.lssp_amd_solve(dev.h, A.h, M.h if M is not None else None, ctypes.byref(prm), x.ptr, b.ptr,
                             ctypes.byref(it), ctypes.byref(res), _p(tr) if trace_cap else None, trace_cap,
                             ctypes.byref(tl)), "solve")
    return Result(it.value, res.value, tr[: min(tl.value, trace_cap)].copy() if trace_cap else np.zeros(0))


def poisson(dim: int, N: int, row0: int = 0, nrows: int | None = None):
    """Rows [row0, row0+nrows) of the 5-pt (dim 2, exam.cxx:4-59) / 7-pt Laplacian."""
    L = _lib.load()
    n = N ** dim
    nrows = n - row0 if nrows is None else nrows
    cap = min(7 if dim == 3 else 5, 7) * nrows
    Ap = np.zeros(nrows + 1, np.int32)
    Aj = np.zeros(cap, np.int32)
    Ax = np.zeros(cap)
    _ck(L.lssp_amd_poisson_rows(dim, N, row0, nrows, _p(Ap), _p(Aj), _p(Ax)), "poisson_rows")
    nnz = int(Ap[-1])
    return Ap, Aj[:nnz].copy(), Ax[:nnz].copy()


def sort_columns(Ap, Aj, Ax, ncols=None):
    """lssp_mat_sort_column (matrix-utils.cxx:387-481) on host arrays, in place on copies."""
    Ap, Aj, Ax = _i32(Ap).copy(), _i32(Aj).copy(), _f64(Ax).copy()
    n = Ap.size - 1
    _ck(_lib.load().lssp_amd_csr_sort_columns(n, n if ncols is None else ncols, _p(Ap), _p(Aj), _p(Ax)),
        "sort_columns")
    return Ap, Aj, Ax
