"""CPU oracle for the LSSP Krylov hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module.  The product package ``lssp_amd`` never imports it
and fails loudly when its HIP library is missing; nothing here is a fallback.

Two libraries are wrapped:

* ``_build/liboracle.so`` -- our C restatement (``lssp_oracle.c``) of
  mvops.cxx / vector.cxx / solver-tri.cxx / pc-iluk.cxx / pc-ilut.cxx /
  matrix-utils.cxx / solver-{bicgstab,gmres,cg}.cxx, with the reference's serial
  reduction order and the GPU's canonical tree / P-rank orders.
* ``_ref/libref.so`` -- the UNMODIFIED reference compiled in place from
  /root/reference (``oracle/Makefile``), driven through its public API by
  ``ref_shim.cxx``.  Present only when it was built; tests that need it skip
  otherwise (the committed fixtures in tests/golden/ pin the oracle without it).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "_build", "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libref.so")

# LSSP_SOLVER_TYPE / LSSP_PC_TYPE values (type-defs.h:63-101, :157-178)
GMRES, LGMRES, RGMRES, BICGSTAB, CG = 0, 1, 2, 4, 7
BICGSAFE, CGS, GPBICG, CR, CRS, BICRSTAB, BICRSAFE, GPBICR, QMRCGSTAB, TFQMR, ORTHOMIN = (
    6, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17)
BICGSTABL, IDRS = 5, 18  # l of BiCGSTAB(l) / s of IDR(s) are passed as `restart` (<= 0: 4)
PC_NON, PC_ILUK, PC_ILUT = 0, 1, 2
SERIAL, TREE = 0, 1

_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_vp = ctypes.c_void_p
_ci, _cd, _cl = ctypes.c_int, ctypes.c_double, ctypes.c_long


def _ptr(a):
    return None if a is None else a.ctypes.data_as(_vp)


_lib = None
_ref = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            raise RuntimeError(f"oracle not built: {ORACLE_SO} (run make -C oracle)")
        _lib = ctypes.CDLL(ORACLE_SO)
        _lib.orc_dot.restype = _cd
        _lib.orc_dot.argtypes = [_ci, _ci, _vp, _vp, _cl]
        _lib.orc_spmv.argtypes = [_ci, _ci, _vp, _vp, _vp, _cd, _vp, _cd, _vp, _vp]
        _lib.orc_ilu_apply.argtypes = [_ci] + [_vp] * 8
        _lib.orc_trisolve.argtypes = [_ci, _ci, _vp, _vp, _vp, _vp, _vp]
        _lib.orc_ilu_create.restype = _vp
        _lib.orc_ilu_create.argtypes = [_ci, _ci, _vp, _vp, _vp, _ci, _cd, _ci, _ci]
        _lib.orc_ilu_sizes.argtypes = [_vp, _vp, _vp]
        _lib.orc_ilu_get.argtypes = [_vp] * 7
        _lib.orc_ilu_free.argtypes = [_vp]
        _lib.orc_solve.restype = _ci
        _lib.orc_solve.argtypes = ([_ci, _ci] + [_vp] * 9 + [_vp, _vp, _cd, _cd, _cd, _ci, _ci, _ci, _ci]
                                   + [_vp, _ci, _vp, _vp])
        _lib.orc_poisson_nnz.restype = _cl
        _lib.orc_poisson_nnz.argtypes = [_ci, _ci]
        _lib.orc_poisson.argtypes = [_ci, _ci, _vp, _vp, _vp]
    return _lib


def ref_available() -> bool:
    return os.path.exists(REF_SO)


def ref():
    global _ref
    if _ref is None:
        if not ref_available():
            raise RuntimeError(f"reference checker not built: {REF_SO}")
        _ref = ctypes.CDLL(REF_SO)
        _ref.ref_quiet()
        _ref.ref_spmv.argtypes = [_ci, _ci, _vp, _vp, _vp, _cd, _vp, _cd, _vp, _vp]
        _ref.ref_dot.restype = _cd
        _ref.ref_dot.argtypes = [_ci, _vp, _vp]
        _ref.ref_vec.restype = _cd
        _ref.ref_vec.argtypes = [_ci, _ci, _cd, _vp, _cd, _vp, _vp]
        _ref.ref_ilu_create.restype = _vp
        _ref.ref_ilu_create.argtypes = [_ci, _ci, _vp, _vp, _vp, _ci, _cd, _ci]
        _ref.ref_ilu_sizes.argtypes = [_vp, _vp, _vp]
        _ref.ref_ilu_get.argtypes = [_vp] * 7
        _ref.ref_ilu_apply.argtypes = [_vp, _vp, _vp]
        _ref.ref_ilu_free.argtypes = [_vp]
        _ref.ref_solve.restype = _ci
        _ref.ref_solve.argtypes = ([_ci, _ci, _ci, _cd, _ci, _ci, _vp, _vp, _vp, _vp, _vp,
                                    _cd, _cd, _cd, _ci, _ci, _vp, _ci, _vp, _vp, _vp, _vp])
        _ref.ref_time.restype = _cd
    return _ref


@dataclass
class CSR:
    n: int
    Ap: np.ndarray
    Aj: np.ndarray
    Ax: np.ndarray

    @property
    def nnz(self) -> int:
        return int(self.Ap[-1])


def poisson(dim: int, N: int) -> CSR:
    """5-pt (dim=2, exam.cxx:4-59) or 7-pt (dim=3) Poisson, natural order."""
    L = lib()
    n = N * N if dim == 2 else N * N * N
    nnz = L.orc_poisson_nnz(dim, N)
    Ap = np.zeros(n + 1, np.int32)
    Aj = np.zeros(nnz, np.int32)
    Ax = np.zeros(nnz, np.float64)
    L.orc_poisson(dim, N, _ptr(Ap), _ptr(Aj), _ptr(Ax))
    return CSR(n, Ap, Aj, Ax)


def dot(x, y, mode=SERIAL, nranks=1) -> float:
    return lib().orc_dot(mode, nranks, _ptr(x), _ptr(y), len(x))


def spmv(op, A: CSR, x, alpha=1.0, beta=0.0, y=None, z=None):
    z = np.zeros(A.n) if z is None else z
    y = z if y is None else y
    lib().orc_spmv(op, A.n, _ptr(A.Ap), _ptr(A.Aj), _ptr(A.Ax), alpha, _ptr(x), beta, _ptr(y), _ptr(z))
    return z


def _ilu_fetch(sizes, get, h, n):
    nl, nu = ctypes.c_int(), ctypes.c_int()
    sizes(h, ctypes.byref(nl), ctypes.byref(nu))
    L = CSR(n, np.zeros(n + 1, np.int32), np.zeros(nl.value, np.int32), np.zeros(nl.value))
    U = CSR(n, np.zeros(n + 1, np.int32), np.zeros(nu.value, np.int32), np.zeros(nu.value))
    get(h, _ptr(L.Ap), _ptr(L.Aj), _ptr(L.Ax), _ptr(U.Ap), _ptr(U.Aj), _ptr(U.Ax))
    return L, U


def ilu(A: CSR, kind="iluk", level=0, tol=1e-3, p=-1, blk=0):
    """ILUK / ILUT factors (L unit-diagonal last, U pivot first)."""
    L_ = lib()
    h = L_.orc_ilu_create(0 if kind == "iluk" else 1, A.n, _ptr(A.Ap), _ptr(A.Aj), _ptr(A.Ax),
                          level, tol, p, blk)
    try:
        return _ilu_fetch(L_.orc_ilu_sizes, L_.orc_ilu_get, h, A.n)
    finally:
        L_.orc_ilu_free(h)


def ilu_apply(L: CSR, U: CSR, rhs):
    x = np.zeros(L.n)
    lib().orc_ilu_apply(L.n, _ptr(L.Ap), _ptr(L.Aj), _ptr(L.Ax), _ptr(U.Ap), _ptr(U.Aj), _ptr(U.Ax),
                        _ptr(x), _ptr(rhs))
    return x


@dataclass
class SolveResult:
    nits: int
    residual: float
    x: np.ndarray
    trace: np.ndarray
    t_setup: float = 0.0
    t_solve: float = 0.0


def solve(solver, A: CSR, b, x0=None, L=None, U=None, rtol=1e-7, atol=1e-7, rbtol=1e-7,
          maxit=1000, restart=30, mode=SERIAL, nranks=1, trace_cap=200000) -> SolveResult:
    x = np.zeros(A.n) if x0 is None else np.array(x0, dtype=np.float64)
    tr = np.zeros(trace_cap)
    tl, res = ctypes.c_int(), ctypes.c_double()
    it = lib().orc_solve(solver, A.n, _ptr(A.Ap), _ptr(A.Aj), _ptr(A.Ax),
                         _ptr(L.Ap) if L else None, _ptr(L.Aj) if L else None, _ptr(L.Ax) if L else None,
                         _ptr(U.Ap) if U else None, _ptr(U.Aj) if U else None, _ptr(U.Ax) if U else None,
                         _ptr(x), _ptr(b), rtol, atol, rbtol, maxit, restart, mode, nranks,
                         _ptr(tr), trace_cap, ctypes.byref(tl), ctypes.byref(res))
    return SolveResult(it, res.value, x, tr[: min(tl.value, trace_cap)].copy())


# ---- the reference itself (oracle/_ref/libref.so) --------------------------

def ref_spmv(op, A: CSR, x, alpha=1.0, beta=0.0, y=None, z=None):
    z = np.zeros(A.n) if z is None else z
    y = z if y is None else y
    ref().ref_spmv(op, A.n, _ptr(A.Ap), _ptr(A.Aj), _ptr(A.Ax), alpha, _ptr(x), beta, _ptr(y), _ptr(z))
    return z


def ref_dot(x, y) -> float:
    return ref().ref_dot(len(x), _ptr(x), _ptr(y))


def ref_ilu(A: CSR, kind="iluk", level=0, tol=1e-3, p=-1):
    R = ref()
    h = R.ref_ilu_create(0 if kind == "iluk" else 1, A.n, _ptr(A.Ap), _ptr(A.Aj), _ptr(A.Ax),
                         level, tol, p)
    try:
        return _ilu_fetch(R.ref_ilu_sizes, R.ref_ilu_get, h, A.n)
    finally:
        R.ref_ilu_free(h)


def ref_ilu_apply(A: CSR, rhs, kind="iluk", level=0, tol=1e-3, p=-1):
    R = ref()
    h = R.ref_ilu_create(0 if kind == "iluk" else 1, A.n, _ptr(A.Ap), _ptr(A.Aj), _ptr(A.Ax),
                         level, tol, p)
    try:
        x = np.zeros(A.n)
        R.ref_ilu_apply(h, _ptr(x), _ptr(np.ascontiguousarray(rhs, dtype=np.float64)))
        return x
    finally:
        R.ref_ilu_free(h)


def ref_solve(solver, A: CSR, b, pc=PC_NON, level=0, ilut_tol=1e-3, ilut_p=-1, x0=None,
              rtol=1e-7, atol=1e-7, rbtol=1e-7, maxit=1000, restart=30, trace_cap=200000) -> SolveResult:
    x = np.zeros(A.n) if x0 is None else np.array(x0, dtype=np.float64)
    tr = np.zeros(trace_cap)
    tl, res, ts, tv = ctypes.c_int(), ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    it = ref().ref_solve(solver, pc, level, ilut_tol, ilut_p, A.n, _ptr(A.Ap), _ptr(A.Aj), _ptr(A.Ax),
                         _ptr(x), _ptr(np.ascontiguousarray(b, dtype=np.float64)), rtol, atol, rbtol,
                         maxit, restart, _ptr(tr), trace_cap, ctypes.byref(tl), ctypes.byref(res),
                         ctypes.byref(ts), ctypes.byref(tv))
    return SolveResult(it, res.value, x, tr[: min(tl.value, trace_cap)].copy(), ts.value, tv.value)


def ref_bj(A: CSR, nblk: int):
    """Block-Jacobi ILU(0) factors composed from the reference's public API."""
    R = ref()
    R.ref_bj_create.restype = _vp
    R.ref_bj_create.argtypes = [_ci, _vp, _vp, _vp, _ci]
    R.ref_bj_free.argtypes = [_vp]
    h = R.ref_bj_create(A.n, _ptr(A.Ap), _ptr(A.Aj), _ptr(A.Ax), nblk)
    try:
        return _ilu_fetch(R.ref_ilu_sizes, R.ref_ilu_get, h, A.n)
    finally:
        R.ref_bj_free(h)


def ref_solve_bj(solver, A: CSR, b, nblk: int, x0=None, rtol=1e-7, atol=1e-7, rbtol=1e-7,
                 maxit=1000, restart=30, trace_cap=200000) -> SolveResult:
    """Solve with block-Jacobi ILU(0) plugged in through LSSP_PC_USER."""
    R = ref()
    R.ref_bj_create.restype = _vp
    R.ref_bj_create.argtypes = [_ci, _vp, _vp, _vp, _ci]
    R.ref_bj_free.argtypes = [_vp]
    R.ref_solve_bj.restype = _ci
    R.ref_solve_bj.argtypes = [_vp, _ci, _ci, _vp, _vp, _vp, _vp, _vp, _cd, _cd, _cd, _ci, _ci,
                               _vp, _ci, _vp, _vp]
    h = R.ref_bj_create(A.n, _ptr(A.Ap), _ptr(A.Aj), _ptr(A.Ax), nblk)
    try:
        x = np.zeros(A.n) if x0 is None else np.array(x0, dtype=np.float64)
        tr = np.zeros(trace_cap)
        tl, res = ctypes.c_int(), ctypes.c_double()
        it = R.ref_solve_bj(h, solver, A.n, _ptr(A.Ap), _ptr(A.Aj), _ptr(A.Ax), _ptr(x),
                            _ptr(np.ascontiguousarray(b, dtype=np.float64)), rtol, atol, rbtol, maxit,
                            restart, _ptr(tr), trace_cap, ctypes.byref(tl), ctypes.byref(res))
        return SolveResult(it, res.value, x, tr[: min(tl.value, trace_cap)].copy())
    finally:
        R.ref_bj_free(h)


# ---- format conversions (matrix-utils.cxx:62-380, :700-765) ------------------
# src "orc": the C restatement; "ref": the reference itself (libref.so)
def _conv_lib(src):
    return lib() if src == "orc" else ref()  # every conversion entry point returns int or void


def csr_to_coo(nrows, ncols, Ap, Aj, Ax, src="orc"):
    L = _conv_lib(src)
    nnz = int(Ap[nrows])
    Ci, Cj, Cx = np.zeros(nnz, np.int32), np.zeros(nnz, np.int32), np.zeros(nnz)
    getattr(L, f"{src}_csr_to_coo")(nrows, ncols, _ptr(Ap), _ptr(Aj), _ptr(Ax), _ptr(Ci), _ptr(Cj), _ptr(Cx))
    return Ci, Cj, Cx


def coo_to_csr(nrows, ncols, Ci, Cj, Cx, src="orc"):
    L = _conv_lib(src)
    nnz = len(Ci)
    Ap = np.zeros(nrows + 1, np.int32)
    Aj, Ax = np.zeros(max(nnz, 1), np.int32), np.zeros(max(nnz, 1))
    getattr(L, f"{src}_coo_to_csr")(nrows, ncols, nnz, _ptr(Ci), _ptr(Cj), _ptr(Cx), _ptr(Ap), _ptr(Aj),
                                    _ptr(Ax))
    return Ap, Aj[:nnz], Ax[:nnz]


def transpose(nrows, ncols, Ap, Aj, Ax, src="orc"):
    L = _conv_lib(src)
    nnz = int(Ap[nrows])
    Tp = np.zeros(ncols + 1, np.int32)
    Tj, Tx = np.zeros(max(nnz, 1), np.int32), np.zeros(max(nnz, 1))
    getattr(L, f"{src}_transpose")(nrows, ncols, _ptr(Ap), _ptr(Aj), _ptr(Ax), _ptr(Tp), _ptr(Tj), _ptr(Tx))
    return Tp, Tj[:nnz], Tx[:nnz]


def csr_to_bcsr(n, bs, Ap, Aj, Ax, src="orc"):
    L = _conv_lib(src)
    nnz = int(Ap[n])
    Bp = np.zeros(n // bs + 1, np.int32)
    Bj, Bx = np.zeros(nnz, np.int32), np.zeros(nnz * bs * bs)
    m = getattr(L, f"{src}_csr_to_bcsr")(n, bs, _ptr(Ap), _ptr(Aj), _ptr(Ax), _ptr(Bp), _ptr(Bj), _ptr(Bx))
    return Bp, Bj[:m].copy(), Bx[:m * bs * bs].copy()


def bcsr_to_csr(nbrows, nbcols, bs, Bp, Bj, Bx, src="orc"):
    L = _conv_lib(src)
    cap = max(int(Bp[nbrows]) * bs * bs, 1)
    Ap = np.zeros(nbrows * bs + 1, np.int32)
    Aj, Ax = np.zeros(cap, np.int32), np.zeros(cap)
    m = getattr(L, f"{src}_bcsr_to_csr")(nbrows, nbcols, bs, _ptr(Bp), _ptr(Bj), _ptr(Bx), _ptr(Ap), _ptr(Aj),
                                         _ptr(Ax))
    return Ap, Aj[:m].copy(), Ax[:m].copy()
