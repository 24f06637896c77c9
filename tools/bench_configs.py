"""Measurement + full-size parity of BASELINE.json's other single-GPU configs.

    python tools/bench_configs.py cg-thermal   [--iters 1000] [--ref-iters 1000]
    python tools/bench_configs.py gmres-ilut   [--grid 256]   [--ref-iters 30]
    python tools/bench_configs.py bicgstab-iluk [--grid 256]  (config 2; --grid 512: config 4's matrix on one GPU)
    python tools/bench_configs.py general-ilu  [--grid 216]   (the packet-sweep ILU path)

Each prints ONE JSON line: GPU throughput (Krylov it/s with HIP-event SpMV
and ILU-apply rooflines), the reference's own CPU timing on a bounded sample
(oracle/_ref/libref.so, 1 core), and a FULL-SIZE parity check: the library in
SERIAL reduction mode is run for the same number of iterations as the
reference and every dot/norm the driver evaluates must be bitwise equal
(trace), plus the final x.  The tree-mode (fast path) run to convergence is
compared with the reference's iteration count.

config 5 (cg-thermal): thermal2-like SPD matrix (lssp_amd.synthetic), CG,
PC_NON, b = 1, x0 = 0, fixed 1000 iterations.
config 3 (gmres-ilut): 7-pt Poisson 256^3, GMRES(30) + ILUT(1e-4, p=20).
general-ilu: the packet-sweep ILU path on a non-grid mesh ILU(0), a 7-pt ILU(1)
and the 7-pt ILU(0) forced off the line sweeps (tracked number for the
general path).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import HBM_PEAK_GBS, ilu_apply_bytes, spmv_bytes  # noqa: E402  (one byte accounting)

T0 = time.perf_counter()


def log(msg):
    """progress on stderr (long host setups must not look like a hang)"""
    print(f"[{time.perf_counter() - T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def _events(dev):
    import torch
    s = torch.cuda.ExternalStream(dev.stream)
    return s, torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def spmv_leg(dev, A, nnz, n, reps=50):
    x = dev.vec(n, np.random.default_rng(1).uniform(-1, 1, n))
    y = dev.vec(n)
    for _ in range(5):
        A.mv_mxy(x, y)
    s, e0, e1 = _events(dev)
    e0.record(s)
    for _ in range(reps):
        A.mv_mxy(x, y)
    e1.record(s)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    # the bytes the kernel moves (1-byte diagonal ids on coded stencils) and the
    # int32-CSR equivalent, as bench.py reports them
    b = spmv_bytes(nnz, n, coded=A.ndiag > 0)
    b32 = spmv_bytes(nnz, n)
    return {"ms": round(ms, 5), "GBps": round(b / ms / 1e6, 1), "frac_hbm_peak": round(b / ms / 1e6 / HBM_PEAK_GBS, 4),
            "bytes": b, "csr_int32_equiv_GBps": round(b32 / ms / 1e6, 1)}


def apply_leg(dev, M, n, reps=5):
    x = dev.vec(n, np.random.default_rng(2).uniform(-1, 1, n))
    z = dev.vec(n)
    M.apply(z, x)
    s, e0, e1 = _events(dev)
    e0.record(s)
    for _ in range(reps):  # queued back to back (the synchronous apply adds a host round trip per call)
        M.apply_async(z, x)
    e1.record(s)
    e1.synchronize()
    M.check()
    ms = e0.elapsed_time(e1) / reps
    b = ilu_apply_bytes(M.nnzL, M.nnzU, n)  # SURVEY 8(d) B_ilu, the bytes bench.py's roofline uses
    return {"ms": round(ms, 4), "GBps": round(b / ms / 1e6, 1), "frac_hbm_peak": round(b / ms / 1e6 / HBM_PEAK_GBS, 4),
            "bytes": b, "levels_L": M.levelsL, "levels_U": M.levelsU}


def timed_solve(dev, A, M, n, solver, iters, restart=30, reduction=None):
    import lssp_amd
    if reduction is not None:
        dev.set_reduction(reduction)
    x = dev.vec(n, np.zeros(n))
    b = dev.vec(n, np.ones(n))
    dev.sync()
    t0 = time.perf_counter()
    r = lssp_amd.solve(dev, A, M, x, b, solver=solver, tol_rel=0.0, tol_abs=0.0, tol_rb=0.0, maxit=iters,
                       restart=restart)
    dev.sync()
    return r, time.perf_counter() - t0


def parity(dev, A, M, n, Ao, solver, ref_kw, iters, restart, out):
    """SERIAL mode vs the reference itself, same iteration count, bitwise"""
    import lssp_amd
    import oracle as O
    log(f"reference: {iters} iterations (setup included)")
    t0 = time.perf_counter()
    ref = O.ref_solve(solver, Ao, np.ones(n), rtol=0.0, atol=0.0, rbtol=0.0, maxit=iters, restart=restart,
                      **ref_kw)
    t_ref = time.perf_counter() - t0
    log("serial-mode run on the GPU")
    dev.set_reduction(lssp_amd.SERIAL)
    x = dev.vec(n, np.zeros(n))
    b = dev.vec(n, np.ones(n))
    r = lssp_amd.solve(dev, A, M, x, b, solver=solver, tol_rel=0.0, tol_abs=0.0, tol_rb=0.0, maxit=iters,
                       restart=restart, trace_cap=ref.trace.size + 16)
    dev.set_reduction(lssp_amd.TREE)
    xs = x.download()
    same = lambda a, b_: bool(np.array_equal(np.asarray(a), np.asarray(b_), equal_nan=True))
    out["parity_serial_vs_reference"] = {
        "iterations": iters, "nits": [r.nits, ref.nits], "trace_len": [int(r.trace.size), int(ref.trace.size)],
        "trace_bitwise": same(r.trace, ref.trace), "x_bitwise": same(xs, ref.x),
        "residual": [r.residual, ref.residual]}
    out["cpu_baseline"] = {"value": round(ref.nits / ref.t_solve, 4), "unit": "iters/s", "cores": 1,
                           "kind": "reference",
                           "sample": f"reference lssp_solver_solve, {ref.nits} iterations in {ref.t_solve:.2f} s "
                                     f"(PC setup {ref.t_setup:.2f} s, wall {t_ref:.1f} s)"}
    return ref


def cg_thermal(args):
    import lssp_amd
    import oracle as O
    from lssp_amd.synthetic import thermal_like
    Ap, Aj, Ax = thermal_like()
    n, nnz = Ap.size - 1, int(Ap[-1])
    dev = lssp_amd.Device(0)
    A = lssp_amd.DMat(dev, Ap, Aj, Ax)
    out = {"config": "thermal2-like SPD (SURVEY 8(d)), CG, PC_NON, b=1, x0=0", "rows": n, "nnz": nnz,
           "spmv": spmv_leg(dev, A, nnz, n)}
    timed_solve(dev, A, None, n, lssp_amd.CG, 20)
    r, t = timed_solve(dev, A, None, n, lssp_amd.CG, args.iters)
    out["gpu"] = {"iters": r.nits, "seconds": round(t, 4), "iters_per_s": round(r.nits / t, 2),
                  "ms_per_iter": round(t / r.nits * 1e3, 4), "residual": r.residual, "reduction": "tree"}
    if O.ref_available():
        ref = parity(dev, A, None, n, O.CSR(n, Ap, Aj, Ax), O.CG, dict(pc=O.PC_NON), args.ref_iters, 30, out)
        out["tree_vs_reference_residual_rel"] = (abs(r.residual - ref.residual) / ref.residual
                                                 if args.ref_iters == args.iters else None)
    dev.close()
    print(json.dumps(out), flush=True)


def gmres_ilut(args):
    import lssp_amd
    import oracle as O
    N = args.grid
    Ap, Aj, Ax = lssp_amd.poisson(3, N)
    n, nnz = Ap.size - 1, int(Ap[-1])
    dev = lssp_amd.Device(0)
    A = lssp_amd.DMat(dev, Ap, Aj, Ax)
    log("ILUT setup")
    t0 = time.perf_counter()
    M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=lssp_amd.ILUT, tol=1e-4, p=20)
    t_pc = time.perf_counter() - t0
    out = {"config": f"7-pt Poisson {N}^3, GMRES(30) + ILUT(1e-4, p=20), b=1, x0=0", "rows": n, "nnz": nnz,
           "ilut": {"nnzL": M.nnzL, "nnzU": M.nnzU, "setup_s": round(t_pc, 2)},
           "spmv": spmv_leg(dev, A, nnz, n), "ilu_apply": apply_leg(dev, M, n)}
    log("GMRES to convergence")
    # to convergence, default tolerances (lssp.cxx:11-13), tree reductions
    x = dev.vec(n, np.zeros(n))
    b = dev.vec(n, np.ones(n))
    dev.sync()
    t0 = time.perf_counter()
    r = lssp_amd.solve(dev, A, M, x, b, solver=lssp_amd.GMRES, maxit=5000, restart=30)
    dev.sync()
    t = time.perf_counter() - t0
    out["gpu"] = {"nits": r.nits, "residual": r.residual, "seconds": round(t, 3),
                  "iters_per_s": round(r.nits / t, 2), "reduction": "tree",
                  "reference_nits_survey": 162 if N == 256 else None}
    print(json.dumps(out), flush=True)  # GPU half first: the reference half is long
    if O.ref_available() and args.ref_iters > 0:
        parity(dev, A, M, n, O.CSR(n, Ap, Aj, Ax), O.GMRES, dict(pc=O.PC_ILUT, ilut_tol=1e-4, ilut_p=20),
               args.ref_iters, 30, out)
    dev.close()
    print(json.dumps(out), flush=True)


def bicgstab_iluk(args):
    """configs 2 (256^3, one GPU) and 4's matrix on one GPU (512^3): BiCGSTAB +
    ILUK(0), tree reductions, zero tolerances (exactly --iters iterations), then
    a solve to the reference's default tolerances; with the reference built, its
    own CPU time on a bounded sample (--ref-iters iterations, 1 core)."""
    import lssp_amd
    import oracle as O
    N = args.grid
    Ap, Aj, Ax = lssp_amd.poisson(3, N)
    n, nnz = Ap.size - 1, int(Ap[-1])
    dev = lssp_amd.Device(0)
    A = lssp_amd.DMat(dev, Ap, Aj, Ax)
    log("ILUK(0) setup")
    t0 = time.perf_counter()
    M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=0)
    t_pc = time.perf_counter() - t0
    out = {"config": f"7-pt Poisson {N}^3, BiCGSTAB + ILUK(0), b=1, x0=0, one GPU", "rows": n, "nnz": nnz,
           "ilu_setup_s": round(t_pc, 2), "spmv": spmv_leg(dev, A, nnz, n), "ilu_apply": apply_leg(dev, M, n)}
    timed_solve(dev, A, M, n, lssp_amd.BICGSTAB, 3)
    r, t = timed_solve(dev, A, M, n, lssp_amd.BICGSTAB, args.iters)
    out["gpu"] = {"iters": r.nits, "iters_per_s": round(r.nits / t, 2), "ms_per_iter": round(t / r.nits * 1e3, 4),
                  "reduction": "tree"}
    x = dev.vec(n, np.zeros(n))
    b = dev.vec(n, np.ones(n))
    dev.sync()
    t0 = time.perf_counter()
    r = lssp_amd.solve(dev, A, M, x, b, solver=lssp_amd.BICGSTAB, maxit=5000)
    dev.sync()
    out["converged"] = {"nits": r.nits, "residual": r.residual, "seconds": round(time.perf_counter() - t0, 3),
                        "reference_nits": {216: 145, 256: 155}.get(N)}
    print(json.dumps(out), flush=True)  # GPU half first
    if args.ref_iters > 0 and O.ref_available():
        log(f"reference: {args.ref_iters} iterations on 1 core")
        ref = O.ref_solve(O.BICGSTAB, O.CSR(n, Ap, Aj, Ax), np.ones(n), rtol=0.0, atol=0.0, rbtol=0.0,
                          maxit=args.ref_iters, pc=O.PC_ILUK, level=0)
        out["cpu_baseline"] = {"value": round(ref.nits / ref.t_solve, 4), "unit": "iters/s", "cores": 1,
                               "kind": "reference",
                               "sample": f"reference lssp_solver_solve, {ref.nits} iterations in {ref.t_solve:.2f} s "
                                         f"(PC setup {ref.t_setup:.2f} s)"}
        out["vs_cpu"] = round(out["gpu"]["iters_per_s"] / out["cpu_baseline"]["value"], 1)
        print(json.dumps(out), flush=True)
    dev.close()


def general_ilu(args):
    """The general (packet-sweep) ILU path on matrices the line sweeps do not
    serve: ILU(0) of the thermal-like mesh matrix (not a grid), ILU(1) of a
    7-pt grid, and the 7-pt ILU(0) forced onto the packet sweeps (LSSP_AMD_LINE=0)
    beside its line sweeps.  Per case: apply time (B_ilu GB/s), BiCGSTAB it/s
    (tree), and for the thermal case a SERIAL-mode run bitwise vs the reference."""
    import lssp_amd
    import oracle as O
    from lssp_amd.synthetic import thermal_like
    dev = lssp_amd.Device(0)
    cases = []

    def case(name, Ap, Aj, Ax, level, line, ref_iters=0, env=None):
        n, nnz = Ap.size - 1, int(Ap[-1])
        log(f"{name}: setup")
        env = dict(env or {})
        if not line:
            env["LSSP_AMD_LINE"] = "0"
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        t0 = time.perf_counter()
        M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=level)
        t_pc = time.perf_counter() - t0
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        A = lssp_amd.DMat(dev, Ap, Aj, Ax)
        out = {"case": name, "rows": n, "nnz": nnz, "ilu": {"level": level, "nnzL": M.nnzL, "nnzU": M.nnzU,
                                                            "setup_s": round(t_pc, 2),
                                                            "sweeps": ["packet", "line ILU(0)", "line ILU(1)"][
                                                                M.sweep_layout()[0]]},
               "ilu_apply": apply_leg(dev, M, n, reps=10)}
        timed_solve(dev, A, M, n, lssp_amd.BICGSTAB, 5)
        r, t = timed_solve(dev, A, M, n, lssp_amd.BICGSTAB, args.iters)
        out["gpu"] = {"iters": r.nits, "seconds": round(t, 4), "iters_per_s": round(r.nits / t, 2),
                      "reduction": "tree"}
        if ref_iters and O.ref_available():
            parity(dev, A, M, n, O.CSR(n, Ap, Aj, Ax), O.BICGSTAB, dict(pc=O.PC_ILUK, level=level),
                   ref_iters, 30, out)
        M.close()
        A.close()
        print(json.dumps(out), flush=True)
        cases.append(out)

    Ap, Aj, Ax = thermal_like()
    case("thermal-like ILU(0)", Ap, Aj, Ax, 0, True, ref_iters=args.ref_iters)
    Ap, Aj, Ax = lssp_amd.poisson(3, 128)
    case("7-pt 128^3 ILU(1), line sweeps", Ap, Aj, Ax, 1, True)
    case("7-pt 128^3 ILU(1), packet sweeps", Ap, Aj, Ax, 1, False)
    Ap, Aj, Ax = lssp_amd.poisson(2, 100)
    case("5-pt 100^2 ILU(1) (exam.cxx's matrix), one-workgroup line sweeps", Ap, Aj, Ax, 1, True)
    case("5-pt 100^2 ILU(1) (exam.cxx's matrix), skewed-tile line sweeps", Ap, Aj, Ax, 1, True,
         env={"LSSP_AMD_LINEG": "0"})
    case("5-pt 100^2 ILU(1) (exam.cxx's matrix), packet sweeps", Ap, Aj, Ax, 1, False)
    Ap, Aj, Ax = lssp_amd.poisson(3, args.grid)
    case(f"7-pt {args.grid}^3 ILU(0), packet sweeps", Ap, Aj, Ax, 0, False)
    case(f"7-pt {args.grid}^3 ILU(0), line sweeps", Ap, Aj, Ax, 0, True)
    case(f"7-pt {args.grid}^3 ILU(1) (the reference's default level), line sweeps", Ap, Aj, Ax, 1, True)
    dev.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("which", choices=["cg-thermal", "gmres-ilut", "bicgstab-iluk", "general-ilu"])
    ap.add_argument("--iters", type=int, default=1000)
    ap.add_argument("--ref-iters", type=int, default=None)
    ap.add_argument("--grid", type=int, default=256)
    args = ap.parse_args()
    if args.which == "cg-thermal":
        args.ref_iters = args.iters if args.ref_iters is None else args.ref_iters
        cg_thermal(args)
    elif args.which == "gmres-ilut":
        # SERIAL-mode dots run on one GPU lane (16.7 M terms each at 256^3), so the
        # bitwise leg is kept to a few Arnoldi steps
        args.ref_iters = 5 if args.ref_iters is None else args.ref_iters
        gmres_ilut(args)
    elif args.which == "general-ilu":
        args.iters = min(args.iters, 100)
        args.ref_iters = 20 if args.ref_iters is None else args.ref_iters
        args.grid = 216 if args.grid == 256 else args.grid
        general_ilu(args)
    else:
        args.iters = min(args.iters, 100)
        args.ref_iters = (3 if args.grid <= 256 else 0) if args.ref_iters is None else args.ref_iters
        bicgstab_iluk(args)


if __name__ == "__main__":
    main()
