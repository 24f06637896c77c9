#!/usr/bin/env python3
"""Generate tests/golden/ from the REFERENCE ITSELF (oracle/_ref/libref.so).

Run in the dev container, where /root/reference exists:
    make -C oracle all ref && python tests/golden/make_golden.py

libref.so is the unmodified reference compiled in place (oracle/Makefile) and
driven through its public API (oracle/ref_shim.cxx).  Only data is written:
golden.npz (arrays; numpy .npz, loaded with allow_pickle=False) and
manifest.json (case parameters, scalars as exact float.hex strings, sha256
digests of larger arrays).  The tests rebuild every input from the manifest
parameters with tests/inputs.py and check the oracle (CPU, -m "not gpu") and
the HIP path (-m gpu) against these vectors.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

import oracle as O  # noqa: E402
from inputs import digest, rand_csr, uniform  # noqa: E402

FULL_MAX = 5000  # store arrays in full up to this many entries, else sha256


def build_matrix(spec) -> O.CSR:
    if spec["type"] == "poisson":
        return O.poisson(spec["dim"], spec["N"])
    Ap, Aj, Ax = rand_csr(spec["n"], spec["per_row"], spec["seed"], spec.get("unsorted", True),
                          spec.get("missing_diag_every", 0), spec.get("diag", 4.0))
    return O.CSR(spec["n"], Ap, Aj, Ax)


def vec(spec, n):
    if spec == "ones":
        return np.ones(n)
    if spec == "zeros":
        return np.zeros(n)
    return uniform(int(spec), n)


class Store:
    def __init__(self):
        self.arrays = {}
        self.cases = []

    def put(self, key, *arrays):
        """full arrays when small, else only a digest"""
        if sum(a.size for a in arrays) <= FULL_MAX:
            for i, a in enumerate(arrays):
                self.arrays[f"{key}__{i}"] = np.ascontiguousarray(a)
            return {"npz": key, "count": len(arrays), "sha256": digest(*arrays)}
        return {"sha256": digest(*arrays)}


def main():
    S = Store()
    P7 = lambda N: {"type": "poisson", "dim": 3, "N": N}  # noqa: E731
    P5 = lambda N: {"type": "poisson", "dim": 2, "N": N}  # noqa: E731
    RND = {"type": "rand", "n": 300, "per_row": 6, "seed": 77, "unsorted": True, "missing_diag_every": 11}
    # same generator with every diagonal present: the reference's ILU(0)/ILUT read past the end
    # of its adjusted copy when a diagonal is missing (matrix-utils.cxx:485 keeps num_nnzs stale),
    # so those paths are pinned only on matrices with full diagonals
    RNDF = {"type": "rand", "n": 300, "per_row": 6, "seed": 77, "unsorted": True, "missing_diag_every": 0}
    RND2 = {"type": "rand", "n": 2000, "per_row": 5, "seed": 4242, "unsorted": True, "missing_diag_every": 0,
            "diag": 3.0}

    # 1. SpMV, all four mvops.cxx entry points
    for mat in [P5(16), P7(8), P7(16), P7(32), P5(256), RND]:
        A = build_matrix(mat)
        for op, alpha, beta in [(0, 1.0, 0.0), (1, -0.75, 0.0), (2, 1.5, -1.25), (3, -1.0, 1.0), (3, 1.0, 0.0)]:
            x = uniform(0x5EED, A.n)
            y = uniform(0x5EED + 1, A.n)
            z = O.ref_spmv(op, A, x, alpha, beta, y.copy(), y.copy())
            S.cases.append({"kind": "spmv", "mat": mat, "op": op, "alpha": alpha.hex(), "beta": beta.hex(),
                            "xseed": 0x5EED, "yseed": 0x5EED + 1,
                            "out": S.put(f"spmv_{len(S.cases)}", z)})

    # 2/3. ILU factors and pc.solve outputs
    pcs = [({"kind": "iluk", "level": 0}, [P7(8), P7(32), P5(64), RNDF, RND2]),
           ({"kind": "iluk", "level": 1}, [P7(8), P7(32), P5(64), RND, RND2]),
           ({"kind": "iluk", "level": 2}, [P7(8), RND]),
           ({"kind": "ilut", "tol": 1e-4, "p": 20}, [P7(8), P7(32), RNDF, RND2]),
           ({"kind": "ilut", "tol": 1e-2, "p": 3}, [P7(8), RNDF, RND2]),
           ({"kind": "ilut", "tol": 1e-3, "p": -1}, [P7(8), RNDF]),
           ({"kind": "bj", "nblk": 2}, [P7(32)]),
           ({"kind": "bj", "nblk": 4}, [P7(32), P7(16)]),
           ({"kind": "bj", "nblk": 8}, [P7(32), P7(16)])]
    for pc, mats in pcs:
        for mat in mats:
            A = build_matrix(mat)
            if pc["kind"] == "iluk":
                L, U = O.ref_ilu(A, "iluk", level=pc["level"])
            elif pc["kind"] == "ilut":
                L, U = O.ref_ilu(A, "ilut", tol=pc["tol"], p=pc["p"])
            else:
                L, U = O.ref_bj(A, pc["nblk"])
            rhs = uniform(0xA11CE, A.n)
            if pc["kind"] == "bj":
                out = O.ilu_apply(L, U, rhs)  # factors are the reference's; apply = solver-tri restated
                applied = None
            else:
                kw = {"level": pc["level"]} if pc["kind"] == "iluk" else {"tol": pc["tol"], "p": pc["p"]}
                applied = O.ref_ilu_apply(A, rhs, pc["kind"], **kw)
                out = applied
            S.cases.append({"kind": "ilu", "mat": mat, "pc": pc, "nnzL": L.nnz, "nnzU": U.nnz,
                            "L": S.put(f"L_{len(S.cases)}", L.Ap, L.Aj, L.Ax),
                            "U": S.put(f"U_{len(S.cases)}", U.Ap, U.Aj, U.Ax),
                            "rhs_seed": 0xA11CE, "apply": S.put(f"apply_{len(S.cases)}", out),
                            "apply_from_ref": applied is not None})

    # 4/5. solver traces (every dot/norm the driver computed, in order)
    B, G, C, RG, LG = O.BICGSTAB, O.GMRES, O.CG, O.RGMRES, O.LGMRES
    solves = [
        (B, {"kind": "iluk", "level": 0}, P7(32), "ones", None, {}),
        (B, {"kind": "iluk", "level": 0}, P7(64), "ones", None, {}),
        (G, {"kind": "ilut", "tol": 1e-4, "p": 20}, P7(32), "ones", None, {"restart": 30}),
        (G, {"kind": "ilut", "tol": 1e-4, "p": 20}, P7(64), "ones", None, {"restart": 30}),
        (C, {"kind": "none"}, P7(32), "ones", None, {}),
        (C, {"kind": "none"}, P7(64), "ones", None, {}),
        (B, {"kind": "iluk", "level": 0}, P5(256), "ones", None, {}),           # config 1
        (G, {"kind": "iluk", "level": 1}, P5(100), "ones", None, {"restart": 60, "maxit": 3000}),  # exam.cxx
        (B, {"kind": "iluk", "level": 1}, P7(24), 0x5EED, 0xB0B, {}),
        (C, {"kind": "iluk", "level": 0}, P7(24), "ones", None, {}),
        (G, {"kind": "none"}, P7(16), "ones", None, {"restart": 10}),
        (B, {"kind": "none"}, P7(16), "ones", None, {}),
        (G, {"kind": "ilut", "tol": 1e-3, "p": 5}, RND2, 0x5EED, None, {"restart": 20}),
        (B, {"kind": "iluk", "level": 1}, RND2, 0x5EED, None, {}),
        (B, {"kind": "iluk", "level": 0}, P7(16), "zeros", None, {}),           # b = 0: immediate exit
        (G, {"kind": "iluk", "level": 0}, P7(16), "zeros", None, {}),
        (C, {"kind": "none"}, P7(16), "ones", None, {"maxit": 7}),              # maxit hit
        (B, {"kind": "iluk", "level": 0}, P7(16), "ones", None, {"maxit": 5}),
        (G, {"kind": "iluk", "level": 0}, P7(16), "ones", None, {"maxit": 13, "restart": 5}),
        (B, {"kind": "bj", "nblk": 2}, P7(32), "ones", None, {}),
        (B, {"kind": "bj", "nblk": 4}, P7(32), "ones", None, {}),
        (B, {"kind": "bj", "nblk": 8}, P7(32), "ones", None, {}),
        (B, {"kind": "bj", "nblk": 8}, P7(64), "ones", None, {}),
        (G, {"kind": "bj", "nblk": 4}, P7(32), "ones", None, {"restart": 30}),
        (C, {"kind": "bj", "nblk": 4}, P7(32), "ones", None, {}),
        # right-preconditioned GMRES (solver-gmres.cxx:257-479)
        (RG, {"kind": "ilut", "tol": 1e-4, "p": 20}, P7(32), "ones", None, {"restart": 30}),
        (RG, {"kind": "iluk", "level": 0}, P7(32), "ones", None, {"restart": 30}),
        (RG, {"kind": "iluk", "level": 1}, P5(100), "ones", None, {"restart": 60, "maxit": 3000}),
        (RG, {"kind": "none"}, P7(16), "ones", None, {"restart": 10}),
        (RG, {"kind": "iluk", "level": 0}, P7(16), "ones", None, {"maxit": 13, "restart": 5}),
        (RG, {"kind": "ilut", "tol": 1e-3, "p": 5}, RND2, 0x5EED, 0xB0B, {"restart": 20}),
        (RG, {"kind": "bj", "nblk": 4}, P7(32), "ones", None, {"restart": 30}),
        (RG, {"kind": "iluk", "level": 0}, P7(16), "zeros", None, {}),
        # LGMRES(m, k = 3) (solver-lgmres.cxx:12-312)
        (LG, {"kind": "ilut", "tol": 1e-4, "p": 20}, P7(32), "ones", None, {"restart": 30}),
        (LG, {"kind": "iluk", "level": 0}, P7(32), "ones", None, {"restart": 10}),
        (LG, {"kind": "iluk", "level": 1}, P5(100), "ones", None, {"restart": 20}),
        (LG, {"kind": "none"}, P7(16), "ones", None, {"restart": 8}),
        (LG, {"kind": "iluk", "level": 0}, P7(16), "ones", None, {"maxit": 13, "restart": 5}),
        (LG, {"kind": "ilut", "tol": 1e-3, "p": 5}, RND2, 0x5EED, 0xB0B, {"restart": 6}),
        (LG, {"kind": "bj", "nblk": 4}, P7(32), "ones", None, {"restart": 12}),
        (LG, {"kind": "iluk", "level": 0}, P7(16), "zeros", None, {}),
    ]
    # the L1-composed drivers (solver-{bicgsafe,cgs,gpbicg,cr,crs,bicrstab,bicrsafe,gpbicr,qmrcgstab,
    # tfqmr}.cxx): SPD and nonsymmetric systems, each PC kind, maxit hit, immediate exit
    for sv in (O.BICGSAFE, O.CGS, O.GPBICG, O.CR, O.CRS, O.BICRSTAB, O.BICRSAFE, O.GPBICR, O.QMRCGSTAB,
               O.TFQMR, O.ORTHOMIN):
        solves += [
            (sv, {"kind": "iluk", "level": 0}, P7(16), "ones", None, {}),
            (sv, {"kind": "none"}, P5(48), "ones", None, {}),
            (sv, {"kind": "ilut", "tol": 1e-3, "p": 5}, RND2, 0x5EED, 0xB0B, {}),
            (sv, {"kind": "iluk", "level": 1}, P7(12), "ones", None, {"maxit": 4}),
            (sv, {"kind": "iluk", "level": 0}, P7(12), "zeros", None, {}),
            (sv, {"kind": "bj", "nblk": 4}, P7(16), "ones", None, {}),
        ]
    # ORTHOMIN(k) with k = restart small enough to cycle its direction ring (solver-orthomin.cxx:102, :120)
    solves += [(O.ORTHOMIN, {"kind": "iluk", "level": 0}, P7(16), "ones", None, {"restart": 3}),
               (O.ORTHOMIN, {"kind": "ilut", "tol": 1e-3, "p": 5}, RND2, 0x5EED, 0xB0B, {"restart": 2})]
    # BiCGSTAB(l) (solver-bicgstabl.cxx:4-217) and IDR(s) (solver-idrs.cxx:86-283); l / s ride in
    # `restart`: the default 4, the special small cases (IDR(1) / IDR(2) have their own unrolled
    # array_solve, solver-idrs.cxx:32-50) and 3 (the general LU)
    for sv in (O.BICGSTABL, O.IDRS):
        solves += [
            (sv, {"kind": "iluk", "level": 0}, P7(16), "ones", None, {"restart": 4}),
            (sv, {"kind": "none"}, P5(48), "ones", None, {"restart": 2}),
            (sv, {"kind": "ilut", "tol": 1e-3, "p": 5}, RND2, 0x5EED, 0xB0B, {"restart": 4}),
            (sv, {"kind": "iluk", "level": 1}, P7(12), "ones", None, {"maxit": 4, "restart": 4}),
            (sv, {"kind": "iluk", "level": 0}, P7(12), "zeros", None, {"restart": 4}),
            (sv, {"kind": "bj", "nblk": 4}, P7(16), "ones", None, {"restart": 4}),
            (sv, {"kind": "iluk", "level": 0}, P7(16), "ones", None, {"restart": 1}),
            (sv, {"kind": "ilut", "tol": 1e-4, "p": 20}, P7(16), "ones", None, {"restart": 3}),
        ]
    pcmap = {"none": O.PC_NON, "iluk": O.PC_ILUK, "ilut": O.PC_ILUT}
    for solver, pc, mat, bspec, x0spec, kw in solves:
        A = build_matrix(mat)
        b = vec(bspec, A.n)
        x0 = None if x0spec is None else vec(x0spec, A.n)
        maxit = kw.get("maxit", 5000)
        restart = kw.get("restart", 30)
        if pc["kind"] == "bj":
            R = O.ref_solve_bj(solver, A, b, pc["nblk"], x0=x0, maxit=maxit, restart=restart)
        else:
            R = O.ref_solve(solver, A, b, pc=pcmap[pc["kind"]], level=pc.get("level", 0),
                            ilut_tol=pc.get("tol", 1e-3), ilut_p=pc.get("p", -1), x0=x0,
                            maxit=maxit, restart=restart)
        S.cases.append({"kind": "solve", "solver": solver, "pc": pc, "mat": mat, "b": bspec, "x0": x0spec,
                        "maxit": maxit, "restart": restart, "rtol": (1e-7).hex(), "atol": (1e-7).hex(),
                        "rbtol": (1e-7).hex(), "nits": R.nits, "residual": R.residual.hex(),
                        "trace": S.put(f"trace_{len(S.cases)}", R.trace),
                        "x": S.put(f"x_{len(S.cases)}", R.x), "x_norm": float(np.linalg.norm(R.x)).hex()})
        print(f"solve {solver} {pc} {mat.get('N', mat.get('n'))}: nits {R.nits} residual {R.residual:.8e}",
              flush=True)

    np.savez_compressed(os.path.join(HERE, "golden.npz"), **S.arrays)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "source": "oracle/_ref/libref.so "
                   "(reference compiled in place from /root/reference, g++ -O2)", "cases": S.cases}, f, indent=1)
    print(f"{len(S.cases)} cases, {len(S.arrays)} arrays")


if __name__ == "__main__":
    main()
