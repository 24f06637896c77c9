"""Load tests/golden/ (generated from the reference by make_golden.py) and
rebuild each case's inputs from its recorded parameters."""
from __future__ import annotations

import json
import os

import numpy as np

import oracle as O
from inputs import digest, rand_csr, uniform

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_cache = {}


def manifest():
    if "m" not in _cache:
        with open(os.path.join(HERE, "manifest.json")) as f:
            _cache["m"] = json.load(f)
        _cache["npz"] = dict(np.load(os.path.join(HERE, "golden.npz"), allow_pickle=False))
    return _cache["m"]


def cases(kind):
    return [c for c in manifest()["cases"] if c["kind"] == kind]


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


def matches(entry, *arrays) -> bool:
    """bitwise: the digest covers dtype and every byte"""
    return digest(*arrays) == entry["sha256"]


def stored(entry):
    manifest()
    if "npz" not in entry:
        return None
    return [_cache["npz"][f"{entry['npz']}__{i}"] for i in range(entry["count"])]


def fx(h: str) -> float:
    return float.fromhex(h)


def case_id(c) -> str:
    m = c["mat"]
    mat = f"p{m['dim'] * 2 + 1 if m['dim'] == 3 else 5}_{m['N']}" if m["type"] == "poisson" else f"rand{m['n']}_{m['seed']}"
    if c["kind"] == "spmv":
        return f"{mat}-op{c['op']}-b{fx(c['beta'])}"
    pc = c["pc"]
    pcs = pc["kind"] + "".join(f"_{k}{v}" for k, v in pc.items() if k != "kind")
    if c["kind"] == "ilu":
        return f"{mat}-{pcs}"
    return f"s{c['solver']}-{pcs}-{mat}-b{c['b']}-m{c['maxit']}"
