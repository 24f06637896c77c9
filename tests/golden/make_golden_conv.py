#!/usr/bin/env python3
"""Generate tests/golden/conv.npz + conv.json: format conversions computed by
the REFERENCE ITSELF (oracle/_ref/libref.so, matrix-utils.cxx:62-380,
:700-765, called through ref_shim.cxx).

Run in the dev container, where /root/reference exists:
    make -C oracle all ref && python tests/golden/make_golden_conv.py

Inputs and outputs are both stored (they are small): conv.npz holds arrays
`<case>__<name>` (loaded with allow_pickle=False), conv.json the case list.
The inputs come from conv_inputs() below (seeded numpy), so the script is the
whole recipe.
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
from inputs import conv_handmade_bcsr, conv_rand  # noqa: E402


def main():
    arrays, cases = {}, []

    def add(kind, name, params, inputs, outputs):
        key = f"{kind}_{name}"
        for k, v in list(inputs.items()) + list(outputs.items()):
            arrays[f"{key}__{k}"] = np.ascontiguousarray(v)
        cases.append({"kind": kind, "name": key, "params": params, "inputs": sorted(inputs),
                      "outputs": sorted(outputs)})

    mats = {}
    for dim, N in ((2, 6), (3, 4)):
        A = O.poisson(dim, N)
        mats[f"p{2 * dim + 1}_{N}"] = (A.n, A.n, A.Ap, A.Aj, A.Ax)
    for name, (nr, nc, k, seed, sp) in {"rnd_sq60": (60, 60, 7, 11, True), "rnd_sq48": (48, 48, 12, 12, False),
                                        "rnd_rect": (37, 53, 6, 13, True), "rnd_tall": (90, 7, 4, 14, False),
                                        "sparse_rows": (20, 20, 1, 15, False), "one_row": (1, 9, 9, 16, True),
                                        "empty": (6, 6, 0, 17, False)}.items():
        mats[name] = (nr, nc) + conv_rand(nr, nc, k, seed, sp)
    for name, (nr, nc, Ap, Aj, Ax) in mats.items():
        Ci, Cj, Cx = O.csr_to_coo(nr, nc, Ap, Aj, Ax, src="ref")
        add("csr_to_coo", name, {"nrows": nr, "ncols": nc}, {"Ap": Ap, "Aj": Aj, "Ax": Ax},
            {"Ci": Ci, "Cj": Cj, "Cx": Cx})
        Tp, Tj, Tx = O.transpose(nr, nc, Ap, Aj, Ax, src="ref")
        add("transpose", name, {"nrows": nr, "ncols": nc}, {"Ap": Ap, "Aj": Aj, "Ax": Ax},
            {"Tp": Tp, "Tj": Tj, "Tx": Tx})
        # coo_to_csr from the entries in a shuffled order (rows scattered, duplicates kept)
        perm = np.random.default_rng(len(name) * 7919 + nr).permutation(Ci.size)
        Si, Sj, Sx = Ci[perm], Cj[perm], Cx[perm]
        Bp, Bj, Bx = O.coo_to_csr(nr, nc, Si, Sj, Sx, src="ref")
        add("coo_to_csr", name, {"nrows": nr, "ncols": nc}, {"Ci": Si, "Cj": Sj, "Cx": Sx},
            {"Ap": Bp, "Aj": Bj, "Ax": Bx})
        if nr != nc or Ap[-1] == 0:
            continue
        for bs in (1, 2, 3, 4, 5, 6, 8):
            if nr % bs:
                continue
            Bp, Bj, Bx = O.csr_to_bcsr(nr, bs, Ap, Aj, Ax, src="ref")
            add("csr_to_bcsr", f"{name}_bs{bs}", {"n": nr, "bs": bs}, {"Ap": Ap, "Aj": Aj, "Ax": Ax},
                {"Bp": Bp, "Bj": Bj, "Bx": Bx})
            nb = nr // bs
            Cp, Cj2, Cx2 = O.bcsr_to_csr(nb, nb, bs, Bp, Bj, Bx, src="ref")
            add("bcsr_to_csr", f"{name}_bs{bs}", {"nbrows": nb, "nbcols": nb, "bs": bs},
                {"Bp": Bp, "Bj": Bj, "Bx": Bx}, {"Ap": Cp, "Aj": Cj2, "Ax": Cx2})
    for name, (nbr, nbc, bs, Bp, Bj, Bx) in conv_handmade_bcsr().items():
        Cp, Cj2, Cx2 = O.bcsr_to_csr(nbr, nbc, bs, Bp, Bj, Bx, src="ref")
        add("bcsr_to_csr", name, {"nbrows": nbr, "nbcols": nbc, "bs": bs}, {"Bp": Bp, "Bj": Bj, "Bx": Bx},
            {"Ap": Cp, "Aj": Cj2, "Ax": Cx2})

    np.savez_compressed(os.path.join(HERE, "conv.npz"), **arrays)
    with open(os.path.join(HERE, "conv.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden_conv.py",
                   "source": "oracle/_ref/libref.so (reference compiled in place, g++ -O2)", "cases": cases},
                  f, indent=1)
    print(f"{len(cases)} cases, {len(arrays)} arrays")


if __name__ == "__main__":
    main()
