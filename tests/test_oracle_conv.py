"""Format conversions (matrix-utils.cxx:62-380, :700-765): the CPU oracle
against the reference's own outputs (tests/golden/conv.*, made by
tests/golden/make_golden_conv.py from oracle/_ref/libref.so), bitwise."""
import numpy as np
import pytest

import oracle as O
from conv_util import conv_cases, same
from inputs import conv_handmade_bcsr, conv_rand

CASES = conv_cases()


def run_oracle(c, src="orc"):
    p, i = c["params"], c["in"]
    k = c["kind"]
    if k == "csr_to_coo":
        return dict(zip(("Ci", "Cj", "Cx"), O.csr_to_coo(p["nrows"], p["ncols"], i["Ap"], i["Aj"], i["Ax"], src)))
    if k == "coo_to_csr":
        return dict(zip(("Ap", "Aj", "Ax"), O.coo_to_csr(p["nrows"], p["ncols"], i["Ci"], i["Cj"], i["Cx"], src)))
    if k == "transpose":
        return dict(zip(("Tp", "Tj", "Tx"), O.transpose(p["nrows"], p["ncols"], i["Ap"], i["Aj"], i["Ax"], src)))
    if k == "csr_to_bcsr":
        return dict(zip(("Bp", "Bj", "Bx"), O.csr_to_bcsr(p["n"], p["bs"], i["Ap"], i["Aj"], i["Ax"], src)))
    return dict(zip(("Ap", "Aj", "Ax"), O.bcsr_to_csr(p["nbrows"], p["nbcols"], p["bs"], i["Bp"], i["Bj"],
                                                        i["Bx"], src)))


def test_fixture_covers_every_conversion_and_edge():
    kinds = {c["kind"] for c in CASES}
    assert kinds == {"csr_to_coo", "coo_to_csr", "transpose", "csr_to_bcsr", "bcsr_to_csr"}
    names = {c["name"] for c in CASES}
    for n in ("transpose_empty", "coo_to_csr_rnd_rect", "bcsr_to_csr_dup_blocks_bs1",
              "bcsr_to_csr_specials_bs3", "bcsr_to_csr_no_blocks", "csr_to_bcsr_rnd_sq60_bs5"):
        assert n in names


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_oracle_matches_reference_fixture(c):
    got = run_oracle(c)
    for k, v in c["out"].items():
        assert same(got[k], v), k


@pytest.mark.skipif(not O.ref_available(), reason="reference checker not built (make -C oracle ref)")
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_oracle_matches_reference_larger(seed):
    nr, nc = 3000 + seed * 17, 2500
    Ap, Aj, Ax = conv_rand(nr, nc, 9, 100 + seed, specials=True)
    for f in (O.csr_to_coo, O.transpose):
        a, b = f(nr, nc, Ap, Aj, Ax, "orc"), f(nr, nc, Ap, Aj, Ax, "ref")
        assert all(same(x, y) for x, y in zip(a, b))
    Ci, Cj, Cx = O.csr_to_coo(nr, nc, Ap, Aj, Ax)
    perm = np.random.default_rng(seed).permutation(Ci.size)
    a = O.coo_to_csr(nr, nc, Ci[perm], Cj[perm], Cx[perm], "orc")
    b = O.coo_to_csr(nr, nc, Ci[perm], Cj[perm], Cx[perm], "ref")
    assert all(same(x, y) for x, y in zip(a, b))
    n = 2520
    Ap, Aj, Ax = conv_rand(n, n, 9, 200 + seed, specials=True)
    for bs in (1, 3, 7, 8):
        a, b = O.csr_to_bcsr(n, bs, Ap, Aj, Ax, "orc"), O.csr_to_bcsr(n, bs, Ap, Aj, Ax, "ref")
        assert all(same(x, y) for x, y in zip(a, b))
        nb = n // bs
        c1 = O.bcsr_to_csr(nb, nb, bs, *a, "orc")
        c2 = O.bcsr_to_csr(nb, nb, bs, *a, "ref")
        assert all(same(x, y) for x, y in zip(c1, c2))


def test_bcsr_round_trip_drops_only_zero_and_nan():
    n = 96
    Ap, Aj, Ax = conv_rand(n, n, 6, 5, specials=True)
    Bp, Bj, Bx = O.csr_to_bcsr(n, 4, Ap, Aj, Ax)
    Cp, Cj, Cx = O.bcsr_to_csr(n // 4, n // 4, 4, Bp, Bj, Bx)
    assert np.all(np.abs(Cx) > 0)
    # every surviving entry is the last value the row stored for its column
    for i in range(n):
        last = {}
        for k in range(Ap[i], Ap[i + 1]):
            last[int(Aj[k])] = Ax[k]
        want = sorted((c, v) for c, v in last.items() if abs(v) > 0)
        got = list(zip(Cj[Cp[i]:Cp[i + 1]].tolist(), Cx[Cp[i]:Cp[i + 1]].tolist()))
        assert got == want


def test_handmade_bcsr_inputs_are_well_formed():
    for nbr, nbc, bs, Bp, Bj, Bx in conv_handmade_bcsr().values():
        assert Bp[0] == 0 and Bp[-1] == Bj.size and Bx.size == Bj.size * bs * bs
        assert np.all(Bj < nbc) and Bp.size == nbr + 1
