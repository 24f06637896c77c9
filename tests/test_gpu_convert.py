"""Format conversions on the device (lssp_amd_csr_to_coo / _coo_to_csr /
_csr_transpose / _csr_to_bcsr / _bcsr_to_csr) -- bitwise:

  * against the reference's own outputs (tests/golden/conv.*),
  * against the CPU oracle (pinned by those fixtures) on random matrices of a
    few hundred thousand rows with repeated columns, empty rows and
    0 / -0.0 / NaN / inf values,
  * at BASELINE's full size (7-pt Poisson 216^3, 70 M entries) through
    properties: A^T == A (symmetric, sorted), coo -> csr and csr -> bcsr ->
    csr round trips return A exactly,
  * malformed inputs return LSSP_AMD_EINVAL instead of faulting.
"""
import numpy as np
import pytest

import oracle as O
from conv_util import conv_cases, same
from inputs import conv_rand

pytestmark = pytest.mark.gpu

CASES = conv_cases()


@pytest.fixture(scope="module")
def dev():
    import lssp_amd
    d = lssp_amd.Device(0)
    yield d
    d.close()


def _csr_to_dev(dev, Ap, Aj, Ax):
    return dev.idx(Ap.size, Ap), dev.idx(Aj.size, Aj), dev.vec(Ax.size, Ax)


def run_device(dev, kind, p, i):
    from lssp_amd import convert as C
    if kind == "csr_to_coo":
        out = C.csr_to_coo(dev, p["nrows"], int(i["Ap"][-1]), *_csr_to_dev(dev, i["Ap"], i["Aj"], i["Ax"]))
        return dict(zip(("Ci", "Cj", "Cx"), (a.download() for a in out)))
    if kind == "coo_to_csr":
        out = C.coo_to_csr(dev, p["nrows"], i["Ci"].size, *_csr_to_dev(dev, i["Ci"], i["Cj"], i["Cx"]))
        return dict(zip(("Ap", "Aj", "Ax"), (a.download() for a in out)))
    if kind == "transpose":
        out = C.transpose(dev, p["nrows"], p["ncols"], int(i["Ap"][-1]),
                          *_csr_to_dev(dev, i["Ap"], i["Aj"], i["Ax"]))
        return dict(zip(("Tp", "Tj", "Tx"), (a.download() for a in out)))
    if kind == "csr_to_bcsr":
        m, *out = C.csr_to_bcsr(dev, p["n"], int(i["Ap"][-1]), p["bs"],
                                *_csr_to_dev(dev, i["Ap"], i["Aj"], i["Ax"]))
        return dict(zip(("Bp", "Bj", "Bx"), (a.download() for a in out)))
    m, *out = C.bcsr_to_csr(dev, p["nbrows"], p["nbcols"], p["bs"], i["Bj"].size,
                            *_csr_to_dev(dev, i["Bp"], i["Bj"], i["Bx"]))
    return dict(zip(("Ap", "Aj", "Ax"), (a.download() for a in out)))


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_conversion_bitwise_vs_reference(dev, c):
    got = run_device(dev, c["kind"], c["params"], c["in"])
    for k, v in c["out"].items():
        assert same(got[k], v), k


@pytest.mark.parametrize("seed", [1, 2])
def test_coo_transpose_bitwise_vs_oracle_large(dev, seed):
    nr, nc = 300_000 + seed, 250_000
    Ap, Aj, Ax = conv_rand(nr, nc, 9, 300 + seed, specials=True)
    p = {"nrows": nr, "ncols": nc}
    got = run_device(dev, "csr_to_coo", p, {"Ap": Ap, "Aj": Aj, "Ax": Ax})
    want = O.csr_to_coo(nr, nc, Ap, Aj, Ax)
    assert all(same(got[k], w) for k, w in zip(("Ci", "Cj", "Cx"), want))
    got = run_device(dev, "transpose", p, {"Ap": Ap, "Aj": Aj, "Ax": Ax})
    want = O.transpose(nr, nc, Ap, Aj, Ax)
    assert all(same(got[k], w) for k, w in zip(("Tp", "Tj", "Tx"), want))
    Ci, Cj, Cx = O.csr_to_coo(nr, nc, Ap, Aj, Ax)
    perm = np.random.default_rng(seed).permutation(Ci.size)
    sh = {"Ci": Ci[perm], "Cj": Cj[perm], "Cx": Cx[perm]}
    got = run_device(dev, "coo_to_csr", p, sh)
    want = O.coo_to_csr(nr, nc, sh["Ci"], sh["Cj"], sh["Cx"])
    assert all(same(got[k], w) for k, w in zip(("Ap", "Aj", "Ax"), want))


@pytest.mark.parametrize("bs", [1, 2, 3, 5, 8])
def test_bcsr_bitwise_vs_oracle_large(dev, bs):
    n = 240_000
    Ap, Aj, Ax = conv_rand(n, n, 9, 400 + bs, specials=True)
    got = run_device(dev, "csr_to_bcsr", {"n": n, "bs": bs}, {"Ap": Ap, "Aj": Aj, "Ax": Ax})
    want = O.csr_to_bcsr(n, bs, Ap, Aj, Ax)
    assert all(same(got[k], w) for k, w in zip(("Bp", "Bj", "Bx"), want))
    nb = n // bs
    back = run_device(dev, "bcsr_to_csr", {"nbrows": nb, "nbcols": nb, "bs": bs},
                      {"Bp": want[0], "Bj": want[1], "Bx": want[2]})
    want2 = O.bcsr_to_csr(nb, nb, bs, *want)
    assert all(same(back[k], w) for k, w in zip(("Ap", "Aj", "Ax"), want2))


def test_bcsr_to_csr_unsorted_duplicate_blocks_vs_oracle(dev):
    # block rows with block columns out of order and repeated: the sort_column path on many rows
    rng = np.random.default_rng(9)
    nb, nbc, bs = 20_000, 5_000, 3
    lens = rng.integers(0, 6, nb)
    Bp = np.zeros(nb + 1, np.int32)
    np.cumsum(lens, out=Bp[1:])
    Bj = rng.integers(0, nbc, Bp[-1]).astype(np.int32)
    Bx = rng.uniform(-1, 1, Bj.size * bs * bs)
    Bx[rng.choice(Bx.size, Bx.size // 10, replace=False)] = 0.0
    got = run_device(dev, "bcsr_to_csr", {"nbrows": nb, "nbcols": nbc, "bs": bs}, {"Bp": Bp, "Bj": Bj, "Bx": Bx})
    want = O.bcsr_to_csr(nb, nbc, bs, Bp, Bj, Bx)
    assert all(same(got[k], w) for k, w in zip(("Ap", "Aj", "Ax"), want))


def test_full_size_round_trips(dev):
    """BASELINE's matrix (7-pt Poisson 216^3): A^T == A, COO and BCSR round trips exact"""
    import lssp_amd
    from lssp_amd import convert as C
    Ap, Aj, Ax = lssp_amd.poisson(3, 216)
    n, nnz = Ap.size - 1, Aj.size
    dAp, dAj, dAx = _csr_to_dev(dev, Ap, Aj, Ax)
    Tp, Tj, Tx = C.transpose(dev, n, n, nnz, dAp, dAj, dAx)
    assert same(Tp.download(), Ap) and same(Tj.download(), Aj) and same(Tx.download(), Ax)
    for a in (Tp, Tj, Tx):
        a.free()
    Ci, Cj, Cx = C.csr_to_coo(dev, n, nnz, dAp, dAj, dAx)
    Bp, Bj, Bx = C.coo_to_csr(dev, n, nnz, Ci, Cj, Cx)
    assert same(Bp.download(), Ap) and same(Bj.download(), Aj) and same(Bx.download(), Ax)
    for a in (Ci, Cj, Cx, Bp, Bj, Bx):
        a.free()
    m, Bp, Bj, Bx = C.csr_to_bcsr(dev, n, nnz, 6, dAp, dAj, dAx)
    k, Rp, Rj, Rx = C.bcsr_to_csr(dev, n // 6, n // 6, 6, m, Bp, Bj, Bx)
    assert k == nnz
    assert same(Rp.download(), Ap) and same(Rj.download(), Aj) and same(Rx.download(), Ax)


def test_malformed_inputs_raise_einval(dev):
    import lssp_amd
    from lssp_amd import convert as C
    Ap, Aj, Ax = conv_rand(100, 100, 5, 77)
    nnz = Aj.size

    def einval(fn, *a):
        with pytest.raises(lssp_amd.LsspError) as e:
            fn(dev, *a)
        assert e.value.status == 1

    bad_ptr = Ap.copy()
    bad_ptr[50] = bad_ptr[51] + 1                 # decreasing row pointers
    einval(C.csr_to_coo, 100, nnz, *_csr_to_dev(dev, bad_ptr, Aj, Ax))
    einval(C.transpose, 100, 100, nnz, *_csr_to_dev(dev, bad_ptr, Aj, Ax))
    einval(C.csr_to_coo, 100, nnz + 1, *_csr_to_dev(dev, Ap, Aj, Ax))   # Ap[n] != nnz
    bad_col = Aj.copy()
    bad_col[3] = 100                              # column out of range
    einval(C.transpose, 100, 100, nnz, *_csr_to_dev(dev, Ap, bad_col, Ax))
    einval(C.csr_to_bcsr, 100, nnz, 4, *_csr_to_dev(dev, Ap, bad_col, Ax))
    einval(C.csr_to_bcsr, 100, nnz, 3, *_csr_to_dev(dev, Ap, Aj, Ax))   # 100 % 3 != 0 (lssp_error there)
    Ci = np.repeat(np.arange(100, dtype=np.int32), np.diff(Ap))
    Ci[7] = -1                                    # row out of range
    einval(C.coo_to_csr, 100, nnz, *_csr_to_dev(dev, Ci, Aj, Ax))
    Bp = np.array([0, 1, 2], np.int32)
    Bj = np.array([0, 2], np.int32)               # block column 2 of 2
    einval(C.bcsr_to_csr, 2, 2, 2, 2, *_csr_to_dev(dev, Bp, Bj, np.ones(8)))
