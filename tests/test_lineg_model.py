"""Model of the one-workgroup 2-D sweeps' dataflow (lssp_amd/csrc/linefill.hip
k_lineg), CPU only.

A restatement in Python of what k_lineg computes: lane j = grid line j, one
level per step (v = i + j for ILU(0), i + 2 j for ILU(1)); the operands of row
(i, j) at level v are the lane's own x(v-1) (W), lane j-1's x(v-1) (ILU(0): S;
ILU(1): SE -- lane 0 of a wave reads the previous wave's lane 63) and, for
ILU(1), lane j-1's x(v-2) (S: the lane's SE of the level before), subtracted in
the reference's column order; rows off the grid hold +0.0.  The U sweep is the
same recurrence in mirrored coordinates on the L sweep's output.  The stream
index map (g2_at: [level][wave][component][64 lanes]) is checked to be a
bijection onto the stream.  Bitwise against the oracle's apply.
"""
import numpy as np
import pytest

import oracle as O
from test_gpu_parity import _box7


def g2_at(v, NW, NC, k, j):
    return ((v * NW + (j >> 6)) * (NC + 1) + k) * 64 + (j & 63)


def sweep(nx, ny, fill, coef, rhs, unit):
    """coef[rs] = (S, (SE,) W, (diag)) of sweep row rs = j nx + i"""
    SK = 2 if fill else 1
    V = nx + SK * (ny - 1)
    xp = np.zeros(ny)  # x(v-1) per lane
    sp = np.zeros(ny)  # ILU(1): lane j-1's x(v-2)
    out = np.zeros(nx * ny)
    for v in range(V):
        se = np.concatenate([[0.0], xp[:-1]])  # lane j-1's x(v-1) (line -1: +0.0)
        x = np.zeros(ny)
        for j in range(ny):
            i = v - SK * j
            if not 0 <= i < nx:
                continue
            c = coef[j * nx + i]
            if fill:
                t = rhs[j * nx + i] - c[0] * sp[j]
                t = t - c[1] * se[j]
                t = t - c[2] * xp[j]
                if not unit:
                    t = t / c[3]
            else:
                t = rhs[j * nx + i] - c[0] * se[j]
                t = t - c[1] * xp[j]
                if not unit:
                    t = t / c[2]
            x[j] = t
            out[j * nx + i] = t
        sp, xp = se, x
    return out


def model_apply(nx, ny, level, seed=3):
    Ap, Aj, Ax = _box7(nx, ny, 1, seed)
    n = Ap.size - 1
    L, U = O.ilu(O.CSR(n, Ap, Aj, Ax), "iluk", level=level)
    fill = level == 1
    offs = [nx, nx - 1, 1] if fill else [nx, 1]  # S, (SE,) W: r - off (L) / r + off (U)
    cl = np.zeros((n, len(offs)))
    cu = np.zeros((n, len(offs) + 1))
    for r in range(n):
        for q in range(L.Ap[r], L.Ap[r + 1] - 1):
            cl[r, offs.index(r - L.Aj[q])] = L.Ax[q]
        rs = n - 1 - r  # U in mirrored (sweep) order
        cu[rs, -1] = U.Ax[U.Ap[r]]
        for q in range(U.Ap[r] + 1, U.Ap[r + 1]):
            cu[rs, offs.index(U.Aj[q] - r)] = U.Ax[q]
    rhs = np.random.default_rng(seed + 1).uniform(-1, 1, n)
    y = sweep(nx, ny, fill, cl, rhs, unit=True)
    xs = sweep(nx, ny, fill, cu, y[::-1].copy(), unit=False)
    return xs[::-1], O.ilu_apply(L, U, rhs)


@pytest.mark.parametrize("nx,ny", [(3, 3), (9, 8), (30, 27), (5, 65), (4, 130)])
@pytest.mark.parametrize("level", [0, 1])
def test_lineg_dataflow_model_bitwise_vs_oracle(nx, ny, level):
    if level == 0 and ny < 8:
        pytest.skip("ILU(0) line sweeps need ny >= 8")
    got, want = model_apply(nx, ny, level)
    assert np.array_equal(got.view(np.int64), want.view(np.int64))


@pytest.mark.parametrize("ny,NC", [(3, 3), (64, 4), (65, 2), (200, 4), (256, 3)])
def test_lineg_stream_index_is_a_bijection(ny, NC):
    NYP = (ny + 63) // 64 * 64
    NW, V = NYP // 64, 7
    idx = [g2_at(v, NW, NC, k, j) for v in range(V) for k in range(NC + 1) for j in range(NYP)]
    assert sorted(idx) == list(range(V * (NC + 1) * NYP))
