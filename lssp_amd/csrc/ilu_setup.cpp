// ilu_setup.cpp -- host setup of the ILU preconditioners and the sync-free
// trisolve schedules.
//
// The factorization runs once per assemble on the host, like the reference
// (SURVEY 3(A)); the apply is the GPU hot path.  The arithmetic is the
// reference's, operation for operation (pc-iluk.cxx, pc-ilut.cxx,
// matrix-utils.cxx), so the factors are bitwise the reference's.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <exception>

#include "internal.h"

namespace lssp_amd {

namespace {

constexpr double ZERO_DIAG_VALUE = 1e-3;  // pc.cxx:6
constexpr double ZERO_DIAG_TOL = 1e-10;   // pc.cxx:7

// matrix-utils.cxx:483-587 -- a row without a diagonal gets (i, tol) at its
// sorted position.  (The reference leaves num_nnzs stale here, so its ILU(0)
// and ILUT then read past the copied arrays; we insert the entry as intended.)
HostCSR adjust_zero_diag(HostCSR &&A, double tol)
{
    const int n = A.n;
    bool all = true;  // the common case: every row has its diagonal -- no copy
    for (int i = 0; i < n && all; i++) {
        bool has = false;
        for (int k = A.Ap[i]; k < A.Ap[i + 1] && !has; k++) has = A.Aj[k] == i;
        all = has;
    }
    if (all) return std::move(A);
    HostCSR M;
    M.n = n;
    M.ncols = A.ncols;
    M.Ap.assign(n + 1, 0);
    M.Aj.reserve(A.Aj.size() + 16);
    M.Ax.reserve(A.Ax.size() + 16);
    for (int i = 0; i < n; i++) {
        bool has = false;
        for (int k = A.Ap[i]; k < A.Ap[i + 1]; k++) has |= A.Aj[k] == i;
        size_t start = M.Aj.size();
        for (int k = A.Ap[i]; k < A.Ap[i + 1]; k++) {
            M.Aj.push_back(A.Aj[k]);
            M.Ax.push_back(A.Ax[k]);
        }
        if (!has) {
            M.Aj.push_back(i);
            M.Ax.push_back(tol);
            for (long j = (long)M.Aj.size() - 2; j >= (long)start; j--) {
                if (M.Aj[j] <= M.Aj[j + 1]) break;
                std::swap(M.Aj[j], M.Aj[j + 1]);
                std::swap(M.Ax[j], M.Ax[j + 1]);
            }
        }
        M.Ap[i + 1] = (int)M.Aj.size();
    }
    return M;
}

// matrix-utils.cxx:589-698
HostCSR block_diag(HostCSR &&A, int blk)
{
    const int n = A.n;
    if (blk >= n) return std::move(A);
    HostCSR M;
    M.n = n;
    M.ncols = A.ncols;
    M.Ap.assign(n + 1, 0);
    for (int i = 0; i < n; i++) {
        const int s = (i / blk) * blk, e = std::min(s + blk, n);
        size_t before = M.Aj.size();
        for (int k = A.Ap[i]; k < A.Ap[i + 1]; k++)
            if (A.Aj[k] >= s && A.Aj[k] < e) {
                M.Aj.push_back(A.Aj[k]);
                M.Ax.push_back(A.Ax[k]);
            }
        if (M.Aj.size() == before) {
            M.Aj.push_back(i);
            M.Ax.push_back(1.0);
        }
        M.Ap[i + 1] = (int)M.Aj.size();
    }
    return M;
}

// pc-iluk.cxx:22-135 (levels of fill), :186-229 (assembly), :231-277 (values)
HostCSR iluk_symbolic(const HostCSR &A, int level)
{
    const int n = A.n;
    if (level < 0) level = 0;
    std::vector<int> lev(n), buf(n), pos(n, -1);
    std::vector<std::vector<int>> Lrow(n), Urow(n), Ulev(n);
    for (int i = 0; i < n; i++) {
        int nl = 0, nu = i;
        for (int k = A.Ap[i]; k < A.Ap[i + 1]; k++) {
            const int col = A.Aj[k];
            if (col < i) {
                buf[nl] = col;
                lev[nl] = 0;
                pos[col] = nl++;
            } else if (col > i) {
                buf[nu] = col;
                lev[nu] = 0;
                pos[col] = nu++;
            }
        }
        for (int piv = 0; piv < nl; piv++) {
            int k = buf[piv], kmin = k, at = piv;
            for (int j = piv + 1; j < nl; j++)
                if (buf[j] < kmin) {
                    kmin = buf[j];
                    at = j;
                }
            if (at != piv) {
                buf[piv] = kmin;
                buf[at] = k;
                pos[kmin] = piv;
                pos[k] = at;
                std::swap(lev[piv], lev[at]);
                k = kmin;
            }
            const std::vector<int> &uc = Urow[k], &ul = Ulev[k];
            for (size_t j = 0; j < uc.size(); j++) {
                const int col = uc[j];
                const int it = ul[j] + lev[piv] + 1;
                if (it > level) continue;
                const int q = pos[col];
                if (q == -1) {
                    if (col < i) {
                        buf[nl] = col;
                        lev[nl] = it;
                        pos[col] = nl++;
                    } else if (col > i) {
                        buf[nu] = col;
                        lev[nu] = it;
                        pos[col] = nu++;
                    }
                } else if (lev[q] < it) {
                    lev[q] = it;
                }
            }
        }
        for (int j = 0; j < nl; j++) pos[buf[j]] = -1;
        for (int j = i; j < nu; j++) pos[buf[j]] = -1;
        Lrow[i].assign(buf.begin(), buf.begin() + nl);
        Urow[i].assign(buf.begin() + i, buf.begin() + nu);
        Ulev[i].assign(lev.begin() + i, lev.begin() + nu);
    }
    HostCSR M;
    M.n = n;
    M.ncols = n;
    M.Ap.assign(n + 1, 0);
    for (int i = 0; i < n; i++) {
        for (int c : Lrow[i]) M.Aj.push_back(c);
        M.Aj.push_back(i);
        for (int c : Urow[i]) M.Aj.push_back(c);
        M.Ap[i + 1] = (int)M.Aj.size();
        Ulev[i].clear();
        Ulev[i].shrink_to_fit();
    }
    M.Ax.assign(M.Aj.size(), 0.0);
    std::vector<double> wk(n, 0.0);
    for (int i = 0; i < n; i++) {
        for (int k = A.Ap[i]; k < A.Ap[i + 1]; k++) wk[A.Aj[k]] = A.Ax[k];
        for (int k = M.Ap[i]; k < M.Ap[i + 1]; k++) M.Ax[k] = wk[M.Aj[k]];
        for (int k = A.Ap[i]; k < A.Ap[i + 1]; k++) wk[A.Aj[k]] = 0;
    }
    sort_columns(M);
    return M;
}

// pc-iluk.cxx:347-409 -- IKJ ILU(0) in place on a sorted local block; the
// multiplier uses the stored reciprocal pivot.
void ilu0_factor(int n, const int *Ap, const int *C, double *Ax)
{
    std::vector<double> wk(n, 0.0), dinv(n);
    double d0 = Ax[Ap[0]];
    if (std::fabs(d0) < ZERO_DIAG_TOL) d0 = d0 > 0 ? ZERO_DIAG_VALUE : -ZERO_DIAG_VALUE;
    dinv[0] = 1. / d0;
    for (int i = 1; i < n; i++) {
        const int end = Ap[i + 1];
        int k = Ap[i];
        for (; k < end && C[k] < i; k++) {
            const int r = C[k];
            for (int q = Ap[r]; q < Ap[r + 1]; q++) wk[C[q]] = Ax[q];
            const double aik = Ax[k] = Ax[k] * dinv[r];
            for (int j = k + 1; j < end; j++)
                if (wk[C[j]] != 0.) Ax[j] = Ax[j] - aik * wk[C[j]];
            for (int q = Ap[r]; q < Ap[r + 1]; q++) wk[C[q]] = 0;
        }
        double d = ZERO_DIAG_VALUE;
        if (k < end && C[k] == i) {
            if (std::fabs(Ax[k]) < ZERO_DIAG_TOL) Ax[k] = ZERO_DIAG_VALUE;
            d = Ax[k];
        }
        dinv[i] = 1. / d;
    }
}

// pc-ilut.cxx:7-49
void qsplit(double *a, int *ind, int n, int ncut)
{
    int first = 0, last = n - 1;
    if (ncut < first || ncut >= last) return;
    for (;;) {
        int mid = first;
        const double key = std::fabs(a[mid]);
        for (int j = first + 1; j <= last; j++)
            if (std::fabs(a[j]) > key) {
                mid++;
                std::swap(a[mid], a[j]);
                std::swap(ind[mid], ind[j]);
            }
        std::swap(a[mid], a[first]);
        std::swap(ind[mid], ind[first]);
        if (mid == ncut) return;
        if (mid > ncut) last = mid - 1;
        else first = mid + 1;
    }
}

// pc-ilut.cxx:51-286 -- ILUT(tol, p) of one local block, written straight into
// the split factors the sweeps use: L (strict entries in the reference's row
// order, then the unit diagonal LAST) and U (pivot FIRST, then the U part).
// The reference stores a row as L part, diagonal, U part; splitting that row
// the way ilu_factor splits any factor (entries before the diagonal to L, the
// diagonal as 1.0 to L and as the pivot to U, the rest to U) gives exactly
// these rows, so no combined factor is kept and no split pass runs.  Row 0 is
// A's row as is (:89-96), so U's row 0 is A's row 0 entry for entry.
void ilut_factor_lu(const HostCSR &A, double tol, int p, HostCSR &L, HostCSR &U)
{
    const int n = A.n;
    L = HostCSR();
    U = HostCSR();
    L.n = L.ncols = U.n = U.ncols = n;
    L.Ap.assign(n + 1, 0);
    U.Ap.assign(n + 1, 0);
    // a row keeps at most p L and p U entries plus its diagonal (:256-274):
    // reserving that bound (address space only; pages are touched as rows are
    // appended) means the factors are never regrown and copied mid-way -- at
    // 256^3 a regrowth moved ~4 GB and first-touched ~8 GB more.  p beyond
    // n-1 keeps no more than a full row; a reservation the host refuses falls
    // back to a modest one and the vectors grow as the reference's realloc does
    // (pc-ilut.cxx:71, :215-222)
    const size_t pc = p >= 0 ? (size_t)std::min(p, std::max(n - 1, 0)) : 0;
    const size_t row0 = (size_t)(A.Ap[1] - A.Ap[0]);
    const size_t capl = p >= 0 ? (size_t)n * (pc + 1) : A.Aj.size() * 2;
    const size_t capu = p >= 0 ? (size_t)n * (pc + 1) + row0 : A.Aj.size() * 2;
    try {
        L.Aj.reserve(capl);
        L.Ax.reserve(capl);
        U.Aj.reserve(capu);
        U.Ax.reserve(capu);
    } catch (const std::exception &) {
        const size_t small = std::max(A.Aj.size() * 2, (size_t)n * 4);
        L.Aj.reserve(std::min(capl, small));
        L.Ax.reserve(std::min(capl, small));
        U.Aj.reserve(std::min(capu, small));
        U.Ax.reserve(std::min(capu, small));
    }
    std::vector<double> w(n), diag(n);
    std::vector<int> jr(n, -1), jw(n);
    for (int k = A.Ap[0]; k < A.Ap[1]; k++) {  // row 0 as is (:89-96)
        if (A.Aj[k] == 0) {
            L.Aj.push_back(0);
            L.Ax.push_back(1.0);
        }
        U.Aj.push_back(A.Aj[k]);
        U.Ax.push_back(A.Ax[k]);
    }
    L.Ap[1] = (int)L.Aj.size();
    U.Ap[1] = (int)U.Aj.size();
    diag[0] = A.Ax[A.Ap[0]];
    if (std::fabs(diag[0]) < ZERO_DIAG_TOL) diag[0] = diag[0] > 0 ? ZERO_DIAG_VALUE : -ZERO_DIAG_VALUE;

    for (int i = 1; i < n; i++) {
        const int b = A.Ap[i], e = A.Ap[i + 1];
        double norm = 0.0;
        for (int k = b; k < e; k++) norm += std::fabs(A.Ax[k]);
        norm /= (double)(e - b);
        const double rel = tol * norm;
        int nl = 0, nu = 0;
        jw[i] = i;
        w[i] = 0.0;
        jr[i] = i;
        for (int k = b; k < e; k++) {
            const int col = A.Aj[k];
            if (col < i) {
                jr[col] = nl;
                jw[nl] = col;
                w[nl] = A.Ax[k];
                nl++;
            } else if (col == i) {
                w[i] = A.Ax[k];
            } else {
                nu++;
                jr[col] = i + nu;
                jw[i + nu] = col;
                w[i + nu] = A.Ax[k];
            }
        }
        for (int j = 0; j < nl; j++) {
            int jrow = jw[j], at = j;
            for (int k = j + 1; k < nl; k++)
                if (jw[k] < jrow) {
                    jrow = jw[k];
                    at = k;
                }
            if (at != j) {
                const int col = jw[j];
                jw[j] = jw[at];
                jw[at] = col;
                jr[jrow] = j;
                jr[col] = at;
                std::swap(w[j], w[at]);
            }
            jr[jrow] = -1;
            const double aik = w[j] = w[j] / diag[jrow];
            // the pivot row's entries past its diagonal, in stored order: U's row
            // without its leading pivot (row 0: A's row, filtered by col)
            for (int k = jrow ? U.Ap[jrow] + 1 : 0; k < U.Ap[jrow + 1]; k++) {
                const int col = U.Aj[k];
                if (col <= jrow) continue;
                const int q = jr[col];
                const double mx = -aik * U.Ax[k];
                if (q == -1 && std::fabs(mx) < rel) continue;
                if (col < i) {
                    if (q == -1) {
                        jw[nl] = col;
                        jr[col] = nl;
                        w[nl] = mx;
                        nl++;
                    } else {
                        w[q] += mx;
                    }
                } else {
                    if (q == -1) {
                        nu++;
                        jw[i + nu] = col;
                        jr[col] = i + nu;
                        w[i + nu] = mx;
                    } else {
                        w[q] += mx;
                    }
                }
            }
        }
        diag[i] = w[i];
        jr[i] = -1;
        for (int j = 0; j < nl; j++) jr[jw[j]] = -1;
        for (int j = 0; j < nu; j++) jr[jw[i + j + 1]] = -1;
        if (std::fabs(diag[i]) < ZERO_DIAG_TOL) diag[i] = diag[i] > 0 ? ZERO_DIAG_VALUE : -ZERO_DIAG_VALUE;
        int len = std::min(nl, p);
        qsplit(w.data(), jw.data(), nl, len);
        for (int k = 0; k < len; k++) {
            L.Ax.push_back(w[k]);
            L.Aj.push_back(jw[k]);
        }
        L.Ax.push_back(1.0);
        L.Aj.push_back(i);
        U.Ax.push_back(diag[i]);
        U.Aj.push_back(i);
        len = std::min(nu, p);
        qsplit(w.data() + i + 1, jw.data() + i + 1, nu, len);
        for (int k = 0; k < len; k++) {
            U.Ax.push_back(w[i + 1 + k]);
            U.Aj.push_back(jw[i + 1 + k]);
        }
        L.Ap[i + 1] = (int)L.Aj.size();
        U.Ap[i + 1] = (int)U.Aj.size();
    }
}

HostCSR local_block(const HostCSR &F, int s, int e)
{
    HostCSR B;
    B.n = B.ncols = e - s;
    const int base = F.Ap[s];
    B.Ap.resize(B.n + 1);
    for (int i = 0; i <= B.n; i++) B.Ap[i] = F.Ap[s + i] - base;
    B.Aj.resize(F.Ap[e] - base);
    B.Ax.resize(F.Ap[e] - base);
    for (size_t k = 0; k < B.Aj.size(); k++) {
        B.Aj[k] = F.Aj[base + k] - s;
        B.Ax[k] = F.Ax[base + k];
    }
    return B;
}

}  // namespace

// matrix-utils.cxx:387-481 -- unsorted rows only; entries bucketed by column
void sort_columns(HostCSR &A)
{
    if (A.n <= 0 || A.ncols <= 0 || A.Aj.empty()) return;
    std::vector<double> val;
    std::vector<int> cols;
    for (int i = 0; i < A.n; i++) {
        const int b = A.Ap[i], e = A.Ap[i + 1];
        bool need = false;
        for (int j = b + 1; j < e; j++)
            if (A.Aj[j - 1] > A.Aj[j]) {
                need = true;
                break;
            }
        if (!need) continue;
        if (val.empty()) val.resize(A.ncols);
        cols.assign(A.Aj.begin() + b, A.Aj.begin() + e);
        for (int j = b; j < e; j++) val[A.Aj[j]] = A.Ax[j];
        std::sort(cols.begin(), cols.end());
        for (int j = b; j < e; j++) {
            A.Aj[j] = cols[j - b];
            A.Ax[j] = val[cols[j - b]];
        }
    }
}

// pc-iluk.cxx:411-581 / pc-ilut.cxx:288-456: adjust_zero_diag, optional
// symbolic ILU(k), block-diagonal extraction, per-block factorization, split
// into L (unit diagonal LAST) and U (pivot FIRST).
void ilu_factor(lssp_amd_ctx *c, int kind, HostCSR &&A0, int level, double tol, int p, int blk, HostCSR &L,
                HostCSR &U, int *status)
{
    *status = LSSP_AMD_OK;
    const int n = A0.n;
    if (kind == LSSP_AMD_ILUT && p <= 0) p = (A0.Ap[n] + n - 1) / n;  // pc-ilut.cxx:436-438
    HostCSR Az = adjust_zero_diag(std::move(A0), ZERO_DIAG_TOL);
    setup_mark("adjust_zero_diag");
    if (blk <= 0 || blk > n) blk = n;
    HostCSR M;
    if (kind == LSSP_AMD_ILUK && level > 0) {
        HostCSR S = iluk_symbolic(Az, level);
        M = block_diag(std::move(S), blk);
    } else {
        M = block_diag(std::move(Az), blk);
    }
    Az = HostCSR();
    setup_mark("symbolic / block_diag");

    HostCSR F;
    static const bool host_ilu0 = getenv("LSSP_AMD_ILU_HOST") && atoi(getenv("LSSP_AMD_ILU_HOST"));
    if (kind == LSSP_AMD_ILUK && c && !host_ilu0) {
        // the numeric ILU(0) of every block at once, on the GPU (ilu_factor.hip)
        *status = ilu0_factor_gpu(c, n, blk, M.Ap, M.Aj, M.Ax);
        if (*status != LSSP_AMD_OK) return;
        F = std::move(M);
    }
    F.n = F.ncols = n;
    if (kind == LSSP_AMD_ILUT) {
        // ILUT writes L and U directly (ilut_factor_lu); one block (the
        // reference's default blk_size = n) needs no block copy at all
        if (blk >= n) {
            ilut_factor_lu(M, tol, p, L, U);
        } else {
            L = HostCSR();
            U = HostCSR();
            L.n = L.ncols = U.n = U.ncols = n;
            L.Ap.assign(n + 1, 0);
            U.Ap.assign(n + 1, 0);
            for (int s = 0; s < n; s += blk) {
                const int e = std::min(s + blk, n);
                HostCSR Lb, Ub;
                ilut_factor_lu(local_block(M, s, e), tol, p, Lb, Ub);
                for (int i = 0; i < Lb.n; i++) {
                    for (int k = Lb.Ap[i]; k < Lb.Ap[i + 1]; k++) {
                        L.Aj.push_back(Lb.Aj[k] + s);
                        L.Ax.push_back(Lb.Ax[k]);
                    }
                    for (int k = Ub.Ap[i]; k < Ub.Ap[i + 1]; k++) {
                        U.Aj.push_back(Ub.Aj[k] + s);
                        U.Ax.push_back(Ub.Ax[k]);
                    }
                    L.Ap[s + i + 1] = (int)L.Aj.size();
                    U.Ap[s + i + 1] = (int)U.Aj.size();
                }
            }
        }
        M = HostCSR();
        setup_mark("numeric factorization (into L, U)");
        return;
    }
    if (F.Ap.empty()) {
    F.Ap.assign(n + 1, 0);
    F.Aj.reserve(M.Aj.size());
    F.Ax.reserve(M.Ax.size());
    for (int s = 0; s < n; s += blk) {
        const int e = std::min(s + blk, n);
        HostCSR B = local_block(M, s, e);
        ilu0_factor(B.n, B.Ap.data(), B.Aj.data(), B.Ax.data());
        for (int i = 0; i < B.n; i++) {
            for (int k = B.Ap[i]; k < B.Ap[i + 1]; k++) {
                F.Aj.push_back(B.Aj[k] + s);
                F.Ax.push_back(B.Ax[k]);
            }
            F.Ap[s + i + 1] = (int)F.Aj.size();
        }
    }
    }
    M = HostCSR();
    setup_mark("numeric factorization");

    // split: row counts first, then every entry written in place
    L.n = U.n = L.ncols = U.ncols = n;
    L.Ap.assign(n + 1, 0);
    U.Ap.assign(n + 1, 0);
    parallel_for(n, [&](long i0, long i1) {
        for (int i = (int)i0; i < (int)i1; i++) {
            int nl = 0, nu = 0;
            for (int k = F.Ap[i]; k < F.Ap[i + 1]; k++) {
                const int c = F.Aj[k];
                nl += c <= i;
                nu += c >= i;
            }
            L.Ap[i + 1] = nl;
            U.Ap[i + 1] = nu;
        }
    });
    for (int i = 0; i < n; i++) {
        L.Ap[i + 1] += L.Ap[i];
        U.Ap[i + 1] += U.Ap[i];
    }
    L.Aj.resize(L.Ap[n]);
    L.Ax.resize(L.Ap[n]);
    U.Aj.resize(U.Ap[n]);
    U.Ax.resize(U.Ap[n]);
    parallel_for(n, [&](long i0, long i1) {
    for (int i = (int)i0; i < (int)i1; i++) {
        int pl = L.Ap[i], pu = U.Ap[i];
        for (int k = F.Ap[i]; k < F.Ap[i + 1]; k++) {
            const int c = F.Aj[k];
            if (c < i) {
                L.Aj[pl] = c;
                L.Ax[pl++] = F.Ax[k];
            } else if (c == i) {
                L.Aj[pl] = c;
                L.Ax[pl++] = 1;
                U.Aj[pu] = c;
                U.Ax[pu++] = F.Ax[k];
            } else {
                U.Aj[pu] = c;
                U.Ax[pu++] = F.Ax[k];
            }
        }
    }
    });
    setup_mark("L/U split");
}

// Level analysis + upload of one triangular factor.
//   lower: diagonal is the LAST entry of each row; strict entries summed in
//          ascending storage order (solver-tri.cxx:13-19)
//   upper: diagonal is the FIRST entry; strict entries summed in DESCENDING
//          storage order (solver-tri.cxx:35-41) -- stored reversed here so the
//          kernel always walks forward.
// dependency levels of a triangular factor's rows (forward for L, backward for
// U); dependencies must point strictly below (lower) / above (upper): a row is
// only ever waited on by later-scheduled rows
int tri_levels(int n, const std::vector<int> &Tp, const std::vector<int> &Tj, bool upper, std::vector<int> &lev)
{
    lev.assign(n, 0);
    for (int i = 0; i < n; i++)
        if (Tp[i + 1] - Tp[i] < 1) return LSSP_AMD_EINVAL;  // no diagonal slot
    if (!upper) {
        for (int i = 0; i < n; i++) {
            int l = 0;
            for (int k = Tp[i]; k < Tp[i + 1] - 1; k++) {
                const int j = Tj[k];
                if (j < 0 || j >= i) return LSSP_AMD_EINVAL;
                l = std::max(l, lev[j] + 1);
            }
            lev[i] = l;
        }
    } else {
        for (int i = n - 1; i >= 0; i--) {
            int l = 0;
            for (int k = Tp[i] + 1; k < Tp[i + 1]; k++) {
                const int j = Tj[k];
                if (j <= i || j >= n) return LSSP_AMD_EINVAL;
                l = std::max(l, lev[j] + 1);
            }
            lev[i] = l;
        }
    }
    return LSSP_AMD_OK;
}

int build_trisched(lssp_amd_ctx *c, int n, const std::vector<int> &Tp, const std::vector<int> &Tj,
                   const std::vector<double> &Tx, bool upper, TriSched &t, const TriSched *prod, bool packets,
                   bool arrays, std::vector<int> *lev_in)
{
    t.n = n;
    std::vector<int> lev;
    SetupTimer tm;
    if (lev_in) lev.swap(*lev_in);
    else LSSP_TRY(tri_levels(n, Tp, Tj, upper, lev));
    tm.mark(upper ? "U levels" : "L levels");
    if ((int)lev.size() != n) return LSSP_AMD_EINVAL;
    long nstrict = 0;
    bool unit = true;
    for (int i = 0; i < n; i++) {
        nstrict += Tp[i + 1] - Tp[i] - 1;
        const double d = upper ? Tx[Tp[i]] : Tx[Tp[i + 1] - 1];
        unit &= d == 1.0;
    }
    int nlev = 0;
    for (int i = 0; i < n; i++) nlev = std::max(nlev, lev[i] + 1);
    t.nlevels = n ? nlev : 0;
    if (packets) LSSP_TRY(build_bp_schedule(c, n, Tp, Tj, Tx, upper, lev, t, prod));
    if (!arrays) return LSSP_AMD_OK;  // line sweeps: only the level count is reported
    // counting sort by level; rows of a level stay in row order (lower) or in
    // descending row order (upper, mirroring the backward sweep)
    std::vector<int> start(nlev + 1, 0), perm(n);
    for (int i = 0; i < n; i++) start[lev[i] + 1]++;
    for (int l = 0; l < nlev; l++) start[l + 1] += start[l];
    t.level_ptr = start;
    t.max_level_rows = 0;
    for (int l = 0; l < nlev; l++) t.max_level_rows = std::max(t.max_level_rows, start[l + 1] - start[l]);
    if (!upper) {
        for (int i = 0; i < n; i++) perm[start[lev[i]]++] = i;
    } else {
        for (int i = n - 1; i >= 0; i--) perm[start[lev[i]]++] = i;
    }
    std::vector<int> rp(n + 1, 0), cols;
    std::vector<double> vals, diag;
    cols.reserve(nstrict);
    vals.reserve(nstrict);
    if (!unit) diag.resize(n);
    for (int p = 0; p < n; p++) {
        const int i = perm[p];
        if (!upper) {
            for (int k = Tp[i]; k < Tp[i + 1] - 1; k++) {
                cols.push_back(Tj[k]);
                vals.push_back(Tx[k]);
            }
            if (!unit) diag[p] = Tx[Tp[i + 1] - 1];
        } else {
            for (int k = Tp[i + 1] - 1; k > Tp[i]; k--) {
                cols.push_back(Tj[k]);
                vals.push_back(Tx[k]);
            }
            if (!unit) diag[p] = Tx[Tp[i]];
        }
        rp[p + 1] = (int)cols.size();
    }
    t.nnz = (int)cols.size();
    t.unit = unit ? 1 : 0;
    LSSP_HIP(hipMalloc(&t.perm, sizeof(int) * std::max(n, 1)));
    LSSP_HIP(hipMalloc(&t.rp, sizeof(int) * (n + 1)));
    LSSP_HIP(hipMalloc(&t.cols, sizeof(int) * std::max<size_t>(cols.size(), 1)));
    LSSP_HIP(hipMalloc(&t.vals, sizeof(double) * std::max<size_t>(vals.size(), 1)));
    LSSP_HIP(hipMemcpy(t.perm, perm.data(), sizeof(int) * n, hipMemcpyHostToDevice));
    LSSP_HIP(hipMemcpy(t.rp, rp.data(), sizeof(int) * (n + 1), hipMemcpyHostToDevice));
    if (!cols.empty()) {
        LSSP_HIP(hipMemcpy(t.cols, cols.data(), sizeof(int) * cols.size(), hipMemcpyHostToDevice));
        LSSP_HIP(hipMemcpy(t.vals, vals.data(), sizeof(double) * vals.size(), hipMemcpyHostToDevice));
    }
    if (!unit) {
        LSSP_HIP(hipMalloc(&t.diag, sizeof(double) * n));
        LSSP_HIP(hipMemcpy(t.diag, diag.data(), sizeof(double) * n, hipMemcpyHostToDevice));
    }
    (void)c;
    return LSSP_AMD_OK;
}

void free_trisched(TriSched &t)
{
    if (t.perm) (void)hipFree(t.perm);
    if (t.rp) (void)hipFree(t.rp);
    if (t.cols) (void)hipFree(t.cols);
    if (t.vals) (void)hipFree(t.vals);
    if (t.diag) (void)hipFree(t.diag);
    for (void *p : {(void *)t.bp_perm, (void *)t.bp_pos, (void *)t.pk6_blk, (void *)t.pk6_desc, (void *)t.pk6_idx, (void *)t.pk6_rec,
                    (void *)t.pk6_claim})
        if (p) (void)hipFree(p);
    t = TriSched();
}

}  // namespace lssp_amd
