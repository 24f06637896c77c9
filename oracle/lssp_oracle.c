/*
 * lssp_oracle.c -- CPU restatement of the LSSP Krylov hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * product path in lssp_amd/.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it.  The product never links it.
 *
 * Every function restates the algorithm of the reference (huiscliu/lssp,
 * mounted read-only at /root/reference) in its own code; the citations give
 * the reference file:line it follows.  Floating-point operation order is kept
 * exactly as in the reference, and the file is compiled with
 * -O2 -ffp-contract=off (no FMA contraction), so results are bit-identical to
 * a g++ -O2 (x86-64 baseline, no -march) build of the reference.  The
 * restatement is pinned against the reference itself: oracle/_ref/libref.so is
 * compiled from the reference sources in place (oracle/Makefile) and
 * tests/golden/ holds the vectors it produced (tests/golden/make_golden.py).
 *
 * Besides the reference's serial dot product (vector.cxx:123-133), the oracle
 * implements the GPU's canonical tree reduction order (LSSP_AMD reduction
 * contract) and the P-rank row-block partitioned order,
 * so that the GPU solvers can be checked bit-for-bit in every mode.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define EXPORT __attribute__((visibility("default")))

/* reference defaults: pc.cxx:6-7 and lssp.cxx:5-14 */
static const double ZERO_DIAG_VALUE = 1e-3;
static const double ZERO_DIAG_TOL = 1e-10;
static const double BREAKDOWN = 1e-40;
static const int DEF_MAXIT = 1000;
static const int DEF_RESTART = 50;
static const double DEF_TOL = 1e-7;

typedef struct {
    int nrows, ncols, nnz;
    int *Ap, *Aj;
    double *Ax;
} csr_t;

static void csr_free(csr_t *A)
{
    free(A->Ap);
    free(A->Aj);
    free(A->Ax);
    memset(A, 0, sizeof(*A));
}

static csr_t csr_alloc(int nrows, int ncols, int nnz)
{
    csr_t A;
    A.nrows = nrows;
    A.ncols = ncols;
    A.nnz = nnz;
    A.Ap = (int *)malloc(sizeof(int) * (size_t)(nrows + 1));
    A.Aj = (int *)malloc(sizeof(int) * (size_t)(nnz > 0 ? nnz : 1));
    A.Ax = (double *)malloc(sizeof(double) * (size_t)(nnz > 0 ? nnz : 1));
    return A;
}

static csr_t csr_copy(int n, int ncols, const int *Ap, const int *Aj, const double *Ax)
{
    csr_t A = csr_alloc(n, ncols, Ap[n]);
    memcpy(A.Ap, Ap, sizeof(int) * (size_t)(n + 1));
    memcpy(A.Aj, Aj, sizeof(int) * (size_t)Ap[n]);
    memcpy(A.Ax, Ax, sizeof(double) * (size_t)Ap[n]);
    return A;
}

/* ------------------------------------------------------------------------ */
/* Reductions                                                               */
/* ------------------------------------------------------------------------ */

enum { RED_SERIAL = 0, RED_TREE = 1 };

/* vector.cxx:123-133: sum += x[i]*y[i], from 0, in index order */
static double dot_serial(const double *x, const double *y, long n)
{
    double s = 0;
    for (long i = 0; i < n; i++) s += x[i] * y[i];
    return s;
}

/* One 64-lane wave: xor-butterfly == halving tree, lane 0 result. */
static double wave64(double *v)
{
    for (int off = 32; off >= 1; off >>= 1)
        for (int l = 0; l < off; l++) v[l] = v[l] + v[l + off];
    return v[0];
}

/* Level 1 of the canonical GPU order: one aligned chunk of 256 products,
 * zero padded, four waves each halving, then (w0+w1)+(w2+w3). */
static double chunk256(const double *x, const double *y, long base, long n)
{
    double w[4];
    for (int q = 0; q < 4; q++) {
        double v[64];
        for (int l = 0; l < 64; l++) {
            long i = base + 64 * q + l;
            v[l] = (i < n) ? x[i] * y[i] : 0.0;
        }
        w[q] = wave64(v);
    }
    return (w[0] + w[1]) + (w[2] + w[3]);
}

/* Level 2: 1024 lanes, lane t adds S[t], S[t+1024], ... onto 0.0 in order,
 * then 16 waves halve, then the 16 wave results halve. */
static double level2(const double *S, long C)
{
    double acc[1024];
    for (int t = 0; t < 1024; t++) {
        double a = 0.0;
        for (long k = t; k < C; k += 1024) a += S[k];
        acc[t] = a;
    }
    double u[16];
    for (int q = 0; q < 16; q++) u[q] = wave64(acc + 64 * q);
    for (int off = 8; off >= 1; off >>= 1)
        for (int l = 0; l < off; l++) u[l] = u[l] + u[l + off];
    return u[0];
}

static double dot_tree(const double *x, const double *y, long n)
{
    long C = (n + 255) / 256;
    if (C == 0) return level2(NULL, 0);
    double *S = (double *)malloc(sizeof(double) * (size_t)C);
    for (long c = 0; c < C; c++) S[c] = chunk256(x, y, 256 * c, n);
    double r = level2(S, C);
    free(S);
    return r;
}

/* Reduction context: mode + P-rank row-block partition (blk = ceil(n/P)). */
typedef struct {
    int mode;
    int nranks;
} red_t;

/* SERIAL: the reference's one sequential sum over the whole vector for any P
 * (the library's ranks continue each other's running sums, comm.cpp);
 * TREE: each rank's block in the canonical tree order, rank sums in rank order. */
static double dot_red(const red_t *R, const double *x, const double *y, long n)
{
    if (R->mode != RED_TREE) return dot_serial(x, y, n);
    int P = R->nranks > 1 ? R->nranks : 1;
    long blk = (n + P - 1) / P;
    double total = 0.0;
    for (int r = 0; r < P; r++) {
        long s = (long)r * blk, e = s + blk;
        if (s > n) s = n;
        if (e > n) e = n;
        double part = dot_tree(x + s, y + s, e - s);
        total = r == 0 ? part : total + part;
    }
    return total;
}

EXPORT double orc_dot(int mode, int nranks, const double *x, const double *y, long n)
{
    red_t R = {mode, nranks};
    return dot_red(&R, x, y, n);
}

/* ------------------------------------------------------------------------ */
/* L1 kernels: SpMV (mvops.cxx), BLAS-1 (vector.cxx), trisolve               */
/* ------------------------------------------------------------------------ */

static double row_sum(const csr_t *A, const double *x, int i)
{
    double sum = 0;
    for (int jj = A->Ap[i]; jj < A->Ap[i + 1]; jj++) sum += x[A->Aj[jj]] * A->Ax[jj];
    return sum;
}

/* mvops.cxx:42-69  z = y*beta + alpha*(A x) */
static void mv_amxpbyz(double alpha, const csr_t *A, const double *x, double beta,
                       const double *y, double *z)
{
    for (int i = 0; i < A->nrows; i++) z[i] = y[i] * beta + alpha * row_sum(A, x, i);
}

/* mvops.cxx:118-142  y = A x */
static void mv_mxy(const csr_t *A, const double *x, double *y)
{
    for (int i = 0; i < A->nrows; i++) y[i] = row_sum(A, x, i);
}

EXPORT void orc_spmv(int op, int n, const int *Ap, const int *Aj, const double *Ax,
                     double alpha, const double *x, double beta, const double *y, double *z)
{
    /* op 0: mxy (mvops.cxx:118), 1: amxy (:81), 2: amxpby in place on z (:5),
     * 3: amxpbyz (:42). Ap == NULL means the zero matrix, as in the reference. */
    for (int i = 0; i < n; i++) {
        double sum = 0;
        if (Ap != NULL)
            for (int jj = Ap[i]; jj < Ap[i + 1]; jj++) sum += x[Aj[jj]] * Ax[jj];
        switch (op) {
        case 0: z[i] = Ap ? sum : 0; break;
        case 1: z[i] = Ap ? sum * alpha : 0; break;
        case 2: z[i] = Ap ? sum * alpha + z[i] * beta : z[i] * beta; break;
        default: z[i] = Ap ? y[i] * beta + alpha * sum : y[i] * beta; break;
        }
    }
}

/* solver-tri.cxx:4-24: diagonal stored LAST, ascending storage-order sum */
static void tri_lower(const csr_t *L, double *x, const double *rhs)
{
    for (int i = 0; i < L->nrows; i++) {
        int end = L->Ap[i + 1] - 1;
        double r = rhs[i];
        for (int j = L->Ap[i]; j < end; j++) r = r - L->Ax[j] * x[L->Aj[j]];
        x[i] = r / L->Ax[end];
    }
}

/* solver-tri.cxx:26-46: diagonal stored FIRST, descending storage-order sum */
static void tri_upper(const csr_t *U, double *x, const double *rhs)
{
    for (int i = U->nrows - 1; i >= 0; i--) {
        int d = U->Ap[i];
        double r = rhs[i];
        for (int j = U->Ap[i + 1] - 1; j > d; j--) r = r - U->Ax[j] * x[U->Aj[j]];
        x[i] = r / U->Ax[d];
    }
}

EXPORT void orc_ilu_apply(int n, const int *Lp, const int *Lj, const double *Lx,
                          const int *Up, const int *Uj, const double *Ux,
                          double *x, const double *rhs)
{
    /* solver-tri.cxx:48-60: cache = L^-1 rhs; x = U^-1 cache */
    csr_t L = {n, n, Lp[n], (int *)Lp, (int *)Lj, (double *)Lx};
    csr_t U = {n, n, Up[n], (int *)Up, (int *)Uj, (double *)Ux};
    double *cache = (double *)malloc(sizeof(double) * (size_t)n);
    tri_lower(&L, cache, rhs);
    tri_upper(&U, x, cache);
    free(cache);
}

EXPORT void orc_trisolve(int upper, int n, const int *Ap, const int *Aj, const double *Ax,
                         double *x, const double *rhs)
{
    csr_t T = {n, n, Ap[n], (int *)Ap, (int *)Aj, (double *)Ax};
    if (upper) tri_upper(&T, x, rhs);
    else tri_lower(&T, x, rhs);
}

/* ------------------------------------------------------------------------ */
/* Matrix utilities (matrix-utils.cxx)                                      */
/* ------------------------------------------------------------------------ */

/* matrix-utils.cxx:387-481: only unsorted rows are touched; entries are
 * bucketed by column (a duplicate column keeps the last value for every
 * occurrence) and the column list is sorted ascending. */
static int cmp_int(const void *a, const void *b)
{
    int x = *(const int *)a, y = *(const int *)b;
    return (x > y) - (x < y);
}

static void sort_columns(csr_t *A)
{
    if (A->nrows <= 0 || A->ncols <= 0 || A->nnz <= 0) return;
    double *val = (double *)malloc(sizeof(double) * (size_t)A->ncols);
    int *cols = (int *)malloc(sizeof(int) * (size_t)A->ncols);
    for (int i = 0; i < A->nrows; i++) {
        int b = A->Ap[i], e = A->Ap[i + 1], need = 0;
        for (int j = b + 1; j < e; j++)
            if (A->Aj[j - 1] > A->Aj[j]) { need = 1; break; }
        if (!need) continue;
        int m = 0;
        for (int j = b; j < e; j++) {
            val[A->Aj[j]] = A->Ax[j];
            cols[m++] = A->Aj[j];
        }
        qsort(cols, (size_t)m, sizeof(int), cmp_int);
        for (int j = b, t = 0; j < e; j++, t++) {
            A->Aj[j] = cols[t];
            A->Ax[j] = val[cols[t]];
        }
    }
    free(val);
    free(cols);
}

/* matrix-utils.cxx:483-587: rows without a diagonal get (i, tol) inserted at
 * its sorted position (appended, then bubbled left). */
static csr_t adjust_zero_diag(const csr_t *A, double tol)
{
    int n = A->nrows, missing = 0;
    char *has = (char *)calloc((size_t)n, 1);
    for (int i = 0; i < n; i++)
        for (int j = A->Ap[i]; j < A->Ap[i + 1]; j++)
            if (A->Aj[j] == i) has[i] = 1;
    for (int i = 0; i < n; i++) missing += !has[i];
    csr_t M = csr_alloc(n, A->ncols, A->nnz + missing);
    M.Ap[0] = 0;
    for (int i = 0; i < n; i++) M.Ap[i + 1] = M.Ap[i] + (A->Ap[i + 1] - A->Ap[i]) + !has[i];
    for (int i = 0; i < n; i++) {
        int o = M.Ap[i];
        for (int j = A->Ap[i]; j < A->Ap[i + 1]; j++, o++) {
            M.Aj[o] = A->Aj[j];
            M.Ax[o] = A->Ax[j];
        }
        if (has[i]) continue;
        M.Aj[o] = i;
        M.Ax[o] = tol;
        for (int j = M.Ap[i + 1] - 2; j >= M.Ap[i]; j--) {
            if (M.Aj[j] <= M.Aj[j + 1]) break;
            int tj = M.Aj[j];
            double tx = M.Ax[j];
            M.Aj[j] = M.Aj[j + 1];
            M.Ax[j] = M.Ax[j + 1];
            M.Aj[j + 1] = tj;
            M.Ax[j + 1] = tx;
        }
    }
    free(has);
    return M;
}

/* matrix-utils.cxx:589-698: keep entries whose column lies in the row's
 * block; an emptied row becomes (j, 1.0).  blk == n is a plain copy. */
static csr_t block_diag(const csr_t *A, int blk)
{
    int n = A->nrows;
    if (blk == n) return csr_copy(n, A->ncols, A->Ap, A->Aj, A->Ax);
    int *cnt = (int *)calloc((size_t)n + 1, sizeof(int));
    long total = 0;
    for (int i = 0; i < n; i++) {
        int s = (i / blk) * blk, e = s + blk < n ? s + blk : n;
        for (int k = A->Ap[i]; k < A->Ap[i + 1]; k++)
            if (A->Aj[k] >= s && A->Aj[k] < e) cnt[i]++;
        if (cnt[i] == 0) cnt[i] = -1;
        total += cnt[i] > 0 ? cnt[i] : 1;
    }
    csr_t M = csr_alloc(n, A->ncols, (int)total);
    M.Ap[0] = 0;
    int o = 0;
    for (int i = 0; i < n; i++) {
        int s = (i / blk) * blk, e = s + blk < n ? s + blk : n;
        if (cnt[i] > 0) {
            for (int k = A->Ap[i]; k < A->Ap[i + 1]; k++)
                if (A->Aj[k] >= s && A->Aj[k] < e) {
                    M.Aj[o] = A->Aj[k];
                    M.Ax[o] = A->Ax[k];
                    o++;
                }
        } else {
            M.Aj[o] = i;
            M.Ax[o] = 1;
            o++;
        }
        M.Ap[i + 1] = o;
    }
    free(cnt);
    return M;
}

/* ------------------------------------------------------------------------ */
/* ILUK (pc-iluk.cxx)                                                       */
/* ------------------------------------------------------------------------ */

/* pc-iluk.cxx:22-135 + :186-229 + :231-277: level-of-fill symbolic ILU(k).
 * Returns the ILU(k) pattern with A's values (0 on fill), rows sorted. */
static csr_t iluk_symbolic(const csr_t *A, int level)
{
    int n = A->nrows;
    if (level < 0) level = 0;
    int *lev = (int *)malloc(sizeof(int) * (size_t)n);
    int *buf = (int *)malloc(sizeof(int) * (size_t)n);
    int *pos = (int *)malloc(sizeof(int) * (size_t)n);
    int **Lrow = (int **)calloc((size_t)n, sizeof(int *));
    int **Urow = (int **)calloc((size_t)n, sizeof(int *));
    int **Ulev = (int **)calloc((size_t)n, sizeof(int *));
    int *Ln = (int *)calloc((size_t)n, sizeof(int));
    int *Un = (int *)calloc((size_t)n, sizeof(int));
    for (int j = 0; j < n; j++) pos[j] = -1;

    for (int i = 0; i < n; i++) {
        int nl = 0, nu = i;
        for (int jj = A->Ap[i]; jj < A->Ap[i + 1]; jj++) {
            int c = A->Aj[jj];
            if (c < i) {
                buf[nl] = c;
                lev[nl] = 0;
                pos[c] = nl++;
            } else if (c > i) {
                buf[nu] = c;
                lev[nu] = 0;
                pos[c] = nu++;
            }
        }
        for (int piv = 0; piv < nl; piv++) {
            /* bring the smallest remaining lower column to slot piv */
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
                int t = lev[piv];
                lev[piv] = lev[at];
                lev[at] = t;
                k = kmin;
            }
            for (int j = 0; j < Un[k]; j++) {
                int c = Urow[k][j];
                int it = Ulev[k][j] + lev[piv] + 1;
                if (it > level) continue;
                int p = pos[c];
                if (p == -1) {
                    if (c < i) {
                        buf[nl] = c;
                        lev[nl] = it;
                        pos[c] = nl++;
                    } else if (c > i) {
                        buf[nu] = c;
                        lev[nu] = it;
                        pos[c] = nu++;
                    }
                } else if (lev[p] < it) {
                    lev[p] = it;
                }
            }
        }
        for (int j = 0; j < nl; j++) pos[buf[j]] = -1;
        for (int j = i; j < nu; j++) pos[buf[j]] = -1;
        Ln[i] = nl;
        if (nl) {
            Lrow[i] = (int *)malloc(sizeof(int) * (size_t)nl);
            memcpy(Lrow[i], buf, sizeof(int) * (size_t)nl);
        }
        Un[i] = nu - i;
        if (Un[i]) {
            Urow[i] = (int *)malloc(sizeof(int) * (size_t)Un[i]);
            Ulev[i] = (int *)malloc(sizeof(int) * (size_t)Un[i]);
            memcpy(Urow[i], buf + i, sizeof(int) * (size_t)Un[i]);
            memcpy(Ulev[i], lev + i, sizeof(int) * (size_t)Un[i]);
        }
    }

    long nnz = 0;
    for (int i = 0; i < n; i++) nnz += Ln[i] + Un[i] + 1;
    csr_t M = csr_alloc(n, n, (int)nnz);
    M.Ap[0] = 0;
    int o = 0;
    for (int i = 0; i < n; i++) {
        for (int j = 0; j < Ln[i]; j++) M.Aj[o++] = Lrow[i][j];
        M.Aj[o++] = i;
        for (int j = 0; j < Un[i]; j++) M.Aj[o++] = Urow[i][j];
        M.Ap[i + 1] = o;
    }
    /* pc-iluk.cxx:231-277: values of A where the pattern matches, else 0 */
    double *wk = (double *)calloc((size_t)n, sizeof(double));
    for (int i = 0; i < n; i++) {
        for (int j = A->Ap[i]; j < A->Ap[i + 1]; j++) wk[A->Aj[j]] = A->Ax[j];
        for (int j = M.Ap[i]; j < M.Ap[i + 1]; j++) M.Ax[j] = wk[M.Aj[j]];
        for (int j = A->Ap[i]; j < A->Ap[i + 1]; j++) wk[A->Aj[j]] = 0;
    }
    free(wk);
    sort_columns(&M);

    for (int i = 0; i < n; i++) {
        free(Lrow[i]);
        free(Urow[i]);
        free(Ulev[i]);
    }
    free(Lrow);
    free(Urow);
    free(Ulev);
    free(Ln);
    free(Un);
    free(lev);
    free(buf);
    free(pos);
    return M;
}

/* pc-iluk.cxx:347-409: in-place IKJ ILU(0) on a sorted local block.
 * Multipliers use the stored reciprocal pivot (diag[] holds 1/pivot). */
static void ilu0_factor(int n, const int *Ap, const int *C, double *Ax)
{
    double *wk = (double *)calloc((size_t)n, sizeof(double));
    double *dinv = (double *)malloc(sizeof(double) * (size_t)n);
    double d0 = Ax[Ap[0]];
    if (fabs(d0) < ZERO_DIAG_TOL) d0 = d0 > 0 ? ZERO_DIAG_VALUE : -ZERO_DIAG_VALUE;
    dinv[0] = 1. / d0;
    for (int i = 1; i < n; i++) {
        int end = Ap[i + 1], k;
        for (k = Ap[i]; k < end && C[k] < i; k++) {
            int r = C[k];
            for (int q = Ap[r]; q < Ap[r + 1]; q++) wk[C[q]] = Ax[q];
            double aik = Ax[k] = Ax[k] * dinv[r];
            for (int j = k + 1; j < end; j++)
                if (wk[C[j]] != 0.) Ax[j] = Ax[j] - aik * wk[C[j]];
            for (int q = Ap[r]; q < Ap[r + 1]; q++) wk[C[q]] = 0;
        }
        double d = ZERO_DIAG_VALUE;
        if (k < end && C[k] == i) {
            if (fabs(Ax[k]) < ZERO_DIAG_TOL) Ax[k] = ZERO_DIAG_VALUE;
            d = Ax[k];
        }
        dinv[i] = 1. / d;
    }
    free(wk);
    free(dinv);
}

/* pc-iluk.cxx:501-532 / pc-ilut.cxx:378-405: split a factored row-set into
 * L (strict lower + unit diagonal LAST) and U (pivot FIRST + upper). */
static void split_lu(const csr_t *F, csr_t *L, csr_t *U)
{
    int n = F->nrows;
    long nl = 0, nu = 0;
    for (int i = 0; i < n; i++)
        for (int k = F->Ap[i]; k < F->Ap[i + 1]; k++) {
            if (F->Aj[k] <= i) nl++;
            if (F->Aj[k] >= i) nu++;
        }
    *L = csr_alloc(n, n, (int)nl);
    *U = csr_alloc(n, n, (int)nu);
    int ol = 0, ou = 0;
    L->Ap[0] = U->Ap[0] = 0;
    for (int i = 0; i < n; i++) {
        for (int k = F->Ap[i]; k < F->Ap[i + 1]; k++) {
            int c = F->Aj[k];
            if (c < i) {
                L->Aj[ol] = c;
                L->Ax[ol++] = F->Ax[k];
            } else if (c == i) {
                L->Aj[ol] = c;
                L->Ax[ol++] = 1;
                U->Aj[ou] = c;
                U->Ax[ou++] = F->Ax[k];
            } else {
                U->Aj[ou] = c;
                U->Ax[ou++] = F->Ax[k];
            }
        }
        L->Ap[i + 1] = ol;
        U->Ap[i + 1] = ou;
    }
}

/* ------------------------------------------------------------------------ */
/* ILUT (pc-ilut.cxx)                                                       */
/* ------------------------------------------------------------------------ */

/* pc-ilut.cxx:7-49: partial quicksort by |a|; the ncut largest end up first */
static void qsplit(double *a, int *ind, int n, int ncut)
{
    int first = 0, last = n - 1;
    if (ncut < first || ncut >= last) return;
    for (;;) {
        int mid = first;
        double key = fabs(a[mid]);
        for (int j = first + 1; j <= last; j++) {
            if (fabs(a[j]) > key) {
                mid++;
                double t = a[mid];
                a[mid] = a[j];
                a[j] = t;
                int ti = ind[mid];
                ind[mid] = ind[j];
                ind[j] = ti;
            }
        }
        double t = a[mid];
        a[mid] = a[first];
        a[first] = t;
        int ti = ind[mid];
        ind[mid] = ind[first];
        ind[first] = ti;
        if (mid == ncut) return;
        if (mid > ncut) last = mid - 1;
        else first = mid + 1;
    }
}

/* pc-ilut.cxx:51-286: row-wise ILUT(tol, p) of one local block. */
static csr_t ilut_factor(const csr_t *A, double tol, int p)
{
    int n = A->nrows;
    const int *Ap = A->Ap, *C = A->Aj;
    const double *Ax = A->Ax;
    long cap = 8L * n + A->nnz + 16;
    csr_t M = csr_alloc(n, n, 0);
    M.Aj = (int *)realloc(M.Aj, sizeof(int) * (size_t)cap);
    M.Ax = (double *)realloc(M.Ax, sizeof(double) * (size_t)cap);
    double *w = (double *)malloc(sizeof(double) * (size_t)n);
    double *diag = (double *)malloc(sizeof(double) * (size_t)n);
    int *jr = (int *)malloc(sizeof(int) * (size_t)n);
    int *jw = (int *)malloc(sizeof(int) * (size_t)n);

    /* row 0 is copied unchanged (pc-ilut.cxx:89-96) */
    long off = 0;
    M.Ap[0] = 0;
    for (int k = Ap[0]; k < Ap[1]; k++, off++) {
        M.Ax[off] = Ax[k];
        M.Aj[off] = C[k];
    }
    M.Ap[1] = (int)off;
    diag[0] = Ax[Ap[0]];
    if (fabs(diag[0]) < ZERO_DIAG_TOL) diag[0] = diag[0] > 0 ? ZERO_DIAG_VALUE : -ZERO_DIAG_VALUE;
    for (int i = 0; i < n; i++) jr[i] = -1;

    for (int i = 1; i < n; i++) {
        int end = Ap[i + 1], nl = 0, nu = 0;
        double norm = 0.0;
        for (int k = Ap[i]; k < end; k++) norm += fabs(Ax[k]);
        norm /= (double)(end - Ap[i]);
        double rel = tol * norm;

        jw[i] = i;
        w[i] = 0.0;
        jr[i] = i;
        for (int k = Ap[i]; k < end; k++) {
            int c = C[k];
            if (c < i) {
                jr[c] = nl;
                jw[nl] = c;
                w[nl] = Ax[k];
                nl++;
            } else if (c == i) {
                w[i] = Ax[k];
            } else {
                nu++;
                jr[c] = i + nu;
                jw[i + nu] = c;
                w[i + nu] = Ax[k];
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
                int c = jw[j];
                jw[j] = jw[at];
                jw[at] = c;
                jr[jrow] = j;
                jr[c] = at;
                double t = w[j];
                w[j] = w[at];
                w[at] = t;
            }
            jr[jrow] = -1;
            double aik = w[j] = w[j] / diag[jrow];
            for (int k = M.Ap[jrow]; k < M.Ap[jrow + 1]; k++) {
                int c = M.Aj[k];
                if (c <= jrow) continue;
                int q = jr[c];
                double mx = -aik * M.Ax[k];
                if (q == -1 && fabs(mx) < rel) continue;
                if (c < i) {
                    if (q == -1) {
                        jw[nl] = c;
                        jr[c] = nl;
                        w[nl] = mx;
                        nl++;
                    } else {
                        w[q] += mx;
                    }
                } else {
                    if (q == -1) {
                        nu++;
                        jw[i + nu] = c;
                        jr[c] = i + nu;
                        w[i + nu] = mx;
                    } else {
                        w[q] += mx;
                    }
                }
            }
        }

        if (cap - off < (long)n + 2) {
            cap += 2L * n + 16;
            M.Aj = (int *)realloc(M.Aj, sizeof(int) * (size_t)cap);
            M.Ax = (double *)realloc(M.Ax, sizeof(double) * (size_t)cap);
        }

        diag[i] = w[i];
        jr[i] = -1;
        for (int j = 0; j < nl; j++) jr[jw[j]] = -1;
        for (int j = 0; j < nu; j++) jr[jw[i + j + 1]] = -1;
        if (fabs(diag[i]) < ZERO_DIAG_TOL) diag[i] = diag[i] > 0 ? ZERO_DIAG_VALUE : -ZERO_DIAG_VALUE;

        int len = nl < p ? nl : p;
        qsplit(w, jw, nl, len);
        for (int k = 0; k < len; k++, off++) {
            M.Ax[off] = w[k];
            M.Aj[off] = jw[k];
        }
        M.Ax[off] = diag[i];
        M.Aj[off] = i;
        off++;
        len = nu < p ? nu : p;
        qsplit(w + i + 1, jw + i + 1, nu, len);
        for (int k = 0; k < len; k++, off++) {
            M.Ax[off] = w[i + 1 + k];
            M.Aj[off] = jw[i + 1 + k];
        }
        M.Ap[i + 1] = (int)off;
    }
    M.nnz = (int)off;
    free(w);
    free(diag);
    free(jr);
    free(jw);
    return M;
}

/* ------------------------------------------------------------------------ */
/* Preconditioner assembly: pc-iluk.cxx:411-581, pc-ilut.cxx:288-456         */
/* ------------------------------------------------------------------------ */

typedef struct {
    csr_t L, U;
} ilu_t;

/* Extract rows [s,e) of F as a local CSR (columns shifted by -s). */
static csr_t local_block(const csr_t *F, int s, int e)
{
    int nb = e - s, base = F->Ap[s];
    csr_t B = csr_alloc(nb, nb, F->Ap[e] - base);
    for (int i = 0; i <= nb; i++) B.Ap[i] = F->Ap[s + i] - base;
    for (int k = 0; k < B.nnz; k++) {
        B.Aj[k] = F->Aj[base + k] - s;
        B.Ax[k] = F->Ax[base + k];
    }
    return B;
}

/* kind 0: ILUK(level), kind 1: ILUT(tol, p).  blk = block-Jacobi block size
 * (the reference API always passes n: pc-iluk.cxx:574, pc-ilut.cxx:449). */
EXPORT void *orc_ilu_create(int kind, int n, const int *Ap, const int *Aj, const double *Ax,
                            int level, double tol, int p, int blk)
{
    csr_t A = csr_copy(n, n, Ap, Aj, Ax);
    sort_columns(&A); /* lssp.cxx:173 (solver assemble sorts its copy) */
    /* pc-ilut.cxx:436-438: p <= 0 becomes ceil(nnz/n) of the solver's matrix */
    if (kind == 1 && p <= 0) p = (A.nnz + n - 1) / n;
    csr_t Az = adjust_zero_diag(&A, ZERO_DIAG_TOL);
    csr_free(&A);
    if (blk <= 0 || blk > n) blk = n;
    csr_t M;
    if (kind == 0 && level > 0) {
        csr_t S = iluk_symbolic(&Az, level);
        M = block_diag(&S, blk);
        csr_free(&S);
    } else {
        M = block_diag(&Az, blk);
    }
    csr_free(&Az);

    /* factor every block locally, re-globalise the columns */
    csr_t F = csr_alloc(n, n, 0);
    long cap = kind == 0 ? M.nnz : (long)M.nnz + 8L * n, o = 0;
    F.Aj = (int *)realloc(F.Aj, sizeof(int) * (size_t)(cap + 1));
    F.Ax = (double *)realloc(F.Ax, sizeof(double) * (size_t)(cap + 1));
    F.Ap[0] = 0;
    for (int s = 0; s < n; s += blk) {
        int e = s + blk < n ? s + blk : n;
        csr_t B = local_block(&M, s, e), T;
        if (kind == 0) {
            ilu0_factor(B.nrows, B.Ap, B.Aj, B.Ax);
            T = B;
        } else {
            T = ilut_factor(&B, tol, p);
            csr_free(&B);
        }
        if (o + T.nnz > cap) {
            cap = o + T.nnz + 2L * n;
            F.Aj = (int *)realloc(F.Aj, sizeof(int) * (size_t)cap);
            F.Ax = (double *)realloc(F.Ax, sizeof(double) * (size_t)cap);
        }
        for (int i = 0; i < T.nrows; i++) {
            for (int k = T.Ap[i]; k < T.Ap[i + 1]; k++, o++) {
                F.Aj[o] = T.Aj[k] + s;
                F.Ax[o] = T.Ax[k];
            }
            F.Ap[s + i + 1] = (int)o;
        }
        csr_free(&T);
    }
    F.nnz = (int)o;
    csr_free(&M);

    ilu_t *h = (ilu_t *)malloc(sizeof(ilu_t));
    split_lu(&F, &h->L, &h->U);
    csr_free(&F);
    return h;
}

EXPORT void orc_ilu_sizes(void *hp, int *nnzL, int *nnzU)
{
    ilu_t *h = (ilu_t *)hp;
    *nnzL = h->L.Ap[h->L.nrows];
    *nnzU = h->U.Ap[h->U.nrows];
}

EXPORT void orc_ilu_get(void *hp, int *Lp, int *Lj, double *Lx, int *Up, int *Uj, double *Ux)
{
    ilu_t *h = (ilu_t *)hp;
    int n = h->L.nrows;
    memcpy(Lp, h->L.Ap, sizeof(int) * (size_t)(n + 1));
    memcpy(Up, h->U.Ap, sizeof(int) * (size_t)(n + 1));
    memcpy(Lj, h->L.Aj, sizeof(int) * (size_t)h->L.Ap[n]);
    memcpy(Lx, h->L.Ax, sizeof(double) * (size_t)h->L.Ap[n]);
    memcpy(Uj, h->U.Aj, sizeof(int) * (size_t)h->U.Ap[n]);
    memcpy(Ux, h->U.Ax, sizeof(double) * (size_t)h->U.Ap[n]);
}

EXPORT void orc_ilu_free(void *hp)
{
    ilu_t *h = (ilu_t *)hp;
    csr_free(&h->L);
    csr_free(&h->U);
    free(h);
}

/* ------------------------------------------------------------------------ */
/* Krylov drivers                                                           */
/* ------------------------------------------------------------------------ */

enum { SOLVER_GMRES = 0, SOLVER_LGMRES = 1, SOLVER_RGMRES = 2, SOLVER_BICGSTAB = 4, SOLVER_CG = 7 }; /* type-defs.h:157-178 */

typedef struct {
    const csr_t *A;
    const csr_t *L, *U; /* NULL => PC_NON (pc.cxx:67-70) */
    double *cache;
    red_t red;
    double *trace;
    int cap, len;
} ctx_t;

static void trace_push(ctx_t *c, double v)
{
    if (c->trace && c->len < c->cap) c->trace[c->len] = v;
    c->len++;
}

static double tdot(ctx_t *c, const double *x, const double *y)
{
    double v = dot_red(&c->red, x, y, c->A->nrows);
    trace_push(c, v);
    return v;
}

static double tnorm(ctx_t *c, const double *x)
{
    double v = sqrt(dot_red(&c->red, x, x, c->A->nrows));
    trace_push(c, v);
    return v;
}

static void pc_apply(ctx_t *c, double *x, const double *rhs)
{
    int n = c->A->nrows;
    if (!c->L) {
        memcpy(x, rhs, sizeof(double) * (size_t)n);
        return;
    }
    tri_lower(c->L, c->cache, rhs);
    tri_upper(c->U, x, c->cache);
}

/* solver-bicgstab.cxx:10-175 */
static int bicgstab(ctx_t *c, double *x, const double *b, double tol_rel, double tol_abs,
                    double tol_rb, int maxit, double *res_out)
{
    const csr_t *A = c->A;
    int n = A->nrows, it;
    if (maxit <= 0) maxit = DEF_MAXIT;
    if (tol_abs < 0) tol_abs = DEF_TOL;
    if (tol_rel < 0) tol_rel = DEF_TOL;
    size_t bytes = sizeof(double) * (size_t)n;
    double *r = malloc(bytes), *rh = malloc(bytes), *p = malloc(bytes), *ph = malloc(bytes);
    double *s = malloc(bytes), *sh = malloc(bytes), *t = malloc(bytes), *v = malloc(bytes);
    double rho0 = 0, rho1 = 0, alpha = 0, beta = 0, omega = 0, res, tol, err_rel;

    mv_amxpbyz(-1, A, x, 1, b, r);
    for (int i = 0; i < n; i++) {
        rh[i] = r[i];
        sh[i] = ph[i] = 0.;
    }
    double bnorm = tnorm(c, b);
    tol_rb *= bnorm;
    res = err_rel = tnorm(c, r);
    if (res <= tol_abs) {
        it = 0;
        goto done;
    }
    tol = res * tol_rel;
    if (tol < tol_abs) tol = tol_abs;
    if (tol < tol_rb) tol = tol_rb;

    for (it = 0; it < maxit; it++) {
        rho1 = tdot(c, r, rh);
        if (rho1 == 0) break;
        if (it == 0) {
            for (int i = 0; i < n; i++) p[i] = r[i];
        } else {
            beta = (rho1 * alpha) / (rho0 * omega);
            for (int i = 0; i < n; i++) p[i] = r[i] + beta * (p[i] - omega * v[i]);
        }
        rho0 = rho1;
        pc_apply(c, ph, p);
        mv_amxpbyz(1, A, ph, 0, p, v);
        alpha = rho1 / tdot(c, rh, v);
        for (int i = 0; i < n; i++) s[i] = r[i] - alpha * v[i];
        if (tnorm(c, s) <= BREAKDOWN) {
            (void)tnorm(c, s); /* the reference prints it (solver-bicgstab.cxx:118) */
            for (int i = 0; i < n; i++) x[i] = x[i] + alpha * ph[i];
            mv_amxpbyz(-1, A, x, 1, b, r);
            res = tnorm(c, r);
            break;
        }
        pc_apply(c, sh, s);
        mv_amxpbyz(1, A, sh, 0, p, t);
        omega = tdot(c, t, s) / tdot(c, t, t);
        for (int i = 0; i < n; i++) {
            x[i] = x[i] + alpha * ph[i] + omega * sh[i];
            r[i] = s[i] - omega * t[i];
        }
        res = tnorm(c, r);
        if (res <= tol) break;
    }
    if (it < maxit) it += 1;
done:
    *res_out = res;
    free(r); free(rh); free(p); free(ph); free(s); free(sh); free(t); free(v);
    return it;
}

/* solver-cg.cxx:8-136 */
static int cg(ctx_t *c, double *x, const double *b, double tol_rel, double tol_abs,
              double tol_rb, int maxit, double *res_out)
{
    const csr_t *A = c->A;
    int n = A->nrows, it;
    if (maxit <= 0) maxit = DEF_MAXIT;
    if (tol_abs < 0) tol_abs = DEF_TOL;
    if (tol_rel < 0) tol_rel = DEF_TOL;
    size_t bytes = sizeof(double) * (size_t)n;
    double *z = malloc(bytes), *r = malloc(bytes), *p = malloc(bytes), *q = malloc(bytes);
    double rho0 = 0, rho1, beta, res, tol;

    double bnorm = tnorm(c, b);
    tol_rb *= bnorm;
    mv_amxpbyz(-1, A, x, 1, b, r);
    res = tnorm(c, r);
    if (res <= tol_abs) {
        it = 0;
        goto done;
    }
    tol = tol_rel * res;
    if (tol < tol_abs) tol = tol_abs;
    if (tol < tol_rb) tol = tol_rb;
    for (int i = 0; i < n; i++) z[i] = 0;
    for (it = 0; it < maxit; it++) {
        pc_apply(c, z, r);
        rho1 = tdot(c, z, r);
        if (it == 0) {
            for (int i = 0; i < n; i++) p[i] = z[i];
        } else {
            beta = rho1 / rho0;
            for (int i = 0; i < n; i++) p[i] = z[i] + beta * p[i];
        }
        mv_mxy(A, p, q);
        double alpha = tdot(c, q, p);
        alpha = rho1 / alpha;
        rho0 = rho1;
        for (int i = 0; i < n; i++) {
            x[i] = x[i] + alpha * p[i];
            r[i] = r[i] - alpha * q[i];
        }
        res = tnorm(c, r);
        if (res <= tol) break;
    }
    if (it < maxit) it += 1;
done:
    *res_out = res;
    free(z); free(r); free(p); free(q);
    return it;
}

/* solver-gmres.cxx:12-255: left-preconditioned GMRES(m), MGS Arnoldi,
 * Givens rotations on the host, true residual at every restart. */
static int gmres(ctx_t *c, double *x, const double *b, double tol_rel, double tol_abs,
                 double tol_rb, int maxit, int m, double *res_out)
{
    const csr_t *A = c->A;
    int n = A->nrows, inner = 0;
    if (m < 0) m = DEF_RESTART;
    if (maxit <= 0) maxit = DEF_MAXIT;
    if (tol_abs < 0) tol_abs = DEF_TOL;
    if (tol_rel < 0) tol_rel = DEF_TOL;
    if (tol_rb < 0) tol_rb = DEF_TOL;
    size_t bytes = sizeof(double) * (size_t)n;
    double *wj = malloc(bytes), *rg = malloc(bytes);
    double **v = malloc(sizeof(double *) * (size_t)m);
    for (int i = 0; i < m; i++) v[i] = malloc(bytes);
    double *gg = malloc(sizeof(double) * (size_t)(m + 1)), *ym = malloc(sizeof(double) * (size_t)m);
    double *H = malloc(sizeof(double) * (size_t)(m + 1) * (size_t)m);
    double *cs = malloc(sizeof(double) * (size_t)m), *sn = malloc(sizeof(double) * (size_t)m);
#define HG(r, col) H[(size_t)(r) * (size_t)m + (size_t)(col)]
    double tol = 0, err_rel = 0, beta, rtol, gstol = 0.;

    double bnorm = tnorm(c, b);
    tol_rb *= bnorm;
    mv_amxpbyz(-1, A, x, 1, b, rg);
    beta = tnorm(c, rg);
    if (beta <= tol_abs) goto done;
    err_rel = beta;
    tol = tol_rel * err_rel;
    if (tol < tol_abs) tol = tol_abs;
    if (tol < tol_rb) tol = tol_rb;
    rtol = tol / beta;

    while (inner < maxit) {
        int i, kk;
        double gs_norm = 0.;
        pc_apply(c, v[0], rg);
        beta = tnorm(c, v[0]);
        gg[0] = beta;
        for (kk = 1; kk <= m; kk++) gg[kk] = 0;
        if (inner == 0) gstol = rtol * beta * 0.5;
        for (size_t q = 0; q < (size_t)(m + 1) * (size_t)m; q++) H[q] = 0;
        for (int q = 0; q < n; q++) v[0][q] /= beta;

        for (i = 0; i < m; i++) {
            double h;
            inner++;
            mv_mxy(A, v[i], rg);
            pc_apply(c, wj, rg);
            for (int j = 0; j <= i; j++) {
                h = tdot(c, wj, v[j]);
                for (int q = 0; q < n; q++) wj[q] = wj[q] * 1 + v[j][q] * (-h); /* vector.cxx:98-107 */
                HG(j, i) = h;
            }
            h = tnorm(c, wj);
            HG(i + 1, i) = h;
            if (fabs(h) <= BREAKDOWN) {
                i--;
                break;
            } else if (i + 1 < m) {
                double a = 1 / h;
                for (int q = 0; q < n; q++) v[i + 1][q] = wj[q] * a; /* vector.cxx:86-95 */
            }
            for (int j = 0; j < i; j++) {
                double h1 = cs[j] * HG(j, i) + sn[j] * HG(j + 1, i);
                double h2 = -sn[j] * HG(j, i) + cs[j] * HG(j + 1, i);
                HG(j, i) = h1;
                HG(j + 1, i) = h2;
            }
            double gma = sqrt(HG(i, i) * HG(i, i) + HG(i + 1, i) * HG(i + 1, i));
            if (fabs(gma) == 0.) gma = 1e-20;
            cs[i] = HG(i, i) / gma;
            sn[i] = HG(i + 1, i) / gma;
            gg[i + 1] = -sn[i] * gg[i];
            gg[i] = cs[i] * gg[i];
            HG(i, i) = cs[i] * HG(i, i) + sn[i] * HG(i + 1, i);
            gs_norm = fabs(gg[i + 1]);
            if (gs_norm <= gstol) break;
        }
        /* i == m after a full cycle; otherwise the last processed column */
        kk = (i == m) ? m : i + 1;
        for (i = kk - 1; i >= 0; i--) {
            ym[i] = gg[i] / HG(i, i);
            for (int j = 0; j < i; j++) gg[j] = gg[j] - ym[i] * HG(j, i);
        }
        for (int q = 0; q < n; q++) {
            double acc = 0;
            for (i = 0; i < kk; i++) acc += v[i][q] * ym[i];
            x[q] += acc;
        }
        mv_amxpbyz(-1, A, x, 1, b, rg);
        beta = tnorm(c, rg);
        if (beta <= tol) break;
        gstol = rtol * gs_norm / (beta / err_rel) * 0.5;
    }
#undef HG
done:
    *res_out = beta;
    free(wj); free(rg);
    for (int i = 0; i < m; i++) free(v[i]);
    free(v); free(gg); free(ym); free(H); free(cs); free(sn);
    return inner;
}

/* solver-gmres.cxx:257-479: right-preconditioned GMRES(m).  The residual it
 * reports is the Givens estimate |g_{i+1}|; b - A x is formed only to restart. */
static int gmres_r(ctx_t *c, double *x, const double *b, double tol_rel, double tol_abs,
                   double tol_rb, int maxit, int m, double *res_out)
{
    const csr_t *A = c->A;
    int n = A->nrows, inner = 0;
    if (m < 0) m = DEF_RESTART;
    if (maxit <= 0) maxit = DEF_MAXIT;
    if (tol_abs < 0) tol_abs = DEF_TOL;
    if (tol_rel < 0) tol_rel = DEF_TOL;
    if (tol_rb < 0) tol_rb = DEF_TOL;
    size_t bytes = sizeof(double) * (size_t)n;
    double *wj = malloc(bytes), *rg = malloc(bytes);
    double **v = malloc(sizeof(double *) * (size_t)m);
    for (int i = 0; i < m; i++) v[i] = malloc(bytes);
    double *gg = malloc(sizeof(double) * (size_t)(m + 1)), *ym = malloc(sizeof(double) * (size_t)m);
    double *H = malloc(sizeof(double) * (size_t)(m + 1) * (size_t)m);
    double *cs = malloc(sizeof(double) * (size_t)m), *sn = malloc(sizeof(double) * (size_t)m);
#define HG(r, col) H[(size_t)(r) * (size_t)m + (size_t)(col)]
    double tol = 0, err_rel = 0, beta;

    double bnorm = tnorm(c, b);
    tol_rb *= bnorm;
    mv_amxpbyz(-1, A, x, 1, b, rg);
    beta = tnorm(c, rg);
    if (beta <= tol_abs) goto done;
    err_rel = beta;
    tol = tol_rel * err_rel;
    if (tol < tol_abs) tol = tol_abs;
    if (tol < tol_rb) tol = tol_rb;

    while (inner < maxit) {
        int i, kk;
        for (kk = 1; kk <= m; kk++) gg[kk] = 0;
        for (size_t q = 0; q < (size_t)(m + 1) * (size_t)m; q++) H[q] = 0;
        gg[0] = beta = tnorm(c, rg);
        {
            double a = 1 / beta;
            for (int q = 0; q < n; q++) v[0][q] = rg[q] * a; /* vector.cxx:86-95 */
        }
        for (i = 0; i < m && inner < maxit; i++) {
            double h;
            inner++;
            pc_apply(c, rg, v[i]);
            mv_mxy(A, rg, wj);
            for (int j = 0; j <= i; j++) {
                h = tdot(c, wj, v[j]);
                for (int q = 0; q < n; q++) wj[q] = wj[q] * 1 + v[j][q] * (-h);
                HG(j, i) = h;
            }
            h = tnorm(c, wj);
            HG(i + 1, i) = h;
            if (fabs(h) <= BREAKDOWN) {
                i--;
                break;
            } else if (i + 1 < m) {
                double a = 1 / h;
                for (int q = 0; q < n; q++) v[i + 1][q] = wj[q] * a;
            }
            for (int j = 0; j < i; j++) {
                double h1 = cs[j] * HG(j, i) + sn[j] * HG(j + 1, i);
                double h2 = -sn[j] * HG(j, i) + cs[j] * HG(j + 1, i);
                HG(j, i) = h1;
                HG(j + 1, i) = h2;
            }
            double gma = sqrt(HG(i, i) * HG(i, i) + HG(i + 1, i) * HG(i + 1, i));
            if (fabs(gma) == 0.) gma = 1e-20;
            cs[i] = HG(i, i) / gma;
            sn[i] = HG(i + 1, i) / gma;
            gg[i + 1] = -sn[i] * gg[i];
            gg[i] = cs[i] * gg[i];
            HG(i, i) = cs[i] * HG(i, i) + sn[i] * HG(i + 1, i);
            beta = fabs(gg[i + 1]);
            if (beta <= tol) break; /* goto solve: i not advanced */
        }
        kk = (i == m) ? m : i + 1;
        for (i = kk - 1; i >= 0; i--) {
            ym[i] = gg[i] / HG(i, i);
            for (int j = 0; j < i; j++) gg[j] = gg[j] - ym[i] * HG(j, i);
        }
        if (kk > 0) {
            for (int q = 0; q < n; q++) rg[q] = v[kk - 1][q] * ym[kk - 1];
            for (i = kk - 2; i >= 0; i--)
                for (int q = 0; q < n; q++) rg[q] = rg[q] * 1 + v[i][q] * ym[i];
            pc_apply(c, wj, rg);
            for (int q = 0; q < n; q++) x[q] = x[q] * 1 + wj[q] * 1;
        }
        if (beta <= tol) break;
        mv_amxpbyz(-1, A, x, 1, b, rg);
    }
#undef HG
done:
    *res_out = beta;
    free(wj); free(rg);
    for (int i = 0; i < m; i++) free(v[i]);
    free(v); free(gg); free(ym); free(H); free(cs); free(sn);
    return inner;
}

/* solver-lgmres.cxx:12-312: LGMRES(m, k), left preconditioned, augmented with
 * the last k corrections (k = LSSP_AUG_K = 3, lssp.cxx:6).  Quirks kept: true
 * divisions for v_0 and v_{i+1}; the solve uses kk = i columns; the x update
 * reads y[m + i] for the first min(cycle, k) z vectors whenever kk > m (y
 * persists across cycles; the reference mallocs it uninitialised, zero here). */
static int lgmres(ctx_t *c, double *x, const double *b, double tol_rel, double tol_abs,
                  double tol_rb, int maxit, int mk, double *res_out)
{
    const csr_t *A = c->A;
    int n = A->nrows, inner = 0, outer = 0, auk = 3;
    if (mk < 0) mk = DEF_RESTART;
    if (maxit <= 0) maxit = DEF_MAXIT;
    if (tol_abs < 0) tol_abs = DEF_TOL;
    if (tol_rel < 0) tol_rel = DEF_TOL;
    if (tol_rb < 0) tol_rb = DEF_TOL;
    int mmax = mk + auk;
    size_t bytes = sizeof(double) * (size_t)n;
    double *wj = malloc(bytes), *rg = malloc(bytes);
    double **v = malloc(sizeof(double *) * (size_t)mmax);
    for (int i = 0; i < mmax; i++) v[i] = malloc(bytes);
    double **z = malloc(sizeof(double *) * (size_t)auk);
    for (int i = 0; i < auk; i++) z[i] = malloc(bytes);
    double *gg = malloc(sizeof(double) * (size_t)(mmax + 1)), *ym = calloc((size_t)mmax, sizeof(double));
    double *H = malloc(sizeof(double) * (size_t)(mmax + 1) * (size_t)mmax);
    double *cs = malloc(sizeof(double) * (size_t)mmax), *sn = malloc(sizeof(double) * (size_t)mmax);
#define HG(r, col) H[(size_t)(r) * (size_t)mmax + (size_t)(col)]
    double tol = 0, err_rel = 0, beta, rtol, gstol = 0.;

    double bnorm = tnorm(c, b);
    tol_rb *= bnorm;
    mv_amxpbyz(-1, A, x, 1, b, rg);
    beta = tnorm(c, rg);
    if (beta <= tol_abs) goto done;
    err_rel = beta;
    tol = tol_rel * err_rel;
    if (tol < tol_abs) tol = tol_abs;
    if (tol < tol_rb) tol = tol_rb;
    rtol = tol / beta;

    while (inner < maxit) {
        int i, kk, m;
        double gs_norm = 0.;
        pc_apply(c, v[0], rg);
        beta = tnorm(c, v[0]);
        m = outer < auk ? mk + outer : mk + auk;
        gg[0] = beta;
        for (kk = 1; kk <= m; kk++) gg[kk] = 0;
        if (outer == 0) gstol = rtol * beta * 0.5;
        for (size_t q = 0; q < (size_t)(mmax + 1) * (size_t)mmax; q++) H[q] = 0;
        for (int q = 0; q < n; q++) v[0][q] /= beta;
        for (i = 0; i < m; i++) {
            double h;
            inner++;
            mv_mxy(A, i < mk ? v[i] : z[i - mk], rg);
            pc_apply(c, wj, rg);
            for (int j = 0; j <= i; j++) {
                h = tdot(c, wj, v[j]);
                for (int q = 0; q < n; q++) wj[q] = wj[q] * 1 + v[j][q] * (-h);
                HG(j, i) = h;
            }
            h = tnorm(c, wj);
            HG(i + 1, i) = h;
            if (fabs(h) <= BREAKDOWN) {
                i--;
                break;
            } else if (i + 1 < m) {
                for (int q = 0; q < n; q++) v[i + 1][q] = wj[q] / h;
            }
            for (int j = 0; j < i; j++) {
                double h1 = cs[j] * HG(j, i) + sn[j] * HG(j + 1, i);
                double h2 = -sn[j] * HG(j, i) + cs[j] * HG(j + 1, i);
                HG(j, i) = h1;
                HG(j + 1, i) = h2;
            }
            double gma = sqrt(HG(i, i) * HG(i, i) + HG(i + 1, i) * HG(i + 1, i));
            if (fabs(gma) == 0.) gma = 1e-20;
            cs[i] = HG(i, i) / gma;
            sn[i] = HG(i + 1, i) / gma;
            gg[i + 1] = -sn[i] * gg[i];
            gg[i] = cs[i] * gg[i];
            HG(i, i) = cs[i] * HG(i, i) + sn[i] * HG(i + 1, i);
            gs_norm = fabs(gg[i + 1]);
            if (gs_norm <= gstol) break;
        }
        kk = i;
        for (i = kk - 1; i >= 0; i--) {
            ym[i] = gg[i] / HG(i, i);
            for (int j = 0; j < i; j++) gg[j] = gg[j] - ym[i] * HG(j, i);
        }
        {
            int zn = outer % auk, nz = outer <= auk ? outer : auk;
            for (int q = 0; q < n; q++) {
                double t = 0;
                if (kk <= mk) {
                    for (i = 0; i < kk; i++) t += v[i][q] * ym[i];
                } else {
                    for (i = 0; i < mk; i++) t += v[i][q] * ym[i];
                    for (i = 0; i < nz; i++) t += z[i][q] * ym[i + mk];
                }
                x[q] += t;
                z[zn][q] = t;
            }
        }
        mv_amxpbyz(-1, A, x, 1, b, rg);
        beta = tnorm(c, rg);
        if (beta <= tol) break;
        gstol = rtol * gs_norm / (beta / err_rel) * 0.5;
        outer++;
    }
#undef HG
done:
    *res_out = beta;
    free(wj); free(rg);
    for (int i = 0; i < mmax; i++) free(v[i]);
    for (int i = 0; i < auk; i++) free(z[i]);
    free(v); free(z); free(gg); free(ym); free(H); free(cs); free(sn);
    return inner;
}

/* ------------------------------------------------------------------------ */
/* The L1-composed drivers: the reference writes these purely as calls of     */
/* its vector API, restated here call for call.  Work vectors are calloc'ed:  */
/* BiCGSafe/BiCRSafe/GPBiCG/GPBiCR read some before writing them (the golden  */
/* runs use zero-initialising malloc, oracle/ref_shim.cxx).                   */
/* ------------------------------------------------------------------------ */

enum { SOLVER_BICGSAFE = 6, SOLVER_CGS = 8, SOLVER_GPBICG = 9, SOLVER_CR = 10, SOLVER_CRS = 11,
       SOLVER_BICRSTAB = 12, SOLVER_BICRSAFE = 13, SOLVER_GPBICR = 14, SOLVER_QMRCGSTAB = 15,
       SOLVER_TFQMR = 16, SOLVER_ORTHOMIN = 17, SOLVER_BICGSTABL = 5, SOLVER_IDRS = 18 };

typedef struct {
    ctx_t *c;
    int n;
    double tol_rel, tol_abs, tol_rb;
    int maxit;
} l1_t;

static void v_axpby(int n, double a, const double *x, double b, double *y) /* vector.cxx:98-107 */
{
    for (int i = 0; i < n; i++) y[i] = y[i] * b + x[i] * a;
}
static void v_axpbyz(int n, double a, const double *x, double b, const double *y, double *z) /* :110-120 */
{
    for (int i = 0; i < n; i++) z[i] = y[i] * b + x[i] * a;
}
static void v_copy(int n, double *d, const double *s) { memcpy(d, s, sizeof(double) * (size_t)n); }
static void v_set(int n, double *x, double v) { for (int i = 0; i < n; i++) x[i] = v; }
static void v_scale(int n, double *x, double a) { for (int i = 0; i < n; i++) x[i] = x[i] * a; } /* :141-146 */
static double *v_new(int n) { return (double *)calloc((size_t)(n > 0 ? n : 1), sizeof(double)); }

#define NV(k) double *k = v_new(n)
#define AXPBY(a, x, b, y) v_axpby(n, a, x, b, y)
#define AXPBYZ(a, x, b, y, z) v_axpbyz(n, a, x, b, y, z)
#define MXY(x, y) mv_mxy(S->c->A, x, y)
#define RESID(x, b, r) mv_amxpbyz(-1, S->c->A, x, 1, b, r)
#define PC(x, r) pc_apply(S->c, x, r)
#define DOT(x, y) tdot(S->c, x, y)
#define NORM(x) tnorm(S->c, x)

static void l1_tol(const l1_t *S, double nrm2, double bnrb, double *tol)
{
    *tol = nrm2 * S->tol_rel;
    if (*tol < S->tol_abs) *tol = S->tol_abs;
    if (*tol < bnrb) *tol = bnrb;
}

/* solver-cgs.cxx:4-133 (vhat aliases uhat, :25) */
static int l1_cgs(l1_t *S, double *x, const double *b, double *res)
{
    int n = S->n, iter;
    NV(r); NV(rtld); NV(p); NV(phat); NV(q); NV(qhat); NV(u); NV(uhat);
    double *vhat = uhat, alpha, beta, rho, rho_old = 1.0, tdot1, nrm2, ires, tol;
    RESID(x, b, r);
    iter = 0;
    nrm2 = ires = NORM(r);
    if (nrm2 <= S->tol_abs) goto end;
    alpha = NORM(b) * S->tol_rb;
    l1_tol(S, nrm2, alpha, &tol);
    v_copy(n, rtld, r);
    v_set(n, q, 0);
    v_set(n, p, 0);
    for (iter = 1; iter <= S->maxit; iter++) {
        rho = DOT(rtld, r);
        if (rho == 0.0) goto end;
        beta = rho / rho_old;
        AXPBYZ(beta, q, 1, r, u);
        AXPBY(1, q, beta, p);
        AXPBY(1, u, beta, p);
        PC(phat, p);
        MXY(phat, vhat);
        tdot1 = DOT(rtld, vhat);
        if (tdot1 == 0.0) goto end;
        alpha = rho / tdot1;
        AXPBYZ(-alpha, vhat, 1, u, q);
        AXPBYZ(1, u, 1, q, phat);
        PC(uhat, phat);
        AXPBY(alpha, uhat, 1, x);
        MXY(uhat, qhat);
        AXPBY(-alpha, qhat, 1, r);
        nrm2 = NORM(r);
        if (tol >= nrm2) goto end;
        rho_old = rho;
    }
end:
    free(r); free(rtld); free(p); free(phat); free(q); free(qhat); free(u); free(uhat);
    *res = nrm2;
    return iter;
}

/* solver-cr.cxx:3-115 */
static int l1_cr(l1_t *S, double *x, const double *b, double *res)
{
    int n = S->n, iter;
    NV(r); NV(z); NV(p); NV(q); NV(qtld); NV(az);
    double alpha, beta, rho, dot_rq, dot_zq, nrm2, ires, tol;
    RESID(x, b, r);
    nrm2 = ires = NORM(r);
    iter = 1;
    if (nrm2 <= S->tol_abs) goto end;
    alpha = NORM(b) * S->tol_rb;
    l1_tol(S, nrm2, alpha, &tol);
    PC(p, r);
    MXY(p, q);
    v_copy(n, z, p);
    for (iter = 1; iter <= S->maxit; iter++) {
        PC(qtld, q);
        rho = DOT(qtld, q);
        if (rho == 0.0) goto end;
        dot_rq = DOT(r, qtld);
        alpha = dot_rq / rho;
        AXPBY(alpha, p, 1, x);
        AXPBY(-alpha, q, 1, r);
        nrm2 = NORM(r);
        if (tol >= nrm2) goto end;
        AXPBY(-alpha, qtld, 1, z);
        MXY(z, az);
        dot_zq = DOT(az, qtld);
        beta = -dot_zq / rho;
        AXPBY(1, z, beta, p);
        AXPBY(1, az, beta, q);
    }
end:
    free(r); free(z); free(p); free(q); free(qtld); free(az);
    *res = nrm2;
    return iter;
}

/* solver-crs.cxx:3-109 (u = uq = z, ap = q, auq = map, :20-25) */
static int l1_crs(l1_t *S, double *x, const double *b, double *res)
{
    int n = S->n, iter;
    NV(r); NV(rtld); NV(p); NV(z); NV(q); NV(map);
    double *u = z, *uq = z, *ap = q, *auq = map;
    double alpha, beta, rho, rho_old, tdot1, nrm2, ires, tol;
    RESID(x, b, r);
    nrm2 = ires = NORM(r);
    iter = 1;
    if (nrm2 <= S->tol_abs) goto end;
    alpha = NORM(b) * S->tol_rb;
    l1_tol(S, nrm2, alpha, &tol);
    v_copy(n, p, r);
    MXY(p, rtld);
    rho_old = 1.0;
    v_set(n, q, 0.);
    v_set(n, p, 0.);
    for (iter = 1; iter <= S->maxit; iter++) {
        PC(z, r);
        rho = DOT(rtld, z);
        if (rho == 0.0) goto end;
        beta = rho / rho_old;
        AXPBYZ(beta, q, 1, z, u);
        AXPBY(1, q, beta, p);
        AXPBY(1, u, beta, p);
        MXY(p, ap);
        PC(map, ap);
        tdot1 = DOT(rtld, map);
        if (tdot1 == 0.0) goto end;
        alpha = rho / tdot1;
        AXPBYZ(-alpha, map, 1, u, q);
        AXPBYZ(1, u, 1, q, uq);
        MXY(uq, auq);
        AXPBY(alpha, uq, 1, x);
        AXPBY(-alpha, auq, 1, r);
        nrm2 = NORM(r);
        if (tol >= nrm2) goto end;
        rho_old = rho;
    }
end:
    free(r); free(rtld); free(p); free(z); free(q); free(map);
    *res = nrm2;
    return iter;
}

/* solver-bicrstab.cxx:3-114 */
static int l1_bicrstab(l1_t *S, double *x, const double *b, double *res)
{
    int n = S->n, iter;
    NV(rtld); NV(r); NV(s); NV(ms); NV(ams); NV(p); NV(ap); NV(map); NV(z);
    double alpha, beta, omega, rho, rho_old, tdot1, tdot2, nrm2, ires, tol;
    RESID(x, b, r);
    nrm2 = ires = NORM(r);
    iter = 1;
    if (nrm2 <= S->tol_abs) goto end;
    alpha = NORM(b) * S->tol_rb;
    l1_tol(S, nrm2, alpha, &tol);
    v_copy(n, p, r);
    MXY(p, rtld);
    PC(z, r);
    v_copy(n, p, z);
    rho_old = DOT(rtld, z);
    for (iter = 1; iter <= S->maxit; iter++) {
        MXY(p, ap);
        PC(map, ap);
        tdot1 = DOT(rtld, map);
        alpha = rho_old / tdot1;
        AXPBYZ(-alpha, ap, 1, r, s);
        nrm2 = NORM(s);
        if (nrm2 <= tol) {
            AXPBY(alpha, p, 1, x);
            goto end;
        }
        AXPBYZ(-alpha, map, 1, z, ms);
        MXY(ms, ams);
        tdot1 = DOT(ams, s);
        tdot2 = DOT(ams, ams);
        omega = tdot1 / tdot2;
        AXPBY(alpha, p, 1, x);
        AXPBY(omega, ms, 1, x);
        AXPBYZ(-omega, ams, 1, s, r);
        nrm2 = NORM(r);
        if (tol >= nrm2) goto end;
        PC(z, r);
        rho = DOT(rtld, z);
        if (rho == 0.0) goto end;
        beta = (rho / rho_old) * (alpha / omega);
        AXPBY(-omega, map, 1, p);
        AXPBY(1, z, beta, p);
        rho_old = rho;
    }
end:
    free(rtld); free(r); free(s); free(ms); free(ams); free(p); free(ap); free(map); free(z);
    *res = nrm2;
    return iter;
}

/* the (qsi, eta) pair, e.g. solver-bicgsafe.cxx:61-75 */
static void l1_safe(l1_t *S, int iter, const double *y, const double *a, const double *r, double *qsi,
                    double *eta)
{
    double td[5], tmp;
    td[0] = DOT(y, y);
    td[1] = DOT(a, r);
    td[2] = DOT(y, r);
    td[3] = DOT(a, y);
    td[4] = DOT(a, a);
    if (iter == 1) {
        *qsi = td[1] / td[4];
        *eta = 0.0;
    } else {
        tmp = td[4] * td[0] - td[3] * td[3];
        *qsi = (td[0] * td[1] - td[2] * td[3]) / tmp;
        *eta = (td[4] * td[2] - td[3] * td[1]) / tmp;
    }
}

/* solver-bicgsafe.cxx:3-155 (cr_ = 0) and solver-bicrsafe.cxx:3-151 (cr_ = 1) */
static int l1_safe_drv(l1_t *S, double *x, const double *b, double *res, int cr_)
{
    int n = S->n, iter;
    NV(rtld); NV(r); NV(mr); NV(amr); NV(p); NV(ap); NV(t); NV(mt); NV(y); NV(u); NV(z); NV(au);
    NV(map); NV(my); NV(artld);
    double alpha, beta, rho, rho_old, qsi, eta, nrm2, ires, tol;
    RESID(x, b, r);
    nrm2 = ires = NORM(r);
    iter = 1;
    if (nrm2 <= S->tol_abs) goto end;
    alpha = NORM(b) * S->tol_rb;
    l1_tol(S, nrm2, alpha, &tol);
    v_copy(n, rtld, r);
    if (cr_) MXY(rtld, artld);
    PC(mr, r);
    MXY(mr, amr);
    rho_old = cr_ ? DOT(rtld, amr) : DOT(rtld, r);
    v_copy(n, ap, amr);
    v_copy(n, p, mr);
    beta = 0.0;
    for (iter = 1; iter <= S->maxit; iter++) {
        if (cr_) {
            PC(map, ap);
            alpha = rho_old / DOT(artld, map);
        } else {
            alpha = rho_old / DOT(rtld, ap);
        }
        l1_safe(S, iter, y, amr, r, &qsi, &eta);
        if (cr_) {
            v_scale(n, u, eta * beta);
            AXPBY(qsi, map, 1, u);
            AXPBY(eta, my, 1, u);
        } else {
            v_copy(n, t, y);
            v_scale(n, t, eta);
            AXPBY(qsi, ap, 1, t);
            PC(mt, t);
            AXPBY(1, mt, eta * beta, u);
        }
        MXY(u, au);
        v_scale(n, z, eta);
        AXPBY(qsi, mr, 1, z);
        AXPBY(-alpha, u, 1, z);
        v_scale(n, y, eta);
        AXPBY(qsi, amr, 1, y);
        AXPBY(-alpha, au, 1, y);
        if (cr_) PC(my, y);
        AXPBY(alpha, p, 1, x);
        AXPBY(1, z, 1, x);
        AXPBY(-alpha, ap, 1, r);
        AXPBY(-1, y, 1.0, r);
        nrm2 = NORM(r);
        if (tol >= nrm2) goto end;
        if (cr_) {
            AXPBY(-alpha, map, 1, mr);
            AXPBY(-1, my, 1, mr);
            MXY(mr, amr);
            rho = DOT(rtld, amr);
            if (rho == 0.0) goto end;
            beta = (rho / rho_old) * (alpha / qsi);
        } else {
            rho = DOT(rtld, r);
            if (rho == 0.0) goto end;
            beta = (rho / rho_old) * (alpha / qsi);
            PC(mr, r);
            MXY(mr, amr);
        }
        AXPBY(-1, u, 1.0, p);
        AXPBY(1, mr, beta, p);
        AXPBY(-1, au, 1.0, ap);
        AXPBY(1, amr, beta, ap);
        rho_old = rho;
    }
end:
    free(rtld); free(r); free(mr); free(amr); free(p); free(ap); free(t); free(mt); free(y); free(u);
    free(z); free(au); free(map); free(my); free(artld);
    *res = nrm2;
    return iter;
}

/* solver-gpbicg.cxx:3-163 (cr_ = 0) and solver-gpbicr.cxx:3-164 (cr_ = 1) */
static int l1_gpbi(l1_t *S, double *x, const double *b, double *res, int cr_)
{
    int n = S->n, iter;
    NV(rtld); NV(r); NV(mr); NV(p); NV(ap); NV(map); NV(t); NV(mt); NV(amt); NV(u); NV(y); NV(w);
    NV(z); NV(mt_old);
    double alpha, beta, rho, rho_old, qsi, eta, tdot0, nrm2, ires, tol;
    RESID(x, b, r);
    nrm2 = ires = NORM(r);
    iter = 1;
    if (nrm2 <= S->tol_abs) {
        iter = 0;
        goto end;
    }
    alpha = NORM(b) * S->tol_rb;
    l1_tol(S, nrm2, alpha, &tol);
    if (cr_) {
        v_copy(n, p, r);
        MXY(p, rtld);
        PC(p, r);
        rho_old = DOT(rtld, p);
    } else {
        v_copy(n, rtld, r);
        PC(p, r);
        rho_old = DOT(rtld, r);
    }
    v_set(n, t, 0.);
    v_set(n, w, 0.);
    beta = 0.0;
    for (iter = 1; iter <= S->maxit; iter++) {
        MXY(p, ap);
        PC(map, ap);
        tdot0 = DOT(rtld, cr_ ? map : ap);
        if (tdot0 == 0.0) goto end;
        alpha = rho_old / tdot0;
        AXPBYZ(-1, w, 1, ap, y);
        AXPBY(1, t, alpha, y);
        AXPBY(-1, r, 1, y);
        AXPBYZ(-alpha, ap, 1, r, t);
        nrm2 = NORM(t);
        if (nrm2 <= tol) {
            AXPBY(alpha, p, 1, x);
            goto end;
        }
        AXPBYZ(-alpha, map, 1, mr, mt);
        MXY(mt, amt);
        l1_safe(S, iter, y, amt, t, &qsi, &eta);
        AXPBY(1., mt_old, beta, u);
        AXPBY(-1, mr, 1, u);
        v_scale(n, u, eta);
        AXPBY(qsi, map, 1, u);
        v_scale(n, z, eta);
        AXPBY(qsi, mr, 1, z);
        AXPBY(-alpha, u, 1, z);
        AXPBY(alpha, p, 1, x);
        AXPBY(1, z, 1., x);
        AXPBYZ(-qsi, amt, 1, t, r);
        AXPBY(-eta, y, 1, r);
        nrm2 = NORM(r);
        if (tol >= nrm2) goto end;
        PC(mr, r);
        rho = DOT(rtld, cr_ ? mr : r);
        if (rho == 0.0) goto end;
        beta = (rho / rho_old) * (alpha / qsi);
        AXPBYZ(beta, ap, 1, amt, w);
        AXPBY(-1, u, 1, p);
        AXPBY(1., mr, beta, p);
        v_copy(n, mt_old, mt);
        rho_old = rho;
    }
end:
    free(rtld); free(r); free(mr); free(p); free(ap); free(map); free(t); free(mt); free(amt); free(u);
    free(y); free(w); free(z); free(mt_old);
    *res = nrm2;
    return iter;
}

/* solver-qmrcgstab.cxx:10-186 */
static int l1_qmrcgstab(l1_t *S, double *xk, const double *bg, double *res)
{
    int n = S->n, itr_out;
    NV(rk); NV(r); NV(br0); NV(pk); NV(vk); NV(sk); NV(dk); NV(tk); NV(bdk); NV(bxk);
    double rho = 1, prho, alpha = 1, beta, omega = 1, theta = 0., btheta, b_eta, eta = 0., tau, btau;
    double residual, c, ires, rerror, tol, tol_rb = S->tol_rb;
    double b_norm = NORM(bg);
    tol_rb *= b_norm;
    RESID(xk, bg, tk);
    residual = NORM(tk);
    if (residual <= S->tol_abs) {
        itr_out = 0;
        goto end;
    }
    tol = residual * S->tol_rel;
    if (tol < S->tol_abs) tol = S->tol_abs;
    if (tol < tol_rb) tol = tol_rb;
    tol = tol / residual;
    PC(rk, tk);
    v_copy(n, br0, rk);
    v_set(n, pk, 0);
    v_set(n, dk, 0);
    v_set(n, vk, 0);
    tau = ires = NORM(rk);
    prho = rho;
    for (itr_out = 0; itr_out < S->maxit; itr_out++) {
        rho = DOT(br0, rk);
        beta = rho * alpha / prho / omega;
        prho = rho;
        AXPBYZ(1, pk, -omega, vk, r);
        AXPBYZ(beta, r, 1, rk, pk);
        MXY(pk, r);
        PC(vk, r);
        alpha = rho / DOT(br0, vk);
        AXPBYZ(-alpha, vk, 1, rk, sk);
        btheta = NORM(sk) / tau;
        c = 1 / sqrt(1. + btheta * btheta);
        btau = tau * btheta * c;
        b_eta = c * c * alpha;
        AXPBYZ(1., pk, theta * theta * eta / alpha, dk, bdk);
        AXPBYZ(1, xk, b_eta, bdk, bxk);
        MXY(sk, r);
        PC(tk, r);
        {
            double num = DOT(sk, tk); /* :146, operands in g++'s evaluation order */
            omega = num / DOT(tk, tk);
        }
        AXPBYZ(1., sk, -omega, tk, rk);
        theta = NORM(rk) / btau;
        c = 1. / sqrt(1. + theta * theta);
        tau = btau * theta * c;
        eta = c * c * omega;
        AXPBYZ(1, sk, btheta * btheta * b_eta / omega, bdk, dk);
        AXPBYZ(1, bxk, eta, dk, xk);
        rerror = NORM(rk) / ires;
        if (rerror <= tol) {
            RESID(xk, bg, tk);
            residual = NORM(tk);
            break;
        }
    }
    if (itr_out < S->maxit) itr_out += 1;
end:
    free(rk); free(r); free(br0); free(pk); free(vk); free(sk); free(dk); free(tk); free(bdk); free(bxk);
    *res = residual;
    return itr_out;
}

/* solver-tfqmr.cxx:3-149 */
static int l1_tfqmr(l1_t *S, double *x, const double *b, double *res)
{
    int n = S->n, iter;
    NV(r); NV(rtld); NV(u); NV(p); NV(d); NV(t); NV(t1); NV(q); NV(v);
    double alpha, beta, rho, rhoold, s, tau, theta, eta, c, w, wold, ww, nrm2, ires, tol;
    RESID(x, b, r);
    nrm2 = ires = NORM(r);
    iter = 1;
    if (nrm2 <= S->tol_abs) {
        iter = 0;
        goto end;
    }
    alpha = NORM(b) * S->tol_rb;
    l1_tol(S, nrm2, alpha, &tol);
    v_copy(n, rtld, r);
    v_copy(n, p, r);
    v_copy(n, u, r);
    v_set(n, d, 0.);
    PC(t, p);
    MXY(t, v);
    rhoold = DOT(r, rtld);
    tau = NORM(r);
    wold = tau;
    theta = 0.0;
    eta = 0.0;
    while (iter <= S->maxit) {
        s = DOT(v, rtld);
        if (fabs(s) == 0.0) goto end;
        alpha = rhoold / s;
        AXPBYZ(-alpha, v, 1, u, q);
        AXPBYZ(1, u, 1., q, t);
        PC(t1, t);
        MXY(t1, v);
        AXPBY(-alpha, v, 1, r);
        w = NORM(r);
        for (int m = 0; m < 2; m++) {
            if (m == 0) {
                ww = sqrt(w * wold);
                AXPBY(1, u, theta * theta * eta / alpha, d);
            } else {
                ww = w;
                AXPBY(1, q, theta * theta * eta / alpha, d);
            }
            theta = ww / tau;
            c = 1.0 / sqrt(1.0 + theta * theta);
            eta = c * c * alpha;
            tau = tau * theta * c;
            PC(t1, d);
            AXPBY(eta, t1, 1, x);
            nrm2 = tau * sqrt(1.0 + m);
            if (tol >= nrm2) goto end;
        }
        rho = DOT(r, rtld);
        if (fabs(rho) == 0.0) goto end;
        beta = rho / rhoold;
        AXPBYZ(beta, q, 1, r, u);
        AXPBY(1, q, beta, p);
        AXPBY(1, u, beta, p);
        PC(t1, p);
        MXY(t1, v);
        rhoold = rho;
        wold = w;
        iter++;
    }
end:
    free(r); free(rtld); free(u); free(p); free(d); free(t); free(t1); free(q); free(v);
    *res = nrm2;
    return iter;
}

/* solver-orthomin.cxx:12-180: ORTHOMIN(k), k = restart */
static int l1_orthomin(l1_t *S, int k, double *x, const double *rhs, double *res)
{
    int n = S->n, itr_out, i, j;
    double tol = -1, err_rel = 0, beta, a_j, tol_rb = S->tol_rb;
    if (k < 0) k = DEF_RESTART;
    NV(z); NV(r); NV(s); NV(sd);
    double *b_j = v_new(k), *c_j = v_new(k), **p = calloc((size_t)k, sizeof(double *));
    double **q = calloc((size_t)k, sizeof(double *));
    for (i = 0; i < k; i++) {
        p[i] = v_new(n);
        q[i] = v_new(n);
    }
    RESID(x, rhs, z);
    v_set(n, r, 0.);
    PC(r, z);
    v_copy(n, p[0], r);
    v_copy(n, sd, r);
    double b_norm = NORM(rhs);
    tol_rb *= b_norm;
    beta = NORM(z);
    if (beta <= S->tol_abs) {
        itr_out = 0;
        goto end;
    }
    err_rel = beta;
    tol = S->tol_rel * err_rel;
    if (tol < S->tol_abs) tol = S->tol_abs;
    if (tol < tol_rb) tol = tol_rb;
    for (itr_out = 0; itr_out < S->maxit; itr_out++) {
        MXY(sd, s);
        j = itr_out % k;
        v_set(n, q[j], 0.);
        PC(q[j], s);
        a_j = DOT(r, q[j]);
        c_j[j] = DOT(q[j], q[j]);
        if (fabs(c_j[j]) <= BREAKDOWN) break;
        a_j = a_j / c_j[j];
        AXPBY(a_j, p[j], 1, x);
        AXPBY(-a_j, q[j], 1, r);
        v_copy(n, sd, r);
        MXY(r, s);
        v_set(n, z, 0.);
        PC(z, s);
        for (i = 0; i < (itr_out >= k - 1 ? k : itr_out + 1); i++) {
            beta = DOT(z, q[i]);
            b_j[i] = -beta / c_j[i];
            AXPBY(b_j[i], p[i], 1, sd);
        }
        j = (itr_out + 1) % k;
        v_copy(n, p[j], sd);
        RESID(x, rhs, z);
        beta = NORM(z);
        if (beta <= tol) break;
    }
    if (itr_out < S->maxit) itr_out += 1;
end:
    for (i = 0; i < k; i++) {
        free(p[i]);
        free(q[i]);
    }
    free(p); free(q); free(b_j); free(c_j); free(z); free(r); free(s); free(sd);
    *res = beta;
    return itr_out;
}

/* solver-bicgstabl.cxx:4-217: BiCGSTAB(l).  x carries the right-preconditioned
 * iterate and is mapped back as x = M^-1 x + x0 on the converged / breakdown
 * exits only (:84-86, :105-107, :131-133, :190-192). */
static void l1_bgsl_back(l1_t *S, double *x, double *t, const double *xp)
{
    int n = S->n;
    PC(t, x);
    v_copy(n, x, t);
    AXPBY(1, xp, 1, x);
}

static int l1_bicgstabl(l1_t *S, int l, double *x, const double *b, double *res)
{
    int n = S->n, iter, i, j, zd = l + 1;
    NV(rtld); NV(xp); NV(bp); NV(t);
    double **r = (double **)malloc(sizeof(double *) * (size_t)zd);
    double **u = (double **)malloc(sizeof(double *) * (size_t)zd);
    for (i = 0; i <= l; i++) { r[i] = v_new(n); u[i] = v_new(n); }
    double *tau = (double *)calloc((size_t)(zd * (4 + zd)), sizeof(double));
    double *gamma = tau + zd * zd, *gamma1 = gamma + zd, *gamma2 = gamma1 + zd, *sigma = gamma2 + zd;
    double alpha, beta, omega, rho0, rho1, nu, nrm2, ires, tol;
    RESID(x, b, r[0]);
    v_copy(n, rtld, r[0]);
    v_copy(n, bp, r[0]);
    v_copy(n, xp, x);
    v_set(n, u[0], 0.);
    iter = 0;
    nrm2 = ires = NORM(r[0]);
    (void)ires;
    if (nrm2 <= S->tol_abs) goto end;
    tol = nrm2 * S->tol_rel;
    alpha = NORM(b) * S->tol_rb;
    if (tol < S->tol_abs) tol = S->tol_abs;
    if (tol < alpha) tol = alpha;
    alpha = 0.0;
    omega = 1.0;
    rho0 = 1.0;
    while (iter <= S->maxit) {
        rho0 = -omega * rho0;
        for (j = 0; j < l; j++) {
            iter++;
            rho1 = DOT(rtld, r[j]);
            if (rho1 == 0.0) { l1_bgsl_back(S, x, t, xp); goto end; }
            beta = alpha * (rho1 / rho0);
            rho0 = rho1;
            for (i = 0; i <= j; i++) AXPBY(1, r[i], -beta, u[i]);
            PC(t, u[j]);
            MXY(t, u[j + 1]);
            nu = DOT(rtld, u[j + 1]);
            if (fabs(nu) == 0.0) { l1_bgsl_back(S, x, t, xp); goto end; }
            alpha = rho1 / nu;
            AXPBY(alpha, u[0], 1, x);
            for (i = 0; i <= j; i++) AXPBY(-alpha, u[i + 1], 1, r[i]);
            nrm2 = NORM(r[0]);
            if (nrm2 <= tol) { l1_bgsl_back(S, x, t, xp); goto end; }
            PC(t, r[j]);
            MXY(t, r[j + 1]);
        }
        for (j = 1; j <= l; j++) { /* MR part :143-154 */
            for (i = 1; i <= j - 1; i++) {
                nu = DOT(r[j], r[i]);
                nu = nu / sigma[i];
                tau[i * zd + j] = nu;
                AXPBY(-nu, r[i], 1, r[j]);
            }
            sigma[j] = DOT(r[j], r[j]);
            nu = DOT(r[0], r[j]);
            gamma1[j] = nu / sigma[j];
        }
        gamma[l] = gamma1[l];
        omega = gamma[l];
        for (j = l - 1; j >= 1; j--) {
            nu = 0.0;
            for (i = j + 1; i <= l; i++) nu += tau[j * zd + i] * gamma[i];
            gamma[j] = gamma1[j] - nu;
        }
        for (j = 1; j <= l - 1; j++) {
            nu = 0.0;
            for (i = j + 1; i <= l - 1; i++) nu += tau[j * zd + i] * gamma[i + 1];
            gamma2[j] = gamma[j + 1] + nu;
        }
        AXPBY(gamma[1], r[0], 1, x); /* UPDATE :174-182 */
        AXPBY(-gamma1[l], r[l], 1, r[0]);
        AXPBY(-gamma[l], u[l], 1, u[0]);
        for (j = 1; j <= l - 1; j++) {
            AXPBY(-gamma[j], u[j], 1, u[0]);
            AXPBY(gamma2[j], r[j], 1, x);
            AXPBY(-gamma1[j], r[j], 1, r[0]);
        }
        nrm2 = NORM(r[0]);
        if (nrm2 < tol) { l1_bgsl_back(S, x, t, xp); goto end; }
    }
end:
    for (i = 0; i <= l; i++) { free(r[i]); free(u[i]); }
    free(r); free(u); free(tau); free(rtld); free(xp); free(bp); free(t);
    *res = nrm2;
    return iter;
}

/* glibc rand() after srand(0) (solver-idrs.cxx:139-144): the additive
 * feedback generator of glibc's default TYPE_3 random(): r[0] = 1 (seed 0 is
 * taken as 1), r[i] = 16807 r[i-1] mod (2^31 - 1) for i < 31, r[i] = r[i-31]
 * for i = 31..33, then r[i] = r[i-31] + r[i-3] (mod 2^32); output k is
 * r[k + 344] >> 1. */
typedef struct { uint32_t r[34]; int k; } glibc_rand_t;

static void glibc_srand0(glibc_rand_t *g)
{
    int64_t w = 1;
    uint32_t seq[344 + 34];
    seq[0] = 1;
    for (int i = 1; i < 31; i++) {
        w = (16807 * w) % 2147483647;
        seq[i] = (uint32_t)w;
    }
    for (int i = 31; i < 34; i++) seq[i] = seq[i - 31];
    for (int i = 34; i < 344; i++) seq[i] = seq[i - 31] + seq[i - 3];
    for (int i = 0; i < 31; i++) g->r[i] = seq[344 - 31 + i]; /* the last 31 values: a ring */
    g->k = 0;
}

static int glibc_rand(glibc_rand_t *g)
{
    /* ring of the last 31 values, oldest at k: new = oldest + (value 3 back) */
    uint32_t v = g->r[g->k] + g->r[(g->k + 28) % 31];
    g->r[g->k] = v;
    g->k = (g->k + 1) % 31;
    return (int)(v >> 1);
}

/* solver-idrs.cxx:23-84 */
static void idrs_array_solve(int n, const double *a, const double *b, double *x, double *w)
{
    int i, j, k;
    double t;
    for (i = 0; i < n * n; i++) w[i] = a[i];
    if (n == 1) {
        x[0] = b[0] / w[0];
    } else if (n == 2) {
        w[0] = 1.0 / w[0];
        w[1] *= w[0];
        w[3] -= w[1] * w[2];
        w[3] = 1.0 / w[3];
        x[0] = b[0];
        x[1] = b[1] - w[1] * x[0];
        x[1] *= w[3];
        x[0] -= w[2] * x[1];
        x[0] *= w[0];
    } else {
        for (k = 0; k < n; k++) {
            w[k + k * n] = 1.0 / w[k + k * n];
            for (i = k + 1; i < n; i++) {
                t = w[i + k * n] * w[k + k * n];
                for (j = k + 1; j < n; j++) w[i + j * n] -= t * w[k + j * n];
                w[i + k * n] = t;
            }
        }
        for (i = 0; i < n; i++) {
            x[i] = b[i];
            for (j = 0; j < i; j++) x[i] -= w[i + j * n] * x[j];
        }
        for (i = n - 1; i >= 0; i--) {
            for (j = i + 1; j < n; j++) x[i] -= w[i + j * n] * x[j];
            x[i] *= w[i + i * n];
        }
    }
}

/* solver-idrs.cxx:86-283: IDR(s) */
static int l1_idrs(l1_t *S, int s, double *x, const double *b, double *res)
{
    int n = S->n, iter, i, j, k, oldest;
    NV(r); NV(t); NV(v); NV(av);
    double **dX = (double **)malloc(sizeof(double *) * (size_t)s);
    double **dR = (double **)malloc(sizeof(double *) * (size_t)s);
    double **P = (double **)malloc(sizeof(double *) * (size_t)s);
    for (i = 0; i < s; i++) { dX[i] = v_new(n); dR[i] = v_new(n); P[i] = v_new(n); }
    double *m = (double *)calloc((size_t)s, sizeof(double)), *cc = (double *)calloc((size_t)s, sizeof(double));
    double *M = (double *)calloc((size_t)(s * s), sizeof(double)), *MM = (double *)calloc((size_t)(s * s), sizeof(double));
    double om = 0, h, nrm2, ires, tol;
    glibc_rand_t g;
    iter = 0;
    RESID(x, b, r);
    nrm2 = ires = NORM(r);
    (void)ires;
    if (nrm2 <= S->tol_abs) goto end;
    tol = nrm2 * S->tol_rel;
    h = NORM(b) * S->tol_rb;
    if (tol < S->tol_abs) tol = S->tol_abs;
    if (tol < h) tol = h;
    glibc_srand0(&g);
    for (k = 0; k < s; k++)
        for (i = 0; i < n; i++) P[k][i] = (glibc_rand(&g) * 1.) / (1. * 2147483647);
    for (j = 0; j < s; j++) { /* idrs_orth :4-21 */
        double rr = NORM(P[j]);
        rr = 1.0 / rr;
        v_scale(n, P[j], rr);
        for (i = j + 1; i < s; i++) {
            double d = DOT(P[j], P[i]);
            AXPBY(-d, P[j], 1, P[i]);
        }
    }
    for (k = 0; k < s; k++) {
        PC(dX[k], r);
        MXY(dX[k], dR[k]);
        h = DOT(dR[k], dR[k]);
        om = DOT(dR[k], r);
        om = om / h;
        v_scale(n, dX[k], om);
        v_scale(n, dR[k], -om);
        AXPBY(1, dX[k], 1, x);
        AXPBY(1, dR[k], 1, r);
        nrm2 = NORM(r);
        if (tol >= nrm2) { iter = k + 1; goto end; }
        for (i = 0; i < s; i++) M[k * s + i] = DOT(P[i], dR[k]);
    }
    iter = s;
    oldest = 0;
    for (i = 0; i < s; i++) m[i] = DOT(P[i], r);
    while (iter <= S->maxit) {
        idrs_array_solve(s, M, m, cc, MM);
        v_copy(n, v, r);
        for (j = 0; j < s; j++) AXPBY(-cc[j], dR[j], 1, v);
        if ((iter % (s + 1)) == s) {
            PC(av, v);
            MXY(av, t);
            h = DOT(t, t);
            om = DOT(t, v);
            om = om / h;
            for (i = 0; i < n; i++) {
                h = om * av[i];
                for (j = 0; j < s; j++) h -= dX[j][i] * cc[j];
                dX[oldest][i] = h;
            }
            for (i = 0; i < n; i++) {
                h = -om * t[i];
                for (j = 0; j < s; j++) h -= dR[j][i] * cc[j];
                dR[oldest][i] = h;
            }
        } else {
            PC(av, v);
            for (i = 0; i < n; i++) {
                h = om * av[i];
                for (j = 0; j < s; j++) h -= dX[j][i] * cc[j];
                dX[oldest][i] = h;
            }
            MXY(dX[oldest], dR[oldest]);
            v_scale(n, dR[oldest], -1.);
        }
        AXPBY(1, dR[oldest], 1, r);
        AXPBY(1, dX[oldest], 1, x);
        iter++;
        nrm2 = NORM(r);
        if (tol >= nrm2) goto end;
        for (i = 0; i < s; i++) {
            h = DOT(P[i], dR[oldest]);
            m[i] += h;
            M[oldest * s + i] = h;
        }
        oldest++;
        if (oldest == s) oldest = 0;
    }
end:
    for (i = 0; i < s; i++) { free(dX[i]); free(dR[i]); free(P[i]); }
    free(dX); free(dR); free(P); free(m); free(cc); free(M); free(MM);
    free(r); free(t); free(v); free(av);
    *res = nrm2;
    return iter;
}

static int l1_solve(ctx_t *c, int solver, double *x, const double *b, double tol_rel, double tol_abs,
                    double tol_rb, int maxit, int restart, double *res)
{
    l1_t S = {c, c->A->nrows, tol_rel < 0 ? DEF_TOL : tol_rel, tol_abs < 0 ? DEF_TOL : tol_abs, tol_rb,
              maxit <= 0 ? DEF_MAXIT : maxit};
    switch (solver) {
    case SOLVER_ORTHOMIN: return restart == 0 ? -1 : l1_orthomin(&S, restart, x, b, res);
    case SOLVER_CGS: return l1_cgs(&S, x, b, res);
    case SOLVER_CR: return l1_cr(&S, x, b, res);
    case SOLVER_CRS: return l1_crs(&S, x, b, res);
    case SOLVER_BICRSTAB: return l1_bicrstab(&S, x, b, res);
    case SOLVER_BICGSAFE: return l1_safe_drv(&S, x, b, res, 0);
    case SOLVER_BICRSAFE: return l1_safe_drv(&S, x, b, res, 1);
    case SOLVER_GPBICG: return l1_gpbi(&S, x, b, res, 0);
    case SOLVER_GPBICR: return l1_gpbi(&S, x, b, res, 1);
    case SOLVER_QMRCGSTAB: return l1_qmrcgstab(&S, x, b, res);
    case SOLVER_TFQMR: return l1_tfqmr(&S, x, b, res);
    /* l of BiCGSTAB(l) / s of IDR(s) ride in `restart` (<= 0: 4, lssp.cxx:7-8) */
    case SOLVER_BICGSTABL: return l1_bicgstabl(&S, restart <= 0 ? 4 : restart, x, b, res);
    case SOLVER_IDRS: return l1_idrs(&S, restart <= 0 ? 4 : restart, x, b, res);
    default: return -1;
    }
}

/* Solve A x = b (x holds x0 on entry).  L/U == NULL => PC_NON.
 * trace receives every dot/norm the driver computes, in call order (the same
 * sequence tests/golden records from the reference). */
EXPORT int orc_solve(int solver, int n, const int *Ap, const int *Aj, const double *Ax,
                     const int *Lp, const int *Lj, const double *Lx,
                     const int *Up, const int *Uj, const double *Ux,
                     double *x, const double *b, double tol_rel, double tol_abs, double tol_rb,
                     int maxit, int restart, int red_mode, int nranks,
                     double *trace, int trace_cap, int *trace_len, double *residual)
{
    csr_t A = csr_copy(n, n, Ap, Aj, Ax);
    sort_columns(&A);
    csr_t L = {n, n, 0, (int *)Lp, (int *)Lj, (double *)Lx};
    csr_t U = {n, n, 0, (int *)Up, (int *)Uj, (double *)Ux};
    ctx_t c;
    memset(&c, 0, sizeof(c));
    c.A = &A;
    c.L = Lp ? &L : NULL;
    c.U = Up ? &U : NULL;
    c.cache = (double *)malloc(sizeof(double) * (size_t)n);
    c.red.mode = red_mode;
    c.red.nranks = nranks;
    c.trace = trace;
    c.cap = trace_cap;
    int it;
    double res = 0;
    switch (solver) {
    case SOLVER_BICGSTAB: it = bicgstab(&c, x, b, tol_rel, tol_abs, tol_rb, maxit, &res); break;
    case SOLVER_CG: it = cg(&c, x, b, tol_rel, tol_abs, tol_rb, maxit, &res); break;
    case SOLVER_GMRES: it = gmres(&c, x, b, tol_rel, tol_abs, tol_rb, maxit, restart, &res); break;
    case SOLVER_RGMRES: it = gmres_r(&c, x, b, tol_rel, tol_abs, tol_rb, maxit, restart, &res); break;
    case SOLVER_LGMRES: it = lgmres(&c, x, b, tol_rel, tol_abs, tol_rb, maxit, restart, &res); break;
    default: it = l1_solve(&c, solver, x, b, tol_rel, tol_abs, tol_rb, maxit, restart, &res);
    }
    if (trace_len) *trace_len = c.len;
    if (residual) *residual = res;
    free(c.cache);
    csr_free(&A);
    return it;
}

/* ------------------------------------------------------------------------ */
/* Synthetic inputs                                                         */
/* ------------------------------------------------------------------------ */

/* example/exam.cxx:4-59 (5-pt, 4/-1) and its 7-pt analogue (6/-1), natural
 * ordering r = (k*N + j)*N + i, columns ascending. */
EXPORT long orc_poisson_nnz(int dim, int N)
{
    long n = N;
    return dim == 2 ? 5 * n * n - 4 * n : 7 * n * n * n - 6 * n * n;
}

EXPORT void orc_poisson(int dim, int N, int *Ap, int *Aj, double *Ax)
{
    long o = 0, r = 0;
    Ap[0] = 0;
    if (dim == 2) {
        for (int i = 0; i < N; i++)
            for (int j = 0; j < N; j++, r++) {
                long idx = (long)N * i + j;
                if (i > 0) { Aj[o] = (int)(idx - N); Ax[o++] = -1; }
                if (j > 0) { Aj[o] = (int)(idx - 1); Ax[o++] = -1; }
                Aj[o] = (int)idx; Ax[o++] = 4;
                if (j < N - 1) { Aj[o] = (int)(idx + 1); Ax[o++] = -1; }
                if (i < N - 1) { Aj[o] = (int)(idx + N); Ax[o++] = -1; }
                Ap[r + 1] = (int)o;
            }
        return;
    }
    long N2 = (long)N * N;
    for (int k = 0; k < N; k++)
        for (int j = 0; j < N; j++)
            for (int i = 0; i < N; i++, r++) {
                if (k > 0) { Aj[o] = (int)(r - N2); Ax[o++] = -1; }
                if (j > 0) { Aj[o] = (int)(r - N); Ax[o++] = -1; }
                if (i > 0) { Aj[o] = (int)(r - 1); Ax[o++] = -1; }
                Aj[o] = (int)r; Ax[o++] = 6;
                if (i < N - 1) { Aj[o] = (int)(r + 1); Ax[o++] = -1; }
                if (j < N - 1) { Aj[o] = (int)(r + N); Ax[o++] = -1; }
                if (k < N - 1) { Aj[o] = (int)(r + N2); Ax[o++] = -1; }
                Ap[r + 1] = (int)o;
            }
}

/* ------------------------------------------------------------------------ */
/* Format conversions (matrix-utils.cxx:62-380, :700-765)                   */
/* ------------------------------------------------------------------------ */

/* matrix-utils.cxx:281-300: the row of every entry; columns / values copied */
EXPORT void orc_csr_to_coo(int nrows, int ncols, const int *Ap, const int *Aj, const double *Ax, int *Ci, int *Cj,
                           double *Cx)
{
    for (int i = 0; i < nrows; i++)
        for (int k = Ap[i]; k < Ap[i + 1]; k++) Ci[k] = i;
    (void)ncols;
    memcpy(Cj, Aj, sizeof(int) * (size_t)Ap[nrows]);
    memcpy(Cx, Ax, sizeof(double) * (size_t)Ap[nrows]);
}

/* matrix-utils.cxx:324-359: counting sort by row; the sequential scatter
 * keeps the input order inside a row */
EXPORT void orc_coo_to_csr(int nrows, int ncols, int nnz, const int *Ci, const int *Cj, const double *Cx, int *Ap,
                           int *Aj, double *Ax)
{
    int *next = (int *)calloc((size_t)nrows + 1, sizeof(int));
    (void)ncols;
    for (int k = 0; k < nnz; k++) next[Ci[k] + 1]++;
    for (int i = 0; i < nrows; i++) next[i + 1] += next[i];
    memcpy(Ap, next, sizeof(int) * ((size_t)nrows + 1));
    for (int k = 0; k < nnz; k++) {
        int d = next[Ci[k]]++;
        Aj[d] = Cj[k];
        Ax[d] = Cx[k];
    }
    free(next);
}

/* matrix-utils.cxx:700-739: counting sort by column, rows visited in order */
EXPORT void orc_transpose(int nrows, int ncols, const int *Ap, const int *Aj, const double *Ax, int *Tp,
                          int *Tj, double *Tx)
{
    int *next = (int *)calloc((size_t)ncols + 1, sizeof(int));
    for (int k = 0; k < Ap[nrows]; k++) next[Aj[k] + 1]++;
    for (int c = 0; c < ncols; c++) next[c + 1] += next[c];
    memcpy(Tp, next, sizeof(int) * ((size_t)ncols + 1));
    for (int i = 0; i < nrows; i++)
        for (int k = Ap[i]; k < Ap[i + 1]; k++) {
            int d = next[Aj[k]]++;
            Tj[d] = i;
            Tx[d] = Ax[k];
        }
    free(next);
}

/* matrix-utils.cxx:62-162: block pattern per block row (distinct block
 * columns, ascending), then the entries written row by row into zeroed
 * column-major bs x bs blocks (a duplicate keeps its last value).  Bj holds
 * up to nnz, Bx up to nnz*bs*bs; returns the number of blocks. */
EXPORT int orc_csr_to_bcsr(int n, int bs, const int *Ap, const int *Aj, const double *Ax, int *Bp, int *Bj,
                           double *Bx)
{
    int nb = n / bs, bs2 = bs * bs;
    int *slot = (int *)malloc(sizeof(int) * (size_t)nb);
    for (int b = 0; b < nb; b++) slot[b] = -1;
    Bp[0] = 0;
    for (int ib = 0; ib < nb; ib++) {
        int m = Bp[ib];
        for (int r = ib * bs; r < (ib + 1) * bs; r++)
            for (int k = Ap[r]; k < Ap[r + 1]; k++) {
                int bc = Aj[k] / bs;
                if (slot[bc] != ib) {
                    slot[bc] = ib;
                    Bj[m++] = bc;
                }
            }
        qsort(Bj + Bp[ib], (size_t)(m - Bp[ib]), sizeof(int), cmp_int);
        Bp[ib + 1] = m;
    }
    memset(Bx, 0, sizeof(double) * (size_t)Bp[nb] * (size_t)bs2);
    for (int b = 0; b < nb; b++) slot[b] = -1;
    for (int ib = 0; ib < nb; ib++) {
        for (int t = Bp[ib]; t < Bp[ib + 1]; t++) slot[Bj[t]] = t;
        for (int r = ib * bs; r < (ib + 1) * bs; r++)
            for (int k = Ap[r]; k < Ap[r + 1]; k++)
                Bx[(size_t)slot[Aj[k] / bs] * bs2 + (size_t)(Aj[k] % bs) * bs + r % bs] = Ax[k];
    }
    free(slot);
    return Bp[nb];
}

/* matrix-utils.cxx:164-215: COO of the entries with fabs(v) > 0 in block
 * order (column-major inside a block), coo_to_csr, then sort_columns
 * (:387-481).  Aj/Ax hold up to bnnz*bs*bs; returns nnz. */
EXPORT int orc_bcsr_to_csr(int nbrows, int nbcols, int bs, const int *Bp, const int *Bj, const double *Bx,
                           int *Ap, int *Aj, double *Ax)
{
    int bs2 = bs * bs;
    size_t cap = (size_t)Bp[nbrows] * (size_t)bs2;
    int *Ci = (int *)malloc(sizeof(int) * (cap ? cap : 1));
    int *Cj = (int *)malloc(sizeof(int) * (cap ? cap : 1));
    double *Cx = (double *)malloc(sizeof(double) * (cap ? cap : 1));
    int m = 0;
    for (int ib = 0; ib < nbrows; ib++)
        for (int t = Bp[ib]; t < Bp[ib + 1]; t++)
            for (int k = 0; k < bs2; k++) {
                double v = Bx[(size_t)t * bs2 + k];
                if (fabs(v) > 0.) {
                    Ci[m] = ib * bs + k % bs;
                    Cj[m] = Bj[t] * bs + k / bs;
                    Cx[m] = v;
                    m++;
                }
            }
    orc_coo_to_csr(nbrows * bs, nbcols * bs, m, Ci, Cj, Cx, Ap, Aj, Ax);
    csr_t A = {nbrows * bs, nbcols * bs, m, Ap, Aj, Ax};
    sort_columns(&A);
    free(Ci);
    free(Cj);
    free(Cx);
    return m;
}
