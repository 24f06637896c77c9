// ref_shim.cxx -- TEST INFRASTRUCTURE ONLY.
//
// A thin extern "C" driver around the UNMODIFIED reference library (compiled
// in place from /root/reference/src by oracle/Makefile into
// oracle/_ref/libref.so).  It only calls the reference's public C++ API, the
// same sequence example/exam.cxx uses (lssp_solver_create -> set_* ->
// lssp_solver_assemble -> lssp_solver_solve), and records every scalar the
// drivers compute through ld --wrap interposition of lssp_vec_dot /
// lssp_vec_norm.  Used to generate tests/golden/ and as the CPU baseline.
#include "lssp.h"

#include <malloc.h>

#include <vector>

static bool g_trace_on = false;
static std::vector<double> g_trace;

extern "C" double __real__Z12lssp_vec_dot9lssp_vec_S_(lssp_vec x, lssp_vec y);
extern "C" double __real__Z13lssp_vec_norm9lssp_vec_(lssp_vec x);

extern "C" double __wrap__Z12lssp_vec_dot9lssp_vec_S_(lssp_vec x, lssp_vec y)
{
    double v = __real__Z12lssp_vec_dot9lssp_vec_S_(x, y);
    if (g_trace_on) g_trace.push_back(v);
    return v;
}

extern "C" double __wrap__Z13lssp_vec_norm9lssp_vec_(lssp_vec x)
{
    double v = __real__Z13lssp_vec_norm9lssp_vec_(x);
    if (g_trace_on) g_trace.push_back(v);
    return v;
}

static lssp_mat_csr view(int n, const int *Ap, const int *Aj, const double *Ax)
{
    lssp_mat_csr A;
    A.num_rows = A.num_cols = n;
    A.num_nnzs = Ap[n];
    A.Ap = const_cast<int *>(Ap);
    A.Aj = const_cast<int *>(Aj);
    A.Ax = const_cast<double *>(Ax);
    return A;
}

static lssp_vec vview(int n, const double *d)
{
    lssp_vec v;
    v.n = n;
    v.d = const_cast<double *>(d);
    return v;
}

extern "C" {

void ref_quiet(void) { lssp_verbosity = 0; }

// op 0: lssp_mv_mxy, 1: lssp_mv_amxy, 2: lssp_mv_amxpby (in place on z),
// 3: lssp_mv_amxpbyz
void ref_spmv(int op, int n, const int *Ap, const int *Aj, const double *Ax, double alpha,
              const double *x, double beta, const double *y, double *z)
{
    lssp_mat_csr A = view(n, Ap, Aj, Ax);
    lssp_vec X = vview(n, x), Y = vview(n, y), Z = vview(n, z);
    switch (op) {
    case 0: lssp_mv_mxy(A, X, Z); break;
    case 1: lssp_mv_amxy(alpha, A, X, Z); break;
    case 2: lssp_mv_amxpby(alpha, A, X, beta, Z); break;
    default: lssp_mv_amxpbyz(alpha, A, X, beta, Y, Z); break;
    }
}

double ref_dot(int n, const double *x, const double *y)
{
    return lssp_vec_dot(vview(n, x), vview(n, y));
}

// BLAS-1: op 0 axpby (y = y*b + x*a), 1 axpbyz (z = y*b + x*a), 2 axy (y = x*a),
// 3 scale (x *= a), 4 norm (returned)
double ref_vec(int op, int n, double a, const double *x, double b, double *y, double *z)
{
    lssp_vec X = vview(n, x), Y = vview(n, y), Z = vview(n, z);
    switch (op) {
    case 0: lssp_vec_axpby(a, X, b, Y); break;
    case 1: lssp_vec_axpbyz(a, X, b, Y, Z); break;
    case 2: lssp_vec_axy(a, X, Y); break;
    case 3: lssp_vec_scale(Y, a); break;
    default: return lssp_vec_norm(X);
    }
    return 0;
}

struct ref_pc {
    LSSP_SOLVER s;
    LSSP_PC pc;
    lssp_mat_csr A;
    std::vector<double> x, b;
};

// Assemble an ILUK (kind 0) or ILUT (kind 1) preconditioner through the
// public API on the n x n matrix (pc-iluk.cxx:566-581, pc-ilut.cxx:429-456).
void *ref_ilu_create(int kind, int n, const int *Ap, const int *Aj, const double *Ax, int level,
                     double tol, int p)
{
    ref_pc *h = new ref_pc();
    h->A = view(n, Ap, Aj, Ax);
    h->x.assign(n, 0.0);
    h->b.assign(n, 1.0);
    lssp_verbosity = 0;
    lssp_solver_create(h->s, LSSP_SOLVER_BICGSTAB, h->pc, kind == 0 ? LSSP_PC_ILUK : LSSP_PC_ILUT);
    if (kind == 0) {
        lssp_pc_iluk_set_level(h->pc, level);
    } else {
        lssp_pc_ilut_set_drop_tol(h->pc, tol);
        lssp_pc_ilut_set_p(h->pc, p);
    }
    lssp_solver_assemble(h->s, h->A, vview(n, h->x.data()), vview(n, h->b.data()), h->pc);
    return h;
}

void ref_ilu_sizes(void *hp, int *nnzL, int *nnzU)
{
    ref_pc *h = (ref_pc *)hp;
    *nnzL = h->pc.L.num_nnzs;
    *nnzU = h->pc.U.num_nnzs;
}

void ref_ilu_get(void *hp, int *Lp, int *Lj, double *Lx, int *Up, int *Uj, double *Ux)
{
    ref_pc *h = (ref_pc *)hp;
    int n = h->pc.L.num_rows;
    memcpy(Lp, h->pc.L.Ap, sizeof(int) * (n + 1));
    memcpy(Lj, h->pc.L.Aj, sizeof(int) * h->pc.L.num_nnzs);
    memcpy(Lx, h->pc.L.Ax, sizeof(double) * h->pc.L.num_nnzs);
    memcpy(Up, h->pc.U.Ap, sizeof(int) * (n + 1));
    memcpy(Uj, h->pc.U.Aj, sizeof(int) * h->pc.U.num_nnzs);
    memcpy(Ux, h->pc.U.Ax, sizeof(double) * h->pc.U.num_nnzs);
}

// pc.solve(&pc, x, rhs): the function pointer the ILU assemble installed
// (lssp_pc_ilu_solve, solver-tri.cxx:57-60)
void ref_ilu_apply(void *hp, double *x, const double *rhs)
{
    ref_pc *h = (ref_pc *)hp;
    int n = h->pc.L.num_rows;
    h->pc.solve(&h->pc, vview(n, x), vview(n, rhs));
}

void ref_ilu_free(void *hp)
{
    ref_pc *h = (ref_pc *)hp;
    lssp_solver_destroy(h->s, h->pc);
    delete h;
}

// Full solve through the API.  solver: LSSP_SOLVER_TYPE (0 GMRES, 4 BICGSTAB,
// 7 CG); pc: 0 none, 1 ILUK, 2 ILUT.  x holds x0 on entry.  Every dot/norm
// the driver evaluates is appended to trace (up to cap), in call order.
int ref_solve(int solver, int pc_type, int level, double ilut_tol, int ilut_p, int n,
              const int *Ap, const int *Aj, const double *Ax, double *x, const double *b,
              double rtol, double atol, double rbtol, int maxit, int restart, double *trace,
              int cap, int *trace_len, double *residual, double *t_setup, double *t_solve)
{
    LSSP_SOLVER s;
    LSSP_PC pc;
    lssp_mat_csr A = view(n, Ap, Aj, Ax);
    lssp_verbosity = 0;
    // BiCGSafe, BiCRSafe, GPBiCG and GPBiCR read work vectors lssp_vec_create
    // left uninitialised (malloc) before writing them; make malloc hand out
    // zeroed bytes (glibc M_PERTURB: allocations filled with ~0xff) so those
    // runs are deterministic -- the device drivers start from zeroed vectors.
    mallopt(M_PERTURB, 0xff);
    lssp_solver_create(s, (LSSP_SOLVER_TYPE)solver, pc, (LSSP_PC_TYPE)pc_type);
    if (pc_type == LSSP_PC_ILUK) lssp_pc_iluk_set_level(pc, level);
    if (pc_type == LSSP_PC_ILUT) {
        lssp_pc_ilut_set_drop_tol(pc, ilut_tol);
        lssp_pc_ilut_set_p(pc, ilut_p);
    }
    lssp_solver_set_rtol(s, rtol);
    lssp_solver_set_atol(s, atol);
    lssp_solver_set_rbtol(s, rbtol);
    lssp_solver_set_maxit(s, maxit);
    if (restart > 0) lssp_solver_set_restart(s, restart);
    // BiCGSTAB(l) / IDR(s): l / s ride in `restart` (lssp_solver_set_bgsl / _idrs, lssp.cxx:495-513)
    if (restart > 0 && solver == LSSP_SOLVER_BICGSTABL) lssp_solver_set_bgsl(s, restart);
    if (restart > 0 && solver == LSSP_SOLVER_IDRS) lssp_solver_set_idrs(s, restart);
    double t0 = lssp_get_time();
    lssp_solver_assemble(s, A, vview(n, x), vview(n, b), pc);
    double t1 = lssp_get_time();
    g_trace.clear();
    g_trace_on = true;
    int it = lssp_solver_solve(s, pc);
    g_trace_on = false;
    double t2 = lssp_get_time();
    if (t_setup) *t_setup = t1 - t0;
    if (t_solve) *t_solve = t2 - t1;
    if (trace_len) *trace_len = (int)g_trace.size();
    for (int i = 0; i < (int)g_trace.size() && i < cap; i++) trace[i] = g_trace[i];
    if (residual) *residual = lssp_solver_get_residual(s);
    lssp_solver_destroy(s, pc);
    return it;
}

double ref_time(void) { return lssp_get_time(); }

} // extern "C"

// ---------------------------------------------------------------------------
// Block-Jacobi ILU(0) composed from the public API: each diagonal block is
// factored by lssp_solver_assemble with ILUK level 0 and the factors are
// stitched with a column shift.  For level 0 this equals the reference's own
// blk_size path (pc-iluk.cxx:411-552 with blk_size < n): adjust_zero_diag
// only inserts in-block diagonals and get_block_diag keeps exactly the block.
// Solves use it through the reference's PC plug-in (LSSP_PC_USER, pc.cxx:219)
// with pc.solve = lssp_pc_ilu_solve.
static lssp_mat_csr g_bjL, g_bjU;

static void bj_assemble(LSSP_PC &pc, LSSP_SOLVER s)
{
    (void)s;
    pc.L = g_bjL;
    pc.U = g_bjU;
    pc.cache = lssp_malloc<double>(pc.L.num_rows);
    pc.solve = lssp_pc_ilu_solve;
    pc.destroy = NULL;
}

static void block_csr(int n, const int *Ap, const int *Aj, const double *Ax, int s, int e,
                      std::vector<int> &bp, std::vector<int> &bj, std::vector<double> &bx)
{
    bp.assign(1, 0);
    bj.clear();
    bx.clear();
    for (int i = s; i < e; i++) {
        for (int k = Ap[i]; k < Ap[i + 1]; k++)
            if (Aj[k] >= s && Aj[k] < e) {
                bj.push_back(Aj[k] - s);
                bx.push_back(Ax[k]);
            }
        bp.push_back((int)bj.size());
    }
    (void)n;
}

extern "C" void *ref_bj_create(int n, const int *Ap, const int *Aj, const double *Ax, int nblk)
{
    int blk = (n + nblk - 1) / nblk;
    std::vector<int> Lp(1, 0), Lj, Up(1, 0), Uj;
    std::vector<double> Lx, Ux;
    for (int s = 0; s < n; s += blk) {
        int e = s + blk < n ? s + blk : n;
        std::vector<int> bp, bj;
        std::vector<double> bx;
        block_csr(n, Ap, Aj, Ax, s, e, bp, bj, bx);
        ref_pc *h = (ref_pc *)ref_ilu_create(0, e - s, bp.data(), bj.data(), bx.data(), 0, 0, 0);
        const lssp_mat_csr &L = h->pc.L, &U = h->pc.U;
        for (int i = 0; i < e - s; i++) {
            for (int k = L.Ap[i]; k < L.Ap[i + 1]; k++) {
                Lj.push_back(L.Aj[k] + s);
                Lx.push_back(L.Ax[k]);
            }
            for (int k = U.Ap[i]; k < U.Ap[i + 1]; k++) {
                Uj.push_back(U.Aj[k] + s);
                Ux.push_back(U.Ax[k]);
            }
            Lp.push_back((int)Lj.size());
            Up.push_back((int)Uj.size());
        }
        ref_ilu_free(h);
    }
    ref_pc *h = new ref_pc();
    h->pc.L.num_rows = h->pc.L.num_cols = n;
    h->pc.U.num_rows = h->pc.U.num_cols = n;
    h->pc.L.num_nnzs = (int)Lj.size();
    h->pc.U.num_nnzs = (int)Uj.size();
    h->pc.L.Ap = lssp_copy_on<int>(Lp.data(), n + 1);
    h->pc.L.Aj = lssp_copy_on<int>(Lj.data(), (int)Lj.size());
    h->pc.L.Ax = lssp_copy_on<double>(Lx.data(), (int)Lx.size());
    h->pc.U.Ap = lssp_copy_on<int>(Up.data(), n + 1);
    h->pc.U.Aj = lssp_copy_on<int>(Uj.data(), (int)Uj.size());
    h->pc.U.Ax = lssp_copy_on<double>(Ux.data(), (int)Ux.size());
    h->pc.cache = lssp_malloc<double>(n);
    h->pc.solve = lssp_pc_ilu_solve;
    return h;
}

extern "C" void ref_bj_free(void *hp)
{
    ref_pc *h = (ref_pc *)hp;
    lssp_mat_destroy(h->pc.L);
    lssp_mat_destroy(h->pc.U);
    lssp_free(h->pc.cache);
    delete h;
}

// Solve with a block-Jacobi handle from ref_bj_create, via LSSP_PC_USER.
extern "C" int ref_solve_bj(void *hp, int solver, int n, const int *Ap, const int *Aj,
                            const double *Ax, double *x, const double *b, double rtol, double atol,
                            double rbtol, int maxit, int restart, double *trace, int cap,
                            int *trace_len, double *residual)
{
    ref_pc *h = (ref_pc *)hp;
    LSSP_SOLVER s;
    LSSP_PC pc;
    lssp_mat_csr A = view(n, Ap, Aj, Ax);
    lssp_verbosity = 0;
    mallopt(M_PERTURB, 0xff);  // as in ref_solve
    lssp_solver_create(s, (LSSP_SOLVER_TYPE)solver, pc, LSSP_PC_USER);
    g_bjL = h->pc.L;
    g_bjU = h->pc.U;
    pc.assemble = bj_assemble;
    lssp_solver_set_rtol(s, rtol);
    lssp_solver_set_atol(s, atol);
    lssp_solver_set_rbtol(s, rbtol);
    lssp_solver_set_maxit(s, maxit);
    if (restart > 0) lssp_solver_set_restart(s, restart);
    // BiCGSTAB(l) / IDR(s): l / s ride in `restart` (lssp_solver_set_bgsl / _idrs, lssp.cxx:495-513)
    if (restart > 0 && solver == LSSP_SOLVER_BICGSTABL) lssp_solver_set_bgsl(s, restart);
    if (restart > 0 && solver == LSSP_SOLVER_IDRS) lssp_solver_set_idrs(s, restart);
    lssp_solver_assemble(s, A, vview(n, x), vview(n, b), pc);
    g_trace.clear();
    g_trace_on = true;
    int it = lssp_solver_solve(s, pc);
    g_trace_on = false;
    if (trace_len) *trace_len = (int)g_trace.size();
    for (int i = 0; i < (int)g_trace.size() && i < cap; i++) trace[i] = g_trace[i];
    if (residual) *residual = lssp_solver_get_residual(s);
    lssp_free(pc.cache);
    lssp_mat_destroy(s.A);
    return it;
}

// ---------------------------------------------------------------------------
// Format conversions through the public API (matrix-utils.h:22-49).  Outputs
// are copied into caller arrays sized as in oracle/lssp_oracle.c's orc_*.
static void put_csr(const lssp_mat_csr &B, int *Ap, int *Aj, double *Ax)
{
    if (B.Ap) memcpy(Ap, B.Ap, sizeof(int) * (B.num_rows + 1));
    else memset(Ap, 0, sizeof(int) * (B.num_rows + 1));
    if (B.num_nnzs > 0) {
        memcpy(Aj, B.Aj, sizeof(int) * B.num_nnzs);
        memcpy(Ax, B.Ax, sizeof(double) * B.num_nnzs);
    }
}

extern "C" void ref_csr_to_coo(int nrows, int ncols, const int *Ap, const int *Aj, const double *Ax, int *Ci,
                               int *Cj, double *Cx)
{
    lssp_mat_csr A = view(nrows, Ap, Aj, Ax);
    A.num_cols = ncols;
    lssp_mat_coo C = lssp_mat_csr_to_coo(A);
    if (C.num_nnzs > 0) {
        memcpy(Ci, C.Ai, sizeof(int) * C.num_nnzs);
        memcpy(Cj, C.Aj, sizeof(int) * C.num_nnzs);
        memcpy(Cx, C.Ax, sizeof(double) * C.num_nnzs);
    }
    lssp_mat_destroy(C);
}

extern "C" void ref_coo_to_csr(int nrows, int ncols, int nnz, const int *Ci, const int *Cj, const double *Cx,
                               int *Ap, int *Aj, double *Ax)
{
    lssp_mat_coo C;
    C.num_rows = nrows;
    C.num_cols = ncols;
    C.num_nnzs = nnz;
    C.Ai = const_cast<int *>(Ci);
    C.Aj = const_cast<int *>(Cj);
    C.Ax = const_cast<double *>(Cx);
    lssp_mat_csr B = lssp_mat_coo_to_csr(C);
    put_csr(B, Ap, Aj, Ax);
    lssp_mat_destroy(B);
}

extern "C" void ref_transpose(int nrows, int ncols, const int *Ap, const int *Aj, const double *Ax, int *Tp,
                              int *Tj, double *Tx)
{
    lssp_mat_csr A = view(nrows, Ap, Aj, Ax);
    A.num_cols = ncols;
    lssp_mat_csr T = lssp_mat_transpose(A);
    put_csr(T, Tp, Tj, Tx);
    lssp_mat_destroy(T);
}

extern "C" int ref_csr_to_bcsr(int n, int bs, const int *Ap, const int *Aj, const double *Ax, int *Bp, int *Bj,
                               double *Bx)
{
    lssp_mat_csr A = view(n, Ap, Aj, Ax);
    lssp_mat_bcsr B = lssp_mat_csr_to_bcsr(A, bs);
    int nb = B.num_rows;
    memcpy(Bp, B.Ap, sizeof(int) * (nb + 1));
    memcpy(Bj, B.Aj, sizeof(int) * B.num_nnzs);
    memcpy(Bx, B.Ax, sizeof(double) * (size_t)B.num_nnzs * bs * bs);
    int m = B.num_nnzs;
    lssp_mat_destroy(B);
    return m;
}

extern "C" int ref_bcsr_to_csr(int nbrows, int nbcols, int bs, const int *Bp, const int *Bj, const double *Bx,
                               int *Ap, int *Aj, double *Ax)
{
    lssp_mat_bcsr B;
    B.num_rows = nbrows;
    B.num_cols = nbcols;
    B.num_nnzs = Bp[nbrows];
    B.blk_size = bs;
    B.Ap = const_cast<int *>(Bp);
    B.Aj = const_cast<int *>(Bj);
    B.Ax = const_cast<double *>(Bx);
    lssp_mat_csr A = lssp_mat_bcsr_to_csr(B);
    put_csr(A, Ap, Aj, Ax);
    int m = A.num_nnzs;
    lssp_mat_destroy(A);
    return m;
}
