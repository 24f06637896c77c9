// solvers.cpp -- BiCGSTAB, GMRES(m) and CG on device-resident vectors.
//
// Each driver replays the reference's scalar recurrences, guards, defaults and
// iteration counting step for step (solver-bicgstab.cxx:10-175,
// solver-gmres.cxx:12-255, solver-cg.cxx:8-136).  The inline host loops of the
// reference become fused elementwise passes (kernels.hip, EwKind); every dot
// or norm becomes a reduction whose finalize program updates the scalar
// recurrence on the device, so an iteration runs without host round trips
// and the host synchronises once per iteration (once per Arnoldi step in
// GMRES) to test convergence, exactly where the reference branches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "internal.h"

namespace lssp_amd {

namespace {

constexpr double BREAKDOWN = 1e-40;  // lssp.cxx:14
constexpr int DEF_MAXIT = 1000;      // lssp.cxx:9
constexpr int DEF_RESTART = 50;      // lssp.cxx:5
constexpr double DEF_TOL = 1e-7;     // lssp.cxx:11-13

enum EwK {  // mirror of kernels.hip EwKind
    K_FILL = 0, K_COPY, K_AXY, K_AXPBY, K_AXPBYZ, K_SCALE, K_DIVS, K_DOT,
    K_BICG_P, K_BICG_S, K_BICG_XR, K_CG_P, K_CG_XR, K_GM_MGS, K_GM_X, K_GMR_Z, K_LGM_X
};

struct Run {
    lssp_amd_ctx *c;
    const lssp_amd_mat *A;
    const lssp_amd_ilu *M;
    long n = 0, nx = 0;
    bool tree = true;
    bool want_trace = false;
    long tcap = 0;
    long tl = 0;  // logical trace length
    std::vector<std::pair<long, double>> patches;
    std::vector<double *> bufs;
    int rank = 0;
    // global preconditioner on P ranks (pc-iluk.cxx:574, blk_size = n): M holds
    // the factors of the WHOLE matrix on every rank; an apply all-gathers the
    // rhs blocks, sweeps the global system and keeps the rank's rows
    bool gpc = false;
    double *g_send = nullptr, *g_rhs = nullptr, *g_x = nullptr;

    ~Run()
    {
        (void)hipStreamSynchronize(c->stream);
        // the gathered-stream cache lives only between a p / s pass and the
        // apply right after it; an error exit between the two must not leave it
        if (M) M->line.lstream_of = nullptr;
        for (double *p : bufs)
            for (auto &w : c->pool)
                if (w.p == p) w.used = false;
    }
    // work vectors come from the context's pool: allocated once, reused by
    // every later solve of the same size
    double *vec(long len = -1)
    {
        const long want = std::max<long>(len < 0 ? nx : len, 1);
        for (auto &w : c->pool)
            if (!w.used && w.n == want) {
                w.used = true;
                bufs.push_back(w.p);
                return w.p;
            }
        double *p = nullptr;
        if (hipMalloc(&p, sizeof(double) * want) != hipSuccess) return nullptr;
        c->pool.push_back({p, want, true});
        bufs.push_back(p);
        return p;
    }
    int T()
    {
        long p = tl++;
        return (want_trace && p < tcap) ? (int)p : -1;
    }
    Fin fin(int op, int nsum, int t0 = -1, int t1 = -1, int dst0 = S_SUM0)
    {
        Fin f;
        f.op = op;
        f.nsum = nsum;
        f.dst[0] = dst0;
        f.tpos[0] = t0;
        f.tpos[1] = t1;
        return f;
    }
    int pc(double *x, const double *rhs)
    {
        if (!M) {
            Ew e;
            e.kind = K_COPY;
            e.n = n;
            e.x = rhs;
            e.out0 = x;
            return launch_ew(c, e);
        }
        if (gpc) return pc_global(x, rhs);
        return launch_ilu_apply(c, M, x, rhs);
    }
    // the rank's rows of U^-1 L^-1 rhs for the global factors: the rows are
    // the canonical blocks of ceil(n/P) (the last one shorter, its send padded),
    // so the gathered blocks are the global rhs in row order
    int pc_global(double *x, const double *rhs)
    {
        const long ng = A->n_global, blk = (ng + c->nranks - 1) / c->nranks;
        if (!g_send) {
            g_send = vec(blk);
            g_rhs = vec(blk * c->nranks);
            g_x = vec(ng);
            if (!g_send || !g_rhs || !g_x) return LSSP_AMD_ENOMEM;
        }
        Ew e;
        e.kind = K_COPY;
        e.x = rhs;
        e.out0 = g_send;
        LSSP_TRY(ew(e));
        LSSP_TRY(comm_allgather(c, g_send, g_rhs, (long)sizeof(double) * blk));
        LSSP_TRY(launch_ilu_apply(c, M, g_x, g_rhs));
        e.x = g_x + A->row0;
        e.out0 = x;
        return ew(e);
    }
    // x = M^-1 rhs, then z = op(A x) (+ fused dots): one rank with a line-swept
    // ILU(0) runs the product in the U sweep's tail, as planes of x become
    // final (launch_line_apply_spmv; bitwise the two steps)
    int pc_spmv(double *x, const double *rhs, int epi, double alpha, double beta, const double *y, double *z,
                int nred = 0, const double *w0 = nullptr, const double *w1 = nullptr)
    {
        if (M && !gpc && M->line.ntiles > 0) {
            const int nr = tree ? nred : 0;
            const int st = launch_line_apply_spmv(c, M->line, x, rhs, A, epi, alpha, beta, y, z, nr, w0, w1);
            if (st == LSSP_AMD_OK && c->nranks > 1)  // the halo round and the chunks that read it
                return spmv_boundary(c, A, epi, alpha, x, beta, y, z, nr, w0, w1);
            if (st != LSSP_AMD_EUNSUPPORTED) return st;
        }
        LSSP_TRY(pc(x, rhs));
        return spmv(epi, alpha, x, beta, y, z, nred, w0, w1);
    }
    int sync(int first, int count)
    {
        LSSP_HIP(hipMemcpyAsync(c->h_scal + first, c->d_scal + first, sizeof(double) * count,
                                hipMemcpyDeviceToHost, c->stream));
        int e = 0;
        LSSP_HIP(hipMemcpyAsync(&e, c->d_err, sizeof(int), hipMemcpyDeviceToHost, c->stream));
        LSSP_HIP(hipStreamSynchronize(c->stream));
        if (e) {
            LSSP_HIP(hipMemset(c->d_err, 0, sizeof(int)));
            // a line sweep that gave up mid-way leaves hand-off entries written
            if (M && M->line.ntiles) LSSP_TRY(line_rearm(c, const_cast<lssp_amd_ilu *>(M)->line));
            LSSP_HIP(hipStreamSynchronize(c->stream));
            return LSSP_AMD_ETIMEOUT;
        }
        return LSSP_AMD_OK;
    }
    // batched iterations, two batches in flight: the stream copies the scalar
    // slots (0 .. S_H + S_HB: the stop flag, the iteration count and the residual
    // history ring) and the error word of the batch just queued into snapshot k
    // and records ev_snap[k]; the host queues the next batch and only then waits
    // for snapshot k, so the GPU runs batch j + 1 while the host reads batch j
    // (the launches past a stop return at once: ctx guard)
    int snap_issue(int k)
    {
        LSSP_HIP(hipMemcpyAsync(c->h_snap + k * (S_H + S_HB), c->d_scal, sizeof(double) * (S_H + S_HB),
                                hipMemcpyDeviceToHost, c->stream));
        LSSP_HIP(hipMemcpyAsync(c->h_snap_err + k, c->d_err, sizeof(int), hipMemcpyDeviceToHost, c->stream));
        LSSP_HIP(hipEventRecord(c->ev_snap[k], c->stream));
        return LSSP_AMD_OK;
    }
    int snap_wait(int k)
    {
        LSSP_HIP(hipEventSynchronize(c->ev_snap[k]));
        memcpy(c->h_scal, c->h_snap + k * (S_H + S_HB), sizeof(double) * (S_H + S_HB));
        if (c->h_snap_err[k]) {
            LSSP_HIP(hipStreamSynchronize(c->stream));  // the batch queued after it runs out first
            LSSP_HIP(hipMemset(c->d_err, 0, sizeof(int)));
            if (M && M->line.ntiles) LSSP_TRY(line_rearm(c, const_cast<lssp_amd_ilu *>(M)->line));
            LSSP_HIP(hipStreamSynchronize(c->stream));
            return LSSP_AMD_ETIMEOUT;
        }
        return LSSP_AMD_OK;
    }
    // start a batched run: stop flag 0, tolerance, iteration count 0
    int batch_begin(double tol)
    {
        c->h_scal[S_DONE] = 0.0;
        c->h_scal[S_TOL] = tol;
        c->h_scal[S_NIT] = 0.0;
        LSSP_HIP(hipMemcpyAsync(c->d_scal + S_DONE, c->h_scal + S_DONE, 3 * sizeof(double), hipMemcpyHostToDevice,
                                c->stream));
        return LSSP_AMD_OK;
    }
    double h(int i) const { return c->h_scal[i]; }
    int spmv(int epi, double alpha, double *x, double beta, const double *y, double *z, int nred = 0,
             const double *w0 = nullptr, const double *w1 = nullptr)
    {
        return spmv_halo(c, A, epi, alpha, x, beta, y, z, tree ? nred : 0, w0, w1);
    }
    int ew(Ew e)
    {
        e.n = n;
        e.scal = c->d_scal;
        if (!tree) e.nred = 0;
        return launch_ew(c, e);
    }
    int fin1(const double *a, const double *b, const Fin &f)
    {
        const double *A_[1] = {a}, *B_[1] = {b};
        return finish_reduce(c, n, 1, A_, B_, f);
    }
    int fin2(const double *a0, const double *b0, const double *a1, const double *b1, const Fin &f)
    {
        const double *A_[2] = {a0, a1}, *B_[2] = {b0, b1};
        return finish_reduce(c, n, 2, A_, B_, f);
    }
    int dot1(const double *a, const double *b, const Fin &f)
    {
        const double *A_[1] = {a}, *B_[1] = {b};
        return reduce_dots(c, n, 1, A_, B_, f);
    }
};

void defaults(const lssp_amd_solve_params &P, double &tol_rel, double &tol_abs, int &maxit)
{
    tol_rel = P.tol_rel < 0 ? DEF_TOL : P.tol_rel;
    tol_abs = P.tol_abs < 0 ? DEF_TOL : P.tol_abs;
    maxit = P.maxit <= 0 ? DEF_MAXIT : P.maxit;
}

// ---------------------------------------------------------------------------
// BiCGSTAB, right preconditioned (solver-bicgstab.cxx:10-175)
// ---------------------------------------------------------------------------
int bicgstab(Run &R, const lssp_amd_solve_params &P, double *x, const double *b, int *nits,
             double *res_out)
{
    const double t_start = wall_time();  // the reference driver's lssp_get_time() ("total time")
    double tol_rel, tol_abs, tol_rb = P.tol_rb, tol;
    int maxit, it;
    defaults(P, tol_rel, tol_abs, maxit);
    if (P.verb >= 2 && R.rank == 0) {
        lprint("bicgstab: maximal iteration: %d\n", maxit);
        lprint("bicgstab: tolerance abs: %g\n", tol_abs);
        lprint("bicgstab: tolerance rel: %g\n", tol_rel);
        lprint("bicgstab: tolerance rbn: %g\n", tol_rb);
    }
    double *r = R.vec(), *rh = R.vec(), *p = R.vec(), *ph = R.vec();
    double *s = R.vec(), *sh = R.vec(), *t = R.vec(), *v = R.vec();
    if (!r || !rh || !p || !ph || !s || !sh || !t || !v) return LSSP_AMD_ENOMEM;

    LSSP_TRY(R.spmv(EPI_AXPBY, -1, x, 1, b, r));  // :67
    {
        Ew e;
        e.kind = K_COPY;
        e.x = r;
        e.out0 = rh;
        LSSP_TRY(R.ew(e));  // :68-71 (the sh/ph zero fill is dead work)
    }
    LSSP_TRY(R.dot1(b, b, R.fin(FIN_NORM, 1, R.T(), -1, S_BNORM)));  // :73
    LSSP_TRY(R.dot1(r, r, R.fin(FIN_NORM, 1, R.T(), -1, S_RES)));    // :76
    LSSP_TRY(R.sync(0, 16));
    const double b_norm = R.h(S_BNORM);
    tol_rb *= b_norm;
    double res = R.h(S_RES);
    const double err_rel = res;
    if (res <= tol_abs) {
        *nits = 0;
        *res_out = res;
        return LSSP_AMD_OK;
    }
    tol = res * tol_rel;
    if (tol < tol_abs) tol = tol_abs;
    if (tol < tol_rb) tol = tol_rb;

    LSSP_TRY(R.dot1(r, rh, R.fin(FIN_BICG_RHO, 1, R.T())));  // :87 (first iteration)
    LSSP_TRY(R.sync(0, 16));
    double rho1 = R.h(S_RHO1);
    bool pending_rho = false;  // a fused next-iteration rho1 sits in the trace

    // tree mode merges ||s||^2 into the omega round (below); SERIAL mode keeps
    // the reference's order of reductions
    const bool merge_s = R.tree;
    // one iteration :94-141 queued on the stream; fin_res: the finalize of its
    // last reduction; *pos_s: the trace position before its ||s|| (:117)
    // line-swept ILU(0): the p and s passes also write the next apply's rhs
    // stream (launch_line_gather_ew), and in tree mode ||s||^2's partials come
    // from the product t = A sh, which reads s anyway (its third fused dot)
    const bool gew = R.M && !R.gpc && line_gather_ew_ok(R.M->line, R.n);
    auto enqueue = [&](int k, int fin_res, long *pos_s) -> int {
        Ew e;
        if (k == 0) {
            e.kind = K_COPY;  // :96
            e.x = r;
            e.out0 = p;
            LSSP_TRY(R.ew(e));
        } else if (gew) {
            LSSP_TRY(launch_line_gather_ew(R.c, R.M->line, GEW_BICG_P, r, v, p, R.c->d_scal));  // :99-102
        } else {
            e.kind = K_BICG_P;  // :99-102
            e.x = r;
            e.y = v;
            e.out0 = p;
            LSSP_TRY(R.ew(e));
        }
        LSSP_TRY(R.pc_spmv(ph, p, EPI_AMX, 1, 0, p, v, 1, rh));  // :107-108, :110
        LSSP_TRY(R.fin1(rh, v, R.fin(FIN_BICG_ALPHA, 1, R.T())));  // :112
        if (gew) {
            LSSP_TRY(launch_line_gather_ew(R.c, R.M->line, GEW_BICG_S, r, v, s, R.c->d_scal));  // :113-115
        } else {
            e = Ew();
            e.kind = K_BICG_S;  // :113-115
            e.x = r;
            e.y = v;
            e.out0 = s;
            e.nred = 1;
            e.r0a = s;
            e.r0b = s;
            // tree mode: ||s||^2's partials go to row 2 and ride with the omega
            // round (t.s, t.t in rows 0, 1 from the product): one level 2 and, on P
            // ranks, one all-gather fewer per iteration.  The break test (:117)
            // only steers the x/r update, which follows the omega round anyway;
            // the preconditioner apply and product on s run in either case.
            if (merge_s) e.pslot = 2;
            LSSP_TRY(R.ew(e));
        }
        *pos_s = R.tl;
        const Fin fs = R.fin(FIN_BICG_S, 1, R.T());          // :117
        if (!merge_s) LSSP_TRY(R.fin1(s, s, fs));
        LSSP_TRY(R.pc_spmv(sh, s, EPI_AMX, 1, 0, p, t, gew && merge_s ? 3 : 2, s, nullptr));  // :130-131, :133
        {
            int t0 = R.T(), t1 = R.T();
            if (merge_s) {
                Fin f = R.fin(FIN_BICG_S_OMEGA, 3, t0, t1);
                f.tpos[2] = fs.tpos[0];
                const double *A_[3] = {t, t, s}, *B_[3] = {s, t, s};
                LSSP_TRY(finish_reduce(R.c, R.n, 3, A_, B_, f));  // :117 + :135
            } else {
                LSSP_TRY(R.fin2(t, s, t, t, R.fin(FIN_BICG_OMEGA, 2, t0, t1)));  // :135
            }
        }
        e = Ew();
        e.kind = K_BICG_XR;  // :136-139
        e.out0 = x;
        e.x = ph;
        e.y = sh;
        e.out1 = r;
        e.u = s;
        e.v = t;
        e.nred = 2;
        e.r0a = r;
        e.r0b = r;
        e.r1a = r;
        e.r1b = rh;
        LSSP_TRY(R.ew(e));
        int t0 = R.T(), t1 = R.T();
        return R.fin2(r, r, r, rh, R.fin(fin_res, 2, t0, t1));  // :141, next :87
    };
    // :117-128 after the device took x += alpha*ph: the reference evaluates
    // ||s|| again (trace), then r = b - A x and its norm
    auto breakdown = [&](long pos_s) -> int {
        if (R.rank == 0) lprint("bicgstab: ||s|| is too small: %f, terminated.\n", R.h(S_SNORM));
        R.tl = pos_s + 1;
        long q = R.tl++;
        R.patches.push_back({q, R.h(S_SNORM)});
        LSSP_TRY(R.spmv(EPI_AXPBY, -1, x, 1, b, r));  // :124
        LSSP_TRY(R.dot1(r, r, R.fin(FIN_NORM, 1, R.T(), -1, S_RES)));
        LSSP_TRY(R.sync(0, 16));
        res = R.h(S_RES);
        return LSSP_AMD_OK;
    };
    auto itr_line = [&](int k, double rk) {
        if (P.verb >= 1 && R.rank == 0)
            lprint("bicgstab: itr: %5d, abs res: %.6e, rel res: %.6e, rbn: %.6e\n", k, rk,
                   (err_rel == 0 ? 0 : rk / err_rel), (b_norm == 0 ? 0 : rk / b_norm));
    };
    const bool batched = !R.M || R.M->line.ntiles > 0;
    if (batched && rho1 == 0) {  // :89-92 at the first iteration
        if (R.rank == 0) lprint("bicgstab: method failed.!\n");
        it = 0;
    } else if (batched) {
        // Line-swept or no preconditioner: iterations are queued in
        // batches and the stop tests run on the device (FIN_BICG_RES_RHO_B:
        // breakdown :117, res <= tol :149, rho1 == 0 :89 of the next); the
        // launches past the stop return at once (ctx guard), and the host reads a
        // batch's residuals from its snapshot while the next batch runs
        // (Run::snap_issue).  Same kernels, same arithmetic.
        constexpr int BATCH = 8;
        static_assert(2 * BATCH <= S_HB, "two batches in the residual history ring");
        lssp_amd_ctx *c = R.c;
        struct Batch {
            int it0 = 0, nb = 0;
            long tl_after[BATCH], pos_s[BATCH];
        } bq[2];
        int queued = 0, nq = 0, nr = 0;  // iterations queued, batches queued, batches read
        auto push = [&]() -> int {
            Batch &B = bq[nq & 1];
            B.it0 = queued;
            B.nb = std::min(BATCH, maxit - queued);
            c->guard = c->d_scal + S_DONE;
            int st = LSSP_AMD_OK;
            for (int j = 0; j < B.nb && st == LSSP_AMD_OK; j++) {
                st = enqueue(queued + j, FIN_BICG_RES_RHO_B, &B.pos_s[j]);
                B.tl_after[j] = R.tl;
            }
            c->guard = nullptr;
            LSSP_TRY(st);
            LSSP_TRY(R.snap_issue(nq & 1));
            queued += B.nb;
            nq++;
            return LSSP_AMD_OK;
        };
        it = 0;
        LSSP_TRY(R.batch_begin(tol));
        LSSP_TRY(push());
        for (;;) {
            if (queued < maxit) LSSP_TRY(push());  // runs while the batch before it is read
            const Batch &B = bq[nr & 1];
            LSSP_TRY(R.snap_wait(nr & 1));
            nr++;
            auto hist = [&](int q) { return R.h(S_H + (B.it0 + q) % S_HB); };
            const int ran = std::max(1, std::min(B.nb, (int)R.h(S_NIT) - B.it0));
            const int code = (int)R.h(S_DONE);
            for (int q = 0; q < ran - (code == 2 ? 1 : 0); q++) itr_line(it + q, hist(q));
            res = hist(ran - 1);
            pending_rho = true;
            if (code == 2) {  // breakdown in iteration it + ran - 1
                it += ran - 1;
                pending_rho = false;
                LSSP_TRY(breakdown(B.pos_s[ran - 1]));
                break;
            } else if (code == 1) {  // converged
                R.tl = B.tl_after[ran - 1];
                it += ran - 1;
                break;
            } else if (code == 3) {  // the next iteration's rho1 == 0
                R.tl = B.tl_after[ran - 1];
                it += ran;
                pending_rho = false;
                if (it < maxit) {
                    if (R.rank == 0) lprint("bicgstab: method failed.!\n");
                    break;
                }
                pending_rho = true;
            } else {
                it += B.nb;
            }
            if (nr == nq) break;  // maxit
        }
    } else {
        for (it = 0; it < maxit; it++) {
            pending_rho = false;
            if (rho1 == 0) {  // :89-92
                if (R.rank == 0) lprint("bicgstab: method failed.!\n");
                break;
            }
            long pos_s = 0;
            LSSP_TRY(enqueue(it, FIN_BICG_RES_RHO, &pos_s));
            LSSP_TRY(R.sync(0, 16));
            if (R.h(S_BREAK) != 0.0) {  // :117-128 -- x += alpha*ph already done on the device
                LSSP_TRY(breakdown(pos_s));
                break;
            }
            pending_rho = true;
            res = R.h(S_RES);
            itr_line(it, res);
            if (res <= tol) break;  // :149
            rho1 = R.h(S_RHO1);
        }
    }
    if (pending_rho) R.tl--;  // the fused next-iteration rho1 is not part of the reference's run
    if (it < maxit) it += 1;  // :152
    if (P.verb >= 2 && R.rank == 0) {
        lprint("bicgstab: total iteration: %d\n", it);
        lprint("bicgstab: total time: %g\n", wall_time() - t_start);
    }
    *nits = it;
    *res_out = res;
    return LSSP_AMD_OK;
}

// ---------------------------------------------------------------------------
// CG (solver-cg.cxx:8-136)
// ---------------------------------------------------------------------------
int cg(Run &R, const lssp_amd_solve_params &P, double *x, const double *b, int *nits, double *res_out)
{
    const double t_start = wall_time();  // the reference driver's lssp_get_time() ("total time")
    double tol_rel, tol_abs, tol_rb = P.tol_rb, tol;
    int maxit, it;
    defaults(P, tol_rel, tol_abs, maxit);
    if (P.verb >= 2 && R.rank == 0) {
        lprint("cg: maximal iteration: %d\n", maxit);
        lprint("cg: tolerance abs: %g\n", tol_abs);
        lprint("cg: tolerance rel: %g\n", tol_rel);
        lprint("cg: tolerance rbn: %g\n", tol_rb);
    }
    double *r = R.vec(), *p = R.vec(), *q = R.vec();
    double *z = R.M ? R.vec() : r;  // PC_NON copies r into z (pc.cxx:67-70): alias instead
    if (!r || !p || !q || !z) return LSSP_AMD_ENOMEM;

    LSSP_TRY(R.dot1(b, b, R.fin(FIN_NORM, 1, R.T(), -1, S_BNORM)));  // :231
    LSSP_TRY(R.spmv(EPI_AXPBY, -1, x, 1, b, r));                      // :234
    LSSP_TRY(R.dot1(r, r, R.fin(FIN_NORM, 1, R.T(), -1, S_RES)));    // :235
    LSSP_TRY(R.sync(0, 16));
    const double b_norm = R.h(S_BNORM);
    tol_rb *= b_norm;
    double res = R.h(S_RES);
    if (res <= tol_abs) {
        *nits = 0;
        *res_out = res;
        return LSSP_AMD_OK;
    }
    const double err_rel = res;
    tol = tol_rel * err_rel;
    if (tol < tol_abs) tol = tol_abs;
    if (tol < tol_rb) tol = tol_rb;
    bool pending_rho = false;

    if (!R.M) {
        // PC_NON: iterations are queued in batches and the stop
        // test :109 runs on the device (FIN_CG_RES_RHO_B); the launches of the
        // iterations after the one that converged return at once (ctx guard),
        // and the host reads a batch's residuals from its snapshot while the
        // next batch runs (Run::snap_issue).  Same kernels, same arithmetic.
#ifndef CG_BATCH
#define CG_BATCH 32  // config 5: 32 against 16 / 8 per batch 21.54-21.84 K / 21.34-21.44 K / 20.98-21.09 K it/s (r06u)
#endif
        constexpr int BATCH = CG_BATCH;  // iterations per batch (A/B: -DCG_BATCH)
        static_assert(2 * BATCH <= S_HB, "two batches in the residual history ring");
        lssp_amd_ctx *c = R.c;
        const bool fuse_l2 = R.tree && c->nranks == 1 && R.n > 0;
        struct Batch {
            int it0 = 0, nb = 0;
            long tl_after[BATCH];
        } bq[2];
        int queued = 0, nq = 0, nr = 0;  // iterations queued, batches queued, batches read
        auto push = [&]() -> int {
            Batch &B = bq[nq & 1];
            B.it0 = queued;
            B.nb = std::min(BATCH, maxit - queued);
            c->guard = c->d_scal + S_DONE;
            int st = LSSP_AMD_OK;
            // one rank, tree reductions: each reduction's level 2 runs inside
            // the vector update that consumes it (k_cg_fused): q.p (partial
            // row 0, from the product) in the x/r update, r.r (row 1) in the
            // next iteration's p update; the batch's last r.r on its own.
            // Stamps are global iteration counts (FIN_CG_RES_RHO_B's S_DONE)
            Fin held;
            bool have_held = false;
            for (int j = 0; j < B.nb && st == LSSP_AMD_OK; j++) {
                const int k = queued + j;
                Ew e;
                if (k == 0) {
                    st = R.dot1(r, r, R.fin(FIN_CG_RHO, 1, R.T()));  // :80 (z == r)
                    e.kind = K_COPY;                                  // :83-86
                } else {
                    e.kind = K_CG_P;  // :88-92
                }
                e.x = z;
                e.out0 = p;
                if (st == LSSP_AMD_OK) {
                    // with the x update of the previous x/r pass (CGF_R): its stop test is stamped k
                    if (have_held) st = launch_cg_fused(c, CGF_PX, R.n, x, p, nullptr, z, nullptr, 1, 1, held, k);
                    else st = R.ew(e);
                }
                have_held = false;
                if (st == LSSP_AMD_OK) st = R.spmv(EPI_MXY, 1, p, 0, nullptr, q, 1, p);  // :95
                const Fin fa = R.fin(FIN_CG_ALPHA, 1, R.T());                            // :96-99
                if (fuse_l2) {
                    // r only: x += alpha p (:102) rides with the next p pass, or the batch's CGF_X
                    if (st == LSSP_AMD_OK) st = launch_cg_fused(c, CGF_R, R.n, x, p, r, nullptr, q, 0, 1, fa);
                } else {
                    if (st == LSSP_AMD_OK) st = R.fin1(q, p, fa);
                    e = Ew();
                    e.kind = K_CG_XR;  // :101-104
                    e.out0 = x;
                    e.x = p;
                    e.out1 = r;
                    e.y = q;
                    e.nred = 1;
                    e.r0a = r;
                    e.r0b = r;
                    if (st == LSSP_AMD_OK) st = R.ew(e);
                }
                int t0 = R.T(), t1 = R.T();
                const Fin fr = R.fin(FIN_CG_RES_RHO_B, 1, t0, t1);  // :106-109, next :80
                if (fuse_l2 && j + 1 < B.nb) {
                    held = fr;
                    have_held = true;
                } else if (fuse_l2) {
                    if (st == LSSP_AMD_OK) st = launch_reduce_tree(c, num_chunks(R.n), 1, fr, 1);
                    if (st == LSSP_AMD_OK)
                        st = launch_cg_fused(c, CGF_X, R.n, x, p, nullptr, nullptr, nullptr, 1, 1, Fin(), k + 1);
                } else {
                    if (st == LSSP_AMD_OK) st = R.fin1(r, r, fr);
                }
                B.tl_after[j] = R.tl;
            }
            c->guard = nullptr;
            LSSP_TRY(st);
            LSSP_TRY(R.snap_issue(nq & 1));
            queued += B.nb;
            nq++;
            return LSSP_AMD_OK;
        };
        it = 0;
        LSSP_TRY(R.batch_begin(tol));
        LSSP_TRY(push());
        for (;;) {
            if (queued < maxit) LSSP_TRY(push());  // runs while the batch before it is read
            const Batch &B = bq[nr & 1];
            LSSP_TRY(R.snap_wait(nr & 1));
            nr++;
            const int ran = std::max(1, std::min(B.nb, (int)R.h(S_NIT) - B.it0));
            for (int q = 0; q < ran; q++) {
                res = R.h(S_H + (B.it0 + q) % S_HB);
                if (P.verb >= 1 && R.rank == 0)
                    lprint("cg: itr: %5d, abs res: %.6e, rel res: %.6e, rbn: %.6e\n", it + q, res,
                           (err_rel == 0 ? 0 : res / err_rel), (b_norm == 0 ? 0 : res / b_norm));
            }
            pending_rho = true;
            if (R.h(S_DONE) != 0.0) {  // :109 held at iteration it + ran - 1
                R.tl = B.tl_after[ran - 1];
                it += ran - 1;
                break;
            }
            it += B.nb;
            if (nr == nq) break;  // maxit
        }
    } else {
        for (it = 0; it < maxit; it++) {
            pending_rho = false;
            if (R.M) {
                LSSP_TRY(R.pc(z, r));                                   // :79
                LSSP_TRY(R.dot1(z, r, R.fin(FIN_CG_RHO, 1, R.T())));   // :80
            } else if (it == 0) {
                LSSP_TRY(R.dot1(r, r, R.fin(FIN_CG_RHO, 1, R.T())));
            }
            Ew e;
            if (it == 0) {
                e.kind = K_COPY;  // :83-86
                e.x = z;
                e.out0 = p;
            } else {
                e.kind = K_CG_P;  // :88-92
                e.x = z;
                e.out0 = p;
            }
            LSSP_TRY(R.ew(e));
            LSSP_TRY(R.spmv(EPI_MXY, 1, p, 0, nullptr, q, 1, p));        // :95
            LSSP_TRY(R.fin1(q, p, R.fin(FIN_CG_ALPHA, 1, R.T())));      // :96-99
            e = Ew();
            e.kind = K_CG_XR;  // :101-104
            e.out0 = x;
            e.x = p;
            e.out1 = r;
            e.y = q;
            e.nred = 1;
            e.r0a = r;
            e.r0b = r;
            LSSP_TRY(R.ew(e));
            if (R.M) {
                LSSP_TRY(R.fin1(r, r, R.fin(FIN_CG_RES, 1, R.T())));  // :106
            } else {
                int t0 = R.T(), t1 = R.T();
                LSSP_TRY(R.fin1(r, r, R.fin(FIN_CG_RES_RHO, 1, t0, t1)));  // :106, next :80 (z == r)
                pending_rho = true;
            }
            LSSP_TRY(R.sync(0, 16));
            res = R.h(S_RES);
            if (P.verb >= 1 && R.rank == 0)
                lprint("cg: itr: %5d, abs res: %.6e, rel res: %.6e, rbn: %.6e\n", it, res,
                       (err_rel == 0 ? 0 : res / err_rel), (b_norm == 0 ? 0 : res / b_norm));
            if (res <= tol) break;  // :109
        }
    }
    if (pending_rho) R.tl--;
    if (it < maxit) it += 1;
    if (P.verb >= 2 && R.rank == 0) {
        lprint("cg: total iteration: %d\n", it);
        lprint("cg: total time: %g\n", wall_time() - t_start);
    }
    *nits = it;
    *res_out = res;
    return LSSP_AMD_OK;
}

// ---------------------------------------------------------------------------
// GMRES(m), left preconditioned, MGS Arnoldi, Givens on the host
// (solver-gmres.cxx:12-255)
// ---------------------------------------------------------------------------
int gmres(Run &R, const lssp_amd_solve_params &P, double *x, const double *b, int *nits, double *res_out)
{
    const double t_start = wall_time();  // the reference driver's lssp_get_time() ("total time")
    lssp_amd_ctx *c = R.c;
    double tol_rel, tol_abs, tol_rb = P.tol_rb;
    int maxit;
    defaults(P, tol_rel, tol_abs, maxit);
    int m = P.restart < 0 ? DEF_RESTART : P.restart;
    if (tol_rb < 0) tol_rb = DEF_TOL;
    if (m <= 0) return LSSP_AMD_EINVAL;
    if (S_H + 2 * m + 2 > NSCAL) return LSSP_AMD_EUNSUPPORTED;  // Hessenberg column + ym staging
    if (P.verb >= 2 && R.rank == 0) {
        lprint("gmres: restart parameter m: %d\n", m);
        lprint("gmres: maximal iteration: %d\n", maxit);
        lprint("gmres: tolerance abs: %g\n", tol_abs);
        lprint("gmres: tolerance rel: %g\n", tol_rel);
        lprint("gmres: tolerance rbn: %g\n", tol_rb);
    }
    double *wj = R.vec(), *rg = R.vec();
    double *V = R.vec(R.nx * (long)m);
    double *d_ym = R.vec(m);
    if (!wj || !rg || !V || !d_ym) return LSSP_AMD_ENOMEM;
    auto Vi = [&](int i) { return V + (long)i * R.nx; };
    std::vector<double> H((size_t)(m + 1) * m), gg(m + 1), cs(m), sn(m), ym(m);
    auto HG = [&](int row, int col) -> double & { return H[(size_t)row * m + col]; };

    LSSP_TRY(R.dot1(b, b, R.fin(FIN_NORM, 1, R.T(), -1, S_BNORM)));  // :85
    LSSP_TRY(R.spmv(EPI_AXPBY, -1, x, 1, b, rg));                     // :88
    LSSP_TRY(R.dot1(rg, rg, R.fin(FIN_NORM, 1, R.T(), -1, S_RES)));  // :89
    LSSP_TRY(R.sync(0, 16));
    const double b_norm = R.h(S_BNORM);
    tol_rb *= b_norm;
    double beta = R.h(S_RES);
    int inner = 0;
    if (beta <= tol_abs) {
        *nits = 0;
        *res_out = beta;
        return LSSP_AMD_OK;
    }
    const double err_rel = beta;
    double tol = tol_rel * err_rel;
    if (tol < tol_abs) tol = tol_abs;
    if (tol < tol_rb) tol = tol_rb;
    const double rtol = tol / beta;
    double gstol = 0.;

    while (inner < maxit) {
        int i, kk;
        double gs_norm = 0.;
        const bool first_cycle = inner == 0;
        LSSP_TRY(R.pc(Vi(0), rg));                                             // :112-113
        LSSP_TRY(R.dot1(Vi(0), Vi(0), R.fin(FIN_NORM, 1, R.T(), -1, S_TMP)));  // :115
        {
            Ew e;
            e.kind = K_DIVS;  // :129-131
            e.out0 = Vi(0);
            e.sidx = S_TMP;
            LSSP_TRY(R.ew(e));
        }
        std::fill(gg.begin(), gg.end(), 0.0);
        std::fill(H.begin(), H.end(), 0.0);
        bool have_beta = false;
        for (i = 0; i < m; i++) {
            inner++;
            LSSP_TRY(R.spmv(EPI_MXY, 1, Vi(i), 0, nullptr, rg));  // :138
            LSSP_TRY(R.pc(wj, rg));                                // :139-140
            LSSP_TRY(R.dot1(wj, Vi(0), R.fin(FIN_STORE, 1, R.T(), -1, S_H)));  // :143, j = 0
            for (int j = 0; j <= i; j++) {  // :142-147, axpy fused with the next dot / the norm
                Ew e;
                e.kind = K_GM_MGS;
                e.out0 = wj;
                e.x = Vi(j);
                e.sidx = S_H + j;
                e.nred = 1;
                e.r0a = wj;
                e.r0b = j < i ? Vi(j + 1) : wj;
                LSSP_TRY(R.ew(e));
                if (j < i)
                    LSSP_TRY(R.fin1(wj, Vi(j + 1), R.fin(FIN_STORE, 1, R.T(), -1, S_H + j + 1)));
                else
                    LSSP_TRY(R.fin1(wj, wj, R.fin(FIN_NORM, 1, R.T(), -1, S_H + i + 1)));  // :149
            }
            LSSP_TRY(R.sync(0, S_H + i + 2));
            if (!have_beta) {
                beta = R.h(S_TMP);
                gg[0] = beta;  // :116
                if (first_cycle) gstol = rtol * beta * 0.5;  // :121-123
                have_beta = true;
            }
            for (int j = 0; j <= i; j++) HG(j, i) = R.h(S_H + j);
            const double hij = R.h(S_H + i + 1);
            HG(i + 1, i) = hij;
            if (std::fabs(hij) <= BREAKDOWN) {  // :152-155
                i--;
                break;
            } else if (i + 1 < m) {
                Ew e;
                e.kind = K_AXY;  // :157
                e.a = 1 / hij;
                e.x = wj;
                e.out0 = Vi(i + 1);
                LSSP_TRY(R.ew(e));
            }
            for (int j = 0; j < i; j++) {  // :160-166
                const double h1 = cs[j] * HG(j, i) + sn[j] * HG(j + 1, i);
                const double h2 = -sn[j] * HG(j, i) + cs[j] * HG(j + 1, i);
                HG(j, i) = h1;
                HG(j + 1, i) = h2;
            }
            double gma = std::sqrt(HG(i, i) * HG(i, i) + HG(i + 1, i) * HG(i + 1, i));  // :168
            if (std::fabs(gma) == 0.) gma = 1e-20;
            cs[i] = HG(i, i) / gma;
            sn[i] = HG(i + 1, i) / gma;
            gg[i + 1] = -sn[i] * gg[i];
            gg[i] = cs[i] * gg[i];
            HG(i, i) = cs[i] * HG(i, i) + sn[i] * HG(i + 1, i);
            gs_norm = std::fabs(gg[i + 1]);
            if (gs_norm <= gstol) break;  // :179-181
        }
        if (!have_beta) {  // (i == 0 breakdown without a sync is impossible; kept for safety)
            LSSP_TRY(R.sync(0, 16));
            beta = R.h(S_TMP);
            gg[0] = beta;
            if (first_cycle) gstol = rtol * beta * 0.5;
        }
        kk = i == m ? m : i + 1;  // :185
        for (i = kk - 1; i >= 0; i--) {  // :186-194
            ym[i] = gg[i] / HG(i, i);
            for (int j = 0; j < i; j++) gg[j] = gg[j] - ym[i] * HG(j, i);
        }
        if (kk > 0) {
            memcpy(c->h_scal + NSCAL - m, ym.data(), sizeof(double) * kk);
            LSSP_HIP(hipMemcpyAsync(d_ym, c->h_scal + NSCAL - m, sizeof(double) * kk,
                                    hipMemcpyHostToDevice, c->stream));
        }
        {
            Ew e;
            e.kind = K_GM_X;  // :196-204
            e.out0 = x;
            e.vbase = V;
            e.k = kk;
            e.u = d_ym;
            e.b = (double)R.nx;  // basis stride
            LSSP_TRY(R.ew(e));
        }
        LSSP_TRY(R.spmv(EPI_AXPBY, -1, x, 1, b, rg));                     // :206
        LSSP_TRY(R.dot1(rg, rg, R.fin(FIN_NORM, 1, R.T(), -1, S_RES)));  // :207
        LSSP_TRY(R.sync(0, 16));
        beta = R.h(S_RES);
        if (P.verb >= 1 && R.rank == 0)
            lprint("gmres: itr: %4d / %5d, abs res: %.6e, rel res: %.6e, rbn: %.6e\n", inner, inner, beta,
                   (err_rel == 0 ? 0 : beta / err_rel), (b_norm == 0 ? 0 : beta / b_norm));
        if (beta <= tol) break;                                  // :215-217
        gstol = rtol * gs_norm / (beta / err_rel) * 0.5;          // :220
    }
    if (P.verb >= 2 && R.rank == 0) {
        lprint("gmres: total iteration: %d\n", inner);
        lprint("gmres: total time: %g\n", wall_time() - t_start);
    }
    *nits = inner;
    *res_out = beta;
    return LSSP_AMD_OK;
}

// ---------------------------------------------------------------------------
// GMRES(m), right preconditioned (solver-gmres.cxx:257-479): A M^-1 u = b,
// x = x0 + M^-1 (V y).  The residual reported is the Givens estimate |g_{i+1}|
// (:370, :427); a true residual b - A x is formed only to restart (:433).
// ---------------------------------------------------------------------------
int gmres_r(Run &R, const lssp_amd_solve_params &P, double *x, const double *b, int *nits, double *res_out)
{
    const double t_start = wall_time();  // the reference driver's lssp_get_time() ("total time")
    lssp_amd_ctx *c = R.c;
    double tol_rel, tol_abs, tol_rb = P.tol_rb;
    int maxit;
    defaults(P, tol_rel, tol_abs, maxit);
    int m = P.restart < 0 ? DEF_RESTART : P.restart;
    if (tol_rb < 0) tol_rb = DEF_TOL;
    if (m <= 0) return LSSP_AMD_EINVAL;
    if (S_H + 2 * m + 2 > NSCAL) return LSSP_AMD_EUNSUPPORTED;
    if (P.verb >= 2 && R.rank == 0) {
        lprint("gmres: restart parameter m: %d\n", m);
        lprint("gmres: maximal iteration: %d\n", maxit);
        lprint("gmres: tolerance abs: %g\n", tol_abs);
        lprint("gmres: tolerance rel: %g\n", tol_rel);
        lprint("gmres: tolerance rbn: %g\n", tol_rb);
    }
    double *wj = R.vec(), *rg = R.vec();
    double *V = R.vec(R.nx * (long)m);
    double *d_ym = R.vec(m);
    if (!wj || !rg || !V || !d_ym) return LSSP_AMD_ENOMEM;
    auto Vi = [&](int i) { return V + (long)i * R.nx; };
    std::vector<double> H((size_t)(m + 1) * m), gg(m + 1), cs(m), sn(m), ym(m);
    auto HG = [&](int row, int col) -> double & { return H[(size_t)row * m + col]; };

    LSSP_TRY(R.dot1(b, b, R.fin(FIN_NORM, 1, R.T(), -1, S_BNORM)));  // :324
    LSSP_TRY(R.spmv(EPI_AXPBY, -1, x, 1, b, rg));                     // :327
    LSSP_TRY(R.dot1(rg, rg, R.fin(FIN_NORM, 1, R.T(), -1, S_RES)));  // :328
    LSSP_TRY(R.sync(0, 16));
    const double b_norm = R.h(S_BNORM);
    tol_rb *= b_norm;
    double beta = R.h(S_RES);
    int inner = 0;
    if (beta <= tol_abs) {  // :330-333
        *nits = 0;
        *res_out = beta;
        return LSSP_AMD_OK;
    }
    const double err_rel = beta;
    double tol = tol_rel * err_rel;
    if (tol < tol_abs) tol = tol_abs;
    if (tol < tol_rb) tol = tol_rb;

    while (inner < maxit) {
        int i, kk;
        std::fill(gg.begin(), gg.end(), 0.0);  // :345-351
        std::fill(H.begin(), H.end(), 0.0);
        LSSP_TRY(R.dot1(rg, rg, R.fin(FIN_NORM, 1, R.T(), -1, S_TMP)));  // :354
        LSSP_TRY(R.sync(0, 16));
        gg[0] = beta = R.h(S_TMP);
        {
            Ew e;
            e.kind = K_AXY;  // :355, a multiply by 1/beta
            e.a = 1 / beta;
            e.x = rg;
            e.out0 = Vi(0);
            LSSP_TRY(R.ew(e));
        }
        bool converged = false;
        for (i = 0; i < m && inner < maxit; i++) {
            inner++;
            LSSP_TRY(R.pc(rg, Vi(i)));                              // :362-363
            LSSP_TRY(R.spmv(EPI_MXY, 1, rg, 0, nullptr, wj));      // :364
            LSSP_TRY(R.dot1(wj, Vi(0), R.fin(FIN_STORE, 1, R.T(), -1, S_H)));  // :367, j = 0
            for (int j = 0; j <= i; j++) {  // :366-371, axpy fused with the next dot / the norm
                Ew e;
                e.kind = K_GM_MGS;
                e.out0 = wj;
                e.x = Vi(j);
                e.sidx = S_H + j;
                e.nred = 1;
                e.r0a = wj;
                e.r0b = j < i ? Vi(j + 1) : wj;
                LSSP_TRY(R.ew(e));
                if (j < i)
                    LSSP_TRY(R.fin1(wj, Vi(j + 1), R.fin(FIN_STORE, 1, R.T(), -1, S_H + j + 1)));
                else
                    LSSP_TRY(R.fin1(wj, wj, R.fin(FIN_NORM, 1, R.T(), -1, S_H + i + 1)));  // :373
            }
            LSSP_TRY(R.sync(0, S_H + i + 2));
            for (int j = 0; j <= i; j++) HG(j, i) = R.h(S_H + j);
            const double hij = R.h(S_H + i + 1);
            HG(i + 1, i) = hij;
            if (std::fabs(hij) <= BREAKDOWN) {  // :377-380
                i--;
                break;
            } else if (i + 1 < m) {
                Ew e;
                e.kind = K_AXY;  // :382
                e.a = 1 / hij;
                e.x = wj;
                e.out0 = Vi(i + 1);
                LSSP_TRY(R.ew(e));
            }
            for (int j = 0; j < i; j++) {  // :385-391
                const double h1 = cs[j] * HG(j, i) + sn[j] * HG(j + 1, i);
                const double h2 = -sn[j] * HG(j, i) + cs[j] * HG(j + 1, i);
                HG(j, i) = h1;
                HG(j + 1, i) = h2;
            }
            double gma = std::sqrt(HG(i, i) * HG(i, i) + HG(i + 1, i) * HG(i + 1, i));  // :393
            if (std::fabs(gma) == 0.) gma = 1e-20;
            cs[i] = HG(i, i) / gma;
            sn[i] = HG(i + 1, i) / gma;
            gg[i + 1] = -sn[i] * gg[i];
            gg[i] = cs[i] * gg[i];
            HG(i, i) = cs[i] * HG(i, i) + sn[i] * HG(i + 1, i);
            beta = std::fabs(gg[i + 1]);
            if (P.verb >= 1 && R.rank == 0)
                lprint("rgmres: itr: %4d, abs res: %.6e, rel res: %.6e, rbn: %.6e\n", inner, beta,
                       (err_rel == 0 ? 0 : beta / err_rel), (b_norm == 0 ? 0 : beta / b_norm));
            if (beta <= tol) {  // :409-411 (goto solve: i is not advanced)
                converged = true;
                break;
            }
        }
        (void)converged;
        kk = i == m ? m : i + 1;  // :414
        for (i = kk - 1; i >= 0; i--) {  // :415-420
            ym[i] = gg[i] / HG(i, i);
            for (int j = 0; j < i; j++) gg[j] = gg[j] - ym[i] * HG(j, i);
        }
        if (kk > 0) {  // :423-431
            memcpy(c->h_scal + NSCAL - m, ym.data(), sizeof(double) * kk);
            LSSP_HIP(hipMemcpyAsync(d_ym, c->h_scal + NSCAL - m, sizeof(double) * kk, hipMemcpyHostToDevice,
                                    c->stream));
            Ew e;
            e.kind = K_GMR_Z;
            e.out0 = rg;
            e.vbase = V;
            e.k = kk;
            e.u = d_ym;
            e.b = (double)R.nx;  // basis stride
            LSSP_TRY(R.ew(e));
            LSSP_TRY(R.pc(wj, rg));  // :429
            Ew xa;
            xa.kind = K_AXPBY;  // :430: x = x*1 + wj*1
            xa.a = 1;
            xa.b = 1;
            xa.x = wj;
            xa.out0 = x;
            LSSP_TRY(R.ew(xa));
        }
        if (beta <= tol) break;                          // :433-435
        LSSP_TRY(R.spmv(EPI_AXPBY, -1, x, 1, b, rg));    // :437
    }
    if (P.verb >= 2 && R.rank == 0) {
        lprint("gmres: total iteration: %d\n", inner);
        lprint("gmres: total time: %g\n", wall_time() - t_start);
    }
    LSSP_TRY(R.sync(0, 1));  // the last x update is complete when the call returns
    *nits = inner;
    *res_out = beta;
    return LSSP_AMD_OK;
}

// ---------------------------------------------------------------------------
// LGMRES(m, k) (solver-lgmres.cxx:12-312): left-preconditioned GMRES(m)
// augmented with the last k corrections z; the cycle's basis grows by one z per
// cycle up to m + k.  Kept exactly as the reference has it:
//   * v_{i+1} = w / h and v_0 /= beta are true divisions (:192-194, :149-151);
//   * the solve uses kk = i columns (:216), so a gstol exit drops the last one;
//   * the x update sums min(kk, m) basis terms, then -- when kk > m -- the
//     first min(cycle, k) z terms with y[m + i] (:226-245), whether or not this
//     cycle set them (y persists across cycles; it starts at zero here).
// ---------------------------------------------------------------------------
int lgmres(Run &R, const lssp_amd_solve_params &P, double *x, const double *b, int *nits, double *res_out)
{
    const double t_start = wall_time();  // the reference driver's lssp_get_time() ("total time")
    lssp_amd_ctx *c = R.c;
    double tol_rel, tol_abs, tol_rb = P.tol_rb;
    int maxit;
    defaults(P, tol_rel, tol_abs, maxit);
    const int mk = P.restart < 0 ? DEF_RESTART : P.restart;
    const int auk = P.aug_k <= 0 ? 3 : P.aug_k;  // lssp.cxx:6
    if (tol_rb < 0) tol_rb = DEF_TOL;
    if (mk <= 0) return LSSP_AMD_EINVAL;
    const int mmax = mk + auk;
    if (S_H + 2 * mmax + 2 > NSCAL || mmax > 0x7fff || auk > 0x7fff) return LSSP_AMD_EUNSUPPORTED;
    if (P.verb >= 2 && R.rank == 0) {
        lprint("lgmres: restart parameter m: %d\n", mk);
        lprint("lgmres: aug k: %d\n", auk);
        lprint("lgmres: maximal iteration: %d\n", maxit);
        lprint("lgmres: tolerance abs: %g\n", tol_abs);
        lprint("lgmres: tolerance rel: %g\n", tol_rel);
        lprint("lgmres: tolerance rbn: %g\n", tol_rb);
    }
    double *wj = R.vec(), *rg = R.vec();
    double *V = R.vec(R.nx * (long)mmax);
    double *Z = R.vec(R.nx * (long)auk);
    double *d_ym = R.vec(mmax);
    if (!wj || !rg || !V || !Z || !d_ym) return LSSP_AMD_ENOMEM;
    auto Vi = [&](int i) { return V + (long)i * R.nx; };
    auto Zi = [&](int i) { return Z + (long)i * R.nx; };
    std::vector<double> H((size_t)(mmax + 1) * mmax), gg(mmax + 1), cs(mmax), sn(mmax), ym(mmax, 0.0);
    auto HG = [&](int row, int col) -> double & { return H[(size_t)row * mmax + col]; };

    LSSP_TRY(R.dot1(b, b, R.fin(FIN_NORM, 1, R.T(), -1, S_BNORM)));  // :108
    LSSP_TRY(R.spmv(EPI_AXPBY, -1, x, 1, b, rg));                     // :111
    LSSP_TRY(R.dot1(rg, rg, R.fin(FIN_NORM, 1, R.T(), -1, S_RES)));  // :112
    LSSP_TRY(R.sync(0, 16));
    const double b_norm = R.h(S_BNORM);
    tol_rb *= b_norm;
    double beta = R.h(S_RES);
    int inner = 0, outer = 0;
    if (beta <= tol_abs) {
        *nits = 0;
        *res_out = beta;
        return LSSP_AMD_OK;
    }
    const double err_rel = beta;
    double tol = tol_rel * err_rel;
    if (tol < tol_abs) tol = tol_abs;
    if (tol < tol_rb) tol = tol_rb;
    const double rtol = tol / beta;
    double gstol = 0.;

    while (inner < maxit) {
        int i, kk;
        double gs_norm = 0.;
        LSSP_TRY(R.pc(Vi(0), rg));                                             // :130-131
        LSSP_TRY(R.dot1(Vi(0), Vi(0), R.fin(FIN_NORM, 1, R.T(), -1, S_TMP)));  // :133
        LSSP_TRY(R.sync(0, 16));
        beta = R.h(S_TMP);
        const int m = outer < auk ? mk + outer : mk + auk;  // :136-141
        std::fill(gg.begin(), gg.end(), 0.0);
        gg[0] = beta;
        if (outer == 0) gstol = rtol * beta * 0.5;  // :148-150
        std::fill(H.begin(), H.end(), 0.0);
        {
            Ew e;
            e.kind = K_DIVS;  // :156-158
            e.out0 = Vi(0);
            e.sidx = S_TMP;
            LSSP_TRY(R.ew(e));
        }
        for (i = 0; i < m; i++) {
            inner++;
            LSSP_TRY(R.spmv(EPI_MXY, 1, i < mk ? Vi(i) : Zi(i - mk), 0, nullptr, rg));  // :165-171
            LSSP_TRY(R.pc(wj, rg));                                                    // :173-174
            LSSP_TRY(R.dot1(wj, Vi(0), R.fin(FIN_STORE, 1, R.T(), -1, S_H)));         // :177, j = 0
            for (int j = 0; j <= i; j++) {  // :176-181
                Ew e;
                e.kind = K_GM_MGS;
                e.out0 = wj;
                e.x = Vi(j);
                e.sidx = S_H + j;
                e.nred = 1;
                e.r0a = wj;
                e.r0b = j < i ? Vi(j + 1) : wj;
                LSSP_TRY(R.ew(e));
                if (j < i)
                    LSSP_TRY(R.fin1(wj, Vi(j + 1), R.fin(FIN_STORE, 1, R.T(), -1, S_H + j + 1)));
                else
                    LSSP_TRY(R.fin1(wj, wj, R.fin(FIN_NORM, 1, R.T(), -1, S_H + i + 1)));  // :183
            }
            LSSP_TRY(R.sync(0, S_H + i + 2));
            for (int j = 0; j <= i; j++) HG(j, i) = R.h(S_H + j);
            const double hij = R.h(S_H + i + 1);
            HG(i + 1, i) = hij;
            if (std::fabs(hij) <= BREAKDOWN) {  // :186-189
                i--;
                break;
            } else if (i + 1 < m) {  // :191-195: v_{i+1} = w / h, a true division
                Ew cp;
                cp.kind = K_COPY;
                cp.x = wj;
                cp.out0 = Vi(i + 1);
                LSSP_TRY(R.ew(cp));
                Ew e;
                e.kind = K_DIVS;
                e.out0 = Vi(i + 1);
                e.sidx = S_H + i + 1;
                LSSP_TRY(R.ew(e));
            }
            for (int j = 0; j < i; j++) {  // :197-203
                const double h1 = cs[j] * HG(j, i) + sn[j] * HG(j + 1, i);
                const double h2 = -sn[j] * HG(j, i) + cs[j] * HG(j + 1, i);
                HG(j, i) = h1;
                HG(j + 1, i) = h2;
            }
            double gma = std::sqrt(HG(i, i) * HG(i, i) + HG(i + 1, i) * HG(i + 1, i));  // :205
            if (std::fabs(gma) == 0.) gma = 1e-20;
            cs[i] = HG(i, i) / gma;
            sn[i] = HG(i + 1, i) / gma;
            gg[i + 1] = -sn[i] * gg[i];
            gg[i] = cs[i] * gg[i];
            HG(i, i) = cs[i] * HG(i, i) + sn[i] * HG(i + 1, i);
            gs_norm = std::fabs(gg[i + 1]);
            if (gs_norm <= gstol) break;  // :216-218 (goto solve: i not advanced)
        }
        kk = i;  // :221
        for (i = kk - 1; i >= 0; i--) {  // :222-230
            ym[i] = gg[i] / HG(i, i);
            for (int j = 0; j < i; j++) gg[j] = gg[j] - ym[i] * HG(j, i);
        }
        memcpy(c->h_scal + NSCAL - mmax, ym.data(), sizeof(double) * mmax);
        LSSP_HIP(hipMemcpyAsync(d_ym, c->h_scal + NSCAL - mmax, sizeof(double) * mmax, hipMemcpyHostToDevice,
                                c->stream));
        {
            const int zn = outer % auk, nz = outer <= auk ? outer : auk;  // :233, :240-246
            Ew e;
            e.kind = K_LGM_X;  // :234-251
            e.out0 = x;
            e.out1 = Zi(zn);
            e.vbase = V;
            e.v = Z;
            e.u = d_ym;
            e.sidx = mk;
            e.k = (kk & 0xffff) | (nz << 16);
            e.b = (double)R.nx;  // basis stride
            LSSP_TRY(R.ew(e));
        }
        LSSP_TRY(R.spmv(EPI_AXPBY, -1, x, 1, b, rg));                     // :253
        LSSP_TRY(R.dot1(rg, rg, R.fin(FIN_NORM, 1, R.T(), -1, S_RES)));  // :254
        LSSP_TRY(R.sync(0, 16));
        beta = R.h(S_RES);
        if (P.verb >= 1 && R.rank == 0)
            lprint("lgmres: itr: %4d / %5d, abs res: %.6e, rel res: %.6e, rbn: %.6e\n", outer, inner, beta,
                   (err_rel == 0 ? 0 : beta / err_rel), (b_norm == 0 ? 0 : beta / b_norm));
        if (beta <= tol) break;                                  // :262
        gstol = rtol * gs_norm / (beta / err_rel) * 0.5;          // :265
        outer++;
    }
    if (P.verb >= 2 && R.rank == 0) {
        lprint("lgmres: total iteration: %d\n", inner);
        lprint("lgmres: total time: %g\n", wall_time() - t_start);
    }
    *nits = inner;
    *res_out = beta;
    return LSSP_AMD_OK;
}


// ===========================================================================
// The remaining Krylov drivers.  Unlike BiCGSTAB / CG / GMRES, the reference
// writes these purely as sequences of its L1 calls (lssp_vec_* vector.cxx,
// lssp_mv_* mvops.cxx, pc.solve) with host scalars, so each is restated here
// call for call over L1K below: the same kernels, operand order and aliasing,
// every dot / norm returned to the host where the reference branches on it.
// Work vectors start zeroed: three drivers read vectors lssp_vec_create left
// uninitialised (malloc, vector.cxx:4-20) before writing them (BiCGSafe y/u/z,
// BiCRSafe u/y/z/my, GPBiCG/GPBiCR mr/u/z/mt_old); the golden runs of the
// reference are made with zero-initialising malloc (oracle/ref_shim.cxx).
// ===========================================================================
struct L1K {
    Run &R;
    int st = LSSP_AMD_OK;  // first failure; every later call is a no-op
    // the last vector update is held back: when dots follow it, they are
    // reduced in the same pass (k_ew with partial sums of its results)
    Ew pend;
    bool has_pend = false;
    explicit L1K(Run &r) : R(r) {}
    ~L1K() { flush(); }  // a driver's last update (x) before it returns
    bool ok() const { return st == LSSP_AMD_OK; }
    void chk(int s)
    {
        if (st == LSSP_AMD_OK && s != LSSP_AMD_OK) st = s;
    }
    void flush()
    {
        if (has_pend && ok()) chk(R.ew(pend));
        has_pend = false;
    }
    double *vec()
    {
        double *p = R.vec();
        if (!p) chk(LSSP_AMD_ENOMEM);
        else set(p, 0.0);
        return p;
    }
    void ew(int kind, double a, double b, const double *x, const double *y, double *out)
    {
        flush();
        if (!ok()) return;
        pend = Ew();
        pend.kind = kind;
        pend.a = a;
        pend.b = b;
        pend.x = x;
        pend.y = y;
        pend.out0 = out;
        has_pend = true;
    }
    // vector.cxx:98-107 y = y*b + x*a;  :110-120 z = y*b + x*a
    void axpby(double a, const double *x, double b, double *y) { ew(K_AXPBY, a, b, x, nullptr, y); }
    void axpbyz(double a, const double *x, double b, const double *y, double *z) { ew(K_AXPBYZ, a, b, x, y, z); }
    void copy(double *dst, const double *src) { ew(K_COPY, 0, 0, src, nullptr, dst); }  // :73-83
    void set(double *x, double v) { ew(K_FILL, v, 0, nullptr, nullptr, x); }          // :31-38
    void scale(double *x, double a) { ew(K_SCALE, a, 0, nullptr, nullptr, x); }       // :141-146
    void mxy(double *x, double *y)  // mvops.cxx:118-150
    {
        flush();
        if (ok()) chk(R.spmv(EPI_MXY, 1, x, 0, nullptr, y));
    }
    void resid(double *x, const double *b, double *r)  // lssp_mv_amxpbyz(-1, A, x, 1, b, r), :42-78
    {
        flush();
        if (ok()) chk(R.spmv(EPI_AXPBY, -1, x, 1, b, r));
    }
    void pc(double *x, const double *rhs)
    {
        flush();
        if (ok()) chk(R.pc(x, rhs));
    }
    // m <= MAX_SLOTS dots / norms the reference evaluates back to back
    // (vector.cxx:123-139): one pass -- the pending updates with the products
    // reduced at their end -- and one host round trip.  The trace gets each
    // value at its position in the reference's call order.
    void fetchn(int m, const bool *isnorm, const double *const *xs, const double *const *ys, double *out)
    {
        int pos[MAX_SLOTS];
        for (int q = 0; q < m; q++) pos[q] = R.T();
        if (ok()) {
            Fin f = R.fin(FIN_STORE, m);
            if (R.tree && has_pend) {  // the held-back update's pass also reduces
                const double **ra[MAX_SLOTS] = {&pend.r0a, &pend.r1a, &pend.r2a, &pend.r3a};
                const double **rb[MAX_SLOTS] = {&pend.r0b, &pend.r1b, &pend.r2b, &pend.r3b};
                for (int q = 0; q < m; q++) {
                    *ra[q] = xs[q];
                    *rb[q] = ys[q];
                }
                pend.nred = m;
                flush();
                if (ok()) chk(finish_reduce(R.c, R.n, m, xs, ys, f));
            } else {
                flush();
                if (ok()) chk(reduce_dots(R.c, R.n, m, xs, ys, f));
            }
            if (ok()) chk(R.sync(0, 32));
        }
        for (int q = 0; q < m; q++) {
            out[q] = ok() ? (isnorm[q] ? sqrt(R.h(S_SUM0 + q)) : R.h(S_SUM0 + q)) : NAN;
            if (ok() && pos[q] >= 0) R.patches.push_back({pos[q], out[q]});
        }
    }
    // two back-to-back evaluations (norm: n0 / n1), one pass and one round trip
    void pair(double &o0, const double *x0, const double *y0, bool n0, double &o1, const double *x1,
              const double *y1, bool n1)
    {
        const bool nm[2] = {n0, n1};
        const double *xs[2] = {x0, x1}, *ys[2] = {y0, y1};
        double v[2];
        fetchn(2, nm, xs, ys, v);
        o0 = v[0];
        o1 = v[1];
    }
    double dot(const double *x, const double *y)  // vector.cxx:123-133
    {
        const bool nm[1] = {false};
        double v;
        fetchn(1, nm, &x, &y, &v);
        return v;
    }
    double norm(const double *x)  // :135-139
    {
        const bool nm[1] = {true};
        double v;
        fetchn(1, nm, &x, &x, &v);
        return v;
    }
};

void tol_setup(const lssp_amd_solve_params &P, double nrm2, double bnorm_rb, double &tol)
{
    // tol = nrm2*rtol; alpha = ||b||*rb; tol = max(tol, atol, alpha)  (e.g. solver-cgs.cxx:41-44)
    double tol_rel, tol_abs;
    int maxit;
    defaults(P, tol_rel, tol_abs, maxit);
    tol = nrm2 * tol_rel;
    if (tol < tol_abs) tol = tol_abs;
    if (tol < bnorm_rb) tol = bnorm_rb;
}

#define L1_DONE()                      \
    do {                               \
        K.flush();                     \
        if (!K.ok()) return K.st;      \
        *nits = iter;                  \
        *res_out = nrm2;               \
        return LSSP_AMD_OK;            \
    } while (0)

// CGS (solver-cgs.cxx:4-133); vhat aliases uhat (:25)
int cgs(Run &R, const lssp_amd_solve_params &P, double *x, const double *b, int *nits, double *res_out)
{
    L1K K(R);
    double tol_rel, tol_abs, tol;
    int maxiter, iter;
    defaults(P, tol_rel, tol_abs, maxiter);
    double *r = K.vec(), *rtld = K.vec(), *p = K.vec(), *phat = K.vec(), *q = K.vec(), *qhat = K.vec();
    double *u = K.vec(), *uhat = K.vec(), *vhat = uhat;
    double alpha = 1.0, beta, rho, rho_old = 1.0, tdot1, nrm2, ires;
    K.resid(x, b, r);
    iter = 0;
    nrm2 = ires = K.norm(r);
    if (!K.ok() || nrm2 <= tol_abs) L1_DONE();
    alpha = K.norm(b) * P.tol_rb;
    tol_setup(P, nrm2, alpha, tol);
    K.copy(rtld, r);
    K.set(q, 0);
    K.set(p, 0);
    for (iter = 1; iter <= maxiter; iter++) {
        rho = K.dot(rtld, r);
        if (!K.ok() || rho == 0.0) L1_DONE();
        beta = rho / rho_old;
        K.axpbyz(beta, q, 1, r, u);
        K.axpby(1, q, beta, p);
        K.axpby(1, u, beta, p);
        K.pc(phat, p);
        K.mxy(phat, vhat);
        tdot1 = K.dot(rtld, vhat);
        if (!K.ok() || tdot1 == 0.0) L1_DONE();
        alpha = rho / tdot1;
        K.axpbyz(-alpha, vhat, 1, u, q);
        K.axpbyz(1, u, 1, q, phat);
        K.pc(uhat, phat);
        K.axpby(alpha, uhat, 1, x);
        K.mxy(uhat, qhat);
        K.axpby(-alpha, qhat, 1, r);
        nrm2 = K.norm(r);
        if (P.verb >= 1 && R.rank == 0)
            lprint("cgs: itr: %5d, abs res: %.6e, rel res: %.6e\n", iter, nrm2, nrm2 / ires);
        if (!K.ok() || tol >= nrm2) L1_DONE();
        rho_old = rho;
    }
    L1_DONE();
}

// CR (solver-cr.cxx:3-115)
int cr(Run &R, const lssp_amd_solve_params &P, double *x, const double *b, int *nits, double *res_out)
{
    L1K K(R);
    double tol_rel, tol_abs, tol;
    int maxiter, iter;
    defaults(P, tol_rel, tol_abs, maxiter);
    double *r = K.vec(), *z = K.vec(), *p = K.vec(), *q = K.vec(), *qtld = K.vec(), *az = K.vec();
    double alpha, beta, rho, dot_rq, dot_zq, nrm2, ires;
    K.resid(x, b, r);
    nrm2 = ires = K.norm(r);
    iter = 1;
    if (!K.ok() || nrm2 <= tol_abs) L1_DONE();  // nits = iter = 1 (:31-35, :105)
    alpha = K.norm(b) * P.tol_rb;
    tol_setup(P, nrm2, alpha, tol);
    K.pc(p, r);
    K.mxy(p, q);
    K.copy(z, p);
    for (iter = 1; iter <= maxiter; iter++) {
        K.pc(qtld, q);
        rho = K.dot(qtld, q);
        if (!K.ok() || rho == 0.0) L1_DONE();
        dot_rq = K.dot(r, qtld);
        alpha = dot_rq / rho;
        K.axpby(alpha, p, 1, x);
        K.axpby(-alpha, q, 1, r);
        nrm2 = K.norm(r);
        if (P.verb >= 1 && R.rank == 0)
            lprint("cr: itr: %5d, abs res: %.6e, rel res: %.6e\n", iter, nrm2, nrm2 / ires);
        if (!K.ok() || tol >= nrm2) L1_DONE();
        K.axpby(-alpha, qtld, 1, z);
        K.mxy(z, az);
        dot_zq = K.dot(az, qtld);
        beta = -dot_zq / rho;
        K.axpby(1, z, beta, p);
        K.axpby(1, az, beta, q);
    }
    L1_DONE();
}

// CRS (solver-crs.cxx:3-109); u = uq = z, ap = q, auq = map (:20-25)
int crs(Run &R, const lssp_amd_solve_params &P, double *x, const double *b, int *nits, double *res_out)
{
    L1K K(R);
    double tol_rel, tol_abs, tol;
    int maxiter, iter;
    defaults(P, tol_rel, tol_abs, maxiter);
    double *r = K.vec(), *rtld = K.vec(), *p = K.vec(), *z = K.vec(), *q = K.vec(), *map = K.vec();
    double *u = z, *uq = z, *ap = q, *auq = map;
    double alpha, beta, rho, rho_old, tdot1, nrm2, ires;
    K.resid(x, b, r);
    nrm2 = ires = K.norm(r);
    iter = 1;
    if (!K.ok() || nrm2 <= tol_abs) L1_DONE();
    alpha = K.norm(b) * P.tol_rb;
    tol_setup(P, nrm2, alpha, tol);
    K.copy(p, r);
    K.mxy(p, rtld);
    rho_old = 1.0;
    K.set(q, 0.);
    K.set(p, 0.);
    for (iter = 1; iter <= maxiter; iter++) {
        K.pc(z, r);
        rho = K.dot(rtld, z);
        if (!K.ok() || rho == 0.0) L1_DONE();
        beta = rho / rho_old;
        K.axpbyz(beta, q, 1, z, u);
        K.axpby(1, q, beta, p);
        K.axpby(1, u, beta, p);
        K.mxy(p, ap);
        K.pc(map, ap);
        tdot1 = K.dot(rtld, map);
        if (!K.ok() || tdot1 == 0.0) L1_DONE();
        alpha = rho / tdot1;
        K.axpbyz(-alpha, map, 1, u, q);
        K.axpbyz(1, u, 1, q, uq);
        K.mxy(uq, auq);
        K.axpby(alpha, uq, 1, x);
        K.axpby(-alpha, auq, 1, r);
        nrm2 = K.norm(r);
        if (P.verb >= 1 && R.rank == 0)
            lprint("crs: itr: %5d, abs res: %.6e, rel res: %.6e\n", iter, nrm2, nrm2 / ires);
        if (!K.ok() || tol >= nrm2) L1_DONE();
        rho_old = rho;
    }
    L1_DONE();
}

// BiCRSTAB (solver-bicrstab.cxx:3-114)
int bicrstab(Run &R, const lssp_amd_solve_params &P, double *x, const double *b, int *nits, double *res_out)
{
    L1K K(R);
    double tol_rel, tol_abs, tol;
    int maxiter, iter;
    defaults(P, tol_rel, tol_abs, maxiter);
    double *rtld = K.vec(), *r = K.vec(), *s = K.vec(), *ms = K.vec(), *ams = K.vec(), *p = K.vec();
    double *ap = K.vec(), *map = K.vec(), *z = K.vec();
    double alpha, beta, omega, rho, rho_old, tdot1, tdot2, nrm2, ires;
    K.resid(x, b, r);
    nrm2 = ires = K.norm(r);
    iter = 1;
    if (!K.ok() || nrm2 <= tol_abs) L1_DONE();
    alpha = K.norm(b) * P.tol_rb;
    tol_setup(P, nrm2, alpha, tol);
    K.copy(p, r);
    K.mxy(p, rtld);
    K.pc(z, r);
    K.copy(p, z);
    rho_old = K.dot(rtld, z);
    for (iter = 1; iter <= maxiter; iter++) {
        K.mxy(p, ap);
        K.pc(map, ap);
        tdot1 = K.dot(rtld, map);
        alpha = rho_old / tdot1;
        K.axpbyz(-alpha, ap, 1, r, s);
        nrm2 = K.norm(s);
        if (!K.ok()) L1_DONE();
        if (nrm2 <= tol) {
            K.axpby(alpha, p, 1, x);
            L1_DONE();
        }
        K.axpbyz(-alpha, map, 1, z, ms);
        K.mxy(ms, ams);
        K.pair(tdot1, ams, s, false, tdot2, ams, ams, false);
        omega = tdot1 / tdot2;
        K.axpby(alpha, p, 1, x);
        K.axpby(omega, ms, 1, x);
        K.axpbyz(-omega, ams, 1, s, r);
        nrm2 = K.norm(r);
        if (P.verb >= 2 && R.rank == 0)
            lprint("bicrstab: itr: %5d, abs res: %.6e, rel res: %.6e\n", iter, nrm2, nrm2 / ires);
        if (!K.ok() || tol >= nrm2) L1_DONE();
        K.pc(z, r);
        rho = K.dot(rtld, z);
        if (!K.ok() || rho == 0.0) L1_DONE();
        beta = (rho / rho_old) * (alpha / omega);
        K.axpby(-omega, map, 1, p);
        K.axpby(1, z, beta, p);
        rho_old = rho;
    }
    L1_DONE();
}

// the (qsi, eta) pair of BiCGSafe / BiCRSafe / GPBiCG / GPBiCR
// (e.g. solver-bicgsafe.cxx:61-75): five dots, then the 2x2 solve
static void safe_coef(L1K &K, int iter, const double *y, const double *a, const double *r, double &qsi,
                      double &eta)
{
    double tdot[5], tmp;
    {  // the five dots back to back: one pass of four, then the fifth
        const bool nm[4] = {false, false, false, false};
        const double *xs[4] = {y, a, y, a}, *ys[4] = {y, r, r, y};
        K.fetchn(4, nm, xs, ys, tdot);
        tdot[4] = K.dot(a, a);
    }
    if (iter == 1) {
        qsi = tdot[1] / tdot[4];
        eta = 0.0;
    } else {
        tmp = tdot[4] * tdot[0] - tdot[3] * tdot[3];
        qsi = (tdot[0] * tdot[1] - tdot[2] * tdot[3]) / tmp;
        eta = (tdot[4] * tdot[2] - tdot[3] * tdot[1]) / tmp;
    }
}

// BiCGSafe (solver-bicgsafe.cxx:3-155)
int bicgsafe(Run &R, const lssp_amd_solve_params &P, double *x, const double *b, int *nits, double *res_out)
{
    L1K K(R);
    double tol_rel, tol_abs, tol;
    int maxiter, iter;
    defaults(P, tol_rel, tol_abs, maxiter);
    double *rtld = K.vec(), *r = K.vec(), *mr = K.vec(), *amr = K.vec(), *p = K.vec(), *ap = K.vec();
    double *t = K.vec(), *mt = K.vec(), *y = K.vec(), *u = K.vec(), *z = K.vec(), *au = K.vec();
    double alpha, beta, rho, rho_old, qsi, eta, nrm2, ires;
    K.resid(x, b, r);
    nrm2 = ires = K.norm(r);
    iter = 1;
    if (!K.ok() || nrm2 <= tol_abs) L1_DONE();
    alpha = K.norm(b) * P.tol_rb;
    tol_setup(P, nrm2, alpha, tol);
    K.copy(rtld, r);
    K.pc(mr, r);
    K.mxy(mr, amr);
    rho_old = K.dot(rtld, r);
    K.copy(ap, amr);
    K.copy(p, mr);
    beta = 0.0;
    for (iter = 1; iter <= maxiter; iter++) {
        alpha = rho_old / K.dot(rtld, ap);
        safe_coef(K, iter, y, amr, r, qsi, eta);
        K.copy(t, y);
        K.scale(t, eta);
        K.axpby(qsi, ap, 1, t);
        K.pc(mt, t);
        K.axpby(1, mt, eta * beta, u);
        K.mxy(u, au);
        K.scale(z, eta);
        K.axpby(qsi, mr, 1, z);
        K.axpby(-alpha, u, 1, z);
        K.scale(y, eta);
        K.axpby(qsi, amr, 1, y);
        K.axpby(-alpha, au, 1, y);
        K.axpby(alpha, p, 1, x);
        K.axpby(1, z, 1, x);
        K.axpby(-alpha, ap, 1, r);
        K.axpby(-1, y, 1.0, r);
        nrm2 = K.norm(r);
        if (P.verb >= 1 && R.rank == 0)
            lprint("bicgsafe: itr: %5d, abs res: %.6e, rel res: %.6e\n", iter, nrm2, nrm2 / ires);
        if (!K.ok() || tol >= nrm2) L1_DONE();
        rho = K.dot(rtld, r);
        if (!K.ok() || rho == 0.0) L1_DONE();
        beta = (rho / rho_old) * (alpha / qsi);
        K.pc(mr, r);
        K.mxy(mr, amr);
        K.axpby(-1, u, 1.0, p);
        K.axpby(1, mr, beta, p);
        K.axpby(-1, au, 1.0, ap);
        K.axpby(1, amr, beta, ap);
        rho_old = rho;
    }
    L1_DONE();
}

// BiCRSafe (solver-bicrsafe.cxx:3-151)
int bicrsafe(Run &R, const lssp_amd_solve_params &P, double *x, const double *b, int *nits, double *res_out)
{
    L1K K(R);
    double tol_rel, tol_abs, tol;
    int maxiter, iter;
    defaults(P, tol_rel, tol_abs, maxiter);
    double *rtld = K.vec(), *r = K.vec(), *mr = K.vec(), *amr = K.vec(), *p = K.vec(), *ap = K.vec();
    double *map = K.vec(), *my = K.vec(), *y = K.vec(), *u = K.vec(), *z = K.vec(), *au = K.vec();
    double *artld = K.vec();
    double alpha, beta, rho, rho_old, qsi, eta, nrm2, ires;
    K.resid(x, b, r);
    nrm2 = ires = K.norm(r);
    iter = 1;
    if (!K.ok() || nrm2 <= tol_abs) L1_DONE();
    alpha = K.norm(b) * P.tol_rb;
    tol_setup(P, nrm2, alpha, tol);
    K.copy(rtld, r);
    K.mxy(rtld, artld);
    K.pc(mr, r);
    K.mxy(mr, amr);
    rho_old = K.dot(rtld, amr);
    K.copy(ap, amr);
    K.copy(p, mr);
    beta = 0.0;
    for (iter = 1; iter <= maxiter; iter++) {
        K.pc(map, ap);
        alpha = rho_old / K.dot(artld, map);
        safe_coef(K, iter, y, amr, r, qsi, eta);
        K.scale(u, eta * beta);
        K.axpby(qsi, map, 1, u);
        K.axpby(eta, my, 1, u);
        K.mxy(u, au);
        K.scale(z, eta);
        K.axpby(qsi, mr, 1, z);
        K.axpby(-alpha, u, 1, z);
        K.scale(y, eta);
        K.axpby(qsi, amr, 1, y);
        K.axpby(-alpha, au, 1, y);
        K.pc(my, y);
        K.axpby(alpha, p, 1, x);
        K.axpby(1, z, 1, x);
        K.axpby(-alpha, ap, 1, r);
        K.axpby(-1, y, 1, r);
        nrm2 = K.norm(r);
        if (P.verb >= 2 && R.rank == 0)
            lprint("bicrsafe: itr: %5d, abs res: %.6e, rel res: %.6e\n", iter, nrm2, nrm2 / ires);
        if (!K.ok() || tol >= nrm2) L1_DONE();
        K.axpby(-alpha, map, 1, mr);
        K.axpby(-1, my, 1, mr);
        K.mxy(mr, amr);
        rho = K.dot(rtld, amr);
        if (!K.ok() || rho == 0.0) L1_DONE();
        beta = (rho / rho_old) * (alpha / qsi);
        K.axpby(-1, u, 1., p);
        K.axpby(1, mr, beta, p);
        K.axpby(-1, au, 1.0, ap);
        K.axpby(1, amr, beta, ap);
        rho_old = rho;
    }
    L1_DONE();
}

// GPBiCG (solver-gpbicg.cxx:3-163) and GPBiCR (solver-gpbicr.cxx:3-164): the
// same recurrence; GPBiCR shadows with A r0 and tests <rtld, M^-1 A p> and
// <rtld, M^-1 r> (gpbicr.cxx:49-54, :62, :129)
int gpbi(Run &R, const lssp_amd_solve_params &P, double *x, const double *b, int *nits, double *res_out, bool cr_)
{
    L1K K(R);
    double tol_rel, tol_abs, tol;
    int maxiter, iter;
    defaults(P, tol_rel, tol_abs, maxiter);
    double *rtld = K.vec(), *r = K.vec(), *mr = K.vec(), *p = K.vec(), *ap = K.vec(), *map = K.vec();
    double *t = K.vec(), *mt = K.vec(), *amt = K.vec(), *u = K.vec(), *y = K.vec(), *w = K.vec();
    double *z = K.vec(), *mt_old = K.vec();
    double alpha, beta, rho, rho_old, qsi, eta, tdot0, nrm2, ires;
    const char *name = cr_ ? "gpbicr" : "gpbicg";
    K.resid(x, b, r);
    nrm2 = ires = K.norm(r);
    iter = 1;
    if (!K.ok()) L1_DONE();
    if (nrm2 <= tol_abs) {
        iter = 0;
        L1_DONE();
    }
    alpha = K.norm(b) * P.tol_rb;
    tol_setup(P, nrm2, alpha, tol);
    if (cr_) {
        K.copy(p, r);
        K.mxy(p, rtld);
        K.pc(p, r);
        rho_old = K.dot(rtld, p);
    } else {
        K.copy(rtld, r);
        K.pc(p, r);
        rho_old = K.dot(rtld, r);
    }
    K.set(t, 0.);
    K.set(w, 0.);
    beta = 0.0;
    for (iter = 1; iter <= maxiter; iter++) {
        K.mxy(p, ap);
        K.pc(map, ap);
        tdot0 = K.dot(rtld, cr_ ? map : ap);
        if (!K.ok() || tdot0 == 0.0) L1_DONE();
        alpha = rho_old / tdot0;
        K.axpbyz(-1, w, 1, ap, y);
        K.axpby(1, t, alpha, y);
        K.axpby(-1, r, 1, y);
        K.axpbyz(-alpha, ap, 1, r, t);
        nrm2 = K.norm(t);
        if (P.verb >= 1 && R.rank == 0)
            lprint("%s: itr: %5d, abs res: %.6e, rel res: %.6e\n", name, iter, nrm2, nrm2 / ires);
        if (!K.ok()) L1_DONE();
        if (nrm2 <= tol) {
            K.axpby(alpha, p, 1, x);
            L1_DONE();
        }
        K.axpbyz(-alpha, map, 1, mr, mt);
        K.mxy(mt, amt);
        safe_coef(K, iter, y, amt, t, qsi, eta);
        K.axpby(1., mt_old, beta, u);
        K.axpby(-1, mr, 1, u);
        K.scale(u, eta);
        K.axpby(qsi, map, 1, u);
        K.scale(z, eta);
        K.axpby(qsi, mr, 1, z);
        K.axpby(-alpha, u, 1, z);
        K.axpby(alpha, p, 1, x);
        K.axpby(1, z, 1., x);
        K.axpbyz(-qsi, amt, 1, t, r);
        K.axpby(-eta, y, 1, r);
        nrm2 = K.norm(r);
        if (P.verb >= 1 && R.rank == 0)
            lprint("%s: itr: %5d, abs res: %.6e, rel res: %.6e\n", name, iter, nrm2, nrm2 / ires);
        if (!K.ok() || tol >= nrm2) L1_DONE();
        K.pc(mr, r);
        rho = K.dot(rtld, cr_ ? mr : r);
        if (!K.ok() || rho == 0.0) L1_DONE();
        beta = (rho / rho_old) * (alpha / qsi);
        K.axpbyz(beta, ap, 1, amt, w);
        K.axpby(-1, u, 1, p);
        K.axpby(1., mr, beta, p);
        K.copy(mt_old, mt);
        rho_old = rho;
    }
    L1_DONE();
}

// QMRCGSTAB (solver-qmrcgstab.cxx:10-186)
int qmrcgstab(Run &R, const lssp_amd_solve_params &P, double *xk, const double *bg, int *nits, double *res_out)
{
    const double t_start = wall_time();  // the reference driver's lssp_get_time() ("total time")
    L1K K(R);
    double tol_rel, tol_abs, tol_rb = P.tol_rb;
    int itr_max, itr_out;
    defaults(P, tol_rel, tol_abs, itr_max);
    if (P.verb >= 2 && R.rank == 0) {
        lprint("qmrcgstab: maximal iteration: %d\n", itr_max);
        lprint("qmrcgstab: tolerance abs: %g\n", tol_abs);
        lprint("qmrcgstab: tolerance rel: %g\n", tol_rel);
        lprint("qmrcgstab: tolerance rbn: %g\n", tol_rb);
    }
    double *rk = K.vec(), *r = K.vec(), *br0 = K.vec(), *pk = K.vec(), *vk = K.vec(), *sk = K.vec();
    double *dk = K.vec(), *tk = K.vec(), *bdk = K.vec(), *bxk = K.vec();
    double rho = 1, prho, alpha = 1, beta, omega = 1, theta = 0., btheta, b_eta, eta = 0., tau, btau;
    double residual, c, ires, rerror, tol;
    const double b_norm = K.norm(bg);
    tol_rb *= b_norm;
    K.resid(xk, bg, tk);
    residual = K.norm(tk);
    if (!K.ok()) return K.st;
    if (residual <= tol_abs) {
        *nits = 0;
        *res_out = residual;
        return LSSP_AMD_OK;
    }
    tol = residual * tol_rel;
    if (tol < tol_abs) tol = tol_abs;
    if (tol < tol_rb) tol = tol_rb;
    tol = tol / residual;
    K.pc(rk, tk);
    K.copy(br0, rk);
    K.set(pk, 0);
    K.set(dk, 0);
    K.set(vk, 0);
    tau = ires = K.norm(rk);
    prho = rho;
    for (itr_out = 0; itr_out < itr_max; itr_out++) {
        rho = K.dot(br0, rk);
        beta = rho * alpha / prho / omega;
        prho = rho;
        K.axpbyz(1, pk, -omega, vk, r);
        K.axpbyz(beta, r, 1, rk, pk);
        K.mxy(pk, r);
        K.pc(vk, r);
        alpha = rho / K.dot(br0, vk);
        K.axpbyz(-alpha, vk, 1, rk, sk);
        btheta = K.norm(sk) / tau;
        c = 1 / sqrt(1. + btheta * btheta);
        btau = tau * btheta * c;
        b_eta = c * c * alpha;
        K.axpbyz(1., pk, theta * theta * eta / alpha, dk, bdk);
        K.axpbyz(1, xk, b_eta, bdk, bxk);
        K.mxy(sk, r);
        K.pc(tk, r);
        {
            // :146 -- operand evaluation order as g++ -O2 built it (the golden traces)
            double num, den;
            K.pair(num, sk, tk, false, den, tk, tk, false);
            omega = num / den;
        }
        K.axpbyz(1., sk, -omega, tk, rk);
        theta = K.norm(rk) / btau;
        c = 1. / sqrt(1. + theta * theta);
        tau = btau * theta * c;
        eta = c * c * omega;
        K.axpbyz(1, sk, btheta * btheta * b_eta / omega, bdk, dk);
        K.axpbyz(1, bxk, eta, dk, xk);
        rerror = K.norm(rk) / ires;
        if (!K.ok()) return K.st;
        if (P.verb >= 1 && R.rank == 0) lprint("qmrcgstab: itr: %4d, rel res: %.6e\n", itr_out, rerror);
        if (rerror <= tol) {
            K.resid(xk, bg, tk);
            residual = K.norm(tk);
            break;
        }
    }
    if (!K.ok()) return K.st;
    if (itr_out < itr_max) itr_out += 1;
    if (P.verb >= 2 && R.rank == 0) {  // solver-qmrcgstab.cxx:178-183
        lprint("qmrcgstab: total iteration: %d\n", itr_out);
        lprint("qmrcgstab: total time: %g\n", wall_time() - t_start);
        lprint("qmrcgstab: absolute error (residual): %g\n", residual);
    }
    *nits = itr_out;
    *res_out = residual;
    return LSSP_AMD_OK;
}

// TFQMR (solver-tfqmr.cxx:3-149)
int tfqmr(Run &R, const lssp_amd_solve_params &P, double *x, const double *b, int *nits, double *res_out)
{
    L1K K(R);
    double tol_rel, tol_abs, tol;
    int maxiter, iter;
    defaults(P, tol_rel, tol_abs, maxiter);
    double *r = K.vec(), *rtld = K.vec(), *u = K.vec(), *p = K.vec(), *d = K.vec(), *t = K.vec();
    double *t1 = K.vec(), *q = K.vec(), *v = K.vec();
    double alpha, beta, rho, rhoold, s, tau, theta, eta, c, w, wold, ww, nrm2, ires;
    K.resid(x, b, r);
    nrm2 = ires = K.norm(r);
    iter = 1;
    if (!K.ok()) L1_DONE();
    if (nrm2 <= tol_abs) {
        iter = 0;
        L1_DONE();
    }
    alpha = K.norm(b) * P.tol_rb;
    tol_setup(P, nrm2, alpha, tol);
    K.copy(rtld, r);
    K.copy(p, r);
    K.copy(u, r);
    K.set(d, 0.);
    K.pc(t, p);
    K.mxy(t, v);
    K.pair(rhoold, r, rtld, false, tau, r, r, true);
    wold = tau;
    theta = 0.0;
    eta = 0.0;
    while (iter <= maxiter) {
        s = K.dot(v, rtld);
        if (!K.ok() || fabs(s) == 0.0) L1_DONE();
        alpha = rhoold / s;
        K.axpbyz(-alpha, v, 1, u, q);
        K.axpbyz(1, u, 1., q, t);
        K.pc(t1, t);
        K.mxy(t1, v);
        K.axpby(-alpha, v, 1, r);
        w = K.norm(r);
        for (int m = 0; m < 2; m++) {
            if (m == 0) {
                ww = sqrt(w * wold);
                K.axpby(1, u, theta * theta * eta / alpha, d);
            } else {
                ww = w;
                K.axpby(1, q, theta * theta * eta / alpha, d);
            }
            theta = ww / tau;
            c = 1.0 / sqrt(1.0 + theta * theta);
            eta = c * c * alpha;
            tau = tau * theta * c;
            K.pc(t1, d);
            K.axpby(eta, t1, 1, x);
            nrm2 = tau * sqrt(1.0 + m);
            if (P.verb >= 1 && R.rank == 0)
                lprint("tfqmr: itr: %5d, abs res: %.6e, rel res: %.6e\n", iter, nrm2, nrm2 / ires);
            if (!K.ok() || tol >= nrm2) L1_DONE();
        }
        rho = K.dot(r, rtld);
        if (!K.ok() || fabs(rho) == 0.0) L1_DONE();
        beta = rho / rhoold;
        K.axpbyz(beta, q, 1, r, u);
        K.axpby(1, q, beta, p);
        K.axpby(1, u, beta, p);
        K.pc(t1, p);
        K.mxy(t1, v);
        rhoold = rho;
        wold = w;
        iter++;
    }
    L1_DONE();
}

// ORTHOMIN(k), k = restart (solver-orthomin.cxx:12-180)
int orthomin(Run &R, const lssp_amd_solve_params &P, double *x, const double *rhs, int *nits, double *res_out)
{
    const double t_start = wall_time();  // the reference driver's lssp_get_time() ("total time")
    L1K K(R);
    double tol_rel, tol_abs, tol_rb = P.tol_rb < 0 ? DEF_TOL : P.tol_rb;
    int itr_max, itr_out, i, j;
    defaults(P, tol_rel, tol_abs, itr_max);
    int k = P.restart < 0 ? DEF_RESTART : P.restart;
    if (k == 0) return LSSP_AMD_EINVAL;  // the reference divides by it (:102)
    if (P.verb >= 2 && R.rank == 0) {
        lprint("orthomin: k parameter m: %d\n", k);
        lprint("orthomin: maximal iteration: %d\n", itr_max);
        lprint("orthomin: tolerance abs: %g\n", tol_abs);
        lprint("orthomin: tolerance rel: %g\n", tol_rel);
        lprint("orthomin: tolerance rbn: %g\n", tol_rb);
    }
    double *z = K.vec(), *r = K.vec(), *s = K.vec(), *sd = K.vec();
    std::vector<double *> p(k), q(k);
    std::vector<double> b_j(k), c_j(k);
    for (i = 0; i < k; i++) {
        p[i] = K.vec();
        q[i] = K.vec();
    }
    double tol = -1, err_rel = 0, beta, a_j;
    K.resid(x, rhs, z);
    K.set(r, 0.);
    K.pc(r, z);
    K.copy(p[0], r);
    K.copy(sd, r);
    const double b_norm = K.norm(rhs);
    tol_rb *= b_norm;
    beta = K.norm(z);
    if (!K.ok()) return K.st;
    if (beta <= tol_abs) {
        *nits = 0;
        *res_out = beta;
        return LSSP_AMD_OK;
    }
    err_rel = beta;
    tol = tol_rel * err_rel;
    if (tol < tol_abs) tol = tol_abs;
    if (tol < tol_rb) tol = tol_rb;
    for (itr_out = 0; itr_out < itr_max; itr_out++) {
        K.mxy(sd, s);
        j = itr_out % k;
        K.set(q[j], 0.);
        K.pc(q[j], s);
        K.pair(a_j, r, q[j], false, c_j[j], q[j], q[j], false);
        if (!K.ok()) return K.st;
        if (fabs(c_j[j]) <= BREAKDOWN) break;
        a_j = a_j / c_j[j];
        K.axpby(a_j, p[j], 1, x);
        K.axpby(-a_j, q[j], 1, r);
        K.copy(sd, r);
        K.mxy(r, s);
        K.set(z, 0.);
        K.pc(z, s);
        const int ni = itr_out >= k - 1 ? k : itr_out + 1;  // :120-136
        for (i = 0; i < ni; i++) {
            beta = K.dot(z, q[i]);
            b_j[i] = -beta / c_j[i];
            K.axpby(b_j[i], p[i], 1, sd);
        }
        j = (itr_out + 1) % k;
        K.copy(p[j], sd);
        K.resid(x, rhs, z);
        beta = K.norm(z);
        if (!K.ok()) return K.st;
        if (P.verb >= 1 && R.rank == 0)
            lprint("orthomin: itr: %5d, abs res: %.6e, rel res: %.6e, rbn: %.6e\n", itr_out, beta,
                   (err_rel == 0 ? 0 : beta / err_rel), (b_norm == 0 ? 0 : beta / b_norm));
        if (beta <= tol) break;
    }
    if (itr_out < itr_max) itr_out += 1;
    if (P.verb >= 2 && R.rank == 0) {
        lprint("orthomin: total iteration: %d\n", itr_out);
        lprint("orthomin: total time: %g\n", wall_time() - t_start);
    }
    *nits = itr_out;
    *res_out = beta;
    return LSSP_AMD_OK;
}

// BiCGSTAB(l) (solver-bicgstabl.cxx:4-217).  x accumulates the right-
// preconditioned iterate; on every converged / breakdown exit the reference
// maps it back as x = M^-1 x + x0 (:84-86, :131-133, :190-192) -- not when
// the outer loop runs out of iterations (iter is tested only there, :73).
int bicgstabl(Run &R, const lssp_amd_solve_params &P, double *x, const double *b, int *nits, double *res_out)
{
    L1K K(R);
    double tol_rel, tol_abs, tol_rb = P.tol_rb < 0 ? DEF_TOL : P.tol_rb, tol = 0;
    int maxiter, iter, i, j;
    defaults(P, tol_rel, tol_abs, maxiter);
    const int l = P.bgsl <= 0 ? 4 : P.bgsl;  // :27-29; LSSP_BGSL = 4 (lssp.cxx:7)
    const int zd = l + 1;
    double *rtld = K.vec(), *xp = K.vec(), *bp = K.vec(), *t = K.vec();
    std::vector<double *> r(l + 1), u(l + 1);
    for (i = 0; i <= l; i++) r[i] = K.vec();
    for (i = 0; i <= l; i++) u[i] = K.vec();
    std::vector<double> tau(zd * zd, 0.), gamma(zd, 0.), gamma1(zd, 0.), gamma2(zd, 0.), sigma(zd, 0.);
    double alpha, beta, omega, rho0, rho1, nu, nrm2, ires;
    auto unprecondition = [&]() {  // pc.solve(t, x); copy(x, t); x = x + xp
        K.pc(t, x);
        K.copy(x, t);
        K.axpby(1, xp, 1, x);
    };
    K.resid(x, b, r[0]);
    K.copy(rtld, r[0]);
    K.copy(bp, r[0]);
    K.copy(xp, x);
    K.set(u[0], 0.);
    iter = 0;
    nrm2 = ires = K.norm(r[0]);
    if (!K.ok() || nrm2 <= tol_abs) L1_DONE();
    tol = nrm2 * tol_rel;
    alpha = K.norm(b) * tol_rb;
    if (tol < tol_abs) tol = tol_abs;
    if (tol < alpha) tol = alpha;
    alpha = 0.0;
    omega = 1.0;
    rho0 = 1.0;
    while (iter <= maxiter) {
        rho0 = -omega * rho0;
        for (j = 0; j < l; j++) {
            iter++;
            rho1 = K.dot(rtld, r[j]);
            if (!K.ok()) return K.st;
            if (rho1 == 0.0) {
                unprecondition();
                L1_DONE();
            }
            beta = alpha * (rho1 / rho0);
            rho0 = rho1;
            for (i = 0; i <= j; i++) K.axpby(1, r[i], -beta, u[i]);
            K.pc(t, u[j]);
            K.mxy(t, u[j + 1]);
            nu = K.dot(rtld, u[j + 1]);
            if (!K.ok()) return K.st;
            if (fabs(nu) == 0.0) {
                unprecondition();
                L1_DONE();
            }
            alpha = rho1 / nu;
            K.axpby(alpha, u[0], 1, x);
            for (i = 0; i <= j; i++) K.axpby(-alpha, u[i + 1], 1, r[i]);
            nrm2 = K.norm(r[0]);
            if (!K.ok()) return K.st;
            if (P.verb >= 1 && R.rank == 0)
                lprint("bicgstabl: itr: %5d, abs res: %.6e, rel res: %.6e\n", iter, nrm2, nrm2 / ires);
            if (nrm2 <= tol) {
                unprecondition();
                L1_DONE();
            }
            K.pc(t, r[j]);
            K.mxy(t, r[j + 1]);
        }
        // MR part (:143-171): modified Gram-Schmidt on r[1..l], then the small triangular solves
        for (j = 1; j <= l; j++) {
            for (i = 1; i <= j - 1; i++) {
                nu = K.dot(r[j], r[i]);
                nu = nu / sigma[i];
                tau[i * zd + j] = nu;
                K.axpby(-nu, r[i], 1, r[j]);
            }
            K.pair(sigma[j], r[j], r[j], false, nu, r[0], r[j], false);
            gamma1[j] = nu / sigma[j];
        }
        if (!K.ok()) return K.st;
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
        // UPDATE (:174-182)
        K.axpby(gamma[1], r[0], 1, x);
        K.axpby(-gamma1[l], r[l], 1, r[0]);
        K.axpby(-gamma[l], u[l], 1, u[0]);
        for (j = 1; j <= l - 1; j++) {
            K.axpby(-gamma[j], u[j], 1, u[0]);
            K.axpby(gamma2[j], r[j], 1, x);
            K.axpby(-gamma1[j], r[j], 1, r[0]);
        }
        nrm2 = K.norm(r[0]);
        if (!K.ok()) return K.st;
        if (P.verb >= 1 && R.rank == 0)
            lprint("bicgstabl: itr: %5d, abs res: %.6e, rel res: %.6e\n", iter, nrm2, nrm2 / ires);
        if (nrm2 < tol) {
            unprecondition();
            L1_DONE();
        }
    }
    L1_DONE();
}

// solver-idrs.cxx:23-84: solve the s x s system M c = m (read column-major),
// LU without pivoting; the s = 1 and s = 2 cases are the reference's own
// unrolled forms.
static void idrs_array_solve(int n, const double *a, const double *b, double *x, double *w)
{
    int i, j, k;
    double t;
    for (i = 0; i < n * n; i++) w[i] = a[i];
    switch (n) {
    case 1: x[0] = b[0] / w[0]; break;
    case 2:
        w[0] = 1.0 / w[0];
        w[1] *= w[0];
        w[3] -= w[1] * w[2];
        w[3] = 1.0 / w[3];
        x[0] = b[0];
        x[1] = b[1] - w[1] * x[0];
        x[1] *= w[3];
        x[0] -= w[2] * x[1];
        x[0] *= w[0];
        break;
    default:
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
        break;
    }
}

// IDR(s) (solver-idrs.cxx:86-283).  The shadow space P is srand(0); rand() /
// RAND_MAX over the GLOBAL vector, k-major (:139-144) -- drawn here from a
// private glibc random_r state seeded the same way (so the caller's rand()
// stream is left alone), each rank keeping its own rows -- then orthonormalised
// with idrs_orth (:4-21).  The inline update loops
//   dX[o][i] = om*av[i] - sum_j dX[j][i]*c[j]   (:198-205, :219-226)
//   dR[o][i] = -om*t[i] - sum_j dR[j][i]*c[j]   (:207-214)
// become one y = x*a pass and s axpby passes (y*1 + x*(-c) is y - x*c
// bitwise) into a spare vector that then takes the place of dX[o] / dR[o].
int idrs(Run &R, const lssp_amd_solve_params &P, double *x, const double *b, int *nits, double *res_out)
{
    L1K K(R);
    double tol_rel, tol_abs, tol_rb = P.tol_rb < 0 ? DEF_TOL : P.tol_rb, tol = 0;
    int maxiter, iter, i, j, k, oldest;
    defaults(P, tol_rel, tol_abs, maxiter);
    const int s = P.idrs <= 0 ? 4 : P.idrs;  // :100-101; LSSP_IDRS = 4 (lssp.cxx:8)
    double *r = K.vec(), *t = K.vec(), *v = K.vec(), *av = K.vec(), *spare = K.vec();
    std::vector<double *> dX(s), dR(s), Pv(s);
    for (i = 0; i < s; i++) {
        dX[i] = K.vec();
        dR[i] = K.vec();
        Pv[i] = K.vec();
    }
    std::vector<double> m(s), c(s), M(s * s), MM(s * s);
    double om = 0, h, nrm2, ires;
    iter = 0;
    K.resid(x, b, r);
    nrm2 = ires = K.norm(r);
    if (!K.ok() || nrm2 <= tol_abs) L1_DONE();
    tol = nrm2 * tol_rel;
    h = K.norm(b) * tol_rb;
    if (tol < tol_abs) tol = tol_abs;
    if (tol < h) tol = h;
    if (!K.ok()) return K.st;
    {
        const long n = R.n, ng = R.A->n_global > 0 ? R.A->n_global : R.n, r0 = R.A->row0;
        std::vector<double> hp(n);
        struct random_data rd;
        char state[128];
        memset(&rd, 0, sizeof(rd));
        memset(state, 0, sizeof(state));
        initstate_r(0, state, sizeof(state), &rd);  // == srand(0) on glibc's default TYPE_3 state
        for (k = 0; k < s; k++) {
            for (long q = 0; q < ng; q++) {
                int32_t v32;
                random_r(&rd, &v32);
                if (q >= r0 && q < r0 + n) hp[q - r0] = (v32 * 1.) / (1. * RAND_MAX);
            }
            K.chk(hipMemcpyAsync(Pv[k], hp.data(), sizeof(double) * n, hipMemcpyHostToDevice, R.c->stream) ==
                          hipSuccess ? LSSP_AMD_OK : LSSP_AMD_EHIP);
            K.chk(hipStreamSynchronize(R.c->stream) == hipSuccess ? LSSP_AMD_OK : LSSP_AMD_EHIP);
        }
    }
    for (j = 0; j < s; j++) {  // idrs_orth (:4-21)
        double rr = K.norm(Pv[j]);
        rr = 1.0 / rr;
        K.scale(Pv[j], rr);
        for (i = j + 1; i < s; i++) {
            const double d = K.dot(Pv[j], Pv[i]);
            K.axpby(-d, Pv[j], 1, Pv[i]);
        }
    }
    for (k = 0; k < s; k++) {
        K.pc(dX[k], r);
        K.mxy(dX[k], dR[k]);
        h = K.dot(dR[k], dR[k]);
        om = K.dot(dR[k], r);
        om = om / h;
        K.scale(dX[k], om);
        K.scale(dR[k], -om);
        K.axpby(1, dX[k], 1, x);
        K.axpby(1, dR[k], 1, r);
        nrm2 = K.norm(r);
        if (!K.ok()) return K.st;
        if (tol >= nrm2) {
            iter = k + 1;
            L1_DONE();
        }
        for (i = 0; i < s; i++) M[k * s + i] = K.dot(Pv[i], dR[k]);
    }
    iter = s;
    oldest = 0;
    for (i = 0; i < s; i++) m[i] = K.dot(Pv[i], r);
    // dst = a*src - sum_j V[j]*c[j], written to the spare vector, which then replaces V[oldest]
    auto combine = [&](double a, const double *src, std::vector<double *> &V) {
        K.ew(K_AXY, a, 0, src, nullptr, spare);
        for (int q = 0; q < s; q++) K.axpby(-c[q], V[q], 1, spare);
        std::swap(spare, V[oldest]);
    };
    while (iter <= maxiter) {
        if (!K.ok()) return K.st;
        idrs_array_solve(s, M.data(), m.data(), c.data(), MM.data());
        K.copy(v, r);
        for (j = 0; j < s; j++) K.axpby(-c[j], dR[j], 1, v);
        if ((iter % (s + 1)) == s) {
            K.pc(av, v);
            K.mxy(av, t);
            h = K.dot(t, t);
            om = K.dot(t, v);
            om = om / h;
            combine(om, av, dX);
            combine(-om, t, dR);
        } else {
            K.pc(av, v);
            combine(om, av, dX);
            K.mxy(dX[oldest], dR[oldest]);
            K.scale(dR[oldest], -1.);
        }
        K.axpby(1, dR[oldest], 1, r);
        K.axpby(1, dX[oldest], 1, x);
        iter++;
        nrm2 = K.norm(r);
        if (!K.ok()) return K.st;
        if (P.verb >= 1 && R.rank == 0)
            lprint("idrs: itr: %5d, abs res: %.6e, rel res: %.6e\n", iter, nrm2, nrm2 / ires);
        if (tol >= nrm2) L1_DONE();
        for (i = 0; i < s; i++) {
            h = K.dot(Pv[i], dR[oldest]);
            m[i] += h;
            M[oldest * s + i] = h;
        }
        oldest++;
        if (oldest == s) oldest = 0;
    }
    L1_DONE();
}

}  // namespace
}  // namespace lssp_amd

using namespace lssp_amd;

extern "C" int lssp_amd_solve(lssp_amd_ctx *c, const lssp_amd_mat *A, const lssp_amd_ilu *M,
                              const lssp_amd_solve_params *prm, double *x, const double *b, int *nits,
                              double *residual, double *trace, int trace_cap, int *trace_len)
{
    if (!c) return LSSP_AMD_EINVAL;
    LSSP_HIP(hipSetDevice(c->device));  // before the agreement below: its scratch and stream are this device's
    // a rank-local argument error still joins the agreement (as -1), so no peer
    // is left waiting in it
    const bool bad_args = !A || !prm || !x || !b || A->nrows != A->ncols - A->nhalo;  // square (lssp.cxx:152)
    // M: the rank's own rows (a block-Jacobi block on P ranks), or on P ranks
    // the factors of the whole matrix (the reference's global ILU)
    const bool gpc = !bad_args && M && c->nranks > 1 && M->n == A->n_global && M->n != A->nrows;
    const bool bad_m = bad_args || (M && M->n != A->nrows && !gpc);
    if (c->nranks > 1) {
        // every rank must take the same preconditioner path (none / its own block /
        // the global factors): the global path all-gathers in every apply, so a
        // mixed choice would leave some ranks waiting there.  Agreed first, so a
        // mismatch fails every rank with EINVAL instead of hanging the job.
        std::vector<int> modes;
        LSSP_TRY(comm_gather_int(c, bad_m ? -1 : !M ? 0 : gpc ? 2 : 1, modes));
        for (int m : modes)
            if (m < 0 || m != modes[0]) return LSSP_AMD_EINVAL;
    }
    if (bad_m) return LSSP_AMD_EINVAL;
    Run R;
    R.c = c;
    R.A = A;
    R.M = M;
    if (M) M->line.lstream_of = nullptr;
    R.gpc = gpc;
    R.n = A->nrows;
    R.nx = (long)A->nrows + A->nhalo;
    R.tree = c->reduce_mode == LSSP_AMD_REDUCE_TREE;
    R.want_trace = trace && trace_cap > 0;
    R.tcap = R.want_trace ? trace_cap : 0;
    R.rank = c->rank;
    if (R.want_trace && c->trace_cap < trace_cap) {
        LSSP_HIP(hipStreamSynchronize(c->stream));
        if (c->d_trace) LSSP_HIP(hipFree(c->d_trace));
        LSSP_HIP(hipMalloc(&c->d_trace, sizeof(double) * trace_cap));
        c->trace_cap = trace_cap;
    }
    double *saved_trace = c->d_trace;
    if (!R.want_trace) c->d_trace = nullptr;
    LSSP_HIP(hipMemsetAsync(c->d_scal, 0, sizeof(double) * NSCAL, c->stream));
    int it = 0, st;
    double res = 0;
    switch (prm->solver) {
    case LSSP_AMD_BICGSTAB: st = bicgstab(R, *prm, x, b, &it, &res); break;
    case LSSP_AMD_CG: st = cg(R, *prm, x, b, &it, &res); break;
    case LSSP_AMD_GMRES: st = gmres(R, *prm, x, b, &it, &res); break;
    case LSSP_AMD_RGMRES: st = gmres_r(R, *prm, x, b, &it, &res); break;
    case LSSP_AMD_LGMRES: st = lgmres(R, *prm, x, b, &it, &res); break;
    case LSSP_AMD_BICGSAFE: st = bicgsafe(R, *prm, x, b, &it, &res); break;
    case LSSP_AMD_CGS: st = cgs(R, *prm, x, b, &it, &res); break;
    case LSSP_AMD_GPBICG: st = gpbi(R, *prm, x, b, &it, &res, false); break;
    case LSSP_AMD_CR: st = cr(R, *prm, x, b, &it, &res); break;
    case LSSP_AMD_CRS: st = crs(R, *prm, x, b, &it, &res); break;
    case LSSP_AMD_BICRSTAB: st = bicrstab(R, *prm, x, b, &it, &res); break;
    case LSSP_AMD_BICRSAFE: st = bicrsafe(R, *prm, x, b, &it, &res); break;
    case LSSP_AMD_GPBICR: st = gpbi(R, *prm, x, b, &it, &res, true); break;
    case LSSP_AMD_QMRCGSTAB: st = qmrcgstab(R, *prm, x, b, &it, &res); break;
    case LSSP_AMD_TFQMR: st = tfqmr(R, *prm, x, b, &it, &res); break;
    case LSSP_AMD_ORTHOMIN: st = orthomin(R, *prm, x, b, &it, &res); break;
    case LSSP_AMD_BICGSTABL: st = bicgstabl(R, *prm, x, b, &it, &res); break;
    case LSSP_AMD_IDRS: st = idrs(R, *prm, x, b, &it, &res); break;
    default: st = LSSP_AMD_EUNSUPPORTED;
    }
    c->d_trace = saved_trace;
    if (st != LSSP_AMD_OK) return st;
    LSSP_HIP(hipStreamSynchronize(c->stream));
    if (nits) *nits = it;
    if (residual) *residual = res;
    if (R.want_trace) {
        long len = std::min<long>(R.tl, trace_cap);
        if (len > 0)
            LSSP_HIP(hipMemcpy(trace, c->d_trace, sizeof(double) * len, hipMemcpyDeviceToHost));
        for (auto &pq : R.patches)
            if (pq.first < trace_cap) trace[pq.first] = pq.second;
    }
    if (trace_len) *trace_len = (int)R.tl;
    return LSSP_AMD_OK;
}
