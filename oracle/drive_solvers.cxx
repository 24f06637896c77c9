// drive_solvers.cxx -- TEST INFRASTRUCTURE (the drop-in check for every driver).
//
// An exam.cxx-style caller of the reference's public API (example/exam.cxx:
// 61-127 call sequence: lssp_solver_create -> set_* -> lssp_solver_assemble ->
// lssp_solver_solve), parameterised by solver, PC and grid, so the same
// program can be linked twice (oracle/Makefile `exam`):
//   _ref/drive_ref  against the reference alone (the checker);
//   _ref/drive_amd  with integration/amd_backend.cxx wrapping the drivers onto
//                   lssp_amd (tests/test_gpu_integration.py).
// It prints the iteration count, the residual and digests of x in %.17e, so
// the two binaries' outputs can be compared as strings.
//
// usage: drive_solvers SOLVER PC LEVEL N MAXIT PARAM [REPEAT]
//   SOLVER  LSSP_SOLVER_TYPE value (type-defs.h:157-178)
//   PC      0 PC_NON, 1 ILUK (LEVEL), 2 ILUT(1e-4, 20), 3 a user PC (LSSP_PC_USER,
//           pc.cxx:219-227) whose assemble calls lssp_pc_iluk_assemble (LEVEL)
//   N       7-pt Poisson N^3 (6 / -1, natural order, b = 1, x0 = 0)
//   PARAM   restart m (GMRES family, ORTHOMIN), l (BiCGSTAB(l)) or s (IDR(s)); <= 0: default
//   REPEAT  1: after the first solve, solve again with b = 2 (same assemble),
//           then scale A by 1.5, re-assemble and solve with b = 1 -- three lines
//           2: after the solve, apply the preconditioner directly through the
//           function pointer, pc.solve(&pc, r, x) and pc.solve(&pc, r, b)
//           (type-defs.h:103-105) -- two "pcsolve" lines
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <malloc.h>

#include "lssp.h"

static lssp_mat_csr poisson7(int N)
{
    const int n = N * N * N;
    lssp_mat_csr A;  // filled as exam.cxx:4-59 fills its 5-pt matrix
    A.num_rows = A.num_cols = n;
    A.Ap = lssp_malloc<int>(n + 1);
    A.Aj = lssp_malloc<int>(7 * n);
    A.Ax = lssp_malloc<double>(7 * n);
    int nnz = 0;
    A.Ap[0] = 0;
    for (int k = 0; k < N; k++)
        for (int j = 0; j < N; j++)
            for (int i = 0; i < N; i++) {
                const int r = (k * N + j) * N + i;
                const int cols[7] = {k > 0 ? r - N * N : -1, j > 0 ? r - N : -1, i > 0 ? r - 1 : -1, r,
                                     i < N - 1 ? r + 1 : -1, j < N - 1 ? r + N : -1, k < N - 1 ? r + N * N : -1};
                for (int q = 0; q < 7; q++)
                    if (cols[q] >= 0) {
                        A.Aj[nnz] = cols[q];
                        A.Ax[nnz] = cols[q] == r ? 6.0 : -1.0;
                        nnz++;
                    }
                A.Ap[r + 1] = nnz;
            }
    A.num_nnzs = nnz;
    return A;
}

static int g_user_level = 0;

// LSSP_PC_USER's assemble: the reference's own ILU(k) setup, which installs
// pc.solve = lssp_pc_ilu_solve (pc-iluk.cxx:566-581)
static void user_ilu_assemble(LSSP_PC &pc, LSSP_SOLVER s)
{
    pc.iluk_level = g_user_level;
    lssp_pc_iluk_assemble(pc, s);
}

int main(int argc, char **argv)
{
    if (argc != 7 && argc != 8) {
        fprintf(stderr, "usage: %s SOLVER PC LEVEL N MAXIT PARAM [REPEAT]\n", argv[0]);
        return 2;
    }
    const int sv = atoi(argv[1]), pct = atoi(argv[2]), level = atoi(argv[3]), N = atoi(argv[4]);
    const int maxit = atoi(argv[5]), param = atoi(argv[6]);
    lssp_verbosity = 0;
    // BiCGSafe, BiCRSafe, GPBiCG and GPBiCR read work vectors lssp_vec_create left
    // uninitialised; zero-filled allocations make the reference run deterministic
    // (the device drivers start from zeroed vectors), as in oracle/ref_shim.cxx
    mallopt(M_PERTURB, 0xff);

    lssp_mat_csr A = poisson7(N);
    const int n = A.num_rows;
    lssp_vec x = lssp_vec_create(n), b = lssp_vec_create(n), r = lssp_vec_create(n);
    lssp_vec_set_value(x, 0.);
    lssp_vec_set_value(b, 1.);

    LSSP_SOLVER solver;
    LSSP_PC pc;
    lssp_solver_create(solver, (LSSP_SOLVER_TYPE)sv, pc,
                       pct == 0 ? LSSP_PC_NON : pct == 1 ? LSSP_PC_ILUK : pct == 2 ? LSSP_PC_ILUT : LSSP_PC_USER);
    if (pct == 1) lssp_pc_iluk_set_level(pc, level);
    if (pct == 3) {
        g_user_level = level;
        pc.assemble = user_ilu_assemble;
    }
    if (pct == 2) {
        lssp_pc_ilut_set_drop_tol(pc, 1e-4);
        lssp_pc_ilut_set_p(pc, 20);
    }
    lssp_solver_set_maxit(solver, maxit);
    if (param > 0) {
        if (sv == LSSP_SOLVER_BICGSTABL) lssp_solver_set_bgsl(solver, param);
        else if (sv == LSSP_SOLVER_IDRS) lssp_solver_set_idrs(solver, param);
        else lssp_solver_set_restart(solver, param);
    }
    const int mode = argc == 8 ? atoi(argv[7]) : 0;
    const bool repeat = mode == 1;
    auto report = [&]() {
        double s1 = 0, s2 = 0;
        for (int i = 0; i < n; i++) {
            s1 += x.d[i];
            s2 += x.d[i] * x.d[i];
        }
        lssp_mv_amxpbyz(-1, A, x, 1, b, r);
        printf("nits %d residual %.17e xsum %.17e xsq %.17e x0 %.17e xlast %.17e true_res %.17e\n", solver.nits,
               solver.residual, s1, s2, x.d[0], x.d[n - 1], lssp_vec_norm(r));
    };
    lssp_solver_assemble(solver, A, x, b, pc);
    lssp_solver_solve(solver, pc);
    report();
    if (mode == 2 && pct != 0) {
        for (int t = 0; t < 2; t++) {
            pc.solve(&pc, r, t == 0 ? x : b);
            double s1 = 0, s2 = 0;
            for (int i = 0; i < n; i++) {
                s1 += r.d[i];
                s2 += r.d[i] * r.d[i];
            }
            printf("pcsolve %d sum %.17e sq %.17e r0 %.17e rlast %.17e\n", t, s1, s2, r.d[0], r.d[n - 1]);
        }
    }
    if (repeat) {
        // the same assembled system, another right-hand side
        lssp_vec_set_value(x, 0.);
        lssp_vec_set_value(b, 2.);
        lssp_solver_solve(solver, pc);
        report();
        // a new matrix: re-assemble (new copy of A, new factors), then solve
        for (int k = 0; k < A.num_nnzs; k++) A.Ax[k] *= 1.5;
        lssp_vec_set_value(x, 0.);
        lssp_vec_set_value(b, 1.);
        lssp_solver_assemble(solver, A, x, b, pc);
        lssp_solver_solve(solver, pc);
        report();
    }

    lssp_solver_destroy(solver, pc);
    lssp_mat_destroy(A);
    lssp_vec_destroy(x);
    lssp_vec_destroy(b);
    lssp_vec_destroy(r);
    return 0;
}
