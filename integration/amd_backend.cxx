// amd_backend.cxx -- the reference-side binding: route LSSP's Krylov hot path
// (all 18 internal Krylov drivers: BiCGSTAB, BiCGSTAB(l), GMRES(m), GMRES-R(m),
// LGMRES(m, k), CG, CGS, CR, CRS, BiCGSafe, BiCRSTAB, BiCRSafe, GPBiCG, GPBiCR,
// QMRCGSTAB, TFQMR, ORTHOMIN, IDR(s), with PC_NON, ILUK or ILUT) to lssp_amd on MI355X.
//
// This is the translation unit a maintainer adds to huiscliu/lssp (as
// src/amd-backend.cxx); INTEGRATION.md describes it.  It compiles against the
// reference's own headers and replaces, at link time, the drivers that
// lssp_solver_solve dispatches to (lssp.cxx:259-336):
//
//     -Wl,--wrap=<mangled lssp_solver_*>   (one per AMD_DRIVER line below)
//
// so lssp.cxx, the drivers and every caller (example/exam.cxx) stay unchanged.
// Everything else (assemble, the column sort, the ILU setup of pc-iluk.cxx /
// pc-ilut.cxx, other solvers and preconditioners) is the reference's own code.
//
// Per solve: A (the sorted copy lssp_solver_assemble made, lssp.cxx:166-173)
// and the factors pc.L / pc.U the reference built are uploaded, x0 and b too;
// the whole iteration runs in HBM (lssp_amd_solve); x is downloaded into the
// caller's view s.x.d (lssp.cxx:175-176) and s.residual / s.nits are set as the
// drivers set them (solver-bicgstab.cxx:156-157, :174).  A non-zero lssp_amd
// status becomes lssp_error(1, ...) -> exit(1), the reference's fatal path
// (utils.cxx:114-135).  LSSP_AMD_REDUCE=serial selects the reference's
// sequential dot order (bitwise-identical runs).
#include "lssp.h"
#include "lssp_amd.h"

static lssp_amd_ctx *amd_ctx()
{
    static lssp_amd_ctx *c = NULL;
    if (c == NULL) {
        const char *d = getenv("LSSP_AMD_DEVICE");
        int st = lssp_amd_ctx_create(d ? atoi(d) : 0, &c);
        if (st != LSSP_AMD_OK) lssp_error(1, "amd: cannot open the device: %s\n", lssp_amd_strerror(st));
    }
    return c;
}

#define AMD_CK(call)                                                                    \
    do {                                                                                \
        int st_ = (call);                                                               \
        if (st_ != LSSP_AMD_OK) lssp_error(1, "amd: %s: %s\n", #call, lssp_amd_strerror(st_)); \
    } while (0)

static bool amd_handles(const LSSP_PC &pc)
{
    return pc.type == LSSP_PC_NON || pc.type == LSSP_PC_ILUK || pc.type == LSSP_PC_ILUT;
}

static int amd_solve(LSSP_SOLVER &s, LSSP_PC &pc, int solver)
{
    lssp_amd_ctx *c = amd_ctx();
    const int n = s.A.num_rows;
    lssp_amd_mat *A = NULL;
    lssp_amd_ilu *M = NULL;
    double *x = NULL, *b = NULL;

    AMD_CK(lssp_amd_mat_upload(c, n, s.A.num_cols, s.A.num_nnzs, s.A.Ap, s.A.Aj, s.A.Ax, &A));
    if (pc.type != LSSP_PC_NON)
        AMD_CK(lssp_amd_ilu_from_factors(c, n, pc.L.Ap, pc.L.Aj, pc.L.Ax, pc.U.Ap, pc.U.Aj, pc.U.Ax, &M));
    AMD_CK(lssp_amd_vec_alloc(c, n, &x));
    AMD_CK(lssp_amd_vec_alloc(c, n, &b));
    AMD_CK(lssp_amd_vec_upload(c, x, s.x.d, n));
    AMD_CK(lssp_amd_vec_upload(c, b, s.rhs.d, n));

    lssp_amd_solve_params p;
    p.solver = solver;
    p.tol_rel = s.tol_rel;
    p.tol_abs = s.tol_abs;
    p.tol_rb = s.tol_rb;
    p.maxit = s.maxit;
    p.restart = s.restart;
    p.verb = s.verb;
    p.aug_k = s.aug_k;
    p.bgsl = s.bgsl;
    p.idrs = s.idrs;
    int nits = 0;
    double res = 0.;
    fflush(stdout);  // the device driver prints with stdio too: keep the line order
    AMD_CK(lssp_amd_solve(c, A, M, &p, x, b, &nits, &res, NULL, 0, NULL));
    fflush(stdout);
    AMD_CK(lssp_amd_vec_download(c, s.x.d, x, n));

    s.residual = res;
    s.nits = nits;
    lssp_amd_vec_free(c, x);
    lssp_amd_vec_free(c, b);
    if (M) lssp_amd_ilu_destroy(M);
    lssp_amd_mat_destroy(A);
    return nits;
}

// One wrapper per driver: the linker's --wrap=SYM sends every call of SYM here
// and names the original __real_SYM; PCs this library does not hold (BILUK,
// ITSOL, AMG, user PCs) fall through to the reference's own driver.
#define AMD_DRIVER(SYM, KIND)                                                   \
    extern "C" int __real_##SYM(LSSP_SOLVER &, LSSP_PC &);                      \
    extern "C" int __wrap_##SYM(LSSP_SOLVER &s, LSSP_PC &pc)                    \
    {                                                                           \
        if (!amd_handles(pc)) return __real_##SYM(s, pc);                       \
        return amd_solve(s, pc, KIND);                                          \
    }

// lssp.cxx:259-336 dispatch targets (mangled names of the drivers in src/solver-*.cxx)
AMD_DRIVER(_Z17lssp_solver_gmresR12LSSP_SOLVER_R8LSSP_PC_, LSSP_AMD_GMRES)
AMD_DRIVER(_Z18lssp_solver_lgmresR12LSSP_SOLVER_R8LSSP_PC_, LSSP_AMD_LGMRES)
AMD_DRIVER(_Z19lssp_solver_gmres_rR12LSSP_SOLVER_R8LSSP_PC_, LSSP_AMD_RGMRES)
AMD_DRIVER(_Z20lssp_solver_bicgstabR12LSSP_SOLVER_R8LSSP_PC_, LSSP_AMD_BICGSTAB)
AMD_DRIVER(_Z21lssp_solver_bicgstablR12LSSP_SOLVER_R8LSSP_PC_, LSSP_AMD_BICGSTABL)
AMD_DRIVER(_Z20lssp_solver_bicgsafeR12LSSP_SOLVER_R8LSSP_PC_, LSSP_AMD_BICGSAFE)
AMD_DRIVER(_Z14lssp_solver_cgR12LSSP_SOLVER_R8LSSP_PC_, LSSP_AMD_CG)
AMD_DRIVER(_Z15lssp_solver_cgsR12LSSP_SOLVER_R8LSSP_PC_, LSSP_AMD_CGS)
AMD_DRIVER(_Z18lssp_solver_gpbicgR12LSSP_SOLVER_R8LSSP_PC_, LSSP_AMD_GPBICG)
AMD_DRIVER(_Z14lssp_solver_crR12LSSP_SOLVER_R8LSSP_PC_, LSSP_AMD_CR)
AMD_DRIVER(_Z15lssp_solver_crsR12LSSP_SOLVER_R8LSSP_PC_, LSSP_AMD_CRS)
AMD_DRIVER(_Z20lssp_solver_bicrstabR12LSSP_SOLVER_R8LSSP_PC_, LSSP_AMD_BICRSTAB)
AMD_DRIVER(_Z20lssp_solver_bicrsafeR12LSSP_SOLVER_R8LSSP_PC_, LSSP_AMD_BICRSAFE)
AMD_DRIVER(_Z18lssp_solver_gpbicrR12LSSP_SOLVER_R8LSSP_PC_, LSSP_AMD_GPBICR)
AMD_DRIVER(_Z21lssp_solver_qmrcgstabR12LSSP_SOLVER_R8LSSP_PC_, LSSP_AMD_QMRCGSTAB)
AMD_DRIVER(_Z17lssp_solver_tfqmrR12LSSP_SOLVER_R8LSSP_PC_, LSSP_AMD_TFQMR)
AMD_DRIVER(_Z20lssp_solver_orthominR12LSSP_SOLVER_R8LSSP_PC_, LSSP_AMD_ORTHOMIN)
AMD_DRIVER(_Z16lssp_solver_idrsR12LSSP_SOLVER_R8LSSP_PC_, LSSP_AMD_IDRS)
