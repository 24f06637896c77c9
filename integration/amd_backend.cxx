// amd_backend.cxx -- the reference-side binding: route LSSP's Krylov hot path
// (all 18 internal Krylov drivers: BiCGSTAB, BiCGSTAB(l), GMRES(m), GMRES-R(m),
// LGMRES(m, k), CG, CGS, CR, CRS, BiCGSafe, BiCRSTAB, BiCRSafe, GPBiCG, GPBiCR,
// QMRCGSTAB, TFQMR, ORTHOMIN, IDR(s), with PC_NON, ILUK, ILUT or a user PC whose
// pc.solve is the ILU apply) and the pc.solve seam itself (lssp_pc_ilu_solve,
// solver-tri.cxx:57-60) to lssp_amd on MI355X.
//
// This is the translation unit a maintainer adds to huiscliu/lssp (as
// src/amd-backend.cxx); INTEGRATION.md describes it.  It compiles against the
// reference's own headers and replaces, at link time, the drivers that
// lssp_solver_solve dispatches to (lssp.cxx:259-336), and hooks the solver /
// PC lifecycle (lssp.cxx:142-200, pc.cxx):
//
//     -Wl,--wrap=<mangled lssp_solver_*>   (one per AMD_DRIVER line below)
//     -Wl,--wrap=<mangled lssp_solver_assemble, lssp_solver_destroy, lssp_pc_assemble>
//     -Wl,--wrap=<mangled lssp_pc_ilu_solve>
//
// so lssp.cxx, the drivers and every caller (example/exam.cxx) stay unchanged.
// Everything else (assemble, the column sort, the ILU setup of pc-iluk.cxx /
// pc-ilut.cxx, other solvers and preconditioners) is the reference's own code.
//
// Device state per LSSP_SOLVER, kept across solves: A (the sorted copy
// lssp_solver_assemble made, lssp.cxx:166-173), the factors pc.L / pc.U the
// reference built with their sweep schedules, and the x / b work vectors.
// They are built at the first solve after an assemble and dropped when the
// solver is re-assembled or destroyed or its PC re-assembled, so a caller that
// solves repeatedly after one lssp_solver_assemble pays the upload and the
// schedule build once; each solve uploads only x0 and b.  The whole iteration
// runs in HBM (lssp_amd_solve); x is downloaded into the caller's view s.x.d
// (lssp.cxx:175-176) and s.residual / s.nits are set as the drivers set them
// (solver-bicgstab.cxx:156-157, :174).  The drivers' messages go through
// lssp_printf (utils.cxx:93-112: stdout and the lssp_set_log file).  A non-zero
// lssp_amd status becomes lssp_error(1, ...) -> exit(1), the reference's fatal
// path (utils.cxx:114-135).  LSSP_AMD_REDUCE=serial selects the reference's
// sequential dot order (bitwise-identical runs).
#include "lssp.h"
#include "lssp_amd.h"

#include <map>

static int amd_print(void *, const char *msg) { return lssp_printf("%s", msg); }

// LSSP_AMD_BINDING_STATS=1: at exit, report to stderr how many solves and
// pc.solve applications ran on the device (which calls the binding took)
static long amd_n_solves = 0, amd_n_applies = 0;
static void amd_stats(void)
{
    fprintf(stderr, "amd: device solves %ld, device pc applies %ld\n", amd_n_solves, amd_n_applies);
}

static lssp_amd_ctx *amd_ctx()
{
    static lssp_amd_ctx *c = NULL;
    if (c == NULL) {
        const char *d = getenv("LSSP_AMD_DEVICE");
        int st = lssp_amd_ctx_create(d ? atoi(d) : 0, &c);
        if (st != LSSP_AMD_OK) lssp_error(1, "amd: cannot open the device: %s\n", lssp_amd_strerror(st));
        lssp_amd_set_print(amd_print, NULL);
        const char *bs = getenv("LSSP_AMD_BINDING_STATS");
        if (bs && atoi(bs) > 0) atexit(amd_stats);
    }
    return c;
}

#define AMD_CK(call)                                                                    \
    do {                                                                                \
        int st_ = (call);                                                               \
        if (st_ != LSSP_AMD_OK) lssp_error(1, "amd: %s: %s\n", #call, lssp_amd_strerror(st_)); \
    } while (0)

// the pc.solve seam (type-defs.h:103-105): lssp_pc_ilu_solve as every object
// linked with --wrap sees it (pc-iluk.cxx:578, pc-ilut.cxx:453, user code)
#define SYM_PC_ILU_SOLVE _Z17lssp_pc_ilu_solveP8LSSP_PC_9lssp_vec_S1_
#define AMD_CAT_(a, b) a##b
#define AMD_CAT(a, b) AMD_CAT_(a, b)
extern "C" void AMD_CAT(__wrap_, SYM_PC_ILU_SOLVE)(LSSP_PC *pc, lssp_vec x, lssp_vec rhs);

// a user PC (LSSP_PC_USER, pc.cxx:219-227) whose assemble installed the ILU
// apply (e.g. by calling lssp_pc_iluk_assemble) is an ILU on pc.L / pc.U too
static bool amd_is_ilu(const LSSP_PC &pc)
{
    return pc.type == LSSP_PC_ILUK || pc.type == LSSP_PC_ILUT ||
           (pc.type == LSSP_PC_USER && pc.solve == AMD_CAT(__wrap_, SYM_PC_ILU_SOLVE));
}

static bool amd_handles(const LSSP_PC &pc) { return pc.type == LSSP_PC_NON || amd_is_ilu(pc); }

// ---- device state per solver ------------------------------------------------
struct AmdState {
    const LSSP_PC *pc = NULL;
    const double *Ax = NULL;  // identity of the uploaded A (s.A)
    int n = 0, nnz = 0;
    lssp_amd_mat *A = NULL;
    const double *Lx = NULL, *Ux = NULL;  // identity of the uploaded factors (pc.L, pc.U)
    lssp_amd_ilu *M = NULL;
    double *x = NULL, *b = NULL;
};
static std::map<const LSSP_SOLVER *, AmdState> amd_states;

static void amd_drop_factors(AmdState &d)
{
    if (d.M) lssp_amd_ilu_destroy(d.M);
    d.M = NULL;
    d.Lx = d.Ux = NULL;
}

static void amd_drop(const LSSP_SOLVER *s)
{
    std::map<const LSSP_SOLVER *, AmdState>::iterator it = amd_states.find(s);
    if (it == amd_states.end()) return;
    AmdState &d = it->second;
    lssp_amd_ctx *c = amd_ctx();
    amd_drop_factors(d);
    if (d.A) lssp_amd_mat_destroy(d.A);
    if (d.x) lssp_amd_vec_free(c, d.x);
    if (d.b) lssp_amd_vec_free(c, d.b);
    amd_states.erase(it);
}

static int amd_solve(LSSP_SOLVER &s, LSSP_PC &pc, int solver)
{
    lssp_amd_ctx *c = amd_ctx();
    const int n = s.A.num_rows;
    AmdState &d = amd_states[&s];
    d.pc = &pc;
    if (d.A && (d.Ax != s.A.Ax || d.n != n || d.nnz != s.A.num_nnzs)) {  // defensive: a different A
        lssp_amd_mat_destroy(d.A);
        d.A = NULL;
    }
    if (!d.A) {
        AMD_CK(lssp_amd_mat_upload(c, n, s.A.num_cols, s.A.num_nnzs, s.A.Ap, s.A.Aj, s.A.Ax, &d.A));
        d.Ax = s.A.Ax;
        d.nnz = s.A.num_nnzs;
    }
    if (d.n != n) {
        if (d.x) lssp_amd_vec_free(c, d.x);
        if (d.b) lssp_amd_vec_free(c, d.b);
        AMD_CK(lssp_amd_vec_alloc(c, n, &d.x));
        AMD_CK(lssp_amd_vec_alloc(c, n, &d.b));
        d.n = n;
    }
    if (pc.type == LSSP_PC_NON) {
        amd_drop_factors(d);
    } else if (!d.M || d.Lx != pc.L.Ax || d.Ux != pc.U.Ax) {
        amd_drop_factors(d);
        AMD_CK(lssp_amd_ilu_from_factors(c, n, pc.L.Ap, pc.L.Aj, pc.L.Ax, pc.U.Ap, pc.U.Aj, pc.U.Ax, &d.M));
        d.Lx = pc.L.Ax;
        d.Ux = pc.U.Ax;
    }
    AMD_CK(lssp_amd_vec_upload(c, d.x, s.x.d, n));
    AMD_CK(lssp_amd_vec_upload(c, d.b, s.rhs.d, n));

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
    AMD_CK(lssp_amd_solve(c, d.A, pc.type == LSSP_PC_NON ? NULL : d.M, &p, d.x, d.b, &nits, &res, NULL, 0, NULL));
    AMD_CK(lssp_amd_vec_download(c, s.x.d, d.x, n));
    amd_n_solves++;

    s.residual = res;
    s.nits = nits;
    return nits;
}

// ---- the pc.solve seam: x = U^-1 L^-1 rhs on the device ------------------------
// A caller that applies the preconditioner itself (pc.solve(&pc, x, rhs)) or a
// driver this library does not replace reaches lssp_pc_ilu_solve through the
// function pointer.  The factors pc->L / pc->U go to the device once per PC
// (identity-checked, dropped with the PC's lifecycle like AmdState); every
// call moves rhs and x over PCIe, as the caller's vectors are host memory.
struct AmdPcState {
    const double *Lx = NULL, *Ux = NULL;
    int n = 0;
    lssp_amd_ilu *M = NULL;
    double *x = NULL, *r = NULL;
};
static std::map<const LSSP_PC *, AmdPcState> amd_pcs;

static void amd_drop_pc(const LSSP_PC *pc)
{
    std::map<const LSSP_PC *, AmdPcState>::iterator it = amd_pcs.find(pc);
    if (it == amd_pcs.end()) return;
    lssp_amd_ctx *c = amd_ctx();
    if (it->second.M) lssp_amd_ilu_destroy(it->second.M);
    if (it->second.x) lssp_amd_vec_free(c, it->second.x);
    if (it->second.r) lssp_amd_vec_free(c, it->second.r);
    amd_pcs.erase(it);
}

extern "C" void AMD_CAT(__wrap_, SYM_PC_ILU_SOLVE)(LSSP_PC *pc, lssp_vec x, lssp_vec rhs)
{
    assert(x.d != NULL && rhs.d != NULL);
    lssp_amd_ctx *c = amd_ctx();
    const int n = pc->L.num_rows;
    std::map<const LSSP_PC *, AmdPcState>::iterator it = amd_pcs.find(pc);
    if (it != amd_pcs.end() && (it->second.Lx != pc->L.Ax || it->second.Ux != pc->U.Ax || it->second.n != n)) {
        amd_drop_pc(pc);  // defensive: factors replaced without lssp_pc_assemble
        it = amd_pcs.end();
    }
    if (it == amd_pcs.end()) {
        AmdPcState e;
        AMD_CK(lssp_amd_ilu_from_factors(c, n, pc->L.Ap, pc->L.Aj, pc->L.Ax, pc->U.Ap, pc->U.Aj, pc->U.Ax, &e.M));
        AMD_CK(lssp_amd_vec_alloc(c, n, &e.x));
        AMD_CK(lssp_amd_vec_alloc(c, n, &e.r));
        e.Lx = pc->L.Ax;
        e.Ux = pc->U.Ax;
        e.n = n;
        it = amd_pcs.insert(std::make_pair(pc, e)).first;
    }
    AmdPcState &e = it->second;
    AMD_CK(lssp_amd_vec_upload(c, e.r, rhs.d, n));
    AMD_CK(lssp_amd_ilu_apply(c, e.M, e.x, e.r));
    AMD_CK(lssp_amd_vec_download(c, x.d, e.x, n));
    amd_n_applies++;
}

// ---- lifecycle hooks: the cached device state follows the reference's objects
#define SYM_SOLVER_ASSEMBLE _Z20lssp_solver_assembleR12LSSP_SOLVER_R13lssp_mat_csr_9lssp_vec_S3_R8LSSP_PC_
#define SYM_SOLVER_DESTROY _Z19lssp_solver_destroyR12LSSP_SOLVER_R8LSSP_PC_
#define SYM_PC_ASSEMBLE _Z16lssp_pc_assembleR8LSSP_PC_12LSSP_SOLVER_

// lssp_solver_assemble (lssp.cxx:142-189): a new copy of A, the PC re-assembled
extern "C" void AMD_CAT(__real_, SYM_SOLVER_ASSEMBLE)(LSSP_SOLVER &, lssp_mat_csr &, lssp_vec, lssp_vec, LSSP_PC &);
extern "C" void AMD_CAT(__wrap_, SYM_SOLVER_ASSEMBLE)(LSSP_SOLVER &s, lssp_mat_csr &A, lssp_vec x, lssp_vec b,
                                                      LSSP_PC &pc)
{
    amd_drop(&s);
    AMD_CAT(__real_, SYM_SOLVER_ASSEMBLE)(s, A, x, b, pc);
}

// lssp_solver_destroy (lssp.cxx:191-208)
extern "C" void AMD_CAT(__real_, SYM_SOLVER_DESTROY)(LSSP_SOLVER &, LSSP_PC &);
extern "C" void AMD_CAT(__wrap_, SYM_SOLVER_DESTROY)(LSSP_SOLVER &s, LSSP_PC &pc)
{
    amd_drop(&s);
    amd_drop_pc(&pc);
    AMD_CAT(__real_, SYM_SOLVER_DESTROY)(s, pc);
}

// lssp_pc_assemble (pc.cxx): new factors for every solver using this PC
extern "C" void AMD_CAT(__real_, SYM_PC_ASSEMBLE)(LSSP_PC &, LSSP_SOLVER);
extern "C" void AMD_CAT(__wrap_, SYM_PC_ASSEMBLE)(LSSP_PC &pc, LSSP_SOLVER s)
{
    for (std::map<const LSSP_SOLVER *, AmdState>::iterator it = amd_states.begin(); it != amd_states.end(); ++it)
        if (it->second.pc == &pc) amd_drop_factors(it->second);
    amd_drop_pc(&pc);
    AMD_CAT(__real_, SYM_PC_ASSEMBLE)(pc, s);
}

// One wrapper per driver: the linker's --wrap=SYM sends every call of SYM here
// and names the original __real_SYM; PCs this library does not hold (BILUK,
// ITSOL, AMG, user PCs with their own solve) fall through to the reference's
// own driver.
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
