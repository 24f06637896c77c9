/*
 * lssp_amd.h -- C-ABI of the MI355X-native LSSP Krylov hot path.
 *
 * Plain pointers and sizes only (no torch, no C++ types).  Device vectors are
 * raw `double *` obtained from lssp_amd_vec_alloc; host arrays are the
 * caller's.  Every entry point returns an int status (LSSP_AMD_OK == 0) and
 * never exits the process; the reference-side binding
 * (integration/amd_backend.cxx) maps a non-zero status to lssp_error(1, ...),
 * which reproduces the reference's exit-on-fatal (utils.cxx:114-135).
 *
 * Each group cites the reference interface it replaces (paths relative to the
 * huiscliu/lssp tree).  The binding a maintainer would add on the reference
 * side is shown in INTEGRATION.md.
 */
#ifndef LSSP_AMD_H
#define LSSP_AMD_H

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status ------------------------------------------------------------ */
enum {
    LSSP_AMD_OK = 0,
    LSSP_AMD_EINVAL = 1,      /* bad argument (the reference asserts / lssp_error) */
    LSSP_AMD_EHIP = 2,        /* HIP runtime error */
    LSSP_AMD_ENOMEM = 3,      /* device or host allocation failed (utils.h:41-57) */
    LSSP_AMD_ETIMEOUT = 4,    /* a sync-free trisolve wait exceeded its bound */
    LSSP_AMD_ECOMM = 5,       /* RCCL error */
    LSSP_AMD_EUNSUPPORTED = 6 /* solver/PC combination not on the hot path */
};

/* reduction order of every dot / norm (vector.cxx:123-139) */
enum {
    LSSP_AMD_REDUCE_SERIAL = 0, /* sequential sum from 0, bitwise == the reference */
    LSSP_AMD_REDUCE_TREE = 1    /* canonical 256-chunk tree, the fast path */
};

/* LSSP_SOLVER_TYPE values of the reference (type-defs.h:157-178) */
enum {
    LSSP_AMD_GMRES = 0, LSSP_AMD_LGMRES = 1, LSSP_AMD_RGMRES = 2, LSSP_AMD_BICGSTAB = 4,
    LSSP_AMD_BICGSAFE = 6, LSSP_AMD_CG = 7, LSSP_AMD_CGS = 8, LSSP_AMD_GPBICG = 9, LSSP_AMD_CR = 10,
    LSSP_AMD_CRS = 11, LSSP_AMD_BICRSTAB = 12, LSSP_AMD_BICRSAFE = 13, LSSP_AMD_GPBICR = 14,
    LSSP_AMD_QMRCGSTAB = 15, LSSP_AMD_TFQMR = 16, LSSP_AMD_ORTHOMIN = 17,
    LSSP_AMD_BICGSTABL = 5, LSSP_AMD_IDRS = 18
};
/* ILU kinds (LSSP_PC_TYPE, type-defs.h:63-101) */
enum { LSSP_AMD_ILUK = 1, LSSP_AMD_ILUT = 2 };

typedef struct lssp_amd_ctx lssp_amd_ctx; /* one device + stream + scratch */
typedef struct lssp_amd_mat lssp_amd_mat; /* device CSR (lssp_mat_csr, type-defs.h:15-24) */
typedef struct lssp_amd_ilu lssp_amd_ilu; /* device L/U + trisolve schedules (LSSP_PC.L/.U) */

const char *lssp_amd_strerror(int status);
int lssp_amd_version(void);

/* Where the drivers' messages go (the lines the reference prints with
 * lssp_printf, utils.cxx:93-112: parameters at verb >= 2, the per-iteration
 * line at verb >= 1, "total iteration" / "total time" at verb >= 2).  fn ==
 * NULL (the default): stdout, flushed after every line.  The reference-side
 * binding routes them through lssp_printf, so a log file set with
 * lssp_set_log receives them too.  Process-wide; fn returns < 0 on error. */
void lssp_amd_set_print(int (*fn)(void *user, const char *msg), void *user);

/* ---- context: replaces the implicit single host thread ------------------ */
int lssp_amd_ctx_create(int device, lssp_amd_ctx **ctx);
int lssp_amd_ctx_destroy(lssp_amd_ctx *ctx);
int lssp_amd_ctx_set_reduction(lssp_amd_ctx *ctx, int mode);
int lssp_amd_ctx_sync(lssp_amd_ctx *ctx);
/* HIP stream the context enqueues on (a hipStream_t), for timing with events */
void *lssp_amd_ctx_stream(lssp_amd_ctx *ctx);

/* ---- device vectors: lssp_vec_create/destroy/set_value_by_array/get_value
 *      (vector.cxx:4-70) ----------------------------------------------- */
int lssp_amd_vec_alloc(lssp_amd_ctx *ctx, long n, double **d);
int lssp_amd_vec_free(lssp_amd_ctx *ctx, double *d);
int lssp_amd_vec_upload(lssp_amd_ctx *ctx, double *d, const double *h, long n);
int lssp_amd_vec_download(lssp_amd_ctx *ctx, double *h, const double *d, long n);

/* ---- CSR matrix: a device copy of an lssp_mat_csr, kept in the given entry
 *      order (SpMV sums in that order, mvops.cxx:55-58).  The solvers expect
 *      the assembled matrix, whose columns lssp_solver_assemble sorts
 *      (lssp.cxx:173): call lssp_amd_csr_sort_columns first, as that does. */
int lssp_amd_csr_sort_columns(int nrows, int ncols, int *Ap, int *Aj, double *Ax); /* matrix-utils.cxx:387-481 */
int lssp_amd_mat_upload(lssp_amd_ctx *ctx, int nrows, int ncols, int nnz, const int *Ap,
                        const int *Aj, const double *Ax, lssp_amd_mat **A);
int lssp_amd_mat_destroy(lssp_amd_mat *A);
int lssp_amd_mat_info(const lssp_amd_mat *A, int *nrows, int *ncols, int *nnz);
/* Device layout of the SpMV's column stream: *ndiag > 0 when every entry's
 * offset col - row is one of ndiag (<= 255) distinct values (stencil
 * matrices); the SpMV then reads a 1-byte offset id per entry instead of the
 * 4-byte column (same entries, same summation order).  0: plain CSR columns.
 * *windowed (may be NULL) = 1 when the columns of every 1024-row block span
 * at most 16384 entries and the product stages that span of x in LDS instead
 * of gathering it from memory (locally numbered meshes); 0 otherwise. */
int lssp_amd_mat_layout(const lssp_amd_mat *A, int *ndiag, int *windowed);
/* Device memory of a matrix: *csr_bytes = the resident CSR (Ap, Aj, Ax: every
 * operation but the two SpMV layouts above reads it), *aux_bytes = what the
 * SpMV layouts add beside it (offset ids + table; window spans and the sliced
 * copy, about as large as Aj + Ax again).  A windowed matrix whose padded
 * sliced copy would exceed 2^30 entries is not windowed (32-bit slice
 * offsets) and runs on the CSR product.  Either pointer may be NULL. */
int lssp_amd_mat_bytes(const lssp_amd_mat *A, long long *csr_bytes, long long *aux_bytes);

/* ---- SpMV: mvops.h:9-19 (mvops.cxx:5-150), bitwise per row --------------
 * x: for a matrix from lssp_amd_mat_upload the first ncols entries are read.
 * For a distributed matrix (lssp_amd_mat_upload_dist) x MUST hold
 * nrows + nhalo entries (lssp_amd_mat_local_rows): the rank's own entries,
 * then room for the halo, which every product OVERWRITES with the peers'
 * values before computing -- hence x is not const. */
/* y = y*beta + alpha*A*x            (lssp_mv_amxpby,  mvops.cxx:33-39)  */
int lssp_amd_mv_amxpby(lssp_amd_ctx *ctx, double alpha, const lssp_amd_mat *A, double *x,
                       double beta, double *y);
/* z = y*beta + alpha*A*x            (lssp_mv_amxpbyz, mvops.cxx:71-78)  */
int lssp_amd_mv_amxpbyz(lssp_amd_ctx *ctx, double alpha, const lssp_amd_mat *A, double *x,
                        double beta, const double *y, double *z);
/* y = a*A*x                         (lssp_mv_amxy,    mvops.cxx:109-115) */
int lssp_amd_mv_amxy(lssp_amd_ctx *ctx, double a, const lssp_amd_mat *A, double *x, double *y);
/* y = A*x                           (lssp_mv_mxy,     mvops.cxx:144-150) */
int lssp_amd_mv_mxy(lssp_amd_ctx *ctx, const lssp_amd_mat *A, double *x, double *y);

/* ---- BLAS-1: vector.h:8-39 (vector.cxx:31-146) -------------------------- */
int lssp_amd_vec_set_value(lssp_amd_ctx *ctx, double *x, long n, double val);
int lssp_amd_vec_copy(lssp_amd_ctx *ctx, double *x, const double *y, long n);
/* Measurement aid (no reference counterpart): read x[0..n) once with 16-byte
 * non-temporal loads and store the XOR of all its 64-bit words (as bits) in
 * the device double *sink -- the HBM streaming-read rate quoted beside the
 * 8 TB/s spec.  n even, x 16-byte aligned (else LSSP_AMD_EINVAL). */
int lssp_amd_stream_read(lssp_amd_ctx *ctx, const double *x, long n, double *sink);
int lssp_amd_vec_axy(lssp_amd_ctx *ctx, double alpha, const double *x, double *y, long n);
int lssp_amd_vec_axpby(lssp_amd_ctx *ctx, double alpha, const double *x, double beta, double *y,
                       long n);
int lssp_amd_vec_axpbyz(lssp_amd_ctx *ctx, double alpha, const double *x, double beta,
                        const double *y, double *z, long n);
int lssp_amd_vec_scale(lssp_amd_ctx *ctx, double *x, long n, double a);
int lssp_amd_vec_dot(lssp_amd_ctx *ctx, const double *x, const double *y, long n, double *result);
int lssp_amd_vec_norm(lssp_amd_ctx *ctx, const double *x, long n, double *result);

/* ---- ILU preconditioner ---------------------------------------------------
 * Setup on the host, exactly the reference algorithm: ILUK
 * (lssp_pc_iluk_assemble, pc-iluk.cxx:566-581) or ILUT (lssp_pc_ilut_assemble,
 * pc-ilut.cxx:429-456); blk > 0 and < n selects block-Jacobi blocks of that
 * size (the blk_size path of pc-iluk.cxx:411-552), used per rank on multi-GPU.
 * Then the factors are uploaded with their sync-free trisolve schedules.
 * Apply: x = U^-1 L^-1 rhs on the device (lssp_pc_ilu_solve,
 * solver-tri.cxx:57-60), bitwise; x may alias rhs. */
int lssp_amd_ilu_create(lssp_amd_ctx *ctx, int kind, int n, const int *Ap, const int *Aj,
                        const double *Ax, int level, double tol, int p, int blk,
                        lssp_amd_ilu **M);
/* upload caller-made factors (L: unit diagonal LAST per row; U: pivot FIRST) */
int lssp_amd_ilu_from_factors(lssp_amd_ctx *ctx, int n, const int *Lp, const int *Lj,
                              const double *Lx, const int *Up, const int *Uj, const double *Ux,
                              lssp_amd_ilu **M);
int lssp_amd_ilu_destroy(lssp_amd_ilu *M);
int lssp_amd_ilu_apply(lssp_amd_ctx *ctx, const lssp_amd_ilu *M, double *x, const double *rhs);
/* The apply enqueued on the context's stream without waiting for it (the
 * synchronous lssp_amd_ilu_apply returns when x is written, like the
 * reference's pc.solve); lssp_amd_ilu_check then waits for the stream and
 * reports a hand-off timeout (LSSP_AMD_ETIMEOUT) of any apply since the last
 * check, re-arming the factor's hand-off buffers.  After an ETIMEOUT, the x of
 * EVERY apply enqueued since the last successful check is invalid (an apply
 * queued behind the one that timed out reads its un-armed hand-off buffers):
 * re-run them. */
int lssp_amd_ilu_apply_async(lssp_amd_ctx *ctx, const lssp_amd_ilu *M, double *x, const double *rhs);
int lssp_amd_ilu_check(lssp_amd_ctx *ctx, const lssp_amd_ilu *M);
/* one triangular sweep: which = 0 lower (solver-tri.cxx:4-24), 1 upper (:26-46) */
int lssp_amd_ilu_trisolve(lssp_amd_ctx *ctx, const lssp_amd_ilu *M, int which, double *x,
                          const double *rhs);
int lssp_amd_ilu_info(const lssp_amd_ilu *M, int *n, int *nnzL, int *nnzU, int *levelsL,
                      int *levelsU, double *setup_seconds);
int lssp_amd_ilu_get_factors(const lssp_amd_ilu *M, int *Lp, int *Lj, double *Lx, int *Up,
                             int *Uj, double *Ux);
/* How an apply sweeps M's factors (no reference counterpart: a query like
 * lssp_amd_mat_layout).  *line = 1 when the factors are a natural-ordered 5-/7-
 * point grid's ILU(0) and run as line sweeps, with tiles of *lines lines x
 * *planes planes (chosen per factor); 2 when they are a 7-point grid's ILU(1)
 * (fill offsets nx-1, nx*ny-nx, nx*ny-1) and run as skewed line sweeps
 * (*lines = 16 lines of j + k, *planes = 8); 0 (and 0 x 0) for the general
 * packet sweeps.  Any pointer may be NULL. */
int lssp_amd_ilu_sweep_layout(const lssp_amd_ilu *M, int *line, int *lines, int *planes);

/* ---- Krylov solve: lssp_solver_solve (lssp.cxx:250-414) for BiCGSTAB
 *      (solver-bicgstab.cxx:10-175), GMRES(m) (solver-gmres.cxx:12-255),
 *      right-preconditioned GMRES(m) (solver-gmres.cxx:257-479), LGMRES(m, k)
 *      (solver-lgmres.cxx:12-312), CG (solver-cg.cxx:8-136), and the other internal
 *      drivers (solver-{bicgstabl,bicgsafe,cgs,gpbicg,cr,crs,bicrstab,bicrsafe,
 *      gpbicr,qmrcgstab,tfqmr,orthomin,idrs}.cxx).  Same recurrences, guards, defaults and
 *      iteration counting; vectors stay in HBM. ------------------------- */
typedef struct {
    int solver;     /* LSSP_AMD_* above (LSSP_SOLVER_TYPE) */
    double tol_rel; /* < 0: default 1e-7 (lssp.cxx:11-13) */
    double tol_abs;
    double tol_rb;
    int maxit;      /* <= 0: default 1000 */
    int restart;    /* GMRES m; < 0: default 50 */
    int verb;       /* >= 1 prints the reference's per-iteration line */
    int aug_k;      /* LGMRES augmentation vectors k; <= 0: default 3 (lssp.cxx:6) */
    int bgsl;       /* BiCGSTAB(l) l; <= 0: default 4 (LSSP_SOLVER.bgsl, lssp.cxx:7, :495-503) */
    int idrs;       /* IDR(s) s; <= 0: default 4 (LSSP_SOLVER.idrs, lssp.cxx:8, :505-513) */
} lssp_amd_solve_params;

/* x: device, x0 on entry, solution on exit; b: device.  M == NULL is PC_NON
 * (pc.cxx:67-70).  trace (host, optional) receives every dot/norm the driver
 * evaluates, in the reference's call order.  On a distributed matrix x and
 * every work vector hold nrows + nhalo entries (the halo part of x is
 * overwritten by the solve's products); b holds nrows. */
int lssp_amd_solve(lssp_amd_ctx *ctx, const lssp_amd_mat *A, const lssp_amd_ilu *M,
                   const lssp_amd_solve_params *prm, double *x, const double *b, int *nits,
                   double *residual, double *trace, int trace_cap, int *trace_len);

/* ---- multi-GPU: one process per GPU, row-block partition, RCCL over xGMI --
 * The reference is serial (README.md:3); this is the SURVEY 8(e) extension.
 * Rank r owns rows [r*ceil(n/P), min((r+1)*ceil(n/P), n)).  A distributed
 * matrix holds the rank's rows with columns renumbered [owned | halo]; SpMV
 * fetches the halo with grouped ncclSend/ncclRecv; dots all-gather the P rank
 * partials and sum them in rank order (deterministic, identical on every
 * rank). */
int lssp_amd_comm_unique_id_size(void);
int lssp_amd_comm_get_unique_id(void *id_out);
/* Collective over the nranks processes (ncclCommInitRank).  Every nranks >= 1
 * creates a real RCCL communicator, nranks == 1 included: the caller must pass
 * an id from lssp_amd_comm_get_unique_id (a placeholder id blocks or fails in
 * RCCL).  A context that never calls it runs single-rank with no communicator;
 * lssp_amd_comm_nranks reports the communicator's rank count (ncclCommCount). */
int lssp_amd_comm_init(lssp_amd_ctx *ctx, int nranks, int rank, const void *id);
int lssp_amd_comm_nranks(lssp_amd_ctx *ctx, int *nranks);
int lssp_amd_comm_barrier(lssp_amd_ctx *ctx);
/* Transport check (collective): an all-gather of every rank's id and a ring
 * round of grouped send/recv (rank r -> r+1, r-1 -> r; a 1-rank communicator
 * sends to itself) driven exactly as the SpMV's halo round is -- packed on the
 * compute stream, the round on the communication stream between two events,
 * the compute stream waiting for it -- then every received word checked.
 * LSSP_AMD_OK, or LSSP_AMD_ECOMM when a value did not arrive.  With nranks = 1
 * lssp_amd_comm_init still creates the (1-rank) RCCL communicator, so a single
 * GPU can run this before a multi-GPU job. */
int lssp_amd_comm_selftest(lssp_amd_ctx *ctx);

/* Host-staged transport: the same protocol with the collective carried by the
 * caller (an MPI library, a torch.distributed gloo group, ...) instead of
 * RCCL.  The library copies the bytes to host memory, calls the hook and
 * copies the result back; used where RCCL is unavailable and to exercise the
 * multi-rank path with several ranks on ONE device (RCCL refuses that).
 * Every hook returns 0 on success; buffers are host memory. */
typedef struct {
    void *user;
    /* recv[q*bytes .. (q+1)*bytes) = rank q's send, for q = 0 .. nranks-1 */
    int (*allgather)(void *user, const void *send, void *recv, long bytes);
    /* one grouped round: nsend messages to peers send_peer[i], nrecv from
     * recv_peer[i]; a rank sends at most one message to each peer per round */
    int (*sendrecv)(void *user, int nsend, const int *send_peer, const void *const *send_buf,
                    const long *send_bytes, int nrecv, const int *recv_peer, void *const *recv_buf,
                    const long *recv_bytes);
} lssp_amd_host_transport;
int lssp_amd_comm_init_host(lssp_amd_ctx *ctx, int nranks, int rank, const lssp_amd_host_transport *t);

/* rows [row0, row0 + nlocal) of a global n x n CSR given by its local rows.
 * Collective: every rank calls it; the input checks are agreed on across the
 * ranks first, so a bad argument on one rank makes EVERY rank return
 * LSSP_AMD_EINVAL (no rank is left waiting in a collective). */
int lssp_amd_mat_upload_dist(lssp_amd_ctx *ctx, int n_global, int row0, int nlocal,
                             const int *Ap, const int *Aj, const double *Ax, lssp_amd_mat **A);
int lssp_amd_mat_local_rows(const lssp_amd_mat *A, int *row0, int *nlocal, int *nhalo);

/* ---- device index arrays: the int members of lssp_mat_csr / lssp_mat_coo /
 *      lssp_mat_bcsr (type-defs.h:15-55) in HBM, as lssp_amd_vec_* for doubles */
int lssp_amd_idx_alloc(lssp_amd_ctx *ctx, long n, int **d);
int lssp_amd_idx_free(lssp_amd_ctx *ctx, int *d);
int lssp_amd_idx_upload(lssp_amd_ctx *ctx, int *d, const int *h, long n);
int lssp_amd_idx_download(lssp_amd_ctx *ctx, int *h, const int *d, long n);

/* ---- format conversions on the device (matrix-utils.h:22-49) --------------
 * Every array is DEVICE memory (idx_alloc / vec_alloc); outputs are caller
 * allocated and must not overlap the inputs.  Results are bitwise those of
 * the reference functions, entry order included.  Input structure is checked
 * on the device first (row pointers non-decreasing from 0 to nnz, indices
 * that address memory in range); a violation returns LSSP_AMD_EINVAL where the
 * reference would assert or read out of bounds.  With nnz == 0 the output row
 * pointers are all 0 (the reference leaves them unallocated). */
/* lssp_mat_csr_to_coo (matrix-utils.cxx:281-322): Ci[k] = row of entry k,
 * Cj/Cx copies.  Cj/Cx may be NULL (the caller keeps using Aj/Ax). */
int lssp_amd_csr_to_coo(lssp_amd_ctx *ctx, int nrows, int nnz, const int *Ap, const int *Aj,
                        const double *Ax, int *Ci, int *Cj, double *Cx);
/* lssp_mat_coo_to_csr (matrix-utils.cxx:324-380): rows bucketed in order,
 * entries of one row kept in input order (a stable sort by row); Ci must lie
 * in [0, nrows), column indices are copied unchecked as in the reference.
 * Ap holds nrows + 1. */
int lssp_amd_coo_to_csr(lssp_amd_ctx *ctx, int nrows, int nnz, const int *Ci, const int *Cj,
                        const double *Cx, int *Ap, int *Aj, double *Ax);
/* lssp_mat_transpose (matrix-utils.cxx:700-765): T (ncols x nrows), row c of
 * T lists the rows of A holding column c in increasing row order (entry
 * order within a row of A for duplicates).  Tp holds ncols + 1. */
int lssp_amd_csr_transpose(lssp_amd_ctx *ctx, int nrows, int ncols, int nnz, const int *Ap,
                           const int *Aj, const double *Ax, int *Tp, int *Tj, double *Tx);
/* lssp_mat_csr_to_bcsr (matrix-utils.cxx:62-162): n x n CSR (n % bs == 0,
 * nnz > 0, else EINVAL as lssp_error/assert there) to (n/bs)^2 blocks of
 * bs x bs, block columns of a block row ascending, each block COLUMN-major
 * (entry (r, c) at Bx[blk*bs*bs + (c%bs)*bs + r%bs]), absent entries 0, and a
 * duplicate (r, c) keeps its last value.  Two calls: with Bj == NULL only
 * *bnnz (number of blocks) is computed; then Bp (n/bs + 1), Bj (*bnnz) and
 * Bx (*bnnz * bs * bs) are filled. */
int lssp_amd_csr_to_bcsr(lssp_amd_ctx *ctx, int n, int nnz, int bs, const int *Ap, const int *Aj,
                         const double *Ax, int *bnnz, int *Bp, int *Bj, double *Bx);
/* lssp_mat_bcsr_to_csr (matrix-utils.cxx:164-215): the entries with
 * fabs(v) > 0 (zeros and NaNs are dropped, as there), each row's columns
 * sorted (lssp_mat_sort_column, :387-481: a row that was out of order gives
 * every duplicate column the value of its last occurrence).  Two calls: with
 * Aj == NULL only *nnz is computed (Ap may be NULL); then Ap (nbrows*bs + 1),
 * Aj and Ax (*nnz) are filled. */
int lssp_amd_bcsr_to_csr(lssp_amd_ctx *ctx, int nbrows, int nbcols, int bs, int bnnz, const int *Bp,
                         const int *Bj, const double *Bx, int *nnz, int *Ap, int *Aj, double *Ax);

/* ---- synthetic inputs (example/exam.cxx:4-59 and its 7-pt analogue) ------ */
long lssp_amd_poisson_nnz(int dim, int N);
/* rows [row0, row0+nrows) of the 5-pt (dim 2) or 7-pt (dim 3) Laplacian */
int lssp_amd_poisson_rows(int dim, int N, long row0, long nrows, int *Ap, int *Aj, double *Ax);

#ifdef __cplusplus
}
#endif
#endif
