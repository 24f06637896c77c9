// internal.h -- shared state of the lssp_amd library (not part of the C-ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <functional>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/lssp_amd.h"

namespace lssp_amd {

// ---- canonical reduction layout ------------------------------
constexpr int CHUNK = 256;       // level 1: one aligned chunk of 256 elements per partial
constexpr int L2_LANES = 1024;   // level 2: one workgroup, lane t sums partials t, t+1024, ...
constexpr int MAX_SLOTS = 4;     // partial sums one pass can produce
constexpr int NSCAL = 4096;      // device scalar slots per context

// sync-free trisolve: the value-as-flag "not yet computed" pattern (a NaN payload
// no arithmetic produces)
constexpr uint64_t TRI_SENTINEL = 0xFFF7DEADBEEFCAFEull;

// scalar slots of the Krylov drivers (device memory, ctx->d_scal)
enum Scal {
    S_RHO0 = 0, S_RHO1, S_ALPHA, S_BETA, S_OMEGA, S_RES, S_SNORM, S_BREAK, S_BNORM, S_TMP,
    S_DONE, S_TOL, S_NIT,  // batched iterations (solvers.cpp cg): stop flag, tolerance, iterations run
    S_SUM0 = 16,   // raw reduced sums of the last reduction
    S_H = 32,      // GMRES Hessenberg column (up to NSCAL - 32 entries); batched residual history ring
    S_HB = 64,     // ... of S_HB entries: iteration k's residual at S_H + k % S_HB (two batches in flight)
};

// finalize programs run by one lane after a reduction (same code for every
// reduction mode, so the scalar recurrences are bit-identical across modes)
enum FinOp {
    FIN_STORE = 0,       // scal[dst[k]] = sum[k]
    FIN_NORM,            // scal[dst[0]] = sqrt(sum[0])
    FIN_BICG_RHO,        // rho1 = s0; beta = (rho1*alpha)/(rho0*omega); rho0 = rho1
    FIN_BICG_ALPHA,      // alpha = rho1 / s0
    FIN_BICG_S,          // snorm = sqrt(s0); break = snorm <= 1e-40
    FIN_BICG_OMEGA,      // omega = s0 / s1
    FIN_BICG_RES_RHO,    // res = sqrt(s0); then FIN_BICG_RHO on s1
    FIN_BICG_RES_RHO_B,  // FIN_BICG_RES_RHO, then res -> history S_H + nit % S_HB, nit += 1, done = 2 breakdown
                         // (S_BREAK), 1 res <= tol, 3 the next iteration's rho1 == 0
    FIN_CG_RHO,          // rho1 = s0; beta = rho1 / rho0
    FIN_CG_ALPHA,        // alpha = rho1 / s0; rho0 = rho1
    FIN_CG_RES,          // res = sqrt(s0)
    FIN_CG_RES_RHO,      // res = sqrt(s0); rho1 = s0; beta = rho1/rho0  (PC_NON: z == r)
    FIN_CG_RES_RHO_B,    // FIN_CG_RES_RHO, then res -> history S_H + nit % S_HB, nit += 1, done = res <= tol
    FIN_BICG_S_OMEGA,    // sums (t.s, t.t, s.s): FIN_BICG_S on s2 (traced at tpos[2]), then FIN_BICG_OMEGA
};

struct Fin {
    int op = FIN_STORE;
    int nsum = 1;
    int dst[MAX_SLOTS] = {S_SUM0, S_SUM0 + 1, S_SUM0 + 2, S_SUM0 + 3};
    int tpos[3] = {-1, -1, -1};  // trace positions of the (up to three) traced values
};

}  // namespace lssp_amd

struct lssp_amd_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    int reduce_mode = LSSP_AMD_REDUCE_TREE;
    int num_cus = 256;
    // reduction scratch
    double *d_part = nullptr;  // [MAX_SLOTS][part_cap] level-1 partials
    long part_cap = 0;
    double *d_sums = nullptr;  // [MAX_SLOTS] rank-local sums
    double *d_wsum = nullptr;  // [MAX_SLOTS][16] level-2 wave sums (k_reduce2m)
    unsigned *d_rcnt = nullptr;  // level-2 arrival counter (k_reduce2m), 0 between launches
    double *d_scal = nullptr;  // [NSCAL] scalar slots
    double *h_scal = nullptr;  // pinned mirror
    double *d_trace = nullptr; // device trace buffer
    long trace_cap = 0;
    int *d_err = nullptr;      // error word (trisolve timeouts)
    // batched iterations: the stream copies each batch's scalars and error word
    // into snapshot k (pinned) and records ev_snap[k], so the host reads batch
    // j while batch j + 1 runs (solvers.cpp Pipe)
    double *h_snap = nullptr;  // [2][S_H + S_HB]
    int *h_snap_err = nullptr; // [2]
    hipEvent_t ev_snap[2] = {nullptr, nullptr};
    // while set: every k_ew / k_spmv3 / reduction launch returns at once when
    // *guard != 0 (batched iterations past the one that converged)
    const double *guard = nullptr;
    // multi-GPU (RCCL)
    int nranks = 1, rank = 0;
    void *comm = nullptr;      // ncclComm_t
    lssp_amd_host_transport host{};  // host-staged transport (comm == nullptr, nranks > 1)
    double *d_gather = nullptr;  // [nranks][MAX_SLOTS]
    double *d_carry = nullptr;   // [MAX_SLOTS] serial mode: running sums of the ranks before this one
    int *d_igather = nullptr;    // [1 + nranks] comm_gather_int scratch (allocated with the communicator)
    // RCCL mode: the halo round runs on comm_stream while the interior rows'
    // product runs on stream (ev_pack: send buffer packed; ev_halo: halo landed)
    hipStream_t comm_stream = nullptr;
    hipEvent_t ev_pack = nullptr, ev_halo = nullptr;
    int tri_blocks_per_cu = 1;  // the sync-free sweep's grid (k_trisolve)
    // Krylov work vectors, kept across solves (no hipMalloc on the solve path)
    struct WsBuf {
        double *p;
        long n;
        bool used;
    };
    std::vector<WsBuf> pool;
};

struct lssp_amd_mat {
    lssp_amd_ctx *ctx = nullptr;
    int nrows = 0, ncols = 0, nnz = 0;  // local rows; ncols = local column space (owned + halo)
    int *Ap = nullptr, *Aj = nullptr;
    double *Ax = nullptr;
    // diagonal-id column coding (SpMV): when the rows use at most 255 distinct
    // offsets col - row (stencil matrices), Ad[k] indexes d_off and the SpMV
    // reads one byte per entry instead of Aj's four; ndiag == 0: not coded
    uint8_t *Ad = nullptr;
    int *d_off = nullptr;
    int ndiag = 0;
    int max_off = 0;  // max |col - row| of the coded offsets
    // max |col - row| over the rows of the halo-free chunks [ich0, ich1) of a
    // distributed matrix (its whole row range on one rank: max_off)
    int max_off_int = 0;
    // windowed x (k_spmv_sell): when every 1024-row block's columns fall in a
    // span of at most WIN_CAP entries, d_win[2b], d_win[2b+1] = that span
    // [lo, hi) and the product stages x[lo, hi) in LDS; nullptr: not windowed
    int *d_win = nullptr;
    // the sliced copy of a windowed matrix that k_spmv_sell reads (build_windows):
    // each 1024-row block's rows sorted by length (stable, descending) into 16
    // slices of 64 rows; slice s keeps entry k of lane l's row at
    // s_meta[2s] + 64 k + l (s_ax) and its column, as a 16-bit offset from the
    // block's staging base (lo rounded down to even), in half (k & 1) of the
    // 32-bit word s_meta[2s] / 2 + 64 (k >> 1) + l (s_col); s_meta[2s + 1] is
    // the slice's longest row; s_row[64 w + l] = local row | length << 10 of
    // thread 64 w + l of its block
    double *s_ax = nullptr;
    uint32_t *s_col = nullptr, *s_row = nullptr;
    int *s_meta = nullptr;
    // device bytes held beside the CSR arrays (offset ids + table, window spans,
    // the sliced copy): lssp_amd_mat_bytes
    long long aux_bytes = 0;
    // k_spmv3's block streams, timed at upload (tune_spmv_streams); 0: the default 8
    int streams = 0;
    // distributed layout
    int n_global = 0, row0 = 0, nhalo = 0;
    // halo exchange plan: for each peer, indices (local) to send and the count to receive
    std::vector<int> send_peer, send_off, send_cnt;  // host plan
    std::vector<int> recv_peer, recv_off, recv_cnt;  // recv_off relative to the halo region
    int *d_send_idx = nullptr;
    double *d_send_buf = nullptr;
    int nsend = 0;
    // the longest run of 256-row chunks [ich0, ich1) none of whose rows reads a
    // halo column: their product does not wait for the halo round (spmv_halo)
    long ich0 = 0, ich1 = 0;
};

namespace lssp_amd {

struct TriSched {
    int n = 0, nnz = 0, nlevels = 0, unit = 0, upper = 0;
    int *perm = nullptr;   // position -> row, rows ordered by level
    int *rp = nullptr;     // [n+1] entry ranges in schedule order
    int *cols = nullptr;   // strict entries, in the reference's summation order
    double *vals = nullptr;
    double *diag = nullptr;  // per position (nullptr when unit)
    std::vector<int> level_ptr;  // host: schedule positions of each level
    int max_level_rows = 0;
    // block-pipelined schedule (tri_bp.cpp): contiguous row blocks of B >=
    // bandwidth rows in sweep order, each walked level by level by one workgroup
    int bp_B = 0, bp_nb = 0, bp_nsteps = 0;
    int *bp_perm = nullptr;  // schedule position -> row
    int *bp_pos = nullptr;   // row -> schedule position (the inverse of bp_perm)
    // packets v6 (k_tri_pk6: schedule-ordered shadow vectors between sweeps)
    int pk6_n = 0, pk6_ep = 4, pk6_rows = 256;
    int pk6_ext = 2;  // HBM operand loads per loader lane per packet (2, 3 or 4; build_packets6)
    int *pk6_blk = nullptr, *pk6_desc = nullptr, *pk6_idx = nullptr;
    uint32_t *pk6_rec = nullptr;
    mutable unsigned long long pk6_base = 0;
    unsigned long long *pk6_claim = nullptr;
    std::vector<int> h_pos;  // L factor: row -> schedule position (for the U factor's build)
};
constexpr int PK3_ROWS = 256;    // v6: rows per packet = compute lanes = loader lanes
constexpr int PK3_EXT = 4;       // v6: HBM x operands per packet row, at most (on average; the kernel
                                 // runs 2, 3 or 4 loads per lane, TriSched::pk6_ext; 2 before round 6)
constexpr int PK3_CAP = 4096;    // v6: packets per block (descriptors staged in LDS)

// ---- line sweeps of structured ILU(0) factors (linesweep.hip) ----------------
// A tile is 256 / P lines x P planes = 256 rows per step, P in {4, 8, 16}
// (chosen per factor, build_line_sweep): a compute wave's 64 lanes are P / 4
// groups of 256 / P lines, each lane holds 2 planes, 2 compute waves.  Squarer
// tiles = fewer tile-to-tile hand-offs on a sweep's critical path (216^3: 56
// hops with 64 x 4 tiles, 26 with 16 x 16).
enum { LT_KIN = 1, LT_JIN = 2, LT_KOUT = 4, LT_JOUT = 8, LT_SKIP = 16 };  // LT_SKIP: k_linef tile wholly off the grid
struct LineGeom {
    int nx = 0, ny = 0, nz = 0;
    std::vector<char> kin;  // plane k has its (k-1) neighbour
    bool unitL = true;
};
struct LineTile {  // one workgroup's unit of work, in its sweep's coordinates
    int j0, nj, k0, np;
    int flags;        // LT_*
    int T;            // levels (k_line2: padded to a whole number of two-level steps)
    int roff;         // (unused)
    int tk, tj;       // producer tiles of the k / j inputs (-1: none)
    int ut;           // L sweep: the mirror U tile (its rhs stream)
    long long cbase;  // first row of the tile in its sweep's streams
    long long ubase;  // L sweep: cbase of the mirror U tile
};
struct LineSweep {
    int nx = 0, ny = 0, nz = 0, ntiles = 0, tmax = 0, NA = 3;
    int P = 4;    // planes per tile
    int NJ = 64;  // lines per tile (k_line2: 16)
    int LV = 1;   // levels per workgroup step (k_line2: 2; its planes P/2.. run one level later)
    long rows_total = 0;
    LineTile *d_tiles = nullptr;
    double *d_coef = nullptr;
    unsigned long long *d_claim = nullptr;
    int *d_order = nullptr;  // k_line2: the tile of each claim (anti-diagonal order)
    mutable unsigned long long base = 0;
    std::vector<LineTile> h_tiles;
};
struct LineILU {
    LineGeom g;
    int P = 4, NJ = 64, LV = 1, W = 0, S = 0, tmax = 0, ntiles = 0;
    int kind = 0;  // 0: 7-point ILU(0) (linesweep.hip); 1: 7-point ILU(1) pattern (linefill.hip)
    LineSweep L, U;
    double *d_ustream = nullptr;  // the U sweep's rhs, written by the L sweep
    double *d_lstream = nullptr;  // the L sweep's rhs in its stream layout (k_line_rhs)
    // the natural-order vector d_lstream already holds (written with it by a
    // solver pass, launch_line_gather_ew): the next apply of exactly that rhs
    // skips its gather; every apply / sweep clears it
    mutable const double *lstream_of = nullptr;
    double *d_hk = nullptr, *d_hj = nullptr;  // hand-off buffers (armed with TRI_SENTINEL)
    long hk_stride = 0, hj_stride = 0, hk_n = 0, hj_n = 0;
    // the U sweep's tail product (launch_line_apply_spmv): U tiles finished per
    // tile row (monotonic), natural plane -> L tile row, chunk claims
    unsigned *d_kdone = nullptr;
    int *d_kof = nullptr;
    unsigned long long *d_tclaim = nullptr;
    mutable unsigned long long tbase = 0;
    mutable unsigned kepoch = 0;
    // kind 1 on a small 2-D grid (linefill.hip k_lineg): ONE workgroup, lines on
    // lanes; level-major streams [level][S, SE, W(, diag), rhs][lane] per sweep
    int g2 = 0, g2fill = 0, g2V = 0, g2NYP = 0, g2NCL = 0, g2NCU = 0;
    double *d_g2L = nullptr, *d_g2U = nullptr;
};

}  // namespace lssp_amd

struct lssp_amd_ilu {
    lssp_amd_ctx *ctx = nullptr;
    int n = 0;
    std::vector<int> Lp, Lj, Up, Uj;  // host copies (for get_factors / tests)
    std::vector<double> Lx, Ux;
    lssp_amd::TriSched lower, upper;
    double *d_cache = nullptr;  // L sweep output, kept all-sentinel between applies
    // packet sweeps: schedule-ordered shadows {L out, L out', U out, U out'} and the
    // apply counter selecting the buffer pair (trisolve.hip launch_ilu_apply)
    mutable double *d_sh[4] = {nullptr, nullptr, nullptr, nullptr};
    mutable double *d_rperm = nullptr;  // the apply's rhs in L order
    mutable unsigned epoch = 0;
    lssp_amd::LineILU line;  // structured factors: line sweeps (ntiles > 0)
    std::mutex sync_free_mu;  // the sync-free arrays, built on first use (ensure_sync_free)
    double setup_seconds = 0;
};

namespace lssp_amd {

// ---- error handling --------------------------------------------------------
#define LSSP_HIP(call)                                                                    \
    do {                                                                                  \
        hipError_t e_ = (call);                                                           \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "lssp_amd: HIP error %s at %s:%d\n", hipGetErrorString(e_), \
                    __FILE__, __LINE__);                                                  \
            return LSSP_AMD_EHIP;                                                         \
        }                                                                                 \
    } while (0)

#define LSSP_TRY(call)               \
    do {                             \
        int s_ = (call);             \
        if (s_ != LSSP_AMD_OK) return s_; \
    } while (0)

// ---- kernel launchers (kernels.hip) ------------------------------------------
enum Epi { EPI_MXY = 0, EPI_AMXY, EPI_AXPBY, EPI_AMX };  // see spmv kernel
int build_diag_ids(lssp_amd_mat *M, const int *Ap, const int *Aj);
int build_windows(lssp_amd_mat *M, const int *Ap, const int *Aj, const double *Ax);
int tune_spmv_streams(lssp_amd_ctx *c, lssp_amd_mat *M);
constexpr int WIN_ROWS = 1024, WIN_CAP = 16384;
int launch_spmv(lssp_amd_ctx *c, const lssp_amd_mat *A, int epi, double alpha, const double *x,
                double beta, const double *y, double *z, int nred, const double *w0,
                const double *w1, long cb = 0, long ce = -1);  // chunks [cb, ce); ce < 0: all
// elementwise + optional partials; kinds in kernels.hip (EwKind)
struct Ew {
    int kind = 0;
    long n = 0;
    double a = 0, b = 0;
    const double *x = nullptr, *y = nullptr, *u = nullptr, *v = nullptr;
    double *out0 = nullptr, *out1 = nullptr;
    const double *scal = nullptr;   // device scalars
    int nred = 0;
    const double *r0a = nullptr, *r0b = nullptr, *r1a = nullptr, *r1b = nullptr;
    const double *r2a = nullptr, *r2b = nullptr, *r3a = nullptr, *r3b = nullptr;  // nred 3, 4
    const double *vbase = nullptr;  // GMRES basis [k][n]
    int k = 0;
    int sidx = 0;                   // scalar index for device-scalar kinds
    int pslot = 0;                  // first partial row the pass's reductions write
};
int launch_ew(lssp_amd_ctx *c, const Ew &e);
// x = y (vector.cxx:73-83): 16-byte vector copy when both are 16-byte aligned
int launch_copy(lssp_amd_ctx *c, double *x, const double *y, long n);
int launch_stream_read(lssp_amd_ctx *c, const double *x, long n, double *sink);

// finish a reduction whose level-1 partials (tree) or operands (serial) are set:
// tree: level-2 over nslot partial rows of C entries; then the finalize program
int launch_reduce_tree(lssp_amd_ctx *c, long C, int nslot, const Fin &f, int slot0 = 0);  // partial rows slot0 ..
// CG's vector updates with the preceding reduction's level 2 folded in (k_cg_fused)
// CGF_R / CGF_PX / CGF_X: the x update x += alpha p is deferred from the x/r
// pass into the next p pass (which reads p anyway), or a batch's last pass
// CGF_X; stamp = the S_DONE value (FIN_CG_RES_RHO_B) that the stop test of
// this pass's own reduction writes -- a guard equal to it still runs the
// pass's x update, any other nonzero guard skips the pass
enum { CGF_P = 0, CGF_XR = 1, CGF_R = 2, CGF_PX = 3, CGF_X = 4 };
int launch_cg_fused(lssp_amd_ctx *c, int kind, long n, double *x, double *p, double *r, const double *z,
                    const double *q, int pin_slot, int pout_slot, const Fin &f, int stamp = 0);
// serial: sums of products a_k[i]*b_k[i] in index order (== vector.cxx:123-133)
int launch_reduce_serial(lssp_amd_ctx *c, long n, int nslot, const double *const *a,
                         const double *const *b, const Fin &f, const double *carry = nullptr);
int launch_finalize(lssp_amd_ctx *c, const double *sums, int nslot, const Fin &f);
int launch_fill(lssp_amd_ctx *c, double *x, long n, uint64_t bits);
int launch_trisolve(lssp_amd_ctx *c, const TriSched &t, const double *rhs, double *x,
                    double *reset);
constexpr int BP_RING = 4096;  // LDS ring of recently computed values (32 KB)
// k_tri_pk6's LDS operand array: the value ring [0, BP_RING), a +0.0 pad slot
// at BP_RING, then the two buffers of landed HBM operands (PK3_EXT per packet
// row of 256).  Byte offset of entry base + par * buffer + k:
constexpr int pk6_xs_off(int base, int par, int k) { return 8 * (base + par * 256 * PK3_EXT + k); }
int build_bp_schedule(lssp_amd_ctx *c, int n, const std::vector<int> &Tp, const std::vector<int> &Tj,
                      const std::vector<double> &Tx, bool upper, const std::vector<int> &lev,
                      TriSched &t, const TriSched *prod = nullptr);
int build_packets6(int n, const std::vector<int> &perm, const std::vector<int> &pos, const std::vector<int> &rp,
                   const int *cols, const double *vals,
                   const std::vector<double> &diag, bool unit, const std::vector<int> &step_pos,
                   const std::vector<int> &blk_step, int nb, long B, const std::vector<int> &rhs_index,
                   TriSched &t);
int launch_ilu_apply(lssp_amd_ctx *c, const lssp_amd_ilu *M, double *x, const double *rhs);
int launch_pack(lssp_amd_ctx *c, const int *idx, const double *x, double *buf, int n);
int launch_sum_ranks(lssp_amd_ctx *c, int nslot, const Fin &f);

long num_chunks(long n);
int ensure_part(lssp_amd_ctx *c, long C);

// ---- host pieces ---------------------------------------------------------------
// the drivers' messages (the reference's lssp_printf lines): to the hook set
// with lssp_amd_set_print, else to stdout (flushed, as lssp_printf does)
int lprint(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
double wall_time();  // seconds, lssp_get_time() (utils.cxx:40-46)
// setup phase timings to stderr when LSSP_AMD_SETUP_TIMES=1 (tuning aid)
void setup_mark(const char *phase);
// a sub-phase's own duration (LSSP_AMD_SETUP_TIMES; thread-safe: no shared clock)
struct SetupTimer {
    double t0;
    SetupTimer();
    void mark(const char *phase);
};
// host setup loops: f(lo, hi) over [0, n) in contiguous chunks on up to 16
// threads (OMP_NUM_THREADS / the hardware concurrency, whichever is smaller)
int host_threads();  // worker threads for host setup: <= 16, <= OMP_NUM_THREADS
// [0, n) cut into at most 16 contiguous ranges of >= grain items, one thread each
void parallel_for(long n, const std::function<void(long, long)> &f, long grain = 4096);

// ILU setup (ilu_setup.cpp), exact restatement of pc-iluk.cxx / pc-ilut.cxx
struct HostCSR {
    int n = 0, ncols = 0;
    std::vector<int> Ap, Aj;
    std::vector<double> Ax;
};
void sort_columns(HostCSR &A);
// c != nullptr: ILUK's numeric ILU(0) runs on c's GPU (ilu_factor.hip), bitwise
// the host restatement (LSSP_AMD_ILU_HOST=1 selects the host one); ILUT stays
// on the host (pc-ilut.cxx:51-286 is sequential by row)
void ilu_factor(lssp_amd_ctx *c, int kind, HostCSR &&A, int level, double tol, int p, int blk, HostCSR &L,
                HostCSR &U, int *status);
int ilu0_factor_gpu(lssp_amd_ctx *c, int n, int blk, const std::vector<int> &Ap, const std::vector<int> &Aj,
                    std::vector<double> &Ax);
int build_trisched(lssp_amd_ctx *c, int n, const std::vector<int> &Tp, const std::vector<int> &Tj,
                   const std::vector<double> &Tx, bool upper, TriSched &t, const TriSched *prod = nullptr,
                   bool packets = true, bool arrays = true, std::vector<int> *lev_in = nullptr);
// the rows' dependency levels alone (build_trisched's first pass; lev_in above
// takes them precomputed, e.g. on another thread)
int tri_levels(int n, const std::vector<int> &Tp, const std::vector<int> &Tj, bool upper, std::vector<int> &lev);
// line sweeps (linesweep.hip): LSSP_AMD_EUNSUPPORTED when the factors are not
// the structured ILU(0) of a 5-/7-point grid
int build_line_sweep(lssp_amd_ctx *c, int n, const std::vector<int> &Lp, const std::vector<int> &Lj,
                     const std::vector<double> &Lx, const std::vector<int> &Up, const std::vector<int> &Uj,
                     const std::vector<double> &Ux, LineILU &li);
int line_rearm(lssp_amd_ctx *c, LineILU &li);
// linefill.hip: the 7-point ILU(1) pattern (EUNSUPPORTED when the factor is not it)
int build_linefill(lssp_amd_ctx *c, int n, const std::vector<int> &Lp, const std::vector<int> &Lj,
                   const std::vector<double> &Lx, const std::vector<int> &Up, const std::vector<int> &Uj,
                   const std::vector<double> &Ux, LineILU &li);
int launch_linefill_apply(lssp_amd_ctx *c, const LineILU &li, double *x, const double *rhs);
struct LineTail;
// small 2-D grids on one workgroup (linefill.hip): cl / cu hold the L / U rows in
// sweep order, components S, (SE,) W (, diag); mode 0 apply, 1 L, 2 U
int build_lineg(lssp_amd_ctx *c, const LineGeom &g, int fill, int ncl, const std::vector<double> &cl,
                const std::vector<double> &cu, LineILU &li);
int launch_lineg(lssp_amd_ctx *c, const LineILU &li, int mode, double *x, const double *rhs);
constexpr int G2_MAXNY = 256;  // k_lineg: lines (lanes) of one workgroup
// k_lineg addresses its streams and output through buffer resources: every
// byte offset (and the dropped-store offset 2^30) within 32 bits
inline bool lineg_fits(const LineGeom &g, int fill)
{
    const long nyp = (g.ny + 63) / 64 * 64, V = g.nx + (fill ? 2L : 1L) * (g.ny - 1);
    return (long)g.nx * g.ny * 8 < (1L << 30) && V * 5 * nyp * 8 + 1024 < (1L << 30);
}  // linesweep_dev.h
int launch_linefill_apply_tail(lssp_amd_ctx *c, const LineILU &li, double *x, const double *rhs, const LineTail &T,
                               long *tail_waves);
int launch_linefill_sweep(lssp_amd_ctx *c, const LineILU &li, int which, double *x, const double *rhs);
void free_line_sweep(LineILU &li);
int launch_line_apply(lssp_amd_ctx *c, const LineILU &li, double *x, const double *rhs);
// the apply followed by z = op(A x) (+ fused dots), the product run by the U
// sweep's workgroups as planes of x become final (k_line2 tail); results are
// bitwise launch_line_apply + launch_spmv.  EUNSUPPORTED when A is not a coded
// single-rank stencil of the factor's grid (the caller then runs the two)
int launch_line_apply_spmv(lssp_amd_ctx *c, const LineILU &li, double *x, const double *rhs, const lssp_amd_mat *A,
                           int epi, double alpha, double beta, const double *y, double *z, int nred,
                           const double *w0, const double *w1);
// the same on P ranks: the tail computes the halo-free chunks [ich0, ich1)
// only; the halo round and the boundary chunks follow it (spmv_boundary)
int spmv_boundary(lssp_amd_ctx *c, const lssp_amd_mat *A, int epi, double alpha, double *x, double beta,
                  const double *y, double *z, int nred, const double *w0, const double *w1);
int launch_line_sweep(lssp_amd_ctx *c, const LineILU &li, int which, double *x, const double *rhs);
// A BiCGSTAB vector pass fused with the next apply's rhs gather: out (natural
// order, n rows) = op(x, y, out) and the same values into the L sweep's
// stream, which the next launch_line_apply of rhs == out then reads as is.
// op: GEW_BICG_P out = x + beta*(out - omega*y), GEW_BICG_S out = x - alpha*y
// (scalars from scal; k_ew's EW_BICG_P / EW_BICG_S arithmetic).  Eligible
// (line_gather_ew_ok) for the k_line2 sweeps of an n-row grid factor.
enum { GEW_BICG_P = 1, GEW_BICG_S = 2 };
bool line_gather_ew_ok(const LineILU &li, long n);
int launch_line_gather_ew(lssp_amd_ctx *c, const LineILU &li, int op, const double *x, const double *y, double *out,
                          const double *scal);
void free_trisched(TriSched &t);

// reductions with the context's mode; result left in d_sums / scal per Fin
int finish_reduce(lssp_amd_ctx *c, long n, int nslot, const double *const *a,
                  const double *const *b, const Fin &f);
int reduce_dots(lssp_amd_ctx *c, long n, int nslot, const double *const *a,
                const double *const *b, const Fin &f);
// multi-rank: all-gather rank sums and sum in rank order, then the finalize
int comm_allgather_sums(lssp_amd_ctx *c, int nslot);
// recv (nranks * bytes, rank order) = every rank's send (bytes), through the
// context's transport (RCCL or the host hooks)
int comm_allgather(lssp_amd_ctx *c, const void *send, void *recv, long bytes);
int comm_gather_int(lssp_amd_ctx *c, int v, std::vector<int> &all);  // collective, rank order
// serial mode, P ranks: receive the running sums of rank-1 (zeros on rank 0)
// into c->d_carry / pass this rank's on to rank+1
int comm_carry_in(lssp_amd_ctx *c);
int comm_carry_out(lssp_amd_ctx *c);
int halo_exchange(const lssp_amd_mat *A, double *x);
// halo round + product, the halo-free chunks overlapped with the round
int spmv_halo(lssp_amd_ctx *c, const lssp_amd_mat *A, int epi, double alpha, double *x, double beta,
              const double *y, double *z, int nred, const double *w0, const double *w1);
int comm_destroy(lssp_amd_ctx *c);

// The canonical level-1 halving tree of one wave: lane 0 gets
// (((v0 + v32) + (v16 + v48)) + ...), the pairs of an xor butterfly over 32,
// 16, 8, 4, 2, 1 -- evaluated for lane 0 only: the 32- and 16-lane steps by
// v_permlane32_swap / v_permlane16_swap, the 8, 4, 2, 1 steps by DPP row
// shifts (row_shl:k), instead of six dependent ds_bpermute round trips per
// half.  Lane 0 adds the same operands in the same pairs, so its value is
// bitwise the butterfly's; the other lanes hold partial sums (every caller
// reads lane 0).  -DWAVE_SUM_BPERM restores the butterfly (A/B).
__device__ __forceinline__ double wave_sum_l0(double v)
{
#ifdef WAVE_SUM_BPERM
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = v + __shfl_xor(v, off, 64);
    return v;
#else
    auto split = [](double x, unsigned &lo, unsigned &hi) {
        const unsigned long long b = (unsigned long long)__double_as_longlong(x);
        lo = (unsigned)b;
        hi = (unsigned)(b >> 32);
    };
    auto join = [](unsigned lo, unsigned hi) {
        return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
    };
    unsigned lo, hi;
    split(v, lo, hi);
    {  // lanes 0..31 <- lanes 32..63
        const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
        const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
        v = v + join(a[1], b[1]);
    }
    split(v, lo, hi);
    {  // lanes 0..15 <- lanes 16..31
        const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
        const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
        v = v + join(a[1], b[1]);
    }
    // lanes l <- l + k inside each 16-lane row (row_shl:k = 0x100 + k)
    split(v, lo, hi);
    v = v + join((unsigned)__builtin_amdgcn_update_dpp((int)lo, (int)lo, 0x108, 0xf, 0xf, false),
                 (unsigned)__builtin_amdgcn_update_dpp((int)hi, (int)hi, 0x108, 0xf, 0xf, false));
    split(v, lo, hi);
    v = v + join((unsigned)__builtin_amdgcn_update_dpp((int)lo, (int)lo, 0x104, 0xf, 0xf, false),
                 (unsigned)__builtin_amdgcn_update_dpp((int)hi, (int)hi, 0x104, 0xf, 0xf, false));
    split(v, lo, hi);
    v = v + join((unsigned)__builtin_amdgcn_update_dpp((int)lo, (int)lo, 0x102, 0xf, 0xf, false),
                 (unsigned)__builtin_amdgcn_update_dpp((int)hi, (int)hi, 0x102, 0xf, 0xf, false));
    split(v, lo, hi);
    v = v + join((unsigned)__builtin_amdgcn_update_dpp((int)lo, (int)lo, 0x101, 0xf, 0xf, false),
                 (unsigned)__builtin_amdgcn_update_dpp((int)hi, (int)hi, 0x101, 0xf, 0xf, false));
    return v;
#endif
}

}  // namespace lssp_amd
