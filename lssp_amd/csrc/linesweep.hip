// linesweep.hip -- ILU(0) triangular sweeps of a structured (5-/7-point grid)
// factor, lines in lanes (solver-tri.cxx:4-46, the same arithmetic bit for bit).
//
// When a factor's strict rows are exactly the grid neighbours -- L row r holds
// {r-nx*ny, r-nx, r-1} (those that exist, ascending, unit diagonal last), U row
// r holds {r, r+1, r+nx, r+nx*ny} -- the sweep is a 3-D wavefront: row
// (i, j, k) needs (i-1, j, k), (i, j-1, k) and (i, j, k-1).  The U sweep is the
// same recurrence in mirrored coordinates (i' = nx-1-i, ...), and its
// descending summation order (solver-tri.cxx:38) is then again k'-1, j'-1, i'-1.
//
// Decomposition.  A TILE is nj <= NJ consecutive lines (j) of np <= P
// consecutive planes (k), P * NJ = 256 (G = 64 / NJ lane groups); one
// workgroup runs it.  A compute wave's lane (g, l) owns line j0+l of the
// group's planes; at step s it computes, for each of its planes p, row
// i = s - l - p.  Then
//   * (i-1, j, k):   the lane's own value of the previous step (a register);
//   * (i, j-1, k):   line l-1's value of the previous step (DPP: wave_shr:1,
//                    or row_shr:1 when the groups are the 16-lane DPP rows);
//   * (i, j, k-1):   the lane's own value of plane p-1 at the previous step
//                    (the group's first plane: LDS, written by the group or
//                    wave holding plane p-1);
// so a step is pure register arithmetic plus one LDS read.  Across tiles the
// two boundary streams (plane np-1 -> the next tile in k, line nj-1 -> the next
// tile in j) go through HBM hand-off buffers with the value as the flag
// (TRI_SENTINEL), indexed by the consumer's step so both sides access them
// coalesced.  A path through the grid crosses W + S tiles instead of nz
// planes: squarer tiles (16 x 16 instead of 64 x 4) halve W + S at the same
// 256 rows per step.
//
// Roles (one barrier per step, LDS only):
//   waves 0..CW-1   compute: read the step's slot, write results to LDS;
//   waves 1..NL     loaders: LDS-DMA (global_load_lds) of the step's
//                   coefficient block (and rhs) D steps ahead, steps q = w mod NL;
//   wave NL+1       poller: LDS-DMA sc1 reads of the hand-off inputs DH steps
//                   ahead; checks them, re-polls what is not yet written;
//   wave NL+2       storer: results -> HBM (natural-order x, the U sweep's rhs
//                   stream, hand-off outputs with sc1 stores), and re-arms the
//                   consumed hand-off inputs with the sentinel.
// Only the compute wave is on the critical path; every VMEM queue (vmcnt is
// in order per wave) belongs to one role with one lead, so no wait ever covers
// another role's slow operations.
//
// Layouts (host, build_line_sweep): per tile, per step, per plane, the rows
// valid at that step (a contiguous lane range [lo, hi]), each row's NA
// coefficients {c_k, c_j, c_i(, diag)} together; steps padded to an even row
// count (16-byte blocks).  The L sweep writes its output into the U
// sweep's rhs stream of the same compact layout (tile, step, plane and lane
// mirrored), so the U sweep reads its rhs as one more coalesced block.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "internal.h"
#include "linesweep_dev.h"

namespace lssp_amd {


// ---------------------------------------------------------------------------
// host: detection of the grid structure
// ---------------------------------------------------------------------------
// kin[k] = plane k has its (k-1) neighbour (false at k = 0 and at block-Jacobi cuts)
static bool detect_grid(int n, const std::vector<int> &Lp, const std::vector<int> &Lj, const std::vector<double> &Lx,
                        const std::vector<int> &Up, const std::vector<int> &Uj, LineGeom &g)
{
    long offs[3];
    int no = 0;
    for (int r = 0; r < n; r++) {
        const int a = Lp[r], b = Lp[r + 1];
        if (b - a < 1 || b - a > 4 || Lj[b - 1] != r) return false;
        for (int k = a; k < b - 1; k++) {
            const long d = (long)r - Lj[k];
            if (d <= 0) return false;
            bool seen = false;
            for (int q = 0; q < no; q++) seen |= offs[q] == d;
            if (!seen) {
                if (no == 3) return false;
                offs[no++] = d;
            }
        }
    }
    std::sort(offs, offs + no);
    if (no < 2 || offs[0] != 1) return false;
    long nx = offs[1], plane = no == 3 ? offs[2] : n;
    if (plane % nx || n % plane) return false;
    g.nx = (int)nx;
    g.ny = (int)(plane / nx);
    g.nz = (int)(n / plane);
    if (g.nx < 2 || g.ny < 8) return false;
    g.kin.assign(g.nz, 0);
    for (int k = 1; k < g.nz; k++) {
        const long r = (long)k * plane;  // row (0, 0, k): its only candidate neighbour is k-1
        g.kin[k] = (Lp[r + 1] - Lp[r] == 2) ? 1 : 0;
    }
    g.unitL = true;
    for (int k = 0; k < g.nz; k++)
        for (int j = 0; j < g.ny; j++)
            for (int i = 0; i < g.nx; i++) {
                const long r = ((long)k * g.ny + j) * g.nx + i;
                long want[3];
                int m = 0;
                if (k > 0 && g.kin[k]) want[m++] = r - plane;
                if (j > 0) want[m++] = r - nx;
                if (i > 0) want[m++] = r - 1;
                const int a = Lp[r], b = Lp[r + 1];
                if (b - a - 1 != m) return false;
                for (int q = 0; q < m; q++)
                    if (Lj[a + q] != want[q]) return false;
                g.unitL &= Lx[b - 1] == 1.0;
                m = 0;
                if (i < g.nx - 1) want[m++] = r + 1;
                if (j < g.ny - 1) want[m++] = r + nx;
                if (k < g.nz - 1 && g.kin[k + 1]) want[m++] = r + plane;
                const int c = Up[r], e = Up[r + 1];
                if (e - c - 1 != m || Uj[c] != r) return false;
                for (int q = 0; q < m; q++)
                    if (Uj[c + 1 + q] != want[q]) return false;
            }
    return true;
}

// k_line2's plane skew: compute wave w owns planes 4w .. 4w+3 and runs
// (LV-1) w levels later, so the k-input of a wave's first plane is one whole
// step (LV levels) old
static inline int line_sigma(int LV, int P, int p) { return LV >= 2 ? (LV - 1) * (p / 4) : 0; }

// rows of a tile (nj lines, np planes) valid at level s, plane p: lanes [lo, hi]
// (row i = s - l - p - sigma(p))
static inline void step_range(int nx, int nj, int np, int s, int p, int sg, int &lo, int &hi)
{
    if (p >= np) {
        lo = 0;
        hi = -1;
        return;
    }
    lo = std::max(0, s - p - sg - nx + 1);
    hi = std::min(nj - 1, s - p - sg);
}

// coefficients of one sweep in that sweep's row order (row r_sweep = r for L,
// n-1-r for U), NA per row: component a = 0 (k-1), 1 (j-1), 2 (i-1), 3
// (diagonal); a missing neighbour gets +0.0 (its operand is +0.0 too)
struct CoefSrc {
    std::vector<double> c;
    int NA = 3;
    void build(const std::vector<int> &Tp, const std::vector<int> &Tj, const std::vector<double> &Tx, bool upper,
               long n, long nx, long plane, int na)
    {
        NA = na;
        c.assign((size_t)n * NA, 0.0);
        parallel_for(n, [&](long r0, long r1) {
        for (long r = r0; r < r1; r++) {
            double *row = c.data() + (size_t)(upper ? n - 1 - r : r) * NA;
            const int b = Tp[r], e = Tp[r + 1];
            if (NA == 4) row[3] = upper ? Tx[b] : Tx[e - 1];
            for (int q = upper ? b + 1 : b; q < (upper ? e : e - 1); q++) {
                const long off = upper ? Tj[q] - r : r - Tj[q];
                const int a = off == plane ? 0 : off == nx ? 1 : 2;  // detect_grid: off is one of 1, nx, plane
                row[a] = Tx[q];
            }
        }
        });
    }
    double get(long r_sweep, int a) const { return c[(size_t)r_sweep * NA + a]; }
};

static int build_tiles(const LineGeom &g, int P, int NJ, int LV, int W, std::vector<LineTile> &tiles, int &S)
{
    (void)NJ;
    // plane segments between cuts, cut into tiles of <= P planes
    std::vector<std::pair<int, int>> kt;  // (k0, np)
    for (int k = 0; k < g.nz;) {
        int e = k + 1;
        while (e < g.nz && g.kin[e]) e++;
        for (int k0 = k; k0 < e; k0 += P) kt.push_back({k0, std::min(P, e - k0)});
        k = e;
    }
    S = (int)kt.size();
    tiles.assign((size_t)S * W, LineTile{});
    const int base = g.ny / W, extra = g.ny % W;
    for (int K = 0; K < S; K++) {
        int j0 = 0;
        for (int J = 0; J < W; J++) {
            LineTile &t = tiles[(size_t)K * W + J];
            t.j0 = j0;
            t.nj = base + (J < extra ? 1 : 0);
            j0 += t.nj;
            t.k0 = kt[K].first;
            t.np = kt[K].second;
            const bool kin = t.k0 > 0 && g.kin[t.k0];
            t.flags = (kin ? LT_KIN : 0) | (J > 0 ? LT_JIN : 0) | (J < W - 1 ? LT_JOUT : 0);
            t.T = g.nx + t.nj + t.np - 2 + line_sigma(LV, P, t.np - 1);
            t.T = (t.T + LV - 1) / LV * LV;
            t.tk = kin ? (K - 1) * W + J : -1;
            t.tj = J > 0 ? K * W + J - 1 : -1;
        }
    }
    for (int K = 0; K + 1 < S; K++)
        for (int J = 0; J < W; J++)
            if (tiles[(size_t)(K + 1) * W + J].flags & LT_KIN) tiles[(size_t)K * W + J].flags |= LT_KOUT;
    return LSSP_AMD_OK;
}

// Stream layout of one sweep: per tile, per step s, a block of P planes x nj
// rows (row (p, l) at p*nj + l; rows not valid at that step are +0.0), each
// row's NA coefficients {c_k, c_j, c_i(, diag)} together.  Fixed strides keep
// every role's addressing to a per-lane base plus immediate offsets.
static int upload_sweep(lssp_amd_ctx *c, const LineGeom &g, const std::vector<LineTile> &tiles, const CoefSrc &src,
                        int NA, LineSweep &ls)
{
    const int nx = g.nx, P = ls.P, LV = ls.LV;
    std::vector<LineTile> tt = tiles;
    long rows_total = 0;
    int tmax = 0;
    for (LineTile &t : tt) {
        t.roff = 0;
        t.cbase = rows_total;
        rows_total += (long)t.T * P * t.nj;
        tmax = std::max(tmax, t.T);
    }
    // + slack for the loaders' whole 1 KB pieces past the last block
    const long slack = 16 * 1024 / 8;
    std::vector<double> coef((size_t)rows_total * NA + slack, 0.0);
    parallel_for((long)tt.size(), [&](long t0, long t1) {
    for (long ti = t0; ti < t1; ti++) {
        const LineTile &t = tt[ti];
        for (int s = 0; s < t.T; s++) {
            double *blk = coef.data() + (size_t)(t.cbase + (long)s * P * t.nj) * NA;
            for (int p = 0; p < t.np; p++) {
                int lo, hi;
                const int sg = line_sigma(LV, P, p);
                step_range(nx, t.nj, t.np, s, p, sg, lo, hi);
                for (int l = lo; l <= hi; l++) {
                    const long i = s - l - p - sg;
                    const long r = ((long)(t.k0 + p) * g.ny + (t.j0 + l)) * nx + i;
                    for (int a = 0; a < NA; a++) blk[(size_t)(p * t.nj + l) * NA + a] = src.get(r, a);
                }
            }
        }
    }
    });
    ls.nx = g.nx;
    ls.ny = g.ny;
    ls.nz = g.nz;
    ls.ntiles = (int)tt.size();
    ls.tmax = tmax;
    ls.rows_total = rows_total;
    ls.NA = NA;
    LSSP_HIP(hipMalloc(&ls.d_tiles, sizeof(LineTile) * tt.size()));
    LSSP_HIP(hipMemcpy(ls.d_tiles, tt.data(), sizeof(LineTile) * tt.size(), hipMemcpyHostToDevice));
    LSSP_HIP(hipMalloc(&ls.d_coef, sizeof(double) * coef.size()));
    LSSP_HIP(hipMemcpy(ls.d_coef, coef.data(), sizeof(double) * coef.size(), hipMemcpyHostToDevice));
    LSSP_HIP(hipMalloc(&ls.d_claim, sizeof(unsigned long long)));
    LSSP_HIP(hipMemset(ls.d_claim, 0, sizeof(unsigned long long)));
    if (LV >= 2) {
        // k_line2 claims tiles by anti-diagonal J + K (then K): a claimed tile's
        // producers (J-1, K) and (J, K-1) were claimed before it, and the
        // workgroups hold tiles of the advancing wavefront instead of tiles
        // many hops ahead of it (row order: the first 256 claims of a 216^3 sweep
        // reach K = 18, whose tiles wait ~30 hops before they can start).
        const int W = (g.ny + ls.NJ - 1) / ls.NJ, nt = (int)tt.size();
        std::vector<int> ord(nt);
        for (int q = 0; q < nt; q++) ord[q] = q;
        std::stable_sort(ord.begin(), ord.end(), [W](int x, int y) {
            const int dx = x % W + x / W, dy = y % W + y / W;
            return dx != dy ? dx < dy : x < y;
        });
        LSSP_HIP(hipMalloc(&ls.d_order, sizeof(int) * nt));
        LSSP_HIP(hipMemcpy(ls.d_order, ord.data(), sizeof(int) * nt, hipMemcpyHostToDevice));
    }
    ls.h_tiles = std::move(tt);
    return LSSP_AMD_OK;
}

// tiles of k_line2: 8 planes x 16 lines, two levels per workgroup step (round 3's
// k_line -- 256 rows and one level per step, 64 x 4 / 32 x 8 / 16 x 16 tiles --
// was removed in round 6 after two rounds as an A/B option only)
static void line_plan(const LineGeom &, int &P, int &NJ, int &LV)
{
    // (the kernel is generic in P = 4 x compute waves; 16-plane tiles measured
    // slower: 216^3 apply 666 against 593 us, 512^3 4.72 against 4.59 ms,
    // profiles/r04/r04e_*, r04f_line2_512_p8_p16.txt)
    P = 8;
    NJ = 16;
    LV = 2;  // levels per workgroup step (4 measured slower)
}

int build_line_sweep(lssp_amd_ctx *c, int n, const std::vector<int> &Lp, const std::vector<int> &Lj,
                     const std::vector<double> &Lx, const std::vector<int> &Up, const std::vector<int> &Uj,
                     const std::vector<double> &Ux, LineILU &li)
{
    const char *env = getenv("LSSP_AMD_LINE");
    if (env && !atoi(env)) return LSSP_AMD_EUNSUPPORTED;
    LineGeom g;
    if (!detect_grid(n, Lp, Lj, Lx, Up, Uj, g)) return build_linefill(c, n, Lp, Lj, Lx, Up, Uj, Ux, li);
    {
        // a small 2-D grid (exam.cxx's 5-point Poisson): one workgroup, lines on
        // lanes (linefill.hip k_lineg); LSSP_AMD_LINEG=0 keeps the tiles
        const char *e = getenv("LSSP_AMD_LINEG");
        if (g.nz == 1 && g.ny <= G2_MAXNY && lineg_fits(g, 0) && !(e && !atoi(e))) {
            const long plane = (long)g.nx * g.ny;
            const int ncl = g.unitL ? 2 : 3;
            CoefSrc sl, su;
            sl.build(Lp, Lj, Lx, false, n, g.nx, plane, g.unitL ? 3 : 4);
            su.build(Up, Uj, Ux, true, n, g.nx, plane, 4);
            // k_lineg's components: S, W (, diag) = CoefSrc's 1, 2 (, 3)
            std::vector<double> cl((size_t)n * ncl), cu((size_t)n * 3);
            for (long r = 0; r < n; r++) {
                for (int k = 0; k < ncl; k++) cl[r * ncl + k] = sl.get(r, 1 + k);
                for (int k = 0; k < 3; k++) cu[r * 3 + k] = su.get(r, 1 + k);
            }
            return build_lineg(c, g, 0, ncl, cl, cu, li);
        }
    }
    int P, NJ, LV;
    line_plan(g, P, NJ, LV);
    const int W = (g.ny + NJ - 1) / NJ;
    std::vector<LineTile> Lt;
    int S = 0;
    LSSP_TRY(build_tiles(g, P, NJ, LV, W, Lt, S));
    // U tiles: exact mirrors of the L tiles (U tile (W-1-J, S-1-K) <-> L tile (J, K))
    std::vector<LineTile> Ut(Lt.size());
    for (int K = 0; K < S; K++)
        for (int J = 0; J < W; J++) {
            const LineTile &l = Lt[(size_t)K * W + J];
            const int Kp = S - 1 - K, Jp = W - 1 - J;
            LineTile &u = Ut[(size_t)Kp * W + Jp];
            u = l;
            u.j0 = g.ny - l.j0 - l.nj;
            u.k0 = g.nz - l.k0 - l.np;
            // U tile Kp takes its k-input from U tile Kp-1 = L tile K+1's k-output side
            const bool kin = K + 1 < S && (Lt[(size_t)(K + 1) * W + J].flags & LT_KIN);
            const bool kout = (l.flags & LT_KIN) != 0;
            u.flags = (kin ? LT_KIN : 0) | (kout ? LT_KOUT : 0) | (Jp > 0 ? LT_JIN : 0) | (Jp < W - 1 ? LT_JOUT : 0);
            u.tk = kin ? (Kp - 1) * W + Jp : -1;
            u.tj = Jp > 0 ? Kp * W + Jp - 1 : -1;
        }
    const long plane = (long)g.nx * g.ny;
    // coefficients per row: c_k, c_j, c_i (unit L), + diag
    const int NAD = 4;
    const int NAL = g.unitL ? 3 : NAD;
    CoefSrc cl, cu;
    cl.build(Lp, Lj, Lx, false, n, g.nx, plane, NAL);
    cu.build(Up, Uj, Ux, true, n, g.nx, plane, NAD);
    li.g = g;
    li.P = li.L.P = li.U.P = P;
    li.NJ = li.L.NJ = li.U.NJ = NJ;
    li.LV = li.L.LV = li.U.LV = LV;
    li.W = W;
    li.S = S;
    LSSP_TRY(upload_sweep(c, g, Lt, cl, NAL, li.L));
    LineGeom gu = g;
    for (int k = 0; k < g.nz; k++) gu.kin[k] = k > 0 ? g.kin[g.nz - k] : 0;
    LSSP_TRY(upload_sweep(c, gu, Ut, cu, NAD, li.U));
    // the L sweep writes its output into the U sweep's rhs stream: per L tile
    // the base row of its mirror U tile
    for (int K = 0; K < S; K++)
        for (int J = 0; J < W; J++) {
            LineTile &l = li.L.h_tiles[(size_t)K * W + J];
            l.ut = (S - 1 - K) * W + (W - 1 - J);
            l.ubase = li.U.h_tiles[l.ut].cbase;
        }
    LSSP_HIP(hipMemcpy(li.L.d_tiles, li.L.h_tiles.data(), sizeof(LineTile) * li.L.h_tiles.size(),
                       hipMemcpyHostToDevice));
    // U rhs stream (written by the L sweep) and the hand-off buffers, shared by
    // both sweeps (they never run at once) and armed with the sentinel
    LSSP_HIP(hipMalloc(&li.d_ustream, sizeof(double) * (li.U.rows_total + 16 * 1024 / 8)));
    LSSP_HIP(hipMemset(li.d_ustream, 0, sizeof(double) * (li.U.rows_total + 16 * 1024 / 8)));  // invalid rows stay +0.0
    // the apply's L sweep reads its rhs as a stream too (k_line_rhs fills the valid rows)
    LSSP_HIP(hipMalloc(&li.d_lstream, sizeof(double) * (li.L.rows_total + 16 * 1024 / 8)));
    LSSP_HIP(hipMemset(li.d_lstream, 0, sizeof(double) * (li.L.rows_total + 16 * 1024 / 8)));
    li.tmax = std::max(li.L.tmax, li.U.tmax);
    li.hk_stride = (long)li.tmax * NJ;
    li.hj_stride = (long)li.tmax * P;
    li.ntiles = (int)Lt.size();
    li.hk_n = li.hk_stride * li.ntiles;
    li.hj_n = li.hj_stride * li.ntiles;
    LSSP_HIP(hipMalloc(&li.d_hk, sizeof(double) * li.hk_n));
    LSSP_HIP(hipMalloc(&li.d_hj, sizeof(double) * li.hj_n));
    LSSP_TRY(line_rearm(c, li));
    LSSP_HIP(hipStreamSynchronize(c->stream));
    return LSSP_AMD_OK;
}

int line_rearm(lssp_amd_ctx *c, LineILU &li)
{
    LSSP_TRY(launch_fill(c, li.d_hk, li.hk_n, TRI_SENTINEL));
    return launch_fill(c, li.d_hj, li.hj_n, TRI_SENTINEL);
}

void free_line_sweep(LineILU &li)
{
    for (LineSweep *s : {&li.L, &li.U}) {
        if (s->d_tiles) (void)hipFree(s->d_tiles);
        if (s->d_coef) (void)hipFree(s->d_coef);
        if (s->d_claim) (void)hipFree(s->d_claim);
        if (s->d_order) (void)hipFree(s->d_order);
        *s = LineSweep{};
    }
    if (li.d_ustream) (void)hipFree(li.d_ustream);
    if (li.d_lstream) (void)hipFree(li.d_lstream);
    if (li.d_hk) (void)hipFree(li.d_hk);
    if (li.d_hj) (void)hipFree(li.d_hj);
    if (li.d_g2L) (void)hipFree(li.d_g2L);
    if (li.d_g2U) (void)hipFree(li.d_g2U);
    li.d_g2L = li.d_g2U = nullptr;
    li.g2 = 0;
    if (li.d_kdone) (void)hipFree(li.d_kdone);
    if (li.d_kof) (void)hipFree(li.d_kof);
    if (li.d_tclaim) (void)hipFree(li.d_tclaim);
    li.d_kdone = nullptr;
    li.d_kof = nullptr;
    li.d_tclaim = nullptr;
    li.d_ustream = li.d_lstream = li.d_hk = li.d_hj = nullptr;
    li.ntiles = 0;
}

// ---------------------------------------------------------------------------
// device
// ---------------------------------------------------------------------------
struct LineArgs {
    int nx, ny, ntiles;
    long n;
    const LineTile *tiles;
    const double *coef;
    const double *rhs;      // natural order (RHS_NAT) or the U rhs stream
    double *out;            // OUT 1: natural-order output; OUT 2: the U rhs stream
    double *hk, *hj;
    long hk_stride, hj_stride;
    unsigned long long *claim;
    unsigned long long base;
    const int *order;       // k_line2: tile of each claim (wavefront order), nullptr: claim order
    int mirror;             // U sweep: natural row = n-1 - sweep row
    int *err;
    // diagnostics (LSSP_AMD_LINE_TRACE): per tile {claim, step 0, end, re-polls,
    // xcc}; per step of tile ttile {compute start, compute end, poller busy,
    // loader wait, loader issue, storer busy}
    unsigned long long *trace;
    int ttile;
    int diag;  // LSSP_AMD_LINE_DIAG timing experiments (wrong results when != 0)
    const double *guard;  // lssp_amd_ctx::guard
    int tail;     // k_line2 OUT 1: run the product tl after the tiles (write-through output, tile counts)
    LineTail tl;
};

// ---------------------------------------------------------------------------
// k_line2: two levels per workgroup step (the default line sweep)
// ---------------------------------------------------------------------------
// A tile is nj <= 16 lines x np <= 8 planes, 128 rows per level.  Two compute
// waves: wave w owns planes 4w .. 4w+3; lane (g, l) = 16 g + l owns line l of
// plane 4w + g -- ONE row per level -- and a step advances TWO levels (v = 2s,
// 2s+1).  The barrier, the loop, the poller's round trip and every role's
// per-step work are paid once per two levels, and a tile moves half the
// bytes per level of k_line's 256-row tiles (the loaders' LDS-DMA issue,
// ~80 clk per 1 KB piece per CU, bounded k_line's level at ~800-950 clk).
// Row (i, l, p) is computed at level v = i + l + p + sigma(p), sigma = 1 on
// wave 1's planes (line_sigma).  The operands of a row at level v:
//   (i-1): the lane's own value of level v-1 (a register);
//   (j-1): line l-1's value of level v-1: DPP row_shr:1 (the 16-lane groups
//          are the DPP rows); line 0 takes the poller's j-input;
//   (k-1): plane p-1's value of level v-1: lane - 16 inside a wave (two
//          permlane swaps); plane 4's k-neighbour (plane 3, wave 0) is, with
//          the skew, level v-2 -- the previous step's result of the same
//          sub-level, read from LDS after the barrier; plane 0 takes the
//          poller's k-input.
// The arithmetic is k_line's, operand for operand (rhs - c_k x_k - c_j x_j -
// c_i x_i, then / diag), so every value is bitwise the same.
// Roles, one barrier per step: 2 compute waves, NL loaders (LDS-DMA of a
// step's two coefficient blocks and its rhs block D steps ahead), 1 poller
// (LDS-DMA sc1 reads of the two levels' hand-off inputs DH steps ahead), SW
// storers (OUT 2: the U sweep's rhs stream; OUT 1: natural-order x in 8-row
// runs of a line).  The rhs always comes from a stream (k_line_rhs gathers it).
// The U sweep's division stays the IEEE division x / d (solver-tri.cxx:44).
// Markstein's three-operation form from y = RN(1/d) (q0 = x y, e = fma(-q0,
// d, x), q = fma(e, y, q0): bitwise IEEE when |x|, |d| lie in [2^-400,
// 2^400], checked on 4e8 operand pairs by tools/probe/div_check.c) measured
// SLOWER in every placement of y: formed by the loader waves into the slot
// (U sweep 394 us), by the compute waves a step early (396 us), stored in the
// coefficient stream at setup (372-376 us) -- against 352-357 us with the
// plain division (profiles/r04/r04d_*, r04e_*, r04f_*): its range checks and
// the extra operand cost as much as the shorter chain saves.


namespace l2 {
constexpr int NJ = 16;  // lines per tile; LV (2 or 4) levels per step; P (8 or 16) planes per tile: 2 or 4 compute waves
constexpr uint64_t GS = 0x0001000100010001ull;  // line 0 of each 16-lane group
constexpr uint64_t G0M = 0xFFFFull;             // group 0 (the wave's first plane)
template <int NA, int P, int LV>
struct Slot {
    static constexpr int ROWS = P * NJ;
    static constexpr int NPC = (LV * ROWS * NA * 8 + 1023) / 1024;  // 1 KB DMA pieces of the two coefficient blocks
    static constexpr int NRP = (LV * ROWS * 8 + 1023) / 1024;       // ... of the two rhs blocks
    static constexpr int COEF = 0;
    static constexpr int RHS = NPC * 1024;
    static constexpr int KFIN = RHS + NRP * 1024;    // double[LV][NJ]
    static constexpr int JFIN = KFIN + LV * NJ * 8;  // double[LV][P]
    static constexpr int BYTES = JFIN + LV * P * 8;
    static_assert(BYTES % 16 == 0, "slot alignment");
};
// levels of results kept in LDS: the storers' source (OUT 1 writes 8-level
// blocks as runs, so it keeps two) and wave 1's k-input (LV levels back)
template <int OUT, int LV>
constexpr int rsl() { return OUT == 1 ? 16 : 2 * LV; }
template <int NA, int OUT, int D, int P, int LV>
constexpr int lds_bytes() { return (D + 1) * Slot<NA, P, LV>::BYTES + rsl<OUT, LV>() * P * NJ * 8 + 16 + 512; }
constexpr int waves(int P, int NL, int SW) { return P / 4 + NL + 1 + SW; }
}  // namespace l2

template <int P, int LV, int NA, int OUT, int NL, int D, int DH, int SW, bool TRACE, bool TL = false>
__global__ __launch_bounds__(64 * l2::waves(P, NL, SW)) void k_line2(LineArgs a)
{
    using namespace l2;
    // TL: the instantiation that can run the tail product (a separate kernel: the
    // product's registers would otherwise raise the plain sweep's VGPRs 113 -> 162
    // and its SGPR spills 63 -> 182, which cost the U sweep ~40 us at 216^3)
    static_assert(!TL || OUT == 1, "the tail product follows the natural-order sweep");
    const bool tail = TL && a.tail;
    using SL = Slot<NA, P, LV>;
    static_assert(LV == 2 || LV == 4, "levels per step");
    constexpr int CW = P / 4, ROWS = P * NJ;
    constexpr int LA = 2;  // the loaders complete step s+LA's slot during step s
    constexpr int R = D + 1;
    constexpr int RSL = rsl<OUT, LV>();
    constexpr int NITEM = SL::NPC + SL::NRP;  // DMA instructions per step, shared by the loaders
    constexpr int KPER = (NITEM + NL - 1) / NL;
    constexpr int S0 = -2 * ((D + 2) / 2);  // first step of every role (even, <= -D-1)
    static_assert(DH >= 2 && DH < D && (D - LA) * KPER <= 63 && 2 * (DH - 1) <= 63, "leads");
    static_assert(OUT == 1 || OUT == 2, "out");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char *ring = smem;
    double *res = reinterpret_cast<double *>(smem + R * SL::BYTES);  // [RSL][P][NJ]
    int *s_tile = reinterpret_cast<int *>(res + RSL * ROWS);
    const unsigned lds0 = (unsigned)(uintptr_t)smem;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int nx = a.nx;
    if (a.guard && *a.guard != 0.0) {  // a batched iteration past the stop: consume the launch's tile claims
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            atomicAdd(a.claim, (unsigned long long)a.ntiles + gridDim.x);
            if (OUT == 1 && tail) {  // ... and the tail's chunk claims and tile counts
                atomicAdd(a.tl.claim, tail_claims(a.tl.nblk, gridDim.x));
                for (int K = 0; K < a.tl.S; K++) atomicAdd(a.tl.kdone + K, (unsigned)a.tl.W);
            }
        }
        return;
    }

    int done_tile = -1;  // the tile this workgroup finished last (its completion is counted at the next claim)
    if (OUT == 1 && tail && a.tl.dbg && threadIdx.x == 0)  // diagnostics: the workgroup's start
        a.tl.dbg[6144 + blockIdx.x] = (unsigned)__builtin_amdgcn_s_memrealtime();
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) {
            if (OUT == 1 && tail && done_tile >= 0) {  // its storers' write-through stores drained before the barrier
                __hip_atomic_fetch_add(a.tl.kdone + done_tile / a.tl.W, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (a.tl.dbg) a.tl.dbg[blockIdx.x] += 1;
            }
            // claims in wavefront order (LineSweep::d_order): every tile's producers
            // have a smaller anti-diagonal J + K and were claimed before it
            const int c = (int)(atomicAdd(a.claim, 1ull) - a.base);
            *s_tile = c < a.ntiles ? (a.order ? a.order[c] : c) : a.ntiles;
        }
        __syncthreads();
        const int t = __builtin_amdgcn_readfirstlane(*s_tile);
        if (t >= a.ntiles) break;
        done_tile = t;
        if (TRACE && threadIdx.x == 0) a.trace[8 * t] = __builtin_amdgcn_s_memrealtime();
        const LineTile d = a.tiles[t];
        const int T = d.T, TS = T / LV, nj = d.nj, np = d.np;
        const long SB = (long)P * nj;  // rows per level block
        const bool kin = d.flags & LT_KIN, jin = d.flags & LT_JIN, kout = d.flags & LT_KOUT,
                   jout = d.flags & LT_JOUT;
        const int ll = lane & (NJ - 1), gl = lane >> 4;
        const int lc = min(ll, nj - 1);
        auto nb = [&](int p, int l) {  // natural row of (i = 0, line l, plane p); + i (mirror: - i)
            const long r = ((long)(d.k0 + p) * a.ny + (d.j0 + l)) * nx;
            return a.mirror ? a.n - 1 - r : r;
        };
        auto sig = [](int p) { return (LV - 1) * (p >> 2); };
        unsigned long long *ts = TRACE ? a.trace + 8 * (long)a.ntiles : nullptr;
        const bool trs = TRACE && t == a.ttile && lane == 0;

        if (wave < CW) {
            // ---------------- compute: plane pw = 4 wave + g, line l ----------------
            const int pw = wave * 4 + gl;
            const int sg = (LV - 1) * wave;  // sigma of the wave's planes
            struct In {
                double ck[LV], cj[LV], ci[LV], dg[LV], rh[LV];
            };
            // the step's inputs, read from LDS one step ahead (their slot was
            // completed before the barrier that ended the previous step)
            auto load = [&](unsigned so, In &in) {
                const char *slot = ring + so;
#pragma unroll
                for (int v = 0; v < LV; v++) {
                    const long r = v * SB + pw * nj + lc;
                    const double *b = reinterpret_cast<const double *>(slot + SL::COEF) + r * NA;
                    in.ck[v] = b[0];
                    in.cj[v] = b[1];
                    in.ci[v] = b[2];
                    if constexpr (NA == 4) in.dg[v] = b[3];
                    in.rh[v] = reinterpret_cast<const double *>(slot + SL::RHS)[r];
                }
            };
            In A, B;
            double xp = 0.0;  // the lane's value of the previous level
            double xs = 0.0;  // lane - 16's value of the previous level (formed at the end of the previous step)
            constexpr int OOB = 0x40000000;  // voffset that drops a buffer store (soffset is not range-checked)
            const __amdgpu_buffer_rsrc_t hko =
                __builtin_amdgcn_make_buffer_rsrc(a.hk + (long)t * a.hk_stride, 0, (int)(a.hk_stride * 8), 0x00020000);
            const __amdgpu_buffer_rsrc_t hjo =
                __builtin_amdgcn_make_buffer_rsrc(a.hj + (long)t * a.hj_stride, 0, (int)(a.hj_stride * 8), 0x00020000);
            const uint64_t njm = (1ull << nj) - 1;
            uint64_t pm = 0;  // lanes of the tile: line < nj, plane < np
#pragma unroll
            for (int g = 0; g < 4; g++)
                if (wave * 4 + g < np) pm |= njm << (16 * g);
            // plane np-1 feeds the next k-tile (group gk of the wave holding it): hk[q][l], q = v - (np-1) - sigma
            const int gk = np - 1 - 4 * wave;
            const bool kw = kout && gk >= 0 && gk < 4;
            const uint64_t kgm = kw ? (0xFFFFull << (16 * (kw ? gk : 0))) : 0ull;
            const int kq = -(np - 1) - sg;
            // line nj-1 feeds the next j-tile: hj[q][p], q = v - (nj-1)
            const uint64_t jgm = jout ? (GS << (nj - 1)) & pm : 0ull;
            const bool lane_in = (pm >> lane) & 1;  // a row of the tile: line < nj, plane < np
            const int loff = ll + pw + sg;           // its row at level v: i = v - loff
            auto publish = [&](int v, uint64_t h, double x) {
                const uint64_t bx = (uint64_t)__double_as_longlong(x);
                if (kw) {  // uniform
                    const int q = v + kq;
                    int vo = ll * 8;
                    asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(vo) : "v"(OOB), "v"(vo), "s"(h & kgm));
                    if (q < 0) vo = OOB;
                    __builtin_amdgcn_raw_buffer_store_b64(split64(bx), hko, vo, max(q, 0) * (NJ * 8), 16);  // sc1
                }
                if (jout) {
                    const int q = v - (nj - 1);
                    int vo = pw * 8;
                    asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(vo) : "v"(OOB), "v"(vo), "s"(h & jgm));
                    if (q < 0) vo = OOB;
                    __builtin_amdgcn_raw_buffer_store_b64(split64(bx), hjo, vo, max(q, 0) * (P * 8), 16);  // sc1
                }
            };
            unsigned so = (unsigned)(((S0 % R) + R) % R) * SL::BYTES;  // slot of step s
            constexpr unsigned RB = (unsigned)(R * SL::BYTES);
            auto body = [&](int s, In &cur, In &nxt) {
                if (TRACE && lane == 0 && wave == 0 && s == 0) a.trace[8 * t + 1] = __builtin_amdgcn_s_memrealtime();
                if (trs && wave == 0 && s >= 0 && s < TS) ts[8 * s] = __builtin_amdgcn_s_memtime();
                const unsigned sn = so + SL::BYTES == RB ? 0u : so + SL::BYTES;  // slot of step s+1
                // k-inputs of group 0 (read first: LDS returns in order): wave 0 the
                // poller's, wave 1 plane 3's results of the previous step
                double kx[LV];
#pragma unroll
                for (int lv = 0; lv < LV; lv++)
                    kx[lv] = wave == 0 ? reinterpret_cast<const double *>(ring + so + SL::KFIN)[lv * NJ + ll]
                                       : res[((LV * s - LV + lv) & (RSL - 1)) * ROWS + (4 * wave - 1) * NJ + ll];
                // j-inputs of line 0, read with the k-inputs at the step that uses
                // them: polled one step later than when they were read a step ahead
                // with the coefficients, so a j-hop's consumer starts a step
                // earlier (216^3 apply 0.489 -> 0.474 ms, bench 650 -> 664 it/s, the
                // 8-rank 512^3 slab 2.405 -> 2.346 ms; profiles/r06/r06i_*)
                double jx[LV];
#pragma unroll
                for (int lv = 0; lv < LV; lv++) jx[lv] = reinterpret_cast<const double *>(ring + so + SL::JFIN)[lv * P + pw];
                asm volatile("" ::: "memory");
                load(sn, nxt);
                // lanes whose row exists at each level: one per-lane compare each
                // (a SALU chain of shifts and per-group start tests measured 3 %
                // slower per apply, profiles/r04/r04n_line2_compute_variants.txt)
                uint64_t h[LV];
#pragma unroll
                for (int lv = 0; lv < LV; lv++)
                    h[lv] = __builtin_amdgcn_ballot_w64(lane_in && (unsigned)(LV * s + lv - loff) < (unsigned)nx);
                if (s >= 0 && s < TS) {
                    double xq = xp;  // the previous level's value
                    double xu = xs;  // lane - 16's value of the previous level
#pragma unroll
                    for (int lv = 0; lv < LV; lv++) {
                        // level LV s + lv
                        const double xk = sel_lanes(G0M, kx[lv], xu);
                        const double xj = dpp_shr1g<4>(xq, jx[lv]);
                        double v = cur.rh[lv] - cur.ck[lv] * xk;
                        v = v - cur.cj[lv] * xj;
                        v = v - cur.ci[lv] * xq;
                        if constexpr (NA == 4) v = v / cur.dg[lv];
                        const double x = sel_lanes(h[lv], v, xq);
                        if (trs && wave == 0 && lv == LV - 1) ts[8 * s + 6] = __builtin_amdgcn_s_memtime();
                        // the next level's k operand (the next step's first, for the
                        // last level) is shuffled BEFORE this level's hand-off and
                        // LDS stores: its ds_bpermute round trip runs under them
                        // instead of after them (~1 %, profiles/r05/r05b_*)
                        xu = up16(x);
                        __builtin_amdgcn_sched_barrier(0);
                        publish(LV * s + lv, h[lv], x);  // its store issues under the next level's arithmetic
                        res[((LV * s + lv) & (RSL - 1)) * ROWS + pw * NJ + ll] = x;
                        xq = x;
                    }
                    xp = xq;
                    xs = xu;  // the next step's first k-operand, off its critical path
                }
                so = sn;
                if (trs && s >= 0 && s < TS) ts[8 * s + (wave == 0 ? 1 : 7)] = __builtin_amdgcn_s_memtime();
                line_barrier();
            };
            for (int s = S0; s <= TS; s += 2) {
                body(s, A, B);
                if (s + 1 <= TS) body(s + 1, B, A);
            }
            if (TRACE && lane == 0 && wave == 0) {
                a.trace[8 * t + 2] = __builtin_amdgcn_s_memrealtime();
                unsigned xcc;
                asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
                a.trace[8 * t + 4] = xcc;
            }
        } else if (wave < CW + NL) {
            // ---------------- loaders: a step's DMAs spread over the NL waves ----------------
            const int w = wave - CW;
            auto issue = [&](int q) {
                const int qc = min(max(q, 0), TS - 1);
                const unsigned sl = lds0 + (unsigned)(((q % R + R) % R) * SL::BYTES);
                const long row = d.cbase + (long)qc * LV * SB;
                const char *cb = reinterpret_cast<const char *>(a.coef) + row * (8L * NA);
                const char *ub = reinterpret_cast<const char *>(a.rhs) + row * 8L;
#pragma unroll
                for (int k = 0; k < KPER; k++) {
                    const int m = w + k * NL;
                    if (m < SL::NPC) {
                        // non-temporal streams (read once): 216^3 apply 539 against
                        // 547 us, bench 597 against 588 it/s; 512^3 unchanged
                        // (profiles/r04/r04s_line2_nt_dma_ab.txt)
                        dma16_nt(cb + m * 1024 + lane * 16, sl + SL::COEF + m * 1024);
                    } else if (m < NITEM) {
                        const int r = m - SL::NPC;
                        dma16_nt(ub + r * 1024 + lane * 16, sl + SL::RHS + r * 1024);
                    } else {
                        dma16(cb + lane * 16, sl + SL::COEF);  // keeps the per-wave count fixed
                    }
                }
            };
            for (int s = S0; s <= TS; s++) {
                const unsigned long long i0 = TRACE ? __builtin_amdgcn_s_memtime() : 0;
                issue(s + D);  // dummies past TS keep the wait counts exact
                const unsigned long long w0 = TRACE ? __builtin_amdgcn_s_memtime() : 0;
                // steps s+LA+1 .. s+D were issued after step s+LA's
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - LA) * KPER) : "memory");
                if (trs && w == 0 && s >= 0 && s < TS) {
                    ts[8 * s + 4] = w0 - i0;
                    ts[8 * s + 3] = __builtin_amdgcn_s_memtime() - w0;
                }
                line_barrier();
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if (wave == CW + NL) {
            // ---------------- poller ----------------
            // At step s: LDS-DMA sc1 reads of step s+DH's k-inputs (two levels x NJ
            // lines: 16 lanes x 16 B) and j-inputs (two levels x P planes: 8 lanes x
            // 16 B); then the k- and j-inputs of step s+1 (issued DH-1 steps ago)
            // are waited for and checked.  A tile without a k (j) input gets +0.0 there (its
            // coefficient is +0.0 too).
            const double *hk = a.hk + (long)max(d.tk, 0) * a.hk_stride;
            const double *hj = a.hj + (long)max(d.tj, 0) * a.hj_stride;
            const int qmax = (int)(a.hk_stride / (NJ * LV)) - 1;  // steps
            const int kl = lane & (NJ - 1), kv = lane >> 4;      // k check: lanes 0..31 = (level, line)
            const int jp = lane & (P - 1), jv = lane / P;        // j check: lanes 0..2P-1 = (level, plane)
            auto kval = [&](int q) {  // q: level
                return lane < LV * NJ && q < T && kl < nj && (unsigned)(q - kl) < (unsigned)nx;
            };
            auto jval = [&](int q) {
                return lane < LV * P && q < T && jp < np && (unsigned)(q - jp - sig(jp)) < (unsigned)nx;
            };
            const unsigned sink = lds0 + (unsigned)(R * SL::BYTES + RSL * ROWS * 8 + 16);
            auto issue = [&](int q) {
                const char *kp = reinterpret_cast<const char *>(hk + (long)min(max(q, 0), qmax) * LV * NJ) + lane * 16;
                const char *jp2 = reinterpret_cast<const char *>(hj + (long)min(max(q, 0), qmax) * LV * P) + lane * 16;
                const unsigned ks = kin ? lds0 + (unsigned)((((q % R) + R) % R) * SL::BYTES + SL::KFIN) : sink;
                const unsigned js = jin ? lds0 + (unsigned)((((q % R) + R) % R) * SL::BYTES + SL::JFIN) : sink;
                if (lane < LV * NJ / 2) dma16_sc1(kp, ks);
                if (lane < LV * P / 2) dma16_sc1(jp2, js);
            };
            if (!kin || !jin) {
                for (int q = 0; q < R; q++) {
                    if (!kin && lane < LV * NJ) reinterpret_cast<double *>(ring + q * SL::BYTES + SL::KFIN)[lane] = 0.0;
                    if (!jin && lane < LV * P) reinterpret_cast<double *>(ring + q * SL::BYTES + SL::JFIN)[lane] = 0.0;
                }
            }
#ifndef LINE2_POLL_PRIO
#define LINE2_POLL_PRIO 3
#endif
            __builtin_amdgcn_s_setprio(LINE2_POLL_PRIO);  // the polls enter the CU's memory queue ahead of the coefficient DMAs
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            unsigned polls = 0;
            for (int s = S0; s <= TS; s++) {
                const unsigned long long w0 = TRACE ? __builtin_amdgcn_s_memtime() : 0;
                issue(s + DH);
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (DH - 1)) : "memory");
                if (s > TS) break;
                const int qk = s + 1, qj = s + 1;  // steps
                double *kslot = reinterpret_cast<double *>(ring + (qk % R) * SL::BYTES + SL::KFIN) + min(lane, LV * NJ - 1);
                double *jslot = reinterpret_cast<double *>(ring + (qj % R) * SL::BYTES + SL::JFIN) + min(lane, LV * P - 1);
                const int lk = LV * qk + kv, lj = LV * qj + jv;  // levels checked by this lane
                const bool vk = kin && kval(lk), vj = jin && jval(lj);
                const uint64_t kvb = vk ? (uint64_t)__double_as_longlong(*kslot) : 0;
                const uint64_t jvb = vj ? (uint64_t)__double_as_longlong(*jslot) : 0;
                const bool bk = vk && kvb == TRI_SENTINEL, bj = vj && jvb == TRI_SENTINEL;
                if (__any(bk || bj)) {
                    // resync episode: drain, wait for these values, re-issue the polls
                    // of the steps after them.  (k_line's episode also waits for the
                    // furthest step in flight, so the re-issued polls cannot miss; that
                    // holds the tile DH steps behind its producer after every episode:
                    // 216^3 apply 528.5 -> 508.9 us without it, bitwise the same,
                    // profiles/r05/r05p_resync_near.txt)
                    polls++;
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    auto spin = [&](const double *src) {
                        for (;;) {
                            const uint64_t b = line_ld_agent(src);
                            if (b != TRI_SENTINEL) return b;
                            if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) {  // 4 s
                                atomicOr(a.err, 8);
                                return (uint64_t)0x7FF8000000000000ull;
                            }
                        }
                    };
                    if (bk) *kslot = __longlong_as_double((long long)spin(hk + (long)lk * NJ + kl));
                    if (bj) *jslot = __longlong_as_double((long long)spin(hj + (long)lj * P + jp));
                    for (int k = 2; k <= DH; k++) issue(s + k);  // the polls issued at steps s+k-DH
                }
                if (trs && s >= 0 && s < TS) ts[8 * s + 2] = __builtin_amdgcn_s_memtime() - w0;
                line_barrier();
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (TRACE) {
                for (int o = 32; o >= 1; o >>= 1) polls += __shfl_xor(polls, o);
                if (lane == 0) a.trace[8 * t + 3] = polls;
            }
        } else {
            // ---------------- storers: results, re-arms ----------------
            // Storer 0 re-arms the consumed j-inputs, storer SW-1 the k-inputs.
            const int w = wave - (CW + NL + 1);
            const int kl = lane & (NJ - 1), kv = lane >> 4, jp = lane & (P - 1), jv = lane / P;
            uint64_t *hki = reinterpret_cast<uint64_t *>(a.hk + (long)max(d.tk, 0) * a.hk_stride) + kl;
            uint64_t *hji = reinterpret_cast<uint64_t *>(a.hj + (long)max(d.tj, 0) * a.hj_stride) + jp;
            const bool rk = w == SW - 1 && kin && lane < LV * NJ && kl < nj;
            const bool rj = w == 0 && jin && lane < LV * P && jp < np;
            auto rearm = [&](int q) {  // step q's entries
                const int vk = LV * q + kv, vj = LV * q + jv;
                if (rk && vk < T && (unsigned)(vk - kl) < (unsigned)nx) hki[(long)vk * NJ] = TRI_SENTINEL;
                if (rj && vj < T && (unsigned)(vj - jp - sig(jp)) < (unsigned)nx)
                    hji[(long)vj * P] = TRI_SENTINEL;
            };
            if constexpr (OUT == 1) {
                // block B (levels 8B .. 8B+7, steps SPB B .. SPB B + SPB-1, SPB =
                // 8 / LV) is written during the next SPB steps, 1 / SPB of it per
                // step: value k of the block is level 8B + (k & 7) of run k >> 3 =
                // (plane, line), so 8 lanes store 8 consecutive rows of one line
                constexpr int SPB = 8 / LV;
                static_assert(RSL == 16 && (ROWS * 8 / SPB) % (64 * SW) == 0, "runs");
                auto slice = [&](int s) {
                    const int B = s / SPB - 1, u = s % SPB;
                    if (B < 0) return;
                    constexpr int PER = ROWS * 8 / SPB / 64 / SW;  // values per lane per step
#pragma unroll
                    for (int it = 0; it < PER; it++) {
                        const int k = u * (ROWS * 8 / SPB) + (w * PER + it) * 64 + lane;
                        const int m = k & 7, r = k >> 3, p = r >> 4, l = r & (NJ - 1);
                        const int q = 8 * B + m;
                        const int i = q - l - p - sig(p);
                        const double x = res[(q & (RSL - 1)) * ROWS + p * NJ + l];
                        if (!(a.diag & 1) && p < np && l < nj && (unsigned)i < (unsigned)nx) {
                            double *o = a.out + (a.mirror ? nb(p, l) - i : nb(p, l) + i);
                            if (tail) st_sc1d(o, x);  // read by the tail product on other CUs
                            else *o = x;
                        }
                    }
                };
                for (int s = S0; s <= TS; s++) {
                    const unsigned long long w0 = TRACE ? __builtin_amdgcn_s_memtime() : 0;
                    if (s >= 0) slice(s);
                    if (s >= 1 && s <= TS) rearm(s - 1);
                    if (trs && w == 0 && s >= 0 && s < TS) ts[8 * s + 5] = __builtin_amdgcn_s_memtime() - w0;
                    line_barrier();
                }
                // the last blocks' remaining quarters (every result is in LDS)
                for (int s = TS + 1; s < SPB * ((T - 1) / 8 + 2); s++) slice(s);
                if (tail) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // before the tile is counted
            } else {
                // step s-1's LV levels: value k = 64 (w + SW it) + lane is level
                // LV(s-1) + k / ROWS, plane (k >> 4) & (P-1), line k & 15; its place in the
                // mirror U tile's rhs stream (same nj, np): level Cp - v with
                // Cp = nx + nj + np - 3 + sigma(p) + sigma(np-1-p)
                constexpr int PS = LV * ROWS / 64 / SW;
                static_assert(LV * ROWS % (64 * SW) == 0, "chunks");
                double *po[PS];
                int vlo[PS], lvs[PS], roff[PS];
#pragma unroll
                for (int u = 0; u < PS; u++) {
                    const int k = (w + u * SW) * 64 + lane;
                    const int lv = k / ROWS, p = (k >> 4) & (P - 1), l = k & (NJ - 1);
                    const int pp = min(p, np - 1), lq = min(l, nj - 1);
                    lvs[u] = lv;
                    roff[u] = (lv * P + p) * NJ + l;
                    vlo[u] = p < np && l < nj ? l + p + sig(p) : 1 << 30;  // valid iff 0 <= v - vlo < nx
                    const long Cp = (long)nx + nj + np - 3 + sig(pp) + sig(np - 1 - pp);
                    po[u] = a.out + d.ubase + Cp * SB + (long)(np - 1 - pp) * nj + (nj - 1 - lq);
                }
                for (int s = S0; s <= TS; s++) {
                    const unsigned long long w0 = TRACE ? __builtin_amdgcn_s_memtime() : 0;
                    const int q = s - 1;
                    if (q >= 0 && q < TS) {
#pragma unroll
                        for (int u = 0; u < PS; u++) {
                            const int v = LV * q + lvs[u];
                            const double x = res[(v & (RSL - 1)) * ROWS + (roff[u] & (ROWS - 1))];
                            if (!(a.diag & 33) && (unsigned)(v - vlo[u]) < (unsigned)nx) po[u][-SB * v] = x;
                        }
                        rearm(q);
                    }
                    if (trs && w == 0 && s >= 0 && s < TS) ts[8 * s + 5] = __builtin_amdgcn_s_memtime() - w0;
                    line_barrier();
                }
            }
        }
    }
    if constexpr (TL) {
        if (a.tail) {  // no tile left for this workgroup: its waves run the tail product
            int *soff = reinterpret_cast<int *>(smem);  // (the ring's LDS is free now; launch_line2_t reserves TAIL_LDS_BYTES)
            __syncthreads();  // (the loop's last barrier already passed; the ring is free)
            if (threadIdx.x < a.tl.ndiag) soff[threadIdx.x] = a.tl.off[threadIdx.x];
            __syncthreads();
            line_tail_wg(a.tl, a.out, a.err, smem);
        }
    }
}

// ---------------------------------------------------------------------------
// launch
// ---------------------------------------------------------------------------
// The apply's rhs (natural order) into the L sweep's stream layout.  A block
// moves 8 consecutive steps of one tile (P x NJ x 8 values): value v of the
// block is (plane p, line l, step q0 + m) with m = v & 7, so 8 neighbouring
// lanes load one 64-byte run of a line from the natural-order vector and, per
// step, 8 lanes store 8 consecutive stream entries.  Block b runs on XCD b % 8
// and the XCD's blocks walk whole tiles in step order.
constexpr int LRHS_RUN = 8;
// P planes x NJ lines per tile; SKEW: k_line2's level map (compute wave w's
// planes SKEW w levels later); mirror: the tiles are a U sweep's (natural row n-1 - r)
template <int P, int NJ, int SKEW>
__global__ __launch_bounds__(256) void k_line_rhs(const LineTile *__restrict__ tiles, int ntiles, int nq, int nx,
                                                 int ny, long n, int mirror, const double *__restrict__ rhs,
                                                 double *__restrict__ out, const double *guard)
{
    if (guard && *guard != 0.0) return;  // a batched iteration past the stop (lssp_amd_ctx::guard)
    const long b = blockIdx.x, j = b >> 3;
    const int t = (int)(b & 7) + 8 * (int)(j / nq), q0 = (int)(j % nq) * LRHS_RUN;
    if (t >= ntiles) return;
    const LineTile d = tiles[t];
    if (q0 >= d.T) return;
    constexpr int NV = P * NJ * LRHS_RUN / 256;  // values per thread
    static_assert(NV >= 1 && P * NJ * LRHS_RUN % 256 == 0, "block");
    double v[NV];
#pragma unroll
    for (int it = 0; it < NV; it++) {
        const int k = it * 256 + threadIdx.x, m = k & 7, l = (k >> 3) % NJ, p = (k >> 3) / NJ;
        const int i = q0 + m - l - p - SKEW * (p / 4);
        const bool ok = q0 + m < d.T && p < d.np && l < d.nj && (unsigned)i < (unsigned)nx;
        const long r = ((long)(d.k0 + p) * ny + (d.j0 + l)) * nx + i;
        v[it] = ok ? rhs[mirror ? n - 1 - r : r] : 0.0;
    }
    const long SB = (long)P * d.nj;
#pragma unroll
    for (int it = 0; it < NV; it++) {
        const int k = it * 256 + threadIdx.x, m = k & 7, l = (k >> 3) % NJ, p = (k >> 3) / NJ;
        const int i = q0 + m - l - p - SKEW * (p / 4);
        if (q0 + m < d.T && p < d.np && l < d.nj && (unsigned)i < (unsigned)nx)
            out[d.cbase + (q0 + m) * SB + p * d.nj + l] = v[it];
    }
}

// k_line2's gather (P = 8 planes x NJ = 16 lines, level skew 1) through LDS:
// a block moves RUN consecutive steps of one tile; it loads every line's RUN
// consecutive entries (a RUN x 8-byte natural-order run per line), then
// stores step by step, 128 consecutive stream entries (1 KB) per step.
// OP as k_line_rhs's.
#ifndef LRHS2_RUN
#define LRHS2_RUN 32
#endif
template <int RUN, int OP>
__global__ __launch_bounds__(256) void k_line_rhs2(const LineTile *__restrict__ tiles, int ntiles, int nq, int nx,
                                                  int ny, const double *__restrict__ rhs, double *__restrict__ out,
                                                  const double *guard, const double *__restrict__ y, double *nat,
                                                  const double *scal)
{
    constexpr int P = 8, NJ = 16, NL = P * NJ, NV = RUN * NL / 256;
    static_assert(NV >= 1 && RUN * NL % 256 == 0, "block");
    __shared__ double tb[RUN][NL + 1];
    if (guard && *guard != 0.0) return;
    const long b = blockIdx.x, j = b >> 3;
    const int t = (int)(b & 7) + 8 * (int)(j / nq), q0 = (int)(j % nq) * RUN;
    if (t >= ntiles) return;
    const LineTile d = tiles[t];
    if (q0 >= d.T) return;
    double c0 = 0.0, c1 = 0.0;
    if (OP == GEW_BICG_P) c0 = scal[S_BETA], c1 = scal[S_OMEGA];
    if (OP == GEW_BICG_S) c0 = scal[S_ALPHA];
    double v[NV];
#pragma unroll
    for (int it = 0; it < NV; it++) {
        const int k = it * 256 + threadIdx.x, m = k % RUN, ln = k / RUN, p = ln / NJ, l = ln % NJ;
        const int i = q0 + m - l - p - p / 4;
        const bool ok = q0 + m < d.T && p < d.np && l < d.nj && (unsigned)i < (unsigned)nx;
        const long r = ((long)(d.k0 + p) * ny + (d.j0 + l)) * nx + i;
        if (OP == 0) {
            v[it] = ok ? rhs[r] : 0.0;
        } else {
            v[it] = 0.0;
            if (ok) {
#if !defined(GEW_TEMPORAL_LOADS)
                // non-temporal operand loads (r, p, v, read once here): 216^3
                // 645.9 -> 658.4 it/s, profiles/r05/r05x_xr_nt_ab.txt; the
                // natural-order output stays temporal (a non-temporal store
                // measured no better).  -DGEW_TEMPORAL_LOADS: plain loads (A/B)
                if (OP == GEW_BICG_P)
                    v[it] = __builtin_nontemporal_load(rhs + r) +
                            c0 * (__builtin_nontemporal_load(nat + r) - c1 * __builtin_nontemporal_load(y + r));
                else v[it] = __builtin_nontemporal_load(rhs + r) - c0 * __builtin_nontemporal_load(y + r);
#else
                if (OP == GEW_BICG_P) v[it] = rhs[r] + c0 * (nat[r] - c1 * y[r]);
                else v[it] = rhs[r] - c0 * y[r];
#endif
#if defined(GEW_NT_STORE)  // tuning builds: the natural-order output non-temporal too
                __builtin_nontemporal_store(v[it], nat + r);
#else
                nat[r] = v[it];
#endif
            }
        }
    }
#pragma unroll
    for (int it = 0; it < NV; it++) {
        const int k = it * 256 + threadIdx.x;
        tb[k % RUN][k / RUN] = v[it];
    }
    __syncthreads();
    const long SB = (long)P * d.nj;
#pragma unroll
    for (int it = 0; it < NV; it++) {
        const int k = it * 256 + threadIdx.x, ln = k % NL, m = k / NL, p = ln / NJ, l = ln % NJ;
        const int i = q0 + m - l - p - p / 4;
        if (q0 + m < d.T && p < d.np && l < d.nj && (unsigned)i < (unsigned)nx)
            out[d.cbase + (q0 + m) * SB + p * d.nj + l] = tb[m][ln];
    }
}

// the natural-order rhs into a sweep's stream layout (stream: li.d_lstream for
// the L sweep, li.d_ustream for the U sweep)
static int launch_line_gather(lssp_amd_ctx *c, const LineSweep &ls, int mirror, const double *rhs, double *stream)
{
    if (ls.LV != 2 || ls.P != 8 || ls.NJ != 16) return LSSP_AMD_EUNSUPPORTED;
    if (!mirror) {
        const int nq2 = (ls.tmax + LRHS2_RUN - 1) / LRHS2_RUN;
        k_line_rhs2<LRHS2_RUN, 0><<<8L * ((ls.ntiles + 7) / 8) * nq2, 256, 0, c->stream>>>(
            ls.d_tiles, ls.ntiles, nq2, ls.nx, ls.ny, rhs, stream, c->guard, nullptr, nullptr, nullptr);
        LSSP_HIP(hipGetLastError());
        return LSSP_AMD_OK;
    }
    const int nq = (ls.tmax + LRHS_RUN - 1) / LRHS_RUN;
    const long grid = 8L * ((ls.ntiles + 7) / 8) * nq;
    auto kr = k_line_rhs<8, 16, 1>;  // (the U sweep's mirrored tiles; the L sweep takes k_line_rhs2 above)
    const long n = (long)ls.nx * ls.ny * ls.nz;
    kr<<<grid, 256, 0, c->stream>>>(ls.d_tiles, ls.ntiles, nq, ls.nx, ls.ny, n, mirror, rhs, stream, c->guard);
    LSSP_HIP(hipGetLastError());
    return LSSP_AMD_OK;
}

// Fusing BiCGSTAB's p / s passes with the gather saves the gather's read of
// the vector just written and its launch: 216^3, 2 x 33.7 us of k_line_rhs per
// iteration become two passes ~10 us longer than k_ew's (the values leave in
// 64-byte runs of a line, the stream in 128-byte steps).  The separate passes
// remain for the factors this does not cover.
bool line_gather_ew_ok(const LineILU &li, long n)
{
    const char *te = getenv("LSSP_AMD_TAIL");  // the tail product gathers itself (and its EINVAL mode)
    return !(te && atoi(te)) && li.ntiles > 0 && li.kind == 0 && !li.g2 && li.LV == 2 && li.L.P == 8 &&
           li.L.NJ == 16 && li.d_lstream && (long)li.L.nx * li.L.ny * li.L.nz == n;
}

int launch_line_gather_ew(lssp_amd_ctx *c, const LineILU &li, int op, const double *x, const double *y, double *out,
                          const double *scal)
{
    const LineSweep &ls = li.L;
    if (!line_gather_ew_ok(li, (long)ls.nx * ls.ny * ls.nz) || (op != GEW_BICG_P && op != GEW_BICG_S))
        return LSSP_AMD_EINVAL;
    const int nq = (ls.tmax + LRHS2_RUN - 1) / LRHS2_RUN;
    const long grid = 8L * ((ls.ntiles + 7) / 8) * nq;
    auto kr = op == GEW_BICG_P ? k_line_rhs2<LRHS2_RUN, GEW_BICG_P> : k_line_rhs2<LRHS2_RUN, GEW_BICG_S>;
    kr<<<grid, 256, 0, c->stream>>>(ls.d_tiles, ls.ntiles, nq, ls.nx, ls.ny, x, li.d_lstream, c->guard, y, out, scal);
    LSSP_HIP(hipGetLastError());
    li.lstream_of = out;
    return LSSP_AMD_OK;
}

// ---- k_line2 launches -------------------------------------------------------
#ifndef LINE2_D
#define LINE2_D 7  // loader lead (steps of two levels; 7 with the near resync: profiles/r05/r05q_line2_leads.txt)
#endif
#ifndef LINE2_DH
#define LINE2_DH 3  // poller lead (steps)
#endif
#ifndef LINE2_NL
#define LINE2_NL 4
#endif
#ifndef LINE2_SW
#define LINE2_SW 4
#endif
// four levels per step (measured with leads 4 / 2 steps) are not instantiated
#ifndef LINE2_D_U
#define LINE2_D_U LINE2_D  // the loader lead of the natural-order-output sweeps (OUT 1)
#endif
template <int LV, int OUT = 2>
constexpr int line2_d() { return LV == 4 ? 4 : OUT == 1 ? LINE2_D_U : LINE2_D; }
#ifndef LINE2_DH_U
#define LINE2_DH_U 2  // the poller lead of the sweeps with natural-order output (OUT 1): 2 with the near resync (U 311 -> 296 us, profiles/r05/r05r_line2_dh.txt)
#endif
template <int LV, int OUT>
constexpr int line2_dh() { return LV == 4 ? 2 : OUT == 1 ? LINE2_DH_U : LINE2_DH; }
template <int P, int LV, int NA, int OUT, bool TRACE, bool TL = false>
static int launch_line2_k(lssp_amd_ctx *c, const LineSweep &ls, const LineArgs &g, int lds)
{
    auto kern = k_line2<P, LV, NA, OUT, LINE2_NL, line2_d<LV, OUT>(), line2_dh<LV, OUT>(), LINE2_SW, TRACE, TL>;
    static int attr = 0;
    if (lds > attr) {
        LSSP_HIP(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        attr = lds;
    }
    const int grid = std::min(ls.ntiles, c->num_cus);
    kern<<<grid, 64 * l2::waves(P, LINE2_NL, LINE2_SW), lds, c->stream>>>(g);
    ls.base += (unsigned long long)ls.ntiles + grid;
    LSSP_HIP(hipGetLastError());
    return LSSP_AMD_OK;
}

template <int P, int LV, int NA, int OUT>
static int launch_line2_t(lssp_amd_ctx *c, const LineSweep &ls, const LineArgs &a)
{
    // (a sweep with natural-order output and the tail product reserves what the product needs)
    constexpr int lds0 = l2::lds_bytes<NA, OUT, line2_d<LV, OUT>(), P, LV>();
    constexpr int ldst = OUT == 1 && lds0 < TAIL_LDS_BYTES(0) ? TAIL_LDS_BYTES(0) : lds0;
    static_assert(ldst <= 160 * 1024, "LDS");
    const int lds = a.tail ? ldst : lds0;
    static_assert(OUT != 1 || l2::waves(P, LINE2_NL, LINE2_SW) >= TAIL_WAVES, "the tail product's roles");
    // diagnostics only: LSSP_AMD_LINE_TRACE=path[:tile] appends one JSON line per sweep
    static const char *trp = getenv("LSSP_AMD_LINE_TRACE");
    if constexpr (OUT == 1)
        if (a.tail) return launch_line2_k<P, LV, NA, OUT, false, true>(c, ls, a, lds);  // (no trace variant)
    if (!trp) return launch_line2_k<P, LV, NA, OUT, false>(c, ls, a, lds);
    LineArgs g = a;
    const size_t tn = 8 * (size_t)ls.ntiles + 8 * (size_t)ls.tmax + 64;
    const char *colon = strrchr(trp, ':');
    g.ttile = colon ? atoi(colon + 1) : ls.ntiles / 2;
    LSSP_HIP(hipMalloc(&g.trace, sizeof(unsigned long long) * tn));
    LSSP_HIP(hipMemsetAsync(g.trace, 0, sizeof(unsigned long long) * tn, c->stream));
    const int grid = std::min(ls.ntiles, c->num_cus);
    LSSP_TRY((launch_line2_k<P, LV, NA, OUT, true>(c, ls, g, lds)));
    std::vector<unsigned long long> h(tn);
    LSSP_HIP(hipMemcpyAsync(h.data(), g.trace, sizeof(unsigned long long) * tn, hipMemcpyDeviceToHost, c->stream));
    LSSP_HIP(hipStreamSynchronize(c->stream));
    (void)hipFree(g.trace);
    std::string path(trp, colon ? colon - trp : strlen(trp));
    FILE *f = fopen(path.c_str(), "a");
    if (f) {
        fprintf(f, "{\"mirror\": %d, \"ntiles\": %d, \"W\": %d, \"ttile\": %d, \"T\": %d, \"LV\": %d, \"grid\": %d, "
                   "\"data\": [",
                a.mirror, ls.ntiles, (ls.ny + ls.NJ - 1) / ls.NJ, g.ttile, ls.h_tiles[g.ttile].T / LV, LV, grid);
        for (size_t i = 0; i < tn; i++) fprintf(f, "%s%llu", i ? ", " : "", h[i]);
        fprintf(f, "]}\n");
        fclose(f);
    }
    return LSSP_AMD_OK;
}

// k_line2 sweep of ls: rhs from a stream; OUT 2: out = the U rhs stream, OUT 1: natural order
// (tail: the product run by the sweep's workgroups after its tiles, OUT 1 only)
static int launch_line2(lssp_amd_ctx *c, const LineILU &li, int which, const double *stream, double *out, int outk,
                        const LineTail *tail = nullptr)
{
    const LineSweep &ls = which ? li.U : li.L;
    LineArgs a{};
    a.nx = ls.nx;
    a.ny = ls.ny;
    a.ntiles = ls.ntiles;
    a.n = (long)ls.nx * ls.ny * ls.nz;
    a.tiles = ls.d_tiles;
    a.coef = ls.d_coef;
    a.rhs = stream;
    a.out = out;
    a.hk = li.d_hk;
    a.hj = li.d_hj;
    a.hk_stride = li.hk_stride;
    a.hj_stride = li.hj_stride;
    a.claim = ls.d_claim;
    a.base = ls.base;
    a.order = ls.d_order;
    a.mirror = which;
    a.err = c->d_err;
    a.guard = c->guard;
    {
        const char *dg = getenv("LSSP_AMD_LINE_DIAG");
        a.diag = dg ? atoi(dg) : 0;
    }
    a.tail = tail != nullptr && outk == 1;
    if (a.tail) a.tl = *tail;
    // (the kernel is generic in LV; four levels per step measured slower)
    if (outk == 2) return ls.NA == 3 ? launch_line2_t<8, 2, 3, 2>(c, ls, a) : launch_line2_t<8, 2, 4, 2>(c, ls, a);
    return ls.NA == 3 ? launch_line2_t<8, 2, 3, 1>(c, ls, a) : launch_line2_t<8, 2, 4, 1>(c, ls, a);
}

int launch_line_apply(lssp_amd_ctx *c, const LineILU &li, double *x, const double *rhs)
{
    const bool ready = rhs == li.lstream_of;  // the stream holds rhs already (launch_line_gather_ew)
    li.lstream_of = nullptr;
    if (li.g2) return launch_lineg(c, li, 0, x, rhs);
    if (li.kind == 1) return launch_linefill_apply(c, li, x, rhs);
    // k_line2: gather, L sweep -> the U rhs stream, U sweep -> x
    if (!ready) LSSP_TRY(launch_line_gather(c, li.L, 0, rhs, li.d_lstream));
    LSSP_TRY(launch_line2(c, li, 0, li.d_lstream, li.d_ustream, 2));
    return launch_line2(c, li, 1, li.d_ustream, x, 1);
}

unsigned *tail_dbg_host = nullptr;  // LSSP_AMD_TAIL_DIAG (lssp_amd_debug_words)

int launch_line_apply_spmv(lssp_amd_ctx *c, const LineILU &li, double *x, const double *rhs, const lssp_amd_mat *A,
                           int epi, double alpha, double beta, const double *y, double *z, int nred,
                           const double *w0, const double *w1)
{
    // Off by default for ILU(0): measured slower than the two steps (216^3 BiCGSTAB 531 vs
    // 559 it/s, ILU(1) 328 vs 335 at the time; profiles/r05/r05c_tail_ab.txt): after the
    // sweep the product moves ~0.75x k_spmv3's rows per us (one 1024-row round
    // per CU in flight, ~6 us each), and during the sweep rows become ready one
    // U tile row (all W tiles) at a time, so the freed workgroups cannot finish
    // the product before the two-step path would.  LSSP_AMD_TAIL=1 selects it
    // (A/B runs); =2: selected, and an ineligible call fails (EINVAL) instead of
    // falling back (tests)
    // The ILU(1) sweeps (k_linef) run it by default: there it gains (216^3
    // BiCGSTAB+ILU(1) 340.2 -> 352.4 it/s, bitwise; profiles/r05/r05v_tail_ilu1.txt);
    // ILU(0) keeps the two steps, whose p / s passes carry the rhs gathers
    // (628.9 against 559.7 it/s with the tail, same session).
    const char *te = getenv("LSSP_AMD_TAIL");
    const int on = te ? atoi(te) : li.kind == 1 ? 1 : 0;
    const long pl = (long)li.g.nx * li.g.ny, n = pl * li.g.nz;
    // one rank: every chunk; P ranks: the halo-free chunks (the caller runs the rest)
    const bool dist = A && A->nhalo > 0;
    const long nall = num_chunks(n);
    const long cb = dist ? A->ich0 : 0, ce = dist ? A->ich1 : nall;
    if (!on || li.kind > 1 || li.g2 || li.LV < 2 || li.ntiles == 0 || !A || (long)A->nrows != n || ce <= cb ||
        (c->nranks > 1) != dist || A->ndiag == 0 || A->max_off_int > pl || nred < 0 || nred > 2 || x == z || !A->Ad ||
        n >= (1L << 28))  // (x is read through a buffer resource: byte offsets below 2^31)
        return on == 2 ? LSSP_AMD_EINVAL : LSSP_AMD_EUNSUPPORTED;
    const int S = li.S, W = li.W, nz = li.g.nz;
    if (!li.d_kdone) {
        // every tile row holds W tiles (build_tiles); natural plane -> its L tile row
        std::vector<int> kof(nz, 0);
        for (int K = 0; K < S; K++) {
            const LineTile &t = li.L.h_tiles[(size_t)K * W];
            for (int k = t.k0; k < t.k0 + t.np; k++) kof[k] = K;
        }
        LineILU &m = const_cast<LineILU &>(li);
        LSSP_HIP(hipMalloc(&m.d_kdone, sizeof(unsigned) * S));
        LSSP_HIP(hipMalloc(&m.d_kof, sizeof(int) * nz));
        LSSP_HIP(hipMalloc(&m.d_tclaim, sizeof(unsigned long long)));
        LSSP_HIP(hipMemsetAsync(m.d_kdone, 0, sizeof(unsigned) * S, c->stream));
        LSSP_HIP(hipMemsetAsync(m.d_tclaim, 0, sizeof(unsigned long long), c->stream));
        LSSP_HIP(hipMemcpyAsync(m.d_kof, kof.data(), sizeof(int) * nz, hipMemcpyHostToDevice, c->stream));
        LSSP_HIP(hipStreamSynchronize(c->stream));
        m.tbase = 0;
        m.kepoch = 0;
    }
    const long nblk = ce - cb;
    LSSP_TRY(ensure_part(c, nall));
    LineTail T{};
    T.Ap = A->Ap;
    T.Aj = A->Aj;
    T.nnz_pad = A->nnz + 4L;
    T.Ax = A->Ax;
    T.Ad = A->Ad;
    T.off = A->d_off;
    T.ndiag = A->ndiag;
    T.nrows = A->nrows;
    T.epi = epi;
    T.nred = nred;
    T.y = y;
    T.z = z;
    T.alpha = alpha;
    T.beta = beta;
    T.w0 = w0;
    T.w1 = w1;
    T.part = c->d_part;
    T.pcap = c->part_cap;
    T.nblk = nblk;
    T.cend = ce;
    T.claim = li.d_tclaim;
    T.base = li.tbase;
    T.kdone = li.d_kdone;
    T.ktarget = (li.kepoch + 1) * (unsigned)W;
    T.kof = li.d_kof;
    T.S = S;
    T.W = W;
    T.nz = nz;
    T.pl = pl;
    static unsigned *dbg_h = nullptr, *dbg_d = nullptr;
    if (getenv("LSSP_AMD_TAIL_DIAG")) {
        if (!dbg_h) {
            LSSP_HIP(hipHostMalloc(&dbg_h, sizeof(unsigned) * 32768, hipHostMallocMapped));
            LSSP_HIP(hipHostGetDevicePointer(reinterpret_cast<void **>(&dbg_d), dbg_h, 0));
        }
        memset(dbg_h, 0, sizeof(unsigned) * 32768);
        tail_dbg_host = dbg_h;
        T.dbg = dbg_d;
    }
    long tail_waves = (long)std::min(li.U.ntiles, c->num_cus);  // (the tail's claimants: workgroups)
    const bool ready = rhs == li.lstream_of;
    li.lstream_of = nullptr;
    if (li.kind == 1) {  // the 7-/5-point ILU(1) line sweeps (linefill.hip)
        LSSP_TRY(launch_linefill_apply_tail(c, li, x, rhs, T, &tail_waves));
    } else {
        if (!ready) LSSP_TRY(launch_line_gather(c, li.L, 0, rhs, li.d_lstream));
        LSSP_TRY(launch_line2(c, li, 0, li.d_lstream, li.d_ustream, 2));
        LSSP_TRY(launch_line2(c, li, 1, li.d_ustream, x, 1, &T));
    }
    // chunks are claimed in pairs and every workgroup of the grid ends on one
    // failed pair claim; every U tile counted once
    li.tbase += tail_claims(nblk, tail_waves);
    li.kepoch++;
    return LSSP_AMD_OK;
}

int launch_line_sweep(lssp_amd_ctx *c, const LineILU &li, int which, double *x, const double *rhs)
{
    li.lstream_of = nullptr;
    if (li.g2) return launch_lineg(c, li, which ? 2 : 1, x, rhs);
    if (li.kind == 1) return launch_linefill_sweep(c, li, which, x, rhs);
    // one sweep: its rhs gathered into its own stream, natural-order output
    double *st = which ? li.d_ustream : li.d_lstream;
    LSSP_TRY(launch_line_gather(c, which ? li.U : li.L, which, rhs, st));
    return launch_line2(c, li, which, st, x, 1);
}

}  // namespace lssp_amd

// diagnostics (LSSP_AMD_TAIL_DIAG): the tail's progress words, readable while a kernel runs
extern "C" int lssp_amd_debug_words(unsigned *out, int n)
{
    if (!lssp_amd::tail_dbg_host || !out) return LSSP_AMD_EINVAL;
    memcpy(out, lssp_amd::tail_dbg_host, sizeof(unsigned) * std::min(n, 32768));
    return LSSP_AMD_OK;
}
