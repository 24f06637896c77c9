// linefill.hip -- triangular sweeps of a 7-point grid's ILU(1) factor (the
// reference's default level, pc.cxx:3) as skewed line sweeps, the arithmetic
// of solver-tri.cxx:4-46 bit for bit.
//
// Pattern.  ILU(1) of the 7-point operator (pc-iluk.cxx:22-135: fills of level
// lev(L) + lev(U) + 1 <= 1) gives L row r = (i, j, k) the strict entries
// {r-pl, r-pl+1, r-pl+nx, r-nx, r-nx+1, r-1} (pl = nx*ny; those inside the
// grid, ascending) and U row r {r+1, r+nx-1, r+nx, r+pl-nx, r+pl-1, r+pl}.  The
// L row (i, j, k) therefore needs
//   B (i, j, k-1), BE (i+1, j, k-1), BN (i, j+1, k-1), S (i, j-1, k),
//   SE (i+1, j-1, k), W (i-1, j, k)
// in that (ascending column) order; its wavefront is v = i + 2j + 3k (6N
// levels).  The U sweep is the same recurrence in mirrored coordinates
// (i' = nx-1-i, ...), and its descending order (solver-tri.cxx:38: T, TW, TS,
// N, NW, E) is then again B, BE, BN, S, SE, W.
//
// Skewed tiles.  In (i, j' = j + k, k) every dependency has dj' <= 0 and
// dk <= 0 (S, SE: dj' = -1; B, BE: dj' = -1, dk = -1; BN: dj' = 0, dk = -1), so
// rectangles of j' x k depend only on their left and lower neighbours, as in
// k_line2 (a rectangle in j would make neighbouring j-tiles need each other at
// every level through BN).  A tile is nj <= 16 lines of j' x np <= 8 planes;
// compute wave w owns planes 4w .. 4w+3, lane (g, l) = 16 g + l line j'0 + l of
// plane p = 4w + g, i.e. grid line j = j'0 + l - (k0 + p) (lanes with j outside
// the grid compute zeros).  At level v the lane computes row
//   i = v - 2 l - p - sigma(p),   sigma = 1 on wave 1's planes,
// and a step advances two levels.  Operands of a row at level v:
//   W:  the lane's own x(v-1);
//   SE: lane l-1's x(v-1) (DPP row_shr:1); line 0: the j-input, row i+1;
//   S:  the lane's SE of level v-1;
//   BN: lane l-16's x(v-1) (plane p-1, one shuffle); plane 0: the k-input;
//       plane 4: plane 3's x(v-2) (wave 0's result of the previous step, LDS);
//   BE: lane l-1's BN of level v-1 (DPP); line 0: line -1 of plane p-1 (the
//       j-input), plane 0: line -1 of plane -1 (the k-input's forwarded entry);
//   B:  the lane's BE of level v-1.
// Only W, SE and BN wait for the previous level: the chain after it is one
// shuffle, one multiply and four subtractions (+ U's division).  Rows outside
// the grid, and rows past the end of a line, hold +0.0, so a missing neighbour's
// product is +0.0 x +0.0 and every value is the reference's.
//
// Hand-offs (value as flag, TRI_SENTINEL; armed by line_rearm, re-armed by
// their consumer).  j-output hj[q + 2][p]: line nj-1 of plane p, row i, for
// q = i + p + sigma(p), rows 0 .. nx (row nx = +0.0, the next tile's SE / BE
// operand of row nx-1).  k-output hk[Q][1 + l]: plane np-1, line l, row i,
// Q = i + 2 l + 2 (the next k-tile's BN operand at its level Q - 2), and
// hk[Q][0] = line -1 of plane np-1 (this tile's j-input), row Q - 1: the next
// k-tile's line 0 BE operand of plane 0, which no other tile of that k-tile
// reads.
//
// Roles and streams are k_line2's (linesweep.hip): 2 compute waves, NL LDS-DMA
// loader waves (the step's coefficient blocks {B, BE, BN, S, SE, W(, diag)}
// and rhs block D steps ahead), 1 poller (the hand-off inputs DH steps ahead),
// SW storers (the U sweep's rhs stream or the natural-order output, re-arms).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <cstdio>
#include <vector>

#include "internal.h"
#include "linesweep_dev.h"

namespace lssp_amd {

namespace lf {
constexpr int P = 8, NJ = 16, LV = 2, HKS = 18, ROWS = P * NJ;
constexpr int HJ0 = 2;  // hj row of q = -2 (the compute runs from level -2)
constexpr uint64_t G0M = 0xFFFFull;  // lane group 0 (the wave's first plane)
constexpr int sig(int p) { return p >> 2; }
template <int NA>
struct Slot {
    static constexpr int NPC = (LV * ROWS * NA * 8 + 1023) / 1024;  // 1 KB DMA pieces of the two coefficient blocks
    static constexpr int NRP = (LV * ROWS * 8 + 1023) / 1024;       // ... of the two rhs blocks
    static constexpr int COEF = 0;
    static constexpr int RHS = NPC * 1024;
    static constexpr int KFIN = RHS + NRP * 1024;      // double[LV][HKS]: hk rows 2s+2, 2s+3
    static constexpr int JFIN = KFIN + LV * HKS * 8;   // double[LV][P]: hj rows of q = 2s+1, 2s+2
    static constexpr int BYTES = JFIN + LV * P * 8;
    static_assert(KFIN % 16 == 0 && JFIN % 16 == 0 && BYTES % 16 == 0, "slot alignment");
};
template <int OUT>
constexpr int rsl() { return OUT == 1 ? 16 : 4; }
template <int NA, int OUT, int D>
constexpr int lds_bytes() { return (D + 1) * Slot<NA>::BYTES + rsl<OUT>() * ROWS * 8 + 16 + 512; }
constexpr int waves(int NL, int SW) { return 2 + NL + 1 + SW; }
}  // namespace lf
constexpr int G2_D = 16;       // k_lineg: levels of DMA lead (ring of D + 1 slots), up to 192 lines
constexpr int G2_DW = 11;      // ... for 193 - 256 lines (4 waves' rings of 12 slots of 3 KB)
constexpr int G2_BND = 2 * 5 * 64 * 8;  // k_lineg's boundary words
// Streams are [level][wave][S, (SE,) W, (diag,) rhs][64 lanes]: each wave DMAs
// only its own lanes' block, so a level's data needs no barrier, only the
// boundary word of the previous wave does.
__host__ __device__ constexpr int g2_pw(int NC) { return (NC + 2) / 2; }  // 1 KB DMA pieces per wave and level
__host__ __device__ inline long g2_at(long v, int NW, int NC, int k, int j)  // stream index of (level, line, component)
{
    return ((v * NW + (j >> 6)) * (NC + 1) + k) * 64 + (j & 63);
}

// ---------------------------------------------------------------------------
// host: detection, tiles, streams
// ---------------------------------------------------------------------------
namespace {

// L / U rows exactly the 7-point ILU(1) pattern of an nx x ny x nz grid, or
// the 5-point one of an nx x ny grid (nz = 1); nx, ny >= 3, no block-Jacobi cuts
bool detect_fill1(int n, const std::vector<int> &Lp, const std::vector<int> &Lj, const std::vector<double> &Lx,
                  const std::vector<int> &Up, const std::vector<int> &Uj, LineGeom &g)
{
    long offs[6];
    int no = 0;
    for (int r = 0; r < n; r++) {
        const int a = Lp[r], b = Lp[r + 1];
        if (b - a < 1 || b - a > 7 || Lj[b - 1] != r) return false;
        for (int k = a; k < b - 1; k++) {
            const long d = (long)r - Lj[k];
            if (d <= 0) return false;
            bool seen = false;
            for (int q = 0; q < no; q++) seen |= offs[q] == d;
            if (!seen) {
                if (no == 6) return false;
                offs[no++] = d;
            }
        }
    }
    // 3-D: {1, nx-1, nx, pl-nx, pl-1, pl}; 2-D (5-point, one plane): {1, nx-1, nx}
    if (no != 6 && no != 3) return false;
    std::sort(offs, offs + no);
    const long nx = offs[2], pl = no == 6 ? offs[5] : n;
    if (offs[0] != 1 || offs[1] != nx - 1) return false;
    if (no == 6 && (offs[3] != pl - nx || offs[4] != pl - 1)) return false;
    if (nx < 3 || pl % nx || n % pl) return false;
    g.nx = (int)nx;
    g.ny = (int)(pl / nx);
    g.nz = (int)(n / pl);
    if (g.ny < 3 || (no == 6) != (g.nz >= 2)) return false;
    std::atomic<bool> ok{true}, unit{true};
    parallel_for(n, [&](long r0, long r1) {
        for (long r = r0; r < r1 && ok.load(std::memory_order_relaxed); r++) {
            const int i = (int)(r % nx), j = (int)((r / nx) % g.ny), k = (int)(r / pl);
            long want[7];
            int m = 0;
            if (k > 0) want[m++] = r - pl;
            if (k > 0 && i < nx - 1) want[m++] = r - pl + 1;
            if (k > 0 && j < g.ny - 1) want[m++] = r - pl + nx;
            if (j > 0) want[m++] = r - nx;
            if (j > 0 && i < nx - 1) want[m++] = r - nx + 1;
            if (i > 0) want[m++] = r - 1;
            const int a = Lp[r], b = Lp[r + 1];
            bool good = b - a - 1 == m;
            for (int q = 0; good && q < m; q++) good = Lj[a + q] == want[q];
            if (good && Lx[b - 1] != 1.0) unit.store(false, std::memory_order_relaxed);
            m = 0;
            if (i < nx - 1) want[m++] = r + 1;
            if (j < g.ny - 1 && i > 0) want[m++] = r + nx - 1;
            if (j < g.ny - 1) want[m++] = r + nx;
            if (k < g.nz - 1 && j > 0) want[m++] = r + pl - nx;
            if (k < g.nz - 1 && i > 0) want[m++] = r + pl - 1;
            if (k < g.nz - 1) want[m++] = r + pl;
            const int c = Up[r], e = Up[r + 1];
            good = good && e - c - 1 == m && Uj[c] == r;
            for (int q = 0; good && q < m; q++) good = Uj[c + 1 + q] == want[q];
            if (!good) ok.store(false, std::memory_order_relaxed);
        }
    });
    if (!ok.load()) return false;
    g.unitL = unit.load();
    g.kin.assign(g.nz, 1);
    g.kin[0] = 0;
    return true;
}

// coefficients of one sweep in its row order (r_sweep = r for L, n-1-r for U):
// {B, BE, BN, S, SE, W(, diag)}; a missing neighbour gets +0.0
struct FillCoef {
    std::vector<double> c;
    int NA = 6;
    void build(const std::vector<int> &Tp, const std::vector<int> &Tj, const std::vector<double> &Tx, bool upper,
               long n, long nx, long pl, int na)
    {
        NA = na;
        c.assign((size_t)n * NA, 0.0);
        parallel_for(n, [&](long r0, long r1) {
            for (long r = r0; r < r1; r++) {
                double *row = c.data() + (size_t)(upper ? n - 1 - r : r) * NA;
                const int b = Tp[r], e = Tp[r + 1];
                if (NA == 7) row[6] = upper ? Tx[b] : Tx[e - 1];
                for (int q = upper ? b + 1 : b; q < (upper ? e : e - 1); q++) {
                    const long off = upper ? Tj[q] - r : r - Tj[q];
                    const int a = off == pl ? 0 : off == pl - 1 ? 1 : off == pl - nx ? 2 : off == nx ? 3 : off == nx - 1 ? 4 : 5;
                    row[a] = Tx[q];
                }
            }
        });
    }
};

// mirror-symmetric widths (<= 16) of the j' = j + k columns, m = ny + nz - 1
std::vector<int> fill_widths(int m)
{
    int W = (m + lf::NJ - 1) / lf::NJ;
    for (;; W++) {
        const int base = m / W, extra = m % W;
        if (W % 2 == 0 && extra % 2) continue;  // an odd surplus needs a middle tile
        std::vector<int> w(W, base);
        for (int q = 0; q < extra / 2; q++) w[q]++, w[W - 1 - q]++;
        if (extra % 2) w[W / 2]++;
        return w;
    }
}

int fill_T(int nx, int nj, int np)
{
    // last row published: row nx of line nj-1, plane np-1
    const int T = nx + 2 * (nj - 1) + (np - 1) + lf::sig(np - 1) + 1;
    return (T + lf::LV - 1) / lf::LV * lf::LV;
}

int fill_upload(lssp_amd_ctx *c, const LineGeom &g, const std::vector<LineTile> &tiles, int W, const FillCoef &src,
                LineSweep &ls)
{
    using namespace lf;
    const int nx = g.nx, NA = src.NA;
    std::vector<LineTile> tt = tiles;
    long rows_total = 0;
    int tmax = 0;
    for (LineTile &t : tt) {
        t.roff = 0;
        t.cbase = rows_total;
        rows_total += (long)t.T * P * t.nj;
        tmax = std::max(tmax, t.T);
    }
    const long slack = 16 * 1024 / 8;  // the loaders' whole 1 KB pieces past the last block
    std::vector<double> coef((size_t)rows_total * NA + slack, 0.0);
    parallel_for((long)tt.size(), [&](long t0, long t1) {
        for (long ti = t0; ti < t1; ti++) {
            const LineTile &t = tt[ti];
            for (int p = 0; p < t.np; p++)
                for (int l = 0; l < t.nj; l++) {
                    const int j = t.j0 + l - (t.k0 + p);
                    if (j < 0 || j >= g.ny) continue;
                    const int off = 2 * l + p + sig(p);
                    for (int i = 0; i < nx; i++) {
                        const long v = i + off;
                        const long r = ((long)(t.k0 + p) * g.ny + j) * nx + i;
                        double *dst = coef.data() + (size_t)(t.cbase + v * P * t.nj + p * t.nj + l) * NA;
                        for (int a = 0; a < NA; a++) dst[a] = src.c[(size_t)r * NA + a];
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
    ls.P = P;
    ls.NJ = NJ;
    ls.LV = LV;
    LSSP_HIP(hipMalloc(&ls.d_tiles, sizeof(LineTile) * tt.size()));
    LSSP_HIP(hipMemcpy(ls.d_tiles, tt.data(), sizeof(LineTile) * tt.size(), hipMemcpyHostToDevice));
    LSSP_HIP(hipMalloc(&ls.d_coef, sizeof(double) * coef.size()));
    LSSP_HIP(hipMemcpy(ls.d_coef, coef.data(), sizeof(double) * coef.size(), hipMemcpyHostToDevice));
    LSSP_HIP(hipMalloc(&ls.d_claim, sizeof(unsigned long long)));
    LSSP_HIP(hipMemset(ls.d_claim, 0, sizeof(unsigned long long)));
    // claims in order of the tile's earliest start: a j-hop costs ~2 nj + 4
    // levels, a k-hop ~np + 1 + 4; both producers of a tile come before it
    const int nt = (int)tt.size();
    std::vector<int> ord(nt);
    for (int q = 0; q < nt; q++) ord[q] = q;
    std::stable_sort(ord.begin(), ord.end(), [W](int x, int y) {
        const long kx = (long)(x % W) * (2 * NJ + 4) + (long)(x / W) * (P + 5);
        const long ky = (long)(y % W) * (2 * NJ + 4) + (long)(y / W) * (P + 5);
        return kx != ky ? kx < ky : x < y;
    });
    LSSP_HIP(hipMalloc(&ls.d_order, sizeof(int) * nt));
    LSSP_HIP(hipMemcpy(ls.d_order, ord.data(), sizeof(int) * nt, hipMemcpyHostToDevice));
    ls.h_tiles = std::move(tt);
    return LSSP_AMD_OK;
}

}  // namespace

// ---------------------------------------------------------------------------
// 2-D grids (5-point ILU(0), and the 5-point ILU(1) pattern, nz = 1; exam.cxx's
// matrices) with at most G2_MAXNY lines: ONE workgroup sweeps the whole grid,
// lane j = line j, one level per step -- v = i + j (ILU(0)) or i + 2 j (ILU(1)),
// row i = v - j or v - 2 j.  Per level the operands are the lane's own x(v-1)
// (W), lane j-1's x(v-1) (ILU(0): S; ILU(1): SE -- DPP wave_shr:1, or the
// previous wave's lane 63 through LDS) and, for ILU(1), lane j-1's x(v-2) (S:
// the lane's SE of the previous level), so a level is one shift, two or three
// multiply-subtracts (+ U's division) and, with more than one wave, one LDS
// word and one barrier -- no hand-offs between CUs.  The tiled sweeps put one
// plane per tile on 16 of 128 lanes and chain the tiles of a 2-D grid through
// cross-CU hand-offs for the same levels.  Streams, level-major: [v][S, (SE,)
// W, (diag,) rhs][lane] (rows off the grid +0.0), the coefficients at build,
// the rhs per apply (k_lineg_rhs gathers the first sweep's; the L sweep writes
// the U sweep's); each wave LDS-DMAs its pieces G2_D levels ahead into a ring.
// ---------------------------------------------------------------------------
int build_lineg(lssp_amd_ctx *c, const LineGeom &g, int fill, int ncl, const std::vector<double> &cl,
                const std::vector<double> &cu, LineILU &li)
{
    const int nx = g.nx, ny = g.ny, NYP = (ny + 63) / 64 * 64, sk = fill ? 2 : 1, V = nx + sk * (ny - 1);
    const int ncu = fill ? 4 : 3;
    const int NW = NYP / 64;
    auto make = [&](const std::vector<double> &src, int NC) {
        std::vector<double> st((size_t)V * (NC + 1) * NYP + 128, 0.0);  // (+1 KB: whole DMA pieces)
        for (int v = 0; v < V; v++)
            for (int j = 0; j < ny; j++) {
                const int i = v - sk * j;
                if (i < 0 || i >= nx) continue;
                const double *cr = src.data() + ((size_t)j * nx + i) * NC;  // (sweep order: U mirrored)
                for (int k = 0; k < NC; k++) st[g2_at(v, NW, NC, k, j)] = cr[k];
            }
        return st;
    };
    const std::vector<double> sl = make(cl, ncl), su = make(cu, ncu);
    LSSP_HIP(hipMalloc(&li.d_g2L, sizeof(double) * sl.size()));
    LSSP_HIP(hipMemcpy(li.d_g2L, sl.data(), sizeof(double) * sl.size(), hipMemcpyHostToDevice));
    LSSP_HIP(hipMalloc(&li.d_g2U, sizeof(double) * su.size()));
    LSSP_HIP(hipMemcpy(li.d_g2U, su.data(), sizeof(double) * su.size(), hipMemcpyHostToDevice));
    li.g = g;
    li.kind = fill;
    li.g2 = 1;
    li.g2fill = fill;
    li.g2V = V;
    li.g2NYP = NYP;
    li.g2NCL = ncl;
    li.g2NCU = ncu;
    li.P = 1;
    li.NJ = ny;
    li.LV = 1;
    li.W = li.S = 1;
    li.ntiles = 1;  // (line sweeps active; no tiles, claims or hand-off buffers)
    return LSSP_AMD_OK;
}

int build_linefill(lssp_amd_ctx *c, int n, const std::vector<int> &Lp, const std::vector<int> &Lj,
                   const std::vector<double> &Lx, const std::vector<int> &Up, const std::vector<int> &Uj,
                   const std::vector<double> &Ux, LineILU &li)
{
    using namespace lf;
    LineGeom g;
    if (!detect_fill1(n, Lp, Lj, Lx, Up, Uj, g)) return LSSP_AMD_EUNSUPPORTED;
    {
        const char *e = getenv("LSSP_AMD_LINEG");  // (read per build: tests select either path)
        if (g.nz == 1 && g.ny <= G2_MAXNY && lineg_fits(g, 1) && !(e && !atoi(e))) {
            const long pl = (long)g.nx * g.ny;
            FillCoef fl, fu;
            fl.build(Lp, Lj, Lx, false, n, g.nx, pl, g.unitL ? 6 : 7);
            fu.build(Up, Uj, Ux, true, n, g.nx, pl, 7);
            // k_lineg's components: S, SE, W (, diag) = FillCoef's 3, 4, 5 (, 6)
            const int ncl = g.unitL ? 3 : 4;
            std::vector<double> cl((size_t)n * ncl), cu((size_t)n * 4);
            for (long r = 0; r < n; r++) {
                for (int k = 0; k < ncl; k++) cl[r * ncl + k] = fl.c[r * fl.NA + 3 + k];
                for (int k = 0; k < 4; k++) cu[r * 4 + k] = fu.c[r * fu.NA + 3 + k];
            }
            return build_lineg(c, g, 1, ncl, cl, cu, li);
        }
    }
    const int m = g.ny + g.nz - 1;
    const std::vector<int> wd = fill_widths(m);
    const int W = (int)wd.size(), S = (g.nz + P - 1) / P;
    std::vector<int> js(W + 1, 0);
    for (int J = 0; J < W; J++) js[J + 1] = js[J] + wd[J];
    std::vector<LineTile> Lt((size_t)S * W), Ut((size_t)S * W);
    auto flags = [&](int K, int J) {
        return (K > 0 ? LT_KIN : 0) | (J > 0 ? LT_JIN : 0) | (K < S - 1 ? LT_KOUT : 0) | (J < W - 1 ? LT_JOUT : 0);
    };
    for (int K = 0; K < S; K++)
        for (int J = 0; J < W; J++) {
            LineTile &t = Lt[(size_t)K * W + J];
            t = LineTile{};
            t.j0 = js[J];
            t.nj = wd[J];
            t.k0 = K * P;
            t.np = std::min(P, g.nz - t.k0);
            t.flags = flags(K, J);
            t.T = fill_T(g.nx, t.nj, t.np);
            t.tk = K > 0 ? (K - 1) * W + J : -1;
            t.tj = J > 0 ? K * W + J - 1 : -1;
            // the U tile (W-1-J, S-1-K) is this tile mirrored
            const int Kp = S - 1 - K, Jp = W - 1 - J;
            LineTile &u = Ut[(size_t)Kp * W + Jp];
            u = t;
            u.j0 = m - t.j0 - t.nj;
            u.k0 = g.nz - t.k0 - t.np;
            u.flags = flags(Kp, Jp);
            u.tk = Kp > 0 ? (Kp - 1) * W + Jp : -1;
            u.tj = Jp > 0 ? Kp * W + Jp - 1 : -1;
        }
    // Tiles wholly off the grid -- every line j = j' - k of every plane outside
    // [0, ny), and so is line -1 (the j-input a tile forwards to its k-successor
    // through hk[Q][0]) -- hold only +0.0 rows: they are marked LT_SKIP (a
    // workgroup that claims one counts it done at once) and their consumers
    // read +0.0 inputs, as on the grid's edges.  In a cube about 40 % of the
    // S x W skewed tiles (j' = j + k spans ny + nz - 1 columns, a plane's lines
    // only ny of them).
    auto skip_off_grid = [&](std::vector<LineTile> &tv) {
        for (LineTile &t : tv) {
            const int lo = t.j0 - 1 - (t.k0 + t.np - 1), hi = t.j0 + t.nj - 1 - t.k0;
            if (hi < 0 || lo > g.ny - 1) t.flags |= LT_SKIP;
        }
        // (a producer of a skipped tile does not publish: the L and U sweeps share
        // the hand-off buffers, and an output no consumer re-arms would reach the
        // other sweep's tile of the same index as a stale value)
        for (LineTile &t : tv) {
            if (!(t.flags & LT_SKIP)) continue;
            if (t.tk >= 0) tv[t.tk].flags &= ~LT_KOUT;
            if (t.tj >= 0) tv[t.tj].flags &= ~LT_JOUT;
        }
        for (LineTile &t : tv) {
            if (t.flags & LT_SKIP) continue;
            if (t.tk >= 0 && (tv[t.tk].flags & LT_SKIP)) {
                t.flags &= ~LT_KIN;
                t.tk = -1;
            }
            if (t.tj >= 0 && (tv[t.tj].flags & LT_SKIP)) {
                t.flags &= ~LT_JIN;
                t.tj = -1;
            }
        }
    };
    skip_off_grid(Lt);
    skip_off_grid(Ut);
    const long pl = (long)g.nx * g.ny;
    const int NAL = g.unitL ? 6 : 7;
    FillCoef cl, cu;
    cl.build(Lp, Lj, Lx, false, n, g.nx, pl, NAL);
    cu.build(Up, Uj, Ux, true, n, g.nx, pl, 7);
    li.g = g;
    li.kind = 1;
    li.P = P;
    li.NJ = NJ;
    li.LV = LV;
    li.W = W;
    li.S = S;
    LSSP_TRY(fill_upload(c, g, Lt, W, cl, li.L));
    LSSP_TRY(fill_upload(c, g, Ut, W, cu, li.U));
    for (int K = 0; K < S; K++)
        for (int J = 0; J < W; J++) {
            LineTile &l = li.L.h_tiles[(size_t)K * W + J];
            l.ut = (S - 1 - K) * W + (W - 1 - J);
            l.ubase = li.U.h_tiles[l.ut].cbase;
        }
    LSSP_HIP(hipMemcpy(li.L.d_tiles, li.L.h_tiles.data(), sizeof(LineTile) * li.L.h_tiles.size(),
                       hipMemcpyHostToDevice));
    const long slack = 16 * 1024 / 8;
    LSSP_HIP(hipMalloc(&li.d_ustream, sizeof(double) * (li.U.rows_total + slack)));
    LSSP_HIP(hipMemset(li.d_ustream, 0, sizeof(double) * (li.U.rows_total + slack)));  // rows off the grid stay +0.0
    LSSP_HIP(hipMalloc(&li.d_lstream, sizeof(double) * (li.L.rows_total + slack)));
    LSSP_HIP(hipMemset(li.d_lstream, 0, sizeof(double) * (li.L.rows_total + slack)));
    li.tmax = std::max(li.L.tmax, li.U.tmax);
    // rows: every step the poller may address (steps up to TS + DH + 1, two rows each, + HJ0)
    const long rows = li.tmax + 32;
    li.hk_stride = rows * HKS;
    li.hj_stride = rows * P;
    li.ntiles = (int)Lt.size();
    li.hk_n = li.hk_stride * li.ntiles;
    li.hj_n = li.hj_stride * li.ntiles;
    LSSP_HIP(hipMalloc(&li.d_hk, sizeof(double) * li.hk_n));
    LSSP_HIP(hipMalloc(&li.d_hj, sizeof(double) * li.hj_n));
    LSSP_TRY(line_rearm(c, li));
    LSSP_HIP(hipStreamSynchronize(c->stream));
    return LSSP_AMD_OK;
}

// ---------------------------------------------------------------------------
// device
// ---------------------------------------------------------------------------
struct FillArgs {
    int nx, ny, ntiles;
    long n;
    const LineTile *tiles;
    const double *coef;
    const double *rhs;  // the sweep's rhs stream
    double *out;        // OUT 1: natural-order output; OUT 2: the U rhs stream
    double *hk, *hj;
    long hk_stride, hj_stride;
    unsigned long long *claim;
    unsigned long long base;
    const int *order;  // the tile of each claim
    int mirror;        // U sweep: natural row = n-1 - sweep row
    int *err;
    const double *guard;  // lssp_amd_ctx::guard
    int tail;     // OUT 1: run the product tl after the tiles (linesweep_dev.h LineTail)
    LineTail tl;
};

template <int NA, int OUT, int NL, int D, int DH, int SW, bool TL = false>
__global__ __launch_bounds__(64 * lf::waves(NL, SW)) void k_linef(FillArgs a)
{
    // TL: the instantiation that can run the tail product (kept apart so the
    // plain sweep does not carry the product's registers; k_line2 alike)
    static_assert(!TL || OUT == 1, "the tail product follows the natural-order sweep");
    const bool tail = TL && a.tail;
    using namespace lf;
    using SL = Slot<NA>;
    constexpr int LA = 2;  // the loaders complete step s+LA's slot during step s
    constexpr int R = D + 1;
    constexpr int RSL = rsl<OUT>();
#ifndef LINEF_NITEM
    constexpr int NITEM = SL::NPC + SL::NRP;
#else
    constexpr int NITEM = LINEF_NITEM;  // timing experiments only: a step's later DMA pieces are not loaded
#endif
    constexpr int KPER = (NITEM + NL - 1) / NL;
    constexpr int S0 = -2 * ((D + 2) / 2);  // first step of every role (even, <= -D-1)
    constexpr int SC = -1;                  // first computed step: levels -2, -1 prime S, B
    static_assert(DH >= 2 && DH < D && (D - LA) * KPER <= 63 && 2 * (DH - 1) <= 63, "leads");
    static_assert(OUT == 1 || OUT == 2, "out");
    static_assert(NA == 6 || NA == 7, "coefficients");
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

    int done_tile = -1;  // the tile this workgroup finished last (counted at the next claim)
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) {
            if (OUT == 1 && tail && done_tile >= 0)  // its storers' write-through stores drained before the barrier
                __hip_atomic_fetch_add(a.tl.kdone + done_tile / a.tl.W, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int c = (int)(atomicAdd(a.claim, 1ull) - a.base);
            *s_tile = c < a.ntiles ? a.order[c] : a.ntiles;
        }
        __syncthreads();
        const int t = __builtin_amdgcn_readfirstlane(*s_tile);
        if (t >= a.ntiles) break;
        done_tile = t;
        const LineTile d = a.tiles[t];
        if (d.flags & LT_SKIP) continue;  // wholly off the grid (build_linefill)
        const int T = d.T, TS = T / LV, nj = d.nj, np = d.np;
        const long SB = (long)P * nj;  // rows per level block
        const bool kin = d.flags & LT_KIN, jin = d.flags & LT_JIN, kout = d.flags & LT_KOUT,
                   jout = d.flags & LT_JOUT;
        const int ll = lane & (NJ - 1), gl = lane >> 4;
        const int lc = min(ll, nj - 1);

        if (wave < 2) {
            // ---------------- compute: plane pw = 4 wave + g, line l ----------------
            const int pw = wave * 4 + gl;
            const int off = 2 * ll + pw + wave;  // row i = v - off
            const int jg = d.j0 + ll - d.k0 - pw;
            const bool lane_ok = pw < np && ll < nj && (unsigned)jg < (unsigned)a.ny;
            struct In {
                double c[NA][LV];
                double rh[LV];
            };
            // the next step's coefficients and rhs from LDS (its slot)
            auto load = [&](unsigned sn, In &in) {
#pragma unroll
                for (int v = 0; v < LV; v++) {
                    const long r = v * SB + pw * nj + lc;
                    const double *b = reinterpret_cast<const double *>(ring + sn + SL::COEF) + r * NA;
#pragma unroll
                    for (int q = 0; q < NA; q++) in.c[q][v] = b[q];
                    in.rh[v] = reinterpret_cast<const double *>(ring + sn + SL::RHS)[r];
                }
            };
            const int pm = max(pw - 1, 0);
            In A, B;
            double xp = 0.0;   // x(v-1)
            double bnp = 0.0;  // BN(v-1)
            double sep = 0.0;  // SE(v-1) = S(v)
            double bep = 0.0;  // BE(v-1) = B(v)
            double xs = 0.0;   // lane - 16's x of the previous step's last level
            constexpr int OOB = 0x40000000;  // voffset that drops a buffer store (soffset is not range-checked)
            const __amdgpu_buffer_rsrc_t hko =
                __builtin_amdgcn_make_buffer_rsrc(a.hk + (long)t * a.hk_stride, 0, (int)(a.hk_stride * 8), 0x00020000);
            const __amdgpu_buffer_rsrc_t hjo =
                __builtin_amdgcn_make_buffer_rsrc(a.hj + (long)t * a.hj_stride, 0, (int)(a.hj_stride * 8), 0x00020000);
            // plane np-1 (group gk of this wave) feeds the next k-tile
            const int gk = np - 1 - 4 * wave;
            const bool kw = kout && gk >= 0 && gk < 4;
            const int sgk = sig(np - 1);
            auto publish = [&](int v, double x, double se) {
                if (kw) {  // uniform
                    const int Q = v - (np - 1) - sgk + 2;
                    const int i = v - 2 * ll - (np - 1) - sgk;
                    const bool m1 = gl == gk && ll < nj && (unsigned)i <= (unsigned)nx;
                    const bool m0 = gl == gk && ll == 0 && (unsigned)(i + 1) <= (unsigned)nx;
                    int vo1 = m1 ? (1 + ll) * 8 : OOB, vo0 = m0 ? 0 : OOB;
                    if (Q < 0) vo1 = vo0 = OOB;
                    const int so = max(Q, 0) * (HKS * 8);
                    __builtin_amdgcn_raw_buffer_store_b64(split64((uint64_t)__double_as_longlong(x)), hko, vo1, so, 16);
                    __builtin_amdgcn_raw_buffer_store_b64(split64((uint64_t)__double_as_longlong(se)), hko, vo0, so, 16);
                }
                if (jout) {
                    const int q = v - 2 * (nj - 1);
                    const bool mj = ll == nj - 1 && pw < np && (unsigned)(q - pw - wave) <= (unsigned)nx;
                    int vo = mj ? pw * 8 : OOB;
                    if (q + HJ0 < 0) vo = OOB;
                    __builtin_amdgcn_raw_buffer_store_b64(split64((uint64_t)__double_as_longlong(x)), hjo, vo,
                                                          max(q + HJ0, 0) * (P * 8), 16);
                }
            };
            unsigned so = (unsigned)(((S0 % R) + R) % R) * SL::BYTES;  // slot of step s
            constexpr unsigned RB = (unsigned)(R * SL::BYTES);
            auto body = [&](int s, In &cur, In &nxt) {
                const unsigned sn = so + SL::BYTES == RB ? 0u : so + SL::BYTES;  // slot of step s+1
                const unsigned sp = so == 0 ? RB - SL::BYTES : so - SL::BYTES;    // slot of step s-1
                // group 0's k-sources: wave 0 the poller's k-input (BN: entry 1+l,
                // line 0's BE: entry 0), wave 1 plane 3's results of the previous step
                double kx0, kx1, kb0 = 0.0, kb1 = 0.0;
                if (wave == 0) {
                    const double *kf = reinterpret_cast<const double *>(ring + so + SL::KFIN);
                    kx0 = kf[1 + ll];
                    kx1 = kf[HKS + 1 + ll];
                    kb0 = kf[0];
                    kb1 = kf[HKS];
                } else {
                    kx0 = res[((2 * s - 2) & (RSL - 1)) * ROWS + 3 * NJ + ll];
                    kx1 = res[((2 * s - 1) & (RSL - 1)) * ROWS + 3 * NJ + ll];
                }
                // the j-inputs, read at the step that uses them (as k_line2's): this
                // step's slot, and the previous step's for the line -1 entries of
                // plane pw-1 one row back (slot rows: q = 2s+1, 2s+2 at [0], [1]; the
                // previous slot's 2s-1, 2s); line -1 of plane pw-1, row i+1: hj q = v - [pw == 4]
                double se0[LV], be0[LV];
                {
                    const double *jc = reinterpret_cast<const double *>(ring + so + SL::JFIN);
                    const double *jp = reinterpret_cast<const double *>(ring + sp + SL::JFIN);
#pragma unroll
                    for (int v = 0; v < LV; v++) {
                        se0[v] = jc[v * P + min(pw, P - 1)];
                        be0[v] = pw == 4 ? jp[v * P + 3] : (v == 0 ? jp[P + pm] : jc[pm]);
                    }
                }
                asm volatile("" ::: "memory");
                load(sn, nxt);
                if (s >= SC && s < TS) {
                    double xu = xs;  // lane - 16's x of the previous level
#pragma unroll
                    for (int lv = 0; lv < LV; lv++) {
                        const int v = 2 * s + lv;
                        const double bn = sel_lanes(G0M, lv == 0 ? kx0 : kx1, xu);
                        const double bel = wave == 0 ? sel_lanes(G0M, lv == 0 ? kb0 : kb1, be0[lv]) : be0[lv];
                        const double be = dpp_shr1g<4>(bnp, bel);
                        const double se = dpp_shr1g<4>(xp, se0[lv]);
                        double r = cur.rh[lv] - cur.c[0][lv] * bep;
                        r = r - cur.c[1][lv] * be;
                        r = r - cur.c[2][lv] * bn;
                        r = r - cur.c[3][lv] * sep;
                        r = r - cur.c[4][lv] * se;
                        r = r - cur.c[5][lv] * xp;
                        if constexpr (NA == 7) r = r / cur.c[6][lv];
                        const bool ok = lane_ok && (unsigned)(v - off) < (unsigned)nx;
                        const double x = sel_lanes(__builtin_amdgcn_ballot_w64(ok), r, 0.0);
                        // the next level's BN shuffle before this level's stores (as k_line2)
                        xu = up16(x);
                        __builtin_amdgcn_sched_barrier(0);
                        publish(v, x, se);
                        res[(v & (RSL - 1)) * ROWS + pw * NJ + ll] = x;
                        bep = be;
                        sep = se;
                        bnp = bn;
                        xp = x;
                    }
                    xs = xu;  // the next step's first BN, off its critical path
                }
                so = sn;
                line_barrier();
            };
            for (int s = S0; s <= TS; s += 2) {
                body(s, A, B);
                if (s + 1 <= TS) body(s + 1, B, A);
            }
        } else if (wave < 2 + NL) {
            // ---------------- loaders: a step's DMAs spread over the NL waves ----------------
            const int w = wave - 2;
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
                        // (non-temporal streams changed nothing here, unlike k_line2:
                        // profiles/r04/r04t_linef_nt_ab_dropped.txt)
                        dma16(cb + m * 1024 + lane * 16, sl + SL::COEF + m * 1024);
                    } else if (m < NITEM) {
                        const int r = m - SL::NPC;
                        dma16(ub + r * 1024 + lane * 16, sl + SL::RHS + r * 1024);
                    } else {
                        dma16(cb + lane * 16, sl + SL::COEF);  // keeps the per-wave count fixed
                    }
                }
            };
            for (int s = S0; s <= TS; s++) {
                issue(s + D);  // dummies past TS keep the wait counts exact
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - LA) * KPER) : "memory");
                line_barrier();
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if (wave == 2 + NL) {
            // ---------------- poller ----------------
            // At step s: LDS-DMA sc1 reads of step s+DH's k rows (hk rows 2q+2,
            // 2q+3: 2 x 18 entries, lanes 0..17 x 16 B) and step s+DH+1's j rows
            // (hj q = 2q+1, 2q+2: 2 x 8 entries, lanes 0..7); then the k-inputs of
            // step s+1 and the j-inputs of step s+2 are waited for and checked
            // (the compute reads the j-inputs one step ahead).  A tile without a
            // k (j) input gets +0.0 there.
            const double *hk = a.hk + (long)max(d.tk, 0) * a.hk_stride;
            const double *hj = a.hj + (long)max(d.tj, 0) * a.hj_stride;
            const int kmax = (int)(a.hk_stride / HKS) - 2, jmax = (int)(a.hj_stride / P) - 2;  // first rows of a pair
            const int ke = lane % HKS, klv = lane / HKS;  // k check: lanes 0..35 = (level, entry)
            const int jp = lane & (P - 1), jlv = lane / P;  // j check: lanes 0..15 = (level, plane)
            auto kval = [&](int q) {  // step q's entry of this lane is a row of the grid's lines
                const int Q = 2 * q + klv + 2, r = ke == 0 ? Q - 1 : Q - 2 * ke;
                return lane < LV * HKS && ke <= nj && r >= 0 && r <= nx;
            };
            auto kaddr = [&](int q) { return hk + (long)(2 * q + klv + 2) * HKS + ke; };
            auto jval = [&](int q) {
                const int qq = 2 * q + jlv + 1, r = qq - jp - sig(jp);
                return lane < LV * P && jp < np && r >= 0 && r <= nx;
            };
            auto jaddr = [&](int q) { return hj + (long)(2 * q + jlv + 1 + HJ0) * P + jp; };
            const unsigned sink = lds0 + (unsigned)(R * SL::BYTES + RSL * ROWS * 8 + 16);
            auto issue = [&](int q) {
                const int Q0 = min(max(2 * q + 2, 0), kmax);
                const int J0 = min(max(2 * q + 1 + HJ0, 0), jmax);
                const char *kp = reinterpret_cast<const char *>(hk + (long)Q0 * HKS) + lane * 16;
                const char *jp2 = reinterpret_cast<const char *>(hj + (long)J0 * P) + lane * 16;
                const unsigned ks = kin ? lds0 + (unsigned)((((q % R) + R) % R) * SL::BYTES + SL::KFIN) : sink;
                const unsigned js = jin ? lds0 + (unsigned)((((q % R) + R) % R) * SL::BYTES + SL::JFIN) : sink;
                if (lane < LV * HKS / 2) dma16_sc1(kp, ks);
                if (lane < LV * P / 2) dma16_sc1(jp2, js);
            };
            if (!kin || !jin) {
                for (int q = 0; q < R; q++) {
                    if (!kin && lane < LV * HKS) reinterpret_cast<double *>(ring + q * SL::BYTES + SL::KFIN)[lane] = 0.0;
                    if (!jin && lane < LV * P) reinterpret_cast<double *>(ring + q * SL::BYTES + SL::JFIN)[lane] = 0.0;
                }
            }
            __builtin_amdgcn_s_setprio(3);  // the polls enter the CU's memory queue ahead of the coefficient DMAs
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            for (int s = S0; s <= TS; s++) {
                issue(s + DH);
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (DH - 1)) : "memory");
                if (s > TS) break;
                const int qk = s + 1, qj = s + 1;  // steps (the j-inputs are read at their own step)
                // (steps from -1 are checked: the ring index of a negative step wraps)
                double *kslot = reinterpret_cast<double *>(ring + ((qk % R + R) % R) * SL::BYTES + SL::KFIN) +
                                min(lane, LV * HKS - 1);
                double *jslot = reinterpret_cast<double *>(ring + ((qj % R + R) % R) * SL::BYTES + SL::JFIN) +
                                min(lane, LV * P - 1);
                const bool vk = kin && qk >= SC && kval(qk), vj = jin && qj >= SC && jval(qj);
                const uint64_t kvb = vk ? (uint64_t)__double_as_longlong(*kslot) : 0;
                const uint64_t jvb = vj ? (uint64_t)__double_as_longlong(*jslot) : 0;
                const bool bk = vk && kvb == TRI_SENTINEL, bj = vj && jvb == TRI_SENTINEL;
                if (__any(bk || bj)) {
                    // resync: drain, wait for these values, re-issue the later polls
                    // (k_line2's episode)
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    auto spin = [&](const double *src) {
                        for (;;) {
                            const uint64_t b = line_ld_agent(src);
                            if (b != TRI_SENTINEL) return b;
                            if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) {  // 4 s
                                atomicOr(a.err, 8);
                                return (uint64_t)0x7FF8000000000000ull;
                            }
                            __builtin_amdgcn_s_sleep(1);
                        }
                    };
                    if (bk) *kslot = __longlong_as_double((long long)spin(kaddr(qk)));
                    if (bj) *jslot = __longlong_as_double((long long)spin(jaddr(qj)));
                    for (int k = 2; k <= DH; k++) issue(s + k);  // the polls issued at steps s+k-DH
                }
                line_barrier();
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            // ---------------- storers: results, re-arms ----------------
            // Storer 0 re-arms the consumed j-inputs, storer SW-1 the k-inputs.
            const int w = wave - (2 + NL + 1);
            const int ke = lane % HKS, klv = lane / HKS, jp = lane & (P - 1), jlv = lane / P;
            uint64_t *hki = reinterpret_cast<uint64_t *>(a.hk + (long)max(d.tk, 0) * a.hk_stride);
            uint64_t *hji = reinterpret_cast<uint64_t *>(a.hj + (long)max(d.tj, 0) * a.hj_stride);
            const bool rk = w == SW - 1 && kin && lane < LV * HKS && ke <= nj;
            const bool rj = w == 0 && jin && lane < LV * P && jp < np;
            auto rearm = [&](int q) {  // step q's entries
                const int Q = 2 * q + klv + 2, r = ke == 0 ? Q - 1 : Q - 2 * ke;
                if (rk && r >= 0 && r <= nx) hki[(long)Q * HKS + ke] = TRI_SENTINEL;
                const int qq = 2 * q + jlv + 1, rr = qq - jp - sig(jp);
                if (rj && rr >= 0 && rr <= nx) hji[(long)(qq + HJ0) * P + jp] = TRI_SENTINEL;
            };
            auto nat = [&](int p, int l, int i) {  // natural row of row i of line l, plane p (valid lane)
                const int j = d.j0 + l - d.k0 - p;
                const long r = ((long)(d.k0 + p) * a.ny + j) * nx + i;
                return a.mirror ? a.n - 1 - r : r;
            };
            if constexpr (OUT == 1) {
                // block B (levels 8B .. 8B+7, steps 4B .. 4B+3) is written during
                // steps 4B+4 .. 4B+7, a quarter per step: value k of the block is
                // level 8B + (k & 7) of run k >> 3 = (plane, line), so 8 lanes store
                // 8 consecutive rows of one line
                static_assert(RSL == 16 && (2 * ROWS) % (64 * SW) == 0, "runs");
                auto slice = [&](int s) {
                    const int Bk = (s >> 2) - 1, u = s & 3;
                    if (Bk < 0) return;
                    constexpr int PER = ROWS * 8 / 4 / 64 / SW;  // values per lane per step
#pragma unroll
                    for (int it = 0; it < PER; it++) {
                        const int k = u * (ROWS * 2) + (w * PER + it) * 64 + lane;
                        const int m = k & 7, r = k >> 3, p = r >> 4, l = r & (NJ - 1);
                        const int q = 8 * Bk + m;
                        const int i = q - 2 * l - p - sig(p);
                        const int j = d.j0 + l - d.k0 - p;
                        const double x = res[(q & (RSL - 1)) * ROWS + p * NJ + l];
                        if (p < np && l < nj && (unsigned)j < (unsigned)a.ny && (unsigned)i < (unsigned)nx) {
                            if (tail) st_sc1d(a.out + nat(p, l, i), x);  // read by the tail product on other CUs
                            else a.out[nat(p, l, i)] = x;
                        }
                    }
                };
                for (int s = S0; s <= TS; s++) {
                    if (s >= 0) slice(s);
                    if (s >= 1 && s <= TS) rearm(s - 1);
                    line_barrier();
                }
                rearm(-1);  // step -1's entries (levels -2, -1)
                // the last blocks' remaining quarters (every result is in LDS)
                for (int s = TS + 1; s < 4 * ((T - 1) / 8) + 8; s++) slice(s);
                if (tail) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // before the tile is counted
            } else {
                // step s-1's two levels: value k = 64 (w + SW u) + lane is level
                // 2(s-1) + (k >> 7), plane (k >> 4) & 7, line k & 15; its place in the
                // mirror U tile's rhs stream (same nj, np): level Cp - v with
                // Cp = nx - 1 + 2 (nj - 1) + np - 1 + sigma(p) + sigma(np-1-p)
                constexpr int PS = LV * ROWS / 64 / SW;
                static_assert(LV * ROWS % (64 * SW) == 0, "chunks");
                double *po[PS];
                int vlo[PS], lvs[PS], roff[PS];
#pragma unroll
                for (int u = 0; u < PS; u++) {
                    const int k = (w + u * SW) * 64 + lane;
                    const int lv = k / ROWS, p = (k >> 4) & (P - 1), l = k & (NJ - 1);
                    const int pp = min(p, np - 1), lq = min(l, nj - 1);
                    const int j = d.j0 + l - d.k0 - p;
                    lvs[u] = lv;
                    roff[u] = p * NJ + l;
                    vlo[u] = p < np && l < nj && (unsigned)j < (unsigned)a.ny ? 2 * l + p + sig(p) : 1 << 30;
                    const long Cp = (long)nx - 1 + 2 * (nj - 1) + np - 1 + sig(pp) + sig(np - 1 - pp);
                    po[u] = a.out + d.ubase + Cp * SB + (long)(np - 1 - pp) * nj + (nj - 1 - lq);
                }
                for (int s = S0; s <= TS; s++) {
                    const int q = s - 1;
                    if (q >= 0 && q < TS) {
#pragma unroll
                        for (int u = 0; u < PS; u++) {
                            const int v = LV * q + lvs[u];
                            const double x = res[(v & (RSL - 1)) * ROWS + roff[u]];
                            if ((unsigned)(v - vlo[u]) < (unsigned)nx) po[u][-SB * v] = x;
                        }
                    }
                    if (q >= SC && q < TS) rearm(q);
                    line_barrier();
                }
            }
        }
    }
    if constexpr (TL) {
        if (a.tail) {  // no tile left for this workgroup: its waves run the tail product
            int *soff = reinterpret_cast<int *>(smem);  // (the ring's LDS is free now; linef_launch_t reserves TAIL_LDS_BYTES)
            __syncthreads();
            if (threadIdx.x < a.tl.ndiag) soff[threadIdx.x] = a.tl.off[threadIdx.x];
            __syncthreads();
            line_tail_wg(a.tl, a.out, a.err, smem);
        }
    }
}

// ---------------------------------------------------------------------------
// rhs gather and launches
// ---------------------------------------------------------------------------
// the natural-order rhs into a sweep's stream: block = (tile, 16 consecutive
// levels); value k of the block is level q0 + (k & 15) of line (k >> 4) & 15 of
// plane k >> 8, so 16 neighbouring lanes read one 128-byte run of a grid line
// (consecutive levels are consecutive rows i); rows off the grid stay +0.0 (the
// stream was zeroed).  All loads are issued before the stores.
constexpr int LF_RUN = 16;
__global__ __launch_bounds__(256) void k_linef_rhs(const LineTile *__restrict__ tiles, int nq, int nx, int ny, long n,
                                                  int mirror, const double *__restrict__ rhs,
                                                  double *__restrict__ out, const double *guard)
{
    using namespace lf;
    if (guard && *guard != 0.0) return;  // a batched iteration past the stop (lssp_amd_ctx::guard)
    const int t = blockIdx.x / nq, q0 = (blockIdx.x % nq) * LF_RUN;
    const LineTile d = tiles[t];
    if (q0 >= d.T) return;
    constexpr int NV = P * NJ * LF_RUN / 256;
    double v[NV];
    long o[NV];
#pragma unroll
    for (int it = 0; it < NV; it++) {
        const int k = it * 256 + threadIdx.x, m = k & (LF_RUN - 1), l = (k >> 4) & (NJ - 1), p = k >> 8;
        const int lv = q0 + m, i = lv - 2 * l - p - sig(p), j = d.j0 + l - d.k0 - p;
        const bool ok = lv < d.T && p < d.np && l < d.nj && (unsigned)j < (unsigned)ny && (unsigned)i < (unsigned)nx;
        const long r = ((long)(d.k0 + p) * ny + j) * nx + i;
        v[it] = ok ? rhs[mirror ? n - 1 - r : r] : 0.0;
        o[it] = ok ? d.cbase + (long)lv * P * d.nj + p * d.nj + l : -1;
    }
#pragma unroll
    for (int it = 0; it < NV; it++)
        if (o[it] >= 0) out[o[it]] = v[it];
}

// ---- k_lineg: the one-workgroup 2-D sweeps (build_lineg) ----
struct G2Args {
    int nx, ny, NYP, V;
    long n;
    double *sL, *sU;  // level-major streams (their rhs slots are written per apply)
    int ncl, ncu;
    int mode;         // 0: apply (L -> the U stream's rhs, U -> out); 1: L only; 2: U only (-> out)
    double *out;      // natural order
    const double *guard;
};
// (a single wave issues every instruction of a level, so the level's cost is
// its instruction count: no branches, no per-level address arithmetic)
template <int FILL, int NC, int D, bool TOU>
__device__ void lineg_sweep(const G2Args &a, const double *st, bool mirror, double *ustream, double *out, char *smem)
{
    constexpr int SK = FILL ? 2 : 1;  // row i = v - SK j
    constexpr int R = D + 1, PW = g2_pw(NC), WSB = PW * 1024;
    const int j = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(j >> 6), lane = j & 63;
    const int NW = blockDim.x >> 6, nx = a.nx, ny = a.ny, V = a.V;
    // boundary words [2][1 + waves][64]: wave w's lanes write row 1 + w, wave w
    // reads lane 63 of row w (row 0 stays +0.0: wave 0's line -1)
    double *bnd = reinterpret_cast<double *>(smem);
    char *wring = smem + G2_BND + wave * R * WSB;  // this wave's ring (slots of its own blocks)
    const unsigned wl0 = (unsigned)(uintptr_t)wring;
    constexpr long BLK = (NC + 1) * 64 * 8;  // bytes of a wave's block per level
    // the DMA cursor: level vi's block (source advanced per level, clamped at
    // V - 1: past it the loads are dummies that keep the counts), its ring slot
    const char *src = reinterpret_cast<const char *>(st) + (long)wave * BLK + lane * 16;
    const long step = (long)NW * BLK;
    int vi = 0, si = 0;
    auto issue = [&]() {
        const unsigned dst = __builtin_amdgcn_readfirstlane(wl0 + (unsigned)(si * WSB));
#pragma unroll
        for (int p = 0; p < PW; p++) dma16(src + p * 1024, dst + p * 1024);
        if (++vi < V) src += step;
        si = si == R - 1 ? 0 : si + 1;
    };
    // per level the wave's vector-memory queue gets one store (level v) and then
    // its PW DMAs (level v + D) -- the prologue a dropped store before each
    // level's DMAs -- so when level v + 2's pieces are waited for (early in
    // level v) exactly (PW + 1)(D - 3) younger operations exist: one count
    constexpr int WAITN = (PW + 1) * (D - 3);
    static_assert(WAITN <= 63, "gfx9 vmcnt");
    constexpr int OOB = 0x40000000;
    // (num_records bound every store: the off-grid lanes' offset OOB lies past them)
    const __amdgpu_buffer_rsrc_t ro = TOU
        ? __builtin_amdgcn_make_buffer_rsrc(ustream, 0, (int)((long)a.V * NW * (a.ncu + 1) * 512), 0x00020000)
        : __builtin_amdgcn_make_buffer_rsrc(out, 0, (int)(a.n * 8), 0x00020000);
    for (int q = j; q < 2 * 5 * 64; q += blockDim.x) bnd[q] = 0.0;  // (before level 0's barrier)
    for (int v = 0; v < D; v++) {
        __builtin_amdgcn_raw_buffer_store_b64(split64(0), ro, OOB, 0, 0);  // (dropped: keeps the counts)
        issue();
    }
    // components of levels v (cf), v + 1 (cn) and v + 2 (cq) in registers: level
    // v+2's LDS reads are issued early in level v, so no level waits for them
    double cf[NC + 1], cn[NC + 1], cq[NC + 1];
    int sr = 0;  // the ring slot of the next level to read
    auto fetch = [&](double (&c)[NC + 1]) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WAITN) : "memory");  // this wave's block of that level landed
        const double *sl = reinterpret_cast<const double *>(wring + sr * WSB);
#pragma unroll
        for (int k = 0; k <= NC; k++) c[k] = sl[k * 64 + lane];
        sr = sr == R - 1 ? 0 : sr + 1;
    };
    // (the first two levels' waits: their blocks have fewer younger operations
    // than the count, so wait for everything once)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    fetch(cf);
    fetch(cn);
    double xp = 0.0, sp = 0.0;  // the lane's x(v-1); lane j-1's x(v-2) (S)
    // per-lane store offsets advance with the level: row i = v - SK j (natural
    // r = j nx + i, mirrored n-1-r), or the U stream's slot of level V-1-v
    const long r0 = (long)j * nx - (long)SK * j;  // r at level 0
#pragma unroll 2
    for (int v = 0; v < V; v++) {
        if (NW > 1) line_barrier();  // level v-1's boundary words written
        const double bprev = bnd[((v - 1) & 1) * 320 + wave * 64 + 63];  // wave w-1's lane 63 (wave 0: +0.0)
        fetch(cq);  // level v + 2 (behind the boundary read in the LDS queue)
        const double se = dpp_shr1(xp, bprev);  // lane j-1's x(v-1) (lane 0: the previous wave's lane 63)
        const double rh = cf[NC];
        double x;
        if constexpr (FILL) {
            // the reference's order: S (r - nx), SE (r - nx + 1), W (r - 1)
            x = rh - cf[0] * sp;
            x = x - cf[1] * se;
            x = x - cf[2] * xp;
            if constexpr (NC == 4) x = x / cf[3];
        } else {
            // S (r - nx) = lane j-1's x(v-1), W (r - 1)
            x = rh - cf[0] * se;
            x = x - cf[1] * xp;
            if constexpr (NC == 3) x = x / cf[2];
        }
        const int i = v - SK * j;
        const bool ok = j < ny && (unsigned)i < (unsigned)nx;
        x = ok ? x : 0.0;  // rows off the grid hold +0.0
        sp = se;
        xp = x;
        bnd[(v & 1) * 320 + (wave + 1) * 64 + lane] = x;
        // one store per wave and level (off-grid lanes dropped): the U stream's rhs
        // slot of its level V-1-v, line ny-1-j (the mirror row), or the output
        int vo;
        if constexpr (TOU) vo = (int)(g2_at(V - 1 - v, NW, a.ncu, a.ncu, ny - 1 - j) * 8);
        else {
            const long r = r0 + v;
            vo = (int)((mirror ? a.n - 1 - r : r) * 8);
        }
        const int msk = -(int)ok;
        vo = (vo & msk) | (OOB & ~msk);  // (a select without a branch)
        __builtin_amdgcn_raw_buffer_store_b64(split64((uint64_t)__double_as_longlong(x)), ro, vo, 0, 0);
        issue();  // level v + D into the slot of level v - 1 (read early in level v - 3)
#pragma unroll
        for (int k = 0; k <= NC; k++) {
            cf[k] = cn[k];
            cn[k] = cq[k];
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int FILL, int NCL, int D>
__global__ __launch_bounds__(G2_MAXNY) void k_lineg(G2Args a)
{
    if (a.guard && *a.guard != 0.0) return;  // a batched iteration past the stop (lssp_amd_ctx::guard)
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (a.mode == 0) lineg_sweep<FILL, NCL, D, true>(a, a.sL, false, a.sU, a.out, smem);
    if (a.mode == 1) lineg_sweep<FILL, NCL, D, false>(a, a.sL, false, nullptr, a.out, smem);
    if (a.mode == 0) {
        // the U stream's rhs slots were written by this workgroup: drained above
        // (vmcnt 0); the workgroup fence and barrier order them before its DMAs
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        __syncthreads();
    }
    if (a.mode != 1) lineg_sweep<FILL, FILL ? 4 : 3, D, false>(a, a.sU, true, nullptr, a.out, smem);
}

// the first sweep's rhs into its stream's rhs slots
__global__ __launch_bounds__(256) void k_lineg_rhs(double *st, int NC, int sk, int V, int NYP, int nx, int ny, long n,
                                                   int mirror, const double *__restrict__ rhs, const double *guard)
{
    if (guard && *guard != 0.0) return;
    const long t = (long)blockIdx.x * 256 + threadIdx.x;
    if (t >= (long)V * NYP) return;
    const int v = (int)(t / NYP), j = (int)(t % NYP), i = v - sk * j;
    if (j >= ny || i < 0 || i >= nx) return;
    const long r = (long)j * nx + i;
    st[g2_at(v, NYP >> 6, NC, NC, j)] = rhs[mirror ? n - 1 - r : r];
}

int launch_lineg(lssp_amd_ctx *c, const LineILU &li, int mode, double *x, const double *rhs)
{
    const LineGeom &g = li.g;
    const long n = (long)g.nx * g.ny;
    const int NYP = li.g2NYP, V = li.g2V;
    // the first sweep's rhs
    double *st0 = mode == 2 ? li.d_g2U : li.d_g2L;
    const int nc0 = mode == 2 ? li.g2NCU : li.g2NCL;
    const long nt = (long)V * NYP;
    k_lineg_rhs<<<(nt + 255) / 256, 256, 0, c->stream>>>(st0, nc0, li.g2fill ? 2 : 1, V, NYP, g.nx, g.ny, n, mode == 2,
                                                         rhs, c->guard);
    LSSP_HIP(hipGetLastError());
    G2Args a{g.nx, g.ny, NYP, V, n, li.d_g2L, li.d_g2U, li.g2NCL, li.g2NCU, mode, x, c->guard};
    // (ILU(1): L 3 or 4 components, U 4; ILU(0): L 2 or 3, U 3).  The DMA lead D
    // covers the memory latency at ~0.1 us per level: 16 levels where the waves'
    // rings of 17 slots fit the LDS (up to 3 waves), 12 for 4 waves
    const int kv = li.g2fill * 2 + (li.g2NCL == (li.g2fill ? 4 : 3));
    const bool wide = NYP > 192;
    const int D = wide ? G2_DW : G2_D;
    const int lds = G2_BND + (NYP >> 6) * (D + 1) * g2_pw(4) * 1024;
    static_assert(G2_BND + 3 * (G2_D + 1) * g2_pw(4) * 1024 <= 160 * 1024 &&
                  G2_BND + 4 * (G2_DW + 1) * g2_pw(4) * 1024 <= 160 * 1024, "k_lineg LDS");
    void (*kern)(G2Args);
    if (wide) kern = kv == 3 ? k_lineg<1, 4, G2_DW> : kv == 2 ? k_lineg<1, 3, G2_DW> : kv == 1 ? k_lineg<0, 3, G2_DW> : k_lineg<0, 2, G2_DW>;
    else kern = kv == 3 ? k_lineg<1, 4, G2_D> : kv == 2 ? k_lineg<1, 3, G2_D> : kv == 1 ? k_lineg<0, 3, G2_D> : k_lineg<0, 2, G2_D>;
    static bool attr[8] = {};
    if (!attr[kv + 4 * wide]) {
        LSSP_HIP(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr[kv + 4 * wide] = true;
    }
    kern<<<1, NYP, lds, c->stream>>>(a);
    LSSP_HIP(hipGetLastError());
    return LSSP_AMD_OK;
}

namespace {
#ifndef LINEF_D
#define LINEF_D 6  // loader lead (steps of two levels)
#endif
#ifndef LINEF_DH
// poller lead (steps): 2 measured faster than 3 on both sweeps (128^3 ILU(1):
// L 382 / U 410 against 409 / 436 us; loading only 4 of the step's 16 KB
// changed little, so the sweeps are bound by their chain and hops, not by the
// loaders; profiles/r04/r04k_linef_variants_128.txt)
#define LINEF_DH 2
#endif
constexpr int LF_NL = 4, LF_SW = 4;

int linef_gather(lssp_amd_ctx *c, const LineSweep &ls, int mirror, const double *rhs, double *stream)
{
    const int nq = (ls.tmax + LF_RUN - 1) / LF_RUN;
    const long grid = (long)ls.ntiles * nq;
    const long n = (long)ls.nx * ls.ny * ls.nz;
    k_linef_rhs<<<grid, 256, 0, c->stream>>>(ls.d_tiles, nq, ls.nx, ls.ny, n, mirror, rhs, stream, c->guard);
    LSSP_HIP(hipGetLastError());
    return LSSP_AMD_OK;
}

template <int NA, int OUT>
int linef_launch_t(lssp_amd_ctx *c, const LineSweep &ls, const FillArgs &a)
{
    // (a sweep with natural-order output and the tail product reserves what the product needs)
    constexpr int lds0 = lf::lds_bytes<NA, OUT, LINEF_D>();
    constexpr int ldst = OUT == 1 && lds0 < TAIL_LDS_BYTES(0) ? TAIL_LDS_BYTES(0) : lds0;
    static_assert(ldst <= 160 * 1024, "LDS");
    const int lds = a.tail ? ldst : lds0;
    static_assert(OUT != 1 || lf::waves(LF_NL, LF_SW) >= TAIL_WAVES, "the tail product's roles");
    auto kern = k_linef<NA, OUT, LF_NL, LINEF_D, LINEF_DH, LF_SW>;
    auto kernt = k_linef<NA, OUT, LF_NL, LINEF_D, LINEF_DH, LF_SW, OUT == 1>;
    static bool attr = false;
    if (!attr) {
        LSSP_HIP(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds0));
        LSSP_HIP(hipFuncSetAttribute((const void *)kernt, hipFuncAttributeMaxDynamicSharedMemorySize, ldst));
        attr = true;
    }
    const int grid = std::min(ls.ntiles, c->num_cus);
    (a.tail ? kernt : kern)<<<grid, 64 * lf::waves(LF_NL, LF_SW), lds, c->stream>>>(a);
    ls.base += (unsigned long long)ls.ntiles + grid;
    LSSP_HIP(hipGetLastError());
    return LSSP_AMD_OK;
}

// one sweep of li (which: 0 L, 1 U) from its rhs stream; OUT 2: out = the U
// rhs stream, OUT 1: natural order (tail: the product after the tiles)
int linef_sweep(lssp_amd_ctx *c, const LineILU &li, int which, const double *stream, double *out, int outk,
                const LineTail *tail = nullptr)
{
    const LineSweep &ls = which ? li.U : li.L;
    FillArgs a{};
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
    a.tail = tail != nullptr && outk == 1;
    if (a.tail) a.tl = *tail;
    if (outk == 2) return ls.NA == 6 ? linef_launch_t<6, 2>(c, ls, a) : linef_launch_t<7, 2>(c, ls, a);
    return ls.NA == 6 ? linef_launch_t<6, 1>(c, ls, a) : linef_launch_t<7, 1>(c, ls, a);
}
}  // namespace

int launch_linefill_apply(lssp_amd_ctx *c, const LineILU &li, double *x, const double *rhs)
{
    if (li.g2) return launch_lineg(c, li, 0, x, rhs);
    LSSP_TRY(linef_gather(c, li.L, 0, rhs, li.d_lstream));
    LSSP_TRY(linef_sweep(c, li, 0, li.d_lstream, li.d_ustream, 2));
    return linef_sweep(c, li, 1, li.d_ustream, x, 1);
}

// the apply with the U sweep's tail product (launch_line_apply_spmv prepared T);
// returns the tail waves of the launch (each ends on one failed chunk claim)
int launch_linefill_apply_tail(lssp_amd_ctx *c, const LineILU &li, double *x, const double *rhs, const LineTail &T,
                               long *tail_waves)
{
    LSSP_TRY(linef_gather(c, li.L, 0, rhs, li.d_lstream));
    LSSP_TRY(linef_sweep(c, li, 0, li.d_lstream, li.d_ustream, 2));
    LSSP_TRY(linef_sweep(c, li, 1, li.d_ustream, x, 1, &T));
    *tail_waves = (long)std::min(li.U.ntiles, c->num_cus);  // (the tail's claimants: workgroups)
    return LSSP_AMD_OK;
}

int launch_linefill_sweep(lssp_amd_ctx *c, const LineILU &li, int which, double *x, const double *rhs)
{
    if (li.g2) return launch_lineg(c, li, which ? 2 : 1, x, rhs);
    double *st = which ? li.d_ustream : li.d_lstream;
    LSSP_TRY(linef_gather(c, which ? li.U : li.L, which, rhs, st));
    return linef_sweep(c, li, which, st, x, 1);
}

}  // namespace lssp_amd
