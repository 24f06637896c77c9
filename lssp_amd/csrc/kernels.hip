// kernels.hip -- gfx950 kernels of the LSSP Krylov hot path.
//
// Compiled with -ffp-contract=off: every a*b+c below is a v_mul_f64 followed
// by a v_add_f64, exactly like the x86-64 -O2 build of the reference, so the
// per-element arithmetic is bit-identical to mvops.cxx / vector.cxx /
// solver-tri.cxx and to the solver drivers' inline loops.
//
// Reductions follow ONE canonical order, shared by every pass
// that produces a dot product, including the SpMV epilogues:
//   level 1: aligned chunks of 256 elements, element 64q+l of a chunk on lane
//            l of wave q; each wave halves (xor butterfly == halving tree,
//            lane 0 result), then (w0 + w1) + (w2 + w3);
//   level 2: one 1024-lane workgroup; lane t adds partials t, t+1024, ... onto
//            0.0 in order; 16 waves halve; the 16 wave sums halve.
// oracle/lssp_oracle.c (dot_tree) restates this order on the CPU.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <type_traits>

#include "internal.h"

namespace lssp_amd {

// ---------------------------------------------------------------------------
// reduction helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v)
{
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = v + __shfl_xor(v, off, 64);
    return v;  // lane 0 holds the halving-tree result
}

// level-1 combine of one 256-element chunk held one element per thread of a
// 256-thread block; the block-combined value is written by thread 0.
template <int NRED>
__device__ __forceinline__ void chunk_reduce(double (&v)[NRED > 0 ? NRED : 1], double *part, long pcap,
                                             long chunk, double (*lds)[4])
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int r = 0; r < NRED; r++) {
        double s = wave_sum(v[r]);
        if (lane == 0) lds[r][wave] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int r = 0; r < NRED; r++)
            part[r * pcap + chunk] = (lds[r][0] + lds[r][1]) + (lds[r][2] + lds[r][3]);
    }
    __syncthreads();
}

__device__ void finalize(const Fin &f, const double *s, double *scal, double *trace)
{
    double t0 = s[0], t1 = f.nsum > 1 ? s[1] : 0.0;
    for (int k = 0; k < f.nsum; k++) scal[S_SUM0 + k] = s[k];
    switch (f.op) {
    case FIN_STORE:
        for (int k = 0; k < f.nsum; k++) scal[f.dst[k]] = s[k];
        break;
    case FIN_NORM:
        t0 = sqrt(s[0]);
        scal[f.dst[0]] = t0;
        break;
    case FIN_BICG_RHO: {  // solver-bicgstab.cxx:87, :99, :105
        double rho1 = s[0];
        scal[S_RHO1] = rho1;
        scal[S_BETA] = (rho1 * scal[S_ALPHA]) / (scal[S_RHO0] * scal[S_OMEGA]);
        scal[S_RHO0] = rho1;
        break;
    }
    case FIN_BICG_ALPHA:  // :112
        scal[S_ALPHA] = scal[S_RHO1] / s[0];
        break;
    case FIN_BICG_S: {  // :117
        t0 = sqrt(s[0]);
        scal[S_SNORM] = t0;
        scal[S_BREAK] = t0 <= 1e-40 ? 1.0 : 0.0;
        break;
    }
    case FIN_BICG_OMEGA:  // :135
        scal[S_OMEGA] = s[0] / s[1];
        break;
    case FIN_BICG_RES_RHO: {  // :141 then the next iteration's :87
        t0 = sqrt(s[0]);
        scal[S_RES] = t0;
        double rho1 = s[1];
        t1 = rho1;
        scal[S_RHO1] = rho1;
        scal[S_BETA] = (rho1 * scal[S_ALPHA]) / (scal[S_RHO0] * scal[S_OMEGA]);
        scal[S_RHO0] = rho1;
        break;
    }
    case FIN_CG_RHO:  // solver-cg.cxx:80, :88
        scal[S_RHO1] = s[0];
        scal[S_BETA] = s[0] / scal[S_RHO0];
        break;
    case FIN_CG_ALPHA:  // :96-99
        scal[S_ALPHA] = scal[S_RHO1] / s[0];
        scal[S_RHO0] = scal[S_RHO1];
        break;
    case FIN_CG_RES:  // :106
        t0 = sqrt(s[0]);
        scal[S_RES] = t0;
        break;
    case FIN_CG_RES_RHO: {  // :106, then the next :80 with z == r (PC_NON)
        t0 = sqrt(s[0]);
        scal[S_RES] = t0;
        t1 = s[0];
        scal[S_RHO1] = s[0];
        scal[S_BETA] = s[0] / scal[S_RHO0];
        break;
    }
    }
    if (trace) {
        if (f.tpos[0] >= 0) trace[f.tpos[0]] = t0;
        if (f.tpos[1] >= 0) trace[f.tpos[1]] = t1;
    }
}

// level 2 (tree) + finalize
__global__ __launch_bounds__(1024) void k_reduce2(const double *__restrict__ part, long pcap, long C,
                                                  int nslot, double *sums, double *scal, double *trace,
                                                  Fin f, int do_fin)
{
    __shared__ double wsum[MAX_SLOTS][16];
    const int t = threadIdx.x;
    for (int s = 0; s < nslot; s++) {
        const double *p = part + s * pcap;
        double a = 0.0;
#pragma unroll 8
        for (long k = t; k < C; k += L2_LANES) a += p[k];
        a = wave_sum(a);
        if ((t & 63) == 0) wsum[s][t >> 6] = a;
    }
    __syncthreads();
    if (t == 0) {
        double r[MAX_SLOTS] = {0, 0, 0, 0};
        for (int s = 0; s < nslot; s++) {
            double u[16];
            for (int q = 0; q < 16; q++) u[q] = wsum[s][q];
            for (int off = 8; off >= 1; off >>= 1)
                for (int l = 0; l < off; l++) u[l] = u[l] + u[l + off];
            r[s] = u[0];
            sums[s] = r[s];
        }
        if (do_fin) finalize(f, r, scal, trace);
    }
}

// serial order: one lane, sum += a[i]*b[i] from 0 (vector.cxx:123-133)
struct SerialArgs {
    const double *a[MAX_SLOTS];
    const double *b[MAX_SLOTS];
};

__global__ void k_dot_serial(SerialArgs g, long n, int nslot, double *sums, double *scal,
                             double *trace, Fin f, int do_fin)
{
    double r[MAX_SLOTS] = {0, 0, 0, 0};
    for (int s = 0; s < nslot; s++) {
        const double *x = g.a[s], *y = g.b[s];
        double acc = 0;
        long i = 0;
        for (; i + 8 <= n; i += 8) {
            double p[8];
#pragma unroll
            for (int u = 0; u < 8; u++) p[u] = x[i + u] * y[i + u];
#pragma unroll
            for (int u = 0; u < 8; u++) acc += p[u];
        }
        for (; i < n; i++) acc += x[i] * y[i];
        r[s] = acc;
        sums[s] = acc;
    }
    if (do_fin) finalize(f, r, scal, trace);
}

__global__ void k_finalize(const double *sums, double *scal, double *trace, Fin f)
{
    double r[MAX_SLOTS];
    for (int s = 0; s < MAX_SLOTS; s++) r[s] = s < f.nsum ? sums[s] : 0.0;
    finalize(f, r, scal, trace);
}

// multi-rank: gathered [P][MAX_SLOTS] rank sums, summed in rank order
__global__ void k_sum_ranks(const double *gath, int P, int nslot, double *sums, double *scal,
                            double *trace, Fin f)
{
    double r[MAX_SLOTS] = {0, 0, 0, 0};
    for (int s = 0; s < nslot; s++) {
        double t = gath[s];
        for (int q = 1; q < P; q++) t = t + gath[q * MAX_SLOTS + s];
        r[s] = t;
        sums[s] = t;
    }
    finalize(f, r, scal, trace);
}

// ---------------------------------------------------------------------------
// SpMV: one 256-row block == one reduction chunk; every row summed by ONE
// lane in CSR order from 0.0 (mvops.cxx:49-62).  The block's Aj/Ax range is
// staged through LDS with coalesced loads when it fits, otherwise the lanes
// read their rows straight from HBM (same arithmetic).
// ---------------------------------------------------------------------------
constexpr int SPMV_CAP = 2048;

struct SpmvArgs {
    int nrows;
    const int *Ap, *Aj;
    const double *Ax, *x, *y;
    double *z;
    double alpha, beta;
    const double *w0, *w1;  // fused dot operands: red0 = z*w0, red1 = z*(w1 ? w1 : z)
    double *part;
    long pcap;
};

// XCD != 0: the 256-row blocks are dealt so that each of the 8 XCDs owns one
// contiguous eighth of the rows (dispatch round-robins workgroups over XCDs,
// workgroup w runs on XCD w % 8); the x entries a block gathers are then
// re-used by the neighbouring blocks of the same XCD out of its L2 (7-pt:
// x is fetched once instead of ~1.3 times, rocprofv3 FETCH_SIZE).
template <int EPI, int NRED, int XCD>
__global__ __launch_bounds__(256) void k_spmv(SpmvArgs a, long nblk)
{
    __shared__ int sj[SPMV_CAP];
    __shared__ double sx[SPMV_CAP];
    __shared__ double lds[MAX_SLOTS][4];
    long blk = blockIdx.x;
    if (XCD) {
        const long per = gridDim.x / 8;
        blk = (blockIdx.x % 8) * per + blockIdx.x / 8;
        if (blk >= nblk) return;
    }
    const int r0 = (int)(blk * 256);
    const int tid = threadIdx.x;
    const int r = r0 + tid;
    const int rend = min(r0 + 256, a.nrows);
    const int base = a.Ap[r0];
    const int cnt = a.Ap[rend] - base;
    double sum = 0;
    if (cnt <= SPMV_CAP) {
        for (int k = tid; k < cnt; k += 256) {
            sj[k] = __builtin_nontemporal_load(a.Aj + base + k);
            sx[k] = __builtin_nontemporal_load(a.Ax + base + k);
        }
        __syncthreads();
        if (r < a.nrows) {
            const int b = a.Ap[r] - base, e = a.Ap[r + 1] - base;
            for (int k = b; k < e; k++) sum += a.x[sj[k]] * sx[k];
        }
    } else if (r < a.nrows) {
        const int b = a.Ap[r], e = a.Ap[r + 1];
        for (int k = b; k < e; k++) sum += a.x[a.Aj[k]] * a.Ax[k];
    }
    double zv = 0;
    if (r < a.nrows) {
        if (EPI == EPI_MXY) zv = sum;                          // mvops.cxx:134
        else if (EPI == EPI_AMXY) zv = sum * a.alpha;          // :99
        else if (EPI == EPI_AXPBY) zv = a.y[r] * a.beta + a.alpha * sum;  // :23, :61
        else zv = a.alpha * sum;  // :61 with beta == 0 and alpha > 0
        a.z[r] = zv;
    }
    if (NRED > 0) {
        double v[NRED > 0 ? NRED : 1];
        if (r < a.nrows) {
            v[0] = zv * a.w0[r];
            if (NRED > 1) v[NRED > 1 ? 1 : 0] = zv * (a.w1 ? a.w1[r] : zv);
        } else {
#pragma unroll
            for (int q = 0; q < NRED; q++) v[q] = 0.0;
        }
        chunk_reduce<NRED>(v, a.part, a.pcap, blk, lds);
    }
}

// Variant 2: the block's Ax / Aj ranges are staged with 16-byte loads (the
// range is widened to 16-byte boundaries; the extra head/tail entries are
// dropped when landing in LDS), all loads of a thread are issued before any
// LDS store, and with XCD != 0 the 256-row blocks are dealt so that each of
// the 8 XCDs owns one contiguous eighth of the rows (dispatch round-robins
// blocks over XCDs: block b runs on XCD b % 8), keeping the x gathers of
// neighbouring blocks in one L2.  Same per-row arithmetic as k_spmv.
constexpr int SPMV2_CAP = 2048;
template <int EPI, int NRED, int XCD>
__global__ __launch_bounds__(256) void k_spmv2(SpmvArgs a, long nblk)
{
    __shared__ __attribute__((aligned(16))) double sx[SPMV2_CAP + 2];
    __shared__ __attribute__((aligned(16))) int sj[SPMV2_CAP + 4];
    __shared__ double lds[MAX_SLOTS][4];
    long blk = blockIdx.x;
    if (XCD) {
        const long per = gridDim.x / 8;
        blk = (blockIdx.x % 8) * per + blockIdx.x / 8;
        if (blk >= nblk) return;
    }
    const int r0 = (int)(blk * 256);
    const int tid = threadIdx.x;
    const int r = r0 + tid;
    const int rend = min(r0 + 256, a.nrows);
    const int base = a.Ap[r0];
    const int cnt = a.Ap[rend] - base;
    double sum = 0;
    if (cnt <= SPMV2_CAP) {
        const int xb = base & ~1, xn = (base + cnt - xb + 1) >> 1;  // double2 count
        const int jb = base & ~3, jn = (base + cnt - jb + 3) >> 2;  // int4 count
        typedef double dbl2_t __attribute__((ext_vector_type(2)));
        typedef int int4_t __attribute__((ext_vector_type(4)));
        const dbl2_t *X2 = reinterpret_cast<const dbl2_t *>(a.Ax + xb);
        const int4_t *J4 = reinterpret_cast<const int4_t *>(a.Aj + jb);
        dbl2_t vx[(SPMV2_CAP / 2 + 1 + 255) / 256];
        int4_t vj[(SPMV2_CAP / 4 + 1 + 255) / 256];
#pragma unroll
        for (int u = 0; u < (int)(sizeof(vx) / sizeof(vx[0])); u++)
            if (tid + 256 * u < xn) vx[u] = __builtin_nontemporal_load(X2 + tid + 256 * u);
#pragma unroll
        for (int u = 0; u < (int)(sizeof(vj) / sizeof(vj[0])); u++)
            if (tid + 256 * u < jn) vj[u] = __builtin_nontemporal_load(J4 + tid + 256 * u);
        const int ox = base - xb, oj = base - jb;  // LDS entry e lives at e + o
#pragma unroll
        for (int u = 0; u < (int)(sizeof(vx) / sizeof(vx[0])); u++)
            if (tid + 256 * u < xn) reinterpret_cast<dbl2_t *>(sx)[tid + 256 * u] = vx[u];
#pragma unroll
        for (int u = 0; u < (int)(sizeof(vj) / sizeof(vj[0])); u++)
            if (tid + 256 * u < jn) reinterpret_cast<int4_t *>(sj)[tid + 256 * u] = vj[u];
        __syncthreads();
        if (r < a.nrows) {
            const int b = a.Ap[r] - base, e = a.Ap[r + 1] - base;
            for (int k = b; k < e; k++) sum += a.x[sj[k + oj]] * sx[k + ox];
        }
    } else if (r < a.nrows) {
        const int b = a.Ap[r], e = a.Ap[r + 1];
        for (int k = b; k < e; k++) sum += a.x[a.Aj[k]] * a.Ax[k];
    }
    double zv = 0;
    if (r < a.nrows) {
        if (EPI == EPI_MXY) zv = sum;
        else if (EPI == EPI_AMXY) zv = sum * a.alpha;
        else if (EPI == EPI_AXPBY) zv = a.y[r] * a.beta + a.alpha * sum;
        else zv = a.alpha * sum;
        a.z[r] = zv;
    }
    if (NRED > 0) {
        double v[NRED > 0 ? NRED : 1];
        if (r < a.nrows) {
            v[0] = zv * a.w0[r];
            if (NRED > 1) v[NRED > 1 ? 1 : 0] = zv * (a.w1 ? a.w1[r] : zv);
        } else {
#pragma unroll
            for (int q = 0; q < NRED; q++) v[q] = 0.0;
        }
        chunk_reduce<NRED>(v, a.part, a.pcap, blk, lds);
    }
}

// Variant 3 of the staged SpMV: as k_spmv (XCD-ordered blocks), but every
// global access a lane makes before the barrier is issued up front and
// branch-free -- the block's Aj / Ax range as 16-byte loads (widened to 16-byte
// boundaries, clamped to the padded arrays; entries outside the block are
// dropped when landing in LDS) and the lane's own Ap[r], Ap[r+1] -- so one
// memory round trip covers the staging and the row bounds.
template <int EPI, int NRED>
__global__ __launch_bounds__(256) void k_spmv3(SpmvArgs a, long nblk, long nnz_pad)
{
    constexpr int NX2 = (SPMV_CAP / 2 + 1 + 255) / 256;  // double2 loads per lane
    constexpr int NJ4 = (SPMV_CAP / 4 + 1 + 255) / 256;  // int4 loads per lane
    __shared__ __attribute__((aligned(16))) double sx[SPMV_CAP + 2];
    __shared__ __attribute__((aligned(16))) int sj[SPMV_CAP + 4];
    __shared__ double lds[MAX_SLOTS][4];
    const long per = gridDim.x / 8;
    const long blk = (blockIdx.x % 8) * per + blockIdx.x / 8;
    if (blk >= nblk) return;
    const int r0 = (int)(blk * 256);
    const int tid = threadIdx.x;
    const int r = r0 + tid;
    const int rend = min(r0 + 256, a.nrows);
    const int base = a.Ap[r0];
    const int cnt = a.Ap[rend] - base;
    const int rr = min(r, a.nrows - 1);
    const int rb = a.Ap[rr], re = a.Ap[rr + 1];
    double sum = 0;
    if (cnt <= SPMV_CAP) {
        typedef double dbl2_t __attribute__((ext_vector_type(2)));
        typedef int int4_t __attribute__((ext_vector_type(4)));
        const long xb = base & ~1L, jb = base & ~3L;
        // clamp to the block's last vector: lanes past the range re-read it
        // (no extra lines), and the padded arrays keep it in bounds
        const long last = cnt > 0 ? (long)base + cnt - 1 : (long)base;
        const long xmax = min(last >> 1, (nnz_pad >> 1) - 1);
        const long jmax = min(last >> 2, (nnz_pad >> 2) - 1);
        const dbl2_t *X2 = reinterpret_cast<const dbl2_t *>(a.Ax);
        const int4_t *J4 = reinterpret_cast<const int4_t *>(a.Aj);
        dbl2_t vx[NX2];
        int4_t vj[NJ4];
#pragma unroll
        for (int u = 0; u < NX2; u++) vx[u] = __builtin_nontemporal_load(X2 + min((xb >> 1) + tid + 256 * u, xmax));
#pragma unroll
        for (int u = 0; u < NJ4; u++) vj[u] = __builtin_nontemporal_load(J4 + min((jb >> 2) + tid + 256 * u, jmax));
        const int xn = (int)(xmax - (xb >> 1)) + 1, jn = (int)(jmax - (jb >> 2)) + 1;  // vectors in range
#pragma unroll
        for (int u = 0; u < NX2; u++)
            if (tid + 256 * u < xn) reinterpret_cast<dbl2_t *>(sx)[tid + 256 * u] = vx[u];
#pragma unroll
        for (int u = 0; u < NJ4; u++)
            if (tid + 256 * u < jn) reinterpret_cast<int4_t *>(sj)[tid + 256 * u] = vj[u];
        __syncthreads();
        if (r < a.nrows) {
            const int ox = (int)(base - xb) - base, oj = (int)(base - jb) - base;
            const int len = re - rb;
            if (len > 0 && len <= 8) {
                // all x gathers of the row in flight at once; the products are
                // then added in CSR order (clamped extra lanes are not added)
                double pr[8];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int k = min(rb + u, re - 1);
                    pr[u] = a.x[sj[k + oj]] * sx[k + ox];
                }
#pragma unroll
                for (int u = 0; u < 8; u++)
                    if (u < len) sum += pr[u];
            } else {
                for (int k = rb; k < re; k++) sum += a.x[sj[k + oj]] * sx[k + ox];
            }
        }
    } else if (r < a.nrows) {
        for (int k = rb; k < re; k++) sum += a.x[a.Aj[k]] * a.Ax[k];
    }
    double zv = 0;
    if (r < a.nrows) {
        if (EPI == EPI_MXY) zv = sum;
        else if (EPI == EPI_AMXY) zv = sum * a.alpha;
        else if (EPI == EPI_AXPBY) zv = a.y[r] * a.beta + a.alpha * sum;
        else zv = a.alpha * sum;
        a.z[r] = zv;
    }
    if (NRED > 0) {
        double v[NRED > 0 ? NRED : 1];
        if (r < a.nrows) {
            v[0] = zv * a.w0[r];
            if (NRED > 1) v[NRED > 1 ? 1 : 0] = zv * (a.w1 ? a.w1[r] : zv);
        } else {
#pragma unroll
            for (int q = 0; q < NRED; q++) v[q] = 0.0;
        }
        chunk_reduce<NRED>(v, a.part, a.pcap, blk, lds);
    }
}

static int g_spmv_variant = -1;  // LSSP_AMD_SPMV: 4 k_spmv3 (default), 3 k_spmv + XCD order,
                                 // 0 k_spmv, 1 k_spmv2, 2 k_spmv2 + XCD order

template <int EPI>
static void spmv_dispatch(const SpmvArgs &a, int nred, long nblocks, hipStream_t s, long nnz_pad)
{
    if (g_spmv_variant < 0) {
        const char *e = getenv("LSSP_AMD_SPMV");
        g_spmv_variant = e ? atoi(e) : 4;
    }
    const long g = (nblocks + 7) / 8 * 8;
    if (g_spmv_variant == 0) {
        if (nred == 0) k_spmv<EPI, 0, 0><<<nblocks, 256, 0, s>>>(a, nblocks);
        else if (nred == 1) k_spmv<EPI, 1, 0><<<nblocks, 256, 0, s>>>(a, nblocks);
        else k_spmv<EPI, 2, 0><<<nblocks, 256, 0, s>>>(a, nblocks);
    } else if (g_spmv_variant == 1) {
        if (nred == 0) k_spmv2<EPI, 0, 0><<<nblocks, 256, 0, s>>>(a, nblocks);
        else if (nred == 1) k_spmv2<EPI, 1, 0><<<nblocks, 256, 0, s>>>(a, nblocks);
        else k_spmv2<EPI, 2, 0><<<nblocks, 256, 0, s>>>(a, nblocks);
    } else if (g_spmv_variant == 2) {
        if (nred == 0) k_spmv2<EPI, 0, 1><<<g, 256, 0, s>>>(a, nblocks);
        else if (nred == 1) k_spmv2<EPI, 1, 1><<<g, 256, 0, s>>>(a, nblocks);
        else k_spmv2<EPI, 2, 1><<<g, 256, 0, s>>>(a, nblocks);
    } else if (g_spmv_variant == 4) {
        if (nred == 0) k_spmv3<EPI, 0><<<g, 256, 0, s>>>(a, nblocks, nnz_pad);
        else if (nred == 1) k_spmv3<EPI, 1><<<g, 256, 0, s>>>(a, nblocks, nnz_pad);
        else k_spmv3<EPI, 2><<<g, 256, 0, s>>>(a, nblocks, nnz_pad);
    } else {
        if (nred == 0) k_spmv<EPI, 0, 1><<<g, 256, 0, s>>>(a, nblocks);
        else if (nred == 1) k_spmv<EPI, 1, 1><<<g, 256, 0, s>>>(a, nblocks);
        else k_spmv<EPI, 2, 1><<<g, 256, 0, s>>>(a, nblocks);
    }
}

int launch_spmv(lssp_amd_ctx *c, const lssp_amd_mat *A, int epi, double alpha, const double *x,
                double beta, const double *y, double *z, int nred, const double *w0,
                const double *w1)
{
    if (A->nrows == 0) return LSSP_AMD_OK;
    long nb = num_chunks(A->nrows);
    LSSP_TRY(ensure_part(c, nb));
    SpmvArgs a{A->nrows, A->Ap, A->Aj, A->Ax, x, y, z, alpha, beta, w0, w1, c->d_part, c->part_cap};
    switch (epi) {
    case EPI_MXY: spmv_dispatch<EPI_MXY>(a, nred, nb, c->stream, A->nnz + 4L); break;
    case EPI_AMXY: spmv_dispatch<EPI_AMXY>(a, nred, nb, c->stream, A->nnz + 4L); break;
    case EPI_AXPBY: spmv_dispatch<EPI_AXPBY>(a, nred, nb, c->stream, A->nnz + 4L); break;
    default: spmv_dispatch<EPI_AMX>(a, nred, nb, c->stream, A->nnz + 4L); break;
    }
    LSSP_HIP(hipGetLastError());
    return LSSP_AMD_OK;
}

// ---------------------------------------------------------------------------
// Elementwise passes (vector.cxx and the drivers' inline loops), one element
// per lane in the canonical chunk layout so any of them can carry partial
// sums.  Operand order inside each expression is the reference's.
// ---------------------------------------------------------------------------
enum EwKind {
    EW_FILL = 0,   // out0 = a                         (vector.cxx:31-38)
    EW_COPY,       // out0 = x                         (:73-83)
    EW_AXY,        // out0 = x * a                     (:86-95)
    EW_AXPBY,      // out0 = out0 * b + x * a          (:98-107)
    EW_AXPBYZ,     // out0 = y * b + x * a             (:110-120)
    EW_SCALE,      // out0 = out0 * a                  (:141-146)
    EW_DIVS,       // out0 = out0 / scal[sidx]         (solver-gmres.cxx:129-131)
    EW_DOT,        // partials only
    EW_BICG_P,     // out0 = x + beta*(out0 - omega*y) (solver-bicgstab.cxx:99-102), x=r, y=v
    EW_BICG_S,     // out0 = x - alpha*y               (:113-115), x=r, y=v
    EW_BICG_XR,    // out0(x) = out0 + alpha*x + omega*y ; out1(r) = u - omega*v   (:136-139)
                   // (break flag set: out0 = out0 + alpha*x only, :120-122)
    EW_CG_P,       // out0 = x + beta*out0             (solver-cg.cxx:90-92)
    EW_CG_XR,      // out0(x) = out0 + alpha*x ; out1(r) = out1 - alpha*y   (:101-104)
    EW_GM_MGS,     // out0 = out0 * 1 + x * (-scal[sidx])  (solver-gmres.cxx:144)
    EW_GM_X,       // out0[q] += sum_{i<k} vbase[i][q] * scal[S_H..]  (:196-204); ym passed in u
};

struct EwArgs {
    int kind;
    long n;
    double a, b;
    const double *x, *y, *u, *v;
    double *out0, *out1;
    const double *scal;
    const double *r0a, *r0b, *r1a, *r1b;
    const double *vbase;
    int k, sidx;
    double *part;
    long pcap;
    long nchunks;
};

template <int NRED>
__global__ __launch_bounds__(256) void k_ew(EwArgs g)
{
    __shared__ double lds[MAX_SLOTS][4];
    for (long c = blockIdx.x; c < g.nchunks; c += gridDim.x) {
        const long i = c * 256 + threadIdx.x;
        const bool in = i < g.n;
        if (in) {
            switch (g.kind) {
            case EW_FILL: g.out0[i] = g.a; break;
            case EW_COPY: g.out0[i] = g.x[i]; break;
            case EW_AXY: g.out0[i] = g.x[i] * g.a; break;
            case EW_AXPBY: g.out0[i] = g.out0[i] * g.b + g.x[i] * g.a; break;
            case EW_AXPBYZ: g.out0[i] = g.y[i] * g.b + g.x[i] * g.a; break;
            case EW_SCALE: g.out0[i] = g.out0[i] * g.a; break;
            case EW_DIVS: g.out0[i] = g.out0[i] / g.scal[g.sidx]; break;
            case EW_DOT: break;
            case EW_BICG_P: {
                const double beta = g.scal[S_BETA], omega = g.scal[S_OMEGA];
                g.out0[i] = g.x[i] + beta * (g.out0[i] - omega * g.y[i]);
                break;
            }
            case EW_BICG_S: g.out0[i] = g.x[i] - g.scal[S_ALPHA] * g.y[i]; break;
            case EW_BICG_XR: {
                const double alpha = g.scal[S_ALPHA];
                if (g.scal[S_BREAK] != 0.0) {
                    g.out0[i] = g.out0[i] + alpha * g.x[i];
                } else {
                    const double omega = g.scal[S_OMEGA];
                    g.out0[i] = g.out0[i] + alpha * g.x[i] + omega * g.y[i];
                    g.out1[i] = g.u[i] - omega * g.v[i];
                }
                break;
            }
            case EW_CG_P: g.out0[i] = g.x[i] + g.scal[S_BETA] * g.out0[i]; break;
            case EW_CG_XR: {
                const double alpha = g.scal[S_ALPHA];
                g.out0[i] = g.out0[i] + alpha * g.x[i];
                g.out1[i] = g.out1[i] - alpha * g.y[i];
                break;
            }
            case EW_GM_MGS: g.out0[i] = g.out0[i] * 1 + g.x[i] * (-g.scal[g.sidx]); break;
            case EW_GM_X: {  // b carries the basis stride (vectors hold owned + halo entries)
                const long ld = (long)g.b;
                double acc = 0;
                for (int q = 0; q < g.k; q++) acc += g.vbase[(long)q * ld + i] * g.u[q];
                g.out0[i] += acc;
                break;
            }
            }
        }
        if (NRED > 0) {
            double v[NRED > 0 ? NRED : 1];
            v[0] = in ? g.r0a[i] * g.r0b[i] : 0.0;
            if (NRED > 1) v[NRED > 1 ? 1 : 0] = in ? g.r1a[i] * g.r1b[i] : 0.0;
            chunk_reduce<NRED>(v, g.part, g.pcap, c, lds);
        }
    }
}

int launch_ew(lssp_amd_ctx *c, const Ew &e)
{
    if (e.n <= 0) return LSSP_AMD_OK;
    long C = num_chunks(e.n);
    LSSP_TRY(ensure_part(c, C));
    EwArgs g{e.kind, e.n, e.a, e.b, e.x, e.y, e.u, e.v, e.out0, e.out1, e.scal,
             e.r0a, e.r0b, e.r1a, e.r1b, e.vbase, e.k, e.sidx, c->d_part, c->part_cap, C};
    // one chunk per block up to a cap; the cap keeps >= 8 blocks per CU resident
    long grid = C < 8L * c->num_cus * 4 ? C : 8L * c->num_cus * 4;
    if (e.nred == 0) k_ew<0><<<grid, 256, 0, c->stream>>>(g);
    else if (e.nred == 1) k_ew<1><<<grid, 256, 0, c->stream>>>(g);
    else k_ew<2><<<grid, 256, 0, c->stream>>>(g);
    LSSP_HIP(hipGetLastError());
    return LSSP_AMD_OK;
}

int launch_reduce_tree(lssp_amd_ctx *c, long C, int nslot, const Fin &f)
{
    int do_fin = c->nranks > 1 ? 0 : 1;
    k_reduce2<<<1, L2_LANES, 0, c->stream>>>(c->d_part, c->part_cap, C, nslot, c->d_sums, c->d_scal,
                                              c->d_trace, f, do_fin);
    LSSP_HIP(hipGetLastError());
    return LSSP_AMD_OK;
}

int launch_reduce_serial(lssp_amd_ctx *c, long n, int nslot, const double *const *a,
                         const double *const *b, const Fin &f)
{
    SerialArgs g{};
    for (int s = 0; s < nslot; s++) {
        g.a[s] = a[s];
        g.b[s] = b[s];
    }
    int do_fin = c->nranks > 1 ? 0 : 1;
    k_dot_serial<<<1, 1, 0, c->stream>>>(g, n, nslot, c->d_sums, c->d_scal, c->d_trace, f, do_fin);
    LSSP_HIP(hipGetLastError());
    return LSSP_AMD_OK;
}

int launch_finalize(lssp_amd_ctx *c, const double *sums, int nslot, const Fin &f)
{
    (void)nslot;
    k_finalize<<<1, 1, 0, c->stream>>>(sums, c->d_scal, c->d_trace, f);
    LSSP_HIP(hipGetLastError());
    return LSSP_AMD_OK;
}

int launch_sum_ranks(lssp_amd_ctx *c, int nslot, const Fin &f)
{
    k_sum_ranks<<<1, 1, 0, c->stream>>>(c->d_gather, c->nranks, nslot, c->d_sums, c->d_scal,
                                         c->d_trace, f);
    LSSP_HIP(hipGetLastError());
    return LSSP_AMD_OK;
}

__global__ void k_fill_bits(uint64_t *x, long n, uint64_t bits)
{
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        x[i] = bits;
}

int launch_fill(lssp_amd_ctx *c, double *x, long n, uint64_t bits)
{
    if (n <= 0) return LSSP_AMD_OK;
    long grid = (n + 255) / 256;
    if (grid > 8L * c->num_cus * 4) grid = 8L * c->num_cus * 4;
    k_fill_bits<<<grid, 256, 0, c->stream>>>(reinterpret_cast<uint64_t *>(x), n, bits);
    LSSP_HIP(hipGetLastError());
    return LSSP_AMD_OK;
}

// ---------------------------------------------------------------------------
// Sync-free level-ordered triangular sweep (solver-tri.cxx:4-46).
//
// Rows are visited in level order (host analysis, ilu_setup.cpp); 64
// consecutive scheduled rows form a chunk and wave w of the persistent grid
// takes chunks w, w+W, w+2W, ... in order.  x starts as TRI_SENTINEL
// everywhere; a row's value is published by ONE 8-byte agent-scope store and
// read by agent-scope (sc1, L1-bypassing) loads -- the data is the flag
// (MI355X_MICROARCH: R2 granule).  Each lane consumes its row's entries in the
// reference's order as they become available, so the arithmetic is exactly
// result = result - val*x[col] ... ; x = result / diag.  The smallest
// unfinished chunk can always progress (its dependencies lie in earlier chunks
// or earlier in the same chunk, and its wave is resident), so the sweep
// cannot deadlock; every wait is still bounded (4 s of s_memrealtime) and a
// timeout raises ctx->d_err instead of hanging the GPU.
// ---------------------------------------------------------------------------
struct TriArgs {
    int n;
    long nchunks;
    const int *perm, *rp, *cols;
    const double *vals, *diag;
    int unit;
    const double *rhs;
    double *x;
    double *reset;  // if set: reset[row] = TRI_SENTINEL once rhs[row] has been read
    int *err;
};

__device__ __forceinline__ uint64_t ld_agent(const double *p)
{
    return __hip_atomic_load(reinterpret_cast<const uint64_t *>(p), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void st_agent(double *p, double v)
{
    __hip_atomic_store(reinterpret_cast<uint64_t *>(p), (uint64_t)__double_as_longlong(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Sync-free sweep.  First pass over a row's entries loads them in batches of
// four; once a dependency is found missing, the lane re-polls only that one
// entry (one load per lane per poll) with an exponential back-off, so waves
// far ahead of the wavefront do not flood the memory system with polls.
template <int BACKOFF>
__global__ __launch_bounds__(256) void k_trisolve(TriArgs a)
{
    const int lane = threadIdx.x & 63;
    const long wave = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const long nwaves = (long)gridDim.x * (blockDim.x >> 6);
    for (long c = wave; c < a.nchunks; c += nwaves) {
        const long p = c * 64 + lane;
        bool active = p < a.n;
        int row = 0, k = 0, end = 0;
        double acc = 0;
        if (active) {
            row = a.perm[p];
            k = a.rp[p];
            end = a.rp[p + 1];
            acc = a.rhs[row];
            if (a.reset) a.reset[row] = __longlong_as_double((long long)TRI_SENTINEL);
        }
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        int nap = 1;
        int mcap = 4;
        for (;;) {
            if (active) {
                while (k < end) {
                    const int m = end - k < mcap ? end - k : mcap;
                    uint64_t bits[4];
#pragma unroll
                    for (int u = 0; u < 4; u++)
                        if (u < m) bits[u] = ld_agent(a.x + a.cols[k + u]);
                    int u = 0;
                    for (; u < m; u++) {
                        if (bits[u] == TRI_SENTINEL) break;
                        acc = acc - a.vals[k] * __longlong_as_double((long long)bits[u]);
                        k++;
                    }
                    if (u < m) {
                        mcap = 1;  // re-poll just the first missing dependency
                        break;
                    }
                    mcap = 4;
                }
                if (k == end) {
                    const double xi = a.unit ? acc : acc / a.diag[p];
                    st_agent(a.x + row, xi);
                    active = false;
                }
            }
            if (!__any(active)) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) {  // 4 s at 100 MHz
                if (active) {
                    atomicOr(a.err, 1);
                    st_agent(a.x + row, __longlong_as_double(0x7FF8000000000000ll));
                }
                break;
            }
            for (int q = 0; q < nap; q++) __builtin_amdgcn_s_sleep(2);
            if (BACKOFF && nap < 32) nap <<= 1;
        }
    }
}

// Level-synchronous alternative: one launch per level, every dependency lies in
// an earlier launch, so plain loads suffice and nothing waits.
__global__ __launch_bounds__(256) void k_trisolve_level(TriArgs a, int lo, int hi)
{
    const int p = lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= hi) return;
    const int row = a.perm[p];
    double acc = a.rhs[row];
    if (a.reset) a.reset[row] = __longlong_as_double((long long)TRI_SENTINEL);
    for (int k = a.rp[p]; k < a.rp[p + 1]; k++) acc = acc - a.vals[k] * a.x[a.cols[k]];
    a.x[row] = a.unit ? acc : acc / a.diag[p];
}

// Block-pipelined sweep (tri_mode 3, schedule from tri_bp.cpp).  Workgroups
// claim blocks in sweep order from a ticket counter (so a block only ever
// waits on a block claimed earlier by a running workgroup: no residency
// assumption, no deadlock), walk the block's steps (levels) in order, read
// same-block values of the last BP_RING positions from LDS and everything else
// with agent-scope loads, and publish "all my rows up to level L are done" in a
// 64-bit progress word {epoch, L+1} after draining their stores (every wave
// s_waitcnt vmcnt(0), barrier, one sc1 store: MI355X_MICROARCH hand-off row 1).
struct BPArgs {
    int B, nb;
    const int *blk_step, *step_pos, *step_need, *step_done, *step_flag;
    const int *perm, *rp, *cols;
    const double *vals, *diag;
    int unit;
    const double *rhs;
    double *x;
    double *reset;
    unsigned long long *prog, *claim;
    unsigned long long base;
    unsigned epoch;
    int *err;
};

__global__ __launch_bounds__(256) void k_tri_bp(BPArgs a)
{
    __shared__ double ring[BP_RING];
    __shared__ int s_blk;
    const int tid = threadIdx.x;
    const unsigned long long tag = (unsigned long long)a.epoch << 32;
    for (;;) {
        __syncthreads();  // ring and s_blk are free again
        if (tid == 0) s_blk = (int)(atomicAdd(a.claim, 1ull) - a.base);
        __syncthreads();
        const int b = s_blk;
        if (b >= a.nb) break;
        const long base = (long)b * a.B;
        unsigned long long seen = 0;
        bool dead = false;
        for (int s = a.blk_step[b]; s < a.blk_step[b + 1]; s++) {
            const int need = a.step_need[s];
            if (need >= 0 && tid == 0 && !dead) {
                const unsigned long long want = tag | (unsigned)(need + 1);
                const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                while (seen < want) {
                    seen = __hip_atomic_load(a.prog + (b - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (seen >= want) break;
                    if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) {  // 4 s
                        atomicOr(a.err, 2);
                        dead = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            __syncthreads();
            const int p0 = a.step_pos[s], p1 = a.step_pos[s + 1];
            for (int p = p0 + tid; p < p1; p += 256) {
                const int row = a.perm[p];
                double acc = a.rhs[row];
                if (a.reset) a.reset[row] = __longlong_as_double((long long)TRI_SENTINEL);
                for (int k = a.rp[p]; k < a.rp[p + 1]; k++) {
                    const int code = a.cols[k];
                    const double xv = code < 0 ? ring[-1 - code] : __longlong_as_double((long long)ld_agent(a.x + code));
                    acc = acc - a.vals[k] * xv;
                }
                const double xi = a.unit ? acc : acc / a.diag[p];
                ring[(p - base) % BP_RING] = xi;
                st_agent(a.x + row, xi);
            }
            if (a.step_flag[s] & 1) {  // drain this block's stores, then publish
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (tid == 0)
                    __hip_atomic_store(a.prog + b, tag | (unsigned)(a.step_done[s] + 1), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

// Packet-streamed block pipeline (tri_mode 4, packets from tri_bp.cpp).
// Blocks are claimed in sweep order as in k_tri_bp.  Inside a block the
// workgroup streams its packets (one level's rows each) through a 3-slot LDS
// ring: while it computes packet q it loads packet q+2 with 16-byte loads and
// gathers the right-hand side of packet q+1, so only the x dependencies are
// on the critical path.  Same-block values of the last BP_RING positions come
// from the LDS value ring; all other x values are read with agent-scope loads
// and, because x is armed with TRI_SENTINEL before the sweep, a value that is
// not yet visible is simply re-read (value-as-flag): no store drains, no
// progress words.  A block only ever waits on the block before it, which was
// claimed earlier by a running workgroup, so the sweep always drains.
struct PkArgs {
    int nb;
    const int *blk, *off;
    const int4 *data;
    int unit;
    const double *rhs;
    double *x;
    double *reset;
    unsigned long long *claim;
    unsigned long long base;
    int *err;
    int diag;  // diagnostics only (LSSP_AMD_TRI_DIAG): 1 = no waiting, 2 = no cross-block loads
};

// Workgroup barrier for LDS hand-offs only.  __syncthreads() is a
// workgroup-scope fence + s_barrier, which on gfx950 also waits vmcnt(0): every
// in-flight global load AND every x store would be waited for at each step.
// Here only LDS traffic must be complete; global loads are waited for where
// their registers are used, the sc1 x stores are never waited for.
__device__ __forceinline__ void lds_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ double ld_ready(const double *p, int *err)
{
    uint64_t bits = ld_agent(p);
    if (bits == TRI_SENTINEL) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        do {
            __builtin_amdgcn_s_sleep(1);
            bits = ld_agent(p);
            if (bits != TRI_SENTINEL) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) {  // 4 s
                atomicOr(err, 4);
                return __longlong_as_double(0x7FF8000000000000ll);
            }
        } while (true);
    }
    return __longlong_as_double((long long)bits);
}

constexpr int PK_VEC = PK_BYTES / 16;         // int4 per packet slot
constexpr int PK_LD = (PK_VEC + 255) / 256;   // int4 loads per thread to stage one packet

__global__ __launch_bounds__(256) void k_tri_pk(PkArgs a)
{
    __shared__ double ring[BP_RING];
    __shared__ int4 pbuf[3][PK_VEC];
    __shared__ double rbuf[3][PK_ROWS];
    __shared__ int s_blk;
    const int tid = threadIdx.x;
    for (;;) {
        __syncthreads();
        if (tid == 0) s_blk = (int)(atomicAdd(a.claim, 1ull) - a.base);
        __syncthreads();
        const int b = s_blk;
        if (b >= a.nb) break;
        const int q0 = a.blk[b], q1 = a.blk[b + 1];
        // prologue: packets q0, q0+1 into slots 0, 1; rhs of q0 into rbuf[0]
        for (int j = 0; j < 2 && q0 + j < q1; j++) {
            const int o = a.off[q0 + j], len = a.off[q0 + j + 1] - o;
            for (int i = tid; i < len; i += 256) pbuf[j][i] = a.data[o + i];
        }
        __syncthreads();
        {
            const int *w = reinterpret_cast<const int *>(pbuf[0]);
            if (tid < w[0]) rbuf[0][tid] = a.rhs[w[4 + tid]];
        }
        __syncthreads();
        for (int q = q0; q < q1; q++) {
            const int cur = (q - q0) % 3, nxt = (cur + 1) % 3, nn = (cur + 2) % 3;
            // (1) stage packet q+2
            int4 st[PK_LD];
            int o2 = 0, len2 = 0;
            if (q + 2 < q1) {
                o2 = a.off[q + 2];
                len2 = a.off[q + 3] - o2;
#pragma unroll
                for (int u = 0; u < PK_LD; u++) {
                    const int i = tid + 256 * u;
                    if (i < len2) st[u] = a.data[o2 + i];
                }
            }
            // (2) gather the right-hand side of packet q+1
            double rh = 0;
            bool have_rh = false;
            if (q + 1 < q1) {
                const int *w = reinterpret_cast<const int *>(pbuf[nxt]);
                if (tid < w[0]) {
                    rh = a.rhs[w[4 + tid]];
                    have_rh = true;
                }
            }
            // (3) packet q
            {
                const int *w = reinterpret_cast<const int *>(pbuf[cur]);
                const int nr = w[0], ne = w[1], pos0 = w[2];
                if (tid < nr) {
                    const int *rows = w + 4, *rp = w + 4 + nr, *codes = w + 5 + 2 * nr;
                    const int vo = (5 + 2 * nr + ne + 1) & ~1;
                    const double *vals = reinterpret_cast<const double *>(w + vo);
                    const int row = rows[tid];
                    double acc = rbuf[cur][tid];
                    if (a.reset) a.reset[row] = __longlong_as_double((long long)TRI_SENTINEL);
                    for (int k = rp[tid]; k < rp[tid + 1]; k++) {
                        const int code = codes[k];
                        double xv;
                        if (code < 0) xv = ring[-1 - code];
                        else if (a.diag == 0) xv = ld_ready(a.x + code, a.err);
                        else if (a.diag == 1) xv = __longlong_as_double((long long)ld_agent(a.x + code));
                        else xv = 0.0;
                        acc = acc - vals[k] * xv;
                    }
                    const double xi = a.unit ? acc : acc / reinterpret_cast<const double *>(w + vo + 2 * ne)[tid];
                    ring[(pos0 + tid) % BP_RING] = xi;
                    st_agent(a.x + row, xi);
                }
            }
            // (4) land the staged data
            if (q + 2 < q1) {
#pragma unroll
                for (int u = 0; u < PK_LD; u++) {
                    const int i = tid + 256 * u;
                    if (i < len2) pbuf[nn][i] = st[u];
                }
            }
            if (have_rh) rbuf[nxt][tid] = rh;
            lds_barrier();
        }
    }
}

// tri_mode 5: k_tri_pk with a deeper software pipeline.  Iteration i computes
// packet i of the block; at that time packets i..i+2 sit in LDS, the loads of
// packet i+3 (issued one iteration earlier) land in LDS at the end of the
// iteration and the loads of packet i+4 are issued; the right-hand side and the
// first PF_E cross-block / far values of packet i+2 are gathered into
// registers and land in LDS one iteration later, two iterations before they
// are used.  Every global load therefore has one to two iterations to arrive
// instead of being waited for inside the iteration that issued it.
constexpr int PF_E = 2;

struct PkRegs {
    int4 pk[PK_LD];
    int len;
    double rh;
    double ev[PF_E];
    int ek[PF_E];
};

__device__ __forceinline__ void pk_issue(const PkArgs &a, int p, int q1, PkRegs &R)
{
    R.len = 0;
    if (p < q1) {
        const int o = a.off[p];
        R.len = a.off[p + 1] - o;
#pragma unroll
        for (int u = 0; u < PK_LD; u++) {
            const int i = threadIdx.x + 256 * u;
            if (i < R.len) R.pk[u] = a.data[o + i];
        }
    }
}

__device__ __forceinline__ void pk_land(int4 *slot, const PkRegs &R)
{
#pragma unroll
    for (int u = 0; u < PK_LD; u++) {
        const int i = threadIdx.x + 256 * u;
        if (i < R.len) slot[i] = R.pk[u];
    }
}

// gather rhs and the first PF_E HBM-resident x values of this thread's row of
// the packet in `slot` (already in LDS)
__device__ __forceinline__ void pk_gather(const PkArgs &a, const int4 *slot, bool valid, PkRegs &R)
{
    R.ek[0] = R.ek[1] = -1;
    if (!valid) return;
    const int *w = reinterpret_cast<const int *>(slot);
    const int nr = w[0];
    const int tid = threadIdx.x;
    if (tid >= nr) return;
    R.rh = a.rhs[w[4 + tid]];
    const int *rp = w + 4 + nr, *codes = w + 5 + 2 * nr;
    int m = 0;
    for (int k = rp[tid]; k < rp[tid + 1] && m < PF_E; k++) {
        const int code = codes[k];
        if (code >= 0) {
            R.ek[m] = k;
            R.ev[m] = __longlong_as_double((long long)ld_agent(a.x + code));
            m++;
        }
    }
}

__global__ __launch_bounds__(256) void k_tri_pk2(PkArgs a)
{
    __shared__ double ring[BP_RING];
    __shared__ int4 pbuf[4][PK_VEC];
    __shared__ double rbuf[4][PK_ROWS];
    __shared__ double ebuf[4][PF_E][PK_ROWS];
    __shared__ int kbuf[4][PF_E][PK_ROWS];
    __shared__ int s_blk;
    const int tid = threadIdx.x;
    for (;;) {
        __syncthreads();
        if (tid == 0) s_blk = (int)(atomicAdd(a.claim, 1ull) - a.base);
        __syncthreads();
        const int b = s_blk;
        if (b >= a.nb) break;
        const int q0 = a.blk[b], q1 = a.blk[b + 1];
        PkRegs RA, RB;
        // prologue: packets 0..2 into slots 0..2
        for (int j = 0; j < 3 && q0 + j < q1; j++) {
            pk_issue(a, q0 + j, q1, RA);
            pk_land(pbuf[j], RA);
        }
        __syncthreads();
        pk_gather(a, pbuf[0], q0 < q1, RA);  // packet 0: straight to LDS
        if (q0 < q1 && tid < PK_ROWS) {
            rbuf[0][tid] = RA.rh;
            for (int e = 0; e < PF_E; e++) {
                ebuf[0][e][tid] = RA.ev[e];
                kbuf[0][e][tid] = RA.ek[e];
            }
        }
        pk_gather(a, pbuf[1], q0 + 1 < q1, RB);  // packet 1: lands at iteration 0
        pk_issue(a, q0 + 3, q1, RA);             // packet 3: lands at iteration 0
        __syncthreads();

        auto iteration = [&](int i, PkRegs &cur, PkRegs &nxt) {
            // cur: loads of packet i+3 + gathers of packet i+1 (issued last iteration)
            // nxt: receives loads of packet i+4 and gathers of packet i+2
            const int p = q0 + i;
            PkRegs G;  // gathers of packet i+2 (registers)
            pk_gather(a, pbuf[(i + 2) & 3], p + 2 < q1, G);
            {
                const int *w = reinterpret_cast<const int *>(pbuf[i & 3]);
                const int nr = w[0], ne = w[1], pos0 = w[2];
                if (tid < nr) {
                    const int *rows = w + 4, *rp = w + 4 + nr, *codes = w + 5 + 2 * nr;
                    const int vo = (5 + 2 * nr + ne + 1) & ~1;
                    const double *vals = reinterpret_cast<const double *>(w + vo);
                    const int row = rows[tid];
                    double acc = rbuf[i & 3][tid];
                    if (a.reset) a.reset[row] = __longlong_as_double((long long)TRI_SENTINEL);
                    const int k0 = kbuf[i & 3][0][tid], k1 = kbuf[i & 3][1][tid];
                    for (int k = rp[tid]; k < rp[tid + 1]; k++) {
                        const int code = codes[k];
                        double xv;
                        if (code < 0) {
                            xv = ring[-1 - code];
                        } else {
                            double pv = 0;
                            bool have = false;
                            if (k == k0) { pv = ebuf[i & 3][0][tid]; have = true; }
                            else if (k == k1) { pv = ebuf[i & 3][1][tid]; have = true; }
                            if (have && __double_as_longlong(pv) != (long long)TRI_SENTINEL) xv = pv;
                            else xv = ld_ready(a.x + code, a.err);
                        }
                        acc = acc - vals[k] * xv;
                    }
                    const double xi = a.unit ? acc : acc / reinterpret_cast<const double *>(w + vo + 2 * ne)[tid];
                    ring[(pos0 + tid) % BP_RING] = xi;
                    st_agent(a.x + row, xi);
                }
            }
            // land packet i+3 and the gathers of packet i+1; issue packet i+4
            pk_land(pbuf[(i + 3) & 3], cur);
            if (p + 1 < q1 && tid < PK_ROWS) {
                rbuf[(i + 1) & 3][tid] = cur.rh;
                ebuf[(i + 1) & 3][0][tid] = cur.ev[0];
                ebuf[(i + 1) & 3][1][tid] = cur.ev[1];
                kbuf[(i + 1) & 3][0][tid] = cur.ek[0];
                kbuf[(i + 1) & 3][1][tid] = cur.ek[1];
            }
            pk_issue(a, p + 4, q1, nxt);
            nxt.rh = G.rh;
            for (int e = 0; e < PF_E; e++) {
                nxt.ev[e] = G.ev[e];
                nxt.ek[e] = G.ek[e];
            }
            lds_barrier();
        };
        // RB holds gathers of packet 1; RA holds loads of packet 3 -- merge into one "cur"
        RA.rh = RB.rh;
        for (int e = 0; e < PF_E; e++) {
            RA.ev[e] = RB.ev[e];
            RA.ek[e] = RB.ek[e];
        }
        const int np = q1 - q0;
        int i = 0;
        for (; i + 1 < np; i += 2) {
            iteration(i, RA, RB);
            iteration(i + 1, RB, RA);
        }
        if (i < np) iteration(i, RA, RB);
    }
}

// tri_mode 6: decoupled loader waves.  On gfx9 one wave's vmcnt covers its
// loads AND its stores, so in a single-role wave every wait for a prefetched
// operand also waited for the write-through x stores of the step before --
// about one HBM round trip per step, whatever the prefetch depth.  Here the
// workgroup is split by role:
//   waves 0-3 (compute): row t of the current packet; operands only from LDS
//     (packet, gathered rhs and HBM x values, value ring), x stored to HBM and
//     never waited for.  Their per-step time is LDS latency + arithmetic.
//   waves 4-7 (loader): every step issue exactly C = PK3_LD + 1 + PK3_EXT loads
//     per lane (unused ones are clamped to a valid address so the count is
//     static): packet j+A into registers, and for packet j+B (already in LDS)
//     its rhs entries and its list of HBM x operands.  Then wait vmcnt(S*C),
//     i.e. only for the group issued S steps earlier, and land it in LDS.
// An HBM operand the producer block has not written yet reads as TRI_SENTINEL
// and is re-polled by its loader lane before landing (value-as-flag again);
// the block-to-block lag settles at about one store + load round trip, which
// is paid once per block instead of once per step.
typedef int v4i __attribute__((ext_vector_type(4)));

struct Pk3Args {
    int nb;
    const int *blk, *off;
    const v4i *data;
    int unit;
    const double *rhs;
    double *x;
    double *reset;
    unsigned long long *claim;
    unsigned long long base;
    int *err;
    int diag;  // timing experiments only (LSSP_AMD_TRI_DIAG bits): 1 no reset stores, 2 no x stores,
               // 4 rhs gathers coalesced, 8 no HBM x gathers (wrong results when != 0)
    unsigned long long *trace;  // diagnostics (LSSP_AMD_TRI_TRACE): per block t_claim, t_end, polls, XCC,
                                // compute/barrier cycles of wave 0, wait/barrier cycles of wave 4
};
constexpr int PK3_VEC = PK3_BYTES / 16;
constexpr int PK3_LD = PK3_VEC / PK3_ROWS;
static_assert(PK3_VEC % PK3_ROWS == 0, "packet slot must split evenly over the loader lanes");

struct Pk3Regs {
    v4i pk[PK3_LD];
    double rh;
    uint64_t ev[PK3_EXT];
};

__device__ __forceinline__ uint64_t poll_ready(const double *p, int *err)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        const uint64_t bits = ld_agent(p);
        if (bits != TRI_SENTINEL) return bits;
        if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) {  // 4 s
            atomicOr(err, 4);
            return 0x7FF8000000000000ull;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

template <int S>
__global__ __launch_bounds__(2 * PK3_ROWS) void k_tri_pk3(Pk3Args a)
{
    constexpr int NS = S + 3;        // packet slots live at once
    constexpr int A = 2 * S + 2;     // packet loads are issued A steps ahead
    constexpr int B = S + 1;         // gathers are issued B steps ahead
    constexpr int C = PK3_LD + 1 + PK3_EXT;
    static_assert(S * C <= 63, "vmcnt is 6 bits");
    __shared__ double ring[BP_RING];
    __shared__ v4i pbuf[NS][PK3_VEC];
    __shared__ double rbuf[2][PK3_ROWS];
    __shared__ double xbuf[2][PK3_ROWS * PK3_EXT];
    __shared__ int offs[PK3_CAP + 1];
    __shared__ int s_blk;
    __shared__ unsigned s_polls;
    const int tid = threadIdx.x;
    // wave-uniform role (readfirstlane): the two roles become separate
    // branches instead of one exec-masked sequence
    const bool loader = __builtin_amdgcn_readfirstlane(tid) >= PK3_ROWS;
    const int t = tid & (PK3_ROWS - 1);
    int prev = -1;
    for (;;) {
        __syncthreads();
        if (tid == 0) {
            if (a.trace && prev >= 0) {
                a.trace[8 * prev + 1] = __builtin_amdgcn_s_memrealtime();
                a.trace[8 * prev + 2] = s_polls;
            }
            s_polls = 0;
            s_blk = (int)(atomicAdd(a.claim, 1ull) - a.base);
        }
        __syncthreads();
        const int b = s_blk;
        if (b >= a.nb) break;
        if (a.trace && tid == 0) {
            unsigned xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            a.trace[8 * b] = __builtin_amdgcn_s_memrealtime();
            a.trace[8 * b + 3] = xcc;
        }
        prev = b;
        const int q0 = a.blk[b], np = a.blk[b + 1] - q0;
        for (int i = tid; i <= np; i += 2 * PK3_ROWS) offs[i] = a.off[q0 + i];
        __syncthreads();

        // the two roles run separate loops with the same number of steps and
        // one s_barrier per step; keeping the roles apart also keeps the
        // compiler's vmcnt bookkeeping of the loader registers exact (a join
        // with the compute path would mark them pending again)
        constexpr int P = S + 1;
        const int nsteps = (np + A + P - 1) / P * P;
        if (!loader) {
            uint64_t c0 = 0, c1 = 0, acc_c = 0, acc_b = 0;
            for (int j = -A; j < nsteps - A; j++) {
                if (a.trace) c0 = __builtin_amdgcn_s_memtime();
                if (j >= 0 && j < np) {
                    const int *w = reinterpret_cast<const int *>(pbuf[j % NS]);
                    const int nr = w[0], ne = w[1], pos0 = w[2], nx = w[3];
                    if (t < nr) {
                        const int *rp = w + 4 + nr, *codes = w + 5 + 2 * nr;
                        const int vo = (5 + 2 * nr + ne + nx + 1) & ~1;
                        const double *vals = reinterpret_cast<const double *>(w + vo);
                        const double *xb = xbuf[j & 1];
                        const int row = w[4 + t];
                        double acc = rbuf[j & 1][t];
                        for (int k = rp[t]; k < rp[t + 1]; k++) {
                            const int code = codes[k];
                            const double xv = code < 0 ? ring[-1 - code] : xb[code];
                            acc = acc - vals[k] * xv;
                        }
                        const double xi = a.unit ? acc : acc / reinterpret_cast<const double *>(w + vo + 2 * ne)[t];
                        ring[(pos0 + t) % BP_RING] = xi;
                        if (!(a.diag & 2)) st_agent(a.x + row, xi);
                        if (a.reset && !(a.diag & 1)) a.reset[row] = __longlong_as_double((long long)TRI_SENTINEL);
                    }
                }
                if (a.trace) c1 = __builtin_amdgcn_s_memtime();
                lds_barrier();
                if (a.trace) {
                    const uint64_t c2 = __builtin_amdgcn_s_memtime();
                    acc_c += c1 - c0;
                    acc_b += c2 - c1;
                }
            }
            if (a.trace && tid == 0) {
                a.trace[8 * b + 4] = acc_c;
                a.trace[8 * b + 5] = acc_b;
            }
        } else {
            uint64_t acc_w = 0, acc_lb = 0;
            auto step = [&](int j, Pk3Regs &Ri, Pk3Regs &Rl) {
                {  // issue group j
                    const int pl = j + A;
                    const v4i *src = a.data + (pl < np ? offs[pl] : 0);
#pragma unroll
                    for (int u = 0; u < PK3_LD; u++) Ri.pk[u] = src[t + PK3_ROWS * u];
                    const int pg = j + B;
                    int row = 0, nxg = 0;
                    const int *xl = reinterpret_cast<const int *>(pbuf[0]);
                    if (pg >= 0 && pg < np) {
                        const int *w = reinterpret_cast<const int *>(pbuf[pg % NS]);
                        const int nrg = w[0];
                        nxg = w[3];
                        if (t < nrg) row = w[4 + t];
                        xl = w + 5 + 2 * nrg + w[1];
                    }
                    Ri.rh = a.rhs[(a.diag & 4) ? t : row];
#pragma unroll
                    for (int e = 0; e < PK3_EXT; e++) {
                        const int idx = t + PK3_ROWS * e;
                        Ri.ev[e] = ld_agent(a.x + (idx < nxg && !(a.diag & 8) ? xl[idx] : 0));
                    }
                }
                uint64_t l0 = 0;
                if (a.trace) l0 = __builtin_amdgcn_s_memtime();
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(S * C) : "memory");
                // touch every landed register once, unconditionally: the
                // compiler then puts its own (equal) wait here rather than
                // inside the divergent branches below, where a skipped branch
                // would leave the load "pending" and cost a vmcnt(0) later
                asm volatile("" ::"v"(Rl.pk[0]), "v"(Rl.pk[1]), "v"(Rl.pk[2]), "v"(Rl.rh), "v"(Rl.ev[0]),
                             "v"(Rl.ev[1]));
                if (a.trace) acc_w += __builtin_amdgcn_s_memtime() - l0;
                if (j - S >= -A) {  // land group j - S
                    const int pl = j + S + 2;
                    if (pl < np) {
#pragma unroll
                        for (int u = 0; u < PK3_LD; u++) pbuf[pl % NS][t + PK3_ROWS * u] = Rl.pk[u];
                    }
                    const int pg = j + 1;
                    if (pg >= 0 && pg < np) {
                        const int *w = reinterpret_cast<const int *>(pbuf[pg % NS]);
                        const int nr = w[0], nx = w[3];
                        const int *xl = w + 5 + 2 * nr + w[1];
                        if (t < nr) rbuf[pg & 1][t] = Rl.rh;
#pragma unroll
                        for (int e = 0; e < PK3_EXT; e++) {
                            const int idx = t + PK3_ROWS * e;
                            if (idx < nx) {
                                uint64_t bits = Rl.ev[e];
                                if (bits == TRI_SENTINEL && !(a.diag & 8)) {
                                    bits = poll_ready(a.x + xl[idx], a.err);
                                    if (a.trace) atomicAdd(&s_polls, 1u);
                                }
                                xbuf[pg & 1][idx] = __longlong_as_double((long long)bits);
                            }
                        }
                    }
                }
                uint64_t l1 = 0;
                if (a.trace) l1 = __builtin_amdgcn_s_memtime();
                lds_barrier();
                if (a.trace) acc_lb += __builtin_amdgcn_s_memtime() - l1;
            };
            // register sets rotate with period S+1; spelled out so they stay
            // in VGPRs (an indexed array would be promoted to LDS or scratch).
            // Steps past the end only issue clamped loads, so every step has
            // exactly C loads per lane.
            Pk3Regs R0, R1, R2, R3;
            for (int j0 = -A; j0 < nsteps - A; j0 += P) {
                if constexpr (S == 2) {
                    step(j0, R0, R1);
                    step(j0 + 1, R1, R2);
                    step(j0 + 2, R2, R0);
                } else {
                    step(j0, R0, R1);
                    step(j0 + 1, R1, R2);
                    step(j0 + 2, R2, R3);
                    step(j0 + 3, R3, R0);
                }
            }
            (void)R3;
            if (a.trace && tid == PK3_ROWS) {
                a.trace[8 * b + 6] = acc_w;
                a.trace[8 * b + 7] = acc_lb;
            }
        }
    }
}

// tri_mode 7: k_tri_pk3's role split plus
//   * a packet layout with each row's entries column-major and padded to the
//     packet's longest row (tri_bp.cpp build_packets4), so a compute lane
//     fetches packet j+1's row description (row, first PK4_EP codes and values,
//     diagonal) into registers while it computes packet j: a step's critical
//     path is one LDS round trip for the operand values, the multiply-adds, the
//     division and the ring write;
//   * the HBM x operands of packet j are gathered only KE steps ahead (the
//     packet words and rhs entries, which depend on nothing, still A and B
//     steps ahead): the producer block is read with KE steps of lead, so the
//     block-to-block lag is about one store + load round trip, not the packet
//     prefetch depth;
//   * the armed ("reset") vector is filled with TRI_SENTINEL over the block's
//     own contiguous row range once the block is done (coalesced stores,
//     after every rhs entry of the block has been read) instead of one
//     scattered store per row per step.
// Loader group of step j, in issue order: x operands of packet j+KE (PK3_EXT),
// packet j+A (PK3_LD), rhs of packet j+B (1).  At the end of step j it lands
// the x operands and rhs of packet j+1 and the words of packet j+A-KE.
struct Pk4Args {
    int nb;
    const int *blk, *off;
    const v4i *data;
    int unit;
    const double *rhs;
    double *x;
    double *reset;
    int n, B, upper;  // block b owns sweep positions [b*B, (b+1)*B)
    unsigned long long *claim;
    unsigned long long base;
    int *err;
    int diag;  // timing experiments only (LSSP_AMD_TRI_DIAG bits, see Pk3Args)
    unsigned long long *trace;
};
constexpr int PK4_EP = 4;  // entries per row held in registers
constexpr int TRW = 12;    // trace words per block (diagnostics)

struct Pk4Regs {
    uint64_t ev[PK3_EXT];
    v4i pk[PK3_LD];
    double rh;
};

template <int KE>
__global__ __launch_bounds__(2 * PK3_ROWS) void k_tri_pk4(Pk4Args a)
{
    constexpr int A = 2 * KE + 3;       // packet words issued A steps ahead
    constexpr int B = KE + 1;           // rhs entries issued B steps ahead
    constexpr int NS = A - KE + 1;      // packet slots live at once
    constexpr int P = KE + 1;           // register-group rotation period
    constexpr int C = PK3_EXT + PK3_LD + 1;
    constexpr int WAITN = (PK3_LD + 1) + (KE - 1) * C;
    static_assert(WAITN + C <= 63, "vmcnt is 6 bits");
    __shared__ double ring[BP_RING + 1];  // [BP_RING] holds +0.0 for PK4_PAD
    __shared__ v4i pbuf[NS][PK3_VEC];
    __shared__ double rbuf[2][PK3_ROWS];
    __shared__ double xbuf[2][PK3_ROWS * PK3_EXT];
    __shared__ int offs[PK3_CAP + 1];
    __shared__ int s_blk;
    __shared__ unsigned s_polls;
    const int tid = threadIdx.x;
    const bool loader = __builtin_amdgcn_readfirstlane(tid) >= PK3_ROWS;
    const int t = tid & (PK3_ROWS - 1);
    if (tid == 0) ring[BP_RING] = 0.0;
    int prev = -1;
    for (;;) {
        __syncthreads();
        if (tid == 0) {
            if (a.trace && prev >= 0) {
                a.trace[TRW * prev + 1] = __builtin_amdgcn_s_memrealtime();
                a.trace[TRW * prev + 2] = s_polls;
            }
            s_polls = 0;
            s_blk = (int)(atomicAdd(a.claim, 1ull) - a.base);
        }
        __syncthreads();
        const int b = s_blk;
        if (b >= a.nb) break;
        if (a.trace && tid == 0) {
            unsigned xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            a.trace[TRW * b] = __builtin_amdgcn_s_memrealtime();
            a.trace[TRW * b + 3] = xcc;
        }
        prev = b;
        const int q0 = a.blk[b], np = a.blk[b + 1] - q0;
        for (int i = tid; i <= np; i += 2 * PK3_ROWS) offs[i] = a.off[q0 + i];
        __syncthreads();
        const int nsteps = (np + A + P - 1) / P * P;
        auto words = [&](int p) { return reinterpret_cast<const int *>(pbuf[p % NS]); };

        if (!loader) {
            // header of packet j+1 (scalars) and row description of packet j (registers)
            int nr1 = 0, em1 = 0, pos1 = 0, nx1 = 0;
            int nr0 = 0, em0 = 0, pos0 = 0, nx0 = 0;
            int row = 0, cd[PK4_EP];
            double vl[PK4_EP], dg = 1.0;
#pragma unroll
            for (int e = 0; e < PK4_EP; e++) {
                cd[e] = PK4_PAD;
                vl[e] = 0.0;
            }
            uint64_t c0 = 0, c1 = 0, acc_c = 0, acc_b = 0;
            for (int j = -A; j < nsteps - A; j++) {
                if (a.trace) c0 = __builtin_amdgcn_s_memtime();
                const bool act = j >= 0 && j < np && t < nr0;
                // (1) operand reads of packet j
                double rb = 0.0, xv[PK4_EP];
                if (act) {
                    rb = rbuf[j & 1][t];
                    const double *xb = xbuf[j & 1];
#pragma unroll
                    for (int e = 0; e < PK4_EP; e++)
                        if (e < em0) xv[e] = cd[e] < 0 ? ring[-1 - cd[e]] : xb[cd[e]];
                }
                // (2) prefetch: header of packet j+2, row description of packet j+1
                int nr2 = 0, em2 = 0, pos2 = 0, nx2 = 0;
                if (j + 2 >= 0 && j + 2 < np) {
                    const int *w = words(j + 2);
                    nr2 = __builtin_amdgcn_readfirstlane(w[0]);
                    em2 = __builtin_amdgcn_readfirstlane(w[1]);
                    pos2 = __builtin_amdgcn_readfirstlane(w[2]);
                    nx2 = __builtin_amdgcn_readfirstlane(w[3]);
                }
                int row1 = 0, cd1[PK4_EP];
                double vl1[PK4_EP], dg1 = 1.0;
#pragma unroll
                for (int e = 0; e < PK4_EP; e++) {
                    cd1[e] = PK4_PAD;
                    vl1[e] = 0.0;
                }
                if (j + 1 >= 0 && j + 1 < np && t < nr1) {
                    const int *w = words(j + 1);
                    const int xo = 4 + nr1 + em1 * nr1;
                    const double *v = reinterpret_cast<const double *>(w + ((xo + nx1 + 1) & ~1));
                    row1 = w[4 + t];
#pragma unroll
                    for (int e = 0; e < PK4_EP; e++)
                        if (e < em1) {
                            cd1[e] = w[4 + nr1 + e * nr1 + t];
                            vl1[e] = v[e * nr1 + t];
                        }
                    if (!a.unit) dg1 = v[em1 * nr1 + t];
                }
                // (3) packet j, in the reference's summation order
                if (act) {
                    double acc = rb;
#pragma unroll
                    for (int e = 0; e < PK4_EP; e++)
                        if (e < em0) acc = acc - vl[e] * xv[e];
                    if (em0 > PK4_EP) {
                        const int *w = words(j);
                        const int xo = 4 + nr0 + em0 * nr0;
                        const double *v = reinterpret_cast<const double *>(w + ((xo + nx0 + 1) & ~1));
                        const double *xb = xbuf[j & 1];
                        for (int e = PK4_EP; e < em0; e++) {
                            const int code = w[4 + nr0 + e * nr0 + t];
                            const double xe = code < 0 ? ring[-1 - code] : xb[code];
                            acc = acc - v[e * nr0 + t] * xe;
                        }
                    }
                    const double xi = a.unit ? acc : acc / dg;
                    ring[(pos0 + t) % BP_RING] = xi;
                    if (!(a.diag & 2)) st_agent(a.x + row, xi);
                }
                nr0 = nr1; em0 = em1; pos0 = pos1; nx0 = nx1;
                nr1 = nr2; em1 = em2; pos1 = pos2; nx1 = nx2;
                row = row1;
                dg = dg1;
#pragma unroll
                for (int e = 0; e < PK4_EP; e++) {
                    cd[e] = cd1[e];
                    vl[e] = vl1[e];
                }
                if (a.trace) c1 = __builtin_amdgcn_s_memtime();
                lds_barrier();
                if (a.trace) {
                    const uint64_t c2 = __builtin_amdgcn_s_memtime();
                    acc_c += c1 - c0;
                    acc_b += c2 - c1;
                }
            }
            // arm the block's own rows for the next sweep that reads them
            if (a.reset && !(a.diag & 1)) {
                const long s0 = (long)b * a.B, s1 = min(s0 + a.B, (long)a.n);
                const long r0 = a.upper ? a.n - s1 : s0, r1 = a.upper ? a.n - s0 : s1;
                uint64_t *rs = reinterpret_cast<uint64_t *>(a.reset);
                for (long i = r0 + t; i < r1; i += PK3_ROWS) rs[i] = TRI_SENTINEL;
            }
            if (a.trace && tid == 0) {
                a.trace[TRW * b + 4] = acc_c;
                a.trace[TRW * b + 5] = acc_b;
            }
        } else {
            // addresses of the next group (prepared one step ahead from LDS)
            int n_off = 0, n_row = 0, n_g[PK3_EXT];
            int lnx = 0, lnr = 0;  // packet j+1: x operand count, rows (landing)
#pragma unroll
            for (int e = 0; e < PK3_EXT; e++) n_g[e] = 0;
            auto prepare = [&](int j) {  // addresses of group j
                const int pl = j + A, pr = j + B, px = j + KE;
                n_off = pl < np ? offs[pl] : 0;
                n_row = 0;
                if (pr >= 0 && pr < np) {
                    const int *w = words(pr);
                    if (t < w[0]) n_row = w[4 + t];
                }
                int nx = 0;
                const int *xl = nullptr;
                if (px >= 0 && px < np) {
                    const int *w = words(px);
                    const int nr = w[0];
                    nx = w[3];
                    xl = w + 4 + nr + w[1] * nr;
                }
#pragma unroll
                for (int e = 0; e < PK3_EXT; e++) {
                    const int idx = t + PK3_ROWS * e;
                    n_g[e] = idx < nx && !(a.diag & 8) ? xl[idx] : 0;
                }
            };
            uint64_t acc_w = 0, acc_lb = 0, acc_is = 0, acc_pr = 0, acc_ld = 0, m0 = 0, m1 = 0;
            auto step = [&](int j, Pk4Regs &Ri, Pk4Regs &Rx, Pk4Regs &Rp) {
                if (a.trace) m0 = __builtin_amdgcn_s_memtime();
                // issue group j (addresses prepared last step)
#pragma unroll
                for (int e = 0; e < PK3_EXT; e++) Ri.ev[e] = ld_agent(a.x + n_g[e]);
                const v4i *src = a.data + n_off;
#pragma unroll
                for (int u = 0; u < PK3_LD; u++) Ri.pk[u] = src[t + PK3_ROWS * u];
                Ri.rh = a.rhs[(a.diag & 4) ? t : n_row];
                if (a.trace) {
                    m1 = __builtin_amdgcn_s_memtime();
                    acc_is += m1 - m0;
                }
                // landing bookkeeping of packet j+1 and addresses of group j+1
                lnr = 0;
                lnx = 0;
                if (j + 1 >= 0 && j + 1 < np) {
                    const int *w = words(j + 1);
                    lnr = __builtin_amdgcn_readfirstlane(w[0]);
                    lnx = __builtin_amdgcn_readfirstlane(w[3]);
                }
                prepare(j + 1);
                uint64_t l0 = 0;
                if (a.trace) {
                    l0 = __builtin_amdgcn_s_memtime();
                    acc_pr += l0 - m1;
                }
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WAITN) : "memory");
                asm volatile("" ::"v"(Rx.ev[0]), "v"(Rx.ev[1]), "v"(Rp.pk[0]), "v"(Rp.pk[1]), "v"(Rp.pk[2]),
                             "v"(Rp.rh));
                uint64_t l2 = 0;
                if (a.trace) {
                    l2 = __builtin_amdgcn_s_memtime();
                    acc_w += l2 - l0;
                }
                // land: words of packet j-KE+A, rhs and x operands of packet j+1
                if (j - KE >= -A) {
                    const int pl = j - KE + A;
                    if (pl < np) {
#pragma unroll
                        for (int u = 0; u < PK3_LD; u++) pbuf[pl % NS][t + PK3_ROWS * u] = Rp.pk[u];
                    }
                }
                if (t < lnr) rbuf[(j + 1) & 1][t] = Rp.rh;
#pragma unroll
                for (int e = 0; e < PK3_EXT; e++) {
                    const int idx = t + PK3_ROWS * e;
                    if (idx < lnx) {
                        uint64_t bits = Rx.ev[e];
                        if (bits == TRI_SENTINEL && !(a.diag & 8)) {
                            bits = poll_ready(a.x + words(j + 1)[4 + lnr + words(j + 1)[1] * lnr + idx], a.err);
                            if (a.trace) atomicAdd(&s_polls, 1u);
                        }
                        xbuf[(j + 1) & 1][idx] = __longlong_as_double((long long)bits);
                    }
                }
                uint64_t l1 = 0;
                if (a.trace) {
                    l1 = __builtin_amdgcn_s_memtime();
                    acc_ld += l1 - l2;
                }
                lds_barrier();
                if (a.trace) acc_lb += __builtin_amdgcn_s_memtime() - l1;
            };
            prepare(-A);
            Pk4Regs R0, R1, R2;
            for (int j0 = -A; j0 < nsteps - A; j0 += P) {
                if constexpr (KE == 1) {  // issue R[j], x operands from R[j], words/rhs from R[j-1]
                    step(j0, R0, R0, R1);
                    step(j0 + 1, R1, R1, R0);
                } else {  // KE == 2: x operands from R[j-1], words/rhs from R[j-2]
                    step(j0, R0, R2, R1);
                    step(j0 + 1, R1, R0, R2);
                    step(j0 + 2, R2, R1, R0);
                }
            }
            (void)R2;
            if (a.trace && tid == PK3_ROWS) {
                a.trace[TRW * b + 6] = acc_w;
                a.trace[TRW * b + 7] = acc_lb;
                a.trace[TRW * b + 8] = acc_is;
                a.trace[TRW * b + 9] = acc_pr;
                a.trace[TRW * b + 10] = acc_ld;
            }
        }
    }
}

// tri_mode 8: packets v5 (tri_bp.cpp build_packets5).  LDS holds only what
// is produced or gathered at run time -- the value ring, the rhs entries and
// the HBM x operands of the next packet -- plus the block's packet descriptors.
// The static part of a packet goes straight from HBM into registers:
//   compute lane t (waves 0-3) loads its row record (row, ring slot, EP codes,
//     EP values, diagonal) for packet j+D while it computes packet j.  Its only
//     other VMEM traffic is the x store, issued D+1 steps before any load it
//     waits for, so the in-order vmcnt wait never waits for a fresh store.
//   loader lane t (waves 4-7) loads packet j+IA's gather indices (row of lane
//     t, x operands t and t+256) and gathers rhs and x for packet j+KE with the
//     indices it loaded IA-KE steps earlier; it lands packet j+1's gathers at
//     the end of step j (polling TRI_SENTINEL values).
// Per step the LDS traffic is ~8 KB (was ~40 KB with staged packets), and a
// compute step's critical path is one LDS round trip plus the arithmetic.
struct Pk5Args {
    int nb;
    const int *blk;
    const int4 *desc;
    const uint32_t *rec;
    const int *idx;
    const double *rhs;
    double *x;
    double *reset;
    int n, B, upper;
    unsigned long long *claim;
    unsigned long long base;
    int *err;
    int diag;
    unsigned long long *trace;
};

template <int EP>
struct Pk5Rec {
    v4i i[EP == 4 ? 2 : 3];
    double v[EP];
    double dg;
    int nr, em;
};
struct Pk5Ld {
    int row, xi[PK3_EXT];
    int nr, nx;
    double rh;
    uint64_t ev[PK3_EXT];
};

template <int EP, int KE>
__global__ __launch_bounds__(2 * PK3_ROWS) void k_tri_pk5(Pk5Args a)
{
    constexpr int IA = KE + 2;   // gather indices are loaded IA steps ahead
    constexpr int D = KE + 2;    // compute records are loaded D steps ahead
    constexpr int Q = D + 1;     // register-set rotation period (both roles)
    constexpr int NI = EP == 4 ? 2 : 3;
    __shared__ double ring[BP_RING + 1];
    __shared__ double rbuf[2][PK3_ROWS];
    __shared__ double xbuf[2][PK3_ROWS * PK3_EXT];
    __shared__ int4 sdesc[PK3_CAP];
    __shared__ int s_blk;
    __shared__ unsigned s_polls;
    const int tid = threadIdx.x;
    const bool loader = __builtin_amdgcn_readfirstlane(tid) >= PK3_ROWS;
    const int t = tid & (PK3_ROWS - 1);
    if (tid == 0) ring[BP_RING] = 0.0;
    int prev = -1;
    for (;;) {
        __syncthreads();
        if (tid == 0) {
            if (a.trace && prev >= 0) {
                a.trace[8 * prev + 1] = __builtin_amdgcn_s_memrealtime();
                a.trace[8 * prev + 2] = s_polls;
            }
            s_polls = 0;
            s_blk = (int)(atomicAdd(a.claim, 1ull) - a.base);
        }
        __syncthreads();
        const int b = s_blk;
        if (b >= a.nb) break;
        if (a.trace && tid == 0) {
            unsigned xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            a.trace[8 * b] = __builtin_amdgcn_s_memrealtime();
            a.trace[8 * b + 3] = xcc;
        }
        prev = b;
        const int q0 = a.blk[b], np = a.blk[b + 1] - q0;
        for (int i = tid; i < np; i += 2 * PK3_ROWS) sdesc[i] = a.desc[q0 + i];
        __syncthreads();
        // both roles run steps j = -D .. -D+T-1, T a multiple of Q; a step's
        // out-of-range operations become loads from valid dummy addresses, so
        // every step issues the same loads and the unrolled loop is uniform
        const int T = (np + D + Q - 1) / Q * Q;
        auto desc = [&](int p) {
            const int4 d = sdesc[p];
            return make_int4(__builtin_amdgcn_readfirstlane(d.x), __builtin_amdgcn_readfirstlane(d.y),
                             __builtin_amdgcn_readfirstlane(d.z), __builtin_amdgcn_readfirstlane(d.w));
        };

        if (!loader) {
            uint64_t c0 = 0, c1 = 0, acc_c = 0, acc_b = 0;
            auto issue = [&](int p, Pk5Rec<EP> &R) {
                int ro = 0, nr = 0, em = 0;
                if (p >= 0 && p < np) {
                    const int4 d = desc(p);
                    ro = d.x;
                    nr = d.z & 0xffff;
                    em = d.w;
                }
                const int n1 = nr > 0 ? nr : 1, tt = min(t, n1 - 1);
                const v4i *base = reinterpret_cast<const v4i *>(a.rec) + ro;
#pragma unroll
                for (int u = 0; u < NI; u++) R.i[u] = base[u * n1 + tt];
                typedef double v2d __attribute__((ext_vector_type(2)));
                const v2d *vb = reinterpret_cast<const v2d *>(base + NI * n1);
#pragma unroll
                for (int q = 0; q < EP / 2; q++) {
                    const v2d v = vb[q * n1 + tt];
                    R.v[2 * q] = v.x;
                    R.v[2 * q + 1] = v.y;
                }
                R.dg = reinterpret_cast<const double *>(vb + (EP / 2) * n1)[tt];
                R.nr = nr;
                R.em = em;
            };
            auto step = [&](int j, Pk5Rec<EP> &Rc, Pk5Rec<EP> &Rn) {
                if (a.trace) c0 = __builtin_amdgcn_s_memtime();
                issue(j + D, Rn);
                // wait for packet j's record here, unconditionally (see k_tri_pk3)
                if constexpr (NI == 2)
                    asm volatile("" ::"v"(Rc.i[0]), "v"(Rc.i[1]), "v"(Rc.v[0]), "v"(Rc.v[1]), "v"(Rc.v[2]),
                                 "v"(Rc.v[3]), "v"(Rc.dg));
                else
                    asm volatile("" ::"v"(Rc.i[0]), "v"(Rc.i[1]), "v"(Rc.i[2]), "v"(Rc.v[0]), "v"(Rc.v[1]),
                                 "v"(Rc.v[2]), "v"(Rc.v[3]), "v"(Rc.v[4]), "v"(Rc.v[5]), "v"(Rc.v[6]),
                                 "v"(Rc.v[7]), "v"(Rc.dg));
                if (j >= 0 && j < np && t < Rc.nr) {
                    int cd[8];
                    cd[0] = Rc.i[0].z;
                    cd[1] = Rc.i[0].w;
                    cd[2] = Rc.i[1].x;
                    cd[3] = Rc.i[1].y;
                    if (EP == 8) {
                        cd[4] = Rc.i[1].z;
                        cd[5] = Rc.i[1].w;
                        cd[6] = Rc.i[2].x;
                        cd[7] = Rc.i[2].y;
                    }
                    const double *xb = xbuf[j & 1];
                    double acc = rbuf[j & 1][t], xv[EP];
#pragma unroll
                    for (int e = 0; e < EP; e++)
                        if (e < Rc.em) xv[e] = cd[e] < 0 ? ring[-1 - cd[e]] : xb[cd[e]];
#pragma unroll
                    for (int e = 0; e < EP; e++)
                        if (e < Rc.em) acc = acc - Rc.v[e] * xv[e];
                    const double xi = acc / Rc.dg;
                    ring[Rc.i[0].y] = xi;
                    if (!(a.diag & 2)) st_agent(a.x + Rc.i[0].x, xi);
                }
                if (a.trace) c1 = __builtin_amdgcn_s_memtime();
                lds_barrier();
                if (a.trace) {
                    const uint64_t c2 = __builtin_amdgcn_s_memtime();
                    acc_c += c1 - c0;
                    acc_b += c2 - c1;
                }
            };
            Pk5Rec<EP> R0, R1, R2, R3, R4;
            R0.nr = R1.nr = R2.nr = R3.nr = R4.nr = 0;
            // packet p lives in R[(p+1) % Q]; the loop starts at j = -D == 1 - Q,
            // so unrolled step u has j == u + 1 (mod Q)
            for (int j0 = -D; j0 < T - D; j0 += Q) {
                if constexpr (Q == 4) {
                    step(j0, R2, R1);
                    step(j0 + 1, R3, R2);
                    step(j0 + 2, R0, R3);
                    step(j0 + 3, R1, R0);
                } else {
                    step(j0, R2, R1);
                    step(j0 + 1, R3, R2);
                    step(j0 + 2, R4, R3);
                    step(j0 + 3, R0, R4);
                    step(j0 + 4, R1, R0);
                }
            }
            (void)R4;
            if (a.reset && !(a.diag & 1)) {
                const long s0 = (long)b * a.B, s1 = min(s0 + a.B, (long)a.n);
                const long r0 = a.upper ? a.n - s1 : s0, r1 = a.upper ? a.n - s0 : s1;
                uint64_t *rs = reinterpret_cast<uint64_t *>(a.reset);
                for (long i = r0 + t; i < r1; i += PK3_ROWS) rs[i] = TRI_SENTINEL;
            }
            if (a.trace && tid == 0) {
                a.trace[8 * b + 4] = acc_c;
                a.trace[8 * b + 5] = acc_b;
            }
        } else {
            uint64_t acc_w = 0, acc_lb = 0;
            auto issue_idx = [&](int p, Pk5Ld &L) {
                int io = 0, nr = 0, nx = 0;
                if (p >= 0 && p < np) {
                    const int4 d = desc(p);
                    io = d.y;
                    nr = d.z & 0xffff;
                    nx = d.z >> 16;
                }
                // clamped, branch-free indices (the buffer ends with one pad entry)
                const int *base = a.idx + io;
                L.row = base[max(min(t, nr - 1), 0)];
#pragma unroll
                for (int e = 0; e < PK3_EXT; e++) L.xi[e] = base[nr + max(min(t + PK3_ROWS * e, nx - 1), 0)];
                L.nr = nr;
                L.nx = nx;
            };
            auto gather = [&](Pk5Ld &L) {
                L.rh = a.rhs[(a.diag & 4) ? t : L.row];
#pragma unroll
                for (int e = 0; e < PK3_EXT; e++) L.ev[e] = ld_agent(a.x + ((a.diag & 8) ? 0 : L.xi[e]));
            };
            auto step = [&](int j, Pk5Ld &Li, Pk5Ld &Lg, Pk5Ld &Ll) {
                issue_idx(j + IA, Li);
                gather(Lg);
                uint64_t l0 = 0;
                if (a.trace) l0 = __builtin_amdgcn_s_memtime();
                asm volatile("" ::"v"(Ll.rh), "v"(Ll.ev[0]), "v"(Ll.ev[1]));
                uint64_t l2 = 0;
                if (a.trace) {
                    l2 = __builtin_amdgcn_s_memtime();
                    acc_w += l2 - l0;
                }
                if (j + 1 >= 0 && j + 1 < np) {  // land packet j+1
                    if (t < Ll.nr) rbuf[(j + 1) & 1][t] = Ll.rh;
#pragma unroll
                    for (int e = 0; e < PK3_EXT; e++) {
                        const int k = t + PK3_ROWS * e;
                        if (k < Ll.nx) {
                            uint64_t bits = Ll.ev[e];
                            if (bits == TRI_SENTINEL && !(a.diag & 8)) {
                                bits = poll_ready(a.x + Ll.xi[e], a.err);
                                if (a.trace) atomicAdd(&s_polls, 1u);
                            }
                            xbuf[(j + 1) & 1][k] = __longlong_as_double((long long)bits);
                        }
                    }
                }
                uint64_t l1 = 0;
                if (a.trace) l1 = __builtin_amdgcn_s_memtime();
                lds_barrier();
                if (a.trace) acc_lb += __builtin_amdgcn_s_memtime() - l1;
            };
            Pk5Ld L0, L1, L2, L3, L4;
            // valid dummy gather indices for the packets before 0
            L0.nr = L1.nr = L2.nr = L3.nr = L4.nr = 0;
            L0.nx = L1.nx = L2.nx = L3.nx = L4.nx = 0;
            L0.row = L1.row = L2.row = L3.row = L4.row = 0;
#pragma unroll
            for (int e = 0; e < PK3_EXT; e++) L0.xi[e] = L1.xi[e] = L2.xi[e] = L3.xi[e] = L4.xi[e] = 0;
            // packet p lives in L[(p+1) % Q]; step j: indices of packet j+IA into
            // L[j % Q], gathers of packet j+KE in L[(j+KE+1) % Q], landing of
            // packet j+1 from L[(j+2) % Q]; j0 == 1 (mod Q)
            for (int j0 = -D; j0 < T - D; j0 += Q) {
                if constexpr (Q == 4) {  // KE == 1: gather and land the same packet
                    step(j0, L1, L3, L3);
                    step(j0 + 1, L2, L0, L0);
                    step(j0 + 2, L3, L1, L1);
                    step(j0 + 3, L0, L2, L2);
                } else {                 // KE == 2
                    step(j0, L1, L4, L3);
                    step(j0 + 1, L2, L0, L4);
                    step(j0 + 2, L3, L1, L0);
                    step(j0 + 3, L4, L2, L1);
                    step(j0 + 4, L0, L3, L2);
                }
            }
            (void)L4;
            if (a.trace && tid == PK3_ROWS) {
                a.trace[8 * b + 6] = acc_w;
                a.trace[8 * b + 7] = acc_lb;
            }
        }
    }
}

// tri_mode 9: packets v6 (tri_bp.cpp build_packets6) with schedule-ordered
// shadow vectors.  k_tri_pk5's role split, plus:
//   * the sweep's output goes to a shadow vector in schedule order with
//     coalesced agent-scope stores (position pos0+t), and the HBM operands of
//     a packet are read from that shadow by schedule position: for a stencil
//     both are contiguous runs (one line per 8 rows instead of one per row);
//   * when the natural-order output is wanted too (the U sweep), a store wave
//     (wave 8) writes it from the LDS value ring one step later with plain
//     stores; it never waits on its vmcnt, so neither do the compute waves;
//   * arming for the next apply: the shadows are double-buffered, and every
//     block fills its own position range of the other buffer with
//     TRI_SENTINEL when it is done (coalesced).
// The compute waves' only VMEM traffic is the coalesced record loads and the
// coalesced shadow stores, so their in-order vmcnt wait for the record of the
// current packet never waits for a slow scattered store.
struct Pk6Args {
    int nb;
    const int *blk;
    const int4 *desc;
    const uint32_t *rec;
    const int *idx;
    const double *rhs;   // rhs entries, indexed by the packet's rhs indices
    double *sh;          // this sweep's shadow (schedule order), armed with TRI_SENTINEL
    double *sh_next;     // the other shadow buffer: armed here for the next apply
    double *nat;         // natural-order output (nullptr: none)
    int n, B;
    unsigned long long *claim;
    unsigned long long base;
    int *err;
    int diag;
    unsigned long long *trace;
    unsigned long long *trace2;  // diagnostics (LSSP_AMD_TRI_TRACE2): per-step clocks of blocks tb0, tb0+1
    int tb0;
};

typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
template <int EP>
struct Pk6Rec {
    typename std::conditional<EP == 4, v2u, v4u>::type c;  // int16 code pairs
    double v[EP];
    double dg;
    int row;
    int nr, pos0;
};

__device__ __forceinline__ int code16(int w, int hi) { return hi ? (w >> 16) : (int)(short)(w & 0xffff); }

template <int I, typename T>
__device__ __forceinline__ T &sel4(T &a, T &b, T &c, T &d)
{
    if constexpr (I == 0) return a;
    else if constexpr (I == 1) return b;
    else if constexpr (I == 2) return c;
    else return d;
}

// KE: steps of lead of the x-operand and rhs gathers; IA: of the gather-index
// loads (IA - KE of 1 or 2); D: of the compute lanes' record loads.  Register
// sets rotate with period Q = 4 (packet p lives in set p mod 4), so D <= 3 and
// IA <= 4.  Shallower prefetch keeps fewer requests in the CU's memory queue,
// which is what a cross-CU hand-off waits behind (MI355X_MICROARCH.md,
// handoff-1to1).
template <int EP, int KE, int IA, int D, bool NAT, int NR>
__global__ __launch_bounds__(NAT ? 2 * NR + 64 : 2 * NR) void k_tri_pk6(Pk6Args a)
{
    constexpr int Q = 4;
    static_assert(D + 1 <= Q && IA <= Q && KE >= 1 && IA - KE >= 1 && IA - KE <= 2, "pipeline depths");
    constexpr int S0 = (IA > D ? IA : D);
    constexpr int J0 = -((S0 + Q - 1) / Q) * Q;  // first step, a multiple of Q
    __shared__ double ring[BP_RING + 1];
    __shared__ double rbuf[2][NR];
    __shared__ double xbuf[2][NR * PK3_EXT];
    __shared__ int rowbuf[2][NR];
    __shared__ int4 sdesc[PK3_CAP];
    __shared__ int s_blk;
    __shared__ unsigned s_polls;
    const int tid = threadIdx.x;
    const int role = __builtin_amdgcn_readfirstlane(tid) / NR;  // 0 compute, 1 loader, 2 store
    static_assert(!NAT || NR == 256, "the store wave needs a 256-row packet");
    const int t = tid & (NR - 1);
    if (tid == 0) ring[BP_RING] = 0.0;
    int prev = -1;
    for (;;) {
        __syncthreads();
        if (tid == 0) {
            if (a.trace && prev >= 0) {
                a.trace[8 * prev + 1] = __builtin_amdgcn_s_memrealtime();
                a.trace[8 * prev + 2] = s_polls;
            }
            s_polls = 0;
            s_blk = (int)(atomicAdd(a.claim, 1ull) - a.base);
        }
        __syncthreads();
        const int b = s_blk;
        if (b >= a.nb) break;
        if (a.trace && tid == 0) {
            unsigned xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            a.trace[8 * b] = __builtin_amdgcn_s_memrealtime();
            a.trace[8 * b + 3] = xcc;
        }
        prev = b;
        const int q0 = a.blk[b], np = a.blk[b + 1] - q0;
        const int bbase = b * a.B;  // first schedule position of the block
        const bool tr2 = a.trace2 && (b == a.tb0 || b == a.tb0 + 1);
        auto mark = [&](int j, int k) {
            if (tr2 && j >= -8 && j < 1016)
                a.trace2[((long)(b - a.tb0) * 1024 + (j + 8)) * 4 + k] = __builtin_amdgcn_s_memrealtime();
        };
        for (int i = tid; i < np; i += blockDim.x) sdesc[i] = a.desc[q0 + i];
        __syncthreads();
        // both roles run steps J0 .. J0+T-1 (T a multiple of Q); out-of-range
        // packets turn into loads from valid dummy addresses
        const int T = (np - J0 + Q - 1) / Q * Q;
        auto desc = [&](int p) {
            const int4 d = sdesc[p];
            return make_int4(__builtin_amdgcn_readfirstlane(d.x), __builtin_amdgcn_readfirstlane(d.y),
                             __builtin_amdgcn_readfirstlane(d.z), __builtin_amdgcn_readfirstlane(d.w));
        };

        // descriptor of a packet, clamped: out-of-range packets get nr = nx = 0
        // and read valid dummy records (no branches around the loads)
        auto descc = [&](int p) {
            int4 d = desc(min(max(p, 0), max(np - 1, 0)));
            if (p < 0 || p >= np) d.z = 0;
            return d;
        };
        if (role == 0) {
            uint64_t c0 = 0, c1 = 0, acc_c = 0, acc_b = 0;
            auto issue = [&](const int4 d, Pk6Rec<EP> &Rr) {
                const int nr = d.z & 0x3ff;
                const int n1 = nr > 0 ? nr : 1, tt = min(t, n1 - 1);
                const uint32_t *base = a.rec + 4L * d.x;
                const int wc = ((EP / 2) * n1 + 3) & ~3, wd = (2 * n1 + 3) & ~3;
                Rr.c = reinterpret_cast<const decltype(Rr.c) *>(base)[tt];
                typedef double v2d __attribute__((ext_vector_type(2)));
                const v2d *vb = reinterpret_cast<const v2d *>(base + wc);
#pragma unroll
                for (int q = 0; q < EP / 2; q++) {
                    const v2d v = vb[q * n1 + tt];
                    Rr.v[2 * q] = v.x;
                    Rr.v[2 * q + 1] = v.y;
                }
                Rr.dg = reinterpret_cast<const double *>(vb + (EP / 2) * n1)[tt];
                if (NAT) Rr.row = reinterpret_cast<const int *>(base + wc + 2 * EP * n1 + wd)[tt];
                Rr.nr = nr;
                Rr.pos0 = d.w;
            };
            int4 dn = descc(J0 + D);  // descriptor of packet j+D, read one step ahead
            auto step = [&](int j, Pk6Rec<EP> &Rc, Pk6Rec<EP> &Rn) {
                if (a.trace) c0 = __builtin_amdgcn_s_memtime();
                issue(dn, Rn);
                dn = descc(j + D + 1);
                if constexpr (EP == 4)
                    asm volatile("" ::"v"(Rc.c), "v"(Rc.v[0]), "v"(Rc.v[1]), "v"(Rc.v[2]), "v"(Rc.v[3]), "v"(Rc.dg));
                else
                    asm volatile("" ::"v"(Rc.c), "v"(Rc.v[0]), "v"(Rc.v[1]), "v"(Rc.v[2]), "v"(Rc.v[3]), "v"(Rc.v[4]),
                                 "v"(Rc.v[5]), "v"(Rc.v[6]), "v"(Rc.v[7]), "v"(Rc.dg));
                if (NAT) asm volatile("" ::"v"(Rc.row));
                if (t < Rc.nr) {  // nr == 0 outside the block's packets
                    const double *xb = xbuf[j & 1];
                    double acc = rbuf[j & 1][t];
                    double xv[EP];
                    // all EP entries: padded ones read +0.0 and subtract +0.0*+0.0
#pragma unroll
                    for (int e = 0; e < EP; e++) {
                        const int cd = code16((int)Rc.c[e / 2], e & 1);
                        xv[e] = cd < 0 ? ring[-1 - cd] : xb[cd];
                    }
#pragma unroll
                    for (int e = 0; e < EP; e++) acc = acc - Rc.v[e] * xv[e];
                    const double xi = acc / Rc.dg;
                    const int pos = Rc.pos0 + t;
                    ring[(pos - bbase) & (BP_RING - 1)] = xi;
                    if (NAT) rowbuf[j & 1][t] = Rc.row;
                    if (!(a.diag & 2)) st_agent(a.sh + pos, xi);
                }
                if (a.trace) c1 = __builtin_amdgcn_s_memtime();
                if (tid == 0) mark(j, 0);
                lds_barrier();
                if (a.trace) {
                    const uint64_t c2 = __builtin_amdgcn_s_memtime();
                    acc_c += c1 - c0;
                    acc_b += c2 - c1;
                }
            };
            Pk6Rec<EP> R0, R1, R2, R3;
            R0.nr = R1.nr = R2.nr = R3.nr = 0;
            for (int j0 = J0; j0 < J0 + T; j0 += Q) {  // j0 == 0 (mod Q): packet p in set p mod Q
                step(j0, sel4<0>(R0, R1, R2, R3), sel4<(0 + D) % Q>(R0, R1, R2, R3));
                step(j0 + 1, sel4<1>(R0, R1, R2, R3), sel4<(1 + D) % Q>(R0, R1, R2, R3));
                step(j0 + 2, sel4<2>(R0, R1, R2, R3), sel4<(2 + D) % Q>(R0, R1, R2, R3));
                step(j0 + 3, sel4<3>(R0, R1, R2, R3), sel4<(3 + D) % Q>(R0, R1, R2, R3));
            }
            // arm the block's positions of the other shadow for the next apply
            if (!(a.diag & 1)) {
                const long s0 = bbase, s1 = min(s0 + a.B, (long)a.n);
                uint64_t *rs = reinterpret_cast<uint64_t *>(a.sh_next);
                for (long i = s0 + t; i < s1; i += NR) rs[i] = TRI_SENTINEL;
            }
            if (a.trace && tid == 0) {
                a.trace[8 * b + 4] = acc_c;
                a.trace[8 * b + 5] = acc_b;
            }
        } else if (role == 1) {
            // The loader's loads are issued from inline asm with explicit
            // vmcnt waits: its register sets rotate across the loop back-edge,
            // where the compiler's own wait counting turns conservative and
            // waited for the previous step's gathers before issuing new ones.
            // Per step, in issue order: 3 index loads (packet j+IA), then 3
            // gathers (packet j+KE) -- so before the gathers, the indices they
            // use (issued at step j-2) have exactly 12 younger loads, and the
            // gathers landed at the end of step j (packet j+1, issued at step
            // j+1-KE) have 6 (KE 2) or 0 (KE 1) younger loads.
            static_assert(PK3_EXT == 2, "wait counts below assume 3 + 3 loads per step");
            constexpr int WAIT_IDX = 6 * (IA - KE);  // younger than the indices the gathers use
            uint64_t acc_w = 0, acc_lb = 0, acc_is = 0, acc_ld = 0, m0 = 0;
            auto issue_idx = [&](const int4 d, Pk5Ld &L) {
                const int nr = d.z & 0x3ff, nx = (d.z >> 10) & 0x7ff;
                const int *base = a.idx + d.y;
                const int *p0 = base + max(min(t, nr - 1), 0);
                const int *p1 = base + nr + max(min(t, nx - 1), 0);
                const int *p2 = base + nr + max(min(t + NR, nx - 1), 0);
                asm volatile("global_load_dword %0, %1, off" : "=v"(L.row) : "v"(p0) : "memory");
                asm volatile("global_load_dword %0, %1, off" : "=v"(L.xi[0]) : "v"(p1) : "memory");
                asm volatile("global_load_dword %0, %1, off" : "=v"(L.xi[1]) : "v"(p2) : "memory");
                L.nr = nr;
                L.nx = nx;
            };
            auto gather = [&](Pk5Ld &L) {
                asm volatile("s_waitcnt vmcnt(%3)" : "+v"(L.row), "+v"(L.xi[0]), "+v"(L.xi[1]) : "n"(WAIT_IDX) : "memory");
                const double *pr = a.rhs + ((a.diag & 4) ? t : L.row);
                const double *px0 = a.sh + ((a.diag & 8) ? 0 : L.xi[0]);
                const double *px1 = a.sh + ((a.diag & 8) ? 0 : L.xi[1]);
                asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(L.rh) : "v"(pr) : "memory");
                asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=v"(L.ev[0]) : "v"(px0) : "memory");
                asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=v"(L.ev[1]) : "v"(px1) : "memory");
            };
            int4 dl = descc(J0 + IA);  // descriptor of packet j+IA, read one step ahead
            auto step = [&](int j, Pk5Ld &Li, Pk5Ld &Lg, Pk5Ld &Ll) {
                if (a.diag & 16) {  // timing experiment: loader idle
                    lds_barrier();
                    return;
                }
                if (a.trace) m0 = __builtin_amdgcn_s_memtime();
                issue_idx(dl, Li);
                gather(Lg);
                dl = descc(j + IA + 1);
                uint64_t l0 = 0;
                if (a.trace) {
                    l0 = __builtin_amdgcn_s_memtime();
                    acc_is += l0 - m0;
                }
                // gathers of packet j+1 were issued at step j+1-KE
                asm volatile("s_waitcnt vmcnt(%3)" : "+v"(Ll.rh), "+v"(Ll.ev[0]), "+v"(Ll.ev[1]) : "n"(6 * (KE - 1)) : "memory");
                uint64_t l2 = 0;
                if (a.trace) {
                    l2 = __builtin_amdgcn_s_memtime();
                    acc_w += l2 - l0;
                }
                if (tid == NR) mark(j, 2);
                // land packet j+1 (nr = nx = 0 outside the block's packets)
                if (t < Ll.nr) rbuf[(j + 1) & 1][t] = Ll.rh;
#pragma unroll
                for (int e = 0; e < PK3_EXT; e++) {
                    const int k = t + NR * e;
                    if (k < Ll.nx) {
                        uint64_t bits = Ll.ev[e];
                        if (bits == TRI_SENTINEL && !(a.diag & 8)) {
                            bits = poll_ready(a.sh + Ll.xi[e], a.err);
                            if (a.trace) atomicAdd(&s_polls, 1u);
                        }
                        xbuf[(j + 1) & 1][k] = __longlong_as_double((long long)bits);
                    }
                }
                uint64_t l1 = 0;
                if (a.trace) {
                    l1 = __builtin_amdgcn_s_memtime();
                    acc_ld += l1 - l2;
                }
                if (tid == NR) {
                    mark(j, 1);
                    if (tr2 && j >= -8 && j < 1016) a.trace2[((long)(b - a.tb0) * 1024 + (j + 8)) * 4 + 3] = s_polls;
                }
                lds_barrier();
                if (a.trace) acc_lb += __builtin_amdgcn_s_memtime() - l1;
            };
            Pk5Ld L0, L1, L2, L3;
            L0.nr = L1.nr = L2.nr = L3.nr = 0;
            L0.nx = L1.nx = L2.nx = L3.nx = 0;
            L0.row = L1.row = L2.row = L3.row = 0;
#pragma unroll
            for (int e = 0; e < PK3_EXT; e++) L0.xi[e] = L1.xi[e] = L2.xi[e] = L3.xi[e] = 0;
            L0.rh = L1.rh = L2.rh = L3.rh = 0;
#define LSSP_PK6_LSTEP(u)                                                                          \
    step(j0 + u, sel4<(u + IA) % Q>(L0, L1, L2, L3), sel4<(u + KE) % Q>(L0, L1, L2, L3), \
         sel4<(u + 1) % Q>(L0, L1, L2, L3))
            for (int j0 = J0; j0 < J0 + T; j0 += Q) {  // packet p in set p mod Q
                LSSP_PK6_LSTEP(0);
                LSSP_PK6_LSTEP(1);
                LSSP_PK6_LSTEP(2);
                LSSP_PK6_LSTEP(3);
            }
#undef LSSP_PK6_LSTEP
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            (void)acc_lb;
            if (a.trace && tid == NR) {  // compute's barrier share is dropped here
                a.trace[8 * b + 5] = acc_w;
                a.trace[8 * b + 6] = acc_is;
                a.trace[8 * b + 7] = acc_ld;
            }
        } else {
            // store wave: at step j write packet j-1's values in natural order
            // (the last step's packet after the loop)
            const int lane = tid & 63;
            auto store = [&](int p) {
                if (NAT && p >= 0 && p < np) {
                    const int4 d = desc(p);
                    const int nr = d.z & 0x3ff;
                    for (int k = lane; k < nr; k += 64)
                        a.nat[rowbuf[p & 1][k]] = ring[(d.w + k - bbase) % BP_RING];
                }
            };
            for (int j = J0; j < J0 + T; j++) {
                store(j - 1);
                lds_barrier();
            }
            store(J0 + T - 1);
        }
    }
}

// diagnostics only (LSSP_AMD_TRI_TRACE): synchronous dump of the per-block
// trace of one packet sweep, one JSON line (tools/tri_trace.py)
static int dump_trace(lssp_amd_ctx *c, unsigned long long *d_trace, int nb, int n, int npk, int grid,
                      const char *path, int width = 8)
{
    std::vector<unsigned long long> h(width * (size_t)nb);
    LSSP_HIP(hipMemcpyAsync(h.data(), d_trace, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost,
                            c->stream));
    LSSP_HIP(hipStreamSynchronize(c->stream));
    (void)hipFree(d_trace);
    FILE *f = fopen(path, "a");
    if (!f) return LSSP_AMD_OK;
    fprintf(f, "{\"n\": %d, \"nb\": %d, \"npk\": %d, \"grid\": %d, \"blocks\": [", n, nb, npk, grid);
    for (int b = 0; b < nb; b++) {
        fprintf(f, "%s[", b ? ", " : "");
        for (int k = 0; k < width; k++) fprintf(f, "%s%llu", k ? ", " : "", h[(size_t)width * b + k]);
        fprintf(f, "]");
    }
    fprintf(f, "]}\n");
    fclose(f);
    return LSSP_AMD_OK;
}

int launch_trisolve(lssp_amd_ctx *c, const TriSched &t, const double *rhs, double *x, double *reset)
{
    if (t.n == 0) return LSSP_AMD_OK;
    long nchunks = (t.n + 63) / 64;
    TriArgs a{t.n, nchunks, t.perm, t.rp, t.cols, t.vals, t.diag, t.unit, rhs, x, reset, c->d_err};
    if (c->tri_mode == 8 && t.pk5_n >= 0) {
        const int grid = std::min(t.bp_nb, c->num_cus);
        const char *trace_path = getenv("LSSP_AMD_TRI_TRACE");
        unsigned long long *d_trace = nullptr;
        if (trace_path) {
            LSSP_HIP(hipMalloc(&d_trace, sizeof(unsigned long long) * 8 * t.bp_nb));
            LSSP_HIP(hipMemsetAsync(d_trace, 0, sizeof(unsigned long long) * 8 * t.bp_nb, c->stream));
        }
        Pk5Args g{t.bp_nb, t.pk5_blk, reinterpret_cast<const int4 *>(t.pk5_desc), t.pk5_rec, t.pk5_idx, rhs, x,
                  reset, t.n, t.bp_B, t.upper, t.pk5_claim, t.pk5_base, c->d_err, c->tri_diag, d_trace};
        const bool ke2 = c->tri_depth == 2;
        if (t.pk5_ep == 4) {
            if (ke2) k_tri_pk5<4, 2><<<grid, 2 * PK3_ROWS, 0, c->stream>>>(g);
            else k_tri_pk5<4, 1><<<grid, 2 * PK3_ROWS, 0, c->stream>>>(g);
        } else {
            if (ke2) k_tri_pk5<8, 2><<<grid, 2 * PK3_ROWS, 0, c->stream>>>(g);
            else k_tri_pk5<8, 1><<<grid, 2 * PK3_ROWS, 0, c->stream>>>(g);
        }
        t.pk5_base += (unsigned long long)t.bp_nb + grid;
        LSSP_HIP(hipGetLastError());
        if (trace_path) LSSP_TRY(dump_trace(c, d_trace, t.bp_nb, t.n, t.pk5_n, grid, trace_path));
        return LSSP_AMD_OK;
    }
    if (c->tri_mode == 7 && t.pk4_n >= 0) {
        const int grid = std::min(t.bp_nb, c->num_cus);
        const char *trace_path = getenv("LSSP_AMD_TRI_TRACE");
        unsigned long long *d_trace = nullptr;
        if (trace_path) {
            LSSP_HIP(hipMalloc(&d_trace, sizeof(unsigned long long) * TRW * t.bp_nb));
            LSSP_HIP(hipMemsetAsync(d_trace, 0, sizeof(unsigned long long) * TRW * t.bp_nb, c->stream));
        }
        Pk4Args g{t.bp_nb, t.pk4_blk, t.pk4_off, reinterpret_cast<const v4i *>(t.pk4_data), t.unit, rhs, x, reset,
                  t.n, t.bp_B, t.upper, t.pk4_claim, t.pk4_base, c->d_err, c->tri_diag, d_trace};
        if (c->tri_depth == 1) k_tri_pk4<1><<<grid, 2 * PK3_ROWS, 0, c->stream>>>(g);
        else k_tri_pk4<2><<<grid, 2 * PK3_ROWS, 0, c->stream>>>(g);
        t.pk4_base += (unsigned long long)t.bp_nb + grid;
        LSSP_HIP(hipGetLastError());
        if (trace_path) LSSP_TRY(dump_trace(c, d_trace, t.bp_nb, t.n, t.pk4_n, grid, trace_path, TRW));
        return LSSP_AMD_OK;
    }
    if (c->tri_mode == 6 && t.pk3_n >= 0) {
        const int grid = std::min(t.bp_nb, c->num_cus);
        const char *trace_path = getenv("LSSP_AMD_TRI_TRACE");
        unsigned long long *d_trace = nullptr;
        if (trace_path) {
            LSSP_HIP(hipMalloc(&d_trace, sizeof(unsigned long long) * 8 * t.bp_nb));
            LSSP_HIP(hipMemsetAsync(d_trace, 0, sizeof(unsigned long long) * 8 * t.bp_nb, c->stream));
        }
        Pk3Args g{t.bp_nb, t.pk3_blk, t.pk3_off, reinterpret_cast<const v4i *>(t.pk3_data), t.unit, rhs, x, reset,
                  t.pk3_claim, t.pk3_base, c->d_err, c->tri_diag, d_trace};
        if (c->tri_depth == 3) k_tri_pk3<3><<<grid, 2 * PK3_ROWS, 0, c->stream>>>(g);
        else k_tri_pk3<2><<<grid, 2 * PK3_ROWS, 0, c->stream>>>(g);
        t.pk3_base += (unsigned long long)t.bp_nb + grid;
        LSSP_HIP(hipGetLastError());
        if (trace_path) LSSP_TRY(dump_trace(c, d_trace, t.bp_nb, t.n, t.pk3_n, grid, trace_path));
        return LSSP_AMD_OK;
    }
    if (c->tri_mode == 5 && t.pk_n >= 0) {
        const int grid = std::min(t.bp_nb, c->num_cus);
        PkArgs g{t.bp_nb, t.pk_blk, t.pk_off, reinterpret_cast<const int4 *>(t.pk_data), t.unit, rhs, x, reset,
                 t.pk_claim, t.pk_base, c->d_err, c->tri_diag};
        k_tri_pk2<<<grid, 256, 0, c->stream>>>(g);
        t.pk_base += (unsigned long long)t.bp_nb + grid;
        LSSP_HIP(hipGetLastError());
        return LSSP_AMD_OK;
    }
    if (c->tri_mode == 4 && t.pk_n >= 0) {
        const int grid = std::min(t.bp_nb, c->num_cus);
        PkArgs g{t.bp_nb, t.pk_blk, t.pk_off, reinterpret_cast<const int4 *>(t.pk_data), t.unit, rhs, x, reset,
                 t.pk_claim, t.pk_base, c->d_err, c->tri_diag};
        k_tri_pk<<<grid, 256, 0, c->stream>>>(g);
        t.pk_base += (unsigned long long)t.bp_nb + grid;
        LSSP_HIP(hipGetLastError());
        return LSSP_AMD_OK;
    }
    if (c->tri_mode == 3) {
        const int grid = std::min(t.bp_nb, c->num_cus);
        t.bp_epoch++;
        BPArgs g{t.bp_B, t.bp_nb, t.bp_blk_step, t.bp_step_pos, t.bp_step_need, t.bp_step_done,
                 t.bp_step_flag, t.bp_perm, t.bp_rp, t.bp_cols, t.bp_vals, t.bp_diag, t.unit, rhs, x,
                 nullptr /* no sentinel protocol here */, t.bp_prog, t.bp_claim, t.bp_base, t.bp_epoch, c->d_err};
        k_tri_bp<<<grid, 256, 0, c->stream>>>(g);
        t.bp_base += (unsigned long long)t.bp_nb + grid;
        LSSP_HIP(hipGetLastError());
        return LSSP_AMD_OK;
    }
    if (c->tri_mode == 1) {
        for (int l = 0; l < t.nlevels; l++) {
            const int lo = t.level_ptr[l], hi = t.level_ptr[l + 1];
            k_trisolve_level<<<(hi - lo + 255) / 256, 256, 0, c->stream>>>(a, lo, hi);
        }
    } else {
        long grid = (long)c->num_cus * c->tri_blocks_per_cu;
        long need = (nchunks + 3) / 4;
        if (grid > need) grid = need;
        if (c->tri_mode == 2) k_trisolve<0><<<grid, 256, 0, c->stream>>>(a);
        else k_trisolve<1><<<grid, 256, 0, c->stream>>>(a);
    }
    LSSP_HIP(hipGetLastError());
    return LSSP_AMD_OK;
}

// tri_mode 9 apply: cache = L^-1 rhs, x = U^-1 cache through the shadows
template <bool NAT>
static int launch_pk6(lssp_amd_ctx *c, const TriSched &t, const double *rhs, double *sh, double *sh_next,
                      double *nat)
{
    const int grid = std::min(t.bp_nb, c->num_cus);
    const char *trace_path = getenv("LSSP_AMD_TRI_TRACE");
    unsigned long long *d_trace = nullptr;
    if (trace_path) {
        LSSP_HIP(hipMalloc(&d_trace, sizeof(unsigned long long) * 8 * t.bp_nb));
        LSSP_HIP(hipMemsetAsync(d_trace, 0, sizeof(unsigned long long) * 8 * t.bp_nb, c->stream));
    }
    const char *t2 = getenv("LSSP_AMD_TRI_TRACE2");  // "path:block"
    unsigned long long *d_t2 = nullptr;
    int tb0 = 0;
    if (t2) {
        const char *colon = strrchr(t2, ':');
        tb0 = colon ? atoi(colon + 1) : t.bp_nb / 2;
        LSSP_HIP(hipMalloc(&d_t2, sizeof(unsigned long long) * 2 * 1024 * 4));
        LSSP_HIP(hipMemsetAsync(d_t2, 0, sizeof(unsigned long long) * 2 * 1024 * 4, c->stream));
    }
    Pk6Args g{t.bp_nb, t.pk6_blk, reinterpret_cast<const int4 *>(t.pk6_desc), t.pk6_rec, t.pk6_idx, rhs, sh,
              sh_next, nat, t.n, t.bp_B, t.pk6_claim, t.pk6_base, c->d_err, c->tri_diag, d_trace, d_t2, tb0};
    // Instantiated: 256-row packets, x operands gathered 2 steps ahead (KE 2),
    // EP 4 or 8 -- the variants whose inline-asm loader tools/check_vmcnt.py
    // (tests/test_isa_vmcnt.py) verifies hazard-free
    if (t.pk6_rows != 256) return LSSP_AMD_EUNSUPPORTED;
    // pipeline depths (LSSP_AMD_TRI_PIPE): 0 = (KE 2, IA 4, D 3), 1 = (2, 3, 3), 2 = (2, 3, 2)
    const int pd = c->tri_pipe;
    if constexpr (NAT) {
        if (t.pk6_ep != 4) return LSSP_AMD_EUNSUPPORTED;
        k_tri_pk6<4, 2, 4, 3, true, 256><<<grid, 2 * 256 + 64, 0, c->stream>>>(g);
    } else if (t.pk6_ep == 4) {
        if (pd == 1) k_tri_pk6<4, 2, 3, 3, false, 256><<<grid, 512, 0, c->stream>>>(g);
        else if (pd == 2) k_tri_pk6<4, 2, 3, 2, false, 256><<<grid, 512, 0, c->stream>>>(g);
        else k_tri_pk6<4, 2, 4, 3, false, 256><<<grid, 512, 0, c->stream>>>(g);
    } else {
        k_tri_pk6<8, 2, 4, 3, false, 256><<<grid, 512, 0, c->stream>>>(g);
    }
    t.pk6_base += (unsigned long long)t.bp_nb + grid;
    LSSP_HIP(hipGetLastError());
    if (trace_path) LSSP_TRY(dump_trace(c, d_trace, t.bp_nb, t.n, t.pk6_n, grid, trace_path));
    if (t2) {  // diagnostics only: per-step clocks of two consecutive blocks
        std::vector<unsigned long long> h(2 * 1024 * 4);
        LSSP_HIP(hipMemcpyAsync(h.data(), d_t2, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost,
                                c->stream));
        LSSP_HIP(hipStreamSynchronize(c->stream));
        (void)hipFree(d_t2);
        std::string path(t2, strrchr(t2, ':') ? strrchr(t2, ':') - t2 : strlen(t2));
        FILE *f = fopen(path.c_str(), "a");
        if (f) {
            fprintf(f, "{\"tb0\": %d, \"steps\": [", tb0);
            for (size_t i = 0; i < h.size(); i++) fprintf(f, "%s%llu", i ? ", " : "", h[i]);
            fprintf(f, "]}\n");
            fclose(f);
        }
    }
    return LSSP_AMD_OK;
}

// permutations between natural order and a sweep's schedule order (positions).
// XCD-aware: workgroup w runs on XCD w % 8 (round-robin dispatch) and walks
// the XCD's contiguous eighth of the positions, so the natural-order lines a
// position range touches (the same few z-planes for a stencil) are reused
// inside one XCD's L2 instead of being fetched once per XCD.
template <bool GATHER>
__global__ __launch_bounds__(256) void k_perm(double *dst, const double *src, const int *perm, int n)
{
    const int nx = 8, per = gridDim.x / nx;
    const int xcd = blockIdx.x % nx, k = blockIdx.x / nx;
    const long chunk = ((long)n + nx - 1) / nx;
    const long lo = xcd * chunk, hi = min((long)n, lo + chunk);
    for (long p = lo + (long)k * 256 + threadIdx.x; p < hi; p += (long)per * 256) {
        if (GATHER) dst[p] = src[perm[p]];
        else dst[perm[p]] = src[p];
    }
}

// tri_mode 9 apply.  The scattered halves of the work -- reading the rhs in L
// order and writing x in natural order -- run as fully parallel permutation
// kernels around the two sweeps, so the pipelined sweeps only touch
// contiguous runs of HBM.  LSSP_AMD_TRI_NAT=1 instead writes x from the U
// sweep's store wave (timing experiments).
int launch_ilu_apply(lssp_amd_ctx *c, const lssp_amd_ilu *M, double *x, const double *rhs)
{
    if (c->tri_mode == 9 && M->lower.pk6_n > 0 && M->upper.pk6_n > 0) {
        const int n = M->n;
        if (!M->d_sh[0]) {
            for (int k = 0; k < 4; k++) {
                LSSP_HIP(hipMalloc(&M->d_sh[k], sizeof(double) * n));
                LSSP_TRY(launch_fill(c, M->d_sh[k], n, TRI_SENTINEL));
            }
            LSSP_HIP(hipMalloc(&M->d_rperm, sizeof(double) * n));
        }
        const int e = M->epoch & 1;
        M->epoch++;
        const int pg = 8 * std::max(1, std::min((n + 2047) / 2048, c->num_cus));  // multiple of 8
        k_perm<true><<<pg, 256, 0, c->stream>>>(M->d_rperm, rhs, M->lower.bp_perm, n);
        LSSP_HIP(hipGetLastError());
        LSSP_TRY(launch_pk6<false>(c, M->lower, M->d_rperm, M->d_sh[e], M->d_sh[e ^ 1], nullptr));
        static const bool nat = getenv("LSSP_AMD_TRI_NAT") && atoi(getenv("LSSP_AMD_TRI_NAT"));
        if (nat && M->upper.pk6_ep == 4)
            return launch_pk6<true>(c, M->upper, M->d_sh[e], M->d_sh[2 + e], M->d_sh[2 + (e ^ 1)], x);
        LSSP_TRY(launch_pk6<false>(c, M->upper, M->d_sh[e], M->d_sh[2 + e], M->d_sh[2 + (e ^ 1)], nullptr));
        k_perm<false><<<pg, 256, 0, c->stream>>>(x, M->d_sh[2 + e], M->upper.bp_perm, n);
        LSSP_HIP(hipGetLastError());
        return LSSP_AMD_OK;
    }
    LSSP_TRY(launch_trisolve(c, M->lower, rhs, M->d_cache, x));
    return launch_trisolve(c, M->upper, M->d_cache, x, M->d_cache);
}

// halo: gather owned entries to send
__global__ void k_pack(const int *idx, const double *x, double *buf, int n)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) buf[i] = x[idx[i]];
}

int launch_pack(lssp_amd_ctx *c, const int *idx, const double *x, double *buf, int n)
{
    if (n <= 0) return LSSP_AMD_OK;
    k_pack<<<(n + 255) / 256, 256, 0, c->stream>>>(idx, x, buf, n);
    LSSP_HIP(hipGetLastError());
    return LSSP_AMD_OK;
}

}  // namespace lssp_amd
