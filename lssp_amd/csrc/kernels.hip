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

template <int EPI, int NRED>
__global__ __launch_bounds__(256) void k_spmv(SpmvArgs a)
{
    __shared__ int sj[SPMV_CAP];
    __shared__ double sx[SPMV_CAP];
    __shared__ double lds[MAX_SLOTS][4];
    const long blk = blockIdx.x;
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

static int g_spmv_variant = -1;  // LSSP_AMD_SPMV: 0 k_spmv, 1 k_spmv2, 2 k_spmv2 + XCD order

template <int EPI>
static void spmv_dispatch(const SpmvArgs &a, int nred, long nblocks, hipStream_t s)
{
    if (g_spmv_variant < 0) {
        const char *e = getenv("LSSP_AMD_SPMV");
        g_spmv_variant = e ? atoi(e) : 0;
    }
    if (g_spmv_variant == 0) {
        if (nred == 0) k_spmv<EPI, 0><<<nblocks, 256, 0, s>>>(a);
        else if (nred == 1) k_spmv<EPI, 1><<<nblocks, 256, 0, s>>>(a);
        else k_spmv<EPI, 2><<<nblocks, 256, 0, s>>>(a);
    } else if (g_spmv_variant == 1) {
        if (nred == 0) k_spmv2<EPI, 0, 0><<<nblocks, 256, 0, s>>>(a, nblocks);
        else if (nred == 1) k_spmv2<EPI, 1, 0><<<nblocks, 256, 0, s>>>(a, nblocks);
        else k_spmv2<EPI, 2, 0><<<nblocks, 256, 0, s>>>(a, nblocks);
    } else {
        const long g = (nblocks + 7) / 8 * 8;
        if (nred == 0) k_spmv2<EPI, 0, 1><<<g, 256, 0, s>>>(a, nblocks);
        else if (nred == 1) k_spmv2<EPI, 1, 1><<<g, 256, 0, s>>>(a, nblocks);
        else k_spmv2<EPI, 2, 1><<<g, 256, 0, s>>>(a, nblocks);
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
    case EPI_MXY: spmv_dispatch<EPI_MXY>(a, nred, nb, c->stream); break;
    case EPI_AMXY: spmv_dispatch<EPI_AMXY>(a, nred, nb, c->stream); break;
    case EPI_AXPBY: spmv_dispatch<EPI_AXPBY>(a, nred, nb, c->stream); break;
    default: spmv_dispatch<EPI_AMX>(a, nred, nb, c->stream); break;
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

int launch_trisolve(lssp_amd_ctx *c, const TriSched &t, const double *rhs, double *x, double *reset)
{
    if (t.n == 0) return LSSP_AMD_OK;
    long nchunks = (t.n + 63) / 64;
    TriArgs a{t.n, nchunks, t.perm, t.rp, t.cols, t.vals, t.diag, t.unit, rhs, x, reset, c->d_err};
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
