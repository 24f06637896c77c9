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

#include <algorithm>
#include <climits>
#include <vector>

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
    return wave_sum_l0(v);  // lane 0 holds the halving-tree result (internal.h)
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
    case FIN_BICG_RES_RHO:  // :141 then the next iteration's :87
    case FIN_BICG_RES_RHO_B: {
        t0 = sqrt(s[0]);
        scal[S_RES] = t0;
        double rho1 = s[1];
        t1 = rho1;
        scal[S_RHO1] = rho1;
        scal[S_BETA] = (rho1 * scal[S_ALPHA]) / (scal[S_RHO0] * scal[S_OMEGA]);
        scal[S_RHO0] = rho1;
        if (f.op == FIN_BICG_RES_RHO_B) {  // :117 / :149 / :89 decided here; the host reads the batch afterwards
            const int k = (int)scal[S_NIT];
            scal[S_H + k % S_HB] = t0;
            scal[S_NIT] = k + 1;
            if (scal[S_BREAK] != 0.0) scal[S_DONE] = 2.0;
            else if (t0 <= scal[S_TOL]) scal[S_DONE] = 1.0;
            else if (rho1 == 0) scal[S_DONE] = 3.0;
        }
        break;
    }
    case FIN_BICG_S_OMEGA: {  // solver-bicgstab.cxx:117, then :135 (one reduction round for both)
        const double sn = sqrt(s[2]);
        scal[S_SNORM] = sn;
        scal[S_BREAK] = sn <= 1e-40 ? 1.0 : 0.0;
        scal[S_OMEGA] = s[0] / s[1];
        if (trace && f.tpos[2] >= 0) trace[f.tpos[2]] = sn;
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
    case FIN_CG_RES_RHO:  // :106, then the next :80 with z == r (PC_NON)
    case FIN_CG_RES_RHO_B: {
        t0 = sqrt(s[0]);
        scal[S_RES] = t0;
        t1 = s[0];
        scal[S_RHO1] = s[0];
        scal[S_BETA] = s[0] / scal[S_RHO0];
        if (f.op == FIN_CG_RES_RHO_B) {  // :109 decided here; the host reads the batch afterwards
            const int k = (int)scal[S_NIT];
            scal[S_H + k % S_HB] = t0;
            scal[S_NIT] = k + 1;
            if (t0 <= scal[S_TOL]) scal[S_DONE] = k + 1;  // the stamp of k_cg_fused's deferred x update
        }
        break;
    }
    }
    if (trace) {
        if (f.tpos[0] >= 0) trace[f.tpos[0]] = t0;
        if (f.tpos[1] >= 0) trace[f.tpos[1]] = t1;
    }
}

// Level 2 of the canonical reduction, spread over L2_LANES / 64
// one-wave workgroups on as many CUs: workgroup q is wave q of the 1024-lane
// level 2 (lanes 64q .. 64q+63, lane t adding partials t, t+1024, ... in order
// onto 0.0, then the wave's halving tree), so the partials are pulled by 16
// CUs instead of one (a single 1024-lane workgroup took ~12 us for the 2 x
// 315 KB of a 10M-row pair of dots, this 7.7 us).  Each wave sum is published
// write-through (sc1) and drained before an arrival ticket; the last arriver
// combines the 16 wave sums with the same halving tree and runs the finalize
// program.
__device__ __forceinline__ void st_sc1(double *p, double v)
{
    __hip_atomic_store(reinterpret_cast<uint64_t *>(p), (uint64_t)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double *p)
{
    return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const uint64_t *>(p),
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

__global__ __launch_bounds__(64) void k_reduce2m(const double *__restrict__ part, long pcap, long C, int nslot,
                                                double *sums, double *scal, double *trace, Fin f, int do_fin,
                                                double *wsum, unsigned *cnt, const double *guard)
{
    if (guard && *guard != 0.0) return;
    const int q = blockIdx.x, t = q * 64 + threadIdx.x;  // lane t of the 1024-lane level 2
    for (int s = 0; s < nslot; s++) {
        const double *p = part + s * pcap;
        double a = 0.0;
        for (long k0 = t; k0 < C; k0 += 32L * L2_LANES) {
            double v[32];
#pragma unroll
            for (int u = 0; u < 32; u++) {
                const long k = k0 + (long)u * L2_LANES;
                v[u] = k < C ? p[k] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 32; u++)
                if (k0 + (long)u * L2_LANES < C) a += v[u];
        }
        a = wave_sum(a);
        if (threadIdx.x == 0) st_sc1(wsum + s * 16 + q, a);
    }
    unsigned last = 0;
    if (threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the wave sums are in memory before the ticket
        last = atomicAdd(cnt, 1u) == gridDim.x - 1;
    }
    last = __shfl(last, 0, 64);
    if (!last) return;
    if (threadIdx.x == 0) {
        double r[MAX_SLOTS] = {0, 0, 0, 0};
        for (int s = 0; s < nslot; s++) {
            double u[16];
            for (int w = 0; w < 16; w++) u[w] = ld_sc1(wsum + s * 16 + w);
            for (int off = 8; off >= 1; off >>= 1)
                for (int l = 0; l < off; l++) u[l] = u[l] + u[l + off];
            r[s] = u[0];
            sums[s] = r[s];
        }
        __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (do_fin) finalize(f, r, scal, trace);
    }
}

// serial order: one lane, sum += a[i]*b[i] from 0 (vector.cxx:123-133)
struct SerialArgs {
    const double *a[MAX_SLOTS];
    const double *b[MAX_SLOTS];
};

// SERIAL reduction mode: sum += x[i]*y[i] for i = 0 .. n-1 from 0.0, exactly
// vector.cxx:123-133.  The additions are ONE dependent chain per slot, so the
// kernel's speed is the f64 add's dependent latency times n; everything else
// is kept off that chain:
//   * wave 0 runs the chains, lane s the chain of slot s (up to MAX_SLOTS dots
//     of one round cost the same as one), with SIMD 0 to itself: the product
//     waves are the 12 waves on SIMDs 1-3 (wave % 4 != 0; waves 4, 8, 12 only
//     take part in the barriers), so no other wave's VALU issue interleaves
//     with the chain;
//   * the products (each rounded as the reference rounds it: -ffp-contract=off)
//     of the next 2048-element chunk are written to the other LDS buffer while
//     the chain adds the current one, slot-major so lane s reads its own two
//     consecutive products with one ds_read_b128;
//   * the chain reads its operands 16 at a time, one batch ahead in registers,
//     so the LDS latency is hidden behind the previous batch's 16 adds.
// A chunk's tail is padded with +0.0: a running sum that starts at +0.0 (or a
// previous rank's running sum, itself such a sum) is never -0.0, and s + 0.0
// == s for every other s, so the padding never changes a bit.
constexpr int SER_C = 2048;  // elements per LDS chunk
#ifndef SER_BATCH
#define SER_BATCH 16
#endif
constexpr int SER_B = SER_BATCH;  // elements per register batch of the chain
static_assert(SER_C % SER_B == 0, "whole batches per chunk");
// carry (multi-rank): the running sums of the ranks before this one, so the
// chain continues theirs and the P ranks add in global index order.
__global__ __launch_bounds__(1024) void k_dot_serial(SerialArgs g, long n, int nslot, double *sums, double *scal,
                                                     double *trace, Fin f, int do_fin, const double *carry,
                                                     const double *guard)
{
    if (guard && *guard != 0.0) return;
    __shared__ __attribute__((aligned(16))) double buf[2][MAX_SLOTS][SER_C];  // read as double2
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const long nch = (n + SER_C - 1) / SER_C;
    const bool producer = (wave & 3) != 0;
    const int pid = (wave - 1 - (wave >> 2)) * 64 + lane;  // 0 .. 767 over the 12 product waves
    auto fill = [&](long k, int bsel) {
        for (int s = 0; s < nslot; s++) {
            const double *x = g.a[s], *y = g.b[s];
            for (int i = pid; i < SER_C; i += 768) {
                const long e = k * SER_C + i;
                buf[bsel][s][i] = e < n ? x[e] * y[e] : 0.0;
            }
        }
    };
    const int sl = lane < nslot ? lane : 0;
    double acc = carry ? carry[sl] : 0.0;
    if (producer && nch > 0) fill(0, 0);
    __syncthreads();
    for (long k = 0; k < nch; k++) {
        if (producer) {
            if (k + 1 < nch) fill(k + 1, (k + 1) & 1);
        } else if (wave == 0) {
            const long m = min((long)SER_C, n - k * SER_C);
            const int nb = (int)((m + SER_B - 1) / SER_B);
            const double2 *B = reinterpret_cast<const double2 *>(&buf[k & 1][sl][0]);
            // two register sets, a batch's reads issued before the previous
            // batch's adds (the empty asm with a memory clobber keeps the reads
            // ahead of them); a read past the chunk's last batch re-reads batch 0
            double2 va[SER_B / 2], vb[SER_B / 2];
            auto rd = [&](double2 (&v)[SER_B / 2], int q) {
                const int qq = q < SER_C / SER_B ? q : 0;
#pragma unroll
                for (int u = 0; u < SER_B / 2; u++) v[u] = B[qq * (SER_B / 2) + u];
            };
            auto add = [&](const double2 (&v)[SER_B / 2]) {
#pragma unroll
                for (int u = 0; u < SER_B / 2; u++) {
                    acc = acc + v[u].x;
                    acc = acc + v[u].y;
                }
            };
            rd(va, 0);
            for (int q = 0; q < nb; q += 2) {
                rd(vb, q + 1);
                asm volatile("" ::: "memory");
                add(va);
                if (q + 1 >= nb) break;
                rd(va, q + 2);
                asm volatile("" ::: "memory");
                add(vb);
            }
        }
        __syncthreads();
    }
    if (wave == 0) {
        double r[MAX_SLOTS];
#pragma unroll
        for (int s = 0; s < MAX_SLOTS; s++) r[s] = __shfl(acc, s, 64);
        if (lane == 0) {
            for (int s = 0; s < nslot; s++) sums[s] = r[s];
            if (do_fin) finalize(f, r, scal, trace);
        }
    }
}

__global__ void k_finalize(const double *sums, double *scal, double *trace, Fin f)
{
    double r[MAX_SLOTS];
    for (int s = 0; s < MAX_SLOTS; s++) r[s] = s < f.nsum ? sums[s] : 0.0;
    finalize(f, r, scal, trace);
}

// multi-rank: gathered [P][MAX_SLOTS] rank sums, summed in rank order (tree
// mode), or the last rank's running sums, which are the global sums (serial)
__global__ void k_sum_ranks(const double *gath, int P, int nslot, double *sums, double *scal,
                            double *trace, Fin f, int serial, const double *guard)
{
    if (guard && *guard != 0.0) return;
    double r[MAX_SLOTS] = {0, 0, 0, 0};
    for (int s = 0; s < nslot; s++) {
        double t = serial ? gath[(P - 1) * MAX_SLOTS + s] : gath[s];
        for (int q = 1; q < P && !serial; q++) t = t + gath[q * MAX_SLOTS + s];
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
    const double *w0, *w1;  // fused dot operands: red0 = z*w0, red1 = z*(w1 ? w1 : z), red2 = w0*w0
    double *part;
    long pcap;
    const uint8_t *Ad;  // diagonal-id column coding (lssp_amd_mat::Ad), CMP kernels
    const int *off;
    int ndiag;
    const double *guard;  // lssp_amd_ctx::guard
    long blk0;            // first chunk of this launch (spmv_halo splits a product)
    int streams;          // concurrent block streams (a multiple of 8, spmv_streams)
    int pbpp, pz, pw;     // column-group block order (spmv_group_env): blocks per plane, planes, group width; 0: natural
    int ntv;              // w0 / w1 / z as non-temporal accesses
};

// The 256-row blocks are dealt so that each of the 8 XCDs owns one contiguous
// eighth of the rows (dispatch round-robins workgroups over XCDs, workgroup w
// runs on XCD w % 8); the x entries a block gathers are then re-used by the
// neighbouring blocks of the same XCD out of its L2 (7-pt: x is fetched once
// instead of ~1.3 times, rocprofv3 FETCH_SIZE).  Every global access a lane
// makes before the barrier is issued up front and branch-free -- the block's Aj / Ax range as 16-byte loads (widened to 16-byte
// boundaries, clamped to the padded arrays; entries outside the block are
// dropped when landing in LDS) and the lane's own Ap[r], Ap[r+1] -- so one
// memory round trip covers the staging and the row bounds.
// CMP: the columns come from the diagonal-id bytes (col = row + off[Ad[k]]),
// 1 byte per entry instead of 4 (7-pt: 0.83 of the CSR bytes per product).
template <int EPI, int NRED, bool CMP>
__global__ __launch_bounds__(256) void k_spmv3(SpmvArgs a, long nblk, long nnz_pad)
{
    constexpr int NX2 = (SPMV_CAP / 2 + 1 + 255) / 256;  // double2 loads per lane
    constexpr int NJ4 = CMP ? 1 : (SPMV_CAP / 4 + 1 + 255) / 256;  // int4 loads per lane (16 ids when CMP)
    __shared__ __attribute__((aligned(16))) double sx[SPMV_CAP + 2];
    __shared__ __attribute__((aligned(16))) int sj[CMP ? SPMV_CAP / 4 + 8 : SPMV_CAP + 4];
    __shared__ int soff[CMP ? 256 : 1];
    __shared__ double lds[MAX_SLOTS][4];
    // the guard is read with the row bounds and tested before the entries are
    // loaded: its round trip overlaps theirs instead of preceding it
    const double gv = a.guard ? *a.guard : 0.0;
    const long per = gridDim.x / a.streams;
    long lb = (blockIdx.x % a.streams) * per + blockIdx.x / a.streams;
    if (lb >= nblk) return;
    if (a.pbpp > 0 && lb < (long)a.pbpp * a.pz) {
        const long gs = (long)a.pw * a.pz, g = lb / gs, rem = lb - g * gs;
        lb = (rem / a.pw) * a.pbpp + g * a.pw + rem % a.pw;
    }
    const long blk = a.blk0 + lb;
    const int r0 = (int)(blk * 256);
    const int tid = threadIdx.x;
    const int r = r0 + tid;
    const int rend = min(r0 + 256, a.nrows);
    const int base = a.Ap[r0];
    const int cnt = a.Ap[rend] - base;
    const int rr = min(r, a.nrows - 1);
    const int rb = a.Ap[rr], re = a.Ap[rr + 1];
    // the fused dots' second operands, loaded up front with the row bounds (the
    // compiler may not move them above the z store: w0 / w1 may alias z, and
    // then they are read as the value just stored, zv, below)
    double w0p = 0.0, w1p = 0.0;
    if (NRED > 0) {
        if (a.ntv) {
            if (a.w0 != a.z) w0p = __builtin_nontemporal_load(a.w0 + rr);
            if (NRED > 1 && a.w1 && a.w1 != a.z) w1p = __builtin_nontemporal_load(a.w1 + rr);
        } else {
            if (a.w0 != a.z) w0p = a.w0[rr];
            if (NRED > 1 && a.w1 && a.w1 != a.z) w1p = a.w1[rr];
        }
    }
    if (gv != 0.0) return;  // a batched iteration past the stop (lssp_amd_ctx::guard)
    double sum = 0;
    if (cnt <= SPMV_CAP) {
        typedef double dbl2_t __attribute__((ext_vector_type(2)));
        typedef int int4_t __attribute__((ext_vector_type(4)));
        // CMP: jb / jmax / jn count 16-byte vectors of ids (16 entries each)
        constexpr int JS = CMP ? 4 : 2;  // log2 entries per 16-byte vector
        const long xb = base & ~1L, jb = base & ~((1L << JS) - 1);
        // clamp to the block's last vector: lanes past the range re-read it
        // (no extra lines), and the padded arrays keep it in bounds
        const long last = cnt > 0 ? (long)base + cnt - 1 : (long)base;
        const long xmax = min(last >> 1, (nnz_pad >> 1) - 1);
        const long jmax = min(last >> JS, (CMP ? (nnz_pad - 4 + 32) >> 4 : nnz_pad >> 2) - 1);
        if (CMP && tid < a.ndiag) soff[tid] = a.off[tid];
        const dbl2_t *X2 = reinterpret_cast<const dbl2_t *>(a.Ax);
        const int4_t *J4 = CMP ? reinterpret_cast<const int4_t *>(a.Ad) : reinterpret_cast<const int4_t *>(a.Aj);
        dbl2_t vx[NX2];
        int4_t vj[NJ4];
#pragma unroll
        for (int u = 0; u < NX2; u++) vx[u] = __builtin_nontemporal_load(X2 + min((xb >> 1) + tid + 256 * u, xmax));
#pragma unroll
        for (int u = 0; u < NJ4; u++) vj[u] = __builtin_nontemporal_load(J4 + min((jb >> JS) + tid + 256 * u, jmax));
        const int xn = (int)(xmax - (xb >> 1)) + 1, jn = (int)(jmax - (jb >> JS)) + 1;  // vectors in range
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
            const unsigned char *sd = reinterpret_cast<const unsigned char *>(sj);
            auto col = [&](int k) { return CMP ? r + soff[sd[k + oj]] : sj[k + oj]; };
            if (len > 0 && len <= 8) {
                // all x gathers of the row in flight at once; the products are
                // then added in CSR order (clamped extra lanes are not added)
                double pr[8];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int k = min(rb + u, re - 1);
                    pr[u] = a.x[col(k)] * sx[k + ox];
                }
#pragma unroll
                for (int u = 0; u < 8; u++)
                    if (u < len) sum += pr[u];
            } else {
                for (int k = rb; k < re; k++) sum += a.x[col(k)] * sx[k + ox];
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
        if (a.ntv) __builtin_nontemporal_store(zv, a.z + r);
        else a.z[r] = zv;
    }
    if (NRED > 0) {
        double v[NRED > 0 ? NRED : 1];
        if (r < a.nrows) {
            v[0] = zv * (a.w0 == a.z ? zv : w0p);
            if (NRED > 1) v[NRED > 1 ? 1 : 0] = zv * (a.w1 && a.w1 != a.z ? w1p : zv);
            if (NRED > 2) v[NRED > 2 ? 2 : 0] = w0p * w0p;  // (launch_spmv: w0 != z)
        } else {
#pragma unroll
            for (int q = 0; q < NRED; q++) v[q] = 0.0;
        }
        chunk_reduce<NRED>(v, a.part, a.pcap, blk, lds);
    }
}

// Windowed-x product for matrices without the diagonal-id coding whose rows
// stay near the diagonal (build_windows, capi.cpp): a 1024-row workgroup (4
// reduction chunks) first stages its x span [lo, hi) (<= WIN_CAP entries)
// into LDS with coalesced loads, then each lane forms its row's products from
// LDS.  The gathers of a locally shuffled numbering (config 5) each hit a
// separate L2 line when read from memory; from LDS they cost a bank access.
// The entries come from the matrix's sliced copy (lssp_amd_mat::s_ax ...):
// the block's rows sorted by length into 64-row slices, entry k of every row
// of a slice in one contiguous 64-lane column, so each load is one coalesced
// wave access (the CSR rows of a wave start at scattered offsets, and their
// per-lane loads were the larger half of the kernel's time).  The column is a
// 16-bit offset into the staged span.  A lane adds its row's products in CSR
// order onto 0.0 -- the arithmetic of k_spmv3 -- and writes the sum to LDS at
// the row's place in the block; after a barrier thread t takes row t, so the
// output store and the fused dots' 256-row chunk partials are those of the
// natural order.
// The product runs persistently (round 6; one workgroup per block before,
// 1.7 % slower on config 5's product, profiles/r06/r06z8_*): one 1024-thread
// workgroup per CU (the LDS ring allows one) walks a contiguous range of
// blocks.  x is staged in an LDS ring of WIN_CAP entries indexed by column
// mod WIN_CAP, and a block loads only the part of its span [lo2, hi) that is
// not already resident from the previous block (consecutive spans of a locally
// shuffled numbering mostly coincide: config 5 loads ~1 K of a block's ~12 K
// span entries).  Two spans of at most WIN_CAP entries that overlap never map
// a needed column onto another needed column, so after the load [lo2, hi) is
// resident whatever was there before.  The next block's entries, row map, dot
// operands and the first XPF x entries of its missing span are loaded into
// registers while the current block is computed; its window and slice bases
// one block earlier still.
template <int EPI, int NRED>
__global__ __launch_bounds__(WIN_ROWS) void k_spmv_sell(SpmvArgs a, const int *__restrict__ win,
                                                         const double *__restrict__ sax,
                                                         const uint32_t *__restrict__ scol,
                                                         const uint32_t *__restrict__ srow,
                                                         const int *__restrict__ smeta, long nblk)
{
    __shared__ double sxw[WIN_CAP];
    __shared__ double zb[WIN_ROWS];
    __shared__ double lds[4][MAX_SLOTS][4];
    constexpr int NK = 10, XPF = 2, MASK = WIN_CAP - 1;
    static_assert((WIN_CAP & MASK) == 0, "ring of a power of two");
    if (a.guard && *a.guard != 0.0) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const long b0 = blockIdx.x * nblk / gridDim.x, b1 = (blockIdx.x + 1) * nblk / gridDim.x;
    if (b0 >= b1) return;
    const double *x = a.x;
    struct Next {
        int lo2, hi;       // the block's span
        uint32_t ri;       // row map word
        uint32_t cw[NK / 2];
        double ax[NK];
        double w0p, w1p;
        double xv[XPF];    // missing-span entries tid, tid + 1024 (flat order: A then B)
        int na, a0, b0c, nmiss;
    };
    // missing part of [lo2, hi) against the resident [vlo, vhi): A = [lo2, min(hi, vlo)),
    // B = [max(lo2, vhi), hi); flat index f < na is A's, else B's
    auto miss_col = [](const Next &q, int f) { return f < q.na ? q.a0 + f : q.b0c + (f - q.na); };
    auto fetch = [&](long b, int mlo, int mhi, int vlo, int vhi, int sb, Next &q) {
        q.lo2 = mlo;
        q.hi = mhi;
        const int ae = min(mhi, vlo);
        q.a0 = mlo;
        q.na = ae > mlo ? ae - mlo : 0;
        q.b0c = max(mlo, vhi);
        const int nbm = mhi > q.b0c ? mhi - q.b0c : 0;
        q.nmiss = q.na + nbm;
#pragma unroll
        for (int u = 0; u < XPF; u++) {
            const int f = tid + WIN_ROWS * u;
            q.xv[u] = f < q.nmiss ? x[miss_col(q, f)] : 0.0;
        }
        q.ri = srow[b * WIN_ROWS + tid];
#pragma unroll
        for (int k = 0; k < NK / 2; k++) q.cw[k] = scol[sb / 2 + 64 * k + lane];
#pragma unroll
        for (int k = 0; k < NK; k++) q.ax[k] = sax[sb + 64 * k + lane];
        const int r = (int)(b * WIN_ROWS) + tid, rr = min(r, a.nrows - 1);
        const int r0 = (int)(b * WIN_ROWS), r1 = min(r0 + WIN_ROWS, a.nrows);
        const bool w0x = NRED > 0 && a.w0 == a.x && a.w0 != a.z && r0 >= mlo && r1 <= mhi;
        q.w0p = 0.0;
        q.w1p = 0.0;
        if (NRED > 0) {
            if (a.w0 != a.z && !w0x) q.w0p = a.w0[rr];
            if (NRED > 1 && a.w1 && a.w1 != a.z) q.w1p = a.w1[rr];
        }
    };
    auto meta = [&](long b, int &mlo, int &mhi, int &sb) {
        mlo = win[2 * b] & ~1;
        mhi = win[2 * b + 1];
        sb = __builtin_amdgcn_readfirstlane(smeta[2 * (b * (WIN_ROWS / 64) + wave)]);
    };
    int vlo = 0, vhi = 0;  // resident span (none)
    int mlo, mhi, msb;
    meta(b0, mlo, mhi, msb);
    Next cur, nxt;
    fetch(b0, mlo, mhi, vlo, vhi, msb, nxt);
    if (b0 + 1 < b1) meta(b0 + 1, mlo, mhi, msb);
    int par = 0;
    for (long b = b0; b < b1; b++, par ^= 1) {
        cur = nxt;
        __syncthreads();  // the previous block's ring and zb reads are done
#pragma unroll
        for (int u = 0; u < XPF; u++) {
            const int f = tid + WIN_ROWS * u;
            if (f < cur.nmiss) sxw[miss_col(cur, f) & MASK] = cur.xv[u];
        }
        for (int f = tid + WIN_ROWS * XPF; f < cur.nmiss; f += WIN_ROWS) {  // a span mostly new
            const int col = miss_col(cur, f);
            sxw[col & MASK] = x[col];
        }
        vlo = cur.lo2;
        vhi = cur.hi;
        __syncthreads();
        if (b + 1 < b1) {
            fetch(b + 1, mlo, mhi, vlo, vhi, msb, nxt);
            if (b + 2 < b1) meta(b + 2, mlo, mhi, msb);
        }
        const int r = (int)(b * WIN_ROWS) + tid;
        const int len = (int)(cur.ri >> 10), lr = (int)(cur.ri & 1023);
        const int lo2 = cur.lo2;
        double sum = 0;
#pragma unroll
        for (int k = 0; k < NK; k++)
            if (k < len) sum += sxw[(lo2 + (int)((cur.cw[k >> 1] >> (16 * (k & 1))) & 0xffffu)) & MASK] * cur.ax[k];
        if (len > NK) {  // rows longer than NK entries
            const long sl = b * (WIN_ROWS / 64) + wave;
            const int sb = __builtin_amdgcn_readfirstlane(smeta[2 * sl]);
            for (int k = NK; k < len; k++) {
                const uint32_t c = scol[sb / 2 + 64 * (k >> 1) + lane];
                sum += sxw[(lo2 + (int)((c >> (16 * (k & 1))) & 0xffffu)) & MASK] * sax[sb + 64L * k + lane];
            }
        }
        zb[lr] = sum;
        __syncthreads();
        sum = zb[tid];
        const int r0 = (int)(b * WIN_ROWS), r1 = min(r0 + WIN_ROWS, a.nrows);
        const bool w0x = NRED > 0 && a.w0 == a.x && a.w0 != a.z && r0 >= cur.lo2 && r1 <= cur.hi;
        double w0p = cur.w0p;
        if (w0x && r < a.nrows) w0p = sxw[r & MASK];
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
                v[0] = zv * (a.w0 == a.z ? zv : w0p);
                if (NRED > 1) v[NRED > 1 ? 1 : 0] = zv * (a.w1 && a.w1 != a.z ? cur.w1p : zv);
            } else {
#pragma unroll
                for (int q = 0; q < NRED; q++) v[q] = 0.0;
            }
            // chunk_reduce's order for each of the 4 chunks (waves 4q .. 4q+3);
            // the next block writes lds only after three more barriers
            const int q = wave >> 2;
#pragma unroll
            for (int t = 0; t < NRED; t++) {
                const double sv = wave_sum(v[t]);
                if (lane == 0) lds[q][t][wave & 3] = sv;
            }
            __syncthreads();
            const long chunk = b * 4 + (tid >> 8);
            if ((tid & 255) == 0 && chunk * 256 < a.nrows) {
                const int cq = tid >> 8;
#pragma unroll
                for (int t = 0; t < NRED; t++)
                    a.part[t * a.pcap + chunk] = (lds[cq][t][0] + lds[cq][t][1]) + (lds[cq][t][2] + lds[cq][t][3]);
            }
        }
    }
}

template <int EPI>
static void spmv_sell_dispatch(const SpmvArgs &a, const lssp_amd_mat *A, int nred, hipStream_t s, int num_cus)
{
    const long nb = (a.nrows + WIN_ROWS - 1) / WIN_ROWS;
    const long g = std::min<long>(nb, num_cus);  // one workgroup per CU (the LDS ring)
    if (nred == 0) k_spmv_sell<EPI, 0><<<g, WIN_ROWS, 0, s>>>(a, A->d_win, A->s_ax, A->s_col, A->s_row, A->s_meta, nb);
    else if (nred == 1) k_spmv_sell<EPI, 1><<<g, WIN_ROWS, 0, s>>>(a, A->d_win, A->s_ax, A->s_col, A->s_row, A->s_meta, nb);
    else k_spmv_sell<EPI, 2><<<g, WIN_ROWS, 0, s>>>(a, A->d_win, A->s_ax, A->s_col, A->s_row, A->s_meta, nb);
}

// Workgroup w of the product takes block (w % K) * (grid / K) + w / K: K
// streams of consecutive blocks, stream q on XCD q % 8 (dispatch deals
// workgroups round-robin over the 8 XCDs), so the x entries a block gathers
// (+-1, +-N, +-N^2 rows away) are re-used by its stream's later blocks out of
// that XCD's L2 / the MALL.  K = 8 walks each XCD's eighth as ONE window; more
// streams spread the concurrent HBM reads over the address space (a streaming
// read of contiguous per-workgroup chunks runs at 7.0 TB/s against 5.3-6.3
// for one narrow window, tools/probe/read_probe.hip) -- but for this product
// K = 8 measured fastest: 143.7 us at 216^3 against 148-159 us for K = 16 ..
// 256 (profiles/r04/r04c_stream_order.txt; the x re-use out of L2 is worth
// more).  LSSP_AMD_SPMV_STREAMS overrides it (A/B runs).
// Column-group block order (stencil matrices whose widest offset, the plane,
// is a whole number of 256-row blocks): the plane's blocks are cut into
// groups of W consecutive blocks, and position t of the traversal takes, group
// by group, block jb of the group in every plane in turn (t -> group, plane,
// block).  With the natural order a block's +-plane gathers are re-read one
// plane of rows later, after ~16 MB of the matrix streamed through the XCD's
// 4 MB L2, so x is fetched ~3 times when the plane is large (512^2 z-slab:
// 1538 MB against 1248 algorithmic, rocprofv3 FETCH_SIZE); in a group its
// neighbours in the traversal are the next plane's blocks, and x is fetched
// ~1.1 times (W = 128: 1277 MB).  The time gained is smaller than the bytes
// (the re-reads mostly hit the MALL): 512^3 y = A x 2.32 -> 2.17 ms, the
// 8-rank slab's BiCGSTAB iteration -1.6 %, 512^2 x 64 alone unchanged
// (profiles/r05/r05l_spmv_group_order.txt).  Automatic for planes of >= 512
// blocks (128 Ki rows; smaller planes keep x in L2 anyway) with W = 128;
// LSSP_AMD_SPMV_ORDER=W forces a width (0: natural order; tests, A/B runs).
static int spmv_group_env()
{
    static const int k = [] {
        const char *e = getenv("LSSP_AMD_SPMV_ORDER");
        return e ? std::max(0, atoi(e)) : -1;
    }();
    return k;
}

// w0 / w1 loads and the z store as non-temporal accesses (no other block
// re-reads them): the 8-rank slab's iteration -0.3 .. -0.6 %.
// LSSP_AMD_SPMV_NTV=0 turns them off (A/B runs).
static int spmv_ntv()
{
    static const int k = [] {
        const char *e = getenv("LSSP_AMD_SPMV_NTV");
        return e ? atoi(e) : 1;
    }();
    return k;
}

// LSSP_AMD_SPMV_STREAMS=K forces K streams (A/B runs); 0: the matrix's own
// choice (tune_spmv_streams), 8 when it has none
static int spmv_streams_env()
{
    static const int k = [] {
        const char *e = getenv("LSSP_AMD_SPMV_STREAMS");
        const int v = e ? atoi(e) : 0;
        return v >= 8 && v % 8 == 0 && v <= 4096 ? v : 0;
    }();
    return k;
}
static int spmv_streams(const lssp_amd_mat *A)
{
    const int e = spmv_streams_env();
    return e ? e : A->streams > 0 ? A->streams : 8;
}

template <int EPI, bool CMP>
static void spmv_dispatch(const SpmvArgs &a, int nred, long nblocks, hipStream_t s, long nnz_pad)
{
    const long g = (nblocks + a.streams - 1) / a.streams * a.streams;  // a multiple of K: whole stream shares
    if (nred == 0) k_spmv3<EPI, 0, CMP><<<g, 256, 0, s>>>(a, nblocks, nnz_pad);
    else if (nred == 1) k_spmv3<EPI, 1, CMP><<<g, 256, 0, s>>>(a, nblocks, nnz_pad);
    else if (nred == 2 || EPI != EPI_AMX) k_spmv3<EPI, 2, CMP><<<g, 256, 0, s>>>(a, nblocks, nnz_pad);
    else k_spmv3<EPI_AMX, 3, CMP><<<g, 256, 0, s>>>(a, nblocks, nnz_pad);
}

template <int EPI>
static void spmv_dispatch(const SpmvArgs &a, int nred, long nblocks, hipStream_t s, long nnz_pad)
{
    if (a.ndiag > 0) spmv_dispatch<EPI, true>(a, nred, nblocks, s, nnz_pad);
    else spmv_dispatch<EPI, false>(a, nred, nblocks, s, nnz_pad);
}

int launch_spmv(lssp_amd_ctx *c, const lssp_amd_mat *A, int epi, double alpha, const double *x,
                double beta, const double *y, double *z, int nred, const double *w0,
                const double *w1, long cb, long ce)
{
    if (A->nrows == 0) return LSSP_AMD_OK;
    const long nall = num_chunks(A->nrows);
    LSSP_TRY(ensure_part(c, nall));
    if (ce < 0) ce = nall;
    if (cb < 0 || cb > ce || ce > nall) return LSSP_AMD_EINVAL;
    // three fused dots (BiCGSTAB's t = A sh with t.s, t.t, s.s): EPI_AMX on k_spmv3
    // only -- a windowed matrix keeps its CSR resident, so k_spmv3 serves it
    if (nred == 3 && (epi != EPI_AMX || !w0 || w0 == z || w1)) return LSSP_AMD_EINVAL;
    const long nb = ce - cb;
    if (nb == 0) return LSSP_AMD_OK;
    SpmvArgs a{A->nrows, A->Ap, A->Aj, A->Ax, x, y, z, alpha, beta, w0, w1, c->d_part, c->part_cap,
               A->Ad, A->d_off, A->ndiag, c->guard, cb, spmv_streams(A), 0, 0, 0, spmv_ntv()};
    const long plane = A->max_off_int;
    if (A->ndiag > 0 && plane >= 256 * 8 && plane % 256 == 0) {
        const long bpp = plane / 256;
        const int env = spmv_group_env();
        const int pw = env >= 0 ? env : (bpp >= 512 && bpp % 128 == 0 ? 128 : 0);
        if (pw > 0 && bpp % pw == 0 && nb / bpp >= 2) {
            a.pbpp = (int)bpp;
            a.pz = (int)(nb / bpp);
            a.pw = pw;
        }
    }
    if (A->d_win && nb == nall && nred <= 2) {
        switch (epi) {
        case EPI_MXY: spmv_sell_dispatch<EPI_MXY>(a, A, nred, c->stream, c->num_cus); break;
        case EPI_AMXY: spmv_sell_dispatch<EPI_AMXY>(a, A, nred, c->stream, c->num_cus); break;
        case EPI_AXPBY: spmv_sell_dispatch<EPI_AXPBY>(a, A, nred, c->stream, c->num_cus); break;
        default: spmv_sell_dispatch<EPI_AMX>(a, A, nred, c->stream, c->num_cus); break;
        }
        LSSP_HIP(hipGetLastError());
        return LSSP_AMD_OK;
    }
    switch (epi) {
    case EPI_MXY: spmv_dispatch<EPI_MXY>(a, nred, nb, c->stream, A->nnz + 4L); break;
    case EPI_AMXY: spmv_dispatch<EPI_AMXY>(a, nred, nb, c->stream, A->nnz + 4L); break;
    case EPI_AXPBY: spmv_dispatch<EPI_AXPBY>(a, nred, nb, c->stream, A->nnz + 4L); break;
    default: spmv_dispatch<EPI_AMX>(a, nred, nb, c->stream, A->nnz + 4L); break;
    }
    LSSP_HIP(hipGetLastError());
    return LSSP_AMD_OK;
}

// The block streams of k_spmv3, measured at upload.  Each XCD walks its
// 1/K of the rows in K/8 contiguous ranges; which K is fastest depends on the
// size (7-pt y = A x, ms, profiles/r06/r06f_spmv_streams.txt: 216^3 K = 8
// 0.145 vs 64 0.155; 256^3 8 0.282 vs 16 0.255; 288^3 8 0.415 vs 64 0.402;
// 320^3 8 0.557 vs 16 0.534) and no address rule we tried explained it
// (skewing each range's start did not, r06e), so matrices of >= 4 Mi rows
// time K = 8, 16, 32, 64 on three products each and keep the fastest unless
// K = 8 is within 2 %.  The product's values do not depend on K (every block
// writes its own rows and chunk partials).
int tune_spmv_streams(lssp_amd_ctx *c, lssp_amd_mat *A)
{
    A->streams = 0;
    if (spmv_streams_env() || A->nrows < (1 << 22) || A->d_win || A->nhalo > 0 || A->n_global != A->nrows)
        return LSSP_AMD_OK;
    double *x = nullptr, *z = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int st = LSSP_AMD_OK;
    auto run = [&]() -> int {
        LSSP_HIP(hipMalloc(&x, sizeof(double) * A->ncols));
        LSSP_HIP(hipMalloc(&z, sizeof(double) * A->nrows));
        LSSP_HIP(hipMemsetAsync(x, 0, sizeof(double) * A->ncols, c->stream));
        LSSP_HIP(hipEventCreate(&e0));
        LSSP_HIP(hipEventCreate(&e1));
        float best = 0.f, t8 = 0.f;
        int kbest = 8;
        for (int k : {8, 16, 32, 64}) {
            A->streams = k;
            LSSP_TRY(launch_spmv(c, A, EPI_MXY, 1.0, x, 0.0, nullptr, z, 0, nullptr, nullptr));
            LSSP_HIP(hipEventRecord(e0, c->stream));
            for (int r = 0; r < 3; r++) LSSP_TRY(launch_spmv(c, A, EPI_MXY, 1.0, x, 0.0, nullptr, z, 0, nullptr, nullptr));
            LSSP_HIP(hipEventRecord(e1, c->stream));
            LSSP_HIP(hipEventSynchronize(e1));
            float ms = 0.f;
            LSSP_HIP(hipEventElapsedTime(&ms, e0, e1));
            if (k == 8) best = t8 = ms;
            else if (ms < best) best = ms, kbest = k;
        }
        A->streams = best < 0.98f * t8 ? kbest : 8;
        return LSSP_AMD_OK;
    };
    st = run();
    if (st != LSSP_AMD_OK) A->streams = 0;
    (void)hipStreamSynchronize(c->stream);
    if (x) (void)hipFree(x);
    if (z) (void)hipFree(z);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    return st;
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
    EW_GMR_Z,      // out0 = v_{k-1}*y_{k-1}, then out0 = out0*1 + v_i*y_i, i = k-2 .. 0
                   // (solver-gmres.cxx:417-423, right-preconditioned GMRES); ym in u
    EW_LGM_X,      // t = sum_{i<min(k,mk)} v_i*y_i (+ sum_{i<nz} z_i*y_{mk+i} when k > mk);
                   // out0 += t; out1 = t  (solver-lgmres.cxx:224-251); ym in u, mk in sidx,
                   // nz in k >> 16, z basis in v (stride as vbase)
};

struct EwArgs {
    int kind;
    long n;
    double a, b;
    const double *x, *y, *u, *v;
    double *out0, *out1;
    const double *scal;
    const double *r0a, *r0b, *r1a, *r1b, *r2a, *r2b, *r3a, *r3b;
    const double *vbase;
    int k, sidx;
    double *part;
    long pcap;
    long nchunks;
    const double *guard;
};

template <int NRED>
__global__ __launch_bounds__(256) void k_ew(EwArgs g)
{
    __shared__ double lds[MAX_SLOTS][4];
    if (g.guard && *g.guard != 0.0) return;
    // grid-strided chunks (a contiguous range of chunks per workgroup measured
    // the same or slower: profiles/r04/r04c_stream_order.txt)
    for (long c = blockIdx.x; c < g.nchunks; c += gridDim.x) {
        const long i = c * 256 + threadIdx.x;
        const bool in = i < g.n;
        // the reduction operands: an output of this pass is read as the value just
        // computed (o0 / o1); any other operand is loaded up front, with the inputs
        // (the compiler may not move a load above the output stores it might alias)
        bool w0 = false, w1 = false;  // this element's out0 / out1 written by the kind below
        double o0 = 0.0, o1 = 0.0, p0a = 0.0, p0b = 0.0, p1a = 0.0, p1b = 0.0;
        double p2a = 0.0, p2b = 0.0, p3a = 0.0, p3b = 0.0;
        auto pre = [&](const double *q) { return (in && q != g.out0 && q != g.out1) ? q[i] : 0.0; };
        if (NRED > 0) {
            p0a = pre(g.r0a);
            p0b = pre(g.r0b);
            if (NRED > 1) {
                p1a = pre(g.r1a);
                p1b = pre(g.r1b);
            }
            if (NRED > 2) {
                p2a = pre(g.r2a);
                p2b = pre(g.r2b);
                p3a = g.r3a ? pre(g.r3a) : 0.0;
                p3b = g.r3b ? pre(g.r3b) : 0.0;
            }
        }
        if (in) {
            switch (g.kind) {
            case EW_FILL: w0 = true, g.out0[i] = o0 = g.a; break;
            case EW_COPY: w0 = true, g.out0[i] = o0 = g.x[i]; break;
            case EW_AXY: w0 = true, g.out0[i] = o0 = g.x[i] * g.a; break;
            case EW_AXPBY: w0 = true, g.out0[i] = o0 = g.out0[i] * g.b + g.x[i] * g.a; break;
            case EW_AXPBYZ: w0 = true, g.out0[i] = o0 = g.y[i] * g.b + g.x[i] * g.a; break;
            case EW_SCALE: w0 = true, g.out0[i] = o0 = g.out0[i] * g.a; break;
            case EW_DIVS: w0 = true, g.out0[i] = o0 = g.out0[i] / g.scal[g.sidx]; break;
            case EW_DOT: break;
            case EW_BICG_P: {
                const double beta = g.scal[S_BETA], omega = g.scal[S_OMEGA];
                w0 = true, g.out0[i] = o0 = g.x[i] + beta * (g.out0[i] - omega * g.y[i]);
                break;
            }
            case EW_BICG_S: w0 = true, g.out0[i] = o0 = g.x[i] - g.scal[S_ALPHA] * g.y[i]; break;
            case EW_BICG_XR: {
                const double alpha = g.scal[S_ALPHA];
                if (g.scal[S_BREAK] != 0.0) {
                    w0 = true, g.out0[i] = o0 = g.out0[i] + alpha * g.x[i];
                } else {
                    // every operand loaded before the first store (the compiler
                    // may not move u, v above a store to out0 they might alias)
                    const double omega = g.scal[S_OMEGA];
                    // x, ph, sh, s, t as non-temporal accesses (none is read again
                    // before the next iteration's sweeps have streamed through the
                    // caches; r, read by the next p pass, stays temporal): 216^3
                    // 632.3 -> 640.9 it/s, profiles/r05/r05x_xr_nt_ab.txt
                    const double xo = __builtin_nontemporal_load(g.out0 + i), xp = __builtin_nontemporal_load(g.x + i),
                                 xs = __builtin_nontemporal_load(g.y + i), su = __builtin_nontemporal_load(g.u + i),
                                 tv = __builtin_nontemporal_load(g.v + i);
                    w0 = true, o0 = xo + alpha * xp + omega * xs;
                    __builtin_nontemporal_store(o0, g.out0 + i);
                    w1 = true, g.out1[i] = o1 = su - omega * tv;
                }
                break;
            }
            case EW_CG_P: w0 = true, g.out0[i] = o0 = g.x[i] + g.scal[S_BETA] * g.out0[i]; break;
            case EW_CG_XR: {
                const double alpha = g.scal[S_ALPHA];
                w0 = true, g.out0[i] = o0 = g.out0[i] + alpha * g.x[i];
                w1 = true, g.out1[i] = o1 = g.out1[i] - alpha * g.y[i];
                break;
            }
            case EW_GM_MGS: w0 = true, g.out0[i] = o0 = g.out0[i] * 1 + g.x[i] * (-g.scal[g.sidx]); break;
            case EW_GM_X: {  // b carries the basis stride (vectors hold owned + halo entries)
                const long ld = (long)g.b;
                double acc = 0;
                for (int q = 0; q < g.k; q++) acc += g.vbase[(long)q * ld + i] * g.u[q];
                g.out0[i] += acc;
                break;
            }
            case EW_LGM_X: {
                const long ld = (long)g.b;
                const int kk = (short)(g.k & 0xffff), nz = g.k >> 16, mk = g.sidx;
                double t = 0;
                if (kk <= mk) {
                    for (int q = 0; q < kk; q++) t += g.vbase[(long)q * ld + i] * g.u[q];
                } else {
                    for (int q = 0; q < mk; q++) t += g.vbase[(long)q * ld + i] * g.u[q];
                    for (int q = 0; q < nz; q++) t += g.v[(long)q * ld + i] * g.u[q + mk];
                }
                g.out0[i] += t;
                w1 = true, g.out1[i] = o1 = t;
                break;
            }
            case EW_GMR_Z: {
                const long ld = (long)g.b;
                double z = g.vbase[(long)(g.k - 1) * ld + i] * g.u[g.k - 1];
                for (int q = g.k - 2; q >= 0; q--) z = z * 1 + g.vbase[(long)q * ld + i] * g.u[q];
                w0 = true, g.out0[i] = o0 = z;
                break;
            }
            }
        }
        if (NRED > 0) {
            double v[NRED > 0 ? NRED : 1];
            auto val = [&](const double *q, double pv) {
                if (q == g.out0 || q == g.out1) {  // an output: the value written, else memory
                    if (q == g.out1 && w1) return o1;
                    if (q == g.out0 && w0) return o0;
                    return q[i];
                }
                return pv;
            };
            v[0] = in ? val(g.r0a, p0a) * val(g.r0b, p0b) : 0.0;
            if (NRED > 1) v[NRED > 1 ? 1 : 0] = in ? val(g.r1a, p1a) * val(g.r1b, p1b) : 0.0;
            if (NRED > 2) {
                v[NRED > 2 ? 2 : 0] = in ? val(g.r2a, p2a) * val(g.r2b, p2b) : 0.0;
                v[NRED > 3 ? 3 : 0] = (in && g.r3a) ? val(g.r3a, p3a) * val(g.r3b, p3b) : 0.0;
            }
            chunk_reduce<NRED>(v, g.part, g.pcap, c, lds);
        }
    }
}

// lssp_vec_copy (vector.cxx:73-83) for 16-byte aligned vectors: four 16-byte
// loads per lane in flight, then the four stores (grid-strided).  It is also
// what bench.py prices HBM with (roofline peak_measured).
typedef double line_dbl2v __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_copy16(const line_dbl2v *__restrict__ s2, line_dbl2v *__restrict__ d2, long n2)
{
    typedef line_dbl2v dbl2v;
    const long stride = (long)gridDim.x * 256;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n2; i += 4 * stride) {
        dbl2v v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) v[u] = i + u * stride < n2 ? __builtin_nontemporal_load(s2 + i + u * stride) : dbl2v{0, 0};
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (i + u * stride < n2) __builtin_nontemporal_store(v[u], d2 + i + u * stride);
    }
}

// Streaming read (the HBM read roofline the bench quotes beside the 8 TB/s
// spec): every word read once by 16-byte non-temporal loads, XOR-folded into
// *sink (64-bit, one atomic per workgroup) so the loads cannot be dropped and
// the result is checkable.  Each workgroup streams its OWN contiguous chunk
// (8 loads in flight per lane): 7.0-7.1 TB/s over 1 GiB, against 5.3-6.3 for
// the same loads grid-strided, where all CUs walk one narrow window of the
// address space (tools/probe/read_probe.hip, profiles/r04/r04a_read_probe.txt).
__global__ __launch_bounds__(256) void k_read16(const line_dbl2v *__restrict__ s2, long n2,
                                               unsigned long long *sink)
{
    typedef unsigned long long u64;
    constexpr int U = 8;
    const long per = (n2 + gridDim.x - 1) / gridDim.x;
    const long b0 = (long)blockIdx.x * per, b1 = b0 + per < n2 ? b0 + per : n2;
    u64 acc = 0;
    for (long i = b0 + threadIdx.x; i < b1; i += U * 256) {
        line_dbl2v v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = i + u * 256 < b1 ? __builtin_nontemporal_load(s2 + i + u * 256)
                                                            : line_dbl2v{0, 0};
#pragma unroll
        for (int u = 0; u < U; u++) acc ^= (u64)__double_as_longlong(v[u][0]) ^ (u64)__double_as_longlong(v[u][1]);
    }
    for (int o = 32; o >= 1; o >>= 1) acc ^= __shfl_xor(acc, o);
    __shared__ u64 w[4];
    if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) atomicXor(sink, w[0] ^ w[1] ^ w[2] ^ w[3]);
}

int launch_stream_read(lssp_amd_ctx *c, const double *x, long n, double *sink)
{
    LSSP_HIP(hipMemsetAsync(sink, 0, sizeof(double), c->stream));
    const long n2 = n / 2;  // n even, x 16-byte aligned (lssp_amd_stream_read)
    unsigned long long *s = reinterpret_cast<unsigned long long *>(sink);
    if (n2 > 0) {
        const long grid = std::max<long>(1, std::min<long>((n2 + 2047) / 2048, 16L * c->num_cus));
        k_read16<<<grid, 256, 0, c->stream>>>(reinterpret_cast<const line_dbl2v *>(x), n2, s);
        LSSP_HIP(hipGetLastError());
    }
    return LSSP_AMD_OK;
}

int launch_copy(lssp_amd_ctx *c, double *x, const double *y, long n)
{
    if (n <= 0) return LSSP_AMD_OK;
    const bool al = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) == 0;
    if (!al || c->guard) {
        Ew e;
        e.kind = EW_COPY;
        e.n = n;
        e.x = y;
        e.out0 = x;
        return launch_ew(c, e);
    }
    const long n2 = n / 2;
    if (n2 > 0) {
        const long grid = std::min<long>((n2 + 1023) / 1024, 8L * c->num_cus * 4);
        k_copy16<<<grid, 256, 0, c->stream>>>(reinterpret_cast<const line_dbl2v *>(y), reinterpret_cast<line_dbl2v *>(x),
                                              n2);
        LSSP_HIP(hipGetLastError());
    }
    if (n & 1) LSSP_HIP(hipMemcpyAsync(x + n - 1, y + n - 1, sizeof(double), hipMemcpyDeviceToDevice, c->stream));
    return LSSP_AMD_OK;
}

int launch_ew(lssp_amd_ctx *c, const Ew &e)
{
    if (e.n <= 0) return LSSP_AMD_OK;
    long C = num_chunks(e.n);
    LSSP_TRY(ensure_part(c, C));
    EwArgs g{e.kind, e.n, e.a, e.b, e.x, e.y, e.u, e.v, e.out0, e.out1, e.scal,
             e.r0a, e.r0b, e.r1a, e.r1b, e.r2a, e.r2b, e.r3a, e.r3b, e.vbase, e.k, e.sidx,
             c->d_part + (long)e.pslot * c->part_cap, c->part_cap, C,
             c->guard};
    // one chunk per block up to a cap; the cap keeps >= 8 blocks per CU resident
    long grid = C < 8L * c->num_cus * 4 ? C : 8L * c->num_cus * 4;
    if (e.nred == 0) k_ew<0><<<grid, 256, 0, c->stream>>>(g);
    else if (e.nred == 1) k_ew<1><<<grid, 256, 0, c->stream>>>(g);
    else if (e.nred == 2) k_ew<2><<<grid, 256, 0, c->stream>>>(g);
    else k_ew<4><<<grid, 256, 0, c->stream>>>(g);  // 3 or 4 (r3a == nullptr: slot 3 sums zeros)
    LSSP_HIP(hipGetLastError());
    return LSSP_AMD_OK;
}

// CG (PC_NON, one rank, tree reductions) with the level 2 of the reduction
// before a vector update folded into that update: every 1024-thread
// workgroup redoes k_reduce2m's level 2 over the C partials at pin (lane t adds
// partials t, t+1024, ... onto 0.0, 16 halving waves, the 16 wave sums halved:
// the same order and sum on every workgroup), derives the scalar its update
// needs exactly as finalize does, and workgroup 0 alone runs the finalize
// program (scalars, trace, residual history, stop flag).  This removes the
// dependent level-2 launch between the reduction's producer and its consumer.
//   CGF_XR: alpha = rho1 / (q.p) [FIN_CG_ALPHA]; x += alpha p, r -= alpha q,
//           r.r partials -> pout (solver-cg.cxx:96-104)
//   CGF_P:  beta = (r.r) / rho0 [FIN_CG_RES_RHO(_B)]; when the stop test
//           (:109) holds no workgroup updates p; else p = r + beta p (:88-92)
//   CGF_R:  CGF_XR without x (3 vectors instead of 6); CGF_PX: CGF_P that
//           first adds the previous alpha p to x (also when the stop test
//           holds) -- p is read once for both; CGF_X: that x update alone (a
//           batch's last iteration).  x gets the same operands in the same
//           order, one pass later: every value is unchanged.  The stop test
//           writes S_DONE = its iteration's stamp, so the pass that finds it
//           still applies its x update while any later pass returns.
// pin and pout are different partial rows: a workgroup still reading pin
// never races another one writing its chunk partials.
struct CgFusedArgs {
    int kind, stamp;
    long n, C;
    double *x, *p, *r;
    const double *z, *q;
    const double *pin;
    double *pout;
    double *sums, *scal, *trace;
    Fin f;
    const double *guard;
};

// lane l's double, uniform (two v_readlane)
__device__ __forceinline__ double lane_bcast(double v, int l)
{
    const long long b = __double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Every global read a workgroup makes before its first store is issued up
// front, ahead of the guard test: the guard, the scalars, the level-2
// partials and the first element's operands (the element loop then loads one
// element ahead).  A pass starts streaming after one memory round trip instead
// of three dependent ones (guard -> partials -> scalars -> operands).
template <int KIND>
__global__ __launch_bounds__(1024) void k_cg_fused(CgFusedArgs a)
{
    __shared__ double wl[16];
    __shared__ double red[2][4][4];
    __shared__ double sc[2];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int kind = KIND;
    const long stride = gridDim.x * 1024L, n = a.n;
    // operands of element i: PX p x z, P p z, R q r, XR q r x p, X x p
    auto load = [&](long i, double (&v)[4]) {
        if (i >= n) return;
        if constexpr (kind == CGF_R || kind == CGF_XR) {
            v[0] = a.q[i];
            v[1] = a.r[i];
            if (kind == CGF_XR) v[2] = a.x[i], v[3] = a.p[i];
        } else {
            v[0] = a.p[i];
            if (kind != CGF_P) v[1] = a.x[i];
            if (kind != CGF_X) v[2] = a.z[i];
        }
    };
    // the scalars and the guard by ONE vector load (lane l reads its own
    // address): scalar loads would share the kernel arguments' lgkmcnt waits
    // and delay the operand loads behind their round trip
    const double *sp = a.scal + (lane == 0 ? S_ALPHA : lane == 1 ? S_RHO1 : lane == 2 ? S_RHO0 : S_TOL);
    if (lane == 4 && a.guard) sp = a.guard;
    const double sv = *sp;
    double cur[4] = {0.0, 0.0, 0.0, 0.0};
    long i = blockIdx.x * 1024L + tid;
    load(i, cur);
    double acc = 0.0;
    if (kind != CGF_X) {
        // lane t adds partials t, t+1024, ... in order; the loads of 8 of them
        // are issued before the adds (k_reduce2m's form)
        for (long k0 = tid; k0 < a.C; k0 += 8L * L2_LANES) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const long k = k0 + (long)u * L2_LANES;
                v[u] = k < a.C ? a.pin[k] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 8; u++)
                if (k0 + (long)u * L2_LANES < a.C) acc += v[u];
        }
    }
    const double al = lane_bcast(sv, 0), rho1 = lane_bcast(sv, 1), rho0 = lane_bcast(sv, 2),
                 tolv = lane_bcast(sv, 3), gv = a.guard ? lane_bcast(sv, 4) : 0.0;
    // a batched iteration past the stop; the stop's own pass keeps its x update
    if (gv != 0.0 && gv != (double)a.stamp) return;
    if (kind == CGF_X) {  // the batch's deferred x update alone
        for (; i < n; i += stride) {
            double nx[4];
            load(i + stride, nx);
            a.x[i] = cur[1] + al * cur[0];
#pragma unroll
            for (int u = 0; u < 4; u++) cur[u] = nx[u];
        }
        return;
    }
    {
        acc = wave_sum(acc);
        if (lane == 0) wl[wave] = acc;
        __syncthreads();
        if (tid == 0) {
            double u[16];
#pragma unroll
            for (int w = 0; w < 16; w++) u[w] = wl[w];
#pragma unroll
            for (int off = 8; off >= 1; off >>= 1)
#pragma unroll
                for (int l = 0; l < off; l++) u[l] = u[l] + u[l + off];
            const double s = u[0];
            double v;
            bool stop = false;
            if (kind == CGF_XR || kind == CGF_R) {
                v = rho1 / s;  // finalize FIN_CG_ALPHA's alpha (S_RHO1 is not written below)
            } else {
                v = s / rho0;  // FIN_CG_RES_RHO's beta (S_RHO0 is not written below)
                stop = a.f.op == FIN_CG_RES_RHO_B && sqrt(s) <= tolv;
            }
            if (blockIdx.x == 0) {
                a.sums[0] = s;
                finalize(a.f, &s, a.scal, a.trace);
            }
            sc[0] = v;
            sc[1] = stop ? 1.0 : 0.0;
        }
        __syncthreads();
    }
    const bool stop = sc[1] != 0.0;
    const double v = sc[0];
    if (kind == CGF_PX) {  // x += alpha p of the previous x/r pass (CGF_R), then p = r + beta p
        // (workgroup 0's finalize does not write S_ALPHA)
        for (; i < n; i += stride) {
            double nx[4];
            load(i + stride, nx);
            const double pv = cur[0];
            a.x[i] = cur[1] + al * pv;
            if (!stop) a.p[i] = cur[2] + v * pv;
#pragma unroll
            for (int u = 0; u < 4; u++) cur[u] = nx[u];
        }
        return;
    }
    if (stop) return;
    int par = 0;
    for (long g = blockIdx.x; g * 1024 < n; g += gridDim.x, par ^= 1, i += stride) {
        double nx[4];
        load(i + stride, nx);
        if (kind == CGF_P) {
            if (i < n) a.p[i] = cur[2] + v * cur[0];
        } else {
            double rr = 0.0;
            if (i < n) {
                if (kind == CGF_XR) a.x[i] = cur[2] + v * cur[3];
                const double rn = cur[1] - v * cur[0];
                a.r[i] = rn;
                rr = rn * rn;
            }
            // chunk_reduce's order for the 4 chunks of this 1024-element group
            const double w = wave_sum(rr);
            if (lane == 0) red[par][wave >> 2][wave & 3] = w;
            __syncthreads();
            const long chunk = g * 4 + (tid >> 8);
            if ((tid & 255) == 0 && chunk * 256 < n) {
                const int cq = tid >> 8;
                a.pout[chunk] = (red[par][cq][0] + red[par][cq][1]) + (red[par][cq][2] + red[par][cq][3]);
            }
        }
#pragma unroll
        for (int u = 0; u < 4; u++) cur[u] = nx[u];
    }
}

int launch_cg_fused(lssp_amd_ctx *c, int kind, long n, double *x, double *p, double *r, const double *z,
                    const double *q, int pin_slot, int pout_slot, const Fin &f, int stamp)
{
    if (n <= 0) return LSSP_AMD_OK;
    const long C = num_chunks(n);
    LSSP_TRY(ensure_part(c, C));
    CgFusedArgs g{kind, stamp, n, C, x, p, r, z, q, c->d_part + pin_slot * c->part_cap,
                  c->d_part + pout_slot * c->part_cap, c->d_sums, c->d_scal, c->d_trace, f, c->guard};
#ifndef CGF_PER_CU
#define CGF_PER_CU 2  // tuning builds override it
#endif
    const long grid = std::min<long>((n + 1023) / 1024, (long)CGF_PER_CU * c->num_cus);  // 2 per CU
    switch (kind) {
    case CGF_P: k_cg_fused<CGF_P><<<grid, 1024, 0, c->stream>>>(g); break;
    case CGF_XR: k_cg_fused<CGF_XR><<<grid, 1024, 0, c->stream>>>(g); break;
    case CGF_R: k_cg_fused<CGF_R><<<grid, 1024, 0, c->stream>>>(g); break;
    case CGF_PX: k_cg_fused<CGF_PX><<<grid, 1024, 0, c->stream>>>(g); break;
    default: k_cg_fused<CGF_X><<<grid, 1024, 0, c->stream>>>(g); break;
    }
    LSSP_HIP(hipGetLastError());
    return LSSP_AMD_OK;
}

int launch_reduce_tree(lssp_amd_ctx *c, long C, int nslot, const Fin &f, int slot0)
{
    int do_fin = c->nranks > 1 ? 0 : 1;
    static_assert(L2_LANES == 16 * 64, "k_reduce2m runs the 16 waves of the level-2 workgroup");
    k_reduce2m<<<L2_LANES / 64, 64, 0, c->stream>>>(c->d_part + slot0 * c->part_cap, c->part_cap, C, nslot,
                                                         c->d_sums, c->d_scal,
                                                         c->d_trace, f, do_fin, c->d_wsum, c->d_rcnt, c->guard);
    LSSP_HIP(hipGetLastError());
    return LSSP_AMD_OK;
}

int launch_reduce_serial(lssp_amd_ctx *c, long n, int nslot, const double *const *a,
                         const double *const *b, const Fin &f, const double *carry)
{
    SerialArgs g{};
    for (int s = 0; s < nslot; s++) {
        g.a[s] = a[s];
        g.b[s] = b[s];
    }
    int do_fin = c->nranks > 1 ? 0 : 1;
    k_dot_serial<<<1, 1024, 0, c->stream>>>(g, n, nslot, c->d_sums, c->d_scal, c->d_trace, f, do_fin, carry,
                                            c->guard);
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
                                         c->d_trace, f, c->reduce_mode == LSSP_AMD_REDUCE_SERIAL, c->guard);
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
