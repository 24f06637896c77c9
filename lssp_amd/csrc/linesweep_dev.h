// linesweep_dev.h -- device helpers shared by the line sweeps (linesweep.hip:
// k_line, k_line2 for ILU(0); linefill.hip: k_linef for the 7-point ILU(1)
// pattern): LDS-DMA issue, the workgroup barrier, agent-scope hand-off loads,
// lane selects, DPP row shifts and the lane - 16 shuffle.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "internal.h"

namespace lssp_amd {

__device__ __forceinline__ void dma16(const void *g, unsigned lds)
{
    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(lds) : "memory", "m0");
}
__device__ __forceinline__ void dma16_nt(const void *g, unsigned lds)
{
    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off nt" ::"v"(g), "s"(lds) : "memory", "m0");
}
__device__ __forceinline__ void dma16_sc1(const void *g, unsigned lds)
{
    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off sc1" ::"v"(g), "s"(__builtin_amdgcn_readfirstlane(lds))
                 : "memory", "m0");
}
// LDS drained, then the workgroup barrier.  The wait is the builtin (not asm),
// so the compiler's wait-count tracking knows every LDS load is complete after
// it and does not re-wait for loads issued before the barrier; the empty asm
// statements keep memory operations from moving across.
__device__ __forceinline__ void line_barrier()
{
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xc07f);  // gfx9: lgkmcnt(0), vmcnt/expcnt unconstrained
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ uint64_t line_ld_agent(const double *p)
{
    return __hip_atomic_load(reinterpret_cast<const uint64_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void line_st_agent(double *p, double v)
{
    uint64_t b = (uint64_t)__double_as_longlong(v);
    if (b == TRI_SENTINEL) b = 0x7FF8000000000000ull;  // never publish the flag pattern as a value
    __hip_atomic_store(reinterpret_cast<uint64_t *>(p), b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// per lane: bit lane of m ? t : f, as two v_cndmask (the compiler cannot turn an
// asm select into a branch around the division that produced t)
__device__ __forceinline__ double sel_lanes(uint64_t m, double t, double f)
{
    const long long tb = __double_as_longlong(t), fb = __double_as_longlong(f);
    int lo, hi;
    asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(lo) : "v"((int)fb), "v"((int)tb), "s"(m));
    asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(hi) : "v"((int)(fb >> 32)), "v"((int)(tb >> 32)), "s"(m));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
typedef unsigned int line_v2u __attribute__((ext_vector_type(2)));
typedef unsigned int line_v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ line_v2u split64(uint64_t b)
{
    line_v2u d;
    d.x = (unsigned)b;
    d.y = (unsigned)(b >> 32);
    return d;
}

__device__ __forceinline__ double dpp_shr1(double v, double old)
{
    const long long b = __double_as_longlong(v), o = __double_as_longlong(old);
    const int lo = __builtin_amdgcn_update_dpp((int)o, (int)b, 0x138, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(b >> 32), 0x138, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// the previous line's value within each lane group; a group's line 0 gets old
// (G = 4: the groups are the DPP rows, row_shr:1 leaves lane 0 of a row alone)
template <int G>
__device__ __forceinline__ double dpp_shr1g(double v, double old)
{
    if constexpr (G == 4) {
        const long long b = __double_as_longlong(v), o = __double_as_longlong(old);
        const int lo = __builtin_amdgcn_update_dpp((int)o, (int)b, 0x111, 0xf, 0xf, false);
        const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(b >> 32), 0x111, 0xf, 0xf, false);
        return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
    } else if constexpr (G == 2) {
        return sel_lanes(1ull << 32, old, dpp_shr1(v, old));
    } else {
        return dpp_shr1(v, old);
    }
}

// the canonical level-1 halving tree of one wave (kernels.hip wave_sum): lane 0
// holds the result
__device__ __forceinline__ double wave_sum_d(double v)
{
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = v + __shfl_xor(v, off, 64);
    return v;
}

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F &&f)
{
    if constexpr (I < N) {
        f(std::integral_constant<int, I>());
        static_for<I + 1, N>(f);
    }
}

// lane l <- lane l - 16 (rows R0..R3 of the wave -> [R0, R0, R1, R2]; row 0 is
// not used): v_permlane16_swap gives [R0, R0, R2, R2] / [R1, R1, R3, R3],
// v_permlane32_swap of those [R0, R0, R1, R1]; rows 1 and 3 from the first,
// row 2 from the second (tools/probe/shfl_probe.hip checks it against ds_bpermute)
// ds_bpermute is the default: 93 against 133 clk per dependent shuffle + f64
// mul/add (profiles/r04/r04a_shfl_probe.txt); -DLINE2_PERMLANE selects the swaps
__device__ __forceinline__ unsigned up16_u32(unsigned x)
{
#ifndef LINE2_PERMLANE
    return (unsigned)__builtin_amdgcn_ds_bpermute((int)(((threadIdx.x & 63) - 16) & 63) * 4, (int)x);
#else
    auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    auto q = __builtin_amdgcn_permlane32_swap(r[0], r[1], false, false);
    unsigned o;
    asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(o) : "v"(r[0]), "v"(q[0]), "s"(0x0000FFFF00000000ull));
    return o;
#endif
}
__device__ __forceinline__ double up16(double v)
{
    const long long b = __double_as_longlong(v);
    const unsigned lo = up16_u32((unsigned)b), hi = up16_u32((unsigned)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | lo);
}

// The product z = op(A x) on the output x of a U sweep, run by the sweep's
// own workgroups once the tile claims are exhausted (launch_line_apply_spmv):
// a workgroup that finds no tile left turns its 11 waves into product waves,
// each claiming whole 256-row reduction chunks from the top of the matrix down
// (the U sweep completes planes in that order) and starting a chunk once every
// plane its rows read (k-1 .. k+1, a 5-/7-point stencil of the sweep's grid)
// is final: the U tiles count their completion per tile row (kdone, agent-
// scope atomics after the storers' write-through stores drained).  Lane l of
// a wave owns rows 64q + l (q = 0..3) of its chunk, forms each row's sum in
// CSR order from 0.0 and the epilogue of k_spmv3, and the chunk's fused-dot
// partials are (w0 + w1) + (w2 + w3) of the four 64-row wave sums -- exactly
// chunk_reduce's order -- so every output and partial is bitwise k_spmv3's.
// Only CUs whose sweep work is over run product waves: the hand-off polls of
// the tiles still running do not queue behind product loads.
struct LineTail {
    const int *Ap;
    const double *Ax;
    const uint8_t *Ad;  // diagonal-id coding (lssp_amd_mat::Ad)
    const int *off;
    int ndiag, nrows, epi, nred;
    const double *y;
    double *z;
    double alpha, beta;
    const double *w0, *w1;
    double *part;
    long pcap, nblk, cend;      // chunks [cend - nblk, cend)
    unsigned long long *claim;  // chunk claims (monotonic)
    unsigned long long base;
    unsigned *kdone;            // U tiles finished per tile row (monotonic)
    unsigned ktarget;           // this launch's count per row (W x launches)
    const int *kof;             // natural plane -> L tile row
    int S, W, nz;
    long pl;                    // rows per plane
    unsigned *dbg;              // LSSP_AMD_TAIL_DIAG: progress words in mapped host memory (diagnostics)
};

__device__ __forceinline__ double ld_sc1d(const double *p)
{
    return __longlong_as_double(
        (long long)__hip_atomic_load(reinterpret_cast<const uint64_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_sc1d(double *p, double v)
{
    __hip_atomic_store(reinterpret_cast<uint64_t *>(p), (uint64_t)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// one wave's share of the tail product (see LineTail); soff: the offset table in LDS
// LDS of the tail: the offset table (<= 255 ints) in the first 1 KB, then
// per wave a TAIL_LDS-byte region: a 64-row group's values (TAIL_CAP + 2
// doubles) and diagonal ids (TAIL_CAP + 32 bytes), staged with coalesced
// 16-byte loads (per-lane row loads cost the texture unit one cache line per
// lane per entry: the first version of this tail took 400 us per product)
constexpr int TAIL_CAP = 448;  // entries of a 64-row group staged (7 per row)
constexpr int TAIL_LDS = 4096;
constexpr int TAIL_LDS_BYTES(int nwaves) { return 1024 + nwaves * TAIL_LDS; }
static __device__ void line_tail_waves(const LineTail &T, const double *x, int *err, char *smem)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int *soff = reinterpret_cast<const int *>(smem);
    double *sx = reinterpret_cast<double *>(smem + 1024 + wave * TAIL_LDS);
    uint8_t *sd = reinterpret_cast<uint8_t *>(smem + 1024 + wave * TAIL_LDS + 8 * (TAIL_CAP + 2));
    typedef double d2_t __attribute__((ext_vector_type(2)));
    typedef int i4_t __attribute__((ext_vector_type(4)));
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        unsigned long long c = 0;
        if (lane == 0) c = atomicAdd(T.claim, 1ull) - T.base;
        const unsigned clo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)c);
        const unsigned chi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(c >> 32));
        const unsigned long long cl = ((unsigned long long)chi << 32) | clo;
        unsigned *dw = T.dbg ? T.dbg + 1024 + 4 * (blockIdx.x * 16 + wave) : nullptr;
        if (dw && lane == 0) {
            dw[0] = 1;
            dw[1] = (unsigned)cl;
        }
        if (cl >= (unsigned long long)T.nblk) {
            if (dw && lane == 0) dw[0] = 9;
            break;
        }
        const long blk = T.cend - 1 - (long)cl;
        const int r0 = (int)(blk * 256), r1 = min(r0 + 256, T.nrows);
        // the planes the chunk's rows read: k-1 .. k+1 of its first / last row
        if (lane == 0) {
            const int ka = max(r0 / (int)T.pl - 1, 0), kb = min((r1 - 1) / (int)T.pl + 1, T.nz - 1);
            const int K0 = T.kof[ka], K1 = T.kof[kb];
            for (int K = K0; K <= K1; K++) {
                unsigned *cnt = T.kdone + (T.S - 1 - K);  // U tile row of L tile row K
                for (;;) {
                    // (an atomic read: coherent with the tiles' atomic increments on every XCD)
                    const unsigned seen = __hip_atomic_fetch_add(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (dw) {
                        dw[2] = (unsigned)K;
                        dw[3] = seen;
                    }
                    if (seen - T.ktarget < 0x80000000u) break;
                    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
                        __builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) {  // 4 s: the sweep gave up
                        atomicOr(err, 8);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (dw && lane == 0) dw[0] = 2;
        double v0[4], v1[4];
        for (int q = 0; q < 4; q++) {
            const int rg = r0 + 64 * q;  // the group's first row
            v0[q] = v1[q] = 0.0;
            if (rg >= T.nrows) continue;  // (uniform)
            const int r = rg + lane, rr = min(r, T.nrows - 1);
            const int rb = T.Ap[rr], re = T.Ap[rr + 1];
            const int e0 = __builtin_amdgcn_readfirstlane(rb);
            const int e1 = __shfl(re, 63, 64);  // the group's last entry + 1
            double sum = 0;
            if (e1 - e0 <= TAIL_CAP) {  // (uniform) stage the group's values and ids
                const int xb = e0 & ~1, db = e0 & ~15;
                const int nv = (e1 - xb + 1) >> 1, nd = (e1 - db + 15) >> 4;
                const d2_t *X2 = reinterpret_cast<const d2_t *>(T.Ax) + (xb >> 1);
                const i4_t *D4 = reinterpret_cast<const i4_t *>(T.Ad) + (db >> 4);
                d2_t vx[4];
                i4_t vd;
#pragma unroll
                for (int u = 0; u < 4; u++) vx[u] = __builtin_nontemporal_load(X2 + min(lane + 64 * u, nv - 1));
                vd = __builtin_nontemporal_load(D4 + min(lane, nd - 1));
#pragma unroll
                for (int u = 0; u < 4; u++)
                    if (lane + 64 * u < nv) reinterpret_cast<d2_t *>(sx)[lane + 64 * u] = vx[u];
                if (lane < nd) reinterpret_cast<i4_t *>(sd)[lane] = vd;
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                double pr[8];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int k = max(min(rb + u, re - 1), 0);
                    pr[u] = ld_sc1d(x + rr + soff[sd[k - db]]) * sx[k - xb];
                }
#pragma unroll
                for (int u = 0; u < 8; u++)
                    if (u < re - rb) sum += pr[u];
                for (int k = rb + 8; k < re; k++) sum += ld_sc1d(x + rr + soff[sd[k - db]]) * sx[k - xb];
                __builtin_amdgcn_wave_barrier();  // the region is rewritten by the next group
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            } else {
                for (int k = rb; k < re; k++) sum += ld_sc1d(x + rr + soff[T.Ad[k]]) * T.Ax[k];
            }
            if (r < T.nrows) {
                double zv;
                if (T.epi == EPI_MXY) zv = sum;
                else if (T.epi == EPI_AMXY) zv = sum * T.alpha;
                else if (T.epi == EPI_AXPBY) zv = ld_sc1d(T.y + r) * T.beta + T.alpha * sum;
                else zv = T.alpha * sum;
                T.z[r] = zv;
                if (T.nred > 0) v0[q] = zv * (T.w0 == T.z ? zv : ld_sc1d(T.w0 + r));
                if (T.nred > 1) v1[q] = zv * (T.w1 && T.w1 != T.z ? ld_sc1d(T.w1 + r) : zv);
            }
        }
        // chunk_reduce's order: the four 64-row groups' halving trees, (w0 + w1) + (w2 + w3)
        if (T.nred > 0) {
            double w[4];
#pragma unroll
            for (int q = 0; q < 4; q++) w[q] = wave_sum_d(v0[q]);
            if (lane == 0) T.part[blk] = (w[0] + w[1]) + (w[2] + w[3]);
        }
        if (T.nred > 1) {
            double w[4];
#pragma unroll
            for (int q = 0; q < 4; q++) w[q] = wave_sum_d(v1[q]);
            if (lane == 0) T.part[T.pcap + blk] = (w[0] + w[1]) + (w[2] + w[3]);
        }
    }
}

}  // namespace lssp_amd
