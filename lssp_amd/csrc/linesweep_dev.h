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
    const int *Aj;              // int32 columns (rows past the staging cap)
    long nnz_pad;               // Ax / Aj padded length (launch_spmv: nnz + 4)
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

// The tail product, workgroup-wide: every round the workgroup claims a PAIR of
// 256-row chunks (threads 0..255 and 256..511 each run one as k_spmv3 runs a
// block; the other waves only take part in the barriers).  The next pair's
// staging loads (row bounds, the chunk's value and id ranges as 16-byte
// vectors, the fused dots' operands -- none of them written by the sweep) are
// in flight while the current pair's x gathers run, so a round costs about one
// memory round trip; only the x gathers wait for the planes to be final.  LDS:
// the offset table (1 KB), two sync words, then two buffers x two chunks of
// TAIL_CH bytes.  (A first version with one 64-row group per wave and three
// dependent round trips per group moved ~80 rows/us per CU and made the
// product slower than k_spmv3: profiles/r05/r05c_tail_ab.txt.)
constexpr int TAIL_CAP = 2048;                                   // staged entries per chunk (k_spmv3's SPMV_CAP)
constexpr int TAIL_SX = 8 * (TAIL_CAP + 2);                      // values
constexpr int TAIL_SD = 4 * (TAIL_CAP / 4 + 8);                  // diagonal ids
constexpr int TAIL_CH = (TAIL_SX + TAIL_SD + 8 * 4 * 4 + 15) / 16 * 16;
constexpr int TAIL_LDS_BYTES(int) { return 1024 + 64 + 4 * TAIL_CH; }
static __device__ void line_tail_wg(const LineTail &T, const double *x, int *err, char *smem)
{
    typedef double d2_t __attribute__((ext_vector_type(2)));
    typedef int i4_t __attribute__((ext_vector_type(4)));
    constexpr int NX2 = (TAIL_CAP / 2 + 1 + 255) / 256;  // 16-byte value loads per thread
    const int tid = threadIdx.x, c = tid >> 8, t = tid & 255;
    const bool act = tid < 512;
    const int *soff = reinterpret_cast<const int *>(smem);
    unsigned *sync = reinterpret_cast<unsigned *>(smem + 1024);
    auto buf = [&](int b) { return smem + 1088 + (2 * b + c) * TAIL_CH; };
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    // the staged state of one chunk (registers)
    struct St {
        long blk;
        int r, rr, rb, re, base, cnt;
        long xb, jb;
        d2_t vx[NX2];
        i4_t vj;
        double w0p, w1p;
    };
    auto claim = [&]() {  // thread 0: the next pair's first chunk index (relative to base)
        const unsigned long long cl = atomicAdd(T.claim, 2ull) - T.base;
        sync[0] = (unsigned)cl;
        sync[1] = (unsigned)(cl >> 32);
    };
    auto read_claim = [&]() { return ((unsigned long long)sync[1] << 32) | sync[0]; };
    auto stage = [&](unsigned long long cl, St &S) {  // loads only; nothing here waits for the sweep
        S.blk = cl + c < (unsigned long long)T.nblk ? T.cend - 1 - (long)(cl + c) : -1;
        if (!act || S.blk < 0) return;
        const int r0 = (int)(S.blk * 256);
        S.r = r0 + t;
        const int rend = min(r0 + 256, T.nrows);
        S.base = T.Ap[r0];
        S.cnt = T.Ap[rend] - S.base;
        S.rr = min(S.r, T.nrows - 1);
        S.rb = T.Ap[S.rr];
        S.re = T.Ap[S.rr + 1];
        S.w0p = S.w1p = 0.0;
        if (T.nred > 0 && T.w0 != T.z) S.w0p = ld_sc1d(T.w0 + S.rr);
        if (T.nred > 1 && T.w1 && T.w1 != T.z) S.w1p = ld_sc1d(T.w1 + S.rr);
        if (S.cnt <= TAIL_CAP) {
            S.xb = S.base & ~1L;
            S.jb = S.base & ~15L;
            const long last = S.cnt > 0 ? (long)S.base + S.cnt - 1 : (long)S.base;
            const long xmax = min(last >> 1, (T.nnz_pad >> 1) - 1);
            const long jmax = min(last >> 4, ((T.nnz_pad - 4 + 32) >> 4) - 1);
            const d2_t *X2 = reinterpret_cast<const d2_t *>(T.Ax);
            const i4_t *J4 = reinterpret_cast<const i4_t *>(T.Ad);
#pragma unroll
            for (int u = 0; u < NX2; u++) S.vx[u] = __builtin_nontemporal_load(X2 + min((S.xb >> 1) + t + 256 * u, xmax));
            S.vj = __builtin_nontemporal_load(J4 + min((S.jb >> 4) + t, jmax));
        }
    };
    auto land = [&](const St &S, int b) {  // the staged vectors into this chunk's LDS buffer
        if (!act || S.blk < 0 || S.cnt > TAIL_CAP) return;
        char *B = buf(b);
        const long last = S.cnt > 0 ? (long)S.base + S.cnt - 1 : (long)S.base;
        const int xn = (int)(min(last >> 1, (T.nnz_pad >> 1) - 1) - (S.xb >> 1)) + 1;
        const int jn = (int)(min(last >> 4, ((T.nnz_pad - 4 + 32) >> 4) - 1) - (S.jb >> 4)) + 1;
#pragma unroll
        for (int u = 0; u < NX2; u++)
            if (t + 256 * u < xn) reinterpret_cast<d2_t *>(B)[t + 256 * u] = S.vx[u];
        if (t < jn) reinterpret_cast<i4_t *>(B + TAIL_SX)[t] = S.vj;
    };
    // thread 0: the pair's rows read final planes only.  U tile rows Kp = S-1-K
    // complete (nearly) in increasing Kp, and the pairs come from the top down,
    // so thread 0 keeps the prefix of rows it has seen complete (kp_done) and
    // asks the counters only about rows past it
    int kp_done = -1;
    auto wait_planes = [&](unsigned long long cl) {
        if (cl >= (unsigned long long)T.nblk) return;
        const long hi = T.cend - 1 - (long)cl;                                   // upper chunk
        const long lo = T.cend - 1 - (long)min(cl + 1, (unsigned long long)T.nblk - 1);
        const int r0 = (int)(lo * 256), r1 = min((int)(hi * 256) + 256, T.nrows);
        const int ka = max(r0 / (int)T.pl - 1, 0), kb = min((r1 - 1) / (int)T.pl + 1, T.nz - 1);
        const int kpb = T.S - 1 - T.kof[ka];  // the highest U tile row needed
        for (int Kp = kp_done + 1; Kp <= kpb; Kp++) {
            unsigned *cnt = T.kdone + Kp;
            for (;;) {
                // (an atomic read: coherent with the tiles' atomic increments on every XCD)
                const unsigned seen = __hip_atomic_fetch_add(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (seen - T.ktarget < 0x80000000u) break;
                if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
                    __builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) {  // 4 s: the sweep gave up
                    atomicOr(err, 8);
                    return;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            kp_done = Kp;
        }
    };
    St A, Bs;
    // pairs are claimed two rounds ahead (a returning atomic costs ~1 us under
    // load); every workgroup ends on exactly one failed claim
    if (tid == 0) {
        claim();
        if (read_claim() < (unsigned long long)T.nblk) {
            const unsigned long long c0 = read_claim();
            claim();
            sync[2] = sync[0];
            sync[3] = sync[1];
            sync[0] = (unsigned)c0;
            sync[1] = (unsigned)(c0 >> 32);
        } else {
            sync[2] = sync[0];
            sync[3] = sync[1];
        }
    }
    __syncthreads();
    unsigned long long cur = read_claim();
    unsigned long long nxt = ((unsigned long long)sync[3] << 32) | sync[2];
    __syncthreads();  // (sync is rewritten below)
    if (cur >= (unsigned long long)T.nblk) return;  // uniform
    stage(cur, A);
    int b = 0;
    for (;;) {
        land(A, b);
        if (tid == 0) {
            wait_planes(cur);
            if (nxt < (unsigned long long)T.nblk) claim();  // the pair after next
        }
        __syncthreads();  // the pair's data in LDS, its planes final, the pair after next claimed
        const unsigned long long nxt2 = nxt < (unsigned long long)T.nblk ? read_claim() : ~0ull;
        stage(nxt, Bs);  // in flight while this pair's gathers run
        double zv = 0.0, v0 = 0.0, v1 = 0.0;
        if (act && A.blk >= 0) {
            const char *B = buf(b);
            const double *sx = reinterpret_cast<const double *>(B);
            const unsigned char *sd = reinterpret_cast<const unsigned char *>(B + TAIL_SX);
            double sum = 0.0;
            if (A.r < T.nrows) {
                if (A.cnt <= TAIL_CAP) {
                    const int ox = (int)(A.base - A.xb) - A.base, oj = (int)(A.base - A.jb) - A.base;
                    const int len = A.re - A.rb;
                    if (len > 0 && len <= 8) {
                        double pr[8];
#pragma unroll
                        for (int u = 0; u < 8; u++) {
                            const int k = min(A.rb + u, A.re - 1);
                            pr[u] = ld_sc1d(x + A.r + soff[sd[k + oj]]) * sx[k + ox];
                        }
#pragma unroll
                        for (int u = 0; u < 8; u++)
                            if (u < len) sum += pr[u];
                    } else {
                        for (int k = A.rb; k < A.re; k++) sum += ld_sc1d(x + A.r + soff[sd[k + oj]]) * sx[k + ox];
                    }
                } else {
                    for (int k = A.rb; k < A.re; k++) sum += ld_sc1d(x + T.Aj[k]) * T.Ax[k];
                }
                if (T.epi == EPI_MXY) zv = sum;
                else if (T.epi == EPI_AMXY) zv = sum * T.alpha;
                else if (T.epi == EPI_AXPBY) zv = ld_sc1d(T.y + A.r) * T.beta + T.alpha * sum;
                else zv = T.alpha * sum;
                T.z[A.r] = zv;
                if (T.nred > 0) v0 = zv * (T.w0 == T.z ? zv : A.w0p);
                if (T.nred > 1) v1 = zv * (T.w1 && T.w1 != T.z ? A.w1p : zv);
            }
        }
        // chunk_reduce's order: the chunk's four wave halving trees, (w0 + w1) + (w2 + w3)
        double *red = reinterpret_cast<double *>(buf(b) + TAIL_SX + TAIL_SD);  // [slot][wave]
        const int wq = (tid >> 6) & 3;
        if (T.nred > 0) {
            const double s0 = wave_sum_d(v0);
            const double s1 = T.nred > 1 ? wave_sum_d(v1) : 0.0;
            if (act && (tid & 63) == 0) {
                red[wq] = s0;
                red[4 + wq] = s1;
            }
        }
        __syncthreads();  // the pair's LDS is read (it is rewritten two rounds later) and reduced
        if (T.nred > 0 && act && t == 0 && A.blk >= 0) {
            T.part[A.blk] = (red[0] + red[1]) + (red[2] + red[3]);
            if (T.nred > 1) T.part[T.pcap + A.blk] = (red[4] + red[5]) + (red[6] + red[7]);
        }
        if (nxt >= (unsigned long long)T.nblk) break;  // uniform
        A = Bs;
        cur = nxt;
        nxt = nxt2;
        b ^= 1;
    }
}

}  // namespace lssp_amd
