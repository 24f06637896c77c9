// linesweep_dev.h -- device helpers shared by the line sweeps (linesweep.hip:
// k_line2 for ILU(0); linefill.hip: k_linef for the 7-point ILU(1)
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
__device__ __forceinline__ double wave_sum_d(double v) { return wave_sum_l0(v); }

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

// The tail product, workgroup-wide, in rounds of a GROUP of TAIL_CPR 256-row
// chunks with split roles: threads 0..511 compute (two rows each, of chunks
// c and c + 2 of the group), loader wave 0 claims groups and polls the tile
// counts, loader waves 1 and 2 load.  Each role waits only for its own memory
// operations (vmcnt is per wave): in round i the compute waves gather x for
// group i from the LDS-staged values and ids, while the loaders LDS-DMA group
// i+1's value and id ranges (from its row pointers, loaded a round earlier),
// load group i+2's row pointers, make sure group i+1's planes are final and
// claim group i+3 -- one memory round trip per round, ~3 us under the sweep's
// load, so a round moves 1024 rows.  LDS (~150 KB; the sweep kernels reserve
// it): the offset table, claims, 3 slots of row pointers, 2 buffers of the
// group's values + ids, the reduction words.  (Earlier versions -- one 64-row
// group per wave with three dependent round trips; staging loads in the
// compute waves' own in-order queue; 512-row rounds -- moved 80 / 150 / 170
// rows/us per CU and made the product slower than k_spmv3:
// profiles/r05/r05c_tail_ab.txt.)
constexpr int TAIL_CPR = 4;                     // chunks per round
constexpr int TAIL_NXP = 15;                    // 1 KB value pieces per chunk
constexpr int TAIL_NDP = 2;                     // 1 KB id pieces per chunk
constexpr int TAIL_CAP = TAIL_NXP * 128 - 1;    // entries per chunk staged (7-pt: <= 1792)
constexpr int TAIL_CHB = (TAIL_NXP + TAIL_NDP) * 1024;
constexpr int TAIL_APC = 260;                   // row pointers per chunk (257 used)
constexpr int TAIL_OFF_SYNC = 1024, TAIL_OFF_AP = 1088;
constexpr int TAIL_OFF_BUF = TAIL_OFF_AP + 3 * TAIL_CPR * TAIL_APC * 4;
constexpr int TAIL_OFF_RED = TAIL_OFF_BUF + 2 * TAIL_CPR * TAIL_CHB;
constexpr int TAIL_WAVES = 11;  // the sweeps' workgroups: 8 compute + 3 loader waves
constexpr int TAIL_LDS_BYTES(int) { return TAIL_OFF_RED + 2 * TAIL_CPR * 8 * 8; }
static_assert(TAIL_LDS_BYTES(0) <= 160 * 1024, "the tail product's LDS");
// claims one launch's tails consume: the groups, then one failed claim per workgroup
__host__ __device__ inline unsigned long long tail_claims(long nblk, long grid)
{
    return (unsigned long long)TAIL_CPR * (unsigned long long)((nblk + TAIL_CPR - 1) / TAIL_CPR + grid);
}
static __device__ void line_tail_wg(const LineTail &T, const double *x, int *err, char *smem)
{
    constexpr int CPR = TAIL_CPR, AP_N = CPR * 257;
    const int tid = threadIdx.x;
    const bool comp = tid < 512;
    const int c = (tid >> 8) & 1, t = tid & 255;  // compute: chunks c, c + 2 of the group; row in the chunk
    const int lt = tid - 512;                     // loader thread 0..191 (waves past 11 idle)
    const bool ldr = !comp && lt < 192;
    const int lw = __builtin_amdgcn_readfirstlane(lt >> 6), lane = tid & 63;
    const int *soff = reinterpret_cast<const int *>(smem);
    unsigned *sync = reinterpret_cast<unsigned *>(smem + TAIL_OFF_SYNC);
    int *aps = reinterpret_cast<int *>(smem + TAIL_OFF_AP);          // [3][CPR][TAIL_APC]
    double *reds = reinterpret_cast<double *>(smem + TAIL_OFF_RED);  // [2][CPR][8]
    const unsigned lds0 = (unsigned)(uintptr_t)smem;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long NB = (unsigned long long)T.nblk;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(x), 0,
                                                                        (int)min((long)T.nrows * 8, 0x7fffffffL), 0x00020000);
    // x (the sweep's output): plain loads, cached in this XCD's L2.  Safe because
    // every line of x a group touches is final before its first load: the group
    // waits for the planes of its rows less the widest offset less 15 rows (a
    // 128-byte line's other rows), x is not read by anything else in the kernel,
    // and its writers' stores are write-through and drained before their tile is
    // counted.
    auto ldx = [&](int col) {
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xr, (int)((unsigned)col * 8u), 0, 0));
    };
    auto ldv = [&](const double *p, int i) { return p == x ? ldx(i) : p[i]; };
    auto blk_of = [&](unsigned long long g, int k) {  // chunk k of a group, -1 past the end
        return g + k < NB ? T.cend - 1 - (long)(g + k) : -1L;
    };
    auto claim = [&]() { return atomicAdd(T.claim, (unsigned long long)CPR) - T.base; };
    // loader waves 1, 2: a group's row pointers into slot q (257 per chunk)
    auto load_ap = [&](unsigned long long g, int q) {
        constexpr int U = (AP_N + 127) / 128;
        int v[U], dst[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int i = lt - 64 + 128 * u, k = i / 257, j = i % 257;
            dst[u] = -1;
            v[u] = 0;
            const long blk = i < AP_N ? blk_of(g, k) : -1L;
            if (blk >= 0) {
                const long r = min(blk * 256 + j, (long)T.nrows);
                v[u] = T.Ap[r];
                dst[u] = (q * CPR + k) * TAIL_APC + j;
            }
        }
#pragma unroll
        for (int u = 0; u < U; u++)
            if (dst[u] >= 0) aps[dst[u]] = v[u];
    };
    // loader waves 1, 2: LDS-DMA of a group's value and id ranges (from slot q) into buffer bb
    auto load_vals = [&](unsigned long long g, int q, int bb) {
#pragma unroll
        for (int k = 0; k < CPR; k++) {
            const long blk = blk_of(g, k);
            if (blk < 0) continue;
            const int *ap = aps + (q * CPR + k) * TAIL_APC;
            const int rows = min(256, T.nrows - (int)(blk * 256));
            const int base = ap[0], cnt = ap[rows] - base;
            if (cnt > TAIL_CAP) continue;  // the compute reads this chunk from HBM
            const long xb = base & ~1L, jb = base & ~15L;
            const int npx = (int)((((long)base + cnt - xb) * 8 + 1023) / 1024);
            const int npd = (int)(((long)base + cnt - jb + 1023) / 1024);
            const unsigned bl = lds0 + TAIL_OFF_BUF + (bb * CPR + k) * TAIL_CHB;
            const long xlast = (T.nnz_pad >> 1) - 1, dlast = ((T.nnz_pad - 4 + 32) >> 4) - 1;
            for (int p = lw - 1; p < npx + npd; p += 2) {
                if (p < npx) {
                    const long v = min((xb >> 1) + p * 64 + lane, xlast);
                    dma16(reinterpret_cast<const char *>(T.Ax) + v * 16, __builtin_amdgcn_readfirstlane(bl + p * 1024));
                } else {
                    const int pd = p - npx;
                    const long v = min((jb >> 4) + pd * 64 + lane, dlast);
                    dma16(reinterpret_cast<const char *>(T.Ad) + v * 16,
                          __builtin_amdgcn_readfirstlane(bl + TAIL_NXP * 1024 + pd * 1024));
                }
            }
        }
    };
    // loader thread 0: the group's rows read final planes only.  U tile rows Kp =
    // S-1-K complete (nearly) in increasing Kp, the groups come from the top down:
    // the prefix of rows seen complete (kp_done) is not asked about again
    int kp_done = -1;
    auto wait_planes = [&](unsigned long long g) {
        if (g >= NB) return;
        const long lo = T.cend - 1 - (long)min(g + CPR - 1, NB - 1);
        const int r0 = (int)(lo * 256);
        const int ka = max(max(r0 - 15, 0) / (int)T.pl - 1, 0);  // (lines of x: 16 rows)
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
    // LSSP_AMD_TAIL_DIAG: per workgroup {target, entry, first group ready, exit, groups, plane-wait ticks}
    unsigned *dw = T.dbg && tid == 512 ? T.dbg + 4096 + 8 * blockIdx.x : nullptr;
    unsigned long long wticks = 0;
    int ngroups = 0;
    if (dw) {
        dw[0] = T.ktarget;
        dw[1] = (unsigned)t0;
    }
    // ---- prologue: claims of groups 0..2 (each only while the previous is valid),
    // row pointers of groups 0 and 1, values of group 0, its planes
    if (tid == 512) {
        unsigned long long q[3] = {~0ull, ~0ull, ~0ull};
        q[0] = claim();
        if (q[0] < NB) q[1] = claim();
        if (q[1] < NB) q[2] = claim();
        for (int k = 0; k < 3; k++) {
            sync[2 * k] = (unsigned)q[k];
            sync[2 * k + 1] = (unsigned)(q[k] >> 32);
        }
    }
    __syncthreads();
    auto rd = [&](int k) { return ((unsigned long long)sync[2 * k + 1] << 32) | sync[2 * k]; };
    unsigned long long g0 = rd(0), g1 = rd(1), g2 = rd(2);
    if (g0 >= NB) {  // uniform
        if (dw) dw[3] = (unsigned)__builtin_amdgcn_s_memrealtime();
        return;
    }
    if (ldr && lw > 0) {
        load_ap(g0, 0);
        load_ap(g1, 1);
    }
    __syncthreads();
    if (ldr) {
        if (lw > 0) load_vals(g0, 0, 0);
        else if (lt == 0) wait_planes(g0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (dw) dw[2] = (unsigned)__builtin_amdgcn_s_memrealtime();
    int b = 0, q = 0;  // buffer and row-pointer slot of the current group
    // diagnostics: busy time per round of compute wave 0 and loader wave 1 (to their barrier)
    unsigned *dwr = T.dbg && (tid == 0 || tid == 576) ? T.dbg + 4096 + 8 * blockIdx.x + (tid == 0 ? 6 : 7) : nullptr;
    unsigned long long rticks = 0;
    for (;;) {
        // g0: this round's group (buffer b, slot q); g1: next (slot q+1); g2: after next
        const uint64_t tr = dwr ? __builtin_amdgcn_s_memrealtime() : 0;
        if (comp) {
            // both rows' loads first (gathers of x, the dot operands), then the sums:
            // no branch between the two rows' loads and the products, so every
            // load of the round is in flight before the first wait (a row that
            // is not computed here loads x out of the buffer's range: +0.0)
            double xv[2][8], av[2][8], w0p[2], w1p[2];
            int len[2], row[2];
            bool big[2];
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int k = c + 2 * h;
                const long blk = blk_of(g0, k);
                const int r0 = blk >= 0 ? (int)(blk * 256) : 0;
                const int rows = blk >= 0 ? min(256, T.nrows - r0) : 0;
                const bool ok = blk >= 0 && t < rows;
                const int *ap = aps + (q * CPR + k) * TAIL_APC;
                const int base = ap[0], cnt = ap[rows] - base;
                const int rb = ap[t], re = ap[t + 1];
                const int r = ok ? r0 + t : 0;
                row[h] = ok ? r : -1;
                len[h] = ok ? re - rb : 0;
                big[h] = ok && (cnt > TAIL_CAP || len[h] > 8);
                const bool fast = ok && !big[h] && len[h] > 0;
                w0p[h] = T.nred > 0 && T.w0 != T.z ? ldv(T.w0, r) : 0.0;
                w1p[h] = T.nred > 1 && T.w1 && T.w1 != T.z ? ldv(T.w1, r) : 0.0;
                const char *B = smem + TAIL_OFF_BUF + (b * CPR + k) * TAIL_CHB;
                const double *sx = reinterpret_cast<const double *>(B);
                const unsigned char *sd = reinterpret_cast<const unsigned char *>(B + TAIL_NXP * 1024);
                const int ox = -(base & ~1), oj = -(base & ~15);
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int kk = min(rb + u, re - 1);
                    const int ij = fast ? kk + oj : 0, ix = fast ? kk + ox : 0;
                    const int col = fast ? r + soff[sd[ij]] : 0x1FFFFFFF;  // (past num_records: +0.0)
                    xv[h][u] = ldx(col);
                    av[h][u] = sx[ix];
                }
            }
            double pr[2][8];
#pragma unroll
            for (int h = 0; h < 2; h++)
#pragma unroll
                for (int u = 0; u < 8; u++) pr[h][u] = xv[h][u] * av[h][u];
            double v0[2] = {0.0, 0.0}, v1[2] = {0.0, 0.0};
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int r = row[h];
                if (r < 0) continue;
                double sum = 0.0;
                if (!big[h]) {
#pragma unroll
                    for (int u = 0; u < 8; u++)
                        if (u < len[h]) sum += pr[h][u];
                } else {
                    const int k = c + 2 * h;
                    const int *ap = aps + (q * CPR + k) * TAIL_APC;
                    const int rb = ap[t], re = ap[t + 1];
                    const int rows = min(256, T.nrows - (r - t)), base = ap[0], cnt = ap[rows] - base;
                    if (cnt <= TAIL_CAP) {
                        const char *B = smem + TAIL_OFF_BUF + (b * CPR + k) * TAIL_CHB;
                        const double *sx = reinterpret_cast<const double *>(B);
                        const unsigned char *sd = reinterpret_cast<const unsigned char *>(B + TAIL_NXP * 1024);
                        const int ox = -(base & ~1), oj = -(base & ~15);
                        for (int kk = rb; kk < re; kk++) sum += ldx(r + soff[sd[kk + oj]]) * sx[kk + ox];
                    } else {
                        for (int kk = rb; kk < re; kk++) sum += ldx(T.Aj[kk]) * T.Ax[kk];
                    }
                }
                double zv;
                if (T.epi == EPI_MXY) zv = sum;
                else if (T.epi == EPI_AMXY) zv = sum * T.alpha;
                else if (T.epi == EPI_AXPBY) zv = ldv(T.y, r) * T.beta + T.alpha * sum;
                else zv = T.alpha * sum;
                T.z[r] = zv;
                if (T.nred > 0) v0[h] = zv * (T.w0 == T.z ? zv : w0p[h]);
                if (T.nred > 1) v1[h] = zv * (T.w1 && T.w1 != T.z ? w1p[h] : zv);
            }
            // chunk_reduce's order: each chunk's four wave halving trees, (w0 + w1) + (w2 + w3)
            if (T.nred > 0) {
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const double s0 = wave_sum_d(v0[h]);
                    const double s1 = T.nred > 1 ? wave_sum_d(v1[h]) : 0.0;
                    if (lane == 0) {
                        double *red = reds + (b * CPR + c + 2 * h) * 8;
                        red[(tid >> 6) & 3] = s0;
                        red[4 + ((tid >> 6) & 3)] = s1;
                    }
                }
            }
        } else if (ldr) {
            // loaders: group g1's values (its row pointers are in slot q+1), group g2's
            // row pointers (waves 1, 2); g1's planes and the claim of the group after
            // g2 (wave 0) -- every wave waits for its own round trips only
            const int q1 = q == 2 ? 0 : q + 1, q2 = q1 == 2 ? 0 : q1 + 1;
            if (lw > 0) {
                if (g1 < NB) load_vals(g1, q1, b ^ 1);
                if (g2 < NB) load_ap(g2, q2);
            } else if (lt == 0) {
                const unsigned long long g3 = g2 < NB ? claim() : ~0ull;
                const uint64_t tw = dw ? __builtin_amdgcn_s_memrealtime() : 0;
                wait_planes(g1);
                if (dw) wticks += __builtin_amdgcn_s_memrealtime() - tw;
                sync[6] = (unsigned)g3;
                sync[7] = (unsigned)(g3 >> 32);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (dwr) rticks += __builtin_amdgcn_s_memrealtime() - tr;
        __syncthreads();  // group g0 computed; g1 staged and its planes final; g2's pointers in; g3 claimed
        if (T.nred > 0 && comp && t == 0) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const long blk = blk_of(g0, c + 2 * h);
                const double *red = reds + (b * CPR + c + 2 * h) * 8;
                if (blk >= 0) {
                    T.part[blk] = (red[0] + red[1]) + (red[2] + red[3]);
                    if (T.nred > 1) T.part[T.pcap + blk] = (red[4] + red[5]) + (red[6] + red[7]);
                }
            }
        }
        const unsigned long long g3 = g2 < NB ? rd(3) : ~0ull;
        ngroups++;
        if (g1 >= NB) break;  // uniform
        __syncthreads();  // (sync word 3 is rewritten next round)
        g0 = g1;
        g1 = g2;
        g2 = g3;
        b ^= 1;
        q = q == 2 ? 0 : q + 1;
    }
    if (dw) {
        dw[3] = (unsigned)__builtin_amdgcn_s_memrealtime();
        dw[4] = ngroups;
        dw[5] = (unsigned)wticks;
    }
    if (dwr) *dwr = (unsigned)rticks;
}

}  // namespace lssp_amd
