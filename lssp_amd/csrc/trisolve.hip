// trisolve.hip -- the ILU triangular sweeps (solver-tri.cxx:4-60) on gfx950.
//
// Structured ILU(0) factors of 5-/7-point grids run the line sweeps
// (linesweep.hip).  Every other factor (ILUK(k>0), ILUT, block-Jacobi, general
// patterns): the role-split packet pipeline through schedule-ordered shadow
// vectors (k_tri_pk6, packets from tri_bp.cpp build_packets6), or -- when a
// factor has rows longer than the longest packet record, and for the
// single-sweep API -- the sync-free level-ordered sweep (k_trisolve).
// DESIGN.md 3.4 has the measurements behind the choice.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "internal.h"

namespace lssp_amd {

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

// a published value never carries the flag pattern: a computed NaN with the
// sentinel's payload (e.g. propagated from such an rhs entry) becomes the
// default quiet NaN, so no reader waits for it
__device__ __forceinline__ void st_agent(double *p, double v)
{
    uint64_t b = (uint64_t)__double_as_longlong(v);
    if (b == TRI_SENTINEL) b = 0x7FF8000000000000ull;
    __hip_atomic_store(reinterpret_cast<uint64_t *>(p), b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Sync-free sweep.  First pass over a row's entries loads them in batches of
// four; once a dependency is found missing, the lane re-polls only that one
// entry (one load per lane per poll) with an exponential back-off, so waves
// far ahead of the wavefront do not flood the memory system with polls.
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
            if (nap < 32) nap <<= 1;
        }
    }
}

// Workgroup barrier for LDS hand-offs only.  __syncthreads() is a
// workgroup-scope fence + s_barrier, which on gfx950 also waits vmcnt(0): every
// in-flight global load AND every x store would be waited for at each step.
// Here only LDS traffic must be complete; global loads are waited for where
// their registers are used, the sc1 x stores are never waited for.
__device__ __forceinline__ void lds_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

typedef int v4i __attribute__((ext_vector_type(4)));

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
#ifndef PK_SPIN_SLEEP
#define PK_SPIN_SLEEP 1
#endif
        if (PK_SPIN_SLEEP) __builtin_amdgcn_s_sleep(PK_SPIN_SLEEP);
    }
}

typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

// v6 record length of a packet of n1 rows, in 16-byte units (tri_bp.cpp
// build_packets6: C, V, D, ROW arrays, each padded to 4 words)
template <int EP>
__device__ __forceinline__ int rec16(int n1)
{
    auto pad4 = [](int w) { return (w + 3) & ~3; };
    return (pad4((EP / 2) * n1) + 2 * EP * n1 + pad4(2 * n1) + pad4(n1)) / 4;
}
constexpr int PK6_REC16 = 1024;  // LREC: record bytes per packet <= 16 KB (4 loads x 256 loader lanes)

struct PkLd {
    int row, xi[PK3_EXT];
    int nr, nx;
    double rh;
    uint64_t ev[PK3_EXT];
    v4u rw[4];  // LREC: the packet's compute record, 4 x 16 B per loader lane
    int rlen;   // record length in 16-byte units (0: none)
};

// Packets v6 (tri_bp.cpp build_packets6) with schedule-ordered shadow vectors:
// compute and loader roles, and
//   * the sweep's output goes to a shadow vector in schedule order with
//     coalesced agent-scope stores (position pos0+t), and the HBM operands of
//     a packet are read from that shadow by schedule position: for a stencil
//     both are contiguous runs (one line per 8 rows instead of one per row);
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
    int n, B;
    int unit;  // unit diagonal (ILUK / ILUT L): x / 1.0 == x, the division is skipped
    unsigned long long *claim;
    unsigned long long base;
    int *err;
    // diagnostics (LSSP_AMD_PK6_TRACE): per block {claim, first step, end,
    // sentinel hits, xcc, packets}; per packet of block tblk {compute start,
    // compute end, loader wait (clk), loader landing end}
    unsigned long long *trace;
    int tblk;
};

template <int EP>
struct Pk6Rec {
    // int16 code pairs: EP/2 words, loaded as uint2 (EP 4) or uint4 chunks
    typedef typename std::conditional<EP == 4, v2u, v4u>::type CW;
    static constexpr int NCW = EP == 4 ? 1 : EP / 8;
    CW c[NCW];
    double v[EP];
    double dg;
    int nr, pos0;
    // byte offset of operand e in the LDS operand array (tri_bp.cpp pk6_xs_off)
    __device__ __forceinline__ unsigned off(int e) const
    {
        const unsigned w = EP == 4 ? c[0][e / 2] : c[e / 8][(e / 2) & 3];
        return (e & 1) ? (w >> 16) : (w & 0xffffu);
    }
};


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
// LREC (long rows, EP 16 / 24): the compute record does not fit in rotating
// registers; the loader lanes fetch it KE steps ahead with the gathers and land
// it in an LDS slot at the end of the step before, and the compute lanes read
// it from there (D unused).
template <int EP, int KE, int IA, int D, int NR, bool LREC = false, bool TRACE = false, int EXT = 2>
__global__ __launch_bounds__(2 * NR) void k_tri_pk6(Pk6Args a)
{
    constexpr int Q = 4;
    static_assert(D + 1 <= Q && IA <= Q && KE >= 1 && IA - KE >= 1 && IA - KE <= 2, "pipeline depths");
    constexpr int S0 = (IA > D ? IA : D);
    constexpr int J0 = -((S0 + Q - 1) / Q) * Q;  // first step, a multiple of Q
    // operands: the value ring, the +0.0 pad slot, the landed HBM operands of
    // two packets (pk6_xs_off); a record addresses each operand by byte offset
    static_assert(NR == 256, "pk6_xs_off assumes 256-row packets");
    __shared__ double xs[BP_RING + 1 + 2 * NR * PK3_EXT];
    double *const ring = xs;
    __shared__ double rbuf[2][NR];
    __shared__ int4 sdesc[PK3_CAP];
    __shared__ v4u recbuf[LREC ? 2 : 1][LREC ? PK6_REC16 : 1];
    __shared__ int s_blk;
    const int tid = threadIdx.x;
    const int role = __builtin_amdgcn_readfirstlane(tid) / NR;  // 0 compute, 1 loader
    const int t = tid & (NR - 1);
    if (tid == 0) ring[BP_RING] = 0.0;
    for (;;) {
        __syncthreads();
        if (tid == 0) s_blk = (int)(atomicAdd(a.claim, 1ull) - a.base);
        __syncthreads();
        const int b = s_blk;
        if (b >= a.nb) break;
        const int q0 = a.blk[b], np = a.blk[b + 1] - q0;
        if (TRACE && tid == 0) {
            a.trace[8L * b] = __builtin_amdgcn_s_memrealtime();
            a.trace[8L * b + 5] = np;
        }
        unsigned long long *ts = TRACE ? a.trace + 8L * a.nb : nullptr;
        const bool trs = TRACE && b == a.tblk && t == 0;
        const int bbase = b * a.B;  // first schedule position of the block
        for (int i = tid; i < np; i += blockDim.x) sdesc[i] = a.desc[q0 + i];
        __syncthreads();
        // both roles run steps J0 .. J0+T-1 (T a multiple of Q); out-of-range
        // packets turn into loads from valid dummy addresses
        const int T = (np - J0 + Q - 1) / Q * Q;
        // descriptor of a packet, clamped: out-of-range packets get nr = nx = 0
        // and read valid dummy records (no branches around the loads).  Read in
        // two halves -- the LDS read one step before its use, the move to
        // scalar registers at the use -- so no step waits for an LDS read at
        // its start (the step's barrier has drained LDS by then).
        auto dread = [&](int p) { return sdesc[min(max(p, 0), max(np - 1, 0))]; };
        auto duni = [&](const int4 r, int p) {
            int4 d = make_int4(__builtin_amdgcn_readfirstlane(r.x), __builtin_amdgcn_readfirstlane(r.y),
                               __builtin_amdgcn_readfirstlane(r.z), __builtin_amdgcn_readfirstlane(r.w));
            if (p < 0 || p >= np) d.z = 0;
            return d;
        };
        auto descc = [&](int p) { return duni(dread(p), p); };
        if (LREC && role == 0) {
            // compute lanes, record from LDS (landed by the loaders one step ahead)
            int4 draw = dread(J0);
            for (int j = J0; j < J0 + T; j++) {
                if (trs && j >= 0 && j < np) ts[4L * j] = __builtin_amdgcn_s_memtime();
                if (TRACE && tid == 0 && j == 0) a.trace[8L * b + 1] = __builtin_amdgcn_s_memrealtime();
                const int4 d = duni(draw, j);
                draw = dread(j + 1);
                const int nr = d.z & 0x3ff;
                if (t < nr) {
                    const unsigned *w = reinterpret_cast<const unsigned *>(recbuf[j & 1]);
                    const int wc = ((EP / 2) * nr + 3) & ~3;
                    typedef double v2d __attribute__((ext_vector_type(2)));
                    const v2d *V = reinterpret_cast<const v2d *>(w + wc);
                    const double dg = reinterpret_cast<const double *>(V + (EP / 2) * nr)[t];
                    double acc = rbuf[j & 1][t];
                    double xv[EP], vv[EP];
                    const char *xsb = reinterpret_cast<const char *>(xs);
#pragma unroll
                    for (int q = 0; q < EP / 8; q++) {
                        const v4u cw = reinterpret_cast<const v4u *>(w)[(EP / 8) * t + q];
#pragma unroll
                        for (int h = 0; h < 8; h++) {
                            const unsigned ww = cw[h / 2];
                            const unsigned o = (h & 1) ? (ww >> 16) : (ww & 0xffffu);
                            xv[8 * q + h] = *reinterpret_cast<const double *>(xsb + o);
                        }
                    }
#pragma unroll
                    for (int q = 0; q < EP / 2; q++) {
                        const v2d v = V[q * nr + t];
                        vv[2 * q] = v.x;
                        vv[2 * q + 1] = v.y;
                    }
#pragma unroll
                    for (int e = 0; e < EP; e++) acc = acc - vv[e] * xv[e];
                    const double xi = a.unit ? acc : acc / dg;
                    const int pos = d.w + t;
                    ring[(pos - bbase) & (BP_RING - 1)] = xi;
                    st_agent(a.sh + pos, xi);
                }
                if (trs && j >= 0 && j < np) ts[4L * j + 1] = __builtin_amdgcn_s_memtime();
                lds_barrier();
            }
            if (TRACE && tid == 0) a.trace[8L * b + 2] = __builtin_amdgcn_s_memrealtime();
            const long s0 = bbase, s1 = min(s0 + a.B, (long)a.n);
            uint64_t *rs = reinterpret_cast<uint64_t *>(a.sh_next);
            for (long i = s0 + t; i < s1; i += NR) rs[i] = TRI_SENTINEL;
        } else if (role == 0) {
            auto issue = [&](const int4 d, Pk6Rec<EP> &Rr) {
                const int nr = d.z & 0x3ff;
                const int n1 = nr > 0 ? nr : 1, tt = min(t, n1 - 1);
                const uint32_t *base = a.rec + 4L * d.x;
                const int wc = ((EP / 2) * n1 + 3) & ~3;
#pragma unroll
                for (int q = 0; q < Pk6Rec<EP>::NCW; q++)
                    Rr.c[q] = reinterpret_cast<const typename Pk6Rec<EP>::CW *>(base)[Pk6Rec<EP>::NCW * tt + q];
                typedef double v2d __attribute__((ext_vector_type(2)));
                const v2d *vb = reinterpret_cast<const v2d *>(base + wc);
#pragma unroll
                for (int q = 0; q < EP / 2; q++) {
                    const v2d v = vb[q * n1 + tt];
                    Rr.v[2 * q] = v.x;
                    Rr.v[2 * q + 1] = v.y;
                }
                // unit diagonal (ILUK / ILUT L): the stored 1.0 is never read -- 8 bytes
                // per row less on the sweep's record stream
                Rr.dg = a.unit ? 1.0 : reinterpret_cast<const double *>(vb + (EP / 2) * n1)[tt];
                Rr.nr = nr;
                Rr.pos0 = d.w;
            };
            int4 dn = descc(J0 + D);    // descriptor of packet j+D, read one step ahead
            int4 dnr = dread(J0 + D + 1);
            auto step = [&](int j, Pk6Rec<EP> &Rc, Pk6Rec<EP> &Rn) {
                if (trs && j >= 0 && j < np) ts[4L * j] = __builtin_amdgcn_s_memtime();
                if (TRACE && tid == 0 && j == 0) a.trace[8L * b + 1] = __builtin_amdgcn_s_memrealtime();
                issue(dn, Rn);
                dn = duni(dnr, j + D + 1);
                dnr = dread(j + D + 2);
                // the current record must be complete here, at one fixed point
#pragma unroll
                for (int q = 0; q < Pk6Rec<EP>::NCW; q++) asm volatile("" ::"v"(Rc.c[q]));
#pragma unroll
                for (int e = 0; e < EP; e++) asm volatile("" ::"v"(Rc.v[e]));
                asm volatile("" ::"v"(Rc.dg));
                if (t < Rc.nr) {  // nr == 0 outside the block's packets
                    double acc = rbuf[j & 1][t];
                    double xv[EP];
                    const char *xsb = reinterpret_cast<const char *>(xs);
                    // all EP entries: padded ones read +0.0 and subtract +0.0*+0.0
#pragma unroll
                    for (int e = 0; e < EP; e++) xv[e] = *reinterpret_cast<const double *>(xsb + Rc.off(e));
#pragma unroll
                    for (int e = 0; e < EP; e++) acc = acc - Rc.v[e] * xv[e];
                    const double xi = a.unit ? acc : acc / Rc.dg;
                    const int pos = Rc.pos0 + t;
                    ring[(pos - bbase) & (BP_RING - 1)] = xi;
                    st_agent(a.sh + pos, xi);
                }
                if (trs && j >= 0 && j < np) ts[4L * j + 1] = __builtin_amdgcn_s_memtime();
                lds_barrier();
            };
            Pk6Rec<EP> R0, R1, R2, R3;
            R0.nr = R1.nr = R2.nr = R3.nr = 0;
            for (int j0 = J0; j0 < J0 + T; j0 += Q) {  // j0 == 0 (mod Q): packet p in set p mod Q
                step(j0, sel4<0>(R0, R1, R2, R3), sel4<(0 + D) % Q>(R0, R1, R2, R3));
                step(j0 + 1, sel4<1>(R0, R1, R2, R3), sel4<(1 + D) % Q>(R0, R1, R2, R3));
                step(j0 + 2, sel4<2>(R0, R1, R2, R3), sel4<(2 + D) % Q>(R0, R1, R2, R3));
                step(j0 + 3, sel4<3>(R0, R1, R2, R3), sel4<(3 + D) % Q>(R0, R1, R2, R3));
            }
            if (TRACE && tid == 0) a.trace[8L * b + 2] = __builtin_amdgcn_s_memrealtime();
            // arm the block's positions of the other shadow for the next apply
            const long s0 = bbase, s1 = min(s0 + a.B, (long)a.n);
            uint64_t *rs = reinterpret_cast<uint64_t *>(a.sh_next);
            for (long i = s0 + t; i < s1; i += NR) rs[i] = TRI_SENTINEL;
        } else {
            // The loader's loads are issued from inline asm with explicit
            // vmcnt waits: its register sets rotate across the loop back-edge,
            // where the compiler's own wait counting turns conservative and
            // waited for the previous step's gathers before issuing new ones.
            // Per step, in issue order: E = 1 + EXT index loads (packet
            // j+IA: the rhs index and EXT operand indices), then E gathers
            // (packet j+KE) -- so before the gathers, the indices they use
            // (issued at step j-(IA-KE)) have E + (IA-KE-1)(RL+2E) + RL + E
            // younger loads, and the gathers landed at the end of step j
            // (packet j+1, issued at step j+1-KE) have (KE-1)(RL+2E).
            // LREC: RL record loads (packet j+KE) open every step, so per step
            // the queue grows by RL + E + E in the order records, indices, gathers
            static_assert(EXT >= 2 && EXT <= 4, "operand loads per lane");
            static_assert(EXT <= PK3_EXT, "the landed-operand buffers hold PK3_EXT per row");
            constexpr int E = 1 + EXT;
            constexpr int RL = LREC ? 4 : 0;
            static_assert(!LREC || PK6_REC16 == RL * NR, "record loads cover one LDS slot");
            constexpr int WAIT_IDX = E + (IA - KE - 1) * (RL + 2 * E) + RL + E;  // younger than the indices the gathers use
            constexpr int WAIT_G = (KE - 1) * (RL + 2 * E);  // younger than packet j+1's gathers (and records)
            static_assert(WAIT_IDX <= 63 && WAIT_G + RL + 2 * E <= 63, "vmcnt range");
            auto issue_rec = [&](const int4 d, PkLd &L) {
                if constexpr (LREC) {
                    const int nr = d.z & 0x3ff, n1 = nr > 0 ? nr : 1;
                    const int len = rec16<EP>(n1);
                    const v4u *base = reinterpret_cast<const v4u *>(a.rec) + d.x;
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const v4u *p = base + min(t + NR * u, len - 1);
                        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(L.rw[u]) : "v"(p) : "memory");
                    }
                    L.rlen = nr > 0 ? len : 0;
                }
            };
            auto issue_idx = [&](const int4 d, PkLd &L) {
                const int nr = d.z & 0x3ff, nx = (d.z >> 10) & 0x7ff;
                const int *base = a.idx + d.y;
                const int *p0 = base + max(min(t, nr - 1), 0);
                asm volatile("global_load_dword %0, %1, off" : "=v"(L.row) : "v"(p0) : "memory");
#pragma unroll
                for (int e = 0; e < EXT; e++) {
                    const int *pe = base + nr + max(min(t + NR * e, nx - 1), 0);
                    asm volatile("global_load_dword %0, %1, off" : "=v"(L.xi[e]) : "v"(pe) : "memory");
                }
                L.nr = nr;
                L.nx = nx;
            };
            auto gather = [&](PkLd &L) {
                if constexpr (EXT == 4)
                    asm volatile("s_waitcnt vmcnt(%5)"
                                 : "+v"(L.row), "+v"(L.xi[0]), "+v"(L.xi[1]), "+v"(L.xi[EXT - 2]), "+v"(L.xi[EXT - 1])
                                 : "n"(WAIT_IDX) : "memory");
                else if constexpr (EXT == 3)
                    asm volatile("s_waitcnt vmcnt(%4)" : "+v"(L.row), "+v"(L.xi[0]), "+v"(L.xi[1]), "+v"(L.xi[EXT - 1])
                                 : "n"(WAIT_IDX) : "memory");
                else
                    asm volatile("s_waitcnt vmcnt(%3)" : "+v"(L.row), "+v"(L.xi[0]), "+v"(L.xi[1]) : "n"(WAIT_IDX) : "memory");
                const double *pr = a.rhs + L.row;
                asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(L.rh) : "v"(pr) : "memory");
#pragma unroll
                for (int e = 0; e < EXT; e++) {
                    const double *pxe = a.sh + L.xi[e];
                    asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=v"(L.ev[e]) : "v"(pxe) : "memory");
                }
            };
            int4 dl = descc(J0 + IA);  // descriptor of packet j+IA, read one step ahead
            int4 dlr = dread(J0 + IA + 1);
            static_assert(!LREC || IA - KE == 1, "LREC: the record's packet j+KE is the index loads' of step j-1");
            int4 dk = descc(J0 + KE);
            unsigned hits = 0;
            auto step = [&](int j, PkLd &Li, PkLd &Lg, PkLd &Ll) {
                issue_rec(dk, Lg);
                issue_idx(dl, Li);
                gather(Lg);
                if constexpr (LREC) dk = dl;
                dl = duni(dlr, j + IA + 1);
                dlr = dread(j + IA + 2);
                const unsigned long long w0 = TRACE ? __builtin_amdgcn_s_memtime() : 0;
                // gathers of packet j+1 were issued at step j+1-KE
                if constexpr (LREC && EXT == 4)
                    asm volatile("s_waitcnt vmcnt(%9)"
                                 : "+v"(Ll.rh), "+v"(Ll.ev[0]), "+v"(Ll.ev[1]), "+v"(Ll.ev[EXT - 2]), "+v"(Ll.ev[EXT - 1]),
                                   "+v"(Ll.rw[0]), "+v"(Ll.rw[1]), "+v"(Ll.rw[2]), "+v"(Ll.rw[3])
                                 : "n"(WAIT_G)
                                 : "memory");
                else if constexpr (LREC && EXT == 3)
                    asm volatile("s_waitcnt vmcnt(%8)"
                                 : "+v"(Ll.rh), "+v"(Ll.ev[0]), "+v"(Ll.ev[1]), "+v"(Ll.ev[EXT - 1]), "+v"(Ll.rw[0]),
                                   "+v"(Ll.rw[1]), "+v"(Ll.rw[2]), "+v"(Ll.rw[3])
                                 : "n"(WAIT_G)
                                 : "memory");
                else if constexpr (LREC)
                    asm volatile("s_waitcnt vmcnt(%7)"
                                 : "+v"(Ll.rh), "+v"(Ll.ev[0]), "+v"(Ll.ev[1]), "+v"(Ll.rw[0]), "+v"(Ll.rw[1]),
                                   "+v"(Ll.rw[2]), "+v"(Ll.rw[3])
                                 : "n"(WAIT_G)
                                 : "memory");
                else if constexpr (EXT == 4)
                    asm volatile("s_waitcnt vmcnt(%5)"
                                 : "+v"(Ll.rh), "+v"(Ll.ev[0]), "+v"(Ll.ev[1]), "+v"(Ll.ev[EXT - 2]), "+v"(Ll.ev[EXT - 1])
                                 : "n"(WAIT_G) : "memory");
                else if constexpr (EXT == 3)
                    asm volatile("s_waitcnt vmcnt(%4)" : "+v"(Ll.rh), "+v"(Ll.ev[0]), "+v"(Ll.ev[1]), "+v"(Ll.ev[EXT - 1])
                                 : "n"(WAIT_G) : "memory");
                else
                    asm volatile("s_waitcnt vmcnt(%3)" : "+v"(Ll.rh), "+v"(Ll.ev[0]), "+v"(Ll.ev[1]) : "n"(WAIT_G) : "memory");
                // land packet j+1 (nr = nx = 0 outside the block's packets)
                if (t < Ll.nr) rbuf[(j + 1) & 1][t] = Ll.rh;
                if constexpr (LREC) {
#pragma unroll
                    for (int u = 0; u < 4; u++)
                        if (t + NR * u < Ll.rlen) recbuf[(j + 1) & 1][t + NR * u] = Ll.rw[u];
                }
#pragma unroll
                for (int e = 0; e < EXT; e++) {
                    const int k = t + NR * e;
                    if (k < Ll.nx) {
                        uint64_t bits = Ll.ev[e];
                        if (bits == TRI_SENTINEL) {
                            if (TRACE) hits++;
                            bits = poll_ready(a.sh + Ll.xi[e], a.err);
                        }
                        xs[BP_RING + 1 + ((j + 1) & 1) * NR * PK3_EXT + k] = __longlong_as_double((long long)bits);
                    }
                }
                if (trs && j + 1 >= 0 && j + 1 < np) {  // the packet landed here is j+1
                    ts[4L * (j + 1) + 2] = __builtin_amdgcn_s_memtime() - w0;
                    ts[4L * (j + 1) + 3] = __builtin_amdgcn_s_memtime();
                }
                lds_barrier();
            };
            PkLd L0, L1, L2, L3;
            L0.nr = L1.nr = L2.nr = L3.nr = 0;
            L0.nx = L1.nx = L2.nx = L3.nx = 0;
            L0.row = L1.row = L2.row = L3.row = 0;
#pragma unroll
            for (int e = 0; e < PK3_EXT; e++) L0.xi[e] = L1.xi[e] = L2.xi[e] = L3.xi[e] = 0;
            L0.rh = L1.rh = L2.rh = L3.rh = 0;
            L0.rlen = L1.rlen = L2.rlen = L3.rlen = 0;
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
            if (TRACE) {
                for (int o = 32; o >= 1; o >>= 1) hits += __shfl_xor(hits, o);
                if ((t & 63) == 0 && hits) atomicAdd(a.trace + 8L * b + 3, (unsigned long long)hits);
                if (t == 0) {
                    unsigned xcc;
                    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
                    a.trace[8L * b + 4] = xcc;
                }
            }
        }
    }
}

int launch_trisolve(lssp_amd_ctx *c, const TriSched &t, const double *rhs, double *x, double *reset)
{
    if (t.n == 0) return LSSP_AMD_OK;
    long nchunks = (t.n + 63) / 64;
    TriArgs a{t.n, nchunks, t.perm, t.rp, t.cols, t.vals, t.diag, t.unit, rhs, x, reset, c->d_err};
    long grid = (long)c->num_cus * c->tri_blocks_per_cu;
    long need = (nchunks + 3) / 4;
    if (grid > need) grid = need;
    k_trisolve<<<grid, 256, 0, c->stream>>>(a);
    LSSP_HIP(hipGetLastError());
    return LSSP_AMD_OK;
}

// packet sweep of one factor: its output to the shadow sh (schedule order)
template <bool TRACE>
static void launch_pk6_k(lssp_amd_ctx *c, const TriSched &t, const Pk6Args &g, int grid)
{
    // Instantiated: 256-row packets, x operands gathered 2 steps ahead (KE 2);
    // EP 4 / 8 with register records, EP 16 / 24 with LDS records -- the
    // variants whose inline-asm loader tools/check_vmcnt.py
    // (tests/test_isa_vmcnt.py) verifies hazard-free
    if (t.pk6_ext == 4) {
        if (t.pk6_ep == 4) k_tri_pk6<4, 2, 4, 3, 256, false, TRACE, 4><<<grid, 512, 0, c->stream>>>(g);
        else if (t.pk6_ep == 8) k_tri_pk6<8, 2, 4, 3, 256, false, TRACE, 4><<<grid, 512, 0, c->stream>>>(g);
        else if (t.pk6_ep == 16) k_tri_pk6<16, 3, 4, 1, 256, true, TRACE, 4><<<grid, 512, 0, c->stream>>>(g);
        else k_tri_pk6<24, 3, 4, 1, 256, true, TRACE, 4><<<grid, 512, 0, c->stream>>>(g);
        return;
    }
    if (t.pk6_ext == 3) {
        if (t.pk6_ep == 4) k_tri_pk6<4, 2, 4, 3, 256, false, TRACE, 3><<<grid, 512, 0, c->stream>>>(g);
        else if (t.pk6_ep == 8) k_tri_pk6<8, 2, 4, 3, 256, false, TRACE, 3><<<grid, 512, 0, c->stream>>>(g);
        else if (t.pk6_ep == 16) k_tri_pk6<16, 3, 4, 1, 256, true, TRACE, 3><<<grid, 512, 0, c->stream>>>(g);
        else k_tri_pk6<24, 3, 4, 1, 256, true, TRACE, 3><<<grid, 512, 0, c->stream>>>(g);
        return;
    }
    if (t.pk6_ep == 4) k_tri_pk6<4, 2, 4, 3, 256, false, TRACE><<<grid, 512, 0, c->stream>>>(g);
    else if (t.pk6_ep == 8) k_tri_pk6<8, 2, 4, 3, 256, false, TRACE><<<grid, 512, 0, c->stream>>>(g);
    else if (t.pk6_ep == 16) k_tri_pk6<16, 3, 4, 1, 256, true, TRACE><<<grid, 512, 0, c->stream>>>(g);
    else k_tri_pk6<24, 3, 4, 1, 256, true, TRACE><<<grid, 512, 0, c->stream>>>(g);
}

static int launch_pk6(lssp_amd_ctx *c, const TriSched &t, const double *rhs, double *sh, double *sh_next)
{
    const int grid = std::min(t.bp_nb, c->num_cus);
    Pk6Args g{t.bp_nb, t.pk6_blk, reinterpret_cast<const int4 *>(t.pk6_desc), t.pk6_rec, t.pk6_idx, rhs, sh,
              sh_next, t.n, t.bp_B, t.unit, t.pk6_claim, t.pk6_base, c->d_err, nullptr, 0};
    if (t.pk6_rows != 256) return LSSP_AMD_EUNSUPPORTED;
    // diagnostics only: LSSP_AMD_PK6_TRACE=path[:block] appends one JSON line per sweep
    static const char *trp = getenv("LSSP_AMD_PK6_TRACE");
    if (!trp) {
        launch_pk6_k<false>(c, t, g, grid);
    } else {
        const char *colon = strrchr(trp, ':');
        g.tblk = colon ? atoi(colon + 1) : t.bp_nb / 2;
        const size_t tn = 8 * (size_t)t.bp_nb + 4 * (size_t)PK3_CAP + 64;
        LSSP_HIP(hipMalloc(&g.trace, sizeof(unsigned long long) * tn));
        LSSP_HIP(hipMemsetAsync(g.trace, 0, sizeof(unsigned long long) * tn, c->stream));
        launch_pk6_k<true>(c, t, g, grid);
        std::vector<unsigned long long> h(tn);
        LSSP_HIP(hipMemcpyAsync(h.data(), g.trace, sizeof(unsigned long long) * tn, hipMemcpyDeviceToHost, c->stream));
        LSSP_HIP(hipStreamSynchronize(c->stream));
        (void)hipFree(g.trace);
        std::string path(trp, colon ? colon - trp : strlen(trp));
        FILE *f = fopen(path.c_str(), "a");
        if (f) {
            fprintf(f, "{\"upper\": %d, \"nb\": %d, \"B\": %d, \"ep\": %d, \"tblk\": %d, \"grid\": %d, \"data\": [",
                    (int)t.upper, t.bp_nb, t.bp_B, t.pk6_ep, g.tblk, grid);
            for (size_t i = 0; i < tn; i++) fprintf(f, "%s%llu", i ? ", " : "", h[i]);
            fprintf(f, "]}\n");
            fclose(f);
        }
    }
    t.pk6_base += (unsigned long long)t.bp_nb + grid;
    LSSP_HIP(hipGetLastError());
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

// the gather as above with four positions per lane: the four indices come in
// one 16-byte load and the four (scattered) operand loads are in flight
// together -- more memory-level parallelism per lane than one dependent
// index -> operand chain at a time
__global__ __launch_bounds__(256) void k_gather4(double *dst, const double *src, const int *perm, int n)
{
    typedef double v2d __attribute__((ext_vector_type(2)));
    const int nx = 8, per = gridDim.x / nx;
    const int xcd = blockIdx.x % nx, k = blockIdx.x / nx;
    const long n4 = (long)n / 4, chunk = (n4 + nx - 1) / nx;
    const long lo = xcd * chunk, hi = min(n4, lo + chunk);
    const int4 *p4 = reinterpret_cast<const int4 *>(perm);
    v2d *d2 = reinterpret_cast<v2d *>(dst);
    for (long q = lo + (long)k * 256 + threadIdx.x; q < hi; q += (long)per * 256) {
        const int4 ix = p4[q];
        const double a0 = src[ix.x], a1 = src[ix.y], a2 = src[ix.z], a3 = src[ix.w];
        d2[2 * q] = v2d{a0, a1};
        d2[2 * q + 1] = v2d{a2, a3};
    }
    if (blockIdx.x == 0)
        for (long p = 4 * n4 + threadIdx.x; p < n; p += 256) dst[p] = src[perm[p]];
}

// ILU apply (solver-tri.cxx:57-60).  Packet sweeps: the scattered halves of
// the work -- reading the rhs in L order and writing x in natural order -- run
// as fully parallel permutation kernels around the two sweeps, so the
// pipelined sweeps only touch contiguous runs of HBM.
int launch_ilu_apply(lssp_amd_ctx *c, const lssp_amd_ilu *M, double *x, const double *rhs)
{
    if (M->line.ntiles) return launch_line_apply(c, M->line, x, rhs);
    if (M->lower.pk6_n > 0 && M->upper.pk6_n > 0) {
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
        if (((uintptr_t)rhs & 15) == 0)
            k_gather4<<<pg, 256, 0, c->stream>>>(M->d_rperm, rhs, M->lower.bp_perm, n);
        else
            k_perm<true><<<pg, 256, 0, c->stream>>>(M->d_rperm, rhs, M->lower.bp_perm, n);
        LSSP_HIP(hipGetLastError());
        LSSP_TRY(launch_pk6(c, M->lower, M->d_rperm, M->d_sh[e], M->d_sh[e ^ 1]));
        LSSP_TRY(launch_pk6(c, M->upper, M->d_sh[e], M->d_sh[2 + e], M->d_sh[2 + (e ^ 1)]));
        // x back to natural order as a gather through the inverse permutation
        // (coalesced stores, scattered loads: faster than scattering the stores)
        if (((uintptr_t)x & 15) == 0)
            k_gather4<<<pg, 256, 0, c->stream>>>(x, M->d_sh[2 + e], M->upper.bp_pos, n);
        else
            k_perm<true><<<pg, 256, 0, c->stream>>>(x, M->d_sh[2 + e], M->upper.bp_pos, n);
        LSSP_HIP(hipGetLastError());
        return LSSP_AMD_OK;
    }
    LSSP_TRY(launch_trisolve(c, M->lower, rhs, M->d_cache, x));
    return launch_trisolve(c, M->upper, M->d_cache, x, M->d_cache);
}

}  // namespace lssp_amd
