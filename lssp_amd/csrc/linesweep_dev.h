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

}  // namespace lssp_amd
