// lat_probe.hip -- calibration of the latencies the ILU sweep design rests on
// (tuning aid, not part of the library).  Build: hipcc -O3 --offload-arch=gfx950
// Prints cycles (s_memtime) per: LDS dependent read, s_barrier (8 waves),
// dependent HBM / L2 loads (plain and sc1), and the cross-CU value hand-off
// (sc1 store -> sc1 poll) between two workgroups.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_lds_chase(int iters, unsigned long long *out)
{
    __shared__ int a[4096];
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) a[i] = (i * 97 + 13) & 4095;
    __syncthreads();
    int p = threadIdx.x;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) p = a[p];
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = p; }
}

__global__ void k_barrier(int iters, unsigned long long *out)
{
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) out[0] = t1 - t0;
}

template <int SC1>
__global__ void k_chase(const long *next, int iters, unsigned long long *out)
{
    long p = 0;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
        if (SC1) p = __hip_atomic_load(next + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else p = next[p];
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = p; }
}

// two workgroups: block 0 writes v[i] = i+1 after seeing w[i-1] == i, block k
// (the partner) waits for v[i] then writes w[i]
__global__ void k_pingpong(unsigned long long *v, unsigned long long *w, int iters, int partner,
                           unsigned long long *out)
{
    if (threadIdx.x != 0) return;
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (blockIdx.x == 0) {
        uint64_t t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < iters; i++) {
            __hip_atomic_store(v + i, (unsigned long long)(i + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (long g = 0; g < (1L << 24) && __hip_atomic_load(w + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != (unsigned long long)(i + 1); g++) {}
        }
        uint64_t t1 = __builtin_amdgcn_s_memtime();
        out[0] = t1 - t0;
        out[2] = xcc;
    } else if ((int)blockIdx.x == partner) {
        for (int i = 0; i < iters; i++) {
            for (long g = 0; g < (1L << 24) && __hip_atomic_load(v + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != (unsigned long long)(i + 1); g++) {}
            __hip_atomic_store(w + i, (unsigned long long)(i + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        out[3] = xcc;
    }
}


// floor of one sweep step: compute waves 0-3 read 4 LDS operands (addresses
// from registers), 4 multiply-subtracts + one division, one LDS write, one
// barrier; waves 4-7 only take part in the barrier.  MODE 1 adds per-step
// coalesced record loads (5 x 16 B per lane, prefetched 3 steps ahead),
// MODE 2 also a coalesced 8-byte store per lane, MODE 3 a scattered store.
template <int MODE>
__global__ __launch_bounds__(512) void k_step(const double *rec, double *out, int iters, unsigned long long *cyc)
{
    __shared__ double ring[4097];
    const int t = threadIdx.x;
    for (int i = t; i < 4097; i += 512) ring[i] = 1.0 + i * 1e-3;
    __syncthreads();
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    if (t < 256) {
        double acc = 1.0;
        int c0 = (t + 7) & 4095, c1 = (t + 300) & 4095, c2 = (t + 1000) & 4095;
        struct R { double a, b, c, d, e; };
        R q0{}, q1{}, q2{}, q3{};
        auto step = [&](int i, R &cur, R &nxt) {
            if (MODE >= 1) {
                const double *b = rec + (size_t)((i + 3) & 1023) * 256 * 10 + t;
                nxt.a = b[0]; nxt.b = b[256]; nxt.c = b[512]; nxt.d = b[768]; nxt.e = b[1024];
                asm volatile("" :: "v"(cur.a), "v"(cur.b), "v"(cur.c), "v"(cur.d), "v"(cur.e));
            }
            double x0 = ring[c0], x1 = ring[c1], x2 = ring[c2], x3 = ring[4096];
            acc = acc - (0.5 + cur.b) * x0;
            acc = acc - (0.25 + cur.c) * x1;
            acc = acc - (0.125 + cur.d) * x2;
            acc = acc - cur.e * x3;
            const double xi = acc / (2.0 + cur.a);
            ring[(i * 256 + t) & 4095] = xi;
            if (MODE == 2) __hip_atomic_store(reinterpret_cast<unsigned long long *>(out) + ((size_t)(i & 1023) * 256 + t), (unsigned long long)__double_as_longlong(xi), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (MODE == 3) __hip_atomic_store(reinterpret_cast<unsigned long long *>(out) + ((size_t)(i & 1023) * 256 + t) * 215 % (1 << 23), (unsigned long long)__double_as_longlong(xi), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            c0 = (c0 + 256) & 4095;
            c1 = (c1 + 256) & 4095;
            c2 = (c2 + 256) & 4095;
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        };
        for (int i = 0; i < iters; i += 4) {
            step(i, q0, q3);
            step(i + 1, q1, q0);
            step(i + 2, q2, q1);
            step(i + 3, q3, q2);
        }
        if (acc == 12345.0) out[0] = acc;
    } else {
        for (int i = 0; i < iters; i++) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (t == 0) cyc[0] = t1 - t0;
}


// ping-pong with explicit cache policies: MODE 0 sc1 store / sc1 load,
// MODE 1 plain store / sc0 load (L2-coherent, same XCD only), MODE 2 sc1 store / sc0 load
template <int MODE>
__device__ __forceinline__ void pp_store(unsigned long long *p, unsigned long long v)
{
    if (MODE == 1) asm volatile("global_store_dwordx2 %0, %1, off" :: "v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx2 %0, %1, off sc1" :: "v"(p), "v"(v) : "memory");
}
template <int MODE>
__device__ __forceinline__ unsigned long long pp_load(const unsigned long long *p)
{
    unsigned long long v;
    if (MODE == 0) asm volatile("global_load_dwordx2 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    else asm volatile("global_load_dwordx2 %0, %1, off sc0\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}
template <int MODE>
__global__ void k_pp2(unsigned long long *v, unsigned long long *w, int iters, int partner, unsigned long long *out)
{
    if (threadIdx.x != 0) return;
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (blockIdx.x == 0) {
        uint64_t t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < iters; i++) {
            pp_store<MODE>(v + i, (unsigned long long)(i + 1));
            for (long g = 0; g < (1L << 14) && pp_load<MODE>(w + i) != (unsigned long long)(i + 1); g++) {}
        }
        uint64_t t1 = __builtin_amdgcn_s_memtime();
        out[0] = t1 - t0;
        out[2] = xcc;
    } else if ((int)blockIdx.x == partner) {
        for (int i = 0; i < iters; i++) {
            for (long g = 0; g < (1L << 14) && pp_load<MODE>(v + i) != (unsigned long long)(i + 1); g++) {}
            pp_store<MODE>(w + i, (unsigned long long)(i + 1));
        }
        out[3] = xcc;
    }
}

int main()
{
    unsigned long long *d_out;
    CK(hipMalloc(&d_out, 64));
    unsigned long long h[8];
    const int it = 10000;
    k_lds_chase<<<1, 64>>>(it, d_out);
    CK(hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost));
    printf("{\"lds_dep_read_cycles\": %.1f}\n", (double)h[0] / it);
    for (int w : {256, 512, 1024}) {
        k_barrier<<<1, w>>>(it, d_out);
        CK(hipMemcpy(h, d_out, 8, hipMemcpyDeviceToHost));
        printf("{\"barrier_cycles\": %.1f, \"threads\": %d}\n", (double)h[0] / it, w);
    }
    // pointer chase over N elements with a large stride permutation
    for (long N : {1L << 12, 1L << 16, 1L << 20, 1L << 26}) {
        std::vector<long> nx(N);
        const long stride = 4099;  // coprime with powers of two
        for (long i = 0; i < N; i++) nx[i] = (i + stride) % N;
        long *d;
        CK(hipMalloc(&d, N * sizeof(long)));
        CK(hipMemcpy(d, nx.data(), N * sizeof(long), hipMemcpyHostToDevice));
        const int ci = 2000;
        k_chase<0><<<1, 1>>>(d, ci, d_out);
        CK(hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost));
        double cold = (double)h[0] / ci;
        k_chase<0><<<1, 1>>>(d, ci, d_out);
        CK(hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost));
        double plain = (double)h[0] / ci;
        printf("{\"chase_bytes\": %ld, \"cold_cycles\": %.1f}\n", N * 8, cold);
        k_chase<1><<<1, 1>>>(d, ci, d_out);
        CK(hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost));
        printf("{\"chase_bytes\": %ld, \"plain_cycles\": %.1f, \"sc1_cycles\": %.1f}\n", N * 8, plain,
               (double)h[0] / ci);
        CK(hipFree(d));
    }
    unsigned long long *v, *w;
    const int pi = 200;
    CK(hipMalloc(&v, pi * 8));
    CK(hipMalloc(&w, pi * 8));
    for (int partner : {1, 2, 8, 16, 100}) {
        CK(hipMemset(v, 0, pi * 8));
        CK(hipMemset(w, 0, pi * 8));
        CK(hipMemset(d_out, 0, 64));
        k_pingpong<<<256, 64>>>(v, w, pi, partner, d_out);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h, d_out, 32, hipMemcpyDeviceToHost));
        printf("{\"pingpong_round_trip_cycles\": %.1f, \"partner\": %d, \"xcc\": [%llu, %llu]}\n",
               (double)h[0] / pi, partner, h[2], h[3]);
    }

    {
        double *rec, *out;
        CK(hipMalloc(&rec, sizeof(double) * 1024 * 256 * 10 + 4096));
        CK(hipMemset(rec, 0, sizeof(double) * 1024 * 256 * 10));
        CK(hipMalloc(&out, sizeof(double) * (1 << 23)));
        const int si = 4000;
        for (int mode = 0; mode < 4; mode++) {
            for (int g : {1, 216}) {
                if (mode == 0) k_step<0><<<g, 512>>>(rec, out, si, d_out);
                if (mode == 1) k_step<1><<<g, 512>>>(rec, out, si, d_out);
                if (mode == 2) k_step<2><<<g, 512>>>(rec, out, si, d_out);
                if (mode == 3) k_step<3><<<g, 512>>>(rec, out, si, d_out);
                CK(hipDeviceSynchronize());
                CK(hipMemcpy(h, d_out, 8, hipMemcpyDeviceToHost));
                printf("{\"step_floor_cycles\": %.1f, \"mode\": %d, \"grid\": %d}\n", (double)h[0] / si, mode, g);
            }
        }
    }
    for (int mode = 0; mode < 3; mode++)
        for (int partner : {8, 1}) {
            if (mode == 1 && partner == 1) continue;  // plain stores are not visible across XCDs
            CK(hipMemset(v, 0, pi * 8));
            CK(hipMemset(w, 0, pi * 8));
            CK(hipMemset(d_out, 0, 64));
            if (mode == 0) k_pp2<0><<<256, 64>>>(v, w, pi, partner, d_out);
            if (mode == 1) k_pp2<1><<<256, 64>>>(v, w, pi, partner, d_out);
            if (mode == 2) k_pp2<2><<<256, 64>>>(v, w, pi, partner, d_out);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h, d_out, 32, hipMemcpyDeviceToHost));
            printf("{\"pp2_round_trip_cycles\": %.1f, \"mode\": %d, \"partner\": %d, \"xcc\": [%llu, %llu]}\n",
                   (double)h[0] / pi, mode, partner, h[2], h[3]);
            fflush(stdout);
        }
    // s_memtime frequency: compare with wall clock
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    k_lds_chase<<<1, 64>>>(2000000, d_out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost));
    printf("{\"memtime_ghz\": %.3f}\n", (double)h[0] / (ms * 1e6));
    return 0;
}
