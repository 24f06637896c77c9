// handoff_probe.hip -- tuning aid (not part of the library): round trip of a
// cross-CU value hand-off between two workgroups, by store / load cache policy,
// same-XCD and cross-XCD partners, on an idle chip and beside an HBM stream
// (the other workgroups copying 1 GiB), to price the line sweeps' k-hand-off.
//   hipcc -O3 --offload-arch=gfx950 handoff_probe.hip -o handoff_probe
// Store policies: 0 plain (the line stays in the XCD's L2), 1 sc1 (write-through,
// the line leaves L2).  Load policies: 0 sc1, 1 nt (both bypass L1).  Every
// poll loop is bounded, so a combination that never sees the value (plain
// store, cross-XCD) ends with a count of misses instead of a hang.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__);          \
            return 1;                                                             \
        }                                                                         \
    } while (0)

template <int ST>
__device__ __forceinline__ void st(unsigned long long *p, unsigned long long v)
{
    if (ST == 0) asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
template <int LD>
__device__ __forceinline__ unsigned long long ld(const unsigned long long *p)
{
    unsigned long long v;
    if (LD == 0) asm volatile("global_load_dwordx2 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    else asm volatile("global_load_dwordx2 %0, %1, off nt\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}

// block 0 and block `partner` ping-pong; every other block streams src -> dst
// when stream != 0 (grid-strided 16-byte copies) until block 0 is done
template <int ST, int LD>
__global__ void k_pp(unsigned long long *v, unsigned long long *w, int iters, int partner, int stream,
                     const double4 *src, double4 *dst, long n4, volatile int *done, unsigned long long *out)
{
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if ((int)blockIdx.x != 0 && (int)blockIdx.x != partner) {
        if (!stream) return;
        for (int rep = 0; rep < 64 && !*done; rep++)
            for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
                dst[i] = src[i];
        return;
    }
    if (threadIdx.x != 0) return;
    unsigned misses = 0;
    if (blockIdx.x == 0) {
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < iters; i++) {
            st<ST>(v + i, (unsigned long long)(i + 1));
            long g = 0;
            for (; g < (1L << 16) && ld<LD>(w + i) != (unsigned long long)(i + 1); g++) {}
            misses += g == (1L << 16);
        }
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        out[0] = t1 - t0;
        out[2] = xcc;
        out[4] = misses;
        *done = 1;
    } else {
        for (int i = 0; i < iters; i++) {
            long g = 0;
            for (; g < (1L << 16) && ld<LD>(v + i) != (unsigned long long)(i + 1); g++) {}
            misses += g == (1L << 16);
            st<ST>(w + i, (unsigned long long)(i + 1));
        }
        out[3] = xcc;
        out[5] = misses;
    }
}

template <int ST, int LD>
static int run(int partner, int stream, unsigned long long *v, unsigned long long *w, const double4 *src, double4 *dst,
               long n4, int *done, unsigned long long *d_out)
{
    const int it = 500;
    CK(hipMemset(v, 0, it * 8));
    CK(hipMemset(w, 0, it * 8));
    CK(hipMemset(d_out, 0, 64));
    CK(hipMemset(done, 0, 4));
    k_pp<ST, LD><<<256, 256>>>(v, w, it, partner, stream, src, dst, n4, done, d_out);
    CK(hipDeviceSynchronize());
    unsigned long long h[8];
    CK(hipMemcpy(h, d_out, 64, hipMemcpyDeviceToHost));
    printf("{\"store\": \"%s\", \"load\": \"%s\", \"partner\": %d, \"xcc\": [%llu, %llu], \"stream\": %d, "
           "\"round_trip_clk\": %.1f, \"misses\": [%llu, %llu]}\n",
           ST ? "sc1" : "plain", LD ? "nt" : "sc1", partner, h[2], h[3], stream, (double)h[0] / it, h[4], h[5]);
    fflush(stdout);
    return 0;
}

int main()
{
    unsigned long long *v, *w, *d_out;
    int *done;
    const long n4 = (1L << 30) / 32;  // 1 GiB of double4
    double4 *src, *dst;
    CK(hipMalloc(&v, 4096));
    CK(hipMalloc(&w, 4096));
    CK(hipMalloc(&d_out, 64));
    CK(hipMalloc(&done, 4));
    CK(hipMalloc(&src, n4 * 32));
    CK(hipMalloc(&dst, n4 * 32));
    CK(hipMemset(src, 0, n4 * 32));
    for (int stream : {0, 1})
        for (int partner : {8, 1}) {  // blocks b and b + 8 share an XCD under round-robin placement
            if (run<1, 0>(partner, stream, v, w, src, dst, n4, done, d_out)) return 1;
            if (run<1, 1>(partner, stream, v, w, src, dst, n4, done, d_out)) return 1;
            if (partner == 8) {  // plain stores are visible in the producer's XCD only
                if (run<0, 0>(partner, stream, v, w, src, dst, n4, done, d_out)) return 1;
                if (run<0, 1>(partner, stream, v, w, src, dst, n4, done, d_out)) return 1;
            }
        }
    return 0;
}
