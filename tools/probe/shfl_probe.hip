// shfl_probe.hip -- checks the lane-16 shift of a 64-bit value built from
// v_permlane16_swap / v_permlane32_swap (gfx950) against ds_bpermute, and
// times both in a dependent chain (the k-input of a line sweep's lane group,
// linesweep.hip k_line2).  Build: hipcc --offload-arch=gfx950 -O3 -o shfl_probe shfl_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ unsigned up16_perm(unsigned x)
{
    auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    auto q = __builtin_amdgcn_permlane32_swap(r[0], r[1], false, false);
    unsigned o;
    asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(o) : "v"(r[0]), "v"(q[0]), "s"(0x0000FFFF00000000ull));
    return o;
}
__device__ __forceinline__ unsigned up16_bperm(unsigned x)
{
    const int lane = threadIdx.x & 63;
    return (unsigned)__builtin_amdgcn_ds_bpermute(((lane - 16) & 63) * 4, (int)x);
}

__global__ void k_check(unsigned *out)
{
    const unsigned x = 1000u + (threadIdx.x & 63) * 7u;
    out[threadIdx.x] = up16_perm(x);
    out[64 + threadIdx.x] = up16_bperm(x);
    auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    out[128 + threadIdx.x] = r[0];
    out[192 + threadIdx.x] = r[1];
}

template <int WHICH>
__global__ void k_chain(double *out, int iters, long long *clk)
{
    double v = threadIdx.x * 1.0;
    const long long t0 = clock64();
    for (int i = 0; i < iters; i++) {
        const long long b = __double_as_longlong(v);
        unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
        if (WHICH == 0) {
            lo = up16_perm(lo);
            hi = up16_perm(hi);
        } else {
            lo = up16_bperm(lo);
            hi = up16_bperm(hi);
        }
        v = __longlong_as_double(((long long)hi << 32) | lo) * 1.0000001 + 0.5;
    }
    const long long t1 = clock64();
    out[threadIdx.x] = v;
    if (threadIdx.x == 0) *clk = t1 - t0;
}

int main()
{
    unsigned *d;
    hipMalloc(&d, 256 * sizeof(unsigned));
    k_check<<<1, 64>>>(d);
    unsigned h[256];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 16; l < 64; l++) {
        const unsigned want = 1000u + (l - 16) * 7u;
        if (h[l] != want || h[64 + l] != want) bad++;
    }
    printf("permlane16_swap(x,x) rows of r[0]:");
    for (int r = 0; r < 4; r++) printf(" %u", (h[128 + 16 * r] - 1000u) / 7u / 16u);
    printf("; r[1]:");
    for (int r = 0; r < 4; r++) printf(" %u", (h[192 + 16 * r] - 1000u) / 7u / 16u);
    printf("\nup16 check: %s (%d bad lanes)\n", bad ? "FAIL" : "ok", bad);
    double *o;
    long long *c;
    hipMalloc(&o, 64 * sizeof(double));
    hipMalloc(&c, sizeof(long long));
    for (int w = 0; w < 2; w++) {
        long long clk = 0;
        for (int rep = 0; rep < 3; rep++) {
            if (w == 0) k_chain<0><<<1, 64>>>(o, 1000, c);
            else k_chain<1><<<1, 64>>>(o, 1000, c);
            hipMemcpy(&clk, c, sizeof(clk), hipMemcpyDeviceToHost);
        }
        printf("%s: %.1f clk per dependent step (incl. one f64 fma-free mul+add)\n", w ? "ds_bpermute" : "permlane",
               clk / 1000.0);
    }
    return bad ? 1 : 0;
}
