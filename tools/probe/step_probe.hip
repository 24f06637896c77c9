// Tuning aid (not product code): cycles per step of a line-sweep-like compute
// body -- LDS operand reads, two planes of the row recurrence (3 multiply-adds
// + a division), the DPP lane shift, the result written to LDS, a barrier --
// with parts switched off by MODE bits, for 1..9 waves per workgroup.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off step_probe.hip -o step_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ double dpp_shr1(double v, double old)
{
    const long long b = __double_as_longlong(v), o = __double_as_longlong(old);
    const int lo = __builtin_amdgcn_update_dpp((int)o, (int)b, 0x138, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(b >> 32), 0x138, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ void bar()
{
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// MODE: 1 LDS operand reads, 2 division, 4 barrier, 8 second plane, 16 dpp
template <int MODE>
__global__ void probe(double *out, unsigned long long *cyc, int iters)
{
    __shared__ double lds[4096];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) lds[i] = 1.0 + 1e-3 * (i & 63);
    __syncthreads();
    double x0 = 1.0 + lane, x1 = 2.0 + lane;
    double c[8], r[2];
    for (int k = 0; k < 8; k++) c[k] = 0.25 + 0.01 * k;
    r[0] = 1.5; r[1] = 2.5;
    const unsigned long long t0 = __builtin_readcyclecounter();
    if (wave == 0) {
        for (int it = 0; it < iters; it++) {
            double kx = 0.5;
            if (MODE & 1) {
                const int o = (it & 7) * 512;
                kx = lds[o + lane];
                for (int k = 0; k < 8; k++) c[k] = lds[o + 64 + 8 * lane + k];
                r[0] = lds[o + 256 + lane];
                r[1] = lds[o + 320 + lane];
            }
            double xj1 = (MODE & 16) ? dpp_shr1(x1, 0.0) : x1;
            double v1 = r[1] - c[0] * x0;
            v1 = v1 - c[1] * xj1;
            v1 = v1 - c[2] * x1;
            if (MODE & 2) v1 = v1 / c[3];
            double v0 = x0;
            if (MODE & 8) {
                double xj0 = (MODE & 16) ? dpp_shr1(x0, 0.0) : x0;
                v0 = r[0] - c[4] * kx;
                v0 = v0 - c[5] * xj0;
                v0 = v0 - c[6] * x0;
                if (MODE & 2) v0 = v0 / c[7];
            }
            x1 = v1;
            x0 = v0;
            lds[3584 + lane] = x0;
            if (MODE & 4) bar();
        }
    } else {
        for (int it = 0; it < iters; it++)
            if (MODE & 4) bar();
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    out[threadIdx.x] = x0 + x1;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <int MODE>
void run(int waves, double *d, unsigned long long *c)
{
    const int iters = 4096;
    probe<MODE><<<1, 64 * waves>>>(d, c, iters);
    unsigned long long h;
    hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("{\"mode\": %d, \"waves\": %d, \"clk_per_step\": %.1f}\n", MODE, waves, (double)h / iters);
}

int main()
{
    double *d;
    unsigned long long *c;
    hipMalloc(&d, 8 * 1024);
    hipMalloc(&c, 8);
    for (int w : {1, 9}) {
        run<0>(w, d, c);
        run<4>(w, d, c);
        run<4 | 16>(w, d, c);
        run<4 | 16 | 8>(w, d, c);
        run<4 | 16 | 8 | 2>(w, d, c);
        run<4 | 16 | 8 | 2 | 1>(w, d, c);
        run<16 | 8 | 2 | 1>(w, d, c);
        run<16 | 8 | 2>(w, d, c);
        run<8 | 2>(w, d, c);
        run<2>(w, d, c);
    }
    return 0;
}
