// Tuning aid (not product code): issue cost and latency of the f64 operations
// of a triangular-sweep row on gfx950 -- NCH independent chains of dependent
// ops, one wave, s_memtime clocks per op.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off valu_probe.hip -o valu_probe
#include <hip/hip_runtime.h>
#include <cstdio>

template <int NCH, int OP>
__global__ void k(double *out, unsigned long long *cyc, int iters)
{
    double x[NCH], y[NCH];
    for (int c = 0; c < NCH; c++) {
        x[c] = 1.0 + threadIdx.x * 1e-3 + c;
        y[c] = 1.0000001 + c * 1e-9;
    }
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            if (OP == 0) x[c] = x[c] * y[c];
            if (OP == 1) x[c] = x[c] - y[c] * x[c];
            if (OP == 2) x[c] = x[c] / y[c];
        }
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    double s = 0;
    for (int c = 0; c < NCH; c++) s += x[c];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <int NCH, int OP>
void run(double *d, unsigned long long *c)
{
    const int iters = 4096;
    k<NCH, OP><<<1, 64>>>(d, c, iters);
    unsigned long long h = 0;
    (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("{\"op\": \"%s\", \"chains\": %d, \"clk_per_chain_step\": %.1f}\n", OP == 0 ? "mul" : OP == 1 ? "mul+sub" : "div",
           NCH, (double)h / iters);
}

int main()
{
    double *d;
    unsigned long long *c;
    (void)hipMalloc(&d, 8 * 1024);
    (void)hipMalloc(&c, 8);
    run<1, 0>(d, c); run<2, 0>(d, c); run<4, 0>(d, c); run<8, 0>(d, c);
    run<1, 1>(d, c); run<4, 1>(d, c); run<8, 1>(d, c);
    run<1, 2>(d, c); run<2, 2>(d, c); run<4, 2>(d, c); run<8, 2>(d, c);
    return 0;
}
