// Dependent-latency probe (tuning aid): one wave runs chains of 1024 dependent
// f64 adds, mul-sub pairs, DPP wave shifts and LDS round trips; prints clocks
// per operation (s_memtime) and the wall time of the whole kernel.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(double *out, unsigned long long *clk, double seed)
{
    __shared__ double lds[64];
    const int lane = threadIdx.x;
    double x = seed + lane, y = 1.0000001;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 1024; i++) x = x + y;  // dependent adds
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 512; i++) x = x - y * x;  // dependent mul + sub pairs
    unsigned long long t2 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 1024; i++) {  // DPP wave_shr:1 of a 64-bit value (2 movs)
        const long long b = __double_as_longlong(x);
        const int lo = __builtin_amdgcn_update_dpp((int)b, (int)b, 0x138, 0xf, 0xf, false);
        const int hi = __builtin_amdgcn_update_dpp((int)(b >> 32), (int)(b >> 32), 0x138, 0xf, 0xf, false);
        x = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
    }
    unsigned long long t3 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 256; i++) {  // LDS write + read round trip
        lds[lane] = x;
        __builtin_amdgcn_s_waitcnt(0xc07f);
        x = lds[(lane + 1) & 63] + 1.0;
    }
    unsigned long long t4 = __builtin_amdgcn_s_memtime();
    out[lane] = x;
    if (lane == 0) {
        clk[0] = t1 - t0;
        clk[1] = t2 - t1;
        clk[2] = t3 - t2;
        clk[3] = t4 - t3;
    }
}

int main()
{
    double *out;
    unsigned long long *clk, h[4];
    hipMalloc(&out, 64 * sizeof(double));
    hipMalloc(&clk, 4 * sizeof(unsigned long long));
    for (int rep = 0; rep < 3; rep++) {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0);
        probe<<<1, 64>>>(out, clk, 1.0);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
        printf("{\"add_clk\": %.1f, \"mulsub_pair_clk\": %.1f, \"dpp64_clk\": %.1f, \"lds_rt_clk\": %.1f, \"kernel_us\": %.1f}\n",
               h[0] / 1024.0, h[1] / 512.0, h[2] / 1024.0, h[3] / 256.0, ms * 1000.0);
    }
    return 0;
}
