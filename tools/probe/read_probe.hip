// read_probe.hip -- HBM streaming-read rate of 16-byte loads over 1 GiB, by
// load policy (plain / non-temporal), loads in flight per lane and grid size:
// picks the form of lssp_amd_stream_read (kernels.hip k_read16).
// Build: hipcc --offload-arch=gfx950 -O3 -o read_probe read_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d2 __attribute__((ext_vector_type(2)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_read(const d2 *__restrict__ s, long n2, unsigned long long *sink)
{
    const long stride = (long)gridDim.x * 256;
    unsigned long long acc = 0;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n2; i += U * stride) {
        d2 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const long k = i + u * stride;
            v[u] = k < n2 ? (NT ? __builtin_nontemporal_load(s + k) : s[k]) : d2{0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; u++) acc ^= (unsigned long long)__double_as_longlong(v[u][0]) ^
                                           (unsigned long long)__double_as_longlong(v[u][1]);
    }
    if (acc == 0x123456789ull) *sink = acc;
}

// contiguous chunk per block (each block streams its own range)
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_read_chunk(const d2 *__restrict__ s, long n2, unsigned long long *sink)
{
    const long per = (n2 + gridDim.x - 1) / gridDim.x;
    const long b0 = (long)blockIdx.x * per, b1 = b0 + per < n2 ? b0 + per : n2;
    unsigned long long acc = 0;
    for (long i = b0 + threadIdx.x; i < b1; i += U * 256) {
        d2 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const long k = i + u * 256;
            v[u] = k < b1 ? (NT ? __builtin_nontemporal_load(s + k) : s[k]) : d2{0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; u++) acc ^= (unsigned long long)__double_as_longlong(v[u][0]) ^
                                           (unsigned long long)__double_as_longlong(v[u][1]);
    }
    if (acc == 0x123456789ull) *sink = acc;
}

template <class K>
static double run(K k, int grid, const d2 *s, long n2, unsigned long long *sink)
{
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int i = 0; i < 3; i++) k<<<grid, 256>>>(s, n2, sink);
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
        (void)hipEventRecord(e0);
        for (int i = 0; i < 10; i++) k<<<grid, 256>>>(s, n2, sink);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    return 16.0 * n2 / (best / 10 * 1e-3) / 1e9;
}

int main()
{
    const long n2 = (1L << 27) / 2;  // 1 GiB of doubles
    d2 *s;
    unsigned long long *sink;
    if (hipMalloc(&s, 16 * n2) != hipSuccess || hipMalloc(&sink, 8) != hipSuccess) return 1;
    (void)hipMemset(s, 1, 16 * n2);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (int gm : {4, 8, 16, 32}) {
        const int grid = gm * cus;
        printf("grid %4d x CUs: stride U4 %.0f  U8 %.0f  U16 %.0f | nt U4 %.0f  U8 %.0f  U16 %.0f | chunk U4 %.0f U8 %.0f | "
               "chunk nt U4 %.0f U8 %.0f GB/s\n", gm, run(k_read<4, false>, grid, s, n2, sink),
               run(k_read<8, false>, grid, s, n2, sink), run(k_read<16, false>, grid, s, n2, sink),
               run(k_read<4, true>, grid, s, n2, sink), run(k_read<8, true>, grid, s, n2, sink),
               run(k_read<16, true>, grid, s, n2, sink), run(k_read_chunk<4, false>, grid, s, n2, sink),
               run(k_read_chunk<8, false>, grid, s, n2, sink), run(k_read_chunk<4, true>, grid, s, n2, sink),
               run(k_read_chunk<8, true>, grid, s, n2, sink));
    }
    return 0;
}
