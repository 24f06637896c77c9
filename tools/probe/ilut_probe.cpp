// ilut_probe.cpp -- tuning aid (not part of the library): times the host ILUT
// numeric factorization (ilu_setup.cpp ilut_factor_lu, pc-ilut.cxx:51-286) on a
// 7-pt Poisson N^3 matrix and prints a checksum of the factor (variants must
// keep it bit for bit).
//   make -C lssp_amd/csrc && hipcc -O2 -std=c++17 -I include -I /opt/rocm/include \
//     tools/probe/ilut_probe.cpp $(ls lssp_amd/lib/obj/*.o | grep -v ilu_setup) -lrccl -o /tmp/ilut_probe
#include "../../lssp_amd/csrc/ilu_setup.cpp"

#include <chrono>

int main(int argc, char **argv)
{
    using namespace lssp_amd;
    const int N = argc > 1 ? atoi(argv[1]) : 96;
    const int n = N * N * N;
    HostCSR A;
    A.n = A.ncols = n;
    A.Ap.assign(n + 1, 0);
    for (int k = 0; k < N; k++)
        for (int j = 0; j < N; j++)
            for (int i = 0; i < N; i++) {
                const int r = (k * N + j) * N + i;
                auto add = [&](int c, double v) {
                    A.Aj.push_back(c);
                    A.Ax.push_back(v);
                };
                if (k > 0) add(r - N * N, -1);
                if (j > 0) add(r - N, -1);
                if (i > 0) add(r - 1, -1);
                add(r, 6);
                if (i < N - 1) add(r + 1, -1);
                if (j < N - 1) add(r + N, -1);
                if (k < N - 1) add(r + N * N, -1);
                A.Ap[r + 1] = (int)A.Aj.size();
            }
    const auto t0 = std::chrono::steady_clock::now();
    HostCSR L, U;
    ilut_factor_lu(A, 1e-4, 20, L, U);
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    uint64_t h = 1469598103934665603ull;
    for (const HostCSR *F : {&L, &U})
        for (size_t k = 0; k < F->Aj.size(); k++) {
            uint64_t b;
            memcpy(&b, &F->Ax[k], 8);
            h = (h ^ b ^ (uint64_t)F->Aj[k]) * 1099511628211ull;
        }
    printf("N %d n %d nnz %zu ilut %.3f s hash %016llx\n", N, n, L.Aj.size() + U.Aj.size(), s, (unsigned long long)h);
    return 0;
}
