// ilu_factor.hip -- ILU(0) numeric factorization on the GPU.
//
// Restates lssp_pc_ilu0_fac (pc-iluk.cxx:347-409), the IKJ elimination the
// reference runs on the host for ILUK(k) on the level-k pattern, operation for
// operation, so the factors are bitwise the reference's:
//   for each strict-lower entry k of row i, ascending:
//       a_ik = a_ik * dinv[c_k]                         (reciprocal pivot, :386)
//       a_ij = a_ij - a_ik * u_kj   for j > k where row c_k holds a NONZERO
//                                   value at column c_j  (:388-390, wk[] != 0)
//   dinv[i] = 1 / a_ii, a tiny pivot replaced first   (:394-399)
// Row i only reads rows c_k < i of its own strict-lower pattern, so rows are
// processed level by level (levels of that DAG, computed on the host; the same
// levels as the L sweep), one lane per row, one launch per level.  Instead of
// the reference's dense scatter array wk[] a lane merges its row with row c_k
// (both sorted): the value wk[c] would hold is the LAST entry of row c_k with
// column c, and an exact zero there skips the update, as the reference's test
// does.  A block-diagonal matrix (block-Jacobi, blk < n) is factored in one
// pass: the first row of every block follows the reference's row-0 rule
// (pivot sign kept, the stored value left untouched, :367-375).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "internal.h"

namespace lssp_amd {

constexpr double ILU_ZERO_DIAG_VALUE = 1e-3;  // pc.cxx:6 (ilu_setup.cpp ZERO_DIAG_VALUE)
constexpr double ILU_ZERO_DIAG_TOL = 1e-10;   // pc.cxx:7

__global__ __launch_bounds__(256) void k_ilu0_level(const int *__restrict__ rows, int cnt, const int *__restrict__ Ap,
                                                    const int *__restrict__ C, double *Ax, double *dinv, int blk)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= cnt) return;
    const int i = rows[t];
    const int s = Ap[i], end = Ap[i + 1];
    if (i % blk == 0) {  // first row of a (block-Jacobi) block
        double d0 = Ax[s];
        if (fabs(d0) < ILU_ZERO_DIAG_TOL) d0 = d0 > 0 ? ILU_ZERO_DIAG_VALUE : -ILU_ZERO_DIAG_VALUE;
        dinv[i] = 1. / d0;
        return;
    }
    int k = s;
    for (; k < end && C[k] < i; k++) {
        const int r = C[k];
        const double aik = Ax[k] * dinv[r];
        Ax[k] = aik;
        int q = Ap[r];
        const int qe = Ap[r + 1];
        for (int j = k + 1; j < end; j++) {
            const int c = C[j];
            while (q < qe && C[q] < c) q++;
            double w = 0.;
            for (int qq = q; qq < qe && C[qq] == c; qq++) w = Ax[qq];  // last duplicate wins, as wk[] does
            if (w != 0.) Ax[j] = Ax[j] - aik * w;
        }
    }
    double d = ILU_ZERO_DIAG_VALUE;
    if (k < end && C[k] == i) {
        if (fabs(Ax[k]) < ILU_ZERO_DIAG_TOL) Ax[k] = ILU_ZERO_DIAG_VALUE;
        d = Ax[k];
    }
    dinv[i] = 1. / d;
}

// In place on the host CSR (sorted rows): upload, level-scheduled launches,
// download of the values.  blk: block size of a block-diagonal matrix (n: one
// block).
int ilu0_factor_gpu(lssp_amd_ctx *c, int n, int blk, const std::vector<int> &Ap, const std::vector<int> &Aj,
                    std::vector<double> &Ax)
{
    if (n <= 0) return LSSP_AMD_OK;
    if (blk <= 0 || blk > n) blk = n;
    const long nnz = Ap[n];
    // levels of the strict-lower DAG; row i waits on rows C[k] < i of its row
    std::vector<int> lev(n, 0);
    int nlev = 0;
    for (int i = 0; i < n; i++) {
        int l = 0;
        for (int k = Ap[i]; k < Ap[i + 1] && Aj[k] < i; k++) l = std::max(l, lev[Aj[k]] + 1);
        lev[i] = l;
        nlev = std::max(nlev, l + 1);
    }
    std::vector<int> off(nlev + 1, 0), rows(n);
    for (int i = 0; i < n; i++) off[lev[i] + 1]++;
    for (int l = 0; l < nlev; l++) off[l + 1] += off[l];
    {
        std::vector<int> fill(off.begin(), off.end() - 1);
        for (int i = 0; i < n; i++) rows[fill[lev[i]]++] = i;
    }
    int *d_Ap = nullptr, *d_Aj = nullptr, *d_rows = nullptr;
    double *d_Ax = nullptr, *d_dinv = nullptr;
    int st = LSSP_AMD_OK;
    auto fail = [&](hipError_t e) {
        if (e != hipSuccess && st == LSSP_AMD_OK) {
            fprintf(stderr, "lssp_amd: HIP error %s in ilu0_factor_gpu\n", hipGetErrorString(e));
            st = LSSP_AMD_EHIP;
        }
    };
    fail(hipMalloc(&d_Ap, sizeof(int) * (n + 1)));
    fail(hipMalloc(&d_Aj, sizeof(int) * std::max<long>(nnz, 1)));
    fail(hipMalloc(&d_Ax, sizeof(double) * std::max<long>(nnz, 1)));
    fail(hipMalloc(&d_rows, sizeof(int) * n));
    fail(hipMalloc(&d_dinv, sizeof(double) * n));
    if (st == LSSP_AMD_OK) {
        fail(hipMemcpyAsync(d_Ap, Ap.data(), sizeof(int) * (n + 1), hipMemcpyHostToDevice, c->stream));
        fail(hipMemcpyAsync(d_Aj, Aj.data(), sizeof(int) * nnz, hipMemcpyHostToDevice, c->stream));
        fail(hipMemcpyAsync(d_Ax, Ax.data(), sizeof(double) * nnz, hipMemcpyHostToDevice, c->stream));
        fail(hipMemcpyAsync(d_rows, rows.data(), sizeof(int) * n, hipMemcpyHostToDevice, c->stream));
    }
    if (st == LSSP_AMD_OK) {
        for (int l = 0; l < nlev; l++) {
            const int cnt = off[l + 1] - off[l];
            k_ilu0_level<<<(cnt + 255) / 256, 256, 0, c->stream>>>(d_rows + off[l], cnt, d_Ap, d_Aj, d_Ax, d_dinv,
                                                                  blk);
        }
        fail(hipGetLastError());
        fail(hipMemcpyAsync(Ax.data(), d_Ax, sizeof(double) * nnz, hipMemcpyDeviceToHost, c->stream));
        fail(hipStreamSynchronize(c->stream));
    }
    for (void *p : {(void *)d_Ap, (void *)d_Aj, (void *)d_Ax, (void *)d_rows, (void *)d_dinv})
        if (p) (void)hipFree(p);
    return st;
}

}  // namespace lssp_amd
