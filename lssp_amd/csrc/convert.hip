// convert.hip -- sparse format conversions on the device.
//
// lssp_mat_csr_to_coo / _coo_to_csr / _transpose / _csr_to_bcsr /
// _bcsr_to_csr (matrix-utils.cxx:62-380, :700-765) for matrices that already
// live in HBM.  All of it is integer / byte movement: no arithmetic on the
// values, so every result is bitwise the reference's, entry order included.
//
// The reference orders entries with counting sorts whose sequential loops
// make them STABLE (coo_to_csr keeps the input order inside a row, transpose
// the row order inside a column).  On the GPU the same orders come from
// stable LSD radix sorts (rocPRIM's device radix sort, keys limited to the bits
// the row / column range needs) of (key, entry index) pairs followed by a
// coalesced gather, and row pointers are lower bounds in the sorted keys.
// Block patterns (csr_to_bcsr) come from one radix sort of packed
// (block row, block column) 64-bit keys and a flag / scan / scatter unique.
// Work where ONE row's entries are written in the reference's sequential
// order (duplicate (r, c) in csr_to_bcsr: last value wins; bcsr_to_csr rows
// in block order) is done by one thread per row, so the order is the same
// by construction.  These kernels are HBM-bound streaming passes; none of
// them is on the solve path.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cstdint>
#include <vector>

#include "internal.h"

namespace {

constexpr int CT = 256;  // threads per block (4 waves)

unsigned grid_for(long n)
{
    long b = (n + CT - 1) / CT;
    return (unsigned)std::max<long>(1, std::min<long>(b, 16384));
}

#define GRID_STRIDE(i, n) for (long i = blockIdx.x * (long)CT + threadIdx.x; i < (n); i += (long)gridDim.x * CT)

int bits_for(unsigned long v)  // bits needed to hold every value in [0, v]
{
    int b = 1;
    while (b < 64 && (v >> b) != 0) b++;
    return b;
}

// Ap[0] == 0, non-decreasing, Ap[nrows] == nnz: afterwards every per-row loop
// stays inside [0, nnz)
__global__ __launch_bounds__(CT) void k_check_ptr(long nrows, int nnz, const int *__restrict__ Ap,
                                                  int *__restrict__ err)
{
    GRID_STRIDE(i, nrows + 1)
    {
        int a = Ap[i];
        bool bad = (i == 0 && a != 0) || (i == nrows && a != nnz) || (i < nrows && Ap[i + 1] < a);
        if (bad) atomicOr(err, 1);
    }
}

__global__ __launch_bounds__(CT) void k_check_idx(long n, const int *__restrict__ v, int lim,
                                                  int *__restrict__ err)
{
    GRID_STRIDE(i, n)
    {
        if ((unsigned)v[i] >= (unsigned)lim) atomicOr(err, 1);
    }
}

// matrix-utils.cxx:287-294: the row of every entry
__global__ __launch_bounds__(CT) void k_expand_rows(long nrows, const int *__restrict__ Ap,
                                                    int *__restrict__ Ci)
{
    GRID_STRIDE(i, nrows)
    {
        int e = Ap[i + 1];
        for (int k = Ap[i]; k < e; k++) Ci[k] = (int)i;
    }
}

__global__ __launch_bounds__(CT) void k_iota(long n, int *__restrict__ v)
{
    GRID_STRIDE(i, n) v[i] = (int)i;
}

// P[r] = first position whose key is >= r, r = 0..nr: the row pointers of
// entries sorted by row (empty rows included)
__global__ __launch_bounds__(CT) void k_row_ptr(long nr, const unsigned *__restrict__ key, int nkeys,
                                                int *__restrict__ P)
{
    GRID_STRIDE(r, nr + 1)
    {
        int lo = 0, hi = nkeys;
        while (lo < hi) {
            int mid = (int)(((unsigned)lo + (unsigned)hi) >> 1);
            if (key[mid] < (unsigned long)r)
                lo = mid + 1;
            else
                hi = mid;
        }
        P[r] = lo;
    }
}

__global__ __launch_bounds__(CT) void k_gather(long n, const int *__restrict__ perm, const int *__restrict__ sj,
                                               const double *__restrict__ sx, int *__restrict__ dj,
                                               double *__restrict__ dx)
{
    GRID_STRIDE(i, n)
    {
        int k = perm[i];
        dj[i] = sj[k];
        dx[i] = sx[k];
    }
}

// csr_to_bcsr: (block row << cbits) | block column of every entry
__global__ __launch_bounds__(CT) void k_block_keys(long n, int bs, int cbits, const int *__restrict__ Ap,
                                                   const int *__restrict__ Aj, uint64_t *__restrict__ key)
{
    GRID_STRIDE(i, n)
    {
        uint64_t hi = (uint64_t)(i / bs) << cbits;
        int e = Ap[i + 1];
        for (int k = Ap[i]; k < e; k++) key[k] = hi | (uint64_t)(unsigned)(Aj[k] / bs);
    }
}

__global__ __launch_bounds__(CT) void k_unique_flag(long n, const uint64_t *__restrict__ key, int *__restrict__ flag)
{
    GRID_STRIDE(i, n) flag[i] = (i == 0 || key[i] != key[i - 1]) ? 1 : 0;
}

__global__ __launch_bounds__(CT) void k_unique_put(long n, const uint64_t *__restrict__ key,
                                                   const int *__restrict__ flag, const int *__restrict__ pos,
                                                   int cbits, int *__restrict__ Bj, unsigned *__restrict__ brow)
{
    GRID_STRIDE(i, n)
    {
        if (flag[i]) {
            uint64_t k = key[i];
            Bj[pos[i]] = (int)(k & ((1ull << cbits) - 1));
            brow[pos[i]] = (unsigned)(k >> cbits);
        }
    }
}

// matrix-utils.cxx:125-156: one thread per CSR row writes its entries in
// order into the zeroed column-major blocks, so a duplicate keeps its last value
__global__ __launch_bounds__(CT) void k_bcsr_fill(long n, int bs, const int *__restrict__ Ap,
                                                  const int *__restrict__ Aj, const double *__restrict__ Ax,
                                                  const int *__restrict__ Bp, const int *__restrict__ Bj,
                                                  double *__restrict__ Bx)
{
    GRID_STRIDE(i, n)
    {
        int ib = (int)(i / bs), ro = (int)(i % bs);
        int b0 = Bp[ib], b1 = Bp[ib + 1];
        int e = Ap[i + 1];
        for (int k = Ap[i]; k < e; k++) {
            int c = Aj[k], bc = c / bs;
            int lo = b0, hi = b1 - 1;  // bc is in the block row's pattern by construction
            while (lo < hi) {
                int mid = (lo + hi) >> 1;
                if (Bj[mid] < bc)
                    lo = mid + 1;
                else
                    hi = mid;
            }
            Bx[(long)lo * bs * bs + (long)(c % bs) * bs + ro] = Ax[k];
        }
    }
}

// bcsr_to_csr (matrix-utils.cxx:185-203): entries of output row i with
// fabs(v) > 0, in block order then block-column offset
__global__ __launch_bounds__(CT) void k_bcsr_count(long n, int bs, const int *__restrict__ Bp,
                                                   const double *__restrict__ Bx, int *__restrict__ cnt)
{
    GRID_STRIDE(i, n)
    {
        int ib = (int)(i / bs), ro = (int)(i % bs), c = 0;
        for (int t = Bp[ib]; t < Bp[ib + 1]; t++) {
            const double *b = Bx + (long)t * bs * bs + ro;
            for (int co = 0; co < bs; co++) c += fabs(b[(long)co * bs]) > 0. ? 1 : 0;
        }
        cnt[i] = c;
    }
}

// fill row i, then lssp_mat_sort_column (matrix-utils.cxx:434-471) on it: a
// row with an inversion is sorted by column and every occurrence of a
// column takes the value stored last for it (the dense row[] buffer there);
// a stable insertion sort keeps equal columns in their original order, so
// that value is the last of each run
__global__ __launch_bounds__(CT) void k_bcsr_rows(long n, int bs, const int *__restrict__ Bp,
                                                  const int *__restrict__ Bj, const double *__restrict__ Bx,
                                                  const int *__restrict__ Ap, int *__restrict__ Aj,
                                                  double *__restrict__ Ax)
{
    GRID_STRIDE(i, n)
    {
        int ib = (int)(i / bs), ro = (int)(i % bs);
        int o = Ap[i], s = o;
        bool sorted = true;
        for (int t = Bp[ib]; t < Bp[ib + 1]; t++) {
            const double *b = Bx + (long)t * bs * bs + ro;
            int c0 = Bj[t] * bs;
            for (int co = 0; co < bs; co++) {
                double v = b[(long)co * bs];
                if (fabs(v) > 0.) {
                    if (o > s && Aj[o - 1] > c0 + co) sorted = false;
                    Aj[o] = c0 + co;
                    Ax[o] = v;
                    o++;
                }
            }
        }
        if (sorted) continue;
        for (int a = s + 1; a < o; a++) {
            int c = Aj[a];
            double v = Ax[a];
            int b = a - 1;
            while (b >= s && Aj[b] > c) {
                Aj[b + 1] = Aj[b];
                Ax[b + 1] = Ax[b];
                b--;
            }
            Aj[b + 1] = c;
            Ax[b + 1] = v;
        }
        for (int a = o - 1; a > s; a--)
            if (Aj[a - 1] == Aj[a]) Ax[a - 1] = Ax[a];
    }
}

// temporary device memory of one call, released after the stream drains
struct Scratch {
    hipStream_t s;
    std::vector<void *> p;
    explicit Scratch(hipStream_t st) : s(st) {}
    template <class T>
    T *get(long count)
    {
        void *q = nullptr;
        if (hipMalloc(&q, std::max<size_t>(sizeof(T) * (size_t)std::max<long>(count, 1), 16)) != hipSuccess)
            return nullptr;
        p.push_back(q);
        return (T *)q;
    }
    ~Scratch()
    {
        (void)hipStreamSynchronize(s);
        for (void *q : p) (void)hipFree(q);
    }
};

#define SCRATCH(var, T, count)                         \
    T *var = S.get<T>(count);                          \
    if (!var) return LSSP_AMD_ENOMEM

int fetch(hipStream_t s, const int *d, int *h)
{
    LSSP_HIP(hipMemcpyAsync(h, d, sizeof(int), hipMemcpyDeviceToHost, s));
    LSSP_HIP(hipStreamSynchronize(s));
    return LSSP_AMD_OK;
}

// run the structure checks queued on err and report
int checked(hipStream_t s, const int *err)
{
    int h = 0;
    int st = fetch(s, err, &h);
    if (st) return st;
    return h ? LSSP_AMD_EINVAL : LSSP_AMD_OK;
}

// rocPRIM's device-wide primitives (the library's own API): the LSD radix
// sort is stable, which is what reproduces the reference's counting sorts
template <class K, class V>
int sort_pairs(Scratch &S, const K *kin, K *kout, const V *vin, V *vout, long n, int bits)
{
    size_t bytes = 0;
    LSSP_HIP(rocprim::radix_sort_pairs(nullptr, bytes, kin, kout, vin, vout, (size_t)n, 0u, (unsigned)bits, S.s));
    SCRATCH(t, char, (long)bytes);
    LSSP_HIP(rocprim::radix_sort_pairs(t, bytes, kin, kout, vin, vout, (size_t)n, 0u, (unsigned)bits, S.s));
    return LSSP_AMD_OK;
}

template <class K>
int sort_keys(Scratch &S, const K *kin, K *kout, long n, int bits)
{
    size_t bytes = 0;
    LSSP_HIP(rocprim::radix_sort_keys(nullptr, bytes, kin, kout, (size_t)n, 0u, (unsigned)bits, S.s));
    SCRATCH(t, char, (long)bytes);
    LSSP_HIP(rocprim::radix_sort_keys(t, bytes, kin, kout, (size_t)n, 0u, (unsigned)bits, S.s));
    return LSSP_AMD_OK;
}

int exclusive_sum(Scratch &S, const int *in, int *out, long n)
{
    size_t bytes = 0;
    LSSP_HIP(rocprim::exclusive_scan(nullptr, bytes, in, out, 0, (size_t)n, rocprim::plus<int>(), S.s));
    SCRATCH(t, char, (long)bytes);
    LSSP_HIP(rocprim::exclusive_scan(t, bytes, in, out, 0, (size_t)n, rocprim::plus<int>(), S.s));
    return LSSP_AMD_OK;
}

#define TRY(x)                     \
    do {                           \
        int st_ = (x);             \
        if (st_) return st_;       \
    } while (0)

// entries (key[k], value k) stably sorted by key, then row pointers over
// [0, nr] and the gathered (sj, sx): the counting sorts of coo_to_csr and
// transpose
int bucket(Scratch &S, long nnz, const int *key, int nr, const int *sj, const double *sx, int *P, int *dj,
           double *dx)
{
    hipStream_t s = S.s;
    SCRATCH(idx, int, nnz);
    SCRATCH(perm, int, nnz);
    SCRATCH(skey, unsigned, nnz);
    k_iota<<<grid_for(nnz), CT, 0, s>>>(nnz, idx);
    TRY(sort_pairs(S, (const unsigned *)key, skey, (const int *)idx, perm, nnz, bits_for((unsigned)std::max(nr - 1, 0))));
    k_row_ptr<<<grid_for((long)nr + 1), CT, 0, s>>>(nr, skey, (int)nnz, P);
    k_gather<<<grid_for(nnz), CT, 0, s>>>(nnz, perm, sj, sx, dj, dx);
    LSSP_HIP(hipGetLastError());
    return LSSP_AMD_OK;
}

}  // namespace

extern "C" {

int lssp_amd_idx_alloc(lssp_amd_ctx *c, long n, int **d)
{
    if (!c || !d || n < 0) return LSSP_AMD_EINVAL;
    if (hipMalloc(d, sizeof(int) * std::max<long>(n, 1)) != hipSuccess) return LSSP_AMD_ENOMEM;
    return LSSP_AMD_OK;
}

int lssp_amd_idx_free(lssp_amd_ctx *c, int *d)
{
    if (!c) return LSSP_AMD_EINVAL;
    LSSP_HIP(hipStreamSynchronize(c->stream));
    if (d) LSSP_HIP(hipFree(d));
    return LSSP_AMD_OK;
}

int lssp_amd_idx_upload(lssp_amd_ctx *c, int *d, const int *h, long n)
{
    if (!c || n < 0 || (n > 0 && (!d || !h))) return LSSP_AMD_EINVAL;
    if (n == 0) return LSSP_AMD_OK;
    LSSP_HIP(hipMemcpyAsync(d, h, sizeof(int) * n, hipMemcpyHostToDevice, c->stream));
    LSSP_HIP(hipStreamSynchronize(c->stream));
    return LSSP_AMD_OK;
}

int lssp_amd_idx_download(lssp_amd_ctx *c, int *h, const int *d, long n)
{
    if (!c || n < 0 || (n > 0 && (!d || !h))) return LSSP_AMD_EINVAL;
    if (n == 0) return LSSP_AMD_OK;
    LSSP_HIP(hipMemcpyAsync(h, d, sizeof(int) * n, hipMemcpyDeviceToHost, c->stream));
    LSSP_HIP(hipStreamSynchronize(c->stream));
    return LSSP_AMD_OK;
}

// matrix-utils.cxx:281-322
int lssp_amd_csr_to_coo(lssp_amd_ctx *c, int nrows, int nnz, const int *Ap, const int *Aj, const double *Ax,
                        int *Ci, int *Cj, double *Cx)
{
    if (!c || nrows < 0 || nnz < 0 || !Ap || (nnz > 0 && (!Aj || !Ax || !Ci))) return LSSP_AMD_EINVAL;
    hipStream_t s = c->stream;
    Scratch S(s);
    SCRATCH(err, int, 1);
    LSSP_HIP(hipMemsetAsync(err, 0, sizeof(int), s));
    k_check_ptr<<<grid_for((long)nrows + 1), CT, 0, s>>>(nrows, nnz, Ap, err);
    TRY(checked(s, err));
    if (nnz == 0) return LSSP_AMD_OK;
    k_expand_rows<<<grid_for(nrows), CT, 0, s>>>(nrows, Ap, Ci);
    LSSP_HIP(hipGetLastError());
    if (Cj) LSSP_HIP(hipMemcpyAsync(Cj, Aj, sizeof(int) * (size_t)nnz, hipMemcpyDeviceToDevice, s));
    if (Cx) LSSP_HIP(hipMemcpyAsync(Cx, Ax, sizeof(double) * (size_t)nnz, hipMemcpyDeviceToDevice, s));
    LSSP_HIP(hipStreamSynchronize(s));
    return LSSP_AMD_OK;
}

// matrix-utils.cxx:324-380
int lssp_amd_coo_to_csr(lssp_amd_ctx *c, int nrows, int nnz, const int *Ci, const int *Cj, const double *Cx,
                        int *Ap, int *Aj, double *Ax)
{
    if (!c || nrows < 0 || nnz < 0 || !Ap || (nnz > 0 && (!Ci || !Cj || !Cx || !Aj || !Ax)))
        return LSSP_AMD_EINVAL;
    hipStream_t s = c->stream;
    Scratch S(s);
    if (nnz == 0) {
        LSSP_HIP(hipMemsetAsync(Ap, 0, sizeof(int) * ((size_t)nrows + 1), s));
        LSSP_HIP(hipStreamSynchronize(s));
        return LSSP_AMD_OK;
    }
    SCRATCH(err, int, 1);
    LSSP_HIP(hipMemsetAsync(err, 0, sizeof(int), s));
    k_check_idx<<<grid_for(nnz), CT, 0, s>>>(nnz, Ci, nrows, err);
    TRY(checked(s, err));
    TRY(bucket(S, nnz, Ci, nrows, Cj, Cx, Ap, Aj, Ax));
    LSSP_HIP(hipStreamSynchronize(s));
    return LSSP_AMD_OK;
}

// matrix-utils.cxx:700-765
int lssp_amd_csr_transpose(lssp_amd_ctx *c, int nrows, int ncols, int nnz, const int *Ap, const int *Aj,
                           const double *Ax, int *Tp, int *Tj, double *Tx)
{
    if (!c || nrows <= 0 || ncols <= 0 || nnz < 0 || !Ap || !Tp || (nnz > 0 && (!Aj || !Ax || !Tj || !Tx)))
        return LSSP_AMD_EINVAL;
    hipStream_t s = c->stream;
    Scratch S(s);
    SCRATCH(err, int, 1);
    LSSP_HIP(hipMemsetAsync(err, 0, sizeof(int), s));
    k_check_ptr<<<grid_for((long)nrows + 1), CT, 0, s>>>(nrows, nnz, Ap, err);
    if (nnz > 0) k_check_idx<<<grid_for(nnz), CT, 0, s>>>(nnz, Aj, ncols, err);
    TRY(checked(s, err));
    if (nnz == 0) {
        LSSP_HIP(hipMemsetAsync(Tp, 0, sizeof(int) * ((size_t)ncols + 1), s));
        LSSP_HIP(hipStreamSynchronize(s));
        return LSSP_AMD_OK;
    }
    SCRATCH(Ci, int, nnz);
    k_expand_rows<<<grid_for(nrows), CT, 0, s>>>(nrows, Ap, Ci);
    TRY(bucket(S, nnz, Aj, ncols, Ci, Ax, Tp, Tj, Tx));
    LSSP_HIP(hipStreamSynchronize(s));
    return LSSP_AMD_OK;
}

// matrix-utils.cxx:62-162
int lssp_amd_csr_to_bcsr(lssp_amd_ctx *c, int n, int nnz, int bs, const int *Ap, const int *Aj,
                         const double *Ax, int *bnnz, int *Bp, int *Bj, double *Bx)
{
    if (!c || n <= 0 || nnz <= 0 || bs <= 0 || n % bs != 0 || !Ap || !Aj || !bnnz) return LSSP_AMD_EINVAL;
    if (Bj && (!Bp || !Bx || !Ax)) return LSSP_AMD_EINVAL;
    hipStream_t s = c->stream;
    Scratch S(s);
    SCRATCH(err, int, 1);
    LSSP_HIP(hipMemsetAsync(err, 0, sizeof(int), s));
    k_check_ptr<<<grid_for((long)n + 1), CT, 0, s>>>(n, nnz, Ap, err);
    k_check_idx<<<grid_for(nnz), CT, 0, s>>>(nnz, Aj, n, err);
    TRY(checked(s, err));
    int nb = n / bs;
    int cbits = bits_for((unsigned)(nb - 1)), rbits = bits_for((unsigned)(nb - 1));
    SCRATCH(key, uint64_t, nnz);
    SCRATCH(skey, uint64_t, nnz);
    SCRATCH(flag, int, nnz);
    SCRATCH(pos, int, nnz);
    k_block_keys<<<grid_for(n), CT, 0, s>>>(n, bs, cbits, Ap, Aj, key);
    TRY(sort_keys(S, (const uint64_t *)key, skey, nnz, cbits + rbits));
    k_unique_flag<<<grid_for(nnz), CT, 0, s>>>(nnz, skey, flag);
    TRY(exclusive_sum(S, flag, pos, nnz));
    int last_pos = 0, last_flag = 0;
    TRY(fetch(s, pos + nnz - 1, &last_pos));
    TRY(fetch(s, flag + nnz - 1, &last_flag));
    *bnnz = last_pos + last_flag;
    if (!Bj) return LSSP_AMD_OK;
    SCRATCH(brow, unsigned, *bnnz);
    k_unique_put<<<grid_for(nnz), CT, 0, s>>>(nnz, skey, flag, pos, cbits, Bj, brow);
    k_row_ptr<<<grid_for((long)nb + 1), CT, 0, s>>>(nb, brow, *bnnz, Bp);
    LSSP_HIP(hipMemsetAsync(Bx, 0, sizeof(double) * (size_t)*bnnz * bs * bs, s));
    k_bcsr_fill<<<grid_for(n), CT, 0, s>>>(n, bs, Ap, Aj, Ax, Bp, Bj, Bx);
    LSSP_HIP(hipGetLastError());
    LSSP_HIP(hipStreamSynchronize(s));
    return LSSP_AMD_OK;
}

// matrix-utils.cxx:164-215 (and :387-481 on its result)
int lssp_amd_bcsr_to_csr(lssp_amd_ctx *c, int nbrows, int nbcols, int bs, int bnnz, const int *Bp,
                         const int *Bj, const double *Bx, int *nnz, int *Ap, int *Aj, double *Ax)
{
    if (!c || nbrows < 0 || nbcols < 0 || bs <= 0 || bnnz < 0 || !Bp || !nnz || (bnnz > 0 && (!Bj || !Bx)))
        return LSSP_AMD_EINVAL;
    if ((long)nbrows * bs > INT32_MAX - 1 || (long)nbcols * bs > INT32_MAX) return LSSP_AMD_EINVAL;
    if (Aj && (!Ap || !Ax)) return LSSP_AMD_EINVAL;
    hipStream_t s = c->stream;
    Scratch S(s);
    SCRATCH(err, int, 1);
    LSSP_HIP(hipMemsetAsync(err, 0, sizeof(int), s));
    k_check_ptr<<<grid_for((long)nbrows + 1), CT, 0, s>>>(nbrows, bnnz, Bp, err);
    if (bnnz > 0) k_check_idx<<<grid_for(bnnz), CT, 0, s>>>(bnnz, Bj, nbcols, err);
    TRY(checked(s, err));
    long n = (long)nbrows * bs;
    SCRATCH(cnt, int, n + 1);
    int *P = Ap;
    if (!P) {
        SCRATCH(Pt, int, n + 1);
        P = Pt;
    }
    LSSP_HIP(hipMemsetAsync(cnt + n, 0, sizeof(int), s));
    k_bcsr_count<<<grid_for(n), CT, 0, s>>>(n, bs, Bp, Bx, cnt);
    TRY(exclusive_sum(S, cnt, P, n + 1));
    TRY(fetch(s, P + n, nnz));
    if (!Aj) return LSSP_AMD_OK;
    k_bcsr_rows<<<grid_for(n), CT, 0, s>>>(n, bs, Bp, Bj, Bx, P, Aj, Ax);
    LSSP_HIP(hipGetLastError());
    LSSP_HIP(hipStreamSynchronize(s));
    return LSSP_AMD_OK;
}

}  // extern "C"
