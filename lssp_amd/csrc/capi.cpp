// capi.cpp -- extern "C" entry points of include/lssp_amd.h (everything except
// the Krylov drivers, solvers.cpp, and the RCCL layer, comm.cpp).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdarg>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <mutex>
#include <thread>

#include "internal.h"

using namespace lssp_amd;

namespace lssp_amd {

long num_chunks(long n) { return (n + CHUNK - 1) / CHUNK; }

int ensure_part(lssp_amd_ctx *c, long C)
{
    if (C <= c->part_cap) return LSSP_AMD_OK;
    LSSP_HIP(hipStreamSynchronize(c->stream));
    if (c->d_part) LSSP_HIP(hipFree(c->d_part));
    long cap = std::max<long>(C, 4096);
    LSSP_HIP(hipMalloc(&c->d_part, sizeof(double) * MAX_SLOTS * cap));
    c->part_cap = cap;
    return LSSP_AMD_OK;
}

// Complete a reduction whose level-1 partials a fused pass already wrote
// (tree) -- or, in serial mode, recompute it in the reference's order from the
// operand pairs -- then combine ranks and run the finalize program.
int finish_reduce(lssp_amd_ctx *c, long n, int nslot, const double *const *a,
                  const double *const *b, const Fin &f)
{
    if (c->reduce_mode == LSSP_AMD_REDUCE_SERIAL && c->nranks > 1) {
        // the reference's one sequential sum (vector.cxx:129) across P ranks: each
        // rank continues the running sums of the ranks before it, in rank order
        LSSP_TRY(comm_carry_in(c));
        LSSP_TRY(launch_reduce_serial(c, n, nslot, a, b, f, c->d_carry));
        LSSP_TRY(comm_carry_out(c));
    } else if (c->reduce_mode == LSSP_AMD_REDUCE_SERIAL) {
        LSSP_TRY(launch_reduce_serial(c, n, nslot, a, b, f));
    } else {
        LSSP_TRY(launch_reduce_tree(c, n > 0 ? num_chunks(n) : 0, nslot, f));
    }
    if (c->nranks > 1) {
        LSSP_TRY(comm_allgather_sums(c, nslot));
        LSSP_TRY(launch_sum_ranks(c, nslot, f));
    }
    return LSSP_AMD_OK;
}

int reduce_dots(lssp_amd_ctx *c, long n, int nslot, const double *const *a, const double *const *b,
                const Fin &f)
{
    if (c->reduce_mode == LSSP_AMD_REDUCE_TREE && n > 0) {
        Ew e;
        e.kind = 7;  // EW_DOT
        e.n = n;
        e.nred = nslot;
        e.r0a = a[0];
        e.r0b = b[0];
        if (nslot > 1) {
            e.r1a = a[1];
            e.r1b = b[1];
        }
        if (nslot > 2) {
            e.r2a = a[2];
            e.r2b = b[2];
        }
        if (nslot > 3) {
            e.r3a = a[3];
            e.r3b = b[3];
        }
        LSSP_TRY(launch_ew(c, e));
    }
    return finish_reduce(c, n, nslot, a, b, f);
}

}  // namespace lssp_amd

namespace lssp_amd {
static int (*g_print_fn)(void *, const char *) = nullptr;
static void *g_print_user = nullptr;

int lprint(const char *fmt, ...)
{
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    const int n = vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (g_print_fn) return g_print_fn(g_print_user, buf);
    fputs(buf, stdout);
    fflush(stdout);
    return n;
}

void setup_mark(const char *phase)
{
    static const bool on = getenv("LSSP_AMD_SETUP_TIMES") && atoi(getenv("LSSP_AMD_SETUP_TIMES"));
    static double last = 0;
    if (!on) return;
    const double t = wall_time();
    if (phase) fprintf(stderr, "lssp_amd setup: %-28s %8.3f s\n", phase, last ? t - last : 0.0);
    last = t;
}

SetupTimer::SetupTimer() : t0(wall_time()) {}
void SetupTimer::mark(const char *phase)
{
    static const bool on = getenv("LSSP_AMD_SETUP_TIMES") && atoi(getenv("LSSP_AMD_SETUP_TIMES"));
    const double t = wall_time();
    if (on) fprintf(stderr, "lssp_amd setup:   %-26s %8.3f s\n", phase, t - t0);
    t0 = t;
}

int host_threads()
{
    static const int nt = [] {
        int t = (int)std::thread::hardware_concurrency();
        const char *e = getenv("OMP_NUM_THREADS");
        if (e && atoi(e) > 0) t = std::min(t, atoi(e));
        return std::max(1, std::min(t, 16));
    }();
    return nt;
}

void parallel_for(long n, const std::function<void(long, long)> &f, long grain)
{
    const int nt = host_threads();
    const int k = (int)std::min<long>(nt, std::max<long>(1, n / std::max<long>(grain, 1)));
    if (k <= 1) {
        f(0, n);
        return;
    }
    std::vector<std::thread> th;
    for (int q = 0; q < k; q++) th.emplace_back([&, q] { f(n * q / k, n * (q + 1) / k); });
    for (std::thread &t : th) t.join();
}

// Diagonal-id column coding of a device CSR (the SpMV's index stream): the
// distinct offsets col - row are collected per thread in small open-addressing
// sets and merged; with at most 255 of them (5- / 7- / 27-point stencils, the
// z-slab halo columns of a distributed stencil) every entry becomes the byte
// index of its offset in the ascending table.  Rows are summed exactly as
// before (same entries, same order): only the way the column is found changes.
namespace {
constexpr int DIAG_MAX = 255, DIAG_HS = 1024;

struct OffSet {
    int key[DIAG_HS];
    unsigned char used[DIAG_HS] = {};
    int count = 0;
    static unsigned slot(int k) { return ((unsigned)k * 2654435761u) >> 22; }  // 10 bits
    int find(int k) const
    {
        for (unsigned h = slot(k);; h = (h + 1) & (DIAG_HS - 1)) {
            if (!used[h]) return -1;
            if (key[h] == k) return (int)h;
        }
    }
    bool add(int k)  // false once more than DIAG_MAX distinct keys were seen
    {
        unsigned h = slot(k);
        for (; used[h]; h = (h + 1) & (DIAG_HS - 1))
            if (key[h] == k) return true;
        if (count == DIAG_MAX) return false;
        used[h] = 1;
        key[h] = k;
        count++;
        return true;
    }
};
}  // namespace

int build_diag_ids(lssp_amd_mat *M, const int *Ap, const int *Aj)
{
    M->ndiag = 0;
    const int n = M->nrows;
    if (M->nnz == 0 || n == 0) return LSSP_AMD_OK;
    std::mutex mu;
    OffSet all;
    std::atomic<bool> too_many{false};
    parallel_for(n, [&](long lo, long hi) {
        OffSet mine;
        for (long i = lo; i < hi && !too_many.load(std::memory_order_relaxed); i++)
            for (int k = Ap[i]; k < Ap[i + 1]; k++)
                if (!mine.add(Aj[k] - (int)i)) {
                    too_many = true;
                    return;
                }
        std::lock_guard<std::mutex> g(mu);
        for (int h = 0; h < DIAG_HS && !too_many; h++)
            if (mine.used[h] && !all.add(mine.key[h])) too_many = true;
    });
    if (too_many) return LSSP_AMD_OK;
    std::vector<int> off;
    for (int h = 0; h < DIAG_HS; h++)
        if (all.used[h]) off.push_back(all.key[h]);
    std::sort(off.begin(), off.end());
    int id_of[DIAG_HS];
    for (int t = 0; t < (int)off.size(); t++) id_of[all.find(off[t])] = t;
    // +32: the SpMV stages the byte stream with 16-byte loads that may touch one
    // vector past the last entry
    std::vector<uint8_t> ad((size_t)M->nnz + 32, 0);
    parallel_for(n, [&](long lo, long hi) {
        for (long i = lo; i < hi; i++)
            for (int k = Ap[i]; k < Ap[i + 1]; k++) ad[k] = (uint8_t)id_of[all.find(Aj[k] - (int)i)];
    });
    LSSP_HIP(hipMalloc(&M->Ad, ad.size()));
    LSSP_HIP(hipMalloc(&M->d_off, sizeof(int) * off.size()));
    LSSP_HIP(hipMemcpy(M->Ad, ad.data(), ad.size(), hipMemcpyHostToDevice));
    LSSP_HIP(hipMemcpy(M->d_off, off.data(), sizeof(int) * off.size(), hipMemcpyHostToDevice));
    M->aux_bytes += (long long)ad.size() + (long long)sizeof(int) * (long long)off.size();
    M->ndiag = (int)off.size();
    M->max_off = 0;
    for (int o : off) M->max_off = std::max(M->max_off, std::abs(o));
    if (M->nhalo == 0) M->max_off_int = M->max_off;  // (distributed: set over the halo-free chunks at upload)
    return LSSP_AMD_OK;
}

// The x spans of the 1024-row blocks of k_spmv_win (kernels.hip), for matrices
// the diagonal-id coding does not cover (more than 255 offsets) whose rows
// nevertheless stay near the diagonal (locally renumbered meshes: config 5).
// entries (padded) of the sliced copy above which k_spmv3 serves the matrix:
// its slice offsets are 32-bit (the 16-bit column pairs halve them).
// LSSP_AMD_SELL_CAP (tests) lowers it to pin the fallback on small matrices.
static long sell_cap()
{
    const char *e = getenv("LSSP_AMD_SELL_CAP");
    const long v = e ? atol(e) : 0;
    return v > 0 && v < INT_MAX / 2 ? v : (long)(INT_MAX / 2);
}

int build_windows(lssp_amd_mat *M, const int *Ap, const int *Aj, const double *Ax)
{
    const int n = M->nrows;
    if (M->ndiag > 0 || M->nnz == 0 || n == 0) return LSSP_AMD_OK;
    const long nb = (n + WIN_ROWS - 1) / WIN_ROWS;
    std::vector<int> win(2 * nb);
    std::atomic<bool> wide{false};
    parallel_for(nb, [&](long b0, long b1) {
        for (long b = b0; b < b1 && !wide.load(std::memory_order_relaxed); b++) {
            int lo = INT_MAX, hi = INT_MIN;
            const int r1 = (int)std::min<long>((b + 1) * WIN_ROWS, n);
            for (int k = Ap[b * WIN_ROWS]; k < Ap[r1]; k++) {
                lo = std::min(lo, Aj[k]);
                hi = std::max(hi, Aj[k] + 1);
            }
            if (lo > hi) lo = hi = 0;  // a block of empty rows
            if ((long)hi - (lo & ~1) > WIN_CAP) wide = true;  // staged from lo rounded down to even
            win[2 * b] = lo;
            win[2 * b + 1] = hi;
        }
    }, 16);
    if (wide) return LSSP_AMD_OK;
    // the sliced copy (lssp_amd_mat::s_ax ...): rows of a block stably sorted
    // by descending length, so a 64-row slice pads to its longest row and every
    // load of k_spmv_sell is one coalesced wave access
    constexpr int NS = WIN_ROWS / 64;
    std::vector<uint16_t> order((size_t)nb * WIN_ROWS);
    std::vector<int> slen((size_t)nb * NS);
    std::vector<uint32_t> srow((size_t)nb * WIN_ROWS);
    parallel_for(nb, [&](long b0, long b1) {
        std::vector<int> len(WIN_ROWS);
        for (long b = b0; b < b1; b++) {
            const long r0 = b * WIN_ROWS;
            const int cnt = (int)std::min<long>(WIN_ROWS, n - r0);
            uint16_t *ord = order.data() + r0;
            for (int q = 0; q < WIN_ROWS; q++) {
                len[q] = q < cnt ? Ap[r0 + q + 1] - Ap[r0 + q] : 0;
                ord[q] = (uint16_t)q;
            }
            std::stable_sort(ord, ord + WIN_ROWS, [&](uint16_t x, uint16_t y) { return len[x] > len[y]; });
            for (int t = 0; t < WIN_ROWS; t++) srow[r0 + t] = (uint32_t)ord[t] | ((uint32_t)len[ord[t]] << 10);
            for (int w = 0; w < NS; w++) slen[b * NS + w] = len[ord[64 * w]];
        }
    }, 16);
    std::vector<int> meta(2 * slen.size());
    long tot = 0;
    for (size_t q = 0; q < slen.size(); q++) {
        meta[2 * q] = (int)tot;
        meta[2 * q + 1] = slen[q];
        tot += 64L * ((slen[q] + 1) & ~1);
        if (tot > sell_cap()) return LSSP_AMD_OK;  // too large for 32-bit slice offsets: k_spmv3 serves it
    }
    constexpr int NPAD = 64 * 16;  // the kernel's unconditional preload may read past the last slice
    std::vector<double> sax((size_t)tot + NPAD, 0.0);
    std::vector<uint32_t> scol((size_t)tot / 2 + NPAD / 2, 0u);
    parallel_for(nb, [&](long b0, long b1) {
        for (long b = b0; b < b1; b++) {
            const long r0 = b * WIN_ROWS;
            const int lo2 = win[2 * b] & ~1;
            for (int w = 0; w < NS; w++) {
                const long base = meta[2 * (b * NS + w)];
                for (int l = 0; l < 64; l++) {
                    const int q = order[r0 + 64 * w + l];
                    if (r0 + q >= n) continue;
                    const int e0 = Ap[r0 + q], len = Ap[r0 + q + 1] - e0;
                    for (int k = 0; k < len; k++) {
                        sax[base + 64L * k + l] = Ax[e0 + k];
                        scol[base / 2 + 64L * (k >> 1) + l] |= (uint32_t)(Aj[e0 + k] - lo2) << (16 * (k & 1));
                    }
                }
            }
        }
    }, 16);
    auto up = [M](void **d, const void *h, size_t bytes) -> int {
        LSSP_HIP(hipMalloc(d, bytes));
        LSSP_HIP(hipMemcpy(*d, h, bytes, hipMemcpyHostToDevice));
        M->aux_bytes += (long long)bytes;
        return LSSP_AMD_OK;
    };
    LSSP_TRY(up((void **)&M->d_win, win.data(), sizeof(int) * win.size()));
    LSSP_TRY(up((void **)&M->s_meta, meta.data(), sizeof(int) * meta.size()));
    LSSP_TRY(up((void **)&M->s_row, srow.data(), sizeof(uint32_t) * srow.size()));
    LSSP_TRY(up((void **)&M->s_ax, sax.data(), sizeof(double) * sax.size()));
    return up((void **)&M->s_col, scol.data(), sizeof(uint32_t) * scol.size());
}

double wall_time()
{
    return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
}
}  // namespace lssp_amd

extern "C" {

void lssp_amd_set_print(int (*fn)(void *user, const char *msg), void *user)
{
    g_print_fn = fn;
    g_print_user = user;
}

const char *lssp_amd_strerror(int s)
{
    switch (s) {
    case LSSP_AMD_OK: return "ok";
    case LSSP_AMD_EINVAL: return "invalid argument";
    case LSSP_AMD_EHIP: return "HIP runtime error";
    case LSSP_AMD_ENOMEM: return "out of memory";
    case LSSP_AMD_ETIMEOUT: return "trisolve dependency wait timed out";
    case LSSP_AMD_ECOMM: return "RCCL error";
    case LSSP_AMD_EUNSUPPORTED: return "unsupported solver / preconditioner";
    default: return "unknown status";
    }
}

int lssp_amd_version(void) { return 10000; }

int lssp_amd_ctx_create(int device, lssp_amd_ctx **out)
{
    if (!out) return LSSP_AMD_EINVAL;
    lssp_amd_ctx *c = new lssp_amd_ctx();
    c->device = device;
    LSSP_HIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    LSSP_HIP(hipGetDeviceProperties(&prop, device));
    c->num_cus = prop.multiProcessorCount;
    LSSP_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    LSSP_HIP(hipMalloc(&c->d_sums, sizeof(double) * MAX_SLOTS));
    LSSP_HIP(hipMalloc(&c->d_wsum, sizeof(double) * MAX_SLOTS * 16));
    LSSP_HIP(hipMalloc(&c->d_rcnt, sizeof(unsigned)));
    LSSP_HIP(hipMemset(c->d_rcnt, 0, sizeof(unsigned)));
    LSSP_HIP(hipMalloc(&c->d_scal, sizeof(double) * NSCAL));
    LSSP_HIP(hipMemset(c->d_scal, 0, sizeof(double) * NSCAL));
    LSSP_HIP(hipHostMalloc(&c->h_scal, sizeof(double) * NSCAL, hipHostMallocDefault));
    LSSP_HIP(hipMalloc(&c->d_err, sizeof(int)));
    LSSP_HIP(hipMemset(c->d_err, 0, sizeof(int)));
    LSSP_HIP(hipHostMalloc(&c->h_snap, sizeof(double) * 2 * (S_H + S_HB), hipHostMallocDefault));
    LSSP_HIP(hipHostMalloc(&c->h_snap_err, sizeof(int) * 2, hipHostMallocDefault));
    for (auto &e : c->ev_snap) LSSP_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    const char *m = getenv("LSSP_AMD_REDUCE");
    if (m && !strcmp(m, "serial")) c->reduce_mode = LSSP_AMD_REDUCE_SERIAL;
    *out = c;
    return LSSP_AMD_OK;
}

int lssp_amd_ctx_destroy(lssp_amd_ctx *c)
{
    if (!c) return LSSP_AMD_OK;
    (void)hipStreamSynchronize(c->stream);
    comm_destroy(c);
    for (auto &w : c->pool) (void)hipFree(w.p);
    if (c->d_part) (void)hipFree(c->d_part);
    if (c->d_trace) (void)hipFree(c->d_trace);
    (void)hipFree(c->d_sums);
    (void)hipFree(c->d_scal);
    if (c->d_wsum) (void)hipFree(c->d_wsum);
    if (c->d_rcnt) (void)hipFree(c->d_rcnt);
    (void)hipHostFree(c->h_scal);
    (void)hipFree(c->d_err);
    if (c->h_snap) (void)hipHostFree(c->h_snap);
    if (c->h_snap_err) (void)hipHostFree(c->h_snap_err);
    for (auto e : c->ev_snap)
        if (e) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(c->stream);
    delete c;
    return LSSP_AMD_OK;
}

int lssp_amd_ctx_set_reduction(lssp_amd_ctx *c, int mode)
{
    if (!c || (mode != LSSP_AMD_REDUCE_SERIAL && mode != LSSP_AMD_REDUCE_TREE)) return LSSP_AMD_EINVAL;
    c->reduce_mode = mode;
    return LSSP_AMD_OK;
}

int lssp_amd_ctx_sync(lssp_amd_ctx *c)
{
    if (!c) return LSSP_AMD_EINVAL;
    LSSP_HIP(hipStreamSynchronize(c->stream));
    return LSSP_AMD_OK;
}

void *lssp_amd_ctx_stream(lssp_amd_ctx *c) { return c ? (void *)c->stream : nullptr; }

// ---- vectors ---------------------------------------------------------------
int lssp_amd_vec_alloc(lssp_amd_ctx *c, long n, double **d)
{
    if (!c || !d || n < 0) return LSSP_AMD_EINVAL;
    if (hipMalloc(d, sizeof(double) * std::max<long>(n, 1)) != hipSuccess) return LSSP_AMD_ENOMEM;
    return LSSP_AMD_OK;
}

int lssp_amd_vec_free(lssp_amd_ctx *c, double *d)
{
    if (!c) return LSSP_AMD_EINVAL;
    LSSP_HIP(hipStreamSynchronize(c->stream));
    if (d) LSSP_HIP(hipFree(d));
    return LSSP_AMD_OK;
}

int lssp_amd_vec_upload(lssp_amd_ctx *c, double *d, const double *h, long n)
{
    if (!c || (n > 0 && (!d || !h))) return LSSP_AMD_EINVAL;
    if (n == 0) return LSSP_AMD_OK;
    LSSP_HIP(hipMemcpyAsync(d, h, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
    LSSP_HIP(hipStreamSynchronize(c->stream));
    return LSSP_AMD_OK;
}

int lssp_amd_vec_download(lssp_amd_ctx *c, double *h, const double *d, long n)
{
    if (!c || (n > 0 && (!d || !h))) return LSSP_AMD_EINVAL;
    if (n == 0) return LSSP_AMD_OK;
    LSSP_HIP(hipMemcpyAsync(h, d, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
    LSSP_HIP(hipStreamSynchronize(c->stream));
    return LSSP_AMD_OK;
}

// ---- matrices --------------------------------------------------------------
static int check_csr(int nrows, int ncols, int nnz, const int *Ap, const int *Aj)
{
    if (nrows < 0 || ncols <= 0 || nnz < 0 || !Ap) return LSSP_AMD_EINVAL;
    if (Ap[0] != 0 || Ap[nrows] != nnz) return LSSP_AMD_EINVAL;
    for (int i = 0; i < nrows; i++)
        if (Ap[i + 1] < Ap[i]) return LSSP_AMD_EINVAL;
    for (int k = 0; k < nnz; k++)
        if (Aj[k] < 0 || Aj[k] >= ncols) return LSSP_AMD_EINVAL;
    return LSSP_AMD_OK;
}

static int upload_csr(lssp_amd_mat *M, const int *Ap, const int *Aj, const double *Ax)
{
    LSSP_HIP(hipMalloc(&M->Ap, sizeof(int) * (M->nrows + 1)));
    // +4 entries: the 16-byte staging loads of k_spmv2 may touch up to one
    // vector past the last entry
    LSSP_HIP(hipMalloc(&M->Aj, sizeof(int) * (M->nnz + 4)));
    LSSP_HIP(hipMalloc(&M->Ax, sizeof(double) * (M->nnz + 4)));
    LSSP_HIP(hipMemcpy(M->Ap, Ap, sizeof(int) * (M->nrows + 1), hipMemcpyHostToDevice));
    if (M->nnz) {
        LSSP_HIP(hipMemcpy(M->Aj, Aj, sizeof(int) * M->nnz, hipMemcpyHostToDevice));
        LSSP_HIP(hipMemcpy(M->Ax, Ax, sizeof(double) * M->nnz, hipMemcpyHostToDevice));
    }
    LSSP_TRY(build_diag_ids(M, Ap, Aj));
    return build_windows(M, Ap, Aj, Ax);
}

int lssp_amd_mat_upload(lssp_amd_ctx *c, int nrows, int ncols, int nnz, const int *Ap, const int *Aj,
                        const double *Ax, lssp_amd_mat **out)
{
    if (!c || !out) return LSSP_AMD_EINVAL;
    LSSP_TRY(check_csr(nrows, ncols, nnz, Ap, Aj));
    LSSP_HIP(hipSetDevice(c->device));
    lssp_amd_mat *M = new lssp_amd_mat();
    M->ctx = c;
    M->nrows = nrows;
    M->ncols = ncols;
    M->nnz = nnz;
    M->n_global = nrows;
    int st = upload_csr(M, Ap, Aj, Ax);
    if (st != LSSP_AMD_OK) {
        lssp_amd_mat_destroy(M);
        return st;
    }
    // a measurement only: if it cannot run (no memory for its two vectors) the
    // product keeps the default block order
    if (tune_spmv_streams(c, M) != LSSP_AMD_OK) (void)hipGetLastError();
    *out = M;
    return LSSP_AMD_OK;
}

int lssp_amd_mat_destroy(lssp_amd_mat *M)
{
    if (!M) return LSSP_AMD_OK;
    if (M->ctx) (void)hipStreamSynchronize(M->ctx->stream);
    if (M->Ap) (void)hipFree(M->Ap);
    if (M->Aj) (void)hipFree(M->Aj);
    if (M->Ax) (void)hipFree(M->Ax);
    if (M->Ad) (void)hipFree(M->Ad);
    if (M->d_off) (void)hipFree(M->d_off);
    if (M->d_win) (void)hipFree(M->d_win);
    for (void *p : {(void *)M->s_ax, (void *)M->s_col, (void *)M->s_row, (void *)M->s_meta})
        if (p) (void)hipFree(p);
    if (M->d_send_idx) (void)hipFree(M->d_send_idx);
    if (M->d_send_buf) (void)hipFree(M->d_send_buf);
    delete M;
    return LSSP_AMD_OK;
}

int lssp_amd_mat_info(const lssp_amd_mat *A, int *nrows, int *ncols, int *nnz)
{
    if (!A) return LSSP_AMD_EINVAL;
    if (nrows) *nrows = A->nrows;
    if (ncols) *ncols = A->ncols;
    if (nnz) *nnz = A->nnz;
    return LSSP_AMD_OK;
}

int lssp_amd_mat_bytes(const lssp_amd_mat *A, long long *csr_bytes, long long *aux_bytes)
{
    if (!A) return LSSP_AMD_EINVAL;
    if (csr_bytes) *csr_bytes = 4LL * (A->nrows + 1) + 12LL * A->nnz;
    if (aux_bytes) *aux_bytes = A->aux_bytes;
    return LSSP_AMD_OK;
}

int lssp_amd_mat_layout(const lssp_amd_mat *A, int *ndiag, int *windowed)
{
    if (!A || !ndiag) return LSSP_AMD_EINVAL;
    *ndiag = A->ndiag;
    if (windowed) *windowed = A->d_win != nullptr;
    return LSSP_AMD_OK;
}

int lssp_amd_mat_local_rows(const lssp_amd_mat *A, int *row0, int *nlocal, int *nhalo)
{
    if (!A) return LSSP_AMD_EINVAL;
    if (row0) *row0 = A->row0;
    if (nlocal) *nlocal = A->nrows;
    if (nhalo) *nhalo = A->nhalo;
    return LSSP_AMD_OK;
}

// ---- SpMV (mvops.cxx) ----------------------------------------------------------
// x must hold nrows + nhalo entries on a distributed matrix; its halo part is
// refreshed here, overlapped with the halo-free rows (spmv_halo, comm.cpp).
int lssp_amd_mv_amxpby(lssp_amd_ctx *c, double alpha, const lssp_amd_mat *A, double *x,
                       double beta, double *y)
{
    if (!c || !A || !x || !y) return LSSP_AMD_EINVAL;
    return spmv_halo(c, A, EPI_AXPBY, alpha, x, beta, y, y, 0, nullptr, nullptr);
}

int lssp_amd_mv_amxpbyz(lssp_amd_ctx *c, double alpha, const lssp_amd_mat *A, double *x,
                        double beta, const double *y, double *z)
{
    if (!c || !A || !x || !y || !z) return LSSP_AMD_EINVAL;
    // y is read even when beta == 0, as the reference does (mvops.cxx:61): a NaN / Inf
    // in y propagates into z (tests/test_gpu_edge.py); only the drivers use the
    // y-free epilogue
    return spmv_halo(c, A, EPI_AXPBY, alpha, x, beta, y, z, 0, nullptr, nullptr);
}

int lssp_amd_mv_amxy(lssp_amd_ctx *c, double a, const lssp_amd_mat *A, double *x, double *y)
{
    if (!c || !A || !x || !y) return LSSP_AMD_EINVAL;
    return spmv_halo(c, A, EPI_AMXY, a, x, 0, nullptr, y, 0, nullptr, nullptr);
}

int lssp_amd_mv_mxy(lssp_amd_ctx *c, const lssp_amd_mat *A, double *x, double *y)
{
    if (!c || !A || !x || !y) return LSSP_AMD_EINVAL;
    return spmv_halo(c, A, EPI_MXY, 1.0, x, 0, nullptr, y, 0, nullptr, nullptr);
}

// ---- BLAS-1 (vector.cxx) -----------------------------------------------------------
static int ew_simple(lssp_amd_ctx *c, int kind, long n, double a, double b, const double *x,
                     const double *y, double *out)
{
    if (!c || n < 0 || (n > 0 && !out)) return LSSP_AMD_EINVAL;
    Ew e;
    e.kind = kind;
    e.n = n;
    e.a = a;
    e.b = b;
    e.x = x;
    e.y = y;
    e.out0 = out;
    return launch_ew(c, e);
}

int lssp_amd_vec_set_value(lssp_amd_ctx *c, double *x, long n, double v)
{
    return ew_simple(c, 0, n, v, 0, nullptr, nullptr, x);
}
int lssp_amd_vec_copy(lssp_amd_ctx *c, double *x, const double *y, long n)
{
    if (!c || n < 0 || (n > 0 && (!x || !y))) return LSSP_AMD_EINVAL;
    return launch_copy(c, x, y, n);
}
int lssp_amd_stream_read(lssp_amd_ctx *c, const double *x, long n, double *sink)
{
    if (!c || !sink || n < 0 || (n & 1) || (n > 0 && !x) || (reinterpret_cast<uintptr_t>(x) & 15)) return LSSP_AMD_EINVAL;
    return launch_stream_read(c, x, n, sink);
}
int lssp_amd_vec_axy(lssp_amd_ctx *c, double alpha, const double *x, double *y, long n)
{
    if (!x && n > 0) return LSSP_AMD_EINVAL;
    return ew_simple(c, 2, n, alpha, 0, x, nullptr, y);
}
int lssp_amd_vec_axpby(lssp_amd_ctx *c, double alpha, const double *x, double beta, double *y, long n)
{
    if (!x && n > 0) return LSSP_AMD_EINVAL;
    return ew_simple(c, 3, n, alpha, beta, x, nullptr, y);
}
int lssp_amd_vec_axpbyz(lssp_amd_ctx *c, double alpha, const double *x, double beta, const double *y,
                        double *z, long n)
{
    if ((!x || !y) && n > 0) return LSSP_AMD_EINVAL;
    return ew_simple(c, 4, n, alpha, beta, x, y, z);
}
int lssp_amd_vec_scale(lssp_amd_ctx *c, double *x, long n, double a)
{
    return ew_simple(c, 5, n, a, 0, nullptr, nullptr, x);
}

int lssp_amd_vec_dot(lssp_amd_ctx *c, const double *x, const double *y, long n, double *result)
{
    if (!c || !result || (n > 0 && (!x || !y))) return LSSP_AMD_EINVAL;
    const double *a[1] = {x}, *b[1] = {y};
    Fin f;
    f.op = FIN_STORE;
    f.dst[0] = S_TMP;
    LSSP_TRY(reduce_dots(c, n, 1, a, b, f));
    LSSP_HIP(hipMemcpyAsync(c->h_scal, c->d_scal + S_TMP, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    LSSP_HIP(hipStreamSynchronize(c->stream));
    *result = c->h_scal[0];
    return LSSP_AMD_OK;
}

int lssp_amd_vec_norm(lssp_amd_ctx *c, const double *x, long n, double *result)
{
    if (!c || !result || (n > 0 && !x)) return LSSP_AMD_EINVAL;
    const double *a[1] = {x}, *b[1] = {x};
    Fin f;
    f.op = FIN_NORM;
    f.dst[0] = S_TMP;
    LSSP_TRY(reduce_dots(c, n, 1, a, b, f));
    LSSP_HIP(hipMemcpyAsync(c->h_scal, c->d_scal + S_TMP, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    LSSP_HIP(hipStreamSynchronize(c->stream));
    *result = c->h_scal[0];
    return LSSP_AMD_OK;
}

// ---- ILU -------------------------------------------------------------------------
// the sync-free sweeps' level-ordered arrays (k_trisolve) of a general factor,
// built on first use: the apply's fallback when a factor has no packet
// schedule, and the single sweeps of lssp_amd_ilu_trisolve
// (the first lssp_amd_ilu_trisolve on a general factor builds them: the handle
// is mutated then, under its own lock).  Each factor is built on its own, and a
// build that fails part-way frees what it allocated, so a retry never
// overwrites live buffers.
static int sync_free_one(lssp_amd_ctx *c, int n, const std::vector<int> &Tp, const std::vector<int> &Tj,
                         const std::vector<double> &Tx, bool upper, TriSched &t)
{
    if (t.rp) return LSSP_AMD_OK;
    int st;
    try {
        st = build_trisched(c, n, Tp, Tj, Tx, upper, t, nullptr, false, true);
    } catch (const std::exception &) {
        st = LSSP_AMD_ENOMEM;
    }
    if (st != LSSP_AMD_OK) {
        for (void *p : {(void *)t.perm, (void *)t.rp, (void *)t.cols, (void *)t.vals, (void *)t.diag})
            if (p) (void)hipFree(p);
        t.perm = t.rp = t.cols = nullptr;
        t.vals = t.diag = nullptr;
    }
    return st;
}
static int ensure_sync_free(lssp_amd_ctx *c, lssp_amd_ilu *M)
{
    std::lock_guard<std::mutex> lk(M->sync_free_mu);
    LSSP_TRY(sync_free_one(c, M->n, M->Lp, M->Lj, M->Lx, false, M->lower));
    return sync_free_one(c, M->n, M->Up, M->Uj, M->Ux, true, M->upper);
}

static int ilu_upload(lssp_amd_ctx *c, lssp_amd_ilu *M)
{
    // structured ILU(0) of a 5-/7-point grid: line sweeps (linesweep.hip); the
    // packet schedules of the general sweeps are then not needed
    setup_mark(nullptr);
    const int ls = build_line_sweep(c, M->n, M->Lp, M->Lj, M->Lx, M->Up, M->Uj, M->Ux, M->line);
    if (ls != LSSP_AMD_OK && ls != LSSP_AMD_EUNSUPPORTED) return ls;
    setup_mark("line sweeps");
    // line sweeps serve every sweep of a structured factor: the packet and
    // sync-free schedules are then not built (only the level counts)
    const bool general = ls != LSSP_AMD_OK;
    // U's level pass (a sequential walk of the whole factor) runs beside L's
    // schedule build; U's build needs L's finished schedule
    std::vector<int> levU;
    int stU = LSSP_AMD_OK, stL = LSSP_AMD_OK;
    std::thread tu([&] {
        try {
            SetupTimer tm;
            stU = tri_levels(M->n, M->Up, M->Uj, true, levU);
            tm.mark("U levels (thread)");
        } catch (const std::exception &) {
            stU = LSSP_AMD_ENOMEM;
        }
    });
    try {  // the thread is joined on every path
        stL = build_trisched(c, M->n, M->Lp, M->Lj, M->Lx, false, M->lower, nullptr, general, false);
    } catch (const std::exception &) {
        stL = LSSP_AMD_ENOMEM;
    }
    tu.join();
    LSSP_TRY(stL);
    LSSP_TRY(stU);
    LSSP_TRY(build_trisched(c, M->n, M->Up, M->Uj, M->Ux, true, M->upper, general ? &M->lower : nullptr, general,
                            false, &levU));
    // the sync-free sweeps' level-ordered arrays only when a factor has no
    // packet schedule (launch_ilu_apply falls back to them): at 256^3 ILUT they
    // are ~8 GB of host copies and uploads nothing else reads
    const bool fallback = general && !(M->lower.pk6_n > 0 && M->upper.pk6_n > 0);
    if (fallback) LSSP_TRY(ensure_sync_free(c, M));
    setup_mark("sweep schedules (L, U)");
    M->lower.h_pos.clear();
    M->lower.h_pos.shrink_to_fit();
    if (fallback) {  // the sync-free sweeps' intermediate vector
        LSSP_HIP(hipMalloc(&M->d_cache, sizeof(double) * std::max(M->n, 1)));
        LSSP_TRY(launch_fill(c, M->d_cache, M->n, TRI_SENTINEL));
    }
    LSSP_HIP(hipStreamSynchronize(c->stream));
    return LSSP_AMD_OK;
}

static int ilu_create(lssp_amd_ctx *c, int kind, int n, const int *Ap, const int *Aj, const double *Ax, int level,
                      double tol, int p, int blk, lssp_amd_ilu **out);
static int ilu_from_factors(lssp_amd_ctx *c, int n, const int *Lp, const int *Lj, const double *Lx, const int *Up,
                            const int *Uj, const double *Ux, lssp_amd_ilu **out);

// host setup allocates multi-GB vectors: an allocation the host refuses
// becomes LSSP_AMD_ENOMEM at the C-ABI instead of an exception
int lssp_amd_ilu_create(lssp_amd_ctx *c, int kind, int n, const int *Ap, const int *Aj,
                        const double *Ax, int level, double tol, int p, int blk, lssp_amd_ilu **out)
{
    try {
        return ilu_create(c, kind, n, Ap, Aj, Ax, level, tol, p, blk, out);
    } catch (const std::exception &) {
        return LSSP_AMD_ENOMEM;
    }
}

int lssp_amd_ilu_from_factors(lssp_amd_ctx *c, int n, const int *Lp, const int *Lj, const double *Lx,
                              const int *Up, const int *Uj, const double *Ux, lssp_amd_ilu **out)
{
    try {
        return ilu_from_factors(c, n, Lp, Lj, Lx, Up, Uj, Ux, out);
    } catch (const std::exception &) {
        return LSSP_AMD_ENOMEM;
    }
}

static int ilu_create(lssp_amd_ctx *c, int kind, int n, const int *Ap, const int *Aj, const double *Ax, int level,
                      double tol, int p, int blk, lssp_amd_ilu **out)
{
    if (!c || !out || n <= 0 || (kind != LSSP_AMD_ILUK && kind != LSSP_AMD_ILUT)) return LSSP_AMD_EINVAL;
    LSSP_TRY(check_csr(n, n, Ap[n], Ap, Aj));
    if (Ap[n] < 1) return LSSP_AMD_EINVAL;
    LSSP_HIP(hipSetDevice(c->device));
    auto t0 = std::chrono::steady_clock::now();
    setup_mark(nullptr);
    HostCSR A;
    A.n = n;
    A.ncols = n;
    A.Ap.assign(Ap, Ap + n + 1);
    A.Aj.assign(Aj, Aj + Ap[n]);
    A.Ax.assign(Ax, Ax + Ap[n]);
    sort_columns(A);  // lssp.cxx:173
    setup_mark("copy + column sort");
    if (kind == LSSP_AMD_ILUK && level < 0) level = 1;  // pc-iluk.cxx:583-592
    HostCSR L, U;
    int fst = LSSP_AMD_OK;
    ilu_factor(c, kind, std::move(A), level, tol < 0 ? 1e-3 : tol, p, blk, L, U, &fst);
    if (fst != LSSP_AMD_OK) return fst;
    lssp_amd_ilu *M = new lssp_amd_ilu();
    M->ctx = c;
    M->n = n;
    M->Lp = std::move(L.Ap);
    M->Lj = std::move(L.Aj);
    M->Lx = std::move(L.Ax);
    M->Up = std::move(U.Ap);
    M->Uj = std::move(U.Aj);
    M->Ux = std::move(U.Ax);
    int st = ilu_upload(c, M);
    if (st != LSSP_AMD_OK) {
        lssp_amd_ilu_destroy(M);
        return st;
    }
    M->setup_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    *out = M;
    return LSSP_AMD_OK;
}

static int ilu_from_factors(lssp_amd_ctx *c, int n, const int *Lp, const int *Lj, const double *Lx, const int *Up,
                            const int *Uj, const double *Ux, lssp_amd_ilu **out)
{
    if (!c || !out || n <= 0) return LSSP_AMD_EINVAL;
    LSSP_TRY(check_csr(n, n, Lp[n], Lp, Lj));
    LSSP_TRY(check_csr(n, n, Up[n], Up, Uj));
    LSSP_HIP(hipSetDevice(c->device));
    auto t0 = std::chrono::steady_clock::now();
    lssp_amd_ilu *M = new lssp_amd_ilu();
    M->ctx = c;
    M->n = n;
    M->Lp.assign(Lp, Lp + n + 1);
    M->Lj.assign(Lj, Lj + Lp[n]);
    M->Lx.assign(Lx, Lx + Lp[n]);
    M->Up.assign(Up, Up + n + 1);
    M->Uj.assign(Uj, Uj + Up[n]);
    M->Ux.assign(Ux, Ux + Up[n]);
    int st = ilu_upload(c, M);
    if (st != LSSP_AMD_OK) {
        lssp_amd_ilu_destroy(M);
        return st;
    }
    M->setup_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    *out = M;
    return LSSP_AMD_OK;
}

int lssp_amd_ilu_destroy(lssp_amd_ilu *M)
{
    if (!M) return LSSP_AMD_OK;
    if (M->ctx) (void)hipStreamSynchronize(M->ctx->stream);
    free_trisched(M->lower);
    free_trisched(M->upper);
    free_line_sweep(M->line);
    if (M->d_cache) (void)hipFree(M->d_cache);
    for (double *p : M->d_sh)
        if (p) (void)hipFree(p);
    if (M->d_rperm) (void)hipFree(M->d_rperm);
    delete M;
    return LSSP_AMD_OK;
}

static int check_err(lssp_amd_ctx *c, const lssp_amd_ilu *M = nullptr)
{
    int e = 0;
    LSSP_HIP(hipMemcpyAsync(&e, c->d_err, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    LSSP_HIP(hipStreamSynchronize(c->stream));
    if (e) {
        LSSP_HIP(hipMemset(c->d_err, 0, sizeof(int)));
        // a sweep that gave up mid-way leaves hand-off entries written: re-arm
        if (M && M->line.ntiles) {
            LSSP_TRY(line_rearm(c, const_cast<lssp_amd_ilu *>(M)->line));
            LSSP_HIP(hipStreamSynchronize(c->stream));
        }
        return LSSP_AMD_ETIMEOUT;
    }
    return LSSP_AMD_OK;
}

// solver-tri.cxx:48-60: cache = L^-1 rhs ; x = U^-1 cache.  The L sweep also
// arms x (sentinel) for the U sweep, the U sweep re-arms the cache.
int lssp_amd_ilu_apply(lssp_amd_ctx *c, const lssp_amd_ilu *M, double *x, const double *rhs)
{
    if (!c || !M || !x || !rhs) return LSSP_AMD_EINVAL;
    LSSP_TRY(launch_ilu_apply(c, M, x, rhs));
    return check_err(c, M);
}

// The same apply, only enqueued on the context's stream (no host round trip):
// for callers that pipeline applies with other work; a hand-off timeout of an
// enqueued apply is reported by lssp_amd_ilu_check.
int lssp_amd_ilu_apply_async(lssp_amd_ctx *c, const lssp_amd_ilu *M, double *x, const double *rhs)
{
    if (!c || !M || !x || !rhs) return LSSP_AMD_EINVAL;
    return launch_ilu_apply(c, M, x, rhs);
}

int lssp_amd_ilu_check(lssp_amd_ctx *c, const lssp_amd_ilu *M)
{
    if (!c || !M) return LSSP_AMD_EINVAL;
    return check_err(c, M);
}

int lssp_amd_ilu_trisolve(lssp_amd_ctx *c, const lssp_amd_ilu *M, int which, double *x, const double *rhs)
{
    if (!c || !M || !x || !rhs || x == rhs) return LSSP_AMD_EINVAL;
    if (M->line.ntiles) {
        LSSP_TRY(launch_line_sweep(c, M->line, which ? 1 : 0, x, rhs));
        return check_err(c, M);
    }
    LSSP_TRY(ensure_sync_free(c, const_cast<lssp_amd_ilu *>(M)));
    LSSP_TRY(launch_fill(c, x, M->n, TRI_SENTINEL));
    LSSP_TRY(launch_trisolve(c, which ? M->upper : M->lower, rhs, x, nullptr));
    return check_err(c);
}

int lssp_amd_ilu_info(const lssp_amd_ilu *M, int *n, int *nnzL, int *nnzU, int *levelsL, int *levelsU,
                      double *setup_seconds)
{
    if (!M) return LSSP_AMD_EINVAL;
    if (n) *n = M->n;
    if (nnzL) *nnzL = (int)M->Lj.size();
    if (nnzU) *nnzU = (int)M->Uj.size();
    if (levelsL) *levelsL = M->lower.nlevels;
    if (levelsU) *levelsU = M->upper.nlevels;
    if (setup_seconds) *setup_seconds = M->setup_seconds;
    return LSSP_AMD_OK;
}

int lssp_amd_ilu_sweep_layout(const lssp_amd_ilu *M, int *line, int *lines, int *planes)
{
    if (!M) return LSSP_AMD_EINVAL;
    const bool ls = M->line.ntiles > 0;
    if (line) *line = ls ? 1 + M->line.kind : 0;
    if (lines) *lines = ls ? M->line.NJ : 0;
    if (planes) *planes = ls ? M->line.P : 0;
    return LSSP_AMD_OK;
}

int lssp_amd_ilu_get_factors(const lssp_amd_ilu *M, int *Lp, int *Lj, double *Lx, int *Up, int *Uj,
                             double *Ux)
{
    if (!M) return LSSP_AMD_EINVAL;
    if (Lp) memcpy(Lp, M->Lp.data(), sizeof(int) * M->Lp.size());
    if (Lj) memcpy(Lj, M->Lj.data(), sizeof(int) * M->Lj.size());
    if (Lx) memcpy(Lx, M->Lx.data(), sizeof(double) * M->Lx.size());
    if (Up) memcpy(Up, M->Up.data(), sizeof(int) * M->Up.size());
    if (Uj) memcpy(Uj, M->Uj.data(), sizeof(int) * M->Uj.size());
    if (Ux) memcpy(Ux, M->Ux.data(), sizeof(double) * M->Ux.size());
    return LSSP_AMD_OK;
}

int lssp_amd_csr_sort_columns(int nrows, int ncols, int *Ap, int *Aj, double *Ax)
{
    if (nrows < 0 || ncols <= 0 || !Ap || !Aj || !Ax) return LSSP_AMD_EINVAL;
    HostCSR H;
    H.n = nrows;
    H.ncols = ncols;
    H.Ap.assign(Ap, Ap + nrows + 1);
    H.Aj.assign(Aj, Aj + Ap[nrows]);
    H.Ax.assign(Ax, Ax + Ap[nrows]);
    sort_columns(H);
    memcpy(Aj, H.Aj.data(), sizeof(int) * H.Aj.size());
    memcpy(Ax, H.Ax.data(), sizeof(double) * H.Ax.size());
    return LSSP_AMD_OK;
}

// ---- synthetic inputs: example/exam.cxx:4-59 (5-pt) and the 7-pt analogue ----------
long lssp_amd_poisson_nnz(int dim, int N)
{
    long n = N;
    return dim == 2 ? 5 * n * n - 4 * n : 7 * n * n * n - 6 * n * n;
}

int lssp_amd_poisson_rows(int dim, int N, long row0, long nrows, int *Ap, int *Aj, double *Ax)
{
    if ((dim != 2 && dim != 3) || N <= 0 || !Ap || !Aj || !Ax) return LSSP_AMD_EINVAL;
    const long N2 = (long)N * N, n = dim == 2 ? N2 : N2 * N;
    if (row0 < 0 || nrows < 0 || row0 + nrows > n) return LSSP_AMD_EINVAL;
    long o = 0;
    Ap[0] = 0;
    for (long q = 0; q < nrows; q++) {
        const long r = row0 + q;
        if (dim == 2) {
            const long i = r / N, j = r % N;
            if (i > 0) { Aj[o] = (int)(r - N); Ax[o++] = -1; }
            if (j > 0) { Aj[o] = (int)(r - 1); Ax[o++] = -1; }
            Aj[o] = (int)r; Ax[o++] = 4;
            if (j < N - 1) { Aj[o] = (int)(r + 1); Ax[o++] = -1; }
            if (i < N - 1) { Aj[o] = (int)(r + N); Ax[o++] = -1; }
        } else {
            const long k = r / N2, j = (r / N) % N, i = r % N;
            if (k > 0) { Aj[o] = (int)(r - N2); Ax[o++] = -1; }
            if (j > 0) { Aj[o] = (int)(r - N); Ax[o++] = -1; }
            if (i > 0) { Aj[o] = (int)(r - 1); Ax[o++] = -1; }
            Aj[o] = (int)r; Ax[o++] = 6;
            if (i < N - 1) { Aj[o] = (int)(r + 1); Ax[o++] = -1; }
            if (j < N - 1) { Aj[o] = (int)(r + N); Ax[o++] = -1; }
            if (k < N - 1) { Aj[o] = (int)(r + N2); Ax[o++] = -1; }
        }
        Ap[q + 1] = (int)o;
    }
    return LSSP_AMD_OK;
}

}  // extern "C"
