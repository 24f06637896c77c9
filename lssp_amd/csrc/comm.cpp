// comm.cpp -- multi-GPU layer: one process per GPU, RCCL over xGMI (or the
// caller's host-staged transport, lssp_amd_comm_init_host).
//
// The reference is serial (README.md:3); this is the SURVEY 8(e) extension of
// the hot path.  Rows are partitioned in contiguous blocks of ceil(n/P) (the
// same blocks the reference's block-Jacobi path uses, pc-iluk.cxx:467-472).
//   * SpMV: each rank holds its rows with columns renumbered [owned | halo];
//     before a product the halo entries are fetched with ONE grouped
//     ncclSend/ncclRecv round to exactly the peers that own them (for the
//     7-pt stencil: one N^2 plane from each z-neighbour).
//   * Dots: each rank reduces its slice in the canonical tree order, the P
//     rank sums are all-gathered (ncclAllGather, P*4 doubles) and every rank
//     adds them in rank order -- deterministic and identical on all ranks.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <climits>
#include <cstring>
#include <map>

#include "internal.h"

namespace lssp_amd {

#define LSSP_NCCL(call)                                                                            \
    do {                                                                                           \
        ncclResult_t r_ = (call);                                                                  \
        if (r_ != ncclSuccess) {                                                                   \
            fprintf(stderr, "lssp_amd: RCCL error %s at %s:%d\n", ncclGetErrorString(r_), __FILE__, \
                    __LINE__);                                                                     \
            return LSSP_AMD_ECOMM;                                                                 \
        }                                                                                          \
    } while (0)

// ---- transport: RCCL, or the caller's host-staged hooks --------------------
struct Msg {
    int peer;
    void *dbuf;  // device buffer
    long bytes;
};

static bool host_mode(const lssp_amd_ctx *c) { return c->comm == nullptr && c->host.allgather != nullptr; }

// recv (device, nranks * bytes) = every rank's send (device, bytes), rank order
static int xfer_allgather(lssp_amd_ctx *c, const void *dsend, void *drecv, long bytes)
{
    if (!host_mode(c)) {
        LSSP_NCCL(ncclAllGather(dsend, drecv, (size_t)bytes, ncclInt8, (ncclComm_t)c->comm, c->stream));
        return LSSP_AMD_OK;
    }
    std::vector<char> hs(std::max<long>(bytes, 1)), hr(std::max<long>(bytes * c->nranks, 1));
    if (bytes) LSSP_HIP(hipMemcpyAsync(hs.data(), dsend, bytes, hipMemcpyDeviceToHost, c->stream));
    LSSP_HIP(hipStreamSynchronize(c->stream));
    if (c->host.allgather(c->host.user, hs.data(), hr.data(), bytes) != 0) return LSSP_AMD_ECOMM;
    if (bytes) LSSP_HIP(hipMemcpyAsync(drecv, hr.data(), bytes * c->nranks, hipMemcpyHostToDevice, c->stream));
    LSSP_HIP(hipStreamSynchronize(c->stream));
    return LSSP_AMD_OK;
}

// one grouped point-to-point round (RCCL: on stream st, default the context's)
static int xfer_group(lssp_amd_ctx *c, const std::vector<Msg> &sends, const std::vector<Msg> &recvs,
                      hipStream_t st = nullptr)
{
    if (!host_mode(c)) {
        if (!st) st = c->stream;
        LSSP_NCCL(ncclGroupStart());
        for (const Msg &m : sends)
            LSSP_NCCL(ncclSend(m.dbuf, (size_t)m.bytes, ncclInt8, m.peer, (ncclComm_t)c->comm, st));
        for (const Msg &m : recvs)
            LSSP_NCCL(ncclRecv(m.dbuf, (size_t)m.bytes, ncclInt8, m.peer, (ncclComm_t)c->comm, st));
        LSSP_NCCL(ncclGroupEnd());
        return LSSP_AMD_OK;
    }
    const int ns = (int)sends.size(), nr = (int)recvs.size();
    std::vector<std::vector<char>> hs(ns), hr(nr);
    std::vector<int> sp(ns), rp(nr);
    std::vector<const void *> sb(ns);
    std::vector<void *> rb(nr);
    std::vector<long> sl(ns), rl(nr);
    for (int i = 0; i < ns; i++) {
        hs[i].resize(std::max<long>(sends[i].bytes, 1));
        if (sends[i].bytes)
            LSSP_HIP(hipMemcpyAsync(hs[i].data(), sends[i].dbuf, sends[i].bytes, hipMemcpyDeviceToHost, c->stream));
        sp[i] = sends[i].peer;
        sb[i] = hs[i].data();
        sl[i] = sends[i].bytes;
    }
    for (int i = 0; i < nr; i++) {
        hr[i].resize(std::max<long>(recvs[i].bytes, 1));
        rp[i] = recvs[i].peer;
        rb[i] = hr[i].data();
        rl[i] = recvs[i].bytes;
    }
    LSSP_HIP(hipStreamSynchronize(c->stream));
    if (c->host.sendrecv(c->host.user, ns, sp.data(), sb.data(), sl.data(), nr, rp.data(), rb.data(), rl.data()) != 0)
        return LSSP_AMD_ECOMM;
    for (int i = 0; i < nr; i++)
        if (recvs[i].bytes)
            LSSP_HIP(hipMemcpyAsync(recvs[i].dbuf, hr[i].data(), recvs[i].bytes, hipMemcpyHostToDevice, c->stream));
    LSSP_HIP(hipStreamSynchronize(c->stream));
    return LSSP_AMD_OK;
}

int comm_allgather_sums(lssp_amd_ctx *c, int nslot)
{
    (void)nslot;
    return xfer_allgather(c, c->d_sums, c->d_gather, (long)sizeof(double) * MAX_SLOTS);
}

int comm_allgather(lssp_amd_ctx *c, const void *send, void *recv, long bytes)
{
    return xfer_allgather(c, send, recv, bytes);
}

int comm_carry_in(lssp_amd_ctx *c)
{
    const long bytes = (long)sizeof(double) * MAX_SLOTS;
    if (c->rank == 0) {
        LSSP_HIP(hipMemsetAsync(c->d_carry, 0, bytes, c->stream));  // +0.0: the reference's sum = 0
        return LSSP_AMD_OK;
    }
    return xfer_group(c, {}, {{c->rank - 1, c->d_carry, bytes}});
}

int comm_carry_out(lssp_amd_ctx *c)
{
    if (c->rank == c->nranks - 1) return LSSP_AMD_OK;
    return xfer_group(c, {{c->rank + 1, c->d_sums, (long)sizeof(double) * MAX_SLOTS}}, {});
}

static void halo_msgs(const lssp_amd_mat *A, double *x, std::vector<Msg> &s, std::vector<Msg> &r)
{
    for (size_t q = 0; q < A->send_peer.size(); q++)
        s.push_back({A->send_peer[q], A->d_send_buf + A->send_off[q], (long)sizeof(double) * A->send_cnt[q]});
    for (size_t q = 0; q < A->recv_peer.size(); q++)
        r.push_back({A->recv_peer[q], x + A->nrows + A->recv_off[q], (long)sizeof(double) * A->recv_cnt[q]});
}

int halo_exchange(const lssp_amd_mat *A, double *x)
{
    if (!A || A->ctx == nullptr || A->ctx->nranks <= 1) return LSSP_AMD_OK;
    if (A->send_peer.empty() && A->recv_peer.empty()) return LSSP_AMD_OK;
    lssp_amd_ctx *c = A->ctx;
    LSSP_TRY(launch_pack(c, A->d_send_idx, x, A->d_send_buf, A->nsend));
    std::vector<Msg> s, r;
    halo_msgs(A, x, s, r);
    return xfer_group(c, s, r);
}

// z = op(A x) with the halo round overlapped: the chunks [ich0, ich1) read no
// halo column, so their product runs while the round is in flight -- on the
// RCCL path the round goes to comm_stream between two events (pack -> round ->
// boundary chunks); on the host transport, which stages through the host
// synchronously, the interior product is simply queued before the round.  Each
// chunk writes its level-1 partials at its own index, so the split product and
// its fused dots are bitwise those of one launch.
int spmv_halo(lssp_amd_ctx *c, const lssp_amd_mat *A, int epi, double alpha, double *x, double beta,
              const double *y, double *z, int nred, const double *w0, const double *w1)
{
    const bool xch = c->nranks > 1 && !(A->send_peer.empty() && A->recv_peer.empty());
    if (!xch || A->ich1 <= A->ich0) {
        LSSP_TRY(halo_exchange(A, x));
        return launch_spmv(c, A, epi, alpha, x, beta, y, z, nred, w0, w1);
    }
    const long nall = num_chunks(A->nrows);
    LSSP_TRY(launch_pack(c, A->d_send_idx, x, A->d_send_buf, A->nsend));
    std::vector<Msg> s, r;
    halo_msgs(A, x, s, r);
    if (!host_mode(c)) {
        LSSP_HIP(hipEventRecord(c->ev_pack, c->stream));
        LSSP_HIP(hipStreamWaitEvent(c->comm_stream, c->ev_pack, 0));
        LSSP_TRY(xfer_group(c, s, r, c->comm_stream));
        LSSP_HIP(hipEventRecord(c->ev_halo, c->comm_stream));
        LSSP_TRY(launch_spmv(c, A, epi, alpha, x, beta, y, z, nred, w0, w1, A->ich0, A->ich1));
        LSSP_HIP(hipStreamWaitEvent(c->stream, c->ev_halo, 0));
    } else {
        LSSP_TRY(launch_spmv(c, A, epi, alpha, x, beta, y, z, nred, w0, w1, A->ich0, A->ich1));
        LSSP_TRY(xfer_group(c, s, r));
    }
    LSSP_TRY(launch_spmv(c, A, epi, alpha, x, beta, y, z, nred, w0, w1, 0, A->ich0));
    return launch_spmv(c, A, epi, alpha, x, beta, y, z, nred, w0, w1, A->ich1, nall);
}

// after a product of the halo-free chunks [ich0, ich1) ran elsewhere (the U
// sweep's tail): the halo round, then the boundary chunks
int spmv_boundary(lssp_amd_ctx *c, const lssp_amd_mat *A, int epi, double alpha, double *x, double beta,
                  const double *y, double *z, int nred, const double *w0, const double *w1)
{
    const long nall = num_chunks(A->nrows);
    LSSP_TRY(halo_exchange(A, x));
    LSSP_TRY(launch_spmv(c, A, epi, alpha, x, beta, y, z, nred, w0, w1, 0, A->ich0));
    return launch_spmv(c, A, epi, alpha, x, beta, y, z, nred, w0, w1, A->ich1, nall);
}

int comm_destroy(lssp_amd_ctx *c)
{
    if (c->comm) {
        ncclCommDestroy((ncclComm_t)c->comm);
        c->comm = nullptr;
    }
    if (c->d_gather) {
        (void)hipFree(c->d_gather);
        c->d_gather = nullptr;
    }
    if (c->d_carry) {
        (void)hipFree(c->d_carry);
        c->d_carry = nullptr;
    }
    if (c->d_igather) {
        (void)hipFree(c->d_igather);
        c->d_igather = nullptr;
    }
    if (c->ev_pack) (void)hipEventDestroy(c->ev_pack);
    if (c->ev_halo) (void)hipEventDestroy(c->ev_halo);
    if (c->comm_stream) (void)hipStreamDestroy(c->comm_stream);
    c->ev_pack = c->ev_halo = nullptr;
    c->comm_stream = nullptr;
    c->host = lssp_amd_host_transport{};
    c->nranks = 1;
    c->rank = 0;
    return LSSP_AMD_OK;
}

// one int per rank, all-gathered in rank order (collective).  The scratch is
// the context's (allocated with the communicator), so nothing here can fail on
// one rank before the all-gather and leave the others waiting in it; a failed
// copy-in on this rank is sent as INT_MIN, which every caller treats as an error.
int comm_gather_int(lssp_amd_ctx *c, int v, std::vector<int> &all)
{
    all.assign(c->nranks, INT_MIN);
    if (c->nranks <= 1) {
        all.assign(c->nranks, v);
        return LSSP_AMD_OK;
    }
    // P ranks without the scratch: lssp_amd_comm_init failed part-way; no
    // agreement can be reported that never happened
    if (!c->d_igather) return LSSP_AMD_EHIP;
    (void)hipSetDevice(c->device);
    int *d = c->d_igather;  // [mine | all ranks]
    if (hipMemcpyAsync(d, &v, sizeof(int), hipMemcpyHostToDevice, c->stream) != hipSuccess) {
        const int bad = INT_MIN;  // still join the gather, with an error code
        (void)hipGetLastError();
        (void)hipMemcpy(d, &bad, sizeof(int), hipMemcpyHostToDevice);
    }
    int st = xfer_allgather(c, d, d + 1, (long)sizeof(int));
    if (st == LSSP_AMD_OK &&
        (hipMemcpyAsync(all.data(), d + 1, sizeof(int) * c->nranks, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
         hipStreamSynchronize(c->stream) != hipSuccess))
        st = LSSP_AMD_EHIP;
    return st;
}

}  // namespace lssp_amd

using namespace lssp_amd;

extern "C" {

namespace {
struct DevMem {  // device scratch, freed when the upload returns
    void *p = nullptr;
    ~DevMem()
    {
        if (p) (void)hipFree(p);
    }
};
struct MatGuard {  // the half-built matrix, destroyed unless released
    lssp_amd_mat *m;
    ~MatGuard() { lssp_amd_mat_destroy(m); }
};
}  // namespace

int lssp_amd_comm_unique_id_size(void) { return (int)sizeof(ncclUniqueId); }

int lssp_amd_comm_get_unique_id(void *out)
{
    if (!out) return LSSP_AMD_EINVAL;
    ncclUniqueId id;
    LSSP_NCCL(ncclGetUniqueId(&id));
    memcpy(out, &id, sizeof(id));
    return LSSP_AMD_OK;
}

int lssp_amd_comm_init(lssp_amd_ctx *c, int nranks, int rank, const void *idp)
{
    if (!c || !idp || nranks < 1 || rank < 0 || rank >= nranks) return LSSP_AMD_EINVAL;
    LSSP_HIP(hipSetDevice(c->device));
    comm_destroy(c);
    // nranks == 1: a 1-rank communicator (the solvers take their single-rank
    // paths; lssp_amd_comm_selftest can drive the RCCL transport on one GPU)
    ncclUniqueId id;
    memcpy(&id, idp, sizeof(id));
    ncclComm_t comm;
    LSSP_NCCL(ncclCommInitRank(&comm, nranks, id, rank));
    c->comm = comm;
    c->nranks = nranks;
    c->rank = rank;
    LSSP_HIP(hipMalloc(&c->d_gather, sizeof(double) * MAX_SLOTS * nranks));
    LSSP_HIP(hipMalloc(&c->d_carry, sizeof(double) * MAX_SLOTS));
    LSSP_HIP(hipMalloc(&c->d_igather, sizeof(int) * (1 + nranks)));
    LSSP_HIP(hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
    LSSP_HIP(hipEventCreateWithFlags(&c->ev_pack, hipEventDisableTiming));
    LSSP_HIP(hipEventCreateWithFlags(&c->ev_halo, hipEventDisableTiming));
    return LSSP_AMD_OK;
}

int lssp_amd_comm_nranks(lssp_amd_ctx *c, int *nranks)
{
    if (!c || !nranks) return LSSP_AMD_EINVAL;
    if (!c->comm) {  // host transport, or no communicator (single rank)
        *nranks = c->nranks;
        return LSSP_AMD_OK;
    }
    int n = 0;
    LSSP_NCCL(ncclCommCount((ncclComm_t)c->comm, &n));
    *nranks = n;
    return LSSP_AMD_OK;
}

int lssp_amd_comm_selftest(lssp_amd_ctx *c)
{
    if (!c) return LSSP_AMD_EINVAL;
    if (!c->comm && !host_mode(c)) return LSSP_AMD_EINVAL;  // no transport
    LSSP_HIP(hipSetDevice(c->device));
    const int P = c->nranks, r = c->rank;
    const long n = 4096 + 8 * r;                              // message sizes differ per rank
    const long nprev = 4096 + 8 * ((r + P - 1) % P);          // what rank r-1 sends
    std::vector<double> h(std::max(n, nprev));
    DevMem d_send, d_recv, d_id, d_ids;
    LSSP_HIP(hipMalloc(&d_send.p, sizeof(double) * n));
    LSSP_HIP(hipMalloc(&d_recv.p, sizeof(double) * nprev));
    LSSP_HIP(hipMalloc(&d_id.p, sizeof(double) * MAX_SLOTS));
    LSSP_HIP(hipMalloc(&d_ids.p, sizeof(double) * MAX_SLOTS * P));
    for (long i = 0; i < n; i++) h[i] = r * 1e6 + i;
    LSSP_HIP(hipMemcpyAsync(d_send.p, h.data(), sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
    LSSP_HIP(hipMemsetAsync(d_recv.p, 0xff, sizeof(double) * nprev, c->stream));
    double mine[MAX_SLOTS] = {(double)r, 1.0 + r, 2.0 * r, -1.0 - r};
    LSSP_HIP(hipMemcpyAsync(d_id.p, mine, sizeof(mine), hipMemcpyHostToDevice, c->stream));
    LSSP_TRY(xfer_allgather(c, d_id.p, d_ids.p, (long)sizeof(mine)));
    // the halo round's plumbing (spmv_halo): event after the pack, the round on
    // comm_stream, the compute stream waits for its event
    const std::vector<Msg> sends{{(r + 1) % P, d_send.p, (long)sizeof(double) * n}};
    const std::vector<Msg> recvs{{(r + P - 1) % P, d_recv.p, (long)sizeof(double) * nprev}};
    if (!host_mode(c)) {
        LSSP_HIP(hipEventRecord(c->ev_pack, c->stream));
        LSSP_HIP(hipStreamWaitEvent(c->comm_stream, c->ev_pack, 0));
        LSSP_TRY(xfer_group(c, sends, recvs, c->comm_stream));
        LSSP_HIP(hipEventRecord(c->ev_halo, c->comm_stream));
        LSSP_HIP(hipStreamWaitEvent(c->stream, c->ev_halo, 0));
    } else {
        LSSP_TRY(xfer_group(c, sends, recvs));
    }
    std::vector<double> ids(MAX_SLOTS * P);
    LSSP_HIP(hipMemcpyAsync(h.data(), d_recv.p, sizeof(double) * nprev, hipMemcpyDeviceToHost, c->stream));
    LSSP_HIP(hipMemcpyAsync(ids.data(), d_ids.p, sizeof(double) * ids.size(), hipMemcpyDeviceToHost, c->stream));
    LSSP_HIP(hipStreamSynchronize(c->stream));
    int st = LSSP_AMD_OK;
    const int rp = (r + P - 1) % P;
    for (long i = 0; i < nprev; i++)
        if (h[i] != rp * 1e6 + i) st = LSSP_AMD_ECOMM;
    for (int q = 0; q < P; q++) {
        const double want[MAX_SLOTS] = {(double)q, 1.0 + q, 2.0 * q, -1.0 - q};
        for (int k = 0; k < MAX_SLOTS; k++)
            if (ids[q * MAX_SLOTS + k] != want[k]) st = LSSP_AMD_ECOMM;
    }
    return st;
}

int lssp_amd_comm_init_host(lssp_amd_ctx *c, int nranks, int rank, const lssp_amd_host_transport *t)
{
    if (!c || nranks < 1 || rank < 0 || rank >= nranks) return LSSP_AMD_EINVAL;
    if (nranks > 1 && (!t || !t->allgather || !t->sendrecv)) return LSSP_AMD_EINVAL;
    LSSP_HIP(hipSetDevice(c->device));
    comm_destroy(c);
    if (nranks == 1) return LSSP_AMD_OK;
    c->host = *t;
    c->nranks = nranks;
    c->rank = rank;
    LSSP_HIP(hipMalloc(&c->d_gather, sizeof(double) * MAX_SLOTS * nranks));
    LSSP_HIP(hipMalloc(&c->d_carry, sizeof(double) * MAX_SLOTS));
    LSSP_HIP(hipMalloc(&c->d_igather, sizeof(int) * (1 + nranks)));
    return LSSP_AMD_OK;
}

int lssp_amd_comm_barrier(lssp_amd_ctx *c)
{
    if (!c) return LSSP_AMD_EINVAL;
    if (c->nranks > 1) {
        // an all-gather of one double per rank: returns on a rank only once every rank has entered
        LSSP_TRY(xfer_allgather(c, c->d_sums, c->d_gather, (long)sizeof(double)));
    }
    LSSP_HIP(hipStreamSynchronize(c->stream));
    return LSSP_AMD_OK;
}

// Local rows [row0, row0+nlocal) of the global matrix, global column indices.
// Collective.  A rank that finds bad input does not return on its own: the
// statuses are agreed on (agree_status) before each collective step, so every
// rank fails together with the same status and none is left waiting in an
// all-gather or send/recv.  Temporary device buffers and the half-built matrix
// are released on every path.

// every rank's status -> the first non-zero one (rank order), identical on all ranks
static int agree_status(lssp_amd_ctx *c, int st)
{
    std::vector<int> all;
    LSSP_TRY(comm_gather_int(c, st, all));
    for (int s : all)
        if (s != LSSP_AMD_OK) return s == INT_MIN ? LSSP_AMD_EHIP : s;
    return LSSP_AMD_OK;
}

int lssp_amd_mat_upload_dist(lssp_amd_ctx *c, int n_global, int row0, int nlocal, const int *Ap,
                             const int *Aj, const double *Ax, lssp_amd_mat **out)
{
    if (!c || !out) return LSSP_AMD_EINVAL;  // no context: nothing to agree through
    const int P = c->nranks;
    // ---- local checks, then agreed on ----
    int st = LSSP_AMD_OK;
    const int blk = n_global > 0 ? (n_global + P - 1) / P : 1;
    const int my0 = std::min(c->rank * blk, std::max(n_global, 0));
    const int myn = std::max(0, std::min(blk, n_global - my0));
    if (!Ap || n_global <= 0 || nlocal < 0 || row0 != my0 || nlocal != myn || Ap[0] != 0)
        st = LSSP_AMD_EINVAL;  // canonical partition only
    const int nnz = st == LSSP_AMD_OK ? Ap[nlocal] : 0;
    if (st == LSSP_AMD_OK && (nnz < 0 || (nnz > 0 && (!Aj || !Ax)))) st = LSSP_AMD_EINVAL;
    for (int k = 0; st == LSSP_AMD_OK && k < nnz; k++)
        if (Aj[k] < 0 || Aj[k] >= n_global) st = LSSP_AMD_EINVAL;
    LSSP_TRY(agree_status(c, st));
    // halo columns, grouped by owner then ascending
    std::map<int, int> halo;  // global col -> slot
    for (int k = 0; k < nnz; k++) {
        const int g = Aj[k];
        if (g < row0 || g >= row0 + nlocal) halo[g] = 0;
    }
    std::vector<int> hcols;
    hcols.reserve(halo.size());
    for (auto &kv : halo) hcols.push_back(kv.first);  // std::map is ordered: owners ascending too
    for (size_t q = 0; q < hcols.size(); q++) halo[hcols[q]] = (int)q;
    std::vector<int> lj(nnz);
    for (int k = 0; k < nnz; k++) {
        const int g = Aj[k];
        lj[k] = (g >= row0 && g < row0 + nlocal) ? g - row0 : nlocal + halo[g];
    }
    MatGuard guard{new lssp_amd_mat()};
    lssp_amd_mat *M = guard.m;
    M->ctx = c;
    M->nrows = nlocal;
    M->nhalo = (int)hcols.size();
    M->ncols = nlocal + M->nhalo;
    M->nnz = nnz;
    M->n_global = n_global;
    M->row0 = row0;
    {  // the longest run of chunks without a halo-reading row (spmv_halo)
        const long nch = num_chunks(nlocal);
        long run0 = 0, best0 = 0, best1 = 0;
        for (long ch = 0; ch <= nch; ch++) {
            bool halo_free = ch < nch;
            for (long i = ch * 256; halo_free && i < std::min<long>((ch + 1) * 256, nlocal); i++)
                for (int k = Ap[i]; k < Ap[i + 1]; k++)
                    if (lj[k] >= nlocal) {
                        halo_free = false;
                        break;
                    }
            if (!halo_free) {
                if (ch - run0 > best1 - best0) best0 = run0, best1 = ch;
                run0 = ch + 1;
            }
        }
        M->ich0 = best0;
        M->ich1 = best1;
        int mo = 0;  // the halo-free rows' widest reach (the U sweep's tail product, linesweep.hip)
        for (long i = best0 * 256; i < std::min<long>(best1 * 256, nlocal); i++)
            for (int k = Ap[i]; k < Ap[i + 1]; k++) mo = std::max(mo, std::abs(lj[k] - (int)i));
        M->max_off_int = mo;
    }
    // receive plan (per owner)
    std::vector<int> need(P, 0);
    for (int g : hcols) need[g / blk]++;
    int off = 0;
    for (int q = 0; q < P; q++) {
        if (need[q]) {
            M->recv_peer.push_back(q);
            M->recv_off.push_back(off);
            M->recv_cnt.push_back(need[q]);
        }
        off += need[q];
    }
    // tell every owner which of its columns we need: counts then index lists
    DevMem d_cnt_mine, d_cnt_all, d_hcols, d_sendg;
    st = hipMalloc(&d_cnt_mine.p, sizeof(int) * P) == hipSuccess &&
                 hipMalloc(&d_cnt_all.p, sizeof(int) * P * P) == hipSuccess &&
                 hipMemcpy(d_cnt_mine.p, need.data(), sizeof(int) * P, hipMemcpyHostToDevice) == hipSuccess
             ? LSSP_AMD_OK
             : LSSP_AMD_ENOMEM;
    LSSP_TRY(agree_status(c, st));
    LSSP_TRY(xfer_allgather(c, d_cnt_mine.p, d_cnt_all.p, (long)sizeof(int) * P));
    std::vector<int> all(P * P);
    LSSP_HIP(hipMemcpyAsync(all.data(), d_cnt_all.p, sizeof(int) * P * P, hipMemcpyDeviceToHost, c->stream));
    LSSP_HIP(hipStreamSynchronize(c->stream));
    int nsend = 0;
    for (int q = 0; q < P; q++) {
        const int cnt = all[q * P + c->rank];  // what rank q needs from me
        if (cnt) {
            M->send_peer.push_back(q);
            M->send_off.push_back(nsend);
            M->send_cnt.push_back(cnt);
            nsend += cnt;
        }
    }
    M->nsend = nsend;
    st = hipMalloc(&d_hcols.p, sizeof(int) * std::max<size_t>(hcols.size(), 1)) == hipSuccess &&
                 hipMalloc(&d_sendg.p, sizeof(int) * std::max(nsend, 1)) == hipSuccess &&
                 (hcols.empty() || hipMemcpy(d_hcols.p, hcols.data(), sizeof(int) * hcols.size(),
                                             hipMemcpyHostToDevice) == hipSuccess)
             ? LSSP_AMD_OK
             : LSSP_AMD_ENOMEM;
    LSSP_TRY(agree_status(c, st));
    {
        std::vector<Msg> s, r;  // my halo columns to their owners; the columns peers need from me
        int *hc = static_cast<int *>(d_hcols.p), *sg = static_cast<int *>(d_sendg.p);
        for (size_t q = 0; q < M->recv_peer.size(); q++)
            s.push_back({M->recv_peer[q], hc + M->recv_off[q], (long)sizeof(int) * M->recv_cnt[q]});
        for (size_t q = 0; q < M->send_peer.size(); q++)
            r.push_back({M->send_peer[q], sg + M->send_off[q], (long)sizeof(int) * M->send_cnt[q]});
        LSSP_TRY(xfer_group(c, s, r));
    }
    std::vector<int> sendg(nsend);
    if (nsend)
        LSSP_HIP(hipMemcpyAsync(sendg.data(), d_sendg.p, sizeof(int) * nsend, hipMemcpyDeviceToHost, c->stream));
    LSSP_HIP(hipStreamSynchronize(c->stream));
    // a peer asking for a column this rank does not own: every rank learns it
    st = LSSP_AMD_OK;
    for (int &g : sendg) {
        if (g < row0 || g >= row0 + nlocal) st = LSSP_AMD_EINVAL;
        g -= row0;
    }
    LSSP_TRY(agree_status(c, st));
    // the matrix's own buffers (the largest allocations of the upload): a
    // failure becomes a status that every rank agrees on, and MatGuard frees
    // whatever was allocated
    auto dev_ok = [](hipError_t e) { return e == hipSuccess; };
    const bool ok =
        dev_ok(hipMalloc(&M->d_send_idx, sizeof(int) * std::max(nsend, 1))) &&
        dev_ok(hipMalloc(&M->d_send_buf, sizeof(double) * std::max(nsend, 1))) &&
        (!nsend || dev_ok(hipMemcpy(M->d_send_idx, sendg.data(), sizeof(int) * nsend, hipMemcpyHostToDevice))) &&
        dev_ok(hipMalloc(&M->Ap, sizeof(int) * (nlocal + 1))) &&
        dev_ok(hipMalloc(&M->Aj, sizeof(int) * ((size_t)nnz + 4))) &&  // +4: see upload_csr (capi.cpp)
        dev_ok(hipMalloc(&M->Ax, sizeof(double) * ((size_t)nnz + 4))) &&
        dev_ok(hipMemcpy(M->Ap, Ap, sizeof(int) * (nlocal + 1), hipMemcpyHostToDevice)) &&
        (!nnz || (dev_ok(hipMemcpy(M->Aj, lj.data(), sizeof(int) * (size_t)nnz, hipMemcpyHostToDevice)) &&
                  dev_ok(hipMemcpy(M->Ax, Ax, sizeof(double) * (size_t)nnz, hipMemcpyHostToDevice))));
    if (!ok) (void)hipGetLastError();  // clear the sticky error of a failed allocation
    LSSP_TRY(agree_status(c, ok ? LSSP_AMD_OK : LSSP_AMD_ENOMEM));
    LSSP_TRY(agree_status(c, build_diag_ids(M, Ap, lj.data())));  // the SpMV's column coding (capi.cpp)
    guard.m = nullptr;
    *out = M;
    return LSSP_AMD_OK;
}

}  // extern "C"
