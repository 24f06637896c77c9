// tri_bp.cpp -- host setup of the block-pipelined triangular sweeps
// (k_tri_pk6, trisolve.hip).
//
// The factor's rows, in sweep order (q = r for L, q = n-1-r for U), are cut
// into contiguous blocks of B rows with B >= the factor's bandwidth, so every
// dependency of a row lies in its own block or in earlier ones.  One
// workgroup takes a block and walks it level by level ("steps"); values it
// needs from its own block come from an LDS ring of recent results, values
// from earlier blocks from HBM, where value-as-flag (TRI_SENTINEL) makes a
// not-yet-written value visible as such.  Only one cross-CU hand-off per block
// boundary is on the critical path instead of one per level.  The per-row
// arithmetic is untouched (entries in the reference's order), so the sweep
// stays bitwise.
#include <algorithm>
#include <atomic>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>

#include "internal.h"

namespace lssp_amd {

int build_bp_schedule(lssp_amd_ctx *c, int n, const std::vector<int> &Tp, const std::vector<int> &Tj,
                      const std::vector<double> &Tx, bool upper, const std::vector<int> &lev, TriSched &t,
                      const TriSched *prod)
{
    (void)c;
    if (n <= 0) return LSSP_AMD_OK;
    SetupTimer tm;
    const char *side = upper ? "U" : "L";
    std::string nm;
    auto mark = [&](const char *what) {
        nm = std::string(side) + " " + what;
        tm.mark(nm.c_str());
    };
    auto Q = [&](int r) { return upper ? n - 1 - r : r; };
    auto strict_begin = [&](int i) { return upper ? Tp[i] + 1 : Tp[i]; };
    auto strict_end = [&](int i) { return upper ? Tp[i + 1] : Tp[i + 1] - 1; };
    bool unit = true;
    int bw = 1;
    {
        std::mutex mu;
        parallel_for(n, [&](long i0, long i1) {
            bool u = true;
            int w = 1;
            for (long i = i0; i < i1; i++) {
                u &= (upper ? Tx[Tp[i]] : Tx[Tp[i + 1] - 1]) == 1.0;
                for (int k = strict_begin((int)i); k < strict_end((int)i); k++) w = std::max(w, std::abs((int)i - Tj[k]));
            }
            std::lock_guard<std::mutex> g(mu);
            unit &= u;
            bw = std::max(bw, w);
        });
    }
    mark("bandwidth");
    long B = std::max(64L, (long)bw);  // one bandwidth per block: measured best
    if (B > n) B = n;
    const int nb = (int)((n + B - 1) / B);

    // rows of each block ordered by (level, q); blocks are independent (threads),
    // their step lists are concatenated in block order
    std::vector<int> perm(n), pos(n);
    std::vector<std::vector<int>> bsp(nb), bsl(nb);
    parallel_for(nb, [&](long b0, long b1) {
        for (long b = b0; b < b1; b++) {
            const long q0 = b * B, q1 = std::min<long>(q0 + B, n);
            int lmin = INT_MAX, lmax = 0;
            for (long q = q0; q < q1; q++) {
                const int r = upper ? n - 1 - (int)q : (int)q;
                lmin = std::min(lmin, lev[r]);
                lmax = std::max(lmax, lev[r]);
            }
            std::vector<int> cnt(lmax - lmin + 2, 0);
            for (long q = q0; q < q1; q++) cnt[lev[upper ? n - 1 - (int)q : (int)q] - lmin + 1]++;
            for (size_t l = 1; l < cnt.size(); l++) cnt[l] += cnt[l - 1];
            for (int l = 0; l <= lmax - lmin; l++)
                if (cnt[l + 1] > cnt[l]) {
                    bsp[b].push_back((int)q0 + cnt[l]);
                    bsl[b].push_back(l + lmin);
                }
            for (long q = q0; q < q1; q++) {
                const int r = upper ? n - 1 - (int)q : (int)q;
                const int p = (int)q0 + cnt[lev[r] - lmin]++;
                perm[p] = r;
                pos[r] = p;
            }
        }
    }, 1);
    mark("block level order");
    std::vector<int> step_pos, blk_step(nb + 1, 0);
    for (int b = 0; b < nb; b++) {
        blk_step[b] = (int)step_pos.size();
        step_pos.insert(step_pos.end(), bsp[b].begin(), bsp[b].end());
    }
    const int nsteps = (int)step_pos.size();
    blk_step[nb] = nsteps;
    step_pos.push_back(n);
    std::vector<int> step_of(n);
    parallel_for(nsteps, [&](long s0, long s1) {
        for (long s = s0; s < s1; s++)
            for (int p = step_pos[s]; p < step_pos[s + 1]; p++) step_of[p] = (int)s;
    }, 64);

    // entries in summation order; intra-block dependencies still inside the
    // ring window come from LDS (code -1 - slot), everything else from HBM
    std::vector<int> rp(n + 1, 0);
    for (int p = 0; p < n; p++) rp[p + 1] = rp[p] + strict_end(perm[p]) - strict_begin(perm[p]);
    // uninitialised: every slot is written below, by the position threads
    std::unique_ptr<int[]> cols(new int[std::max(rp[n], 1)]);
    std::unique_ptr<double[]> vals(new double[std::max(rp[n], 1)]);
    std::vector<double> diag;
    if (!unit) diag.resize(n);
    parallel_for(n, [&](long p0, long p1) {
        for (long p = p0; p < p1; p++) {
            const int i = perm[p], b = (int)(Q(i) / B), s = step_of[p];
            int o = rp[p];
            auto take = [&](int k) {
                const int j = Tj[k];
                const int bj = (int)(Q(j) / B);
                int code = j;
                if (bj == b) {
                    const int pd = pos[j];
                    if (step_pos[s + 1] - pd <= BP_RING) code = -1 - (int)((pd - (long)b * B) % BP_RING);
                }
                cols[o] = code;
                vals[o] = Tx[k];
                o++;
            };
            if (!upper)
                for (int k = Tp[i]; k < Tp[i + 1] - 1; k++) take(k);
            else
                for (int k = Tp[i + 1] - 1; k > Tp[i]; k--) take(k);
            if (!unit) diag[p] = upper ? Tx[Tp[i]] : Tx[Tp[i + 1] - 1];
        }
    });
    mark("entries in sweep order");
    {
        // v6 packets; the rhs of the U sweep is the L sweep's output, read in
        // L's schedule order (the L sweep's rhs is permuted into L order first)
        std::vector<int> rhs_index(n);
        parallel_for(n, [&](long r0, long r1) {
            for (long r = r0; r < r1; r++) rhs_index[r] = prod && !prod->h_pos.empty() ? prod->h_pos[r] : pos[r];
        });
        const int st6 = build_packets6(n, perm, pos, rp, cols.get(), vals.get(), diag, unit, step_pos, blk_step, nb, B,
                                       rhs_index, t);
        // a row longer than the longest record: the sync-free sweep serves the factor
        if (st6 == LSSP_AMD_EUNSUPPORTED) t.pk6_n = -1;
        else if (st6 != LSSP_AMD_OK) return st6;
        if (!upper) t.h_pos = pos;
    }
    mark("packets (incl. upload)");
    t.bp_B = (int)B;
    t.upper = upper;
    t.bp_nb = nb;
    t.bp_nsteps = nsteps;
    auto up = [](auto *&d, const auto &h) -> int {
        using T = typename std::remove_reference<decltype(h)>::type::value_type;
        LSSP_HIP(hipMalloc(&d, sizeof(T) * std::max<size_t>(h.size(), 1)));
        if (!h.empty()) LSSP_HIP(hipMemcpy(d, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice));
        return LSSP_AMD_OK;
    };
    LSSP_TRY(up(t.bp_perm, perm));  // position -> row: the apply's permutation kernels
    LSSP_TRY(up(t.bp_pos, pos));    // row -> position: x back to natural order as a gather
    mark("permutation upload");
    return LSSP_AMD_OK;
}

// Packets v6 (trisolve.hip k_tri_pk6).  The sweeps exchange values
// through "shadow" vectors kept in schedule order (position p holds the value
// of row perm[p]), so the cross-block operands of a packet and its output are
// contiguous runs instead of one cache line per row.  Per packet:
//   desc  int4 {record offset (16 B units), index offset (4 B units),
//               nr | nx << 10 | emax << 21, schedule position of the first row}
//   records (compute lanes), arrays over the packet's rows, 16-byte aligned:
//     C  operand addresses as uint16 pairs, EP/2 words per row: uint2 (EP 4) or
//        uint4 chunks (EP 8, 16, 24) -- the operand's byte offset in the
//        kernel's LDS operand array (pk6_xs_off: a value-ring slot, the +0.0
//        pad slot, or the packet's landed HBM operand, whose buffer is the
//        packet's parity within its block), so the compute lanes read each
//        operand with no decoding
//     V[EP/2] double2 entry values, D double diagonal, ROW int (natural row)
//   indices (loader lanes): rhs[nr] (the rhs entry of each row: its L-schedule
//     position, for both sweeps -- the L sweep reads the rhs permuted into L
//     order, the U sweep reads the L sweep's shadow), xidx[nx] (schedule
//     positions of the HBM operands in this sweep's own shadow)
int build_packets6(int n, const std::vector<int> &perm, const std::vector<int> &pos, const std::vector<int> &rp,
                   const int *cols, const double *vals,
                   const std::vector<double> &diag, bool unit, const std::vector<int> &step_pos,
                   const std::vector<int> &blk_step, int nb, long B, const std::vector<int> &rhs_index,
                   TriSched &t)
{
    const int ROWS = 256;  // rows per packet = compute lanes (512 measured slower)
    int maxlen = 0;
    for (int p = 0; p < n; p++) maxlen = std::max(maxlen, rp[p + 1] - rp[p]);
    if (maxlen > 24) return LSSP_AMD_EUNSUPPORTED;  // ILUT(tol, p <= 24), ILU(k) of stencils
    const int EP = maxlen <= 4 ? 4 : maxlen <= 8 ? 8 : maxlen <= 16 ? 16 : 24;
    // record words of a packet of n rows (C, V, D, ROW, each padded to 4 words);
    // EP >= 16 records are staged through a 16 KB LDS slot (trisolve.hip LREC)
    auto rec_words = [&](long nrow) {
        auto p4 = [](long w) { return (w + 3) & ~3L; };
        return p4((long)(EP / 2) * nrow) + 2L * EP * nrow + p4(2 * nrow) + p4(nrow);
    };
    constexpr long PK6_REC_WORDS16 = 1024;  // 16-byte units (trisolve.hip PK6_REC16)
    auto pack = [](int a, int b) { return (uint32_t)((a & 0xffff) | ((uint32_t)(b & 0xffff) << 16)); };
    // blocks are independent: each thread builds its blocks' packets with
    // block-relative record / index offsets and its own operand stamps; the
    // blocks are then laid out in order and the offsets made absolute
    struct BlkPk {
        std::vector<int> desc;
        std::vector<uint32_t> rec;
        std::vector<int> idx;
    };
    // The HBM operands a packet may gather (xcap = EXT x 256: the loader lanes
    // fetch EXT each).  A packet is closed early when its rows' new operands
    // would pass the cap, so a small cap splits levels into several packets,
    // and every packet is a step of its block (7-pt 256^3 ILUT: 512 split 1,580
    // levels into 2,546 packets per block, profiles/r06/r06k_*; the U factor
    // needs 1,024).  Each extra load per lane costs the step ~3 %, so the
    // packets are first counted for EXT = 2, 3, 4 and the smallest EXT whose
    // count is within 1 % of EXT = 4's is kept.
    auto packets_at = [&](int cap) {
        std::atomic<long> total{0};
        parallel_for(nb, [&](long b0, long b1) {
            std::vector<int> stamp(n, -1);
            int pid = 0;
            long cnt = 0;
            for (long b = b0; b < b1; b++)
                for (int s = blk_step[b]; s < blk_step[b + 1]; s++) {
                    int p = step_pos[s];
                    while (p < step_pos[s + 1]) {
                        int nr = 0, nx = 0;
                        while (p + nr < step_pos[s + 1] && nr < ROWS) {
                            const int r = p + nr;
                            if (EP >= 16 && rec_words(nr + 1) > 4 * PK6_REC_WORDS16) break;
                            int newx = 0;
                            for (int k = rp[r]; k < rp[r + 1]; k++)
                                if (cols[k] >= 0 && stamp[cols[k]] != pid) newx++;
                            if (nx + newx > cap) break;
                            for (int k = rp[r]; k < rp[r + 1]; k++)
                                if (cols[k] >= 0 && stamp[cols[k]] != pid) stamp[cols[k]] = pid, nx++;
                            nr++;
                        }
                        p += nr;
                        pid++;
                        cnt++;
                    }
                }
            total += cnt;
        }, 1);
        return total.load();
    };
    int ext = PK3_EXT;
    {
        const long c4 = packets_at(ROWS * PK3_EXT);
        for (int e = 2; e < PK3_EXT; e++)
            if (packets_at(ROWS * e) <= c4 + c4 / 100) {
                ext = e;
                break;
            }
    }
    const int xcap = ROWS * ext;
    std::vector<BlkPk> bp(nb);
    std::atomic<int> status{LSSP_AMD_OK};
    parallel_for(nb, [&](long b0, long b1) {
        std::vector<int> stamp(n, -1), slot(n, 0), xl;
        int pid = 0;
        for (long b = b0; b < b1 && status.load() == LSSP_AMD_OK; b++) {
            std::vector<int> &desc = bp[b].desc, &idx = bp[b].idx;
            std::vector<uint32_t> &rec = bp[b].rec;
            {
                // the block's packets at most: one per row, each array padded by
                // < 4 words -- reserved so the multi-MB vectors never regrow
                const long rows = std::min<long>((b + 1) * B, n) - b * B;
                const int steps = blk_step[b + 1] - blk_step[b];
                rec.reserve((size_t)(rows * ((EP / 2) + 2 * EP + 3) + 12L * (rows / 8 + steps + 1)));
                idx.reserve((size_t)(rows * (1 + PK3_EXT) + 8));
                desc.reserve((size_t)4 * (rows / 8 + steps + 1));
            }
            static_assert(pk6_xs_off(BP_RING + 1, 1, ROWS * PK3_EXT - 1) <= 0xffff, "16-bit operand offsets");
            for (int s = blk_step[b]; s < blk_step[b + 1]; s++) {
                int p = step_pos[s];
                while (p < step_pos[s + 1]) {
                    int nr = 0, emax = 0;
                    xl.clear();
                    while (p + nr < step_pos[s + 1] && nr < ROWS) {
                        const int r = p + nr;
                        if (EP >= 16 && rec_words(nr + 1) > 4 * PK6_REC_WORDS16) break;  // LDS record slot
                        int newx = 0;
                        for (int k = rp[r]; k < rp[r + 1]; k++)
                            if (cols[k] >= 0 && stamp[cols[k]] != pid) newx++;
                        if ((long)xl.size() + newx > (long)xcap) break;
                        for (int k = rp[r]; k < rp[r + 1]; k++) {
                            const int g = cols[k];
                            if (g >= 0 && stamp[g] != pid) {
                                stamp[g] = pid;
                                slot[g] = (int)xl.size();
                                xl.push_back(g);
                            }
                        }
                        emax = std::max(emax, rp[r + 1] - rp[r]);
                        nr++;
                    }
                    const int nx = (int)xl.size();
                    const int par = (int)(desc.size() / 4) & 1;  // the packet's index in its block, mod 2
                    const long ro = (long)rec.size() / 4, io = (long)idx.size();  // block-relative
                    desc.push_back((int)ro);
                    desc.push_back((int)io);
                    desc.push_back(nr | (nx << 10) | (emax << 21));
                    desc.push_back(p);
                    // C: (EP/2) words per row, V: 2*EP, D: 2, ROW: 1 -- each array padded to 4 words
                    auto pad4 = [](long w) { return (w + 3) & ~3L; };
                    const long wc = pad4((long)(EP / 2) * nr), wv = 2L * EP * nr, wd = pad4(2L * nr), wr = pad4(nr);
                    rec.resize(rec.size() + wc + wv + wd + wr, 0u);
                    uint32_t *w = rec.data() + 4 * ro;
                    double *V = reinterpret_cast<double *>(w + wc);
                    double *D = V + (long)EP * nr;
                    uint32_t *ROW = w + wc + wv + wd;
                    for (int r = 0; r < nr; r++) {
                        const int k0 = rp[p + r], len = rp[p + r + 1] - k0;
                        int cc[24];
                        for (int e = 0; e < 24; e++) cc[e] = pk6_xs_off(BP_RING, 0, 0);  // the +0.0 pad slot
                        for (int e = 0; e < len; e++) {
                            const int g = cols[k0 + e];
                            cc[e] = g < 0 ? pk6_xs_off(-1 - g, 0, 0) : pk6_xs_off(BP_RING + 1, par, slot[g]);
                            V[2L * ((long)(e / 2) * nr + r) + (e & 1)] = vals[k0 + e];
                        }
                        for (int q = 0; q < EP / 2; q++) w[(long)(EP / 2) * r + q] = pack(cc[2 * q], cc[2 * q + 1]);
                        D[r] = unit ? 1.0 : diag[p + r];
                        ROW[r] = (uint32_t)perm[p + r];
                    }
                    for (int r = 0; r < nr; r++) idx.push_back(rhs_index[perm[p + r]]);
                    for (int x = 0; x < nx; x++) idx.push_back(pos[xl[x]]);
                    p += nr;
                    pid++;
                }
            }
            if ((int)desc.size() / 4 > PK3_CAP) status = LSSP_AMD_EUNSUPPORTED;
        }
    }, 1);
    if (status.load() != LSSP_AMD_OK) return status.load();
    // lay the blocks out in order; offsets absolute
    std::vector<int> blk(nb + 1, 0);
    std::vector<long> rec_off(nb + 1, 0), idx_off(nb + 1, 0);
    for (int b = 0; b < nb; b++) {
        blk[b + 1] = blk[b] + (int)bp[b].desc.size() / 4;
        rec_off[b + 1] = rec_off[b] + (long)bp[b].rec.size();
        idx_off[b + 1] = idx_off[b] + (long)bp[b].idx.size();
    }
    if (rec_off[nb] / 4 > INT_MAX || idx_off[nb] > INT_MAX) return LSSP_AMD_EUNSUPPORTED;
    // the blocks laid out in order (offsets made absolute) in uninitialised
    // host arrays, filled by the block threads in parallel -- no single-thread
    // zero fill of the multi-GB record stream -- then one upload each
    SetupTimer tm;
    t.pk6_n = blk[nb];
    t.pk6_ep = EP;
    t.pk6_ext = ext;
    t.pk6_rows = ROWS;
    const size_t ndesc = std::max<size_t>(4L * blk[nb], 1), nrec = rec_off[nb] + 4, nidx = idx_off[nb] + 1;
    std::unique_ptr<int[]> desc(new int[ndesc]);
    std::unique_ptr<uint32_t[]> rec(new uint32_t[nrec]);
    std::unique_ptr<int[]> idx(new int[nidx]);
    std::fill(rec.get() + rec_off[nb], rec.get() + nrec, 0u);  // the kernels' whole-unit reads past the end
    idx[nidx - 1] = 0;
    desc[0] = 0;
    parallel_for(nb, [&](long b0, long b1) {
        for (long b = b0; b < b1; b++) {
            BlkPk &k = bp[b];
            int *d = desc.get() + 4L * blk[b];
            for (size_t e = 0; e < k.desc.size(); e += 4) {
                d[e] = k.desc[e] + (int)(rec_off[b] / 4);
                d[e + 1] = k.desc[e + 1] + (int)idx_off[b];
                d[e + 2] = k.desc[e + 2];
                d[e + 3] = k.desc[e + 3];
            }
            std::copy(k.rec.begin(), k.rec.end(), rec.get() + rec_off[b]);
            std::copy(k.idx.begin(), k.idx.end(), idx.get() + idx_off[b]);
            k = BlkPk();  // the block's host copy is done with
        }
    }, 1);
    bp.clear();
    auto up = [](auto *&d, const auto *h, size_t cnt) -> int {
        using T = typename std::remove_const<typename std::remove_pointer<decltype(h)>::type>::type;
        LSSP_HIP(hipMalloc(&d, sizeof(T) * cnt));
        LSSP_HIP(hipMemcpy(d, h, sizeof(T) * cnt, hipMemcpyHostToDevice));
        return LSSP_AMD_OK;
    };
    LSSP_TRY(up(t.pk6_blk, blk.data(), blk.size()));
    LSSP_TRY(up(t.pk6_desc, desc.get(), ndesc));
    LSSP_TRY(up(t.pk6_rec, rec.get(), nrec));
    LSSP_TRY(up(t.pk6_idx, idx.get(), nidx));
    tm.mark("packet upload");
    LSSP_HIP(hipMalloc(&t.pk6_claim, sizeof(unsigned long long)));
    LSSP_HIP(hipMemset(t.pk6_claim, 0, sizeof(unsigned long long)));
    t.pk6_base = 0;
    return LSSP_AMD_OK;
}

}  // namespace lssp_amd
