// tri_bp.cpp -- host setup of the block-pipelined triangular sweep (tri_mode 3).
//
// The factor's rows, in sweep order (q = r for L, q = n-1-r for U), are cut
// into contiguous blocks of B rows with B >= the factor's bandwidth, so every
// dependency of a row lies in its own block or in the previous one.  One
// workgroup takes a block and walks it level by level ("steps"); values it
// needs from its own block come from an LDS ring of recent results, values
// from the previous block are read once that block's progress word says the
// needed level is complete.  Only one cross-CU hand-off per block boundary is
// on the critical path instead of one per level.  The per-row arithmetic is
// untouched (entries in the reference's order), so the sweep stays bitwise.
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>

#include "internal.h"

namespace lssp_amd {

int build_bp_schedule(lssp_amd_ctx *c, int n, const std::vector<int> &Tp, const std::vector<int> &Tj,
                      const std::vector<double> &Tx, bool upper, const std::vector<int> &lev, TriSched &t)
{
    (void)c;
    if (n <= 0) return LSSP_AMD_OK;
    auto Q = [&](int r) { return upper ? n - 1 - r : r; };
    auto strict_begin = [&](int i) { return upper ? Tp[i] + 1 : Tp[i]; };
    auto strict_end = [&](int i) { return upper ? Tp[i + 1] : Tp[i + 1] - 1; };
    bool unit = true;
    int bw = 1;
    for (int i = 0; i < n; i++) {
        unit &= (upper ? Tx[Tp[i]] : Tx[Tp[i + 1] - 1]) == 1.0;
        for (int k = strict_begin(i); k < strict_end(i); k++) bw = std::max(bw, std::abs(i - Tj[k]));
    }
    const char *em = getenv("LSSP_AMD_TRI_BP_MULT");
    long mult = em ? atol(em) : 0;
    const long nbw = (n + (long)bw - 1) / bw;
    if (mult <= 0) mult = 1;  // measured best on 7-pt 216^3 (tools/bench_trisolve.py)
    (void)nbw;
    long B = std::max(64L, mult * (long)bw);
    if (B > n) B = n;
    const int nb = (int)((n + B - 1) / B);
    const char *ep = getenv("LSSP_AMD_TRI_BP_PUBLISH");
    const int publish_every = ep ? std::max(1, atoi(ep)) : 1;

    // rows of each block ordered by (level, q)
    std::vector<int> perm(n), pos(n);
    std::vector<int> step_pos, step_lev, blk_step(nb + 1, 0);
    for (int b = 0; b < nb; b++) {
        const long q0 = (long)b * B, q1 = std::min<long>(q0 + B, n);
        int lmin = INT_MAX, lmax = 0;
        for (long q = q0; q < q1; q++) {
            const int r = upper ? n - 1 - (int)q : (int)q;
            lmin = std::min(lmin, lev[r]);
            lmax = std::max(lmax, lev[r]);
        }
        std::vector<int> cnt(lmax - lmin + 2, 0);
        for (long q = q0; q < q1; q++) cnt[lev[upper ? n - 1 - (int)q : (int)q] - lmin + 1]++;
        for (size_t l = 1; l < cnt.size(); l++) cnt[l] += cnt[l - 1];
        blk_step[b] = (int)step_lev.size();
        for (int l = 0; l <= lmax - lmin; l++)
            if (cnt[l + 1] > cnt[l]) {
                step_pos.push_back((int)q0 + cnt[l]);
                step_lev.push_back(l + lmin);
            }
        for (long q = q0; q < q1; q++) {
            const int r = upper ? n - 1 - (int)q : (int)q;
            const int p = (int)q0 + cnt[lev[r] - lmin]++;
            perm[p] = r;
            pos[r] = p;
        }
    }
    const int nsteps = (int)step_lev.size();
    blk_step[nb] = nsteps;
    step_pos.push_back(n);
    std::vector<int> step_of(n);
    for (int s = 0; s < nsteps; s++)
        for (int p = step_pos[s]; p < step_pos[s + 1]; p++) step_of[p] = s;

    // entries in summation order; intra-block dependencies still inside the
    // ring window come from LDS (code -1 - slot), everything else from HBM
    std::vector<int> rp(n + 1, 0), cols, need(nsteps, -1), done(nsteps), flag(nsteps, 0);
    std::vector<double> vals, diag;
    if (!unit) diag.resize(n);
    cols.reserve(Tj.size());
    vals.reserve(Tj.size());
    for (int p = 0; p < n; p++) {
        const int i = perm[p], b = (int)(Q(i) / B), s = step_of[p];
        auto take = [&](int k) {
            const int j = Tj[k];
            const int bj = (int)(Q(j) / B);
            int code = j;
            if (bj == b) {
                const int pd = pos[j];
                if (step_pos[s + 1] - pd <= BP_RING) code = -1 - (int)((pd - (long)b * B) % BP_RING);
                else flag[step_of[pd]] |= 1;  // drain right after the producing step
            } else {
                need[s] = std::max(need[s], lev[j]);
            }
            cols.push_back(code);
            vals.push_back(Tx[k]);
        };
        if (!upper)
            for (int k = Tp[i]; k < Tp[i + 1] - 1; k++) take(k);
        else
            for (int k = Tp[i + 1] - 1; k > Tp[i]; k--) take(k);
        if (!unit) diag[p] = upper ? Tx[Tp[i]] : Tx[Tp[i + 1] - 1];
        rp[p + 1] = (int)cols.size();
    }
    for (int b = 0; b < nb; b++)
        for (int s = blk_step[b], k = 0; s < blk_step[b + 1]; s++, k++) {
            const bool last = s + 1 == blk_step[b + 1];
            done[s] = last ? INT_MAX - 2 : step_lev[s + 1] - 1;
            if (last || (k + 1) % publish_every == 0) flag[s] |= 1;
        }

    {
        const int st = build_packets(n, perm, rp, cols, vals, diag, unit, step_pos, blk_step, nb, B, t);
        if (st == LSSP_AMD_EUNSUPPORTED) t.pk_n = -1;  // a row too long for a packet: mode 2 serves it
        else if (st != LSSP_AMD_OK) return st;
    }
    t.bp_B = (int)B;
    t.bp_nb = nb;
    t.bp_nsteps = nsteps;
    auto up = [](auto *&d, const auto &h) -> int {
        using T = typename std::remove_reference<decltype(h)>::type::value_type;
        LSSP_HIP(hipMalloc(&d, sizeof(T) * std::max<size_t>(h.size(), 1)));
        if (!h.empty()) LSSP_HIP(hipMemcpy(d, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice));
        return LSSP_AMD_OK;
    };
    LSSP_TRY(up(t.bp_perm, perm));
    LSSP_TRY(up(t.bp_rp, rp));
    LSSP_TRY(up(t.bp_cols, cols));
    LSSP_TRY(up(t.bp_vals, vals));
    if (!unit) LSSP_TRY(up(t.bp_diag, diag));
    LSSP_TRY(up(t.bp_step_pos, step_pos));
    LSSP_TRY(up(t.bp_step_need, need));
    LSSP_TRY(up(t.bp_step_done, done));
    LSSP_TRY(up(t.bp_step_flag, flag));
    LSSP_TRY(up(t.bp_blk_step, blk_step));
    LSSP_HIP(hipMalloc(&t.bp_prog, sizeof(unsigned long long) * nb));
    LSSP_HIP(hipMemset(t.bp_prog, 0, sizeof(unsigned long long) * nb));
    LSSP_HIP(hipMalloc(&t.bp_claim, sizeof(unsigned long long)));
    LSSP_HIP(hipMemset(t.bp_claim, 0, sizeof(unsigned long long)));
    t.bp_base = 0;
    t.bp_epoch = 0;
    return LSSP_AMD_OK;
}

// Packet layout (4-byte words, every packet 16-byte aligned):
//   [0] nrows  [1] nent  [2] block-local position of the first row  [3] 0
//   rows[nrows]  rp[nrows+1] (packet-local)  codes[nent]  (pad to 8 bytes)
//   vals[nent] (double)  diag[nrows] (double, only when the diagonal is not 1)
// A packet holds rows of ONE step (level) of one block, in schedule order.
int build_packets(int n, const std::vector<int> &perm, const std::vector<int> &rp,
                  const std::vector<int> &cols, const std::vector<double> &vals,
                  const std::vector<double> &diag, bool unit, const std::vector<int> &step_pos,
                  const std::vector<int> &blk_step, int nb, long B, TriSched &t)
{
    auto words = [&](int nr, int ne) {
        long w = 5 + 2L * nr + ne;
        w = (w + 1) & ~1L;
        w += 2L * ne + (unit ? 0 : 2L * nr);
        return (w + 3) & ~3L;
    };
    std::vector<int> blk(nb + 1, 0), off(1, 0);
    std::vector<uint32_t> data;
    for (int b = 0; b < nb; b++) {
        blk[b] = (int)off.size() - 1;
        for (int s = blk_step[b]; s < blk_step[b + 1]; s++) {
            int p = step_pos[s];
            while (p < step_pos[s + 1]) {
                int nr = 0, ne = 0;
                while (p + nr < step_pos[s + 1] && nr < PK_ROWS) {
                    const int e = rp[p + nr + 1] - rp[p + nr];
                    if (words(nr + 1, ne + e) * 4 > PK_BYTES) break;
                    nr++;
                    ne += e;
                }
                if (nr == 0) return LSSP_AMD_EUNSUPPORTED;  // one row does not fit a packet
                const size_t o = data.size();
                data.resize(o + words(nr, ne), 0u);
                uint32_t *w = data.data() + o;
                w[0] = nr;
                w[1] = ne;
                w[2] = (uint32_t)(p - (long)b * B);
                for (int r = 0; r < nr; r++) w[4 + r] = (uint32_t)perm[p + r];
                for (int r = 0; r <= nr; r++) w[4 + nr + r] = (uint32_t)(rp[p + r] - rp[p]);
                for (int e = 0; e < ne; e++) w[5 + 2 * nr + e] = (uint32_t)cols[rp[p] + e];
                long vo = (5 + 2L * nr + ne + 1) & ~1L;
                memcpy(w + vo, vals.data() + rp[p], sizeof(double) * ne);
                if (!unit) memcpy(w + vo + 2L * ne, diag.data() + p, sizeof(double) * nr);
                off.push_back((int)(data.size() / 4));
                p += nr;
            }
        }
    }
    blk[nb] = (int)off.size() - 1;
    t.pk_n = (int)off.size() - 1;
    LSSP_HIP(hipMalloc(&t.pk_blk, sizeof(int) * (nb + 1)));
    LSSP_HIP(hipMemcpy(t.pk_blk, blk.data(), sizeof(int) * (nb + 1), hipMemcpyHostToDevice));
    LSSP_HIP(hipMalloc(&t.pk_off, sizeof(int) * off.size()));
    LSSP_HIP(hipMemcpy(t.pk_off, off.data(), sizeof(int) * off.size(), hipMemcpyHostToDevice));
    LSSP_HIP(hipMalloc(&t.pk_data, sizeof(uint32_t) * std::max<size_t>(data.size(), 4)));
    if (!data.empty())
        LSSP_HIP(hipMemcpy(t.pk_data, data.data(), sizeof(uint32_t) * data.size(), hipMemcpyHostToDevice));
    LSSP_HIP(hipMalloc(&t.pk_claim, sizeof(unsigned long long)));
    LSSP_HIP(hipMemset(t.pk_claim, 0, sizeof(unsigned long long)));
    t.pk_base = 0;
    (void)n;
    return LSSP_AMD_OK;
}

}  // namespace lssp_amd
