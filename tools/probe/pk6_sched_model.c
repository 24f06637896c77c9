// packet-DAG model of build_packets6 + k_tri_pk6 (analysis aid): ring size R,
// HBM-operand cap X per packet, row cap RC per packet
#include <stdlib.h>
#include <string.h>
void model2(int n, const int *Lp, const int *Lj, int B, int R, int X, int RC, double tau, double hop, double *out)
{
    int *lev = malloc(sizeof(int) * n);
    int maxl = 0;
    for (int i = 0; i < n; i++) {
        int l = 0;
        for (int k = Lp[i]; k < Lp[i + 1]; k++) if (Lj[k] < i && lev[Lj[k]] + 1 > l) l = lev[Lj[k]] + 1;
        lev[i] = l; if (l > maxl) maxl = l;
    }
    int nb = (n + B - 1) / B;
    int *pos = malloc(sizeof(int) * n), *perm = malloc(sizeof(int) * n), *pk = malloc(sizeof(int) * n);
    int *cnt = malloc(sizeof(int) * (maxl + 2));
    int *stamp = malloc(sizeof(int) * n);
    for (int i = 0; i < n; i++) stamp[i] = -1;
    // pass 1: positions (block, level, q)
    for (int b = 0; b < nb; b++) {
        int q0 = b * B, q1 = q0 + B < n ? q0 + B : n;
        memset(cnt, 0, sizeof(int) * (maxl + 2));
        for (int q = q0; q < q1; q++) cnt[lev[q] + 1]++;
        for (int l = 1; l <= maxl + 1; l++) cnt[l] += cnt[l - 1];
        for (int q = q0; q < q1; q++) { int p = q0 + cnt[lev[q]]++; perm[p] = q; pos[q] = p; }
    }
    // pass 2: packets
    long npk = 0; int pid = 0;
    long *bstart = malloc(sizeof(long) * (nb + 1));
    double *T = malloc(sizeof(double) * (long)n);  // per packet (<= n packets)
    double *dep = malloc(sizeof(double) * (long)n);
    double span = 0, lagsum = 0, prevstart = 0;
    for (int b = 0; b < nb; b++) {
        int q0 = b * B, q1 = q0 + B < n ? q0 + B : n;
        bstart[b] = npk;
        int p = q0;
        while (p < q1) {
            int l = lev[perm[p]];
            int e = p; while (e < q1 && lev[perm[e]] == l) e++;   // the level's rows [p, e)
            while (p < e) {
                int nr = 0, nx = 0;
                while (p + nr < e && nr < RC) {
                    int r = perm[p + nr], newx = 0;
                    for (int k = Lp[r]; k < Lp[r + 1]; k++) {
                        int c = Lj[k]; if (c >= r) continue;
                        int ring = (c >= q0) && (e - pos[c] <= R);
                        if (!ring && stamp[c] != pid) newx++;
                    }
                    if (nx + newx > X) break;
                    for (int k = Lp[r]; k < Lp[r + 1]; k++) {
                        int c = Lj[k]; if (c >= r) continue;
                        int ring = (c >= q0) && (e - pos[c] <= R);
                        if (!ring && stamp[c] != pid) { stamp[c] = pid; nx++; }
                    }
                    pk[r] = (int)npk;
                    nr++;
                }
                dep[npk] = 0;
                p += nr; npk++; pid++;
            }
        }
        // timing of this block's packets
        for (long a = bstart[b]; a < npk; a++) dep[a] = 0;
        for (int q = q0; q < q1; q++) {
            long a = pk[q];
            for (int k = Lp[q]; k < Lp[q + 1]; k++) { int c = Lj[k]; if (c < q0) { double t = T[pk[c]] + hop; if (t > dep[a]) dep[a] = t; } }
        }
        double t = 0;
        for (long a = bstart[b]; a < npk; a++) { double s = t > dep[a] ? t : dep[a]; if (a == bstart[b]) { if (b) lagsum += s - prevstart; prevstart = s; } T[a] = s + tau; t = T[a]; }
        if (t > span) span = t;
    }
    out[0] = maxl + 1; out[1] = npk / (double)nb; out[2] = span; out[3] = lagsum / (nb > 1 ? nb - 1 : 1);
    free(lev); free(pos); free(perm); free(pk); free(cnt); free(stamp); free(bstart); free(T); free(dep);
}
