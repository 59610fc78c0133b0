// psx_sweep_unit.h — one wave unit of the tiled sweep (k = 2, 3) as a device
// function, shared by k_sweep (psx_sweep.hip) and the k = 3 fast kernel's
// in-launch level-2 blocks (psx_sweep3.hip).
#ifndef PSX_SWEEP_UNIT_H
#define PSX_SWEEP_UNIT_H

#include "psx_sweep_dev.h"

namespace psx {

// LDS of one k_sweep unit (one wave)
struct SweepUnitSmem {
    Acc5 slot[64];     // c accumulators, ownership rotates every step
    Acc5 sacc[2][64];  // [0] a, [1] b accumulators, lane-owned
};

// One union set: per-study subset weights (n, mu) for the 2^K subsets (bit j =
// member j), zero-weighted where a member is absent from the study.  Folds the
// 3^K assignments (postcal.cpp:907-1030) into per-member records and the set's
// scalar record.
//
// notSharedLL (member j unshared) sums over assignment groups whose maximum sits
// Gll - GN_j bits below the set maximum.  The fast variant rescales the group
// sum by that gap (exact while the gap is <= 900 bits, i.e. unless j's
// quadratic gain exceeds ~900 bits in both studies) and raises *flag otherwise;
// the host then reruns the level with EXACT = true, which rescales each group's
// subset weights to the group's own maximum.
template <int K, bool EXACT>
__device__ __forceinline__ void fold_set_patterns(const TileArgs& A, const int (&nn)[2][1 << K],
                                                  const double (&mu)[2][1 << K], int Sm0, int Sm1,
                                                  double wcount, int* flag, Acc5 (&out)[K], SetRec& sr) {
    constexpr int NS = 1 << K;
    constexpr int FULL = NS - 1;
    constexpr int NP = (K == 2) ? 9 : 27;
    // pre-scale each study to its own top exponent (exact powers of two)
    const int nb0 = nn[0][FULL], nb1 = nn[1][FULL];
    double E0[NS], E1[NS];
#pragma unroll
    for (int T = 0; T < NS; T++) {
        E0[T] = ((T & ~Sm0) == 0) ? ldexp(mu[0][T], nn[0][T] - nb0) : 0.0;
        E1[T] = ((T & ~Sm1) == 0) ? ldexp(mu[1][T], nn[1][T] - nb1) : 0.0;
    }
    const int Gll = nb0 + nb1;  // E0 E1 < 4: values stay below 2^2 relative to Gll
    double Sw[K][3], Sl[K][3];
#pragma unroll
    for (int j = 0; j < K; j++)
#pragma unroll
        for (int x = 0; x < 3; x++) Sw[j][x] = Sl[j][x] = 0.0;
#pragma unroll
    for (int p = 0; p < NP; p++) {
        int c0 = 0, c1 = 0, nsh = 0, r = p;
        int x[K];
#pragma unroll
        for (int j = 0; j < K; j++) {
            x[j] = r % 3;  // 0: study0 only, 1: study1 only, 2: both
            r /= 3;
            if (x[j] != 1) c0 |= 1 << j;
            if (x[j] != 0) c1 |= 1 << j;
            if (x[j] == 2) nsh++;
        }
        const double wll = E0[c0] * E1[c1];
        const double w = wll * A.pit[nsh];
#pragma unroll
        for (int j = 0; j < K; j++) {
            Sw[j][x[j]] += w;
            Sl[j][x[j]] += wll;
        }
    }
    // notSharedLL groups: member j unshared, max pattern 2^{GN_j - 2}
    int GN[K], dmax = 0;
#pragma unroll
    for (int j = 0; j < K; j++) {
        const int bj = 1 << j;
        GN[j] = max(nb0 + nn[1][FULL ^ bj], nn[0][FULL ^ bj] + nb1);
        dmax = max(dmax, Gll - GN[j]);
    }
    double ns[K];
    if (!EXACT) {
        if (dmax > 900) atomicOr(flag, 1);
#pragma unroll
        for (int j = 0; j < K; j++) ns[j] = ldexp(Sl[j][0] + Sl[j][1], Gll - GN[j]);
    } else {
#pragma unroll
        for (int j = 0; j < K; j++) {
            const int bj = 1 << j;
            // group x_j = study0 only: C0 contains j, C1 within FULL ^ bj
            const int g1 = nb0 + nn[1][FULL ^ bj];
            // group x_j = study1 only: C1 contains j, C0 within FULL ^ bj
            const int g2 = nn[0][FULL ^ bj] + nb1;
            double s1 = 0.0, s2 = 0.0;
#pragma unroll
            for (int p = 0; p < NP; p++) {
                int c0 = 0, c1 = 0, r = p, xj = 0;
#pragma unroll
                for (int i = 0; i < K; i++) {
                    const int xi = r % 3;
                    r /= 3;
                    if (xi != 1) c0 |= 1 << i;
                    if (xi != 0) c1 |= 1 << i;
                    if (i == j) xj = xi;
                }
                if (xj == 2) continue;
                const bool ok = ((c0 & ~Sm0) == 0) && ((c1 & ~Sm1) == 0);
                const double m = ok ? mu[0][c0] * mu[1][c1] : 0.0;
                if (xj == 0) s1 += ldexp(m, nn[0][c0] + nn[1][c1] - g1);
                else s2 += ldexp(m, nn[0][c0] + nn[1][c1] - g2);
            }
            const int G = max(s1 != 0.0 ? g1 : EMPTY, s2 != 0.0 ? g2 : EMPTY);
            ns[j] = ldexp(s1, g1 - G) + ldexp(s2, g2 - G);
            GN[j] = G;
        }
    }
    const int GS = Gll + A.Ck;
#pragma unroll
    for (int j = 0; j < K; j++) {
        out[j].post0 = Sw[j][0] + Sw[j][2];
        out[j].post1 = Sw[j][1] + Sw[j][2];
        out[j].shared = Sw[j][2];
        out[j].mP = nz_shift(GS, out[j].post0 + out[j].post1);
        out[j].sll = Sl[j][2];
        out[j].mS = nz_shift(Gll, out[j].sll);
        out[j].nsll = ns[j];
        out[j].mN = nz_shift(GN[j], ns[j]);
        out[j].pad = 0;
    }
    sr.tot = Sw[0][0] + Sw[0][1] + Sw[0][2];
    sr.m = nz_shift(GS, sr.tot);
    // noCausal[s]: the assignment with C_s empty (all members in the other study)
    sr.nc0 = E1[FULL] * A.pit[0];
    sr.m0 = nz_shift(nb1 + A.Ck, sr.nc0);
    sr.nc1 = E0[FULL] * A.pit[0];
    sr.m1 = nz_shift(nb0 + A.Ck, sr.nc1);
    sr.pad = 0;
    sr.score = 1e300;
    sr.npat = wcount;
}


// Unit = (a-chunk or j-range, B, T): lane t owns b = 64B + t and walks the
// 64 x 64 (b, c) tile of T diagonally (psx_sweep.hip header comment).
template <int K, bool EXACT>
__device__ __forceinline__ void sweep_unit(const TileArgs& A, int unit, const int4* __restrict__ units,
                                           Acc5* __restrict__ rec, SetRec* __restrict__ srec, int rec_stride,
                                           int* __restrict__ flag, const int* __restrict__ pos, SweepUnitSmem& sm) {
    Acc5 (&slot)[64] = sm.slot;
    Acc5 (&sacc)[2][64] = sm.sacc;
    const int t = threadIdx.x;
    const int4 un = units[unit];
    const int a0 = un.x, a1 = un.y, B = un.z, T = un.w;
    const int b = 64 * B + t;
    const bool bvalid = b < A.U;
    const int tile = T * (T + 1) / 2 + B;
    const int ldg = A.ldg;
    slot[t] = acc_zero();
    sacc[1][t] = acc_zero();
    SetRec accs = set_zero();
    accs.m = accs.m0 = accs.m1 = EMPTY;
    const unsigned pb = bvalid ? A.pres[b] : 0u;
    // per-lane b terms
    double Abb[2], yb[2], iAbb[2], qb[2], rPb[2];
#pragma unroll
    for (int s = 0; s < 2; s++) {
        Abb[s] = A.Ad[s][b];
        yb[s] = A.y[s][b];
        const double r = rsqrt_nr(Abb[s]);
        iAbb[s] = r * r;
        qb[s] = yb[s] * yb[s] * iAbb[s];
        rPb[s] = r * A.rsd[s];
    }
    const int na = (K == 3) ? (a1 - a0) : 1;
    for (int ai = 0; ai < na; ai++) {
        const int a = a0 + ai;
        sacc[0][t] = acc_zero();
        constexpr int NS = 1 << K;
        double mu[2][NS];
        int nn[2][NS];
        // ---- hoisted prefix: subsets without c ------------------------------------------
        double iAaa[2], ya[2], Gab[2], qa[2], rPa[2], Dab[2], iDab[2], wab[2], qab[2], rPab[2];
        unsigned pa = 0;
#pragma unroll
        for (int s = 0; s < 2; s++) {
            mu[s][0] = 1.0;
            nn[s][0] = 0;
            if (K == 3) {
                const double Aaa = A.Ad[s][a];
                const double ra = rsqrt_nr(Aaa);
                iAaa[s] = ra * ra;
                ya[s] = A.y[s][a];
                Gab[s] = A.G[s][(size_t)a * ldg + b];
                qa[s] = ya[s] * ya[s] * iAaa[s];
                rPa[s] = ra * A.rsd[s];
                const double l = Gab[s] * iAaa[s];
                Dab[s] = Abb[s] - l * Gab[s];
                const double rab = rsqrt_nr(Dab[s]);
                iDab[s] = rab * rab;
                wab[s] = yb[s] - l * ya[s];
                qab[s] = qa[s] + wab[s] * wab[s] * iDab[s];
                rPab[s] = rPa[s] * rab * A.rsd[s];
                split2(0.5 * qa[s] * PSX_LOG2E, rPa[s], nn[s][1], mu[s][1]);     // {a}
                split2(0.5 * qb[s] * PSX_LOG2E, rPb[s], nn[s][2], mu[s][2]);     // {b}
                split2(0.5 * qab[s] * PSX_LOG2E, rPab[s], nn[s][3], mu[s][3]);   // {a,b}
            } else {
                split2(0.5 * qb[s] * PSX_LOG2E, rPb[s], nn[s][1], mu[s][1]);     // {b}
            }
        }
        if (K == 3) pa = A.pres[a];
        const bool abvalid = bvalid && (K == 2 || a < b);
        const double wab_cnt = memb_weight(pb) * (K == 3 ? memb_weight(pa) : 1.0);
        // k = 2 units carry a j-range of the diagonal walk in (a0, a1)
        const int j0 = (K == 2) ? a0 : 0, j1 = (K == 2) ? a1 : 64;
        for (int j = j0; j < j1; j++) {
            const int cc = (t + j) & 63;
            const int c = 64 * T + cc;
            const bool act = abvalid && c < A.U && (B < T || cc > t);
            if (act) {
                const unsigned pc = A.pres[c];
#pragma unroll
                for (int s = 0; s < 2; s++) {
                    const double Acc_ = A.Ad[s][c];
                    const double yc = A.y[s][c];
                    const double Gbc = A.skew[s][(size_t)tile * 4096 + j * 64 + t];
                    constexpr int IC = (K == 3) ? 4 : 2, IBC = (K == 3) ? 6 : 3;
                    mu[s][IC] = A.muS[s][c];  // {c}: precomputed per SNP
                    nn[s][IC] = A.nS[s][c];
                    // {b, c}
                    const double l2 = Gbc * iAbb[s];
                    const double D2 = Acc_ - l2 * Gbc;
                    const double w2 = yc - l2 * yb[s];
                    const double r2 = rsqrt_nr(D2);
                    const double t2 = w2 * r2;
                    split2(0.5 * (qb[s] + t2 * t2) * PSX_LOG2E, rPb[s] * r2 * A.rsd[s], nn[s][IBC], mu[s][IBC]);
                    if (K == 3) {
                        const double Gac = A.G[s][(size_t)a * ldg + c];
                        // {a, c}
                        const double l1 = Gac * iAaa[s];
                        const double D1 = Acc_ - l1 * Gac;
                        const double w1 = yc - l1 * ya[s];
                        const double r1 = rsqrt_nr(D1);
                        const double t1 = w1 * r1;
                        split2(0.5 * (qa[s] + t1 * t1) * PSX_LOG2E, rPa[s] * r1 * A.rsd[s], nn[s][5], mu[s][5]);
                        // {a, b, c}: extend the (a, b) factor by the c row
                        const double lcb = (Gbc - l1 * Gab[s]) * iDab[s];
                        const double D3 = D1 - lcb * lcb * Dab[s];
                        const double w3 = w1 - lcb * wab[s];
                        const double r3 = rsqrt_nr(D3);
                        const double t3 = w3 * r3;
                        split2(0.5 * (qab[s] + t3 * t3) * PSX_LOG2E, rPab[s] * r3 * A.rsd[s], nn[s][7], mu[s][7]);
                    }
                }
                int Sm0, Sm1;
                if (K == 3) {
                    Sm0 = (pa & 1) | ((pb & 1) << 1) | ((pc & 1) << 2);
                    Sm1 = ((pa >> 1) & 1) | (((pb >> 1) & 1) << 1) | (((pc >> 1) & 1) << 2);
                } else {
                    Sm0 = (pb & 1) | ((pc & 1) << 1);
                    Sm1 = ((pb >> 1) & 1) | (((pc >> 1) & 1) << 1);
                }
                Acc5 out[K];
                SetRec sr;
                fold_set_patterns<K, EXACT>(A, nn, mu, Sm0, Sm1, wab_cnt * memb_weight(pc), flag, out, sr);
                ffold1(accs.m, accs.tot, sr.m, sr.tot);
                ffold1(accs.m0, accs.nc0, sr.m0, sr.nc0);
                ffold1(accs.m1, accs.nc1, sr.m1, sr.nc1);
                accs.npat += sr.npat;
                if (K == 3) {
                    Acc5 x = sacc[0][t];
                    ffold_acc(x, out[0]);
                    sacc[0][t] = x;
                }
                {
                    Acc5 x = sacc[1][t];
                    ffold_acc(x, out[K - 2]);
                    sacc[1][t] = x;
                }
                Acc5 sl = slot[cc];
                ffold_acc(sl, out[K - 1]);
                slot[cc] = sl;
            }
            __syncthreads();  // slot[] ownership rotates across lanes every step
        }
        if (K == 3) {
            Acc5 acca = sacc[0][t];
            wave_fold_acc(acca);
            if (t == 0) put_rec(rec, pos, (size_t)unit * rec_stride + 128 + ai, acca);
        }
    }
    __syncthreads();
    put_rec(rec, pos, (size_t)unit * rec_stride + t, slot[t]);
    put_rec(rec, pos, (size_t)unit * rec_stride + 64 + t, sacc[1][t]);
    wave_fold_set(accs);
    if (t == 0) store_rec(srec + unit, accs);
}

}  // namespace psx
#endif
