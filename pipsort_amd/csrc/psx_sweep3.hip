// psx_sweep3.hip — the k = 3 exhaustive level (postcal.cpp:716-1092 for
// |union set| = 3), the dominant kernel of the sweep.
//
// Same tiling as k_sweep (psx_sweep.hip): a unit is (a-chunk, B, T), lane t
// owns b = 64B + t and walks c = 64T + ((t + j) & 63) diagonally, so the 64
// per-c accumulators rotate through LDS without atomics.  This kernel is
// VALU-issue bound (every wave64 VALU op costs ~4 cycles, FP64 or integer
// alike; HBM traffic is negligible), so it is built to minimise the VALU
// instruction count per union set:
//
//  * everything indexed by c (A diag, scaled y, singleton weights, presence
//    factors) and the Sigma~ row of a are staged in LDS once per unit / per a
//    and read with immediate offsets — no per-step address arithmetic;
//  * y is pre-scaled by sqrt(log2(e)/2), so every quadratic form is directly
//    the base-2 exponent h_T of the subset weight;
//  * 1/sqrt(pivot) is v_rsq_f64 (5e-8 relative on gfx950, tools/rsq_acc.hip)
//    plus ONE Newton step (4e-15), kept scaled by 2 so it costs three ops;
//  * 2^h is split as 2^n * mu by a round-to-nearest magic add, a 256-entry
//    2^(i/256) table in LDS and a degree-4 polynomial on |t| < 0.00136;
//  * the prior is multiplicative per member (prior_nats, postcal.cpp:198-212):
//    pit[nsh] = pit0 * rho^nsh, so the 27 assignments are folded with shared
//    row / column partial sums and pit0 is applied once per record;
//  * accumulators keep a lazy shift: a contribution at shift G is added with
//    one power-of-two scale and the shift only moves (rarely, in one
//    wave-uniform branch) when G exceeds it by > 960 bits.  Contributions more than ~1022 bits below
//    an accumulator's own running maximum vanish, exactly as in the
//    branch-free fold they replace.
//
// Absent members (mixed loci) are masked by zeroing their pivot factor, which
// zeroes every subset weight containing them (checkOR of postcal.cpp:907-955).
// notSharedLL groups more than ~900 bits below a set's scale raise *flag; the
// host then reruns the level with k_sweep<3, true> (exact group scaling).
#include <hip/hip_runtime.h>

#include <string>

#include "psx_sweep.h"
#include "psx_sweep_dev.h"

namespace psx {

constexpr double kMagic = 6755399441055744.0;  // 1.5 * 2^52: round-to-nearest-integer add
constexpr double kTinyNs = 0x1p-900;            // notSharedLL group floor of the fast path
// e^{f ln2 / 256} = sum_k q_k f^k, |f| <= 1/2 (degree 4, error < 4e-17)
constexpr double kQ1 = PSX_LN2 / 256.0;
constexpr double kQ2 = kQ1 * kQ1 / 2.0;
constexpr double kQ3 = kQ2 * kQ1 / 3.0;
constexpr double kQ4 = kQ3 * kQ1 / 4.0;

// lane-local accumulator with a lazy shift: value = 2^m * s
struct LAcc {
    int m;
    double p0, p1, sh, sl, ns;
};

__device__ __forceinline__ void lacc_zero(LAcc& a) {
    a.m = EMPTY;
    a.p0 = a.p1 = a.sh = a.sl = a.ns = 0.0;
}

// 2/sqrt(x): v_rsq_f64 + one Newton step y (3 - x y^2) without its exact 1/2
// (3 VALU ops; the factor 2 is absorbed by halved y and rsd in the c step)
__device__ __forceinline__ double rsq2x(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    const double u = x * y;
    return y * fma(-u, y, 3.0);
}

// 2^h * rP = 2^n * mu (mu in [0.99, 2.01) * rP): N = round(256 h), n = N >> 8,
// mu = tab[N & 255] * 2^{f/256} * rP with f = 256 h - N (exact)
__device__ __forceinline__ void split3(double h, double rP, const double* tab, int& n, double& mu) {
    const double xr = fma(h, 256.0, kMagic);
    const int N = __double2loint(xr);
    const double kf = xr - kMagic;
    const double f = fma(h, 256.0, -kf);
    double p = fma(kQ4, f, kQ3);
    p = fma(p, f, kQ2);
    p = fma(p, f, kQ1);
    p = fma(p, f, 1.0);
    n = N >> 8;
    mu = tab[N & 255] * p * rP;
}

// lazy accumulator: move the shift up to G (values scale down exactly)
__device__ __forceinline__ void lacc_shift(LAcc& a, int G) {
    const int d = a.m - G;
    a.p0 = ldexp(a.p0, d);
    a.p1 = ldexp(a.p1, d);
    a.sh = ldexp(a.sh, d);
    a.sl = ldexp(a.sl, d);
    a.ns = ldexp(a.ns, d);
    a.m = G;
}

// add a contribution already scaled to the accumulator's shift by f = 2^{G - m}
__device__ __forceinline__ void lacc_add(LAcc& a, double f, double p0, double p1, double sh, double sl, double ns) {
    a.p0 = fma(p0, f, a.p0);
    a.p1 = fma(p1, f, a.p1);
    a.sh = fma(sh, f, a.sh);
    a.sl = fma(sl, f, a.sl);
    a.ns = fma(ns, f, a.ns);
}

// lazy accumulator -> merge record (Acc5 convention: P at +Ck, values * pit0)
__device__ __forceinline__ Acc5 lacc_rec(const LAcc& a, int Ck, double pit0) {
    Acc5 r;
    r.post0 = a.p0 * pit0;
    r.post1 = a.p1 * pit0;
    r.shared = a.sh * pit0;
    r.sll = a.sl;
    r.nsll = a.ns;
    r.mP = (r.post0 + r.post1 != 0.0) ? a.m + Ck : EMPTY;
    r.mS = (a.sl != 0.0) ? a.m : EMPTY;
    r.mN = (a.ns != 0.0) ? a.m : EMPTY;
    r.pad = 0;
    return r;
}

template <bool ALLPRES>
__global__ __launch_bounds__(64, 2) void k_sweep3(Sweep3Args A, const int4* __restrict__ units,
                                                  Acc5* __restrict__ rec, SetRec* __restrict__ srec, int rec_stride,
                                                  int* __restrict__ flag) {
    __shared__ double tab[256];
    __shared__ double cA[2][64], cY[2][64], cMu[2][64], cR[2][64], gA[2][64];
    __shared__ int cN[2][64];
    __shared__ double cW[64];
    __shared__ double sP0[64], sP1[64], sSh[64], sSl[64], sNs[64];
    __shared__ int sM[64];

    const int unit = blockIdx.x;
    const int t = threadIdx.x;
    const int4 un = units[unit];
    const int a0 = un.x, a1 = un.y, B = un.z, T = un.w;
    const int b = 64 * B + t;
    const bool bvalid = b < A.U;
    const int tile = T * (T + 1) / 2 + B;
    const int ldg = A.ldg;
    const double rho = A.rho;

    // ---- unit prologue: stage the c-tile ------------------------------------------
    for (int i = t; i < 256; i += 64) tab[i] = A.tab[i];
    {
        const int c = 64 * T + t;  // < ldg: arrays are padded to ldg
        const unsigned pc = A.pres[c];
#pragma unroll
        for (int s = 0; s < 2; s++) {
            const bool in = ALLPRES || ((pc >> s) & 1u);
            cA[s][t] = A.Ad[s][c];
            cY[s][t] = 0.5 * A.ys[s][c];  // halved: pivots come out as 2/sqrt(D)
            cMu[s][t] = in ? A.muS[s][c] : 0.0;
            cN[s][t] = A.nS[s][c];
            cR[s][t] = in ? 0.5 * A.rsd[s] : 0.0;
        }
        cW[t] = memb_weight(pc);
    }
    sM[t] = EMPTY;
    sP0[t] = sP1[t] = sSh[t] = sSl[t] = sNs[t] = 0.0;
    __syncthreads();

    // ---- per-lane b terms ------------------------------------------------------------
    const unsigned pb = bvalid ? A.pres[b] : 0u;
    // rP*X: pivot-factor products, times one more rsd when every SNP is in both
    // studies (then the c pivot factor is r_c alone; otherwise r_c * cR[c])
    double Abb[2], yb[2], ybh[2], iAbb[2], hb[2], rPb[2], rPbX[2], chib[2], muB[2];
    int nB[2];
#pragma unroll
    for (int s = 0; s < 2; s++) {
        chib[s] = (ALLPRES || ((pb >> s) & 1u)) ? 1.0 : 0.0;
        Abb[s] = A.Ad[s][b];
        yb[s] = A.ys[s][b];
        ybh[s] = 0.5 * yb[s];
        const double r = rsqrt_nr(Abb[s]);
        iAbb[s] = r * r;
        hb[s] = yb[s] * yb[s] * iAbb[s];
        rPb[s] = r * A.rsd[s] * chib[s];
        rPbX[s] = ALLPRES ? rPb[s] * (0.5 * A.rsd[s]) : rPb[s];
        split3(hb[s], rPb[s], tab, nB[s], muB[s]);
    }
    const double wb = memb_weight(pb);

    LAcc accB;
    lacc_zero(accB);
    double totB = 0.0;
    int m0 = EMPTY, m1 = EMPTY;
    double nc0 = 0.0, nc1 = 0.0, npat = 0.0;

    const double* sk0 = A.skew[0] + (size_t)tile * 4096 + t;
    const double* sk1 = A.skew[1] + (size_t)tile * 4096 + t;

    for (int ai = 0; ai < a1 - a0; ai++) {
        const int a = a0 + ai;
        // Sigma~ row of a over the c-tile
#pragma unroll
        for (int s = 0; s < 2; s++) gA[s][t] = A.G[s][(size_t)a * ldg + 64 * T + t];
        const unsigned pa = A.pres[a];
        double iAaa[2], yah[2], rPaX[2], Gab[2], Dab[2], iDab[2], wabh[2], hab[2], ha[2], rPabX[2];
        // c-free subsets relative to 2^{n_ab}: E'[0] = {}, [1] = {a}, [2] = {b}, [3] = {a,b}
        double Ep[2][4];
        int nAB[2];
#pragma unroll
        for (int s = 0; s < 2; s++) {
            const double chia = (ALLPRES || ((pa >> s) & 1u)) ? 1.0 : 0.0;
            const double ra = rsqrt_nr(A.Ad[s][a]);
            iAaa[s] = ra * ra;
            const double ya = A.ys[s][a];
            yah[s] = 0.5 * ya;
            ha[s] = ya * ya * iAaa[s];
            const double rPa = ra * A.rsd[s] * chia;
            rPaX[s] = ALLPRES ? rPa * (0.5 * A.rsd[s]) : rPa;
            int nA;
            double muA, muAB;
            split3(ha[s], rPa, tab, nA, muA);
            Gab[s] = A.G[s][(size_t)a * ldg + b];
            const double l = Gab[s] * iAaa[s];
            Dab[s] = fma(-l, Gab[s], Abb[s]);
            const double rab = rsqrt_nr(Dab[s]);
            iDab[s] = rab * rab;
            const double wab = fma(-l, ya, yb[s]);
            wabh[s] = 0.5 * wab;
            hab[s] = fma(wab * wab, iDab[s], ha[s]);
            const double rPab = rPa * rab * A.rsd[s] * chib[s];
            rPabX[s] = ALLPRES ? rPab * (0.5 * A.rsd[s]) : rPab;
            split3(hab[s], rPab, tab, nAB[s], muAB);
            // n_ab >= n_a, n_b (nested quadratic forms), so these never overflow; a
            // term that underflows sits > 1022 bits below its set's {a,b} weight
            Ep[s][0] = ldexp(1.0, -nAB[s]);
            Ep[s][1] = ldexp(muA, nA - nAB[s]);
            Ep[s][2] = ldexp(muB[s], nB[s] - nAB[s]);
            Ep[s][3] = muAB;
        }
        const bool abvalid = bvalid && a < b;
        const double wab_cnt = wb * memb_weight(pa);
        LAcc accA;
        lacc_zero(accA);
        __syncthreads();  // gA visible

        for (int j = 0; j < 64; j++) {
            const int cc = (t + j) & 63;
            const int c = 64 * T + cc;
            const bool act = abvalid && c < A.U && (B < T || cc > t);
            if (act) {
                double E[2][8];
                int nb[2];
#pragma unroll
                for (int s = 0; s < 2; s++) {
                    const double Acc_ = cA[s][cc];
                    const double yc = cY[s][cc];
                    const double Gbc = (s ? sk1 : sk0)[j * 64];
                    const double Gac = gA[s][cc];
                    // {b, c}
                    const double l2 = Gbc * iAbb[s];
                    const double D2 = fma(-l2, Gbc, Acc_);
                    const double w2 = fma(-l2, ybh[s], yc);
                    const double r2 = rsq2x(D2);
                    const double t2 = w2 * r2;
                    const double h2 = fma(t2, t2, hb[s]);
                    // {a, c}
                    const double l1 = Gac * iAaa[s];
                    const double D1 = fma(-l1, Gac, Acc_);
                    const double w1 = fma(-l1, yah[s], yc);
                    const double r1 = rsq2x(D1);
                    const double t1 = w1 * r1;
                    const double h1 = fma(t1, t1, ha[s]);
                    // {a, b, c}: extend the (a, b) factor by the c row
                    const double lcb = fma(-l1, Gab[s], Gbc) * iDab[s];
                    const double u3 = lcb * Dab[s];
                    const double D3 = fma(-u3, lcb, D1);
                    const double w3 = fma(-lcb, wabh[s], w1);
                    const double r3 = rsq2x(D3);
                    const double t3 = w3 * r3;
                    const double h3 = fma(t3, t3, hab[s]);
                    double rP2, rP1, rP3;
                    if (ALLPRES) {
                        rP2 = rPbX[s] * r2;
                        rP1 = rPaX[s] * r1;
                        rP3 = rPabX[s] * r3;
                    } else {
                        const double rc = cR[s][cc];  // rsd_s, or 0 when c is absent from study s
                        rP2 = rPbX[s] * (r2 * rc);
                        rP1 = rPaX[s] * (r1 * rc);
                        rP3 = rPabX[s] * (r3 * rc);
                    }
                    int n1, n2, n3;
                    double mu1, mu2, mu3;
                    split3(h2, rP2, tab, n2, mu2);
                    split3(h1, rP1, tab, n1, mu1);
                    split3(h3, rP3, tab, n3, mu3);
                    const int nbs = n3;
                    nb[s] = nbs;
                    // subset weights relative to 2^nb (bit 0 = a, bit 1 = b, bit 2 = c)
                    const int dd = nAB[s] - nbs;
                    E[s][0] = ldexp(Ep[s][0], dd);
                    E[s][1] = ldexp(Ep[s][1], dd);
                    E[s][2] = ldexp(Ep[s][2], dd);
                    E[s][3] = ldexp(Ep[s][3], dd);
                    E[s][4] = ldexp(cMu[s][cc], cN[s][cc] - nbs);
                    E[s][5] = ldexp(mu1, n1 - nbs);
                    E[s][6] = ldexp(mu2, n2 - nbs);
                    E[s][7] = mu3;
                }
                const int Gll = nb[0] + nb[1];
                // ---- 27 study assignments: x = 0 study0 only, 1 study1 only, 2 both ----
                // wll = E0[C0] E1[C1];  C0 = {j : x_j != 1},  C1 = {j : x_j != 0}
                double A1[3], Ar[3], A22[3];
                double sllA = 0.0, nsA = 0.0, sllB = 0.0, nsB = 0.0;
                double SwA[3], SwB[3];
#pragma unroll
                for (int xa = 0; xa < 3; xa++) {
#pragma unroll
                    for (int xb = 0; xb < 3; xb++) {
                        double w[3];
#pragma unroll
                        for (int xc = 0; xc < 3; xc++) {
                            const int c0 = (xa != 1) | ((xb != 1) << 1) | ((xc != 1) << 2);
                            const int c1 = (xa != 0) | ((xb != 0) << 1) | ((xc != 0) << 2);
                            w[xc] = E[0][c0] * E[1][c1];
                        }
                        const double s01 = w[0] + w[1];
                        const double Pl = s01 + w[2];
                        const double Pw = fma(rho, w[2], s01);
                        // column partials by how many of (a, b) are shared
                        const int cls = (xa == 2) + (xb == 2);
#pragma unroll
                        for (int xc = 0; xc < 3; xc++) {
                            if (cls == 0) A1[xc] = (xa == 0 && xb == 0) ? w[xc] : A1[xc] + w[xc];
                            else if (cls == 1) Ar[xc] = (xa == 0 && xb == 2) ? w[xc] : Ar[xc] + w[xc];
                            else A22[xc] = w[xc];
                        }
                        // member a / member b marginals
                        if (xa == 2) sllA = (xb == 0) ? Pl : sllA + Pl;
                        else nsA = (xa == 0 && xb == 0) ? Pl : nsA + Pl;
                        if (xb == 2) sllB = (xa == 0) ? Pl : sllB + Pl;
                        else nsB = (xa == 0 && xb == 0) ? Pl : nsB + Pl;
                        if (xb == 0) SwA[xa] = Pw;
                        else if (xb == 1) SwA[xa] += Pw;
                        else SwA[xa] = fma(rho, Pw, SwA[xa]);
                        if (xa == 0) SwB[xb] = Pw;
                        else if (xa == 1) SwB[xb] += Pw;
                        else SwB[xb] = fma(rho, Pw, SwB[xb]);
                    }
                }
                SwA[2] *= rho;
                SwB[2] *= rho;
                double SwC[3], Rl[3];
#pragma unroll
                for (int xc = 0; xc < 3; xc++) {
                    Rl[xc] = A1[xc] + Ar[xc] + A22[xc];
                    SwC[xc] = fma(rho, fma(rho, A22[xc], Ar[xc]), A1[xc]);
                }
                SwC[2] *= rho;
                const double sllC = Rl[2];
                const double nsC = Rl[0] + Rl[1];
                const double tot = SwA[0] + SwA[1] + SwA[2];
                if (__builtin_amdgcn_ballot_w64((nsA < kTinyNs) | (nsB < kTinyNs) | (nsC < kTinyNs)))
                    if (nsA < kTinyNs || nsB < kTinyNs || nsC < kTinyNs) atomicOr(flag, 1);
                const bool nz = tot != 0.0;
                // ---- folds: a, b (registers), c (LDS slot, rotating owner), noCausal ----
                LAcc sl;
                sl.m = sM[cc];
                sl.p0 = sP0[cc];
                sl.p1 = sP1[cc];
                sl.sh = sSh[cc];
                sl.sl = sSl[cc];
                sl.ns = sNs[cc];
                int dA = Gll - accA.m, dB = Gll - accB.m, dS = Gll - sl.m;
                // noCausal[s]: the assignment with C_s empty (every member in the other study)
                double x0 = ldexp(E[1][7], nb[1] - m0), x1 = ldexp(E[0][7], nb[0] - m1);
                const bool up = (nz & (max(dA, max(dB, dS)) > 960)) | (x0 > 0x1p960) | (x1 > 0x1p960);
                if (__builtin_amdgcn_ballot_w64(up)) {  // wave-uniform, rare: move shifts up
                    if (nz && dA > 960) { lacc_shift(accA, Gll); dA = 0; }
                    if (nz && dB > 960) { lacc_shift(accB, Gll); totB = ldexp(totB, -dB); dB = 0; }
                    if (nz && dS > 960) { lacc_shift(sl, Gll); dS = 0; }
                    if (x0 > 0x1p960) { nc0 = ldexp(nc0, m0 - nb[1]); m0 = nb[1]; x0 = E[1][7]; }
                    if (x1 > 0x1p960) { nc1 = ldexp(nc1, m1 - nb[0]); m1 = nb[0]; x1 = E[0][7]; }
                }
                nc0 += x0;
                nc1 += x1;
                lacc_add(accA, ldexp(1.0, min(dA, 1000)), SwA[0] + SwA[2], SwA[1] + SwA[2], SwA[2], sllA, nsA);
                const double fB = ldexp(1.0, min(dB, 1000));
                lacc_add(accB, fB, SwB[0] + SwB[2], SwB[1] + SwB[2], SwB[2], sllB, nsB);
                totB = fma(tot, fB, totB);
                lacc_add(sl, ldexp(1.0, min(dS, 1000)), SwC[0] + SwC[2], SwC[1] + SwC[2], SwC[2], sllC, nsC);
                sM[cc] = sl.m;
                sP0[cc] = sl.p0;
                sP1[cc] = sl.p1;
                sSh[cc] = sl.sh;
                sSl[cc] = sl.sl;
                sNs[cc] = sl.ns;
                npat += ALLPRES ? 27.0 : wab_cnt * cW[cc];
            }
            __syncthreads();  // slot ownership rotates across lanes every step
        }
        Acc5 ra = lacc_rec(accA, A.Ck, A.pit0);
        wave_fold_acc(ra);
        if (t == 0) rec[(size_t)unit * rec_stride + 128 + ai] = ra;
    }
    {
        LAcc sl;
        sl.m = sM[t];
        sl.p0 = sP0[t];
        sl.p1 = sP1[t];
        sl.sh = sSh[t];
        sl.sl = sSl[t];
        sl.ns = sNs[t];
        rec[(size_t)unit * rec_stride + t] = lacc_rec(sl, A.Ck, A.pit0);
    }
    rec[(size_t)unit * rec_stride + 64 + t] = lacc_rec(accB, A.Ck, A.pit0);
    SetRec sr;
    sr.tot = totB * A.pit0;
    sr.m = (sr.tot != 0.0) ? accB.m + A.Ck : EMPTY;
    sr.nc0 = nc0 * A.pit0;
    sr.m0 = (sr.nc0 != 0.0) ? m0 + A.Ck : EMPTY;
    sr.nc1 = nc1 * A.pit0;
    sr.m1 = (sr.nc1 != 0.0) ? m1 + A.Ck : EMPTY;
    sr.pad = 0;
    sr.score = 1e300;
    sr.npat = npat;
    wave_fold_set(sr);
    if (t == 0) srec[unit] = sr;
}

int launch_sweep3(bool allpres, const Sweep3Args& A, int n_units, const int4* units, Acc5* rec, SetRec* srec,
                  int rec_stride, int* flag, hipStream_t st) {
    if (allpres)
        hipLaunchKernelGGL((k_sweep3<true>), dim3(n_units), dim3(64), 0, st, A, units, rec, srec, rec_stride, flag);
    else
        hipLaunchKernelGGL((k_sweep3<false>), dim3(n_units), dim3(64), 0, st, A, units, rec, srec, rec_stride, flag);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// y * sqrt(log2(e) / 2): quadratic forms of the scaled y are base-2 exponents
__global__ void k_scale_y(const double* __restrict__ y, int n, double* __restrict__ ys) {
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u < n) ys[u] = y[u] * 0.84932180028801904272;  // sqrt(log2(e) / 2)
}

int launch_scale_y(const double* y, int n, double* ys, hipStream_t st) {
    hipLaunchKernelGGL(k_scale_y, dim3((n + 255) / 256), dim3(256), 0, st, y, n, ys);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace psx
