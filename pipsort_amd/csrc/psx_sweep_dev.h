// psx_sweep_dev.h — device helpers shared by the sweep kernels (psx_sweep.hip,
// psx_sweep3.hip): tile arguments, branch-free (m, s) folds, wave reductions,
// full-precision rsqrt and the base-2 split of subset weights.
#ifndef PSX_SWEEP_DEV_H
#define PSX_SWEEP_DEV_H

#include <hip/hip_runtime.h>

#include "psx_math.h"

namespace psx {

struct TileArgs {
    const double* G[2];
    const double* Ad[2];
    const double* y[2];
    const double* skew[2];
    const double* muS[2];  // singleton weights {c}: mu of 2^{h_c} (d A_cc)^{-1/2}
    const int* nS[2];      // and its integer exponent floor(h_c)
    const unsigned char* pres;
    double d[2], rsd[2];   // d_s and d_s^{-1/2}
    int U, ldg, Ck;
    double pit[4];
};

// level-2 units launched as extra blocks of the k = 3 fast kernel
struct Level2Blocks {
    int n;
    TileArgs A;
    const int4* units;
    Acc5* rec;
    SetRec* srec;
    const int* pos;
};

constexpr int EMPTY = -(1 << 28);  // shift of an empty accumulator (value 0)

__device__ inline Acc5 acc_zero() {
    Acc5 a;
    a.mP = a.mS = a.mN = EMPTY;
    a.pad = 0;
    a.post0 = a.post1 = a.shared = a.sll = a.nsll = 0.0;
    return a;
}

__device__ inline Acc5 shfl_acc5(const Acc5& a, int o) {
    Acc5 b;
    b.mP = __shfl_xor(a.mP, o);
    b.mS = __shfl_xor(a.mS, o);
    b.mN = __shfl_xor(a.mN, o);
    b.pad = 0;
    b.post0 = __shfl_xor(a.post0, o);
    b.post1 = __shfl_xor(a.post1, o);
    b.shared = __shfl_xor(a.shared, o);
    b.sll = __shfl_xor(a.sll, o);
    b.nsll = __shfl_xor(a.nsll, o);
    return b;
}

__device__ inline SetRec shfl_set(const SetRec& a, int o) {
    SetRec b;
    b.m = __shfl_xor(a.m, o);
    b.m0 = __shfl_xor(a.m0, o);
    b.m1 = __shfl_xor(a.m1, o);
    b.pad = 0;
    b.tot = __shfl_xor(a.tot, o);
    b.nc0 = __shfl_xor(a.nc0, o);
    b.nc1 = __shfl_xor(a.nc1, o);
    b.score = __shfl_xor(a.score, o);
    b.npat = __shfl_xor(a.npat, o);
    return b;
}

__device__ inline void wave_fold_acc(Acc5& a) {
    for (int o = 1; o < 64; o <<= 1) {
        Acc5 b = shfl_acc5(a, o);
        fold_acc(a, b);
    }
}
__device__ inline void wave_fold_set(SetRec& a) {
    for (int o = 1; o < 64; o <<= 1) {
        SetRec b = shfl_set(a, o);
        fold_set(a, b);
    }
}

// Branch-free folds for the hot loop.  Empty accumulators and empty
// contributions carry shift EMPTY, so max() never lets a zero raise a shift.
__device__ __forceinline__ void ffold1(int32_t& m, double& s, int32_t m2, double s2) {
    const int M = max(m, m2);
    s = ldexp(s, m - M) + ldexp(s2, m2 - M);
    m = M;
}
__device__ __forceinline__ void ffold_acc(Acc5& a, const Acc5& b) {
    const int M = max(a.mP, b.mP);
    a.post0 = ldexp(a.post0, a.mP - M) + ldexp(b.post0, b.mP - M);
    a.post1 = ldexp(a.post1, a.mP - M) + ldexp(b.post1, b.mP - M);
    a.shared = ldexp(a.shared, a.mP - M) + ldexp(b.shared, b.mP - M);
    a.mP = M;
    ffold1(a.mS, a.sll, b.mS, b.sll);
    ffold1(a.mN, a.nsll, b.mN, b.nsll);
}
__device__ __forceinline__ int nz_shift(int m, double s) { return s != 0.0 ? m : EMPTY; }

// 1/sqrt(x) to full double precision: v_rsq_f64 + two Newton steps
__device__ __forceinline__ double rsqrt_nr(double x) {
    double y = __builtin_amdgcn_rsq(x);
    double e = fma(-x * y, y, 1.0);
    y = fma(0.5 * y, e, y);
    e = fma(-x * y, y, 1.0);
    return fma(0.5 * y, e, y);
}

// 2^f for f in [0, 1): sqrt(2) e^t, t = (f - 1/2) ln 2, degree-12 Taylor (|err| < 2e-16)
__device__ __forceinline__ double exp2_frac(double f) {
    const double t = (f - 0.5) * PSX_LN2;
    double p = 2.08767569878680989792e-09;      // 1/12!
    p = fma(p, t, 2.50521083854417187751e-08);  // 1/11!
    p = fma(p, t, 2.75573192239858906526e-07);  // 1/10!
    p = fma(p, t, 2.75573192239858906526e-06);  // 1/9!
    p = fma(p, t, 2.48015873015873015873e-05);  // 1/8!
    p = fma(p, t, 1.98412698412698412698e-04);  // 1/7!
    p = fma(p, t, 1.38888888888888888889e-03);  // 1/6!
    p = fma(p, t, 8.33333333333333333333e-03);  // 1/5!
    p = fma(p, t, 4.16666666666666666667e-02);  // 1/4!
    p = fma(p, t, 1.66666666666666666667e-01);  // 1/3!
    p = fma(p, t, 0.5);
    p = fma(p, t, 1.0);
    p = fma(p, t, 1.0);
    return p * 1.41421356237309504880;
}

// weight 2^h * rP as (n, mu), n = floor(h), mu in (0, 2)
__device__ __forceinline__ void split2(double h, double rP, int& n, double& mu) {
    const double fl = floor(h);
    n = (int)fl;
    mu = exp2_frac(h - fl) * rP;
}

// Record stores (plain stores: non-temporal ones were measured neutral at
// world 1 and slower at world 8, EXPERIMENTS.md A).
template <typename T>
__device__ __forceinline__ void store_rec(T* dst, const T& v) {
    *dst = v;
}

// record slot i goes to buffer position pos[i] (-1: no SNP; the merges gather by SNP)
__device__ __forceinline__ void put_rec(Acc5* rec, const int* pos, size_t i, const Acc5& v) {
    const int q = pos[i];
    if (q >= 0) store_rec(rec + q, v);
}

__device__ __forceinline__ double memb_weight(unsigned p) { return p == 3u ? 3.0 : (p ? 1.0 : 0.0); }

}  // namespace psx
#endif
