// psx_math.h — numerics shared by the MI355X kernels and the host orchestration.
//
// Representation.  Every PostCal accumulator (postcal.h:62-78) is a log-sum-exp
// of per-configuration log values.  The reference keeps it as a double in log
// space and folds terms with addlogSpace (postcal.h:102-112).  On the GPU each
// accumulator is a pair (m, s) meaning  value = 2^m * s  (m an int32 shift in
// base 2, s >= 0 a double), with the configuration-independent constant
// K = -||S'||^2 / 2 (postcal.cpp:285-287, 799-803) factored out.  Folding two
// pairs needs only max / ldexp / add — no log or exp — so partial sums from
// lanes, waves, workgroups and GPUs merge exactly and associatively, every
// accumulator keeps its own dynamic range (the reference's LL columns span
// thousands of nats), and terms more than ~1074 bits below the running value
// vanish exactly as addlogSpace drops terms > 700 nats down.
//
// Per configuration (postcal.cpp:214-304 with postcal.cpp:250 keeping only the
// diagonal of sigmaC and model.h:239 making B block diagonal), the low-rank
// likelihood separates by study:
//   ll = K + sum_s f_s(C_s),  f_s(T) = q_T/2 - ln(P_T)/2,
//   A_T = diag(1/d_s) + Sigma~_s[T,T] = L D L^T,  q_T = y_T^T A_T^-1 y_T,
//   P_T = prod_i d_s D_i = det(I + D_s Sigma~_s[T,T])
// (Woodbury + Sylvester on the reference's tmp_CC = I + U V).  The weight of a
// subset is kept split as  2^{h_T} P_T^{-1/2} = 2^n * mu,  h_T = q_T log2(e)/2,
// n = floor(h_T), mu = 2^{h_T - n} P_T^{-1/2} in (0, 2).
#ifndef PSX_MATH_H
#define PSX_MATH_H

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#define PSX_KMAX 6            // largest union set the generic evaluator handles (3^6 patterns)
#define PSX_LOG2E 1.4426950408889634074
#define PSX_LN2 0.69314718055994530942

namespace psx {

// Per-SNP accumulator / per-member partial record (5 PostCal quantities).
//   group P (shift mP): post0, post1, shared   — PIP-type, judged relative to total
//   group S (shift mS): sll  (sharedLL)
//   group N (shift mN): nsll (notSharedLL)
struct Acc5 {
    int32_t mP, mS, mN, pad;
    double post0, post1, shared, sll, nsll;
};

// Per-set (or per-unit) scalar record: total, noCausal[0], noCausal[1], each with
// its own shift (noCausal[s] can sit thousands of nats below the total).
struct SetRec {
    int32_t m, m0, m1, pad;
    double tot, nc0, nc1;
    double score;  // min over patterns of L' (nats, K excluded) == SSS max|L| pattern
    double npat;   // configurations folded in (exact integer in a double)
};

// Last slot of a partial image: which shard of which plan the image holds.  A
// merge folds images in rank order and refuses a set whose tags disagree (a
// rank that cut another plan — other PSX_K3_* knobs, another build — would
// leave configurations uncounted or counted twice).
constexpr int32_t kPlanMagic = 0x54585350;  // "PSXT"
struct PlanTag {
    int32_t magic, world, rank, U;
    uint64_t hash;  // U, ldg, c, presence bits, world and the plan knobs (rank excluded)
    uint64_t pad[4];
};

static_assert(sizeof(Acc5) == 56 && sizeof(SetRec) == 56 && sizeof(PlanTag) == 56, "partial-image slot layout");

__host__ __device__ inline int imax(int a, int b) { return a > b ? a : b; }

__host__ __device__ inline SetRec set_zero() {
    SetRec r;
    r.m = r.m0 = r.m1 = r.pad = 0;
    r.tot = r.nc0 = r.nc1 = 0.0;
    r.score = 1e300;
    r.npat = 0.0;
    return r;
}

// fold (m2, s2[0..n)) into (m, s[0..n)) — shared shift within the group
__host__ __device__ inline void fold_group(int32_t& m, double* s, int n, int32_t m2, const double* s2) {
    bool nz2 = false, nz = false;
    for (int i = 0; i < n; i++) { nz2 |= (s2[i] != 0.0); nz |= (s[i] != 0.0); }
    if (!nz2) return;
    if (!nz) {
        m = m2;
        for (int i = 0; i < n; i++) s[i] = s2[i];
        return;
    }
    int M = imax(m, m2);
    for (int i = 0; i < n; i++) s[i] = ldexp(s[i], m - M) + ldexp(s2[i], m2 - M);
    m = M;
}

__host__ __device__ inline void fold1(int32_t& m, double& s, int32_t m2, double s2) {
    if (s2 == 0.0) return;
    if (s == 0.0) { m = m2; s = s2; return; }
    int M = imax(m, m2);
    s = ldexp(s, m - M) + ldexp(s2, m2 - M);
    m = M;
}

__host__ __device__ inline void fold_acc(Acc5& a, const Acc5& b) {
    double sa[3] = {a.post0, a.post1, a.shared};
    const double sb[3] = {b.post0, b.post1, b.shared};
    fold_group(a.mP, sa, 3, b.mP, sb);
    a.post0 = sa[0]; a.post1 = sa[1]; a.shared = sa[2];
    fold1(a.mS, a.sll, b.mS, b.sll);
    fold1(a.mN, a.nsll, b.mN, b.nsll);
}

__host__ __device__ inline void fold_set(SetRec& a, const SetRec& b) {
    fold1(a.m, a.tot, b.m, b.tot);
    fold1(a.m0, a.nc0, b.m0, b.nc0);
    fold1(a.m1, a.nc1, b.m1, b.nc1);
    a.score = fmin(a.score, b.score);
    a.npat += b.npat;
}

// 2^{h} * rP as (n, mu): n = floor(h), mu = 2^{h-n} * rP
__host__ __device__ inline void split_exp(double h, double rP, int& n, double& mu) {
    double fl = floor(h);
    n = (int)fl;
    mu = exp2(h - fl) * rP;
}

// LDL^T of A_T for the members idx[0..t) of one study (union-indexed arrays):
//   A_ij = G[idx_i][idx_j] (i != j), A_ii = Ad[idx_i]; returns q = y^T A^-1 y and
//   P = prod d*D_i.  Used by the generic evaluator (any t <= PSX_KMAX).
__host__ __device__ inline void ldlt_terms(const double* G, int ldg, const double* Ad, const double* y,
                                           double dval, const int* idx, int t, double& q, double& P) {
    double L[PSX_KMAX][PSX_KMAX];
    double D[PSX_KMAX], Rd[PSX_KMAX], w[PSX_KMAX];
    q = 0.0;
    P = 1.0;
    for (int i = 0; i < t; i++) {
        const double* Gi = G + (size_t)idx[i] * ldg;
        for (int j = 0; j < i; j++) {
            double acc = Gi[idx[j]];
            for (int k = 0; k < j; k++) acc -= L[i][k] * L[j][k] * D[k];
            L[i][j] = acc * Rd[j];  // one division per pivot (below)
        }
        double di = Ad[idx[i]];
        double wi = y[idx[i]];
        for (int k = 0; k < i; k++) {
            di -= L[i][k] * L[i][k] * D[k];
            wi -= L[i][k] * w[k];
        }
        D[i] = di;
        Rd[i] = 1.0 / di;
        w[i] = wi;
        q += wi * wi * Rd[i];
        P *= dval * di;
    }
}

}  // namespace psx
#endif
