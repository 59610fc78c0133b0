// psx_sweep3.hip — the k = 3 exhaustive level (postcal.cpp:716-1092 for
// |union set| = 3), the dominant kernel of the sweep.
//
// A unit is (a-chunk, b-block K, c-block C), K <= C, in the padded index space:
// lane t owns c = 64C + t and at step j takes b-slot (t + j) & 63 of block K,
// so the 64 b-slot accumulators rotate through LDS without atomics.  Triples
// are routed by block pattern (plan_units3c): off-diagonal tiles (K < C) only
// see a before block K, so every lane is active every step; triples with two
// members in one block go to that block's diagonal tile (K == C), walked
// folded (steps 1..32, each pair of the block once) with a before, after or
// inside the block.  This kernel is VALU-issue bound (every wave64 VALU op
// costs ~4 cycles, FP64 or integer alike; HBM traffic is negligible), so it is
// built to minimise the VALU instruction count per union set:
//
//  * per step only the {a, b, c} extension is computed: the a-independent
//    {b, c} weights come precomputed (k_build_bc3, once per locus) and are
//    streamed with the tile row of Sigma~, both one step ahead of use;
//  * the (a, c) terms (lane-owned) and (a, b) terms (lane-parallel, into LDS)
//    are hoisted per a; everything else indexed by b is staged in LDS once per
//    unit and read with immediate offsets;
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
//    wave-uniform branch) when G exceeds it by > 960 bits.  Contributions more
//    than ~1022 bits below an accumulator's own running maximum vanish,
//    exactly as in the branch-free fold they replace.
//
// Absent members (mixed loci) are masked by zeroing their pivot factor, which
// zeroes every subset weight containing them (checkOR of postcal.cpp:907-955).
// notSharedLL groups more than ~900 bits below a set's scale raise *flag; the
// host then reruns the level with k_sweep<3, true> (exact group scaling).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <string>
#include <type_traits>

#include "psx_sweep.h"
#include "psx_sweep_dev.h"
#include "psx_sweep_unit.h"
#include "psx_wave.h"

// device-library wave reductions (DPP, result in every lane)
extern "C" __device__ __attribute__((const)) int __ockl_wfred_max_i32(int);
extern "C" __device__ __attribute__((const)) double __ockl_wfred_add_f64(double);
extern "C" __device__ __attribute__((const)) double __ockl_wfred_min_f64(double);

namespace psx {

constexpr double kMagic = 6755399441055744.0;  // 1.5 * 2^52: round-to-nearest-integer add
constexpr double kTinyNs = 0x1p-900;            // notSharedLL group floor of the fast path
// e^{f ln2 / 256} = sum_k q_k f^k, |f| <= 1/2 (degree 4, error < 4e-17)
constexpr double kQ1 = PSX_LN2 / 256.0;
constexpr double kQ2 = kQ1 * kQ1 / 2.0;
constexpr double kQ3 = kQ2 * kQ1 / 3.0;
constexpr double kQ4 = kQ3 * kQ1 / 4.0;
// the walk's cubic: Chebyshev interpolant of 2^{f/256} on |f| <= 1/2 (nodes
// cos((2i+1) pi / 8) / 2), max relative error 1.8e-14 (the Taylor quartic above:
// 3.8e-17); it saves the walk two FP64 operations per union set (-2.2 %, r03)
constexpr double kC0 = 0.9999999999999825;
constexpr double kC1 = 0.002707606174062277;
constexpr double kC2 = 3.665566156758823e-06;
constexpr double kC3 = 3.3083029835781016e-09;

// an opaque point in the instruction stream for a loaded value: no use of it can
// be scheduled before this statement (the wait for the load lands here)
__device__ __forceinline__ void pin_vgpr(double2& v) {
    double x = v.x, y = v.y;
    asm volatile("" : "+v"(x), "+v"(y));
    v = make_double2(x, y);
}
__device__ __forceinline__ void pin_vgpr(int2& v) {
    int x = v.x, y = v.y;
    asm volatile("" : "+v"(x), "+v"(y));
    v = make_int2(x, y);
}

// A unit's set record across the wave by DPP reductions: each (shift, sum) pair
// is taken at the wave's largest shift among lanes holding a value (empty lanes
// carry EMPTY), then summed; a term more than ~1074 bits below that shift
// vanishes, as in the pairwise fold it replaces.  The result is in every lane.
__device__ __forceinline__ void wave_pair_dpp(int& m, double& s) {
    const int M = __ockl_wfred_max_i32(s != 0.0 ? m : EMPTY);
    const double S = __ockl_wfred_add_f64(s != 0.0 ? ldexp(s, m - M) : 0.0);
    m = S != 0.0 ? M : EMPTY;
    s = S;
}
__device__ __forceinline__ void wave_fold_set_dpp(SetRec& r) {
    wave_pair_dpp(r.m, r.tot);
    wave_pair_dpp(r.m0, r.nc0);
    wave_pair_dpp(r.m1, r.nc1);
    r.score = __ockl_wfred_min_f64(r.score);
    r.npat = __ockl_wfred_add_f64(r.npat);
}


// Order LDS accesses across the lanes of a ONE-wave workgroup: a wave's LDS
// instructions execute in issue order, so program order suffices.  __syncthreads
// would add s_barrier and, through its fence, a vmcnt(0) drain that waits for
// every global load in flight (the prefetched tile rows and next-a Sigma~
// entries): ~1 us per a prologue (tools/unit_trace.py, r04i).
__device__ __forceinline__ void wave_lds_order() { asm volatile("" ::: "memory"); }

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

// the table-free first half of split3: N = round(256 h), q = 2^{f/256} * rP
// (the caller completes mu = tab[N & 255] * q, n = N >> 8)
__device__ __forceinline__ void split3a(double h, double rP, int& N, double& q) {
    const double xr = fma(h, 256.0, kMagic);
    N = __double2loint(xr);
    const double kf = xr - kMagic;
    const double f = fma(h, 256.0, -kf);
    double p = fma(kQ4, f, kQ3);
    p = fma(p, f, kQ2);
    p = fma(p, f, kQ1);
    p = fma(p, f, 1.0);
    q = p * rP;
}

// split3a with the rounding offset by an integer R (cmag = kMagic - 256 R):
// N = round(256 (h - R)), so the caller's exponent is N >> 8 = n - R directly;
// the fraction's exponential by the walk's cubic (kC*).  k256 = 256 and kc3 = kC3
// in SGPRs, kc2 = kC2 in a VGPR: opaque values the caller holds for the walk, so
// the compiler emits one VOP3 v_fma_f64 instead of copying the addend (a
// loop-carried VGPR, or a constant it cannot put on the constant bus beside
// another) for the two-address v_fmac_f64 with a literal: a v_mov_b64 per use
__device__ __forceinline__ void split3r(double h, double rP, double cmag, double k256, double kc3, double kc2,
                                        int& N, double& q) {
    const double xr = fma(h, k256, cmag);
    N = __double2loint(xr);
    const double kf = xr - cmag;
    const double f = fma(h, k256, -kf);
    double p = fma(f, kc3, kc2);
    p = fma(p, f, kC1);
    p = fma(p, f, kC0);
    q = p * rP;
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

// fast-variant accumulator (shift m; W0, W1, W2 = prior-weighted sums over
// the member's assignments study 0 only / study 1 only / both, W2 without the
// member's own rho) -> merge record (Acc5 convention, as lacc_rec)
__device__ __forceinline__ Acc5 wrec(int m, double W0, double W1, double W2, double sl, double ns, double rho, int Ck,
                                     double pit0) {
    Acc5 r;
    const double sh = rho * W2;
    r.post0 = (W0 + sh) * pit0;
    r.post1 = (W1 + sh) * pit0;
    r.shared = sh * pit0;
    r.sll = sl;
    r.nsll = ns;
    r.mP = (r.post0 + r.post1 != 0.0) ? m + Ck : EMPTY;
    r.mS = (sl != 0.0) ? m : EMPTY;
    r.mN = (ns != 0.0) ? m : EMPTY;
    r.pad = 0;
    return r;
}

// b-block terms of SNP v (v space) in study s: 1/A_bb, y_b / 2, the {b}
// quadratic form and its pivot factor (x the c step's rsd / 2)
struct BTerms {
    double I, Yh, H, R, chi;
};
template <bool ALLPRES>
__device__ __forceinline__ BTerms b_terms(const Sweep3Args& A, int s, int v) {
    const int u = v - A.pad;
    const bool ok = v >= A.pad;
    const unsigned p = ok ? A.pres[u] : 0u;
    BTerms b;
    b.chi = (ok && (ALLPRES || ((p >> s) & 1u))) ? 1.0 : 0.0;
    const double Abb = ok ? A.Ad[s][u] : 1.0;
    const double yb = ok ? A.ys[s][u] : 0.0;
    const double r = rsqrt_nr(Abb);
    b.I = r * r;
    b.Yh = 0.5 * yb;
    b.H = yb * yb * r * r;
    b.R = r * A.rsd[s] * b.chi * (0.5 * A.rsd[s]);  // {b} factor x (c's rsd / 2)
    return b;
}

// the {b, c} subset weight 2^n2 * mu2 (LDL^T of {b, c}, c extending b)
__device__ __forceinline__ void bc_weight(double Gbc, const BTerms& b, double Acc, double ych, double chic,
                                          const double* tab, int& n2, double& mu2) {
    const double l2 = Gbc * b.I;
    const double D2 = fma(-l2, Gbc, Acc);
    const double w2 = fma(-l2, b.Yh, ych);
    const double r2 = rsq2x(D2);
    const double t2 = w2 * r2;
    const double h2 = fma(t2, t2, b.H);
    split3(h2, b.R * r2 * chic, tab, n2, mu2);
}

// mu01[tile][j][t] (both studies), bcn[tile][j][t]: the {b, c} weights of the k = 3 walk,
// b = 64K + ((t + j) & 63), c = 64C + t (the folded diagonal walk uses the same
// (slot, lane) pairs).  One block per (tile, step), lane t.
template <bool ALLPRES>
__global__ void k_build_bc3(Sweep3Args A, double2* __restrict__ mu01, int2* __restrict__ nn) {
    const int tile = blockIdx.x, j = blockIdx.y, t = threadIdx.x;
    int C = 0;
    while ((C + 1) * (C + 2) / 2 <= tile) C++;
    const int K = tile - C * (C + 1) / 2;
    const int vb = 64 * K + ((t + j) & 63), vc = 64 * C + t, uc = vc - A.pad;
    const bool okc = vc >= A.pad;
    const unsigned pcm = okc ? A.pres[uc] : 0u;
    const size_t o = (size_t)tile * 4096 + j * 64 + t;
    int n[2];
    double mu[2];
#pragma unroll
    for (int s = 0; s < 2; s++) {
        const BTerms b = b_terms<ALLPRES>(A, s, vb);
        const double chic = (okc && (ALLPRES || ((pcm >> s) & 1u))) ? 1.0 : 0.0;
        const double Acc = okc ? A.Ad[s][uc] : 1.0;
        const double ych = 0.5 * (okc ? A.ys[s][uc] : 0.0);
        bc_weight(A.skewT[s][o], b, Acc, ych, chic, A.tab, n[s], mu[s]);
    }
    mu01[o] = make_double2(mu[0], mu[1]);
    nn[o] = make_int2(n[0], n[1]);
}

// Unit = (a-chunk [a0, a1), b-block K, c-chunk C), K <= C, in the padded index
// space v = u + pad (the partial 64-block is the lowest one, where the sweep
// has the least work).  Lane t owns c = 64C + t for the whole unit; at step j
// it takes b = 64K + ((t + j) & 63), so the 64 b-slot accumulators rotate
// through LDS without conflicts.  Per a, the {a,c} pivot (lane-owned) and the
// {a,b} pivots of the 64 b's (lane-parallel, into LDS) are computed once; per
// step only {b,c} and {a,b,c} are new.
//
// Pivot factors: P_T^{-1/2} = prod_i r_i rsd over the LDL^T pivots of T.  The
// step computes r2x = 2 / sqrt(D), so the staged factors carry rsd / 2.
// LDS: what other lanes read — the exp2 table, the per-a (a, b) terms of the
// rotating b slot, the slot accumulators; what a lane reads only for itself (its b
// slot's and c's constants, record positions, the next a's Sigma~ row entries)
// is held in registers.  (Three waves per SIMD, <= 13,312 bytes per block and 168
// VGPRs, were measured 17 % slower: the walk state left no registers for the
// per-a state, which the compiler parked in scratch behind dependent waits,
// profiles/archive/r03d_k3_three_waves_rejected.txt.)
//
// LDS of a k = 3 unit, ROBUST variant: (a, b) terms (per a), indexed [study][b
// slot], the exp2 table and the rotating b-slot accumulators
struct Sweep3Smem {
    double tab[256];
    double abG[2][64], abI[2][64], abW[2][64], abH[2][64], abR[2][64], abMu[2][64], abMuB[2][64];
    int abN[2][64];
    float bW[64];
    double sP0[64], sP1[64], sSh[64], sSl[64], sNs[64];
    int sM[64];
    int aPos[kMaxChunkA3];  // a record positions
    // lane constants the a prologues read, parked across the walks (registers
    // would spill): this lane's b slot ({b} quadratic form, pivot factor) and c
    double lbH[2][64], lbR[2][64], lAcc[2][64], lyc[2][64], lmuC[2][64];
    int lnC[2][64];
};
// LDS of the fast k = 3 variant: the per-b terms of both studies side by side
// (one 16-byte read per term and step; lane t reads slot (t + j) & 63, so the
// reads are conflict-free), and the b-slot accumulators (one shift sM for every
// slot: all slots move up to the wave's largest a shift together)
struct Sweep3FastSmem {
    double tab[256];
    double2 aAd[kMaxChunkA3], aY[kMaxChunkA3];  // the unit's a: A_aa, y_a (both studies), presence
    unsigned aP[kMaxChunkA3];
    int aPos[kMaxChunkA3];  // a record positions
    double2 abG[64], abI[64], abIW[64], abH[64], abR[64];
    double2 abMu[64], abMuB[64];  // the slot's {a, b} / {b} weights relative to 2^Ru_s (wave reference)
    float bW[64];  // membership weight of the slot's b (0, 1 or 3)
    double sW0[64], sW1[64], sW2[64], sSl[64], sNs[64];
    double sW2w[64], sSlw[64];  // the current a's walk part of sW2 / sSl, at 2^(Ru_0 + Ru_1)
    union {
        struct {  // off-diagonal units (closed-form sums, sweep3_unit_fast): this lane's c terms
            double2 bcsm[64];   // the {b, c} weights of this lane's c summed over the block, both studies
            int2 bcsn[64];
            double2 bccm[64];   // the {b, c} weights of slot b summed over the tile's c, both studies
            int2 bccn[64];
        };
        struct {  // the other units: lane constants the a prologues read, parked across the walks
            double2 lmuB[64];   // this lane's slot {b} weight, both studies (2^lnB * lmuB)
            int2 lnB[64];
            double2 lmuC[64];   // this lane's c {c} weight, both studies (2^lnC * lmuC)
            int2 lnC[64];
            double2 lAbb[64];   // this lane's b slot / c: A_bb, y_b, A_cc, y_c, both studies
            double2 lyb[64];
            double2 lAcc[64];
            double2 lyc[64];
        };
    };
    double pbS[2];              // sum of the block's {b} weights, both studies: 2^pbM * pbS
    double kc2;                 // the walk's kC2 (non-SEP units read it per a)
    int pbM[2];
};
union SweepSmem {  // a block runs either a k = 3 unit or a level-2 unit
    Sweep3Smem s3;
    Sweep3FastSmem f3;
    SweepUnitSmem u2;
};
// PSX_K3_WAVES one-wave blocks per SIMD: 160 KiB / (4 x waves) per block, in 512-byte granules
static_assert(sizeof(SweepSmem) <= (163840 / (4 * PSX_K3_WAVES)) / 512 * 512, "k_sweep3 LDS above its occupancy budget");

// One k = 3 unit, ROBUST variant: every step's subset weights are taken
// relative to the set's own top exponent (n_abc per study) and the lane / slot
// accumulators shift lazily, so any dynamic range is handled.  Run for the
// units the fast variant (below) flags.
template <bool ALLPRES>
__device__ __forceinline__ void sweep3_unit_robust(const Sweep3Args& A, int unit, const int4* __restrict__ units,
                                                Acc5* __restrict__ rec, SetRec* __restrict__ srec, int rec_stride,
                                                int* __restrict__ flag, const int* __restrict__ pos, SweepSmem& sm) {
    double (&tab)[256] = sm.s3.tab;
    double (&abG)[2][64] = sm.s3.abG;
    double (&abI)[2][64] = sm.s3.abI;
    double (&abW)[2][64] = sm.s3.abW;
    double (&abH)[2][64] = sm.s3.abH;
    double (&abR)[2][64] = sm.s3.abR;
    double (&abMu)[2][64] = sm.s3.abMu;
    double (&abMuB)[2][64] = sm.s3.abMuB;
    int (&abN)[2][64] = sm.s3.abN;
    float (&bW)[64] = sm.s3.bW;
    double (&sP0)[64] = sm.s3.sP0;
    double (&sP1)[64] = sm.s3.sP1;
    double (&sSh)[64] = sm.s3.sSh;
    double (&sSl)[64] = sm.s3.sSl;
    double (&sNs)[64] = sm.s3.sNs;
    int (&sM)[64] = sm.s3.sM;

    const int t = threadIdx.x;
    const int4 un = units[unit];
    const int a0 = un.x, a1 = un.y, K = un.z & 0xffff, C = un.w & 0xffff;
    // b-walk steps of this (half) unit.  A diagonal tile (K == C) is walked
    // folded: at step j lane t pairs with slot (t + j) & 63 whichever of the two
    // is larger, so steps 1..31 (+ step 32 on lanes < 32) visit every pair of
    // the block once — half the steps of the triangular walk, no idle lanes.
    // The set {a, slot, t} is factored in the order (a, slot, t) either way.
    const bool diag = K == C;
    const int j0 = diag ? 1 + (un.z >> 17) : un.z >> 16;
    const int j1 = diag ? 1 + (un.w >> 17) : un.w >> 16;
    const int pad = A.pad, ldg = A.ldg;
    const int tile = C * (C + 1) / 2 + K;
    const double rho = A.rho;

    // ---- unit prologue -------------------------------------------------------------
    for (int i = t; i < 256; i += 64) tab[i] = A.tab[i];
    // this lane's b of the b-block (v-space; u = v - pad)
    const int vbl = 64 * K + t, ubl = vbl - pad;
    const bool okb = vbl >= pad;
    const unsigned pbl = okb ? A.pres[ubl] : 0u;
#pragma unroll
    for (int s = 0; s < 2; s++) {  // this lane's b slot: {b} quadratic form and pivot factor
        const BTerms b = b_terms<ALLPRES>(A, s, vbl);
        sm.s3.lbH[s][t] = b.H;
        sm.s3.lbR[s][t] = b.R;
    }
    bW[t] = (float)memb_weight(pbl);
    sM[t] = EMPTY;
    sP0[t] = sP1[t] = sSh[t] = sSl[t] = sNs[t] = 0.0;

    // c terms: lane-owned for the whole unit
    const int vc = 64 * C + t, uc = vc - pad;
    const bool okc = vc >= pad;
    const unsigned pcm = okc ? A.pres[uc] : 0u;
#pragma unroll
    for (int s = 0; s < 2; s++) {
        const double chic = (okc && (ALLPRES || ((pcm >> s) & 1u))) ? 1.0 : 0.0;
        sm.s3.lAcc[s][t] = okc ? A.Ad[s][uc] : 1.0;
        sm.s3.lyc[s][t] = okc ? A.ys[s][uc] : 0.0;
        sm.s3.lmuC[s][t] = okc ? A.muS[s][uc] * chic : 0.0;
        sm.s3.lnC[s][t] = okc ? A.nS[s][uc] : 0;
    }
    const double wc = memb_weight(pcm);

    LAcc accC;
    lacc_zero(accC);
    double totC = 0.0;
    int m0 = EMPTY, m1 = EMPTY;
    double nc0 = 0.0, nc1 = 0.0, npat = 0.0;
    // the tile row: both studies' skewed Sigma~ entries and {b, c} weights as
    // 16-byte pairs (three loads per step)
    const double2* g01 = A.g01 + (size_t)tile * 4096 + t;
    const double2* m01 = A.mu01 + (size_t)tile * 4096 + t;
    const int2* bnn = A.bcn + (size_t)tile * 4096 + t;

    // record positions (CSR map) of this unit's c / b-slot / a records, and the
    // first a's Sigma~ row entries, loaded with the unit prologue
    const size_t rbase = (size_t)unit * rec_stride;
    const int posC = pos[rbase + t], posB = pos[rbase + 64 + t];
    if (t < a1 - a0) sm.s3.aPos[t] = pos[rbase + 128 + t];

    for (int ai = 0; ai < a1 - a0; ai++) {
        const int va = a0 + ai, ua = va - pad;  // a0 >= pad: a is always a real SNP
        const unsigned pa = A.pres[ua];
        double l1[2], D1[2], w1h[2], Ep[2][4];  // Ep: {}, {a}, {c}, {a,c} relative to 2^{n_ac}
        int R[2];
        // step j0 of the tile row: issued before the a prologue, whose work hides it
        double2 gnx = g01[j0 * 64], mnx = m01[j0 * 64];
        int2 nnx = bnn[j0 * 64];
        __syncthreads();  // previous a's (a, b) terms fully consumed
#pragma unroll
        for (int s = 0; s < 2; s++) {
            const double chia = (ALLPRES || ((pa >> s) & 1u)) ? 1.0 : 0.0;
            const double ya = A.ys[s][ua];
            const double ra = rsqrt_nr(A.Ad[s][ua]);
            const double iAaa = ra * ra;
            const double ha = ya * ya * iAaa;
            const double rPa = ra * A.rsd[s] * chia;
            int nA;
            double muA;
            split3(ha, rPa, tab, nA, muA);
            {
                // {a, b} and {b} for this lane's b, into LDS
                const double Gab = okb ? A.G[s][(size_t)ua * ldg + ubl] : 0.0;
                const double Abb = okb ? A.Ad[s][ubl] : 1.0;
                const double yb = okb ? A.ys[s][ubl] : 0.0;
                const double l = Gab * iAaa;
                const double Dab = fma(-l, Gab, Abb);
                const double rab = rsqrt_nr(Dab);
                const double wab = fma(-l, ya, yb);
                const double hab = fma(wab * wab, rab * rab, ha);
                // this lane's b absent from study s (or padding): the {a, b} weight is 0
                const bool chib = okb && (ALLPRES || ((pbl >> s) & 1u));
                const double rPab = chib ? rPa * rab * A.rsd[s] : 0.0;
                int nAB, nB;
                double muAB, muB;
                split3(hab, rPab, tab, nAB, muAB);
                split3(sm.s3.lbH[s][t], sm.s3.lbR[s][t] * (2.0 / A.rsd[s]), tab, nB, muB);
                abG[s][t] = Gab;
                abI[s][t] = rab * rab;
                abW[s][t] = 0.5 * wab;
                abH[s][t] = hab;
                abR[s][t] = rPab * (0.5 * A.rsd[s]);
                abMu[s][t] = muAB;
                abMuB[s][t] = ldexp(muB, nB - nAB);  // n_ab >= n_b: nested quadratic forms
                abN[s][t] = nAB;
            }
            // {a, c}: lane-owned
            const double Gac = okc ? A.G[s][(size_t)ua * ldg + uc] : 0.0;
            const double chic = (okc && (ALLPRES || ((pcm >> s) & 1u))) ? 1.0 : 0.0;
            l1[s] = Gac * iAaa;
            D1[s] = fma(-l1[s], Gac, sm.s3.lAcc[s][t]);
            const double w1 = fma(-l1[s], ya, sm.s3.lyc[s][t]);
            w1h[s] = 0.5 * w1;
            const double r1 = rsqrt_nr(D1[s]);
            const double h1 = fma(w1 * w1, r1 * r1, ha);
            const double rP1 = rPa * r1 * A.rsd[s] * chic;
            int n1;
            double mu1;
            split3(h1, rP1, tab, n1, mu1);
            // {}, {a}, {c} never exceed {a,c} (nested forms), so these cannot overflow
            R[s] = n1;
            Ep[s][0] = ldexp(1.0, -n1);
            Ep[s][1] = ldexp(muA, nA - n1);
            Ep[s][2] = ldexp(sm.s3.lmuC[s][t], sm.s3.lnC[s][t] - n1);
            Ep[s][3] = mu1;
        }
        const double wac = wc * memb_weight(pa);
        LAcc accA;
        lacc_zero(accA);
        __syncthreads();  // (a, b) terms visible

        // the next step's skewed Sigma~ entries and {b, c} weights are loaded one
        // step ahead (L2 / MALL latency is longer than the VALU work between)
        for (int j = j0; j < j1; j++) {
            const double gcur0 = gnx.x, gcur1 = gnx.y, mcur0 = mnx.x, mcur1 = mnx.y;
            const int2 ncur = nnx;
            if (j + 1 < j1) {
                gnx = g01[(j + 1) * 64];
                mnx = m01[(j + 1) * 64];
                nnx = bnn[(j + 1) * 64];
            }
            const int bs = (t + j) & 63;
            const int vb = 64 * K + bs;
            // diagonal tile: the pair {slot, t} of the block with a below both,
            // or any real pair when a lies after the block
            const bool act = diag ? (((vb > va && vc > va) || (va >= 64 * K + 64 && vb >= pad && vc >= pad)) &&
                                     (j < 32 || t < 32))
                                  : (okc && vb > va && vb < vc);
            if (act) {
                double E[2][8];
                int nb[2];
#pragma unroll
                for (int s = 0; s < 2; s++) {
                    const double Gbc = s ? gcur1 : gcur0;
                    // {b, c}: precomputed (k_build_bc3, a-independent)
                    const int n2 = s ? ncur.y : ncur.x;
                    const double mu2 = s ? mcur1 : mcur0;
                    // {a, b, c}: extend the (a, b) factor by the c row (x = the
                    // unnormalised L entry; D_ab I_ab = 1 folds the pivot away)
                    const double x = fma(-l1[s], abG[s][bs], Gbc);
                    const double lcb = x * abI[s][bs];
                    const double D3 = fma(-x, lcb, D1[s]);
                    const double w3 = fma(-lcb, abW[s][bs], w1h[s]);
                    const double r3 = rsq2x(D3);
                    const double t3 = w3 * r3;
                    const double h3 = fma(t3, t3, abH[s][bs]);
                    double rP3 = abR[s][bs] * r3;
                    if (!ALLPRES && !((pcm >> s) & 1u)) rP3 = 0.0;  // c absent from study s
                    int n3;
                    double mu3;
                    split3(h3, rP3, tab, n3, mu3);
                    nb[s] = n3;
                    // subset weights relative to 2^n_abc (bit 0 = a, bit 1 = b, bit 2 = c)
                    const int dR = R[s] - n3, dAB = abN[s][bs] - n3;
                    E[s][0] = ldexp(Ep[s][0], dR);
                    E[s][1] = ldexp(Ep[s][1], dR);
                    E[s][2] = ldexp(abMuB[s][bs], dAB);
                    E[s][3] = ldexp(abMu[s][bs], dAB);
                    E[s][4] = ldexp(Ep[s][2], dR);
                    E[s][5] = ldexp(Ep[s][3], dR);
                    E[s][6] = ldexp(mu2, n2 - n3);
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
                // ---- folds: a, c (registers), b (LDS slot, rotating owner), noCausal ----
                LAcc sl;
                sl.m = sM[bs];
                sl.p0 = sP0[bs];
                sl.p1 = sP1[bs];
                sl.sh = sSh[bs];
                sl.sl = sSl[bs];
                sl.ns = sNs[bs];
                int dA = Gll - accA.m, dC = Gll - accC.m, dS = Gll - sl.m;
                // noCausal[s]: the assignment with C_s empty (every member in the other study)
                double x0 = ldexp(E[1][7], nb[1] - m0), x1 = ldexp(E[0][7], nb[0] - m1);
                const bool up = (nz & (max(dA, max(dC, dS)) > 960)) | (x0 > 0x1p960) | (x1 > 0x1p960);
                if (__builtin_amdgcn_ballot_w64(up)) {  // wave-uniform, rare: move shifts up
                    if (nz && dA > 960) { lacc_shift(accA, Gll); dA = 0; }
                    if (nz && dC > 960) { lacc_shift(accC, Gll); totC = ldexp(totC, -dC); dC = 0; }
                    if (nz && dS > 960) { lacc_shift(sl, Gll); dS = 0; }
                    if (x0 > 0x1p960) { nc0 = ldexp(nc0, m0 - nb[1]); m0 = nb[1]; x0 = E[1][7]; }
                    if (x1 > 0x1p960) { nc1 = ldexp(nc1, m1 - nb[0]); m1 = nb[0]; x1 = E[0][7]; }
                }
                nc0 += x0;
                nc1 += x1;
                lacc_add(accA, ldexp(1.0, min(dA, 1000)), SwA[0] + SwA[2], SwA[1] + SwA[2], SwA[2], sllA, nsA);
                lacc_add(sl, ldexp(1.0, min(dS, 1000)), SwB[0] + SwB[2], SwB[1] + SwB[2], SwB[2], sllB, nsB);
                const double fC = ldexp(1.0, min(dC, 1000));
                lacc_add(accC, fC, SwC[0] + SwC[2], SwC[1] + SwC[2], SwC[2], sllC, nsC);
                totC = fma(tot, fC, totC);
                sM[bs] = sl.m;
                sP0[bs] = sl.p0;
                sP1[bs] = sl.p1;
                sSh[bs] = sl.sh;
                sSl[bs] = sl.sl;
                sNs[bs] = sl.ns;
                npat += ALLPRES ? 27.0 : wac * bW[bs];
            }
            // b-slot ownership rotates across lanes every step: the workgroup is one
            // wave and LDS executes a wave's instructions in issue order, so only the
            // compiler must keep program order (no lgkmcnt drain per step)
            __builtin_amdgcn_wave_barrier();
        }
        Acc5 ra = lacc_rec(accA, A.Ck, A.pit0);
        wave_fold_acc(ra);
        const int qa = sm.s3.aPos[ai];
        if (t == 0 && qa >= 0) store_rec(rec + qa, ra);
    }
    __syncthreads();
    {
        LAcc sl;
        sl.m = sM[t];
        sl.p0 = sP0[t];
        sl.p1 = sP1[t];
        sl.sh = sSh[t];
        sl.sl = sSl[t];
        sl.ns = sNs[t];
        Acc5 rc = lacc_rec(accC, A.Ck, A.pit0);
        const Acc5 rb = lacc_rec(sl, A.Ck, A.pit0);
        if (diag) fold_acc(rc, rb);  // one SNP: c = b slot t (the plan keys one record)
        if (posC >= 0) store_rec(rec + posC, rc);
        if (!diag && posB >= 0) store_rec(rec + posB, rb);
    }
    SetRec sr;
    sr.tot = totC * A.pit0;
    sr.m = (sr.tot != 0.0) ? accC.m + A.Ck : EMPTY;
    sr.nc0 = nc0 * A.pit0;
    sr.m0 = (sr.nc0 != 0.0) ? m0 + A.Ck : EMPTY;
    sr.nc1 = nc1 * A.pit0;
    sr.m1 = (sr.nc1 != 0.0) ? m1 + A.Ck : EMPTY;
    sr.pad = 0;
    sr.score = 1e300;
    sr.npat = npat;
    wave_fold_set(sr);
    if (t == 0) store_rec(srec + unit, sr);
}

constexpr int kMaxRefGap = 960;  // fast variant: largest n_abc - n_ac (bits, both studies) it accepts
constexpr int kMaxSpread = 240;  // fast variant: largest Ru_s - R_s (bits, per study) within a wave

// One k = 3 unit, FAST variant.  All of a lane's subset weights for one a are
// taken relative to R_s = n_{ac} (the {a, c} exponent of study s, fixed for the
// whole b-walk), so per step only the four weights that involve b are rescaled
// and the accumulators need no per-step shift: the a accumulator sits at G =
// R_0 + R_1, the c accumulator and noCausal move their shift once per a, and
// every b slot is moved once per a to the wave's largest G.  Weights relative
// to 2^R stay below 2^(n_abc - n_ac + 2); a unit in which some set exceeds
// kMaxRefGap bits over both studies (a very strong b given {a, c}) is redone by
// the ROBUST variant in the same block.
//
// The 27 assignments are folded in factored form (E_s[m]: weight of subset m
// of {a, b, c}, bit 0 a, bit 1 b, bit 2 c; P_s = E_s without c, Q_s = with c):
//  * members a, b: for the 9 (x_a, x_b), with c marginalised,
//      Pl = Q0[al] (P1 + Q1)[be] + P0[al] Q1[be],  Pw = Q0[al] (P1 + rho Q1)[be] + P0[al] Q1[be]
//  * member c: bilinear forms Q0' M P1 etc. with M = m (x) m over (a, b),
//      m = [[0, 1], [1, rho]] (prior-weighted) or [[0, 1], [1, 1]] (LL sums)
// (101 VALU operations instead of 27 products and ~90 partial sums).  Each
// member's own rho (x = 2) is applied when its record is written.
template <bool ALLPRES, bool SEP>
__device__ __forceinline__ void sweep3_unit_fast(const Sweep3Args& A, int unit, const int4* __restrict__ units,
                                                 Acc5* __restrict__ rec, SetRec* __restrict__ srec, int rec_stride,
                                                 int* __restrict__ flag, const int* __restrict__ pos, SweepSmem& sm,
                                                 bool& redo) {
    Sweep3FastSmem& F = sm.f3;
    double (&tab)[256] = F.tab;
    float (&bW)[64] = F.bW;
    double (&sW0)[64] = F.sW0;  // b slots: W0, W1, W2 (own rho deferred), sharedLL, notSharedLL
    double (&sW1)[64] = F.sW1;
    double (&sW2)[64] = F.sW2;
    double (&sSl)[64] = F.sSl;
    double (&sNs)[64] = F.sNs;
    double (&sW2w)[64] = F.sW2w;
    double (&sSlw)[64] = F.sSlw;

    const int t = threadIdx.x;
    const unsigned long long t_start = A.trace ? wall_clock64() : 0ull;
    const int4 un = units[unit];
    const int a0 = un.x, a1 = un.y, K = un.z & 0xffff, C = un.w & 0xffff;
    const bool diag = K == C;
    const int j0 = diag ? 1 + (un.z >> 17) : un.z >> 16;
    const int j1 = diag ? 1 + (un.w >> 17) : un.w >> 16;
    const int pad = A.pad, ldg = A.ldg;
    const int tile = C * (C + 1) / 2 + K;
    const double rho = A.rho;

    // ---- unit prologue: the unit's constants are loaded once, into LDS where other
    // lanes read them and into registers where a lane reads only its own ---------------
    for (int i = t; i < 256; i += 64) tab[i] = A.tab[i];
    if (t == 0) F.kc2 = kC2;
    const int vbl = 64 * K + t, ubl = vbl - pad;
    const bool okb = vbl >= pad;
    const int ib = okb ? ubl : 0;  // clamped index: the loads are unconditional
    const unsigned pbl = okb ? A.pres[ib] : 0u;
    double Abb[2], yb[2];
#pragma unroll
    for (int s = 0; s < 2; s++) {
        Abb[s] = okb ? A.Ad[s][ib] : 1.0;
        yb[s] = okb ? A.ys[s][ib] : 0.0;
    }
    if (t < a1 - a0) {  // the unit's a (at most kMaxChunkA3)
        const int u = a0 + t - pad;
        F.aAd[t] = make_double2(A.Ad[0][u], A.Ad[1][u]);
        F.aY[t] = make_double2(A.ys[0][u], A.ys[1][u]);
        F.aP[t] = A.pres[u];
        F.aPos[t] = pos[(size_t)unit * rec_stride + 128 + t];
    }
    bW[t] = (float)memb_weight(pbl);
    int sMt = EMPTY;  // shift of the b slots (wave-uniform: every a moves all slots alike)
    int eZ = 0;       // this a's walk scale of the sW2 / sSl parts: 2^eZ of the slot shift
    sW0[t] = sW1[t] = sW2[t] = sSl[t] = sNs[t] = 0.0;
    sW2w[t] = sSlw[t] = 0.0;

    const int vc = 64 * C + t, uc = vc - pad;
    const bool okc = vc >= pad;
    const int ic = okc ? uc : 0;
    const unsigned pcm = okc ? A.pres[ic] : 0u;
    double Acc[2], yc[2], chic[2], muC[2];  // (chic: recomputed where used after the prologue)
    int nC[2];
#pragma unroll
    for (int s = 0; s < 2; s++) {
        chic[s] = (okc && (ALLPRES || ((pcm >> s) & 1u))) ? 1.0 : 0.0;
        Acc[s] = okc ? A.Ad[s][ic] : 1.0;
        yc[s] = okc ? A.ys[s][ic] : 0.0;
        muC[s] = okc ? A.muS[s][ic] * chic[s] : 0.0;
        nC[s] = okc ? A.nS[s][ic] : 0;
    }
    const double wc = memb_weight(pcm);

    // c accumulator (shift mC), noCausal (shifts m0, m1), redo gap
    int mC = EMPTY, m0 = EMPTY, m1 = EMPTY, dmax = 0;
    bool wide = false;  // some a's lanes spread more than kMaxSpread below the wave: redo
    double cW0 = 0.0, cW1 = 0.0, cW2 = 0.0, cSl = 0.0, cNs = 0.0;
    double nc0 = 0.0, nc1 = 0.0, npat = 0.0;
    const double2* g01 = A.g01 + (size_t)tile * 4096 + t;
    const double2* m01 = A.mu01 + (size_t)tile * 4096 + t;
    const int2* bnn = A.bcn + (size_t)tile * 4096 + t;
    // record positions (CSR map) of this unit's c / b-slot records; this a's
    // Sigma~ row entries (g1ab: this lane's b slot, g1ac: its c)
    const size_t rbase = (size_t)unit * rec_stride;
    int posC = 0, posB = 0;
    if (SEP) {
        posC = pos[rbase + t];
        posB = pos[rbase + 64 + t];
    }
    double g1ab[2], g1ac[2];
#pragma unroll
    for (int s = 0; s < 2; s++) {
        const double* row = A.G[s] + (size_t)(a0 - pad) * ldg;
        const double gb = row[ib], gc = row[ic];
        g1ab[s] = okb ? gb : 0.0;
        g1ac[s] = okc ? gc : 0.0;
    }
    // off-diagonal units' closed-form tile sums, issued with the other unit loads
    double2 l_bcsm = make_double2(0.0, 0.0), l_bccm = make_double2(0.0, 0.0);
    int2 l_bcsn = make_int2(0, 0), l_bccn = make_int2(0, 0);
    if (SEP) {
        l_bcsm = A.bcsm[(size_t)tile * 64 + t];
        l_bcsn = A.bcsn[(size_t)tile * 64 + t];
        l_bccm = A.bccm[(size_t)tile * 64 + t];
        l_bccn = A.bccn[(size_t)tile * 64 + t];
    }
    wave_lds_order();  // exp2 table staged
    // the {b} weight of this lane's slot: unit-constant (the a prologues rescale it)
    int nBb[2];
    double muBb[2];
#pragma unroll
    for (int s = 0; s < 2; s++) {
        const double chib = (okb && (ALLPRES || ((pbl >> s) & 1u))) ? 1.0 : 0.0;
        const double r = rsqrt_nr(Abb[s]);
        split3(yb[s] * yb[s] * r * r, r * A.rsd[s] * chib, tab, nBb[s], muBb[s]);
    }
    // Off-diagonal units walk every b of block K on every lane (a < 64K <= b <
    // 64C <= c, all lanes active, steps 0 .. 63), so the parts of the per-step fold
    // that factor into (b-only or a,b-only) x (a,c-only) terms have closed forms
    // (sep): the walk sums V_s of the {b}, {a, b} and {b, c} weights, and the b
    // slot's one-study dot products over {b} and {a, b} (see below).
    constexpr bool sep = SEP;  // the caller checked !diag && j0 == 0 && j1 == 64
    if (!sep) {
        F.lmuB[t] = make_double2(muBb[0], muBb[1]);
        F.lnB[t] = make_int2(nBb[0], nBb[1]);
        F.lmuC[t] = make_double2(muC[0], muC[1]);
        F.lnC[t] = make_int2(nC[0], nC[1]);
        F.lAbb[t] = make_double2(Abb[0], Abb[1]);
        F.lyb[t] = make_double2(yb[0], yb[1]);
        F.lAcc[t] = make_double2(Acc[0], Acc[1]);
        F.lyc[t] = make_double2(yc[0], yc[1]);
    }
    if (sep) {
        F.bcsm[t] = l_bcsm;
        F.bcsn[t] = l_bcsn;
        F.bccm[t] = l_bccm;
        F.bccn[t] = l_bccn;
        int m2[2] = {nBb[0], nBb[1]};
        double x2[2] = {muBb[0], muBb[1]};
        wave_pair_k(m2, x2);
        if (t == 0) {
#pragma unroll
            for (int s = 0; s < 2; s++) {
                F.pbS[s] = x2[s];
                F.pbM[s] = m2[s];
            }
        }
    }

    // diagnostics (PSX_UNIT_TRACE): phases of the first a (t_ph), and finer stamps
    // inside its prologue / fold (t_fn: loads + barrier, per-study terms, slot
    // shift, closed forms; fold arithmetic)
    unsigned long long t_ph[4] = {0ull, 0ull, 0ull, 0ull}, t_fn[6] = {0ull, 0ull, 0ull, 0ull, 0ull, 0ull};
    unsigned long long t_la[2] = {0ull, 0ull};
    if (A.trace) t_ph[0] = wall_clock64();
    // The a record (the a's five sums over the wave) is reduced with the NEXT a's
    // prologue batch, or with the unit's set record after the last a: one round
    // of batched wave reductions per a instead of two.  rG = EMPTY: none pending.
    double rW[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    int rG = EMPTY, rq = -1;
    // global loads of each a, all consumed late (no wait in the prologue): the
    // walk's first tile row, and the next a's Sigma~ row entries; the first a's
    // are issued here, in flight with the unit prologue's, in off-diagonal units
    // (their wait at the loop entry was ~1 us of the first a's prologue, r04p;
    // the other units' registers would spill)
    double2 gnx = make_double2(0.0, 0.0), mnx = make_double2(0.0, 0.0);
    int2 nnx = make_int2(0, 0);
    double nGab[2] = {0.0, 0.0}, nGac[2] = {0.0, 0.0};
    if (SEP) {
        gnx = g01[j0 * 64];
        mnx = m01[j0 * 64];
        nnx = bnn[j0 * 64];
#pragma unroll
        for (int s = 0; s < 2; s++) {
            const double* row = A.G[s] + (size_t)(a1 - a0 > 1 ? a0 + 1 - pad : a0 - pad) * ldg;
            nGab[s] = row[ib];
            nGac[s] = row[ic];
        }
    }
    for (int ai = 0; ai < a1 - a0; ai++) {
        const int va = a0 + ai, ua = va - pad;
        double l1[2], D1[2], w1h[2], Ep[2][4];  // Ep: {}, {a}, {c}, {a,c} relative to 2^R
        int R[2];
        const bool nxt = ai + 1 < a1 - a0;
        if (A.trace && ai > 0 && !nxt) t_la[0] = wall_clock64();  // the last a's prologue (units of > 1 a)
        if (!SEP || ai > 0) {
            gnx = g01[j0 * 64];
            mnx = m01[j0 * 64];
            nnx = bnn[j0 * 64];
#pragma unroll
            for (int s = 0; s < 2; s++) {
                const double* row = A.G[s] + (size_t)(nxt ? ua + 1 : ua) * ldg;
                nGab[s] = row[ib];
                nGac[s] = row[ic];
            }
        }
        wave_lds_order();  // previous a's (a, b) terms and slots fully consumed
        if (A.trace && ai == 0) t_fn[0] = wall_clock64();
        // this lane's {b} and {c} weights: registers (SEP), or re-read from LDS
        double uB[2] = {muBb[0], muBb[1]}, uC[2] = {muC[0], muC[1]};
        int uNB[2] = {nBb[0], nBb[1]}, uNC[2] = {nC[0], nC[1]};
        if (!sep) {
            const double2 x = F.lmuB[t], y = F.lmuC[t];
            const int2 nx = F.lnB[t], ny = F.lnC[t];
            uB[0] = x.x; uB[1] = x.y; uC[0] = y.x; uC[1] = y.y;
            uNB[0] = nx.x; uNB[1] = nx.y; uNC[0] = ny.x; uNC[1] = ny.y;
        }
        // this lane's A_bb, y_b, A_cc, y_c: registers (SEP), or re-read from LDS
        double vAbb[2] = {Abb[0], Abb[1]}, vyb[2] = {yb[0], yb[1]}, vAcc[2] = {Acc[0], Acc[1]}, vyc[2] = {yc[0], yc[1]};
        if (!sep) {
            const double2 p = F.lAbb[t], q = F.lyb[t], r = F.lAcc[t], u = F.lyc[t];
            vAbb[0] = p.x; vAbb[1] = p.y; vyb[0] = q.x; vyb[1] = q.y;
            vAcc[0] = r.x; vAcc[1] = r.y; vyc[0] = u.x; vyc[1] = u.y;
        }
        const unsigned pa = F.aP[ai];
        const double2 aAd = F.aAd[ai], aY = F.aY[ai];
        double pG[2], pI[2], pIW[2], pH[2], pR[2], pMu[2], pMuB[2];
        int pN[2];
#pragma unroll
        for (int s = 0; s < 2; s++) {
            const double chia = (ALLPRES || ((pa >> s) & 1u)) ? 1.0 : 0.0;
            const double ya = s ? aY.y : aY.x;
            const double ra = rsqrt_nr(s ? aAd.y : aAd.x);
            const double iAaa = ra * ra;
            const double ha = ya * ya * iAaa;
            const double rPa = ra * A.rsd[s] * chia;
            int nA;
            double muA;
            split3(ha, rPa, tab, nA, muA);
            {
                const double Gab = g1ab[s];
                const double l = Gab * iAaa;
                const double Dab = fma(-l, Gab, vAbb[s]);
                const double rab = rsqrt_nr(Dab);
                const double wab = fma(-l, ya, vyb[s]);
                const double hab = fma(wab * wab, rab * rab, ha);
                const bool chib = okb && (ALLPRES || ((pbl >> s) & 1u));
                const double rPab = chib ? rPa * rab * A.rsd[s] : 0.0;
                int nAB;
                double muAB;
                split3(hab, rPab, tab, nAB, muAB);
                const int nB = uNB[s];
                const double muB = uB[s];
                pG[s] = Gab;
                pI[s] = rab * rab;
                pIW[s] = rab * rab * (0.5 * wab);  // I_ab w_ab / 2 (the pivot itself is not needed)
                pH[s] = hab;
                pR[s] = rPab * (0.5 * A.rsd[s]);
                pMu[s] = muAB;
                pMuB[s] = ldexp(muB, nB - nAB);
                pN[s] = nAB;
            }
            const double Gac = g1ac[s];
            l1[s] = Gac * iAaa;
            D1[s] = fma(-l1[s], Gac, vAcc[s]);
            const double w1 = fma(-l1[s], ya, vyc[s]);
            w1h[s] = 0.5 * w1;
            const double r1 = rsqrt_nr(D1[s]);
            const double h1 = fma(w1 * w1, r1 * r1, ha);
            const double chic = (okc && (ALLPRES || ((pcm >> s) & 1u))) ? 1.0 : 0.0;
            const double rP1 = rPa * r1 * A.rsd[s] * chic;
            int n1;
            double mu1;
            split3(h1, rP1, tab, n1, mu1);
            R[s] = n1;
            Ep[s][0] = ldexp(1.0, -n1);
            Ep[s][1] = ldexp(muA, nA - n1);
            Ep[s][2] = ldexp(uC[s], uNC[s] - n1);
            Ep[s][3] = mu1;
        }
        F.abG[t] = make_double2(pG[0], pG[1]);
        F.abI[t] = make_double2(pI[0], pI[1]);
        F.abIW[t] = make_double2(pIW[0], pIW[1]);
        F.abH[t] = make_double2(pH[0], pH[1]);
        F.abR[t] = make_double2(pR[0], pR[1]);
        const double wac = wc * memb_weight(pa);
        if (A.trace && ai == 0) t_fn[1] = wall_clock64();
        // this a's reference G: the a accumulator sits at it; c / noCausal / the b
        // slots move their shift up to it (values scale down exactly) once per a
        const int G = R[0] + R[1];
        // Deferred fold.  Over subsets A of {a, c} (bit 0 a, bit 1 c) let c_s[A] =
        // E_s[A] (fixed for this a: Ep) and v_s[A] = E_s[A + b] (new every step).
        // An assignment puts b in study 0 only (weight v_0[A0] c_1[A1]), study 1 only
        // (c_0[A0] v_1[A1]) or both (v_0[A0] v_1[A1]).  Members a and c sit at a
        // fixed shift for the whole b-walk, so their marginals need only the sums
        // V_s = sum_j v_s and ZS[xa][xc] = sum_j v_0[A0] v_1[A1] (one per assignment
        // of the pair), folded once after the walk.  The rotating b slot takes its
        // marginals per step: b in one study are dot products with the fixed
        // vectors uW_s = (m (x) m) c_s (m = [[0, 1], [1, rho]], prior-weighted) and
        // uL_s = (m1 (x) m1) c_s (m1 = [[0, 1], [1, 1]]); b in both from the 9 products.
        double uW[2][4], uL[2][4];
#pragma unroll
        for (int s = 0; s < 2; s++) {
            const double* c = Ep[s];
            uW[s][0] = c[3];
            uW[s][1] = fma(rho, c[3], c[2]);
            uW[s][2] = fma(rho, c[3], c[1]);
            uW[s][3] = fma(rho, fma(rho, c[3], c[1] + c[2]), c[0]);
            uL[s][0] = c[3];
            uL[s][1] = c[2] + c[3];
            uL[s][2] = c[1] + c[3];
            uL[s][3] = (c[0] + c[1]) + uL[s][1];
        }
        double ZS[3][3], V0[4], V1[4];
#pragma unroll
        for (int i = 0; i < 4; i++) V0[i] = V1[i] = 0.0;
#pragma unroll
        for (int xa = 0; xa < 3; xa++)
#pragma unroll
            for (int xc = 0; xc < 3; xc++) ZS[xa][xc] = 0.0;
        int nact = 0;  // masked steps this lane took part in
        {
            const int M = max(mC, G), d = mC - M;
            cW0 = ldexp(cW0, d); cW1 = ldexp(cW1, d); cW2 = ldexp(cW2, d); cSl = ldexp(cSl, d); cNs = ldexp(cNs, d);
            mC = M;
            const int M0 = max(m0, R[1]), M1 = max(m1, R[0]);
            nc0 = ldexp(nc0, m0 - M0);
            nc1 = ldexp(nc1, m1 - M1);
            m0 = M0;
            m1 = M1;
        }
        // the walk's split constants as opaque registers (split3r)
        double k256 = 256.0, kc3 = kC3, kc2 = kC2;
        if (!SEP) kc2 = F.kc2;  // (re-read per a: not live across the walk)
        asm volatile("" : "+s"(k256), "+s"(kc3), "+v"(kc2));
        // this a's wave maxima in one batch: G (the slot shift) and, for the closed
        // forms of off-diagonal units, R_s and the slots' {a, b} exponents
        // (and the previous a's record shift)
        int mx[8] = {G, rG, R[0], R[1], pMu[0] != 0.0 ? pN[0] : EMPTY, pMu[1] != 0.0 ? pN[1] : EMPTY, EMPTY, EMPTY};
        if (sep) {
            wave_max_t(mx);
        } else {
            int g4[4] = {G, rG, R[0], R[1]};
            wave_max_t(g4);
#pragma unroll
            for (int i = 0; i < 4; i++) mx[i] = g4[i];
        }
        // The walk's b-weights are taken relative to the wave's largest R_s (Ru_s)
        // instead of the lane's own: the {b} / {a, b} weights of a slot are then
        // one value for every lane (scaled here, once per a, instead of per step
        // and lane), and each lane's factor lam_s = 2^(Ru_s - R_s) folds into the
        // lane vectors it meets (uW, uL, the slot scale) and into the walk sums
        // after the walk.  A lane more than kMaxSpread below the wave in a study
        // would lose its low terms to underflow: the unit is redone (robust).
        const int Ru[2] = {mx[2], mx[3]};
        const int sp0 = Ru[0] - R[0], sp1 = Ru[1] - R[1];
        wide |= __builtin_amdgcn_ballot_w64(max(sp0, sp1) > kMaxSpread) != 0;
        const double lam0 = ldexp(1.0, min(sp0, kMaxSpread)), lam1 = ldexp(1.0, min(sp1, kMaxSpread));
        F.abMuB[t] = make_double2(ldexp(pMuB[0], pN[0] - Ru[0]), ldexp(pMuB[1], pN[1] - Ru[1]));
        F.abMu[t] = make_double2(ldexp(pMu[0], pN[0] - Ru[0]), ldexp(pMu[1], pN[1] - Ru[1]));
        // round-to-nearest magic offset by Ru: N = round(256 (h3 - Ru)), so n3 - Ru = N >> 8
        const double cmag[2] = {kMagic - 256.0 * Ru[0], kMagic - 256.0 * Ru[1]};
        // the previous a's record: its sums at the wave's largest shift
        const int rGw = mx[1], rdg = rG != EMPTY ? rG - rGw : -2000;
        double abS[2] = {0.0, 0.0};  // sum over the slots of the {a, b} weights, at 2^abM
        int abM[2] = {EMPTY, EMPTY};
        double fS;  // a lane's contribution to the b slots is scaled by 2^(G - sM)
        {
            const int Gm = mx[0];
            const int Ms = max(sMt, Gm), d = sMt - Ms;
            sW0[t] = ldexp(sW0[t], d);
            sW1[t] = ldexp(sW1[t], d);
            sW2[t] = ldexp(sW2[t] + ldexp(sW2w[t], eZ), d);  // the previous a's walk part joins
            sSl[t] = ldexp(sSl[t] + ldexp(sSlw[t], eZ), d);
            sW2w[t] = sSlw[t] = 0.0;
            sNs[t] = ldexp(sNs[t], d);
            sMt = Ms;
            fS = ldexp(1.0, G - Ms);
            // The slot's b-in-both-studies sums take fS lam_0 lam_1 = 2^(G - Ms +
            // Ru_0 - R_0 + Ru_1 - R_1) = 2^(Ru_0 + Ru_1 - Ms) per lane: one scale for
            // the wave (a lane clamped at kMaxSpread makes the unit wide: redone), so
            // the walk adds them unscaled into sW2w / sSlw and the scale is applied
            // once, when the next a (or the unit end) folds them into sW2 / sSl
            eZ = Ru[0] + Ru[1] - Ms;
        }
        if (A.trace && ai == 0) t_fn[2] = wall_clock64();
        if (sep) {
            // b in one study, subsets {} and {a} of {a, c} with b: over the walk
            // slot b receives from every lane c once
            //   v_0[A](b, c) uW_1[A](c) 2^(G(c) - sM[b]) = E_0[A + b] 2^(-sM[b]) uW_1[A](c) 2^(R_1(c)),
            // A in {{}, {a}}, i.e. E_0[A + b] 2^(-sM[b]) times a wave sum over c
            // (likewise study 1); the walk then only takes their {b, c} and {a, b, c}
            // terms.  Lane t adds slot t's share.
            // (likewise the plain one-study sums of notSharedLL, uL: uL_s[0] = uW_s[0])
            // (and the walk sum of the {a, b} weights over the slots, V_s[1]: one batch)
            const int Qm[2] = {mx[2], mx[3]};
            double ws[16];
            ws[13] = ws[14] = ws[15] = 0.0;  // (batch padded to a multiple of 4)
#pragma unroll
            for (int s = 0; s < 2; s++) {
                ws[2 * s] = ldexp(uW[s][0], R[s] - Qm[s]);
                ws[2 * s + 1] = ldexp(uW[s][1], R[s] - Qm[s]);
                ws[4 + s] = ldexp(uL[s][1], R[s] - Qm[s]);
                ws[6 + s] = pMu[s] != 0.0 ? ldexp(pMu[s], pN[s] - mx[4 + s]) : 0.0;
            }
#pragma unroll
            for (int i = 0; i < 5; i++) ws[8 + i] = ldexp(rW[i], rdg);
            wave_sum_t(ws);
            const double QW[2][2] = {{ws[0], ws[1]}, {ws[2], ws[3]}}, QL[2] = {ws[4], ws[5]};
#pragma unroll
            for (int s = 0; s < 2; s++) {
                abS[s] = ws[6 + s];
                abM[s] = ws[6 + s] != 0.0 ? mx[4 + s] : EMPTY;
            }
#pragma unroll
            for (int i = 0; i < 5; i++) rW[i] = ws[8 + i];
            // E_s[A + b] of this lane's slot: {b} = pMuB 2^pN, {a, b} = pMu 2^pN
            const double e0 = ldexp(1.0, pN[0] + Qm[1] - sMt), e1 = ldexp(1.0, pN[1] + Qm[0] - sMt);
            sW0[t] += fma(pMuB[0], QW[1][0], pMu[0] * QW[1][1]) * e0;
            sW1[t] += fma(pMuB[1], QW[0][0], pMu[1] * QW[0][1]) * e1;
            sNs[t] += fma(fma(pMuB[0], QW[1][0], pMu[0] * QL[1]), e0, fma(pMuB[1], QW[0][0], pMu[1] * QL[0]) * e1);
            // b in both studies, a and c each in one (different) study, b's partner
            // subsets {a, b} in one study and {b, c} in the other: per step
            //   v_0[{b,c}] v_1[{a,b}] 2^(G - sM[b]) = E_0[b, c] E_1[a, b] 2^(-sM[b])
            // (no lane scale left), summed over c: E_1[a, b] x the tile's column sum
            // of the {b, c} weights, for both prior-weighted (W2) and plain (sharedLL)
            // sums (their coefficient in Z0 is 1)
            const double2 cs = F.bccm[t];
            const int2 cn = F.bccn[t];
            const double z0 = fma(pMu[1] * cs.x, ldexp(1.0, pN[1] + cn.x - sMt), pMu[0] * cs.y * ldexp(1.0, pN[0] + cn.y - sMt));
            sW2[t] += z0;
            sSl[t] += z0;
        }
        if (!sep) {
            double r5[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int i = 0; i < 5; i++) r5[i] = ldexp(rW[i], rdg);
            wave_sum_t(r5);
#pragma unroll
            for (int i = 0; i < 5; i++) rW[i] = r5[i];
        }
        if (t == 0 && rq >= 0) store_rec(rec + rq, wrec(rGw, rW[0], rW[1], rW[2], rW[3], rW[4], rho, A.Ck, A.pit0));
        if (A.trace && ai == 0) t_fn[3] = wall_clock64();
        // the slot scale rides in the prior-weighted vectors (only the b-slot dot
        // products use them from here on; a power of two, so exact above underflow)
        // (uW_s / uL_s meet study 1 - s's b-weights: lam_(1 - s); the {b, c} x
        // {a, b, c} products, lam_0 lam_1 with the slot scale: 2^eZ, applied per a)
        const double fW[2] = {fS * lam1, fS * lam0};
#pragma unroll
        for (int s = 0; s < 2; s++)
#pragma unroll
            for (int i = 0; i < 4; i++) uW[s][i] *= fW[s];
        // SEP: so does the notSharedLL vector (its whole-value check is on the slot
        // totals), the {b, c} / {a, b, c} entries the walk uses
        if (sep) {
#pragma unroll
            for (int s = 0; s < 2; s++)
#pragma unroll
                for (int i = 2; i < 4; i++) uL[s][i] *= fW[s];
        } else {
#pragma unroll
            for (int i = 0; i < 4; i++) {
                uL[0][i] *= lam1;
                uL[1][i] *= lam0;
            }
        }
        wave_lds_order();  // (a, b) terms and slot shifts visible
        if (nxt) {
#pragma unroll
            for (int s = 0; s < 2; s++) {
                g1ab[s] = okb ? nGab[s] : 0.0;
                g1ac[s] = okc ? nGac[s] : 0.0;
            }
        }
        if (A.trace && ai == 0) t_ph[1] = wall_clock64();
        if (A.trace && ai > 0 && !nxt) t_la[1] = wall_clock64();

        // The b-walk.  chain(j) is step j's dependent {a, b, c} extension up to
        // the split of 2^h3 (N = round(256 h3), q = 2^(f/256) P^(-1/2)); finish(j)
        // takes the table entry, rescales the four b weights, folds the 27
        // assignments and accumulates.  Off-diagonal tiles (every lane active every
        // step) run chain(j + 1) beside finish(j), so the serial chain of one step
        // overlaps the wide fold of the previous one; the Sigma~ tile row is
        // fetched two steps ahead, the {b, c} weights one.
        bool tiny = false;
        int dA = -(1 << 20);  // largest n_abc - Ru over the walk (both studies)
        // Step j's b slot is bs = (t + j) & 63; the lambdas take its LDS byte
        // offsets (o16 = 16 bs into the double2 slot arrays, o8 = 8 bs into the
        // double ones), stepped by the walk (one add and mask per step)
        auto slot = [](const auto& arr, unsigned off) -> const auto& {
            return *reinterpret_cast<const std::remove_reference_t<decltype(arr[0])>*>(
                reinterpret_cast<const char*>(arr) + off);
        };
        auto chain = [&](unsigned o16, double2 g, int (&N)[2], double (&q)[2]) {
            const double2 aG = slot(F.abG, o16), aI = slot(F.abI, o16), aIW = slot(F.abIW, o16),
                          aH = slot(F.abH, o16), aR = slot(F.abR, o16);
#pragma unroll
            for (int s = 0; s < 2; s++) {
                // x = the unnormalised L entry of c against b; D_ab I_ab = 1 folds the pivot away
                const double Gbc = s ? g.y : g.x;
                const double x = fma(-l1[s], s ? aG.y : aG.x, Gbc);
                const double lcb = x * (s ? aI.y : aI.x);
                const double D3 = fma(-x, lcb, D1[s]);
                const double w3 = fma(-x, s ? aIW.y : aIW.x, w1h[s]);
                const double r3 = rsq2x(D3);
                const double t3 = w3 * r3;
                const double h3 = fma(t3, t3, s ? aH.y : aH.x);
                double rP3 = (s ? aR.y : aR.x) * r3;
                if (!ALLPRES && !((pcm >> s) & 1u)) rP3 = 0.0;  // c absent from study s
                split3r(h3, rP3, cmag[s], k256, kc3, kc2, N[s], q[s]);
            }
        };
        // SEP (off-diagonal units): the {} / {a} parts of the prior-weighted one-study
        // dot products and the walk sums V_s[0 .. 2] have closed forms (a prologue,
        // after the walk).  Their notSharedLL (NB) holds only the {b, c} / {a, b, c}
        // part, so it is not checked per step: the b slot's whole notSharedLL total
        // (closed-form + walk parts) is checked against kTinyNs once, after the
        // unit (the `low` flag below).  Diagonal units keep the per-step NB check.
        // finish(j)'s LDS operands: its slot's {b} / {a, b} terms and scale, and the
        // exp2 table entries of the chain's split (read as soon as the chain ends)
        struct FTt {
            double2 muB, mu;  // the slot's {b} / {a, b} weights relative to 2^Ru_s
            double tb0, tb1;
        };
        auto ld_ft = [&](unsigned o16, const int (&N)[2]) {
            return FTt{slot(F.abMuB, o16), slot(F.abMu, o16), tab[N[0] & 255], tab[N[1] & 255]};
        };
        auto finish_ft = [&](unsigned o8, const FTt& ft, const int (&N)[2], const double (&q)[2], double2 mcur,
                             int2 ncur) {
            constexpr bool sepc = SEP;
            auto acc = [&](double (&arr)[64]) -> double* { return reinterpret_cast<double*>(reinterpret_cast<char*>(arr) + o8); };
            const double2 aMuB = ft.muB, aMu = ft.mu;
            // v[s][A] = E_s[A + b] relative to 2^{Ru_s}: {b}, {a, b}, {b, c}, {a, b, c}
            double v[2][4];
            int d3s = 0;
#pragma unroll
            for (int s = 0; s < 2; s++) {
                const int d3 = N[s] >> 8;  // n3 - Ru (N is Ru-relative)
                const double mu3 = (s ? ft.tb1 : ft.tb0) * q[s];
                const int n2 = s ? ncur.y : ncur.x;
                const double mu2 = s ? mcur.y : mcur.x;
                d3s += d3;
                v[s][0] = s ? aMuB.y : aMuB.x;
                v[s][1] = s ? aMu.y : aMu.x;
                v[s][2] = ldexp(mu2, n2 - Ru[s]);
                v[s][3] = ldexp(mu3, d3);
            }
            dA = max(dA, d3s);
            auto dot4 = [](const double (&u)[4], const double (&x)[4], double acc0) {
                return fma(u[3], x[3], fma(u[2], x[2], fma(u[1], x[1], fma(u[0], x[0], acc0))));
            };
            auto dot2 = [](const double (&u)[4], const double (&x)[4], double acc0) {  // the {b, c} and {a, b, c} terms
                return fma(u[3], x[3], fma(u[2], x[2], acc0));
            };
            // ---- member b (this step's slot): b in study 0 only / study 1 only ----
            const double WB0 = sepc ? dot2(v[0], uW[1], 0.0) : dot4(v[0], uW[1], 0.0);
            const double WB1 = sepc ? dot2(v[1], uW[0], 0.0) : dot4(v[1], uW[0], 0.0);
            const double NB = sepc ? dot2(v[0], uL[1], dot2(v[1], uL[0], 0.0)) : dot4(v[0], uL[1], dot4(v[1], uL[0], 0.0));
            // ---- b in both studies: the 9 assignments of (a, c); their sums for a and c ----
#pragma unroll
            for (int xa = 0; xa < 3; xa++)
#pragma unroll
                for (int xc = 0; xc < 3; xc++) {
                    const int i0 = (xa != 1) | ((xc != 1) << 1), i1 = (xa != 0) | ((xc != 0) << 1);
                    ZS[xa][xc] = fma(v[0][i0], v[1][i1], ZS[xa][xc]);
                }
            // Z0: (xa, xc) in {0,1}^2 -> (i0, i1) = (3,0), (1,2), (2,1), (0,3); SEP: the
            // {b, c} x {a, b} pairs (1,2), (2,1) in closed form (a prologue)
            const double Z0 = sepc ? fma(v[0][0], v[1][3], v[0][3] * v[1][0])
                                   : fma(v[0][0], v[1][3], fma(v[0][2], v[1][1], fma(v[0][1], v[1][2], v[0][3] * v[1][0])));
            // Z1: one of a, c in both studies -> (3,1), (1,3), (3,2), (2,3)
            const double Z1 = fma(v[0][2], v[1][3], fma(v[0][3], v[1][2], fma(v[0][1], v[1][3], v[0][3] * v[1][1])));
            const double z22 = v[0][3] * v[1][3];
            const double WB2 = fma(rho, fma(rho, z22, Z1), Z0);
            const double LB2 = (Z0 + Z1) + z22;
#pragma unroll
            for (int i = sepc ? 3 : 0; i < 4; i++) {
                V0[i] += v[0][i];
                V1[i] += v[1][i];
            }
            // (SEP: NB is a part of the set's notSharedLL; the slot's total is checked
            // after the unit instead)
            if (!sepc) tiny |= NB < kTinyNs;
            // ---- b slot (LDS, x fS: WB0 / WB1 carry it from uW) ----
            // LDS float adds: no read round trip; one lane per slot per step, and a
            // wave's LDS instructions execute in issue order (deterministic)
            __hip_atomic_fetch_add(acc(sW0), WB0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add(acc(sW1), WB1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add(acc(sW2w), WB2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add(acc(sSlw), LB2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add(acc(sNs), sepc ? NB : NB * fS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (!ALLPRES) npat += wac * *reinterpret_cast<const float*>(reinterpret_cast<const char*>(bW) + (o8 >> 1));
        };
        auto o16of = [&](int j) { return (unsigned)((t + j) & 63) << 4; };
        auto finish = [&](int j, const int (&N)[2], const double (&q)[2], double2 mcur, int2 ncur) {
            finish_ft(o16of(j) >> 1, ld_ft(o16of(j), N), N, q, mcur, ncur);
        };
        // Steps on which every lane is active run pipelined: the whole walk of an
        // off-diagonal tile, and steps 1..30 of a diagonal tile whose a lies
        // outside its block (pairs {slot, t} of the block, no padding lane).  The
        // rest (a inside the block, step 31 / 32, padding) take the masked loop.
        int je = j0;
        if (!diag)
            je = j0 + ((j1 - j0) & ~1);
        else if ((va < 64 * K || va >= 64 * K + 64) && 64 * K >= pad)
            je = j0 + ((min(j1, 32) - j0) & ~1);
        auto walk = [&]() {
            // unrolled by two: the chained state alternates between (NA, qA) and (NB, qB).
            // Loads run up to three rows ahead unclamped (the buffers carry
            // kTileRowPad rows past the last tile; what lies past je is not used),
            // so they address off one lane offset with immediate row offsets
            // (the tile bases are wave-uniform and the lane's row offset a 32-bit
            // unsigned byte count: base + offset + row immediates, one add per pair)
            const char* gb = (const char*)(A.g01 + (size_t)tile * 4096);
            const char* mb = (const char*)(A.mu01 + (size_t)tile * 4096);
            const char* nb = (const char*)(A.bcn + (size_t)tile * 4096);
            unsigned o16 = (unsigned)(j0 * 64 + t) * 16u, o8 = o16 >> 1;  // double2 / int2 rows: 1024 / 512 bytes
            double2 g_next = *(const double2*)(gb + o16 + 1024);
            double2 m_cur = mnx;
            int2 n_cur = nnx;
            int NA[2], NB[2];
            double qA[2], qB[2];
            unsigned s8 = o16of(j0) >> 1;  // step j's slot offset (8-byte arrays)
            chain(s8 << 1, gnx, NA, qA);
            // each finish's LDS operands are read right after the chain it follows,
            // one half step pair before the finish runs
            FTt ftA = ld_ft(s8 << 1, NA);
            for (int j = j0; j < je; j += 2) {
                // (advanced first: the pair's loads all address off the new offsets,
                // so the old ones die here and the loop carries no register copy)
                o16 += 2048u;
                o8 += 1024u;
                double2 m_nxt = *(const double2*)(mb + o16 - 1024);
                int2 n_nxt = *(const int2*)(nb + o8 - 512);
                double2 g_after = *(const double2*)(gb + o16);
                const unsigned s8b = (s8 + 8u) & 504u;
                chain(s8b << 1, g_next, NB, qB);
                finish_ft(s8, ftA, NA, qA, m_cur, n_cur);
                const FTt ftB = ld_ft(s8b << 1, NB);
                s8 = (s8b + 8u) & 504u;  // step j + 2 (the old offset is dead: no loop copy)
                // b-slot ownership rotates across lanes every step: the workgroup is
                // one wave and LDS executes a wave's instructions in issue order
                __builtin_amdgcn_wave_barrier();
                m_cur = *(const double2*)(mb + o16);
                n_cur = *(const int2*)(nb + o8);
                g_next = *(const double2*)(gb + o16 + 1024);
                // the row loads at the top of this pair of steps are first used here
                // (and this half's loads first in the next pair): pinned, so the
                // scheduler cannot hoist a use to where it would wait for a load
                // issued only ~80 instructions earlier (the tile rows come from the
                // MALL).  Same-box A/B: world 1 1.043 -> 1.016 ms.
                pin_vgpr(m_nxt);
                pin_vgpr(n_nxt);
                pin_vgpr(g_after);
                chain(s8 << 1, g_after, NA, qA);  // (the last pair's is not used)
                finish_ft(s8b, ftB, NB, qB, m_nxt, n_nxt);
                ftA = ld_ft(s8 << 1, NA);
                __builtin_amdgcn_wave_barrier();
                pin_vgpr(m_cur);
                pin_vgpr(n_cur);
                pin_vgpr(g_next);
            }
        };
        if (je > j0) {
            walk();
            if (je < j1) {
                gnx = g01[je * 64];
                mnx = m01[je * 64];
                nnx = bnn[je * 64];
            }
        }
        for (int j = je; j < j1; j++) {
            const double2 gcur = gnx, mcur = mnx;
            const int2 ncur = nnx;
            if (j + 1 < j1) {
                gnx = g01[(j + 1) * 64];
                mnx = m01[(j + 1) * 64];
                nnx = bnn[(j + 1) * 64];
            }
            const int bs = (t + j) & 63;
            const int vb = 64 * K + bs;
            // off-diagonal: a < block K < block C.  Diagonal: the pair {slot, t} of
            // the block with a below both, or any real pair when a lies after the
            // block (steps 1..31, + 32 on lanes < 32)
            const bool act = diag ? (((vb > va && vc > va) || (va >= 64 * K + 64 && vb >= pad && vc >= pad)) &&
                                     (j < 32 || t < 32))
                                  : (okc && vb > va && vb < vc);
            if (act) {
                int N[2];
                double q[2];
                chain(o16of(j), gcur, N, q);
                finish(j, N, q, mcur, ncur);  // (never in SEP units: their walk is all pipelined)
                nact++;
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (A.trace && ai == 0) t_ph[2] = wall_clock64();
        // the walk sums back to the lane's own R_s (and n_abc - R for the redo test);
        // the lane factors are recomputed here from R_s (not held across the walk)
        {
            int ru0 = Ru[0], ru1 = Ru[1];
            asm volatile("" : "+s"(ru0), "+s"(ru1));
            const int q0 = ru0 - R[0], q1 = ru1 - R[1];
            dmax = max(dmax, dA + q0 + q1);
            const double m0f = ldexp(1.0, min(q0, kMaxSpread)), m1f = ldexp(1.0, min(q1, kMaxSpread));
#pragma unroll
            for (int i = sep ? 3 : 0; i < 4; i++) {
                V0[i] *= m0f;
                V1[i] *= m1f;
            }
            const double l01 = m0f * m1f;
#pragma unroll
            for (int xa = 0; xa < 3; xa++)
#pragma unroll
                for (int xc = 0; xc < 3; xc++) ZS[xa][xc] *= l01;
        }
        nact += je - j0;
        if (ALLPRES) npat += 27.0 * nact;
        if (sep) {
            // the walk sums of the {b}, {a, b} and {b, c} weights relative to 2^R_s:
            // the block's {b} sum (unit prologue), this a's {a, b} sum over the slots
            // (wave sum of the slot owners' LDS terms) and the tile row's {b, c} sum
            const double2 bsm = F.bcsm[t];
            const int2 bsn = F.bcsn[t];
#pragma unroll
            for (int s = 0; s < 2; s++) {
                double* Vs = s ? V1 : V0;
                Vs[0] = ldexp(F.pbS[s], F.pbM[s] - R[s]);
                Vs[1] = ldexp(abS[s], abM[s] - R[s]);  // (a prologue's batch)
                Vs[2] = ldexp(s ? bsm.y : bsm.x, (s ? bsn.y : bsn.x) - R[s]);
            }
        }
        // ---- members a and c: fold the walk's sums.  Per assignment (xa, xc) of the
        // pair, L = (b in study 0 only) + (b in study 1 only), then b in both from ZS
        double Cw[3][3], Cu[3][3];  // prior-weighted (b's rho, not a's or c's) / plain
#pragma unroll
        for (int xa = 0; xa < 3; xa++)
#pragma unroll
            for (int xc = 0; xc < 3; xc++) {
                const int i0 = (xa != 1) | ((xc != 1) << 1), i1 = (xa != 0) | ((xc != 0) << 1);
                const double L = fma(V0[i0], Ep[1][i1], Ep[0][i0] * V1[i1]);
                Cw[xa][xc] = fma(rho, ZS[xa][xc], L);
                Cu[xa][xc] = L + ZS[xa][xc];
            }
        double WA[3], WC[3];
#pragma unroll
        for (int x = 0; x < 3; x++) {
            WA[x] = fma(rho, Cw[x][2], Cw[x][0] + Cw[x][1]);
            WC[x] = fma(rho, Cw[2][x], Cw[0][x] + Cw[1][x]);
        }
        const double LA2 = (Cu[2][0] + Cu[2][1]) + Cu[2][2];
        const double NA = ((Cu[0][0] + Cu[0][1]) + Cu[0][2]) + ((Cu[1][0] + Cu[1][1]) + Cu[1][2]);
        const double LC2 = (Cu[0][2] + Cu[1][2]) + Cu[2][2];
        const double NC = ((Cu[0][0] + Cu[1][0]) + Cu[2][0]) + ((Cu[0][1] + Cu[1][1]) + Cu[2][1]);
        // a notSharedLL sum far below the shift loses precision: exact rerun
        if (nact > 0) tiny |= (NA < kTinyNs) | (NC < kTinyNs);
        const double fC = ldexp(1.0, G - mC), f0 = ldexp(1.0, R[1] - m0), f1 = ldexp(1.0, R[0] - m1);
        cW0 = fma(WC[0], fC, cW0);
        cW1 = fma(WC[1], fC, cW1);
        cW2 = fma(WC[2], fC, cW2);
        cSl = fma(LC2, fC, cSl);
        cNs = fma(NC, fC, cNs);
        // noCausal[s]: every member in the other study only
        nc0 = fma(V1[3], f0, nc0);
        nc1 = fma(V0[3], f1, nc1);
        if (!wide && __builtin_amdgcn_ballot_w64(tiny))  // (a wide unit is redone: its values are void)
            if (tiny) atomicOr(flag, 1);
        if (A.trace && ai == 0) t_fn[4] = wall_clock64();
        {
            // the a record, pending: every lane's five sums share its shift G, so the
            // wave folds them at the largest G among lanes with content (a lane's
            // notSharedLL is >= 2^-900 of its own G, so nothing that matters is
            // lost), in the next batch of wave reductions
            const bool has = (WA[0] + WA[1] + WA[2] + LA2 + NA) != 0.0;
            rW[0] = WA[0];
            rW[1] = WA[1];
            rW[2] = WA[2];
            rW[3] = LA2;
            rW[4] = NA;
            rG = has ? G : EMPTY;
            rq = F.aPos[ai];
        }
        if (A.trace && ai == 0) t_ph[3] = wall_clock64();
    }
    if (!SEP) {  // (non-SEP units: loaded late, so they are not live across the walks)
        posC = pos[rbase + t];
        posB = pos[rbase + 64 + t];
    }
    wave_lds_order();
    {
        // a diagonal tile's lane t and b slot t are one SNP: one record (the plan
        // keys no b records there), folded here instead of in the merge
        Acc5 rc = wrec(mC, cW0, cW1, cW2, cSl, cNs, rho, A.Ck, A.pit0);
        const Acc5 rb = wrec(sMt, sW0[t], sW1[t], sW2[t] + ldexp(sW2w[t], eZ), sSl[t] + ldexp(sSlw[t], eZ), sNs[t],
                             rho, A.Ck, A.pit0);
        if (sep) {
            // the b slot's notSharedLL total (closed-form and walk parts) against the
            // fast path's floor: at or above 2^-900 of the slot shift, every term lost
            // to underflow (< 2^-1074 each) is below 2^-174 of it; below, exact rerun
            const bool low = okb && sNs[t] < kTinyNs;
            if (!wide && __builtin_amdgcn_ballot_w64(low))
                if (low) atomicOr(flag, 2);  // bit 1: the SEP b-slot trigger (psx_timing.exact_rerun)
        }
        if (diag) fold_acc(rc, rb);
        if (posC >= 0) store_rec(rec + posC, rc);
        if (!diag && posB >= 0) store_rec(rec + posB, rb);
    }
    SetRec sr;
    sr.tot = ((cW0 + cW1) + rho * cW2) * A.pit0;  // every assignment of the lane's sets
    sr.m = (sr.tot != 0.0) ? mC + A.Ck : EMPTY;
    sr.nc0 = nc0 * A.pit0;
    sr.m0 = (sr.nc0 != 0.0) ? m0 + A.Ck : EMPTY;
    sr.nc1 = nc1 * A.pit0;
    sr.m1 = (sr.nc1 != 0.0) ? m1 + A.Ck : EMPTY;
    sr.pad = 0;
    sr.score = 1e300;
    sr.npat = npat;
    {
        // the unit's set record across the wave: three (shift, sum) pairs and the
        // pattern count, with the last a's pending record, in one batch (score:
        // 1e300 in every lane)
        int m3[3] = {sr.m, sr.m0, sr.m1};
        double x3[3] = {sr.tot, sr.nc0, sr.nc1};
        int M3[4];
#pragma unroll
        for (int k = 0; k < 3; k++) M3[k] = x3[k] != 0.0 ? m3[k] : EMPTY;
        M3[3] = rG;
        wave_max_t(M3);
        const int rdg = rG != EMPTY ? rG - M3[3] : -2000;
        double x4[12] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < 3; k++) x4[k] = x3[k] != 0.0 ? ldexp(x3[k], m3[k] - M3[k]) : 0.0;
        x4[3] = sr.npat;
#pragma unroll
        for (int i = 0; i < 5; i++) x4[4 + i] = ldexp(rW[i], rdg);
        wave_sum_t(x4);
        if (t == 0 && rq >= 0) store_rec(rec + rq, wrec(M3[3], x4[4], x4[5], x4[6], x4[7], x4[8], rho, A.Ck, A.pit0));
        sr.tot = x4[0];
        sr.m = x4[0] != 0.0 ? M3[0] : EMPTY;
        sr.nc0 = x4[1];
        sr.m0 = x4[1] != 0.0 ? M3[1] : EMPTY;
        sr.nc1 = x4[2];
        sr.m1 = x4[2] != 0.0 ? M3[2] : EMPTY;
        sr.npat = x4[3];
    }
    if (t == 0) store_rec(srec + unit, sr);
    redo = wide || __builtin_amdgcn_ballot_w64(dmax > kMaxRefGap) != 0;
    if (A.trace && t == 0) {
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        unsigned long long* tr = A.trace + kTraceWords * (size_t)unit;
        tr[0] = t_start;
        tr[1] = wall_clock64();
        tr[2] = hw | ((unsigned long long)xcc << 32) | ((unsigned long long)K << 40) | ((unsigned long long)C << 48);
        tr[3] = (unsigned long long)unit | ((unsigned long long)diag << 32) | ((unsigned long long)(a1 - a0) << 33) |
                ((unsigned long long)redo << 40);
        for (int i = 0; i < 4; i++) tr[4 + i] = t_ph[i];
        for (int i = 0; i < 6; i++) tr[8 + i] = t_fn[i];
        tr[14] = t_la[0];
        tr[15] = t_la[1];
    }
}

// The k = 3 sweep: one block per unit (fast variant, redone robustly in the same
// block when flagged); level-2 units ride in the same launch, after them.
template <bool ALLPRES>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(PSX_K3_WAVES, PSX_K3_WAVES))) void k_sweep3(Sweep3Args A, const int4* __restrict__ units,
                                                  Acc5* __restrict__ rec, SetRec* __restrict__ srec, int rec_stride,
                                                  int* __restrict__ flag, const int* __restrict__ pos, int nk3,
                                                  TileArgs A2, const int4* __restrict__ units2,
                                                  Acc5* __restrict__ rec2, SetRec* __restrict__ srec2,
                                                  const int* __restrict__ pos2) {
    __shared__ SweepSmem sm;
    // a single pass times its sweep without dispatch events (their packets left
    // ~5 us between the sweep and the merge): the launch's first block stamps
    // its start, the merge's first block its own (k_merge_rec)
    if (A.tstamp && blockIdx.x == 0 && threadIdx.x == 0) *A.tstamp = wall_clock64();
    if ((int)blockIdx.x >= nk3) {
        sweep_unit<2, false>(A2, blockIdx.x - nk3, units2, rec2, srec2, 128, flag, pos2, sm.u2);
        return;
    }
    bool redo = false;
    // off-diagonal units with the whole b-walk (all of them, as plan_units3c
    // cuts them) take the closed-form variant; a copy of the unit code each, so
    // each copy's walk loop gets its own register assignment (one function with
    // both loops rotated ~14 loop-carried registers per step pair in the other)
    const int4 un = units[blockIdx.x];
    if ((un.z & 0xffff) != (un.w & 0xffff) && (un.z >> 16) == 0 && (un.w >> 16) == 64)
        sweep3_unit_fast<ALLPRES, true>(A, blockIdx.x, units, rec, srec, rec_stride, flag, pos, sm, redo);
    else
        sweep3_unit_fast<ALLPRES, false>(A, blockIdx.x, units, rec, srec, rec_stride, flag, pos, sm, redo);
    if (redo) {
        if (threadIdx.x == 0 && A.redo_count) atomicAdd(A.redo_count, 1);
        __syncthreads();
        sweep3_unit_robust<ALLPRES>(A, blockIdx.x, units, rec, srec, rec_stride, flag, pos, sm);
    }
}

// skewT[tile(K, C)][j][t] = G~[64C + t][64K + ((t + j) & 63)] for K <= C, in the
// padded index space v = u + pad (zero where either index is padding)
__global__ void k_build_skewT(const double* __restrict__ G, int ldg, int pad, double* __restrict__ skew) {
    const int tile = blockIdx.x;
    const int j = blockIdx.y;
    const int t = threadIdx.x;
    int C = 0;
    while ((C + 1) * (C + 2) / 2 <= tile) C++;
    const int K = tile - C * (C + 1) / 2;
    const int v = 64 * C + t, w = 64 * K + ((t + j) & 63);
    skew[(size_t)tile * 4096 + j * 64 + t] = (v >= pad && w >= pad) ? G[(size_t)(v - pad) * ldg + (w - pad)] : 0.0;
}

int launch_build_skewT(const double* G, int ldg, int pad, double* skew, hipStream_t st) {
    const int nblk = ldg / 64;
    hipLaunchKernelGGL(k_build_skewT, dim3(nblk * (nblk + 1) / 2, 64), dim3(64), 0, st, G, ldg, pad, skew);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_build_bc3(const Sweep3Args& A, int ntile, double2* mu01, int2* n, hipStream_t st) {
    // a non-ALLPRES build is exact for every locus (chi factors of present SNPs are 1)
    hipLaunchKernelGGL((k_build_bc3<false>), dim3(ntile, 64), dim3(64), 0, st, A, mu01, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// per tile and lane t (c = 64C + t): sum over the 64 steps j (every b of block K)
// of the {b, c} weights 2^bcn * mu01, both studies, at the largest exponent of
// the lane's nonzero terms (in step order)
__global__ __launch_bounds__(64) void k_bc3_rowsum(const double2* __restrict__ mu01, const int2* __restrict__ n,
                                                   double2* __restrict__ sm, int2* __restrict__ sn) {
    const size_t base = (size_t)blockIdx.x * 4096 + threadIdx.x;
    int M0 = EMPTY, M1 = EMPTY;
    for (int j = 0; j < 64; j++) {
        const double2 m = mu01[base + 64 * j];
        const int2 e = n[base + 64 * j];
        if (m.x != 0.0) M0 = max(M0, e.x);
        if (m.y != 0.0) M1 = max(M1, e.y);
    }
    double S0 = 0.0, S1 = 0.0;
    for (int j = 0; j < 64; j++) {
        const double2 m = mu01[base + 64 * j];
        const int2 e = n[base + 64 * j];
        if (m.x != 0.0) S0 += ldexp(m.x, e.x - M0);
        if (m.y != 0.0) S1 += ldexp(m.y, e.y - M1);
    }
    sm[(size_t)blockIdx.x * 64 + threadIdx.x] = make_double2(S0, S1);
    sn[(size_t)blockIdx.x * 64 + threadIdx.x] = make_int2(M0, M1);
}

int launch_bc3_rowsum(int ntile, const double2* mu01, const int2* n, double2* sm, int2* sn, hipStream_t st) {
    hipLaunchKernelGGL(k_bc3_rowsum, dim3(ntile), dim3(64), 0, st, mu01, n, sm, sn);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// per tile and b slot (thread b): the same sum over the 64 c of the tile; slot b
// sits at step j in lane (b - j) & 63
__global__ __launch_bounds__(64) void k_bc3_colsum(const double2* __restrict__ mu01, const int2* __restrict__ n,
                                                   double2* __restrict__ sm, int2* __restrict__ sn) {
    const size_t base = (size_t)blockIdx.x * 4096;
    const int b = threadIdx.x;
    int M0 = EMPTY, M1 = EMPTY;
    for (int j = 0; j < 64; j++) {
        const size_t o = base + 64 * j + ((b - j) & 63);
        const double2 m = mu01[o];
        const int2 e = n[o];
        if (m.x != 0.0) M0 = max(M0, e.x);
        if (m.y != 0.0) M1 = max(M1, e.y);
    }
    double S0 = 0.0, S1 = 0.0;
    for (int j = 0; j < 64; j++) {
        const size_t o = base + 64 * j + ((b - j) & 63);
        const double2 m = mu01[o];
        const int2 e = n[o];
        if (m.x != 0.0) S0 += ldexp(m.x, e.x - M0);
        if (m.y != 0.0) S1 += ldexp(m.y, e.y - M1);
    }
    sm[(size_t)blockIdx.x * 64 + b] = make_double2(S0, S1);
    sn[(size_t)blockIdx.x * 64 + b] = make_int2(M0, M1);
}

int launch_bc3_colsum(int ntile, const double2* mu01, const int2* n, double2* sm, int2* sn, hipStream_t st) {
    hipLaunchKernelGGL(k_bc3_colsum, dim3(ntile), dim3(64), 0, st, mu01, n, sm, sn);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

__global__ void k_interleave2(const double* __restrict__ a, const double* __restrict__ b, size_t n,
                              double2* __restrict__ out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = make_double2(a[i], b[i]);
}

int launch_interleave2(const double* a, const double* b, size_t n, double2* out, hipStream_t st) {
    hipLaunchKernelGGL(k_interleave2, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a, b, n, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_sweep3(bool allpres, const Sweep3Args& A, int n_units, const int4* units, Acc5* rec, SetRec* srec,
                  int rec_stride, int* flag, const int* pos, hipStream_t st, const Level2Blocks* l2, hipEvent_t ev0,
                  hipEvent_t ev1) {
    const Level2Blocks none{0, TileArgs{}, nullptr, nullptr, nullptr, nullptr};
    const Level2Blocks& b = l2 ? *l2 : none;
    const dim3 grid(n_units + b.n);
    // with events: their timestamps / completion ride in the dispatch packet
    // itself (no marker packets between back-to-back passes)
    if (allpres)
        hipExtLaunchKernelGGL((k_sweep3<true>), grid, dim3(64), 0, st, ev0, ev1, 0, A, units, rec, srec, rec_stride,
                              flag, pos, n_units, b.A, b.units, b.rec, b.srec, b.pos);
    else
        hipExtLaunchKernelGGL((k_sweep3<false>), grid, dim3(64), 0, st, ev0, ev1, 0, A, units, rec, srec, rec_stride,
                              flag, pos, n_units, b.A, b.units, b.rec, b.srec, b.pos);
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

// load this translation unit's device code on the current device (psx_warmup)
int warm_module_sweep3() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, (const void*)k_scale_y) == hipSuccess ? 0 : -1;
}

}  // namespace psx
