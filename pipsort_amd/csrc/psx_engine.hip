// psx_engine.hip — MI355X (gfx950) posterior-calculation engine for PIPSORT.
//
// Replaces PostCal's configuration sweep (postcal.cpp:400-1092,
// sss_postcal.cpp:102-685) with HIP kernels.  See DESIGN.md for the data layout
// and the kernel inventory; psx_math.h for the accumulator representation.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <map>
#include <random>
#include <string>
#include <tuple>
#include <vector>
#include <thread>

#include "../../include/pipsort_engine.h"
#include "../../include/pipsort_model.h"
#include "psx_configs.h"
#include "psx_math.h"
#include "psx_sample.h"
#include "psx_setup.h"
#include "psx_sweep.h"
#include "psx_sweep_dev.h"
#include "psx_mem.h"
#include "psx_wave.h"

extern "C" __device__ __attribute__((const)) double __ockl_wfred_min_f64(double);

using psx::Acc5;
using psx::kPlanMagic;
using psx::PlanTag;
using psx::SetRec;

namespace {

thread_local std::string g_err;
constexpr int kPlanMismatchWord = 8;  // status word raised by k_merge_partials

constexpr size_t kStatBytes = 3 * 56;  // SetRec, PlanTag, status words (EXACT flag first)

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(expr)                                                                          \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess)                                                                 \
            return fail(PSX_EHIP, std::string("HIP error ") + hipGetErrorString(_e) + " at " + \
                                      __FILE__ + ":" + std::to_string(__LINE__) + ": " #expr); \
    } while (0)

// ---------------------------------------------------------------------------
// Device problem description (union-indexed, see DESIGN.md "HBM layout")
// ---------------------------------------------------------------------------
struct DevProb {
    int U, ldg;                   // union SNPs, padded leading dimension (multiple of 64)
    const double* G[2];           // Sigma~_s in union coordinates, ldg x ldg, 0 where absent
    const double* Ad[2];          // 1/d_s + Sigma~_s[u,u]  (1/d_s where absent / padding)
    const double* y[2];           // y_s = B_s^T S'_s in union coordinates (0 where absent)
    const unsigned char* pres;    // bit s set when union SNP u is in study s
    double dval[2];               // d_s = s^2 n_s / min(n) + t^2   (postcal.cpp:89)
    int Ck[PSX_KMAX + 1];         // integer prior shift per causal-set size
    double pit[PSX_KMAX + 1][PSX_KMAX + 1];    // 2^{prior(k,nsh) log2e - Ck[k]}
    double prior[PSX_KMAX + 1][PSX_KMAX + 1];  // prior(k, nsh) in nats (postcal.cpp:19-59)
};

__device__ inline double wave_sum(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ inline double wave_min(double v) {
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
    return v;
}

// ---------------------------------------------------------------------------
// Setup kernels: Sigma~_s = B_s^T B_s (FP64, LDS tiled), y_s = B_s^T S'_s
// ---------------------------------------------------------------------------
// B column-major M x M: Sigma~[i][j] = sum_r B[i*M + r] * B[j*M + r]
__global__ __launch_bounds__(256) void k_btb(const double* __restrict__ B, int M, double* __restrict__ out) {
    __shared__ double ti[16][17], tj[16][17];
    int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    int i0 = blockIdx.y * 16, j0 = blockIdx.x * 16;
    double acc = 0.0;
    for (int r0 = 0; r0 < M; r0 += 16) {
        int r = r0 + tx;
        int ci = i0 + ty, cj = j0 + ty;
        ti[ty][tx] = (ci < M && r < M) ? B[(size_t)ci * M + r] : 0.0;
        tj[ty][tx] = (cj < M && r < M) ? B[(size_t)cj * M + r] : 0.0;
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < 16; kk++) acc = fma(ti[ty][kk], tj[tx][kk], acc);
        __syncthreads();
    }
    int i = i0 + ty, j = j0 + tx;
    if (i < M && j < M) out[(size_t)i * M + j] = acc;
}

__global__ void k_bts(const double* __restrict__ B, const double* __restrict__ sp, int M, double* __restrict__ y) {
    int i = blockIdx.x;
    double acc = 0.0;
    for (int r = threadIdx.x; r < M; r += 64) acc = fma(B[(size_t)i * M + r], sp[r], acc);
    acc = wave_sum(acc);
    if (threadIdx.x == 0) y[i] = acc;
}

__global__ void k_diag(const double* __restrict__ S, int M, double* __restrict__ d) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < M) d[i] = S[(size_t)i * M + i];
}

// scatter study-local Sigma~ into union coordinates
__global__ void k_to_union(const double* __restrict__ S, int M, const int* __restrict__ u2l, int U, int ldg,
                           double* __restrict__ G) {
    int v = blockIdx.x * blockDim.x + threadIdx.x;
    int u = blockIdx.y;
    if (v >= ldg) return;
    double val = 0.0;
    if (u < U && v < U) {
        int lu = u2l[u], lv = u2l[v];
        if (lu >= 0 && lv >= 0) val = S[(size_t)lu * M + lv];
    }
    G[(size_t)u * ldg + v] = val;
}

// ---------------------------------------------------------------------------
// Generic evaluator: one wave per union set (any k <= PSX_KMAX).  Lanes first
// factor the 2^k per-study subsets (LDL^T), then stride over the 3^k study
// assignments (x_j in {1: study0 only, 2: study1 only, 3: both}), i.e. exactly
// the masks of postcal.cpp:907-955 that pass checkOR.  Used for SSS neighbour
// batches, the -b configs path, levels the tiled sweep does not cover.
// forced[set] = (C0 mask, C1 mask) restricts a set to one pattern (configs rows).
// ---------------------------------------------------------------------------
// Register-resident: the set's Sigma~ sub-blocks, Ad and y are gathered into
// LDS in one round trip; every loop runs over PSX_KMAX with `j < k` guards so
// the per-lane arrays stay in VGPRs (no scratch); members outside a lane's
// subset enter its LDL^T as zero rows, which leaves the in-subset arithmetic
// (and its rounding) exactly that of psx::ldlt_terms.
// One union set S (stride entries, -1 padded) by the calling wave: its set
// record (*so), its member records (mo[0 .. k), if mo) and its SSS score (*sc,
// if sc); fpair = (C0 mask, C1 mask) restricts the set to one pattern.
// the 3^KMAX assignments as (c0, c1) member masks: assignment p gives member j
// digit j of p (base 3): study 0 only / study 1 only / both (postcal.cpp:928-943's
// mask order restated); a set of k < KMAX members takes the first 3^k entries,
// masked to its k members
struct PatTab {
    unsigned short v[729];
};
constexpr PatTab make_pat() {
    PatTab t{};
    for (int p = 0; p < 729; p++) {
        int r = p, c0 = 0, c1 = 0;
        for (int j = 0; j < 6; j++) {
            const int x = r % 3 + 1;
            r /= 3;
            if (x & 1) c0 |= 1 << j;
            if (x & 2) c1 |= 1 << j;
        }
        t.v[p] = (unsigned short)(c0 | (c1 << 8));
    }
    return t;
}
static_assert(PSX_KMAX == 6, "the assignment table covers 3^6");
__constant__ PatTab kPat = make_pat();

// A set's operands (its members' Sigma~ sub-blocks, A_d, y and presence), staged
// in two halves so that a caller can put other loads between them
// (k_sss_eval's map probe): eval_gather issues the global loads into
// registers, eval_stage waits for them and writes LDS.
struct EvalShm {
    double g[2][PSX_KMAX][PSX_KMAX];
    double ad[2][PSX_KMAX], y[2][PSX_KMAX];
    double mu[2][64], f[2][64];
    int n[2][64];
    int mem[PSX_KMAX];
};
struct EvalOps {
    double g[2];     // this lane's (<= 2) lower-triangle Sigma~ entries: e = lane, lane + 64
    double ad, y;    // lanes < 2 KMAX: (study lane / KMAX, member lane % KMAX)
    unsigned pr;     // lanes < KMAX: presence bits of member lane
    int k;
};
__device__ __forceinline__ EvalOps eval_gather(const DevProb& P, const int* __restrict__ S, int stride,
                                               EvalShm& sh) {
    constexpr int KM = PSX_KMAX;
    const int lane = threadIdx.x;
    EvalOps o;
    int mem[KM];  // the members (S's non-negative entries, in order)
    int k = 0;
#pragma unroll
    for (int j = 0; j < KM; j++) {
        mem[j] = -1;
        const int v = j < stride ? S[j] : -1;
#pragma unroll
        for (int c = 0; c <= j; c++)
            if (v >= 0 && c == k) mem[c] = v;
        k += v >= 0;
    }
    o.k = k;
    // Every load below is unconditional (clamped indices, results selected
    // after) and every study pointer a select between the two kernel-argument
    // values: indexing P.G[s] with a per-lane s read the pointer from the
    // kernel arguments by a vector load, and each guarded load waited for the
    // one before — five dependent round trips per set instead of one (late r06)
    // (the kernel-argument pointers pinned in scalar registers: otherwise the
    // compiler folds the selects below back into a per-lane pointer load)
    const double *G0 = P.G[0], *G1 = P.G[1], *A0 = P.Ad[0], *A1 = P.Ad[1], *Y0 = P.y[0], *Y1 = P.y[1];
    const unsigned char* PR = P.pres;
    asm volatile("" : "+s"(G0), "+s"(G1), "+s"(A0), "+s"(A1), "+s"(Y0), "+s"(Y1), "+s"(PR));
    double gv[2];
    bool gok[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int e = lane + 64 * h;
        const int s = e / (KM * KM), i = (e / KM) % KM, j = e % KM;
        int mi = -1, mj = -1;
#pragma unroll
        for (int c = 0; c < KM; c++) {
            mi = c == i ? mem[c] : mi;
            mj = c == j ? mem[c] : mj;
        }
        gok[h] = e < 2 * KM * KM && i < k && j < i;
        const size_t off = gok[h] ? (size_t)mi * P.ldg + mj : 0;
        gv[h] = (s ? G1 : G0)[off];
    }
    {
        const int s = lane / KM, i = lane % KM;
        int mi = -1;
#pragma unroll
        for (int c = 0; c < KM; c++) mi = c == i ? mem[c] : mi;
        const bool ok = lane < 2 * KM && i < k;
        const bool okp = lane < KM && lane < k;
        const int ia = ok ? mi : 0, ip = okp ? mi : 0;
        const double av = (s ? A1 : A0)[ia];
        const double yv = (s ? Y1 : Y0)[ia];
        const unsigned pv = PR[ip];
        o.ad = ok ? av : 0.0;
        o.y = ok ? yv : 0.0;
        o.pr = okp ? pv : 0u;
        if (lane < KM) sh.mem[lane] = mi;
    }
#pragma unroll
    for (int h = 0; h < 2; h++) o.g[h] = gok[h] ? gv[h] : 0.0;
    return o;
}
__device__ __forceinline__ void eval_stage(const EvalOps& o, EvalShm& sh) {
    constexpr int KM = PSX_KMAX;
    const int lane = threadIdx.x;
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int e = lane + 64 * h;
        const int s = e / (KM * KM), i = (e / KM) % KM, j = e % KM;
        if (e < 2 * KM * KM && i < o.k && j < i) sh.g[s][i][j] = o.g[h];
    }
    if (lane < 2 * KM && lane % KM < o.k) {
        sh.ad[lane / KM][lane % KM] = o.ad;
        sh.y[lane / KM][lane % KM] = o.y;
    }
}

// the set's 2^k subset weights per study and its 3^k assignments (after
// eval_gather / eval_stage): set record, member records, score.  KM: the most
// members the caller's sets have (KM = 5 for batches of at most 5: fewer live
// registers in the unrolled factorisations and pattern sums)
template <int KM = PSX_KMAX>
__device__ void eval_compute(const DevProb& P, const EvalOps& o, EvalShm& shm, const int* __restrict__ fpair,
                             SetRec* __restrict__ so, Acc5* __restrict__ mo, double* __restrict__ sc,
                             unsigned long long* tr = nullptr) {
    static_assert(KM >= 1 && KM <= PSX_KMAX, "members per set");
    double (&s_g)[2][PSX_KMAX][PSX_KMAX] = shm.g;
    double (&s_ad)[2][PSX_KMAX] = shm.ad;
    double (&s_y)[2][PSX_KMAX] = shm.y;
    double (&s_mu)[2][64] = shm.mu;
    double (&s_f)[2][64] = shm.f;
    int (&s_n)[2][64] = shm.n;
    const int lane = threadIdx.x;
    const int k = o.k;
    int pmask[2];
    pmask[0] = (int)(__ballot(o.pr & 1u) & 0x3f);
    pmask[1] = (int)(__ballot(o.pr & 2u) & 0x3f);
    __syncthreads();
    const int nsub = 1 << k;
    // one (study, subset) per lane: 2^k subsets of both studies (one pass for
    // k <= 5, two for k = 6) — half the serial chain of a lane doing both studies
    for (int wk = lane; wk < 2 * nsub; wk += 64) {
        const int s = wk >> k, sub = wk & (nsub - 1);
        {
            double L[KM][KM], D[KM], Rd[KM], w[KM];
            double q = 0.0, Pd = 1.0;
            const double dv = s ? P.dval[1] : P.dval[0];
#pragma unroll
            for (int i = 0; i < KM; i++) {
                const bool in = i < k && ((sub >> i) & 1);
                double di = 1.0, wi = 0.0;
#pragma unroll
                for (int j = 0; j < i; j++) {
                    double acc = s_g[s][i][j];
#pragma unroll
                    for (int m = 0; m < j; m++) acc -= L[i][m] * L[j][m] * D[m];
                    // L[j][*] = 0 and D[j] = 1 for j outside the subset
                    L[i][j] = in && ((sub >> j) & 1) ? acc * Rd[j] : 0.0;
                }
                if (in) {
                    di = s_ad[s][i];
                    wi = s_y[s][i];
#pragma unroll
                    for (int m = 0; m < i; m++) {
                        di -= L[i][m] * L[i][m] * D[m];
                        wi -= L[i][m] * w[m];
                    }
                }
                // one division per pivot (ldlt_terms' rounding): the L entries
                // below it and the quadratic form multiply by its reciprocal
                Rd[i] = 1.0 / di;
                if (in) {
                    q += wi * wi * Rd[i];
                    Pd *= dv * di;
                }
                D[i] = di;
                w[i] = wi;
            }
            int n;
            double mu;
            psx::split_exp(0.5 * q * PSX_LOG2E, 1.0 / sqrt(Pd), n, mu);
            s_mu[s][sub] = mu;
            s_n[s][sub] = n;
            s_f[s][sub] = 0.5 * q - 0.5 * log(Pd);
        }
    }
    __syncthreads();
    if (tr) tr[3] = wall_clock64();
    const int S0 = pmask[0], S1 = pmask[1];
    const int Gll = s_n[0][S0] + s_n[1][S1] + 2;
    int GN[KM];
#pragma unroll
    for (int j = 0; j < KM; j++) {
        const int bj = 1 << j;
        const int g1 = s_n[0][S0] + s_n[1][S1 & ~bj];
        const int g2 = s_n[0][S0 & ~bj] + s_n[1][S1];
        GN[j] = psx::imax(g1, g2) + 2;
    }
    const int Ck = P.Ck[k];
    const int GS = Gll + Ck;
    int npat = 1;
    for (int j = 0; j < k; j++) npat *= 3;
    int fc0 = -1, fc1 = -1;
    if (fpair) {
        fc0 = fpair[0];
        fc1 = fpair[1];
    }
    double pit[KM + 1], pri[KM + 1];
#pragma unroll
    for (int j = 0; j <= KM; j++) {
        pit[j] = P.pit[k][j];
        pri[j] = P.prior[k][j];
    }
    double tot = 0, nc0 = 0, nc1 = 0, smin = 1e300, npatv = 0;
    // noCausal[s] terms live on their own shifts (C_s empty => the other study is full)
    const int Gnc0 = s_n[1][S1] + Ck, Gnc1 = s_n[0][S0] + Ck;
    double p0[KM], p1[KM], sh[KM], sl[KM], ns[KM];
#pragma unroll
    for (int j = 0; j < KM; j++) p0[j] = p1[j] = sh[j] = sl[j] = ns[j] = 0.0;
    const int full = (1 << k) - 1;
    for (int p = lane; p < npat; p += 64) {
        const unsigned pt = kPat.v[p];
        const int c0 = (int)(pt & 0xffu) & full, c1 = (int)(pt >> 8) & full;
        int x[KM];
#pragma unroll
        for (int j = 0; j < KM; j++) x[j] = ((c0 >> j) & 1) | (((c1 >> j) & 1) << 1);
        if ((c0 & ~S0) || (c1 & ~S1)) continue;  // (study, SNP) pair not present: no mask bit
        if (fc0 >= 0 && (c0 != fc0 || c1 != fc1)) continue;
        const int nsh = __popc(c0 & c1);
        double pitv = pit[0], priv = pri[0];
#pragma unroll
        for (int j = 1; j <= KM; j++)
            if (nsh == j) { pitv = pit[j]; priv = pri[j]; }
        const double mup = s_mu[0][c0] * s_mu[1][c1];
        const int np = s_n[0][c0] + s_n[1][c1];
        const double wll = ldexp(mup, np - Gll);
        const double w = wll * pitv;
        npatv += 1.0;
        tot += w;
        // value = 2^{np} mup 2^{prior log2e}; pit carries 2^{-Ck}, the shift +Ck
        if (c0 == 0) nc0 += ldexp(mup * pit[0], np - (Gnc0 - Ck));
        if (c1 == 0) nc1 += ldexp(mup * pit[0], np - (Gnc1 - Ck));
        smin = fmin(smin, s_f[0][c0] + s_f[1][c1] + priv);
#pragma unroll
        for (int j = 0; j < KM; j++) {
            if (x[j] & 1) p0[j] += w;
            if (x[j] & 2) p1[j] += w;
            if (x[j] == 3) {
                sh[j] += w;
                sl[j] += wll;
            } else if (x[j]) {
                ns[j] += ldexp(mup, np - GN[j]);
            }
        }
    }
    if (tr) tr[4] = wall_clock64();
    // every sum in one transposed batch (~7 instructions per value instead of
    // six dependent LDS shuffles each); the score's minimum by DPP
    constexpr int RK = (4 + 5 * KM + 3) / 4 * 4;  // the reduction batch (a multiple of 4)
    double red[RK];
    red[0] = tot; red[1] = nc0; red[2] = nc1; red[3] = npatv;
#pragma unroll
    for (int j = 0; j < KM; j++) {
        red[4 + 5 * j] = p0[j]; red[5 + 5 * j] = p1[j]; red[6 + 5 * j] = sh[j];
        red[7 + 5 * j] = sl[j]; red[8 + 5 * j] = ns[j];
    }
#pragma unroll
    for (int i = 4 + 5 * KM; i < RK; i++) red[i] = 0.0;
    psx::wave_sum_t(red);
    tot = red[0]; nc0 = red[1]; nc1 = red[2]; npatv = red[3];
    smin = __ockl_wfred_min_f64(smin);
    if (tr) tr[5] = wall_clock64();
    double vp0 = 0, vp1 = 0, vsh = 0, vsl = 0, vns = 0;
#pragma unroll
    for (int j = 0; j < KM; j++)
        if (j == lane) {
            vp0 = red[4 + 5 * j]; vp1 = red[5 + 5 * j]; vsh = red[6 + 5 * j];
            vsl = red[7 + 5 * j]; vns = red[8 + 5 * j];
        }
    if (lane == 0) {
        SetRec rr = psx::set_zero();
        rr.m = GS;
        rr.m0 = Gnc0;
        rr.m1 = Gnc1;
        rr.tot = tot;
        rr.nc0 = nc0;
        rr.nc1 = nc1;
        rr.score = smin;
        rr.npat = npatv;
        *so = rr;
        if (sc) *sc = smin;
    }
    if (lane < k && mo) {
        Acc5 a;
        a.mP = GS;
        a.mS = Gll;
        a.mN = GN[0];
#pragma unroll
        for (int j = 1; j < KM; j++)
            if (j == lane) a.mN = GN[j];
        a.pad = 0;
        a.post0 = vp0;
        a.post1 = vp1;
        a.shared = vsh;
        a.sll = vsl;
        a.nsll = vns;
        mo[lane] = a;
    }
    if (tr) tr[6] = wall_clock64();
}


// one set (sorted members, -1 padded, in global or LDS memory): gather, stage, compute
template <int KM = PSX_KMAX>
__device__ void eval_set(const DevProb& P, const int* __restrict__ S, int stride, const int* __restrict__ fpair,
                         SetRec* __restrict__ so, Acc5* __restrict__ mo, double* __restrict__ sc) {
    __shared__ EvalShm shm;
    const EvalOps o = eval_gather(P, S, stride, shm);
    eval_stage(o, shm);
    eval_compute<KM>(P, o, shm, fpair, so, mo, sc);
}

// span (optional, device [lo, hi)): block b evaluates set lo + b of `sets`, the
// blocks past hi - lo exit (a batch whose size the device decided); outputs
// stay indexed by b
__global__ __launch_bounds__(64) void k_eval_sets(DevProb P, const int* __restrict__ sets, int stride,
                                                  const int* __restrict__ forced, SetRec* __restrict__ srec,
                                                  Acc5* __restrict__ mrec, double* __restrict__ score,
                                                  const int* __restrict__ span = nullptr) {
    const int set = blockIdx.x;
    int base = 0;
    if (span) {
        base = span[0];
        if (set >= span[1] - base) return;
    }
    eval_set(P, sets + (size_t)(base + set) * stride, stride, forced ? forced + 2 * set : nullptr, srec + set,
             mrec ? mrec + (size_t)set * stride : nullptr, score ? score + set : nullptr);
}

// A user batch (psx_eval_union_batch), one wave per row: the row is validated
// (its members, the non-negative entries, strictly ascending union indices;
// else *bad = badv and the row adds nothing: the merges then skip the whole
// batch and the host reports the error), compacted in place (record j of the
// set is its j-th member: the merges' keys) and evaluated.  A row without
// members is the null configuration (sss_postcal.cpp:463-499): set record
// null1, score L0 (the host adds K, as for every score).
// The rows are read from `in` and written compacted to `out` (device; may be the
// same rows); scores and the validity word go to pinned host memory (no readback
// copy), the word also to `bad` (device) for the merges.
template <int KM>
__device__ __forceinline__ void eval_batch_row(const DevProb& P, const int* in, int* out, int stride, SetRec null1,
                                               double L0, unsigned long long badv, unsigned long long* __restrict__ bad,
                                               unsigned long long* __restrict__ hbad, SetRec* __restrict__ srec,
                                               Acc5* __restrict__ mrec, double* __restrict__ score) {
    __shared__ int row[PSX_KMAX];
    const int set = blockIdx.x, lane = threadIdx.x;
    int* S = out + (size_t)set * stride;
    const int v = lane < stride ? in[(size_t)set * stride + lane] : -1;
    __builtin_amdgcn_wave_barrier();  // (in may alias out: every lane has read its entry)
    const unsigned long long m = __ballot(v >= 0);
    const unsigned long long below = m & ((1ull << lane) - 1ull);
    const int k = __popcll(m), pos = __popcll(below);
    const int pl = below ? 63 - __clzll(below) : 0;  // the previous member's lane
    const int pv = __shfl(v, pl);
    const bool bad_lane = v >= 0 && (v >= P.U || (below != 0ull && v <= pv));
    const bool ok = __ballot(bad_lane) == 0ull;
    if (lane < PSX_KMAX) row[lane] = -1;
    __builtin_amdgcn_wave_barrier();
    if (ok && v >= 0) row[pos] = v;
    __builtin_amdgcn_wave_barrier();
    if (lane < stride) S[lane] = row[lane];
    if (!ok || k == 0) {
        if (lane == 0) {
            if (!ok) {
                *bad = badv;
                *hbad = badv;
            }
            srec[set] = ok ? null1 : psx::set_zero();
            if (score) score[set] = ok ? L0 : 0.0;
        }
        return;
    }
    eval_set<KM>(P, row, stride, nullptr, srec + set, mrec + (size_t)set * stride, score ? score + set : nullptr);
}
// tstamp (optional, pinned host): block 0 stores its start clock (the batch's
// kernel time without dispatch events, see eval_generic_staged)
#define PSX_EVAL_BATCH_ARGS                                                                                   \
    DevProb P, const int *in, int *out, int stride, SetRec null1, double L0, unsigned long long badv,         \
        unsigned long long *__restrict__ bad, unsigned long long *__restrict__ hbad, SetRec *__restrict__ srec, \
        Acc5 *__restrict__ mrec, double *__restrict__ score, unsigned long long *__restrict__ tstamp
__global__ __launch_bounds__(64) void k_eval_batch(PSX_EVAL_BATCH_ARGS) {
    if (tstamp && blockIdx.x == 0 && threadIdx.x == 0) *tstamp = wall_clock64();
    eval_batch_row<PSX_KMAX>(P, in, out, stride, null1, L0, badv, bad, hbad, srec, mrec, score);
}
// rows of at most 5 members: 96 registers, 5 waves per SIMD (the 6-member
// instance needs 113: 4 waves)
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(5))) void k_eval_batch5(PSX_EVAL_BATCH_ARGS) {
    if (tstamp && blockIdx.x == 0 && threadIdx.x == 0) *tstamp = wall_clock64();
    eval_batch_row<5>(P, in, out, stride, null1, L0, badv, bad, hbad, srec, mrec, score);
}

// n ints out of pinned host memory (the staging buffer) into device memory,
// 16 bytes a lane, the last lane the tail: an SDMA copy instead costs a ~16 us
// engine hand-off before the next launch on the stream (r06t)
__global__ __launch_bounds__(256) void k_stage_rows(const int* __restrict__ src, size_t n, int* __restrict__ dst) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x, n4 = n / 4;
    if (i < n4) {
        reinterpret_cast<int4*>(dst)[i] = reinterpret_cast<const int4*>(src)[i];
    } else if (i == n4) {
        for (size_t j = 4 * n4; j < n; j++) dst[j] = src[j];
    }
}
#undef PSX_EVAL_BATCH_ARGS

// One lane copies the status block (SetRec, PlanTag, status words: kStatBytes
// from the scalars' slot) and the robust-redo count to pinned host memory, so
// psx_sync needs no read-out launch after the merges that end a pass or an
// exchange (k_merge_fin, k_merge_partials).  The lane wrote the scalars and the
// flag words itself; the rest comes from earlier launches.
__device__ void status_to_host(const int* stat, const int* redo, int* host) {
    // 16-byte pieces (the block is 8-byte aligned: pairs of 8-byte words) —
    // each store to host memory is a fabric write the kernel's end waits for
    constexpr int nq = (int)(kStatBytes / 8);
    static_assert(kStatBytes % 8 == 0, "status block of 8-byte words");
    // the lane's own stores to the block (scalars, flag words; through other
    // pointers of the caller) complete before it reads the block back: no
    // compiler reordering across the volatile loads, no load passing the stores
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0);
    const volatile unsigned long long* vs = reinterpret_cast<const volatile unsigned long long*>(stat);
    unsigned long long w[nq + 1];
#pragma unroll
    for (int i = 0; i < nq; i++) w[i] = vs[i];
    w[nq] = (unsigned long long)(unsigned)(redo ? *redo : 0);
    unsigned long long* h = reinterpret_cast<unsigned long long*>(host);
#pragma unroll
    for (int i = 0; i + 1 <= nq; i += 2) {
        if (i + 1 <= nq) {
            ulonglong2 v;
            v.x = w[i];
            v.y = w[i + 1];
            *reinterpret_cast<ulonglong2*>(h + i) = v;  // (hstat: pinned, 64-byte aligned)
        }
    }
    if ((nq + 1) % 2) h[nq] = w[nq];
}

// merge `count` concatenated partial images (rank order) into acc / sacc.
// Image layout: Acc5[ldg] followed by one Acc5-sized slot holding the SetRec
// and one holding the PlanTag.  The images must be shards 0 .. count - 1 of one
// plan: every thread checks the tags first (the same few lines for all), and
// when they disagree nothing is written — the accumulators keep their values —
// and status word kPlanMismatchWord is raised (psx_sync / psx_merge_partials
// report and clear it).  Grid: (U + 63) / 64 per-SNP blocks + one scalar block.
__global__ __launch_bounds__(64) void k_merge_partials(const Acc5* __restrict__ parts, int U, int ldg, int count,
                                                       Acc5* __restrict__ acc, SetRec* sacc,
                                                       int* flag,  // (the status block: no restrict)
                                                       const int* __restrict__ redo, int* __restrict__ host) {
    const size_t stride = (size_t)ldg + 2;  // ldg Acc5, SetRec, PlanTag
    const int tid = threadIdx.x;
    const bool scal = blockIdx.x == gridDim.x - 1;
    const int u = blockIdx.x * 64 + tid;
    // the first eight images' entries of this SNP, issued before the tag check
    // (unconditional loads from clamped indices: conditional ones put a wait
    // after each image's load, one round trip per rank)
    const int uc = (!scal && u < U) ? u : 0;
    Acc5 x[8];
#pragma unroll
    for (int q = 0; q < 8; q++) x[q] = parts[(size_t)(q < count ? q : 0) * stride + uc];
    // the tags, one rank per lane, in parallel (late r06: a lane walking the
    // ranks' tags field by field was a chain of dependent scalar loads, ~1 us
    // per rank — most of the merge at world 8)
    const PlanTag* const tag0 = reinterpret_cast<const PlanTag*>(parts + ldg + 1);
    const unsigned long long h0 = tag0->hash;
    bool bad = false;
    for (int r0 = 0; r0 < count; r0 += 64) {
        const int r = r0 + tid;
        bool b = false;
        if (r < count) {
            const PlanTag t = *reinterpret_cast<const PlanTag*>(parts + (size_t)r * stride + ldg + 1);
            b = (t.magic != kPlanMagic) | (t.hash != h0) | (t.world != count) | (t.rank != r) | (t.U != U);
        }
        bad |= __ballot(b) != 0ull;
    }
    if (scal) {  // the scalars, in rank order on lane 0
        if (bad) {
            if (tid == 0) {
                flag[kPlanMismatchWord] = 1;
                if (host) status_to_host(reinterpret_cast<const int*>(sacc), redo, host);
            }
            return;
        }
        SetRec s = psx::set_zero();
        int f = 0;
        for (int r0 = 0; r0 < count; r0 += 64) {
            SetRec y0 = psx::set_zero();
            if (r0 + tid < count) y0 = *reinterpret_cast<const SetRec*>(parts + (size_t)(r0 + tid) * stride + ldg);
            const int m = min(64, count - r0);
            for (int q = 0; q < m; q++) {
                SetRec y;
                y.m = __shfl(y0.m, q); y.m0 = __shfl(y0.m0, q); y.m1 = __shfl(y0.m1, q); y.pad = __shfl(y0.pad, q);
                y.tot = __shfl(y0.tot, q); y.nc0 = __shfl(y0.nc0, q); y.nc1 = __shfl(y0.nc1, q);
                y.score = __shfl(y0.score, q); y.npat = __shfl(y0.npat, q);
                psx::fold_set(s, y);
                f |= y.pad;  // any rank's EXACT flag
            }
        }
        if (tid == 0) {
            s.pad = f;
            flag[1] |= f;
            *sacc = s;
            if (host) status_to_host(reinterpret_cast<const int*>(sacc), redo, host);
        }
        return;
    }
    if (u >= U) return;
    Acc5 a = {0, 0, 0, 0, 0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < 8; q++)
        if (q < count) psx::fold_acc(a, x[q]);
    for (int r0 = 8; r0 < count; r0 += 8) {  // eight image loads in flight, folded in rank order
#pragma unroll
        for (int q = 0; q < 8; q++) x[q] = parts[(size_t)(r0 + q < count ? r0 + q : r0) * stride + u];
#pragma unroll
        for (int q = 0; q < 8; q++)
            if (r0 + q < count) psx::fold_acc(a, x[q]);
    }
    if (!bad) acc[u] = a;
}

// the partial image (ldg + 2 slots) to a caller's buffer, 16 bytes per thread
__global__ __launch_bounds__(256) void k_copy_image(const int4* __restrict__ src, size_t n16, int4* __restrict__ dst) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n16) dst[i] = src[i];
}

// psx_sync's status read-out: the status block (SetRec, PlanTag, status words)
// and the robust-redo count straight to pinned host memory, then the words the
// host consumes are re-armed (sticky EXACT flag, plan mismatch).  One launch in
// place of two copies and a memset.
__global__ __launch_bounds__(64) void k_status_out(int* __restrict__ stat, const int* __restrict__ redo,
                                                   int* __restrict__ host) {
    constexpr int nw = (int)(kStatBytes / sizeof(int));
    const int i = threadIdx.x;
    if (i < nw) {
        host[i] = stat[i];
        constexpr int base = 2 * (int)(sizeof(SetRec) / sizeof(int));  // status words after SetRec + PlanTag
        if (i == base + 1 || i == base + kPlanMismatchWord) stat[i] = 0;
    }
    if (i == nw) host[nw] = redo ? *redo : 0;
}

// Level 1 for one union SNP u, per thread: k_eval_sets with k = 1 written out
// (subsets {} and {u} per study; assignments x in {study0, study1, both}
// filtered by presence, postcal.cpp:907-955), same arithmetic and fold order.
__device__ void eval_single(const DevProb& P, int u, Acc5& a, SetRec& r) {
    const unsigned pr = P.pres[u];
    const int S0 = pr & 1u, S1 = (pr >> 1) & 1u;
    double mu[2][2], f[2][2];
    int n[2][2];
    for (int s = 0; s < 2; s++) {
        mu[s][0] = 1.0;
        n[s][0] = 0;
        f[s][0] = 0.0;
        double q, Pd;
        psx::ldlt_terms(P.G[s], P.ldg, P.Ad[s], P.y[s], P.dval[s], &u, 1, q, Pd);
        psx::split_exp(0.5 * q * PSX_LOG2E, 1.0 / sqrt(Pd), n[s][1], mu[s][1]);
        f[s][1] = 0.5 * q - 0.5 * log(Pd);
    }
    const int Ck = P.Ck[1];
    const int Gll = n[0][S0] + n[1][S1] + 2;
    const int GN = psx::imax(n[0][S0] + n[1][0], n[0][0] + n[1][S1]) + 2;
    const int GS = Gll + Ck;
    const int Gnc0 = n[1][S1] + Ck, Gnc1 = n[0][S0] + Ck;
    double tot = 0, nc0 = 0, nc1 = 0, smin = 1e300, npat = 0;
    double p0 = 0, p1 = 0, sh = 0, sl = 0, ns = 0;
    for (int x = 1; x <= 3; x++) {
        const int c0 = x & 1, c1 = (x >> 1) & 1;
        if ((c0 & ~S0) || (c1 & ~S1)) continue;
        const int nsh = c0 & c1;
        const double mup = mu[0][c0] * mu[1][c1];
        const int np = n[0][c0] + n[1][c1];
        const double wll = ldexp(mup, np - Gll);
        const double w = wll * P.pit[1][nsh];
        npat += 1.0;
        tot += w;
        if (c0 == 0) nc0 += ldexp(mup * P.pit[1][0], np - (Gnc0 - Ck));
        if (c1 == 0) nc1 += ldexp(mup * P.pit[1][0], np - (Gnc1 - Ck));
        smin = fmin(smin, f[0][c0] + f[1][c1] + P.prior[1][nsh]);
        if (x & 1) p0 += w;
        if (x & 2) p1 += w;
        if (x == 3) {
            sh += w;
            sl += wll;
        } else {
            ns += ldexp(mup, np - GN);
        }
    }
    a.mP = GS; a.mS = Gll; a.mN = GN; a.pad = 0;
    a.post0 = p0; a.post1 = p1; a.shared = sh; a.sll = sl; a.nsll = ns;
    r = psx::set_zero();
    r.m = GS; r.m0 = Gnc0; r.m1 = Gnc1;
    r.tot = tot; r.nc0 = nc0; r.nc1 = nc1; r.score = smin; r.npat = npat;
}

// The whole-pass merge of the fused exhaustive pass, with level 1 folded in,
// in two launches of one-wave blocks (r06; r01-r05 had one launch whose block
// 0 folded every scalar record in one wave: 86 us of a 0.84 ms single pass at
// world 1, 26 us of 0.23 ms at world 8, profiles/r06a_*):
//   k_merge_rec   blocks [0, nch):    scalar chunk c -> spart[c]: first the level-1
//                                     sets of this shard, 64 per chunk (one per
//                                     lane, late r06), then the unit records
//                                     srec[0, nsrec), kScalChunk per chunk
//                 block nch + V u + v: slice v of V of SNP u's record run (level A
//                                     then level B, dense per-SNP runs) -> apart[V u + v]
//   k_merge_fin   block 0:            scalars = extra (null configuration), then
//                                     spart in chunk order (one wave, fixed tree)
//                 blocks 1..:         thread u: acc[u] = level-1 record of u (if in
//                                     this shard), then apart[V u .. V u + V) in order
// One-wave blocks throughout: a pipelined pass's merge runs beside the next
// sweep, whose one-wave blocks hold every wave slot, and takes the first slot
// any sweep block frees (a wider block waits for several free slots on one CU
// at once and was starved for the whole sweep, r02).  V (slices per SNP) is a
// function of the plan only, and every pass runs the same two launches, so
// synchronous, pipelined and single passes give bitwise-identical results.
// Fixed fold order: deterministic.
constexpr int kScalChunk = 512;   // scalar items per chunk wave (8 per lane)
constexpr int kMergeWaysMax = 8;  // slices per SNP run
constexpr int kMergeDepth = 8;    // record loads in flight per lane

__global__ __launch_bounds__(64) void k_merge_rec(DevProb P, int lo, int nsingle, const Acc5* __restrict__ recA,
                                                  const int* __restrict__ dptrA, const int* __restrict__ gidxA,
                                                  const Acc5* __restrict__ recB, const int* __restrict__ dptrB,
                                                  const int* __restrict__ gidxB, const SetRec* __restrict__ srec,
                                                  long nsrec, int nch, int V, SetRec* __restrict__ spart,
                                                  Acc5* __restrict__ apart, unsigned long long* __restrict__ ts) {
    constexpr int T = 64;
    const int tid = threadIdx.x;
    const int b = blockIdx.x;
    if (ts && b == 0 && tid == 0) ts[1] = wall_clock64();  // a single pass: the sweep's end (its start: ts[0])
    const int nchs = (nsingle + T - 1) / T;  // level-1 chunks: one set per lane
    if (b < nchs) {
        // the level-1 sets of this shard, one per lane (eval_single is a chain of
        // divisions and transcendentals: eight of them in series per lane held
        // the whole merge up at world 1, late r06)
        const int i = b * T + tid;
        SetRec a = psx::set_zero();
        if (i < nsingle) {
            Acc5 dummy;
            eval_single(P, lo + i, dummy, a);
        }
        psx::wave_fold_set(a);
        if (tid == 0) spart[b] = a;
        return;
    }
    if (b < nch) {  // the unit set records, kScalChunk per chunk
        const long i0 = (long)(b - nchs) * kScalChunk + tid;
        SetRec r[kScalChunk / T];
        // unconditional loads from clamped indices (a conditional load put a
        // wait after each one: eight round trips in series per lane), then the
        // records past the end replaced by zero records
#pragma unroll
        for (int q = 0; q < kScalChunk / T; q++) {
            const long i = i0 + (long)q * T;
            r[q] = srec[i < nsrec ? i : nsrec - 1];
        }
#pragma unroll
        for (int q = 0; q < kScalChunk / T; q++)
            if (i0 + (long)q * T >= nsrec) r[q] = psx::set_zero();
        SetRec a = psx::set_zero();
#pragma unroll
        for (int q = 0; q < kScalChunk / T; q++) psx::fold_set(a, r[q]);
        psx::wave_fold_set(a);
        if (tid == 0) spart[b] = a;
        return;
    }
    const int item = b - nch;
    const int u = item / V, v = item - u * V;
    if (u >= P.U) return;
    const int a0 = dptrA ? dptrA[u] : 0, na = dptrA ? dptrA[u + 1] - a0 : 0;
    const int b0 = dptrB ? dptrB[u] : 0, nb = dptrB ? dptrB[u + 1] - b0 : 0;
    const int n = na + nb;
    const int j0 = (int)((long)n * v / V), j1 = (int)((long)n * (v + 1) / V);
    Acc5 a = psx::acc_zero();
    // each lane folds its records in record order, kMergeDepth loads in flight
    // (their gather indices loaded one round ahead)
    constexpr int D = kMergeDepth;
    auto gidx_of = [&](int j) {
        return j < na ? (gidxA ? gidxA[a0 + j] : a0 + j) : (gidxB ? gidxB[b0 + j - na] : b0 + j - na);
    };
    int g[D];
#pragma unroll
    for (int q = 0; q < D; q++) {
        const int j = j0 + tid + q * T;
        g[q] = j < j1 ? gidx_of(j) : 0;
    }
    for (int i = j0 + tid; i < j1; i += D * T) {
        Acc5 x[D];
#pragma unroll
        for (int q = 0; q < D; q++) {
            const int j = i + q * T;
            if (j < j1) x[q] = j < na ? recA[g[q]] : recB[g[q]];
        }
#pragma unroll
        for (int q = 0; q < D; q++) {
            const int j = i + (D + q) * T;
            g[q] = j < j1 ? gidx_of(j) : 0;
        }
#pragma unroll
        for (int q = 0; q < D; q++)
            if (i + q * T < j1) psx::fold_acc(a, x[q]);
    }
    psx::wave_fold_acc(a);
    if (tid == 0) apart[item] = a;
}

__global__ __launch_bounds__(64) void k_merge_fin(DevProb P, int lo, int hi, int nch, int V,
                                                  const SetRec* __restrict__ spart, const Acc5* __restrict__ apart,
                                                  SetRec extra, Acc5* __restrict__ acc, SetRec* sacc,
                                                  int* flag, int* sticky,  // (the status block: no restrict)
                                                  const int* __restrict__ redo, int* __restrict__ host,
                                                  const unsigned long long* __restrict__ ts,
                                                  unsigned long long* __restrict__ hts) {
    const int tid = threadIdx.x;
    if (blockIdx.x == 0) {
        if (ts && tid < 2) hts[tid] = ts[tid];  // the pass's clock stamps (earlier launches) to the host
        SetRec a = psx::set_zero();
        for (int c = tid; c < nch; c += 64) psx::fold_set(a, spart[c]);
        psx::wave_fold_set(a);
        if (tid == 0) {
            SetRec g = psx::set_zero();
            psx::fold_set(g, extra);
            psx::fold_set(g, a);
            // hand the pass's EXACT flag to the host in the status record and re-arm
            // it for the next pass (the kernels that raise it have completed)
            // (atomic exchange: with pipelined passes the next pass's sweep may
            // already be raising its own flag word; the sticky word collects all)
            g.pad = atomicExch(flag, 0);
            atomicOr(sticky, g.pad);  // sticky copy for asynchronous passes (psx_sync)
            *sacc = g;
            if (host) status_to_host(reinterpret_cast<const int*>(sacc), redo, host);
        }
        return;
    }
    const int u = (blockIdx.x - 1) * 64 + tid;
    if (u >= P.U) return;
    Acc5 x[kMergeWaysMax];
#pragma unroll
    for (int v = 0; v < kMergeWaysMax; v++)
        if (v < V) x[v] = apart[(size_t)u * V + v];
    Acc5 g = {0, 0, 0, 0, 0.0, 0.0, 0.0, 0.0, 0.0};
    if (u >= lo && u < hi) {
        SetRec dummy;
        eval_single(P, u, g, dummy);
    }
#pragma unroll
    for (int v = 0; v < kMergeWaysMax; v++)
        if (v < V) psx::fold_acc(g, x[v]);
    acc[u] = g;
}

}  // namespace

namespace {
struct SssDev;                 // the SSS walk's workspace (kept across walks)
void sss_release(SssDev* d);
}  // namespace

// ===========================================================================
// Host engine
// ===========================================================================
struct psx_engine {
    int dev = 0;
    hipStream_t stream = nullptr;
    hipStream_t own_stream = nullptr;  // from the stream pool (psx_create)
    int own_pr = 0;                    // its priority (pool key)
    bool external_stream = false;      // psx_set_stream: caller orders export/merge
    int S = 2;
    int m[2] = {0, 0};
    int N = 0, U = 0, ldg = 0, maxc = 0;
    int rank = 0, world = 1;
    std::vector<int> u2l;     // [2][U]
    std::vector<unsigned char> pres;
    double K = 0;             // -||S'||^2/2
    double L0 = 0;            // null configuration L' (K excluded), postcal.cpp:797-803
    double dval[2] = {0, 0};
    DevProb dp;
    // device buffers
    double* dG[2] = {nullptr, nullptr};
    double* dAd[2] = {nullptr, nullptr};
    double* dy[2] = {nullptr, nullptr};
    unsigned char* dpres = nullptr;
    // accumulator image, one allocation of ldg + 3 slots: per-SNP Acc5[ldg], then
    // the SetRec scalars (slot ldg), the PlanTag (slot ldg + 1), then the status
    // words (slot ldg + 2: [0] EXACT flag, [1] its sticky copy, [2..3] the other
    // record buffers' flags, [8] plan mismatch); the first ldg + 2 slots are the
    // exported partial image
    Acc5* dacc = nullptr;
    SetRec* dsacc = nullptr;   // = slot ldg
    PlanTag* dtag = nullptr;   // = slot ldg + 1
    int* dflag = nullptr;      // = slot ldg + 2
    unsigned char* hstat = nullptr;  // pinned host copy of the status block
    // fused exhaustive pass: every unit set record of the pass in one buffer
    SetRec* dpass = nullptr;
    size_t cap_pass = 0;
    // the pass merge's partials: per scalar chunk, per (SNP, slice)
    SetRec* dspart = nullptr;
    size_t cap_spart = 0;
    Acc5* dapart = nullptr;
    size_t cap_apart = 0;
    // sweep workspace (tiled kernel)
    psx::SweepPlanCache plans;
    // generic workspace
    // the sets of one batch, uploaded with one copy from pinned staging; their
    // member records' CSR (dptr[U + 1] | gidx), built on the device
    int* dgen = nullptr;
    size_t cap_gen = 0;
    int* dgcsr = nullptr;
    size_t cap_gcsr = 0;
    psx::PlanScratch gscratch;
    unsigned char* dbm = nullptr;  // chunked batch merge scratch (psx::launch_merge_batch)
    size_t cap_bm = 0;
    uint32_t batch_seq = 0;        // user batches so far (their validity words)
    int* hstage = nullptr;
    size_t cap_stage = 0;
    hipEvent_t stage_ev = nullptr;  // last upload out of hstage (reuse waits on it)
    unsigned long long* hbclk = nullptr;  // [2] pinned coherent: a user batch's kernel clocks
    bool stage_rec = false;
    bool stage_open = false;  // an upload out of hstage is enqueued, its event not yet
    double* dscore = nullptr;       // per-set scores (SSS), read back compactly
    size_t cap_score = 0;
    double* hscore = nullptr;
    size_t cap_hscore = 0;
    SetRec* dsrec = nullptr;
    size_t cap_srec = 0;
    Acc5* dmrec = nullptr;
    size_t cap_mrec = 0;
    // cached generic exhaustive levels (level 1, levels > 3 when small): (k, rank, world)
    struct GenLevel {
        int* d_sets = nullptr;
        int* d_csr = nullptr;
        SetRec* d_srec = nullptr;
        Acc5* d_mrec = nullptr;
        size_t nsets = 0;
        int lo = 0;  // first set's rank in lexicographic order
        int ptr_len = 0, idx_len = 0, n_rows = 0;
        hipEvent_t ev[2] = {nullptr, nullptr};
        bool ran = false;
    };
    std::map<std::tuple<int, int, int>, GenLevel> glevels;
    // asynchronous passes (psx_run_exhaustive_async): ring of (start, end)
    // event pairs around the dominant kernel, consumed oldest-first
    static constexpr int kRing = 64;
    // pipelined asynchronous passes: sweeps on a compute stream, merges (and the
    // caller's exchange) on `stream`; record buffers alternate by pass parity
    hipStream_t cstream = nullptr;
    static constexpr int kCuMasked = 1 << 30;  // cstream_pr of a CU-masked (not pooled) stream
    int cstream_pr = 0;                        // its priority (stream pool key)
    // overlapped passes (PSX_OVERLAP = n reserved CUs): two compute streams
    // masked off n CUs, alternating, so pass i + 1's units fill pass i's drain;
    // the merges and the caller's exchange keep the reserved CUs
    hipStream_t cstream2 = nullptr;
    int ovl = -1;                     // reserved CUs (0: no overlap), read once
    int a_alt = 0;
    int a_first = -1;                 // ring slot of the first pass since the last sync (start: span0)
    hipEvent_t span0 = nullptr;       // start of that pass
    double a_span = 0;                // span0 to the last consumed pass's end (ms)

    static constexpr int kBufs = psx::kRecBufs;  // record buffer sets: sweep i waits for merge i - kBufs
    hipEvent_t mdone[kBufs] = {};
    bool mdone_rec[kBufs] = {};
    bool mdone_lazy[kBufs] = {};  // merge of a single pass on the engine stream, no event recorded
    // Passes whose sweep runs on the engine stream (a single pass — nothing in
    // flight at its call — or every pass under PSX_SERIAL): no dispatch events;
    // the sweep's first block and the merge's first block stamp their start
    // clocks into dstamps[slot], k_merge_fin copies the pair to hstamps[slot]
    // (pinned), psx_sync sums them
    int a_stamped = 0;
    double a_sspan = 0;  // the stamped passes' summed sweep time (their part of the span)
    unsigned long long* dstamps = nullptr;  // [kRing][2] device
    unsigned long long* hstamps = nullptr;  // [kRing][2] pinned host
    int wclk_khz = 100000;  // wall_clock64 rate (hipDeviceAttributeWallClockRate)
    // hstat holds the status of the last merge enqueued (k_merge_fin /
    // k_merge_partials write it to pinned host memory) and nothing that changes
    // the status was enqueued since: psx_sync needs no read-out launch
    bool stat_fresh = false;
    int a_par = kBufs - 1;
    hipEvent_t aev[2 * kRing] = {};
    int a_head = 0, a_pending = 0, a_count = 0;
    double a_kms = 0;
    // configs-file enumerator (psx_configs.hip): index maps on the device, workspace
    int* d_cfg_maps = nullptr;  // l2u[N] | u2l[2 * U]
    psx::CfgWork cfg;
    // SSS walk workspace: the set map, per-item rows / marks and the pinned
    // host buffers, grown on demand and reused by the next walk
    SssDev* sss = nullptr;
    // timing
    hipEvent_t ev[4];
    psx_timing timing;
    double prep_ms = 0;  // host wall of the last run's plan / layout preparation
    uint64_t n_configs = 0;

    ~psx_engine();
};

psx_engine::~psx_engine() {
    hipSetDevice(dev);
    // one device synchronisation, then every block goes back to the pool as is
    hipDeviceSynchronize();
    psx::IdleScope idle;
    for (int s = 0; s < 2; s++) { psx::dfree(dG[s]); psx::dfree(dAd[s]); psx::dfree(dy[s]); }
    psx::dfree(dpres); psx::dfree(dacc);
    if (hstat) psx::hfree(hstat);
    if (stage_ev) { hipEventSynchronize(stage_ev); hipEventDestroy(stage_ev); }
    if (hstage) psx::hfree(hstage);
    if (hbclk) psx::hfree(hbclk);
    if (hscore) psx::hfree(hscore);
    psx::dfree(dgen); psx::dfree(dgcsr); psx::dfree(dbm); psx::dfree(gscratch.p); psx::dfree(dscore); psx::dfree(dsrec); psx::dfree(dmrec); psx::dfree(dpass); psx::dfree(dspart); psx::dfree(dapart); psx::dfree(dstamps);
    if (hstamps) psx::hfree(hstamps);
    psx::sweep_free(plans);
    psx::configs_free(cfg);
    psx::dfree(d_cfg_maps);
    sss_release(sss);
    for (auto& kv : glevels) {
        GenLevel& g = kv.second;
        psx::dfree(g.d_sets); psx::dfree(g.d_csr); psx::dfree(g.d_srec); psx::dfree(g.d_mrec);
        for (int i = 0; i < 2; i++) if (g.ev[i]) hipEventDestroy(g.ev[i]);
    }
    for (int i = 0; i < 4; i++) hipEventDestroy(ev[i]);
    for (int i = 0; i < 2 * kRing; i++) if (aev[i]) hipEventDestroy(aev[i]);
    if (span0) hipEventDestroy(span0);
    for (int i = 0; i < kBufs; i++)
        if (mdone[i]) hipEventDestroy(mdone[i]);
    if (cstream2) { hipStreamSynchronize(cstream2); hipStreamDestroy(cstream2); }
    if (cstream && cstream_pr == kCuMasked) {
        hipStreamSynchronize(cstream);
        hipStreamDestroy(cstream);
    } else if (cstream) {
        psx::stream_put(cstream, cstream_pr);
    }
    if (own_stream) psx::stream_put(own_stream, own_pr);
}

namespace {

template <typename T>
int ensure(T*& p, size_t& cap, size_t n) {
    if (n <= cap) return 0;
    psx::dfree(p);
    p = nullptr;
    size_t nc = std::max(n, cap * 2);
    HIPCHK(psx::dmalloc(&p, nc * sizeof(T)));
    cap = nc;
    return 0;
}

// pinned host buffer of at least n elements (contents not preserved)
template <typename T>
int ensure_host(T*& p, size_t& cap, size_t n) {
    if (n <= cap) return 0;
    const size_t nc = std::max(n, cap * 2);
    if (p) psx::hfree(p);
    p = nullptr;
    cap = 0;
    HIPCHK(psx::hmalloc(reinterpret_cast<void**>(&p), nc * sizeof(T)));
    cap = nc;
    return 0;
}

double logval(const psx_engine* e, int32_t m, double s) {
    if (!(s > 0)) return 0.0;  // reference "empty" sentinel
    return e->K + ((double)m + std::log2(s)) * PSX_LN2;
}

// prior(k, nsh) in nats exactly as postcal.cpp:19-59 accumulates it
double prior_nats(const psx_problem* p, int U, int k, int nsh) {
    double pc = 0;
    if (p->sharing_param != 0) pc += nsh * std::log(p->sharing_param) + (k - nsh) * std::log((1 - p->sharing_param) * 0.5);
    pc += k * std::log(p->gamma);
    pc += (U - k) * std::log(1 - p->gamma);
    return pc;
}

// Build a CSR (SNP -> record indices) for records laid out as [set][stride]
// with member SNPs `sets`; records in set order, so folds are deterministic.
void build_csr(const std::vector<int>& sets, int stride, size_t nsets, int U, std::vector<int>& ptr,
               std::vector<int>& idx, std::vector<int>& rows) {
    std::vector<int> cnt(U + 1, 0);
    for (size_t i = 0; i < nsets * stride; i++)
        if (sets[i] >= 0) cnt[sets[i]]++;
    rows.clear();
    ptr.assign(1, 0);
    std::vector<int> start(U, -1);
    int acc = 0;
    for (int u = 0; u < U; u++)
        if (cnt[u]) {
            start[u] = acc;
            rows.push_back(u);
            acc += cnt[u];
            ptr.push_back(acc);
        }
    idx.assign(acc, 0);
    std::vector<int> fill(U, 0);
    for (size_t i = 0; i < nsets * stride; i++) {
        int u = sets[i];
        if (u >= 0) idx[start[u] + fill[u]++] = (int)i;
    }
}

// The pinned staging buffer, n ints, once its previous upload is done.
int stage_acquire(psx_engine* e, size_t n, int** out) {
    if (e->stage_open) {
        HIPCHK(hipStreamSynchronize(e->stream));  // (an upload whose call failed before its event)
        e->stage_open = false;
    } else if (e->stage_rec) {
        HIPCHK(hipEventSynchronize(e->stage_ev));
    }
    int rc = ensure_host(e->hstage, e->cap_stage, n);
    if (rc) return rc;
    *out = e->hstage;
    return 0;
}

// Evaluate nsets union sets staged in e->hstage ([set][stride], members first,
// -1 after them) with the generic kernel: one upload, k_eval_sets, then
// (accumulate) the deterministic merges of its member and set records; scores
// (SSS) copied back.  Batches of up to kBatchChunks chunks (an SSS
// neighbourhood) merge in two launches (psx::launch_merge_batch); larger ones
// (generic exhaustive levels) through the records' CSR, built by a device radix
// sort (psx::csr_from_keys_device).
constexpr int kBatchChunks = 256;  // psx::k_batch_fold's limit
SetRec null_rec(const psx_engine* e, double count);

// user = true: a psx_eval_union_batch slice (rows validated, compacted and
// null rows handled on the device by k_eval_batch; at most kBatchChunks merge
// chunks); false: internal sets (canonical rows, k_eval_sets).
int eval_generic_staged(psx_engine* e, int stride, size_t nsets, bool accumulate, double* scores, double* kernel_ms,
                        bool user = false) {
    if (nsets == 0) return 0;
    if (stride > PSX_KMAX) return fail(PSX_ERANGE, "union set larger than PSX_KMAX");
    int rc;
    const size_t n_sets = nsets * stride;
    const bool chunked = accumulate && psx::batch_merge_chunks((long)nsets, stride) <= kBatchChunks && e->U <= 131072;
    // the batch's validity word: after the scores (user batches), a 64-bit
    // pattern unique to this call
    const unsigned long long badv = ((unsigned long long)(++e->batch_seq) << 32) | 0xBADBA7C4ull;
    if ((rc = ensure(e->dgen, e->cap_gen, n_sets))) return rc;
    if ((rc = ensure(e->dsrec, e->cap_srec, nsets))) return rc;
    if ((rc = ensure(e->dmrec, e->cap_mrec, n_sets))) return rc;
    if (!user && scores && (rc = ensure(e->dscore, e->cap_score, nsets))) return rc;
    if (user && (rc = ensure_host(e->hscore, e->cap_hscore, nsets + 1))) return rc;
    // (user batches) the validity word: device status slot words 10-11 for the
    // merges, pinned hscore[nsets] for the host
    unsigned long long* dbad = user ? reinterpret_cast<unsigned long long*>(e->dflag + 10) : nullptr;
    if (chunked && (rc = ensure(e->dbm, e->cap_bm, psx::batch_merge_bytes((long)nsets, stride, e->U)))) return rc;
    if (accumulate && !chunked && (rc = ensure(e->dgcsr, e->cap_gcsr, (size_t)e->U + 1 + n_sets))) return rc;
    // the rows: one upload out of the pinned staging buffer, by a copy kernel on
    // the stream (a kernel reading them from host memory in the evaluation
    // itself measured 36 -> 55 us, r05w)
    hipLaunchKernelGGL(k_stage_rows, dim3((unsigned)((n_sets / 4 + 1 + 255) / 256)), dim3(256), 0, e->stream,
                       e->hstage, n_sets, e->dgen);
    e->stage_open = true;
    HIPCHK(hipGetLastError());
    // the kernel time of a user batch merged in chunks: in-kernel clocks (the
    // evaluation's first block start -> the chunk merge's first block start,
    // pinned host), no timing events around the launch (each costs a ~5 us gap)
    const bool clocks = kernel_ms && user && chunked;
    if (clocks && !e->hbclk) HIPCHK(psx::hmalloc_coherent_raw(reinterpret_cast<void**>(&e->hbclk), 64));
    unsigned long long* const bclk = clocks ? e->hbclk : nullptr;
    if (bclk) bclk[0] = bclk[1] = 0;
    if (kernel_ms && !clocks) HIPCHK(hipEventRecord(e->ev[2], e->stream));
    if (user)  // (rows of at most 5 members: the 5-member instance, fewer live registers)
        hipLaunchKernelGGL(stride <= 5 ? k_eval_batch5 : k_eval_batch, dim3((unsigned)nsets), dim3(64), 0,
                           e->stream, e->dp, e->dgen, e->dgen, stride, null_rec(e, 1.0), e->L0, badv, dbad,
                           reinterpret_cast<unsigned long long*>(e->hscore + nsets), e->dsrec, e->dmrec,
                           scores ? e->hscore : nullptr, bclk);
    else
        hipLaunchKernelGGL(k_eval_sets, dim3((unsigned)nsets), dim3(64), 0, e->stream, e->dp, e->dgen, stride,
                           nullptr, e->dsrec, e->dmrec, scores ? e->dscore : nullptr);
    HIPCHK(hipGetLastError());
    if (kernel_ms && !clocks) HIPCHK(hipEventRecord(e->ev[3], e->stream));
    if (chunked) {
        if (psx::launch_merge_batch(e->dgen, stride, (long)nsets, e->U, e->dmrec, e->dsrec, e->dbm, e->dacc,
                                    e->dsacc, e->stream, dbad, badv, bclk ? bclk + 1 : nullptr))
            return fail(PSX_EHIP, "set-batch merge failed");
    } else if (accumulate) {
        if (user) {
            // (a user batch beyond the chunked merge, U > 131072: its validity is
            // known before the CSR merges are enqueued, which do not check it)
            HIPCHK(hipStreamSynchronize(e->stream));
            if (*reinterpret_cast<const unsigned long long*>(e->hscore + nsets) == badv)
                return fail(PSX_EINVAL, "sets must be ascending union indices");
        }
        int* dptr = e->dgcsr;
        int* gidx = e->dgcsr + e->U + 1;
        if (psx::csr_from_keys_device(e->dgen, (long)n_sets, e->U, dptr, gidx, e->gscratch, e->stream))
            return fail(PSX_EHIP, "device CSR of a set batch failed");
        if (psx::launch_merge_dptr(e->dmrec, dptr, gidx, e->U, e->dacc, e->stream))
            return fail(PSX_EHIP, psx::sweep_error());
        SetRec none = psx::set_zero();
        if (psx::launch_merge_sets(e->dsrec, (long)nsets, none, e->dsacc, e->stream))
            return fail(PSX_EHIP, psx::sweep_error());
    }
    // hstage's reuse waits for this event: recorded after the launches (one
    // between the copy and the evaluation costs a ~6 us gap, r06u)
    if (!e->stage_ev) HIPCHK(hipEventCreateWithFlags(&e->stage_ev, hipEventDisableTiming));
    HIPCHK(hipEventRecord(e->stage_ev, e->stream));
    e->stage_rec = true;
    e->stage_open = false;
    if (scores && !user) {
        if ((rc = ensure_host(e->hscore, e->cap_hscore, nsets))) return rc;
        HIPCHK(hipMemcpyAsync(e->hscore, e->dscore, nsets * sizeof(double), hipMemcpyDeviceToHost, e->stream));
    }
    if (!scores && !kernel_ms && !user) return 0;
    HIPCHK(hipStreamSynchronize(e->stream));
    if (user && *reinterpret_cast<const unsigned long long*>(e->hscore + nsets) == badv)
        return fail(PSX_EINVAL, "sets must be ascending union indices");
    if (scores)
        for (size_t i = 0; i < nsets; i++) scores[i] = e->K + e->hscore[i];
    if (clocks) {
        const unsigned long long t0 = bclk[0], t1 = bclk[1];
        *kernel_ms += t1 > t0 ? (double)(t1 - t0) / (double)e->wclk_khz : 0.0;
    } else if (kernel_ms) {
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, e->ev[2], e->ev[3]));
        *kernel_ms += ms;
    }
    return 0;
}

// `count` null configurations (postcal.cpp:793-822) as a set record
SetRec null_rec(const psx_engine* e, double count) {
    double h = e->L0 * PSX_LOG2E;
    double fl = std::floor(h);
    SetRec x = psx::set_zero();
    x.m = x.m0 = x.m1 = (int32_t)fl;
    x.score = e->L0;
    x.npat = count;
    double v = std::exp2(h - fl) * count;
    x.tot = x.nc0 = x.nc1 = v;
    return x;
}

// fold `count` null configurations into the scalars
int fold_null(psx_engine* e, double count) {
    if (count <= 0) return 0;
    if (psx::launch_merge_sets(nullptr, 0L, null_rec(e, count), e->dsacc, e->stream))
        return fail(PSX_EHIP, psx::sweep_error());
    return 0;
}

// lexicographic k-subset enumeration over [0, U)
long double choose_ld(int n, int k) {
    if (k < 0 || k > n) return 0;
    long double r = 1;
    for (int i = 1; i <= k; i++) r = r * (n - k + i) / i;
    return r;
}
uint64_t choose_u64(int n, int k) {
    if (k < 0 || k > n) return 0;
    unsigned __int128 r = 1;
    for (int i = 1; i <= k; i++) r = r * (unsigned)(n - k + i) / (unsigned)i;
    return (uint64_t)r;
}
void unrank_lex(uint64_t r, int U, int k, int* out) {
    int x = 0;
    for (int i = 0; i < k; i++) {
        for (;;) {
            uint64_t c = choose_u64(U - x - 1, k - i - 1);
            if (r < c) break;
            r -= c;
            x++;
        }
        out[i] = x++;
    }
}
bool next_lex(int* c, int U, int k) {
    int i = k - 1;
    while (i >= 0 && c[i] == U - k + i) i--;
    if (i < 0) return false;
    c[i]++;
    for (int j = i + 1; j < k; j++) c[j] = c[j - 1] + 1;
    return true;
}

// exhaustive level k through the generic evaluator, shard-restricted
int run_level_generic(psx_engine* e, int k, double* kms) {
    uint64_t total = choose_u64(e->U, k);
    uint64_t lo = total * (uint64_t)e->rank / e->world;
    uint64_t hi = total * (uint64_t)(e->rank + 1) / e->world;
    if (lo >= hi) return 0;
    const uint64_t CH = 1u << 20;
    std::vector<int> c(k);
    unrank_lex(lo, e->U, k, c.data());
    uint64_t r = lo;
    while (r < hi) {
        uint64_t n = std::min<uint64_t>(CH, hi - r);
        int* h = nullptr;
        int rc = stage_acquire(e, n * k, &h);
        if (rc) return rc;
        for (uint64_t i = 0; i < n; i++) {
            std::copy(c.begin(), c.end(), h + i * k);
            next_lex(c.data(), e->U, k);
        }
        if ((rc = eval_generic_staged(e, k, n, true, nullptr, kms))) return rc;
        r += n;
    }
    return 0;
}

// the shard plan every rank of a job must share (PlanTag.hash): the locus shape,
// c, the world size and the plan knobs / compiled plan constants
uint64_t plan_hash(const psx_engine* e) {
    uint64_t h = psx::plan_knobs_hash();
    auto mix = [&](const void* p, size_t n) {
        for (size_t i = 0; i < n; i++) h = (h ^ ((const unsigned char*)p)[i]) * 1099511628211ull;
    };
    const int v[4] = {e->U, e->ldg, e->maxc, e->world};
    mix(v, sizeof(v));
    mix(e->pres.data(), e->pres.size());
    return h;
}

int write_tag(psx_engine* e) {
    PlanTag t;
    std::memset(&t, 0, sizeof(t));
    t.magic = kPlanMagic;
    t.world = e->world;
    t.rank = e->rank;
    t.U = e->U;
    t.hash = plan_hash(e);
    HIPCHK(hipMemcpyAsync(e->dtag, &t, sizeof(t), hipMemcpyHostToDevice, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return 0;
}

// after a synchronous merge of partial images
// (reported once: the word is cleared; the refused merge wrote nothing)
int check_plan_mismatch(psx_engine* e) {
    HIPCHK(hipStreamSynchronize(e->stream));  // k_merge_partials wrote the status block to hstat
    const int* const words = reinterpret_cast<const int*>(e->hstat + 2 * sizeof(SetRec));
    if (words[kPlanMismatchWord]) {
        HIPCHK(hipMemsetAsync(e->dflag + kPlanMismatchWord, 0, sizeof(int), e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        e->stat_fresh = false;
        return fail(PSX_EINVAL, "merged partial images are not shards 0..world-1 of one plan "
                                "(ranks with different PSX_K3_* knobs, builds or shard settings); "
                                "nothing was merged");
    }
    return 0;
}

int reset_acc(psx_engine* e) {
    HIPCHK(hipMemsetAsync(e->dacc, 0, sizeof(Acc5) * e->ldg, e->stream));
    SetRec z = psx::set_zero();
    HIPCHK(hipMemcpyAsync(e->dsacc, &z, sizeof(SetRec), hipMemcpyHostToDevice, e->stream));
    return 0;
}


// Enqueue an exhaustive level through the generic evaluator with its sets and
// record CSR cached on the device (built once per (k, rank, world)).
int enqueue_generic_level(psx_engine* e, int k) {
    auto key = std::make_tuple(k, e->rank, e->world);
    auto it = e->glevels.find(key);
    if (it == e->glevels.end()) {
        psx_engine::GenLevel g;
        uint64_t total = choose_u64(e->U, k);
        uint64_t lo = total * (uint64_t)e->rank / e->world;
        uint64_t hi = total * (uint64_t)(e->rank + 1) / e->world;
        g.nsets = (size_t)(hi - lo);
        std::vector<int> sets(g.nsets * k);
        if (g.nsets) {
            std::vector<int> c(k);
            unrank_lex(lo, e->U, k, c.data());
            for (size_t i = 0; i < g.nsets; i++) {
                std::copy(c.begin(), c.end(), sets.begin() + i * k);
                next_lex(c.data(), e->U, k);
            }
        }
        std::vector<int> ptr, idx, rows;
        build_csr(sets, k, g.nsets, e->U, ptr, idx, rows);
        g.ptr_len = (int)ptr.size();
        g.idx_len = (int)idx.size();
        g.n_rows = (int)rows.size();
        std::vector<int> packed(ptr);
        packed.insert(packed.end(), idx.begin(), idx.end());
        packed.insert(packed.end(), rows.begin(), rows.end());
        if (g.nsets) {
            HIPCHK(psx::dmalloc(&g.d_sets, sizeof(int) * sets.size()));
            HIPCHK(hipMemcpy(g.d_sets, sets.data(), sizeof(int) * sets.size(), hipMemcpyHostToDevice));
            HIPCHK(psx::dmalloc(&g.d_csr, sizeof(int) * packed.size()));
            HIPCHK(hipMemcpy(g.d_csr, packed.data(), sizeof(int) * packed.size(), hipMemcpyHostToDevice));
            HIPCHK(psx::dmalloc(&g.d_srec, sizeof(SetRec) * g.nsets));
            HIPCHK(psx::dmalloc(&g.d_mrec, sizeof(Acc5) * g.nsets * k));
        }
        for (int i = 0; i < 2; i++) HIPCHK(hipEventCreate(&g.ev[i]));
        it = e->glevels.emplace(key, g).first;
    }
    psx_engine::GenLevel& g = it->second;
    g.ran = false;
    if (g.nsets == 0) return 0;
    HIPCHK(hipEventRecord(g.ev[0], e->stream));
    hipLaunchKernelGGL(k_eval_sets, dim3((unsigned)g.nsets), dim3(64), 0, e->stream, e->dp, g.d_sets, k,
                       (const int*)nullptr, g.d_srec, g.d_mrec, (double*)nullptr);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(g.ev[1], e->stream));
    if (psx::launch_merge_members(g.d_mrec, g.d_csr, g.d_csr + g.ptr_len, g.d_csr + g.ptr_len + g.idx_len,
                                  g.n_rows, e->dacc, e->stream))
        return fail(PSX_EHIP, psx::sweep_error());
    if (psx::launch_merge_sets(g.d_srec, (long)g.nsets, psx::set_zero(), e->dsacc, e->stream))
        return fail(PSX_EHIP, psx::sweep_error());
    g.ran = true;
    return 0;
}

// Level 1 of a pass: its member records ARE the initial per-SNP accumulators
// (set i of this shard is SNP lo + i), so they are written in place into the
// zeroed dacc; the set records initialise the scalars together with `extra`
// (the null configuration on rank 0) and the EXACT flag is cleared.
int get_level1(psx_engine* e, psx_engine::GenLevel** out) {
    auto key = std::make_tuple(1, e->rank, e->world);
    auto it = e->glevels.find(key);
    if (it == e->glevels.end()) {
        psx_engine::GenLevel g;
        uint64_t lo = (uint64_t)e->U * e->rank / e->world, hi = (uint64_t)e->U * (e->rank + 1) / e->world;
        g.lo = (int)lo;
        g.nsets = (size_t)(hi - lo);
        if (g.nsets) {
            std::vector<int> sets(g.nsets);
            for (size_t i = 0; i < g.nsets; i++) sets[i] = (int)(lo + i);
            HIPCHK(psx::dmalloc(&g.d_sets, sizeof(int) * g.nsets));
            HIPCHK(hipMemcpy(g.d_sets, sets.data(), sizeof(int) * g.nsets, hipMemcpyHostToDevice));
            HIPCHK(psx::dmalloc(&g.d_srec, sizeof(SetRec) * g.nsets));
        }
        for (int i = 0; i < 2; i++) HIPCHK(hipEventCreate(&g.ev[i]));
        it = e->glevels.emplace(key, g).first;
    }
    *out = &it->second;
    return 0;
}

int enqueue_level1(psx_engine* e, const SetRec& extra) {
    psx_engine::GenLevel* gp = nullptr;
    int rc = get_level1(e, &gp);
    if (rc) return rc;
    psx_engine::GenLevel& g = *gp;
    HIPCHK(hipEventRecord(g.ev[0], e->stream));
    if (g.nsets)
        hipLaunchKernelGGL(k_eval_sets, dim3((unsigned)g.nsets), dim3(64), 0, e->stream, e->dp, g.d_sets, 1,
                           (const int*)nullptr, g.d_srec, e->dacc + g.lo, (double*)nullptr);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(g.ev[1], e->stream));
    if (psx::launch_merge_sets(g.d_srec, (long)g.nsets, extra, e->dsacc, e->stream, true, e->dflag))
        return fail(PSX_EHIP, psx::sweep_error());
    g.ran = true;
    return 0;
}

// One exhaustive pass, everything enqueued on the engine stream; the status
// block (scalars + EXACT flag) comes back with one async copy and one sync.
int exhaustive_pass(psx_engine* e, bool exact, double* generic_ms) {
    int rc;
    HIPCHK(hipMemsetAsync(e->dacc, 0, sizeof(Acc5) * e->ldg, e->stream));
    HIPCHK(hipEventRecord(e->ev[0], e->stream));
    if ((rc = enqueue_level1(e, e->rank == 0 ? null_rec(e, 1.0) : psx::set_zero()))) return rc;
    double kms = 0;
    for (int k = 2; k <= e->maxc; k++) {
        if (psx::sweep_supports(k, e->U)) {
            psx::SweepArgs sa{e->dG[0], e->dG[1], e->dAd[0], e->dAd[1], e->dy[0], e->dy[1], e->dpres,
                              e->dval[0], e->dval[1], e->dp.Ck, &e->dp.pit[0][0], PSX_KMAX + 1};
            if (psx::sweep_level(e->plans, k, e->U, e->ldg, e->rank, e->world, e->stream, sa, e->dacc, e->dsacc,
                                 exact))
                return fail(PSX_EHIP, std::string("sweep level ") + std::to_string(k) + ": " + psx::sweep_error());
        } else if (choose_u64(e->U, k) / (uint64_t)e->world <= (4u << 20)) {
            if ((rc = enqueue_generic_level(e, k))) return rc;
        } else {
            if ((rc = run_level_generic(e, k, &kms))) return rc;  // very large generic level: chunked
        }
    }
    HIPCHK(hipEventRecord(e->ev[1], e->stream));
    HIPCHK(hipMemcpyAsync(e->hstat, e->dsacc, kStatBytes, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    for (int k = 1; k <= e->maxc; k++) {
        auto it = e->glevels.find(std::make_tuple(k, e->rank, e->world));
        if (it != e->glevels.end() && it->second.ran) {
            float ms = 0;
            HIPCHK(hipEventElapsedTime(&ms, it->second.ev[0], it->second.ev[1]));
            kms += ms;
        }
    }
    *generic_ms = kms;
    return 0;
}

psx::SweepArgs sweep_args(psx_engine* e) {
    return psx::SweepArgs{e->dG[0], e->dG[1], e->dAd[0], e->dAd[1], e->dy[0], e->dy[1], e->dpres,
                          e->dval[0], e->dval[1], e->dp.Ck, &e->dp.pit[0][0], PSX_KMAX + 1};
}

// The fused pass is the shape of every BASELINE config: c in {2, 3}, all
// levels >= 2 on the tiled sweep.
bool fused_eligible(const psx_engine* e) {
    return (e->maxc == 2 || e->maxc == 3) && psx::sweep_supports(2, e->U) && psx::sweep_supports(e->maxc, e->U);
}

// One exhaustive pass with the fast kernels and a single merge, four device
// operations on one stream:
//   zero image + flag | top level (k = c) | level 2 (c = 3) | merge (+ level 1) | status copy
// The dominant kernel is the second call the host makes, level 1 is computed
// inside the merge (it is one 1x1 factor per SNP), and all record folds (per
// SNP: level 1, then 2, then 3; scalars: null configuration, level-1 sets,
// every unit record) are one launch.  Deterministic: the fold order is fixed
// by the plans, not by scheduling.
// consume the oldest recorded asynchronous kernel interval
int consume_async(psx_engine* e) {
    const int r = ((e->a_head - e->a_pending) % psx_engine::kRing + psx_engine::kRing) % psx_engine::kRing;
    HIPCHK(hipEventSynchronize(e->aev[2 * r + 1]));
    float ms = 0, sp = 0;
    HIPCHK(hipEventElapsedTime(&ms, r == e->a_first ? e->span0 : e->aev[2 * r], e->aev[2 * r + 1]));
    HIPCHK(hipEventElapsedTime(&sp, e->span0, e->aev[2 * r + 1]));
    if (r == e->a_first) e->a_first = -2;  // consumed: later passes of this span use their own starts
    e->a_kms += ms;
    e->a_span = sp;
    e->a_count++;
    e->a_pending--;
    return 0;
}

// the stamped passes since the last take (their k_merge_fin completed): each
// sweep from its first block's start to the merge's first block's start
// (in-kernel wall clocks; the merge starts ~1 us after the sweep's end)
void take_stamps(psx_engine* e) {
    for (int i = 0; i < e->a_stamped; i++) {
        const unsigned long long t0 = e->hstamps[2 * i], t1 = e->hstamps[2 * i + 1];
        const double ms = t1 > t0 ? (double)(t1 - t0) / (double)e->wclk_khz : 0.0;
        e->a_kms += ms;
        e->a_sspan += ms;
        e->a_count++;
    }
    e->a_stamped = 0;
}

// Asynchronous passes are pipelined: pass i's sweep runs on the compute stream
// into the record buffers of parity i & 1 while the merge of pass i - 1 and the
// caller's exchange (export / collective / merge of partials) run on the engine
// stream.  Sweep i waits for merge i - 2 (same buffers), merge i for sweep i.
int fused_pass(psx_engine* e, int* flag, bool async = false) {
    const psx::SweepArgs sa = sweep_args(e);
    psx::SweepPlan* P2 = nullptr;
    psx::SweepPlan* P3 = nullptr;
    const auto tp = std::chrono::steady_clock::now();
    if (psx::sweep_prepare(e->plans, 2, e->U, e->ldg, e->rank, e->world, e->stream, sa, false, &P2) ||
        (e->maxc == 3 && psx::sweep_prepare(e->plans, 3, e->U, e->ldg, e->rank, e->world, e->stream, sa, false, &P3)))
        return fail(PSX_EHIP, std::string("sweep plan: ") + psx::sweep_error());
    e->prep_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp).count();
    psx::SweepPlan* top = P3 ? P3 : P2;
    psx::SweepPlan* low = P3 ? P2 : nullptr;
    const size_t nl = low ? (size_t)low->n_units : 0, nt = (size_t)top->n_units;
    const size_t npass = nl + nt + 1;
    int rc;
    if ((rc = ensure(e->dpass, e->cap_pass, psx_engine::kBufs * npass))) return rc;
    hipStream_t X = e->stream;  // merges (and the caller's exchange)
    hipStream_t S = X;          // sweeps
    int par = 0;
    if (async) {
        if (!e->cstream) {
            // reserved CUs for overlapped sweeps, decided at the handle's first
            // asynchronous pass (rebuilding the streams when a handle's world
            // changed was 20-25 % slower, r04u).  Default: one XCD's CUs (32 of
            // MI355X's 256) at world >= 8, none below; PSX_OVERLAP = n overrides.
            // Measured on one box, alternating rounds (profiles/r05zi_*, r05zj_*):
            // world 8 step 0.132 -> 0.112 ms with 32 (16 / 24 / 48 / 64: 0.12-0.127,
            // a whole XCD for the merges and the exchange is the sweet spot);
            // worlds 2 and 4 are 2-7 % slower with any reservation.
            int ncu = 0;
            HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, e->dev));
            const char* ovl_env = getenv("PSX_OVERLAP");
            e->ovl = ovl_env ? std::max(0, atoi(ovl_env)) : (e->world >= 8 ? ncu / 8 : 0);
            if (e->ovl > 0 && e->ovl < ncu) {
                // Two compute streams on their own queues, masked off e->ovl CUs
                // (bits ncu - 1 - k * stride, PSX_RESERVE_STRIDE, default 1):
                // consecutive sweeps overlap, each one's last dispatch round filled
                // by the next one's units, and the merge / exchange kernels (often
                // multi-wave blocks, which a CU full of one-wave sweep blocks never
                // frees room for) run on the reserved CUs.
                const char* st = getenv("PSX_RESERVE_STRIDE");
                const int stride = st ? std::max(1, atoi(st)) : 1;
                std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
                for (int c = 0; c < ncu; c++) mask[c / 32] |= 1u << (c % 32);
                for (int k = 0; k < e->ovl; k++) {
                    const int c = ncu - 1 - k * stride;
                    if (c >= 0) mask[c / 32] &= ~(1u << (c % 32));
                }
                HIPCHK(hipExtStreamCreateWithCUMask(&e->cstream, (uint32_t)mask.size(), mask.data()));
                HIPCHK(hipExtStreamCreateWithCUMask(&e->cstream2, (uint32_t)mask.size(), mask.data()));
                e->cstream_pr = psx_engine::kCuMasked;  // not pooled
            } else {
                // the compute stream sits below the engine / exchange stream in
                // priority, so merges and the exchange get wave slots first.  (Two
                // alternating unmasked compute streams, overlapping one sweep's
                // tail with the next: neutral at world 1, 2-7 % slower at worlds 2
                // and 4, r05zm, profiles/r05zm_overlap_unmasked.txt.)
                int lo_pr = 0, hi_pr = 0;
                HIPCHK(hipDeviceGetStreamPriorityRange(&lo_pr, &hi_pr));
                e->cstream_pr = (lo_pr + hi_pr) / 2;
                HIPCHK(psx::stream_get(&e->cstream, e->cstream_pr));
            }
            for (int i = 0; i < psx_engine::kBufs; i++)
                if (!e->mdone[i]) HIPCHK(hipEventCreateWithFlags(&e->mdone[i], hipEventDisableTiming));
        }
        // Serial passes at world 1 (PSX_SERIAL = 0 / 1 overrides): every pass's
        // sweep and merge back to back on the engine stream.  With nothing to
        // exchange, overlapping the merge with the next sweep bought nothing: same
        // step, 0.788 vs 0.789 ms at syn1000c3, the overlapped sweep itself 7 %
        // longer (0.808 vs 0.753 ms) for the merge's waves beside it (r06f).  At
        // world > 1 the next sweep hides the exchange (and at world >= 8 the
        // previous sweep's drain): pipelined.
        static const char* ser_env = getenv("PSX_SERIAL");
        const bool serial = ser_env ? atoi(ser_env) != 0 : e->world == 1;
        if ((e->a_pending == 0 && e->a_stamped == 0) || serial) {
            // nothing in flight since the last psx_sync: a single pass (one locus
            // swept once) — sweep and merge back to back on the engine stream, on
            // the whole GPU, with no cross-stream event between them (9 us, r06a)
            S = X;
        } else {
            S = e->cstream;
            if (e->cstream2) {
                S = e->a_alt ? e->cstream2 : e->cstream;
                e->a_alt ^= 1;
            }
        }
        par = e->a_par = (e->a_par + 1) % psx_engine::kBufs;
        // the merge that last read this buffer set (pass i - kBufs) must be done.
        // Host-side flow control: blocking here only when the device is more than
        // kBufs - 1 passes behind keeps barrier packets off the compute stream
        // (back-to-back sweeps then dispatch with no marker between them).
        // A single pass's merge (on X, like its sweep) records no event (an event
        // packet put ~5 us between the merge and the caller's exchange, r06b):
        // a later sweep on a compute stream that reuses its buffers records one
        // on X now, which completes after that merge (X is in order).
        if (S != X && e->mdone_lazy[par]) {
            HIPCHK(hipEventRecord(e->mdone[par], X));
            e->mdone_rec[par] = true;
            e->mdone_lazy[par] = false;
        }
        if (S != X && e->mdone_rec[par]) HIPCHK(hipEventSynchronize(e->mdone[par]));
    }
    SetRec* const dpass = e->dpass + par * npass;
    // EXACT flag word of this buffer set ([1]: sticky word); the words share one image slot
    static_assert(sizeof(int) * (psx_engine::kBufs + 1) <= sizeof(Acc5), "flag words fit the status slot");
    int* const pflag = e->dflag + (par ? 1 + par : 0);
    // no zeroing pass: the merge overwrites every per-SNP slot and the scalars,
    // padding slots stay zero from psx_create, and the EXACT flag word was
    // re-armed by the merge that last used it (or psx_create)
    int slot = 0;
    hipEvent_t k0 = nullptr, k1 = nullptr;  // the sweep launch's own start / stop events
    // the k = 3 fast kernel on the engine stream: no dispatch events, clock stamps
    const bool single = async && S == X && top->k == 3 && top->variant == 1;
    unsigned long long* stamp = nullptr;
    unsigned long long* hstamp = nullptr;
    if (single) {
        if (!e->dstamps) {
            HIPCHK(psx::dmalloc(&e->dstamps, sizeof(unsigned long long) * 2 * psx_engine::kRing));
            HIPCHK(psx::hmalloc(&e->hstamps, sizeof(unsigned long long) * 2 * psx_engine::kRing));
        }
        if (e->a_stamped == psx_engine::kRing) {  // the ring is full: take its passes now
            HIPCHK(hipStreamSynchronize(X));
            take_stamps(e);
        }
        stamp = e->dstamps + 2 * e->a_stamped;
        hstamp = e->hstamps + 2 * e->a_stamped;
        e->plans.stamp = stamp;
    } else if (async) {
        if (e->a_pending == psx_engine::kRing && (rc = consume_async(e))) return rc;
        slot = e->a_head;
        for (int i = 0; i < 2; i++)
            if (!e->aev[2 * slot + i]) HIPCHK(hipEventCreate(&e->aev[2 * slot + i]));
        k0 = e->aev[2 * slot];
        if (e->a_first == -1) {  // the first pass since the last sync starts the span
            if (!e->span0) HIPCHK(hipEventCreate(&e->span0));
            e->a_first = slot;
            k0 = e->span0;
        }
        k1 = e->aev[2 * slot + 1];
    } else {
        HIPCHK(hipEventRecord(e->ev[0], S));
    }
    // the top level; level 2 (c = 3) rides in the same launch
    const int src = psx::sweep_kernel(e->plans, *top, S, sa, dpass + nl, false, low, dpass, par, pflag, !async, k0, k1);
    e->plans.stamp = nullptr;
    if (src) return fail(PSX_EHIP, std::string("sweep level ") + std::to_string(top->k) + ": " + psx::sweep_error());
    if (single) e->a_stamped++;
    if (async && !single) {
        e->a_head = (e->a_head + 1) % psx_engine::kRing;
        e->a_pending++;
        if (S != X) HIPCHK(hipStreamWaitEvent(X, k1, 0));  // merge i after sweep i (stop event of its dispatch)
    }
    const int lo = (int)((int64_t)e->U * e->rank / e->world), hi = (int)((int64_t)e->U * (e->rank + 1) / e->world);
    const SetRec extra = e->rank == 0 ? null_rec(e, 1.0) : psx::set_zero();
    psx::SweepPlan* mA = low ? low : top;
    psx::SweepPlan* mB = low ? top : nullptr;
    // the pass merge (k_merge_rec + k_merge_fin): V slices per SNP run, sized
    // from the plan's records per SNP (about 256 records per slice on average)
    const long nrec = (long)mA->rec_len + (mB ? (long)mB->rec_len : 0);
    const int V = (int)std::min<long>(kMergeWaysMax, std::max<long>(1, (2 * nrec / std::max(e->U, 1) + 511) / 512));
    const long nsingle = hi - lo, nsrec = (long)(nl + nt);
    const int nch = (int)((nsingle + 63) / 64 + (nsrec + kScalChunk - 1) / kScalChunk);
    if ((rc = ensure(e->dspart, e->cap_spart, (size_t)std::max(nch, 1)))) return rc;
    if ((rc = ensure(e->dapart, e->cap_apart, (size_t)e->U * V))) return rc;
    // (-DPSX_ABLATE_MERGE, a separate timing build only: the pass's merge is
    // skipped and its results are wrong; measures what the merge beside the next
    // sweep costs.  No environment switch: a shipped library always merges.)
    const bool csr = mA->csr_pos && (!mB || mB->csr_pos);
#ifndef PSX_ABLATE_MERGE
    hipLaunchKernelGGL(k_merge_rec, dim3((unsigned)(nch + (size_t)e->U * V)), dim3(64), 0, X, e->dp, lo, (int)nsingle,
                       psx::plan_records(*mA, par), mA->d_dptr, csr ? (const int*)nullptr : mA->d_gidx,
                       mB ? psx::plan_records(*mB, par) : nullptr, mB ? mB->d_dptr : nullptr,
                       csr || !mB ? (const int*)nullptr : mB->d_gidx,  // runs contiguous: gidx the identity
                       dpass, nsrec, nch, V, e->dspart, e->dapart, stamp);
    hipLaunchKernelGGL(k_merge_fin, dim3(1 + (e->U + 63) / 64), dim3(64), 0, X, e->dp, lo, hi, nch, V, e->dspart,
                       e->dapart, extra, e->dacc, e->dsacc, pflag, e->dflag + 1, (const int*)e->plans.d_redo,
                       reinterpret_cast<int*>(e->hstat), stamp, hstamp);
#endif
    HIPCHK(hipGetLastError());
    if (async) {
        if (S == X) {
            e->mdone_lazy[par] = true;
            e->mdone_rec[par] = false;
        } else {
            HIPCHK(hipEventRecord(e->mdone[par], X));
            e->mdone_rec[par] = true;
            e->mdone_lazy[par] = false;
        }
        *flag = 0;
        e->stat_fresh = true;  // k_merge_fin wrote the status to hstat
        return 0;
    }
    HIPCHK(hipEventRecord(e->ev[1], X));
    HIPCHK(hipStreamSynchronize(X));  // (k_merge_fin wrote the status block to hstat)
    SetRec s;
    std::memcpy(&s, e->hstat, sizeof(SetRec));
    *flag = s.pad;
    return 0;
}

int fill_timing(psx_engine* e, double gms, int flag);

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int32_t psx_abi_version(void) { return PSX_ABI_VERSION; }
int32_t psx_overlap_cus(const psx_engine* e) { return e ? e->ovl : -1; }
const char* psx_last_error(void) { return g_err.c_str(); }

int psx_pool_trim(void) {
    psx::pool_trim();
    return 0;
}
int64_t psx_pool_cached_bytes(void) { return (int64_t)psx::pool_cached_bytes(); }

int psx_device_count(int* count) {
    int c = 0;
    hipError_t err = hipGetDeviceCount(&c);
    if (err != hipSuccess) c = 0;
    *count = c;
    return 0;
}

uint64_t psx_count_configs(const psx_problem* p) {
    // e_k of weights w_u = 2^{b_u} - 1 (postcal.cpp:903 masks minus checkOR failures = prod (2^b - 1))
    int U = p->n_union, c = p->max_causal;
    std::vector<long double> e(c + 1, 0.0L);
    e[0] = 1;
    for (int u = 0; u < U; u++) {
        int b = 0;
        for (int s = 0; s < p->n_studies; s++) b += p->union_to_local[s * U + u] >= 0;
        long double w = (long double)((1 << b) - 1);
        for (int k = c; k >= 1; k--) e[k] += e[k - 1] * w;
    }
    long double t = 0;
    for (int k = 0; k <= c; k++) t += e[k];
    return (uint64_t)(t + 0.5L);
}

namespace {

// PostCal::PostCal (postcal.h:118-195) from either the low-rank seam inputs
// (p->B, p->s_prime) or, with ld != nullptr, the Model inputs (LD + z) through
// the GPU Model setup (psx_setup.hip).
int create_impl(const psx_problem* p, const psx_ld_problem* ld, int device, psx_engine** out, psx_setup_info* info) {
    *out = nullptr;
    auto tc0 = std::chrono::steady_clock::now();
    if (!p || p->n_studies != 2) return fail(PSX_EINVAL, "only two studies are supported (postcal.cpp:20-23)");
    if (p->max_causal < 0 || p->max_causal > PSX_KMAX) return fail(PSX_ERANGE, "max_causal outside [0, 6]");
    if (p->n_union <= 0 || p->m[0] <= 0 || p->m[1] <= 0) return fail(PSX_EINVAL, "empty problem");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(PSX_ENODEV, "no HIP device: the engine has no CPU fallback");
    if (device < 0 || device >= ndev) return fail(PSX_EINVAL, "device index out of range");
    HIPCHK(hipSetDevice(device));
    psx_engine* e = new psx_engine();
    e->dev = device;
    {
        int khz = 0;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) == hipSuccess && khz > 0)
            e->wclk_khz = khz;
    }
    auto bail = [&](int rc) { delete e; return rc; };
    // the engine stream carries merges and the exchange: highest priority, so its
    // short kernels get wave slots ahead of the sweeps (which run on lower-
    // priority compute streams in pipelined mode)
    int pr_lo = 0, pr_hi = 0;
    if (hipDeviceGetStreamPriorityRange(&pr_lo, &pr_hi) != hipSuccess ||
        psx::stream_get(&e->own_stream, pr_hi) != hipSuccess)
        return bail(fail(PSX_EHIP, "stream"));
    e->own_pr = pr_hi;
    e->stream = e->own_stream;
    for (int i = 0; i < 4; i++)
        if (hipEventCreate(&e->ev[i]) != hipSuccess) return bail(fail(PSX_EHIP, "event"));
    e->m[0] = p->m[0];
    e->m[1] = p->m[1];
    e->N = p->m[0] + p->m[1];
    e->U = p->n_union;
    e->ldg = (e->U + 63) / 64 * 64;
    e->maxc = p->max_causal;
    e->u2l.assign(p->union_to_local, p->union_to_local + 2 * e->U);
    e->pres.assign(e->ldg, 0);
    for (int s = 0; s < 2; s++) {
        int cnt = 0;
        for (int u = 0; u < e->U; u++) {
            int l = e->u2l[s * e->U + u];
            if (l >= p->m[s]) return bail(fail(PSX_EINVAL, "snp map index outside the study"));
            if (l >= 0) { e->pres[u] |= (unsigned char)(1 << s); cnt++; }
        }
        if (cnt != p->m[s]) return bail(fail(PSX_EINVAL, "Invariant does not hold (model.h:140-143)"));
    }
    // the exhaustive pass's unit plans (host decomposition + record CSR) depend
    // only on the locus shape: built on host threads while the setup runs
    e->plans.pres_host = e->pres;
    if (fused_eligible(e)) {
        psx::plan_prefetch(e->plans, device, 2, e->U, e->ldg, 0, 1, false);
        if (e->maxc == 3) psx::plan_prefetch(e->plans, device, 3, e->U, e->ldg, 0, 1, false);
    }
    // d_s (postcal.cpp:66,89): s^2 * (n_s / min n) + t^2 with integer sample sizes
    int mn = std::min(p->sample_sizes[0], p->sample_sizes[1]);
    for (int s = 0; s < 2; s++) e->dval[s] = p->s_squared * (double(p->sample_sizes[s]) / mn) + p->t_squared;
    double spsq = 0;
    if (!ld)
        for (int i = 0; i < e->N; i++) spsq += p->s_prime[i] * p->s_prime[i];
    // null configuration (postcal.cpp:799-803): -res/2 - sqrt(|1|) + U log(1-gamma); K factored out
    e->L0 = -std::sqrt(std::fabs(1.0)) + e->U * std::log(1 - p->gamma);

    // prior tables
    DevProb& dp = e->dp;
    std::memset(&dp, 0, sizeof(dp));
    dp.U = e->U;
    dp.ldg = e->ldg;
    dp.dval[0] = e->dval[0];
    dp.dval[1] = e->dval[1];
    for (int k = 0; k <= PSX_KMAX; k++) {
        double mx = -INFINITY;
        for (int n = 0; n <= k; n++) {
            double pr = prior_nats(p, e->U, k, n);
            dp.prior[k][n] = pr;
            if (std::isfinite(pr)) mx = std::max(mx, pr * PSX_LOG2E);
        }
        dp.Ck[k] = std::isfinite(mx) ? (int)std::ceil(mx) : 0;
        for (int n = 0; n <= k; n++) {
            double v = dp.prior[k][n] * PSX_LOG2E - dp.Ck[k];
            dp.pit[k][n] = std::isfinite(v) ? std::exp2(v) : 0.0;
        }
    }

    // device data: Sigma~ = B^T B, y = B^T S' per study, in union coordinates.
    // The two studies are independent (BIG_SIGMA is block-diagonal, model.h:239):
    // study 1 runs on a second host thread and stream beside study 0.
    using clk = std::chrono::steady_clock;
    auto since = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
    size_t gsz = (size_t)e->ldg * e->ldg;
    struct Scratch {
        double *dB = nullptr, *dS = nullptr, *dsp = nullptr, *dyl = nullptr;
        int* du2l = nullptr;
        hipStream_t st = nullptr;
        std::string err;
        int code = 0;
        double spsq = 0;
        psx::LdStudyResult r;
    } sc[2];
    auto cleanup = [&]() {
        for (auto& x : sc)
            if (x.st) hipStreamSynchronize(x.st);
        psx::IdleScope idle;  // the scratch was used on these two streams only
        for (auto& x : sc) {
            psx::dfree(x.dB); psx::dfree(x.dS); psx::dfree(x.dsp); psx::dfree(x.dyl); psx::dfree(x.du2l);
            if (x.st && x.st != e->stream) psx::stream_put(x.st, 0);
        }
    };
    const clk::time_point ta = clk::now();
    for (int s = 0; s < 2; s++) {
        const int M = p->m[s];
        Scratch& x = sc[s];
        if (psx::dmalloc(&x.dB, (size_t)M * M * sizeof(double)) != hipSuccess ||
            psx::dmalloc(&x.dS, (size_t)M * M * sizeof(double)) != hipSuccess ||
            psx::dmalloc(&x.dsp, (size_t)M * sizeof(double)) != hipSuccess ||
            psx::dmalloc(&x.dyl, (size_t)M * sizeof(double)) != hipSuccess ||
            psx::dmalloc(&x.du2l, (size_t)e->U * sizeof(int)) != hipSuccess ||
            psx::dmalloc(&e->dG[s], gsz * sizeof(double)) != hipSuccess ||
            psx::dmalloc(&e->dAd[s], e->ldg * sizeof(double)) != hipSuccess ||
            psx::dmalloc(&e->dy[s], e->ldg * sizeof(double)) != hipSuccess) {
            cleanup();
            return bail(fail(PSX_EHIP, "out of device memory (setup)"));
        }
    }
    sc[0].st = e->stream;
    if (psx::stream_get(&sc[1].st, 0) != hipSuccess) {
        sc[1].st = nullptr;
        cleanup();
        return bail(fail(PSX_EHIP, "stream"));
    }
    const double alloc_ms = since(ta);
    const clk::time_point tb = clk::now();
    psx::LuJoin join;  // the two studies' first elimination in joint launches
    static const char* lj = getenv("PSX_LU_JOINT");  // A/B: 0 = each study's own launches
    const bool joint = !(lj && atoi(lj) == 0);
    auto study = [&](int s) {
        struct Leave {  // however this study ends, the other does not wait for it
            psx::LuJoin& j;
            int s;
            ~Leave() { j.leave(s); }
        } leave{join, s};
        Scratch& x = sc[s];
        auto die = [&](int code, const std::string& msg) { x.code = code; x.err = msg; };
        if (hipSetDevice(device) != hipSuccess) return die(PSX_EHIP, "set device");
        const int M = p->m[s];
        const size_t boff = s ? (size_t)p->m[0] * p->m[0] : 0;
        const int soff = s ? p->m[0] : 0;
        hipStream_t st = x.st;
        hipMemcpyAsync(x.du2l, p->union_to_local + s * e->U, e->U * sizeof(int), hipMemcpyHostToDevice, st);
        bool lowrank = true;  // Sigma~ = B^T B, y = B^T S' from (B, S')
        const double* Bs = ld ? nullptr : p->B + boff;
        const double* Ss = ld ? nullptr : p->s_prime + soff;
        std::vector<double> hB, hS;
        if (ld) {
            psx::LdStudyResult& r = x.r;
            std::string err;
            if (psx::ld_study_setup(ld->ld + boff, ld->z + soff, M, st, x.dS, x.dyl, &r, &err, joint ? &join : nullptr, s))
                return die(PSX_EHIP, "GPU model setup: " + err);
            if (r.path == 0) {
                lowrank = false;
                x.spsq += r.spsq;
            } else {
                // Sigma' not (comfortably) positive definite: the reference's eigen
                // route (model.h:213-259) on the GPU, B and S' left in dB / dsp
                // (PSX_HOST_EIGEN=1: the host restatement instead, for tests)
                std::vector<double> sig(ld->ld + boff, ld->ld + boff + (size_t)M * M);
                for (int i = 0; i < M; i++) sig[(size_t)i * M + i] += r.added;
                const char* he = getenv("PSX_HOST_EIGEN");
                if (he && atoi(he)) {
                    hB.resize((size_t)M * M);
                    hS.resize(M);
                    if (psx_lowrank_study(sig.data(), ld->z + soff, M, hB.data(), hS.data()))
                        return die(PSX_EINVAL, "eigen route failed");
                    for (int i = 0; i < M; i++) x.spsq += hS[i] * hS[i];
                    Bs = hB.data();
                    Ss = hS.data();
                } else {
                    double sq = 0;
                    if (psx::eigen_lowrank_device(sig.data(), ld->z + soff, M, st, x.dS, x.dB, x.dsp, &sq, &err))
                        return die(PSX_EHIP, "GPU eigen route: " + err);
                    x.spsq += sq;
                    Bs = Ss = nullptr;  // already on the device
                }
            }
        }
        if (lowrank) {
            if (Bs) hipMemcpyAsync(x.dB, Bs, (size_t)M * M * sizeof(double), hipMemcpyHostToDevice, st);
            if (Ss) hipMemcpyAsync(x.dsp, Ss, (size_t)M * sizeof(double), hipMemcpyHostToDevice, st);
            dim3 g((M + 15) / 16, (M + 15) / 16);
            hipLaunchKernelGGL(k_btb, g, dim3(256), 0, st, x.dB, M, x.dS);
            hipLaunchKernelGGL(k_bts, dim3(M), dim3(64), 0, st, x.dB, x.dsp, M, x.dyl);
        }
        hipLaunchKernelGGL(k_to_union, dim3((e->ldg + 255) / 256, e->ldg), dim3(256), 0, st, x.dS, M, x.du2l, e->U,
                           e->ldg, e->dG[s]);
        if (hipGetLastError() != hipSuccess) return die(PSX_EHIP, "setup kernel launch");
        std::vector<double> Sd((size_t)M), yl(M);
        // diagonal of Sigma~ (into the B staging buffer, no longer needed) and y
        hipLaunchKernelGGL(k_diag, dim3((M + 255) / 256), dim3(256), 0, st, x.dS, M, x.dB);
        hipMemcpyAsync(Sd.data(), x.dB, M * sizeof(double), hipMemcpyDeviceToHost, st);
        hipMemcpyAsync(yl.data(), x.dyl, M * sizeof(double), hipMemcpyDeviceToHost, st);
        if (hipStreamSynchronize(st) != hipSuccess) return die(PSX_EHIP, "setup sync");
        std::vector<double> ad(e->ldg), yu(e->ldg);
        for (int u = 0; u < e->ldg; u++) {
            int l = (u < e->U) ? e->u2l[s * e->U + u] : -1;
            ad[u] = 1.0 / e->dval[s] + (l >= 0 ? Sd[l] : 0.0);
            yu[u] = (l >= 0) ? yl[l] : 0.0;
        }
        hipMemcpyAsync(e->dAd[s], ad.data(), e->ldg * sizeof(double), hipMemcpyHostToDevice, st);
        hipMemcpyAsync(e->dy[s], yu.data(), e->ldg * sizeof(double), hipMemcpyHostToDevice, st);
        if (hipStreamSynchronize(st) != hipSuccess) return die(PSX_EHIP, "setup copy");
    };
    {
        std::thread t1(study, 1);
        study(0);
        t1.join();
    }
    const double studies_ms = since(tb);
    for (int s = 0; s < 2; s++) {
        if (sc[s].code) {
            const int code = sc[s].code;
            const std::string msg = sc[s].err;
            cleanup();
            return bail(fail(code, msg));
        }
        spsq += sc[s].spsq;
        if (ld && info) {
            const psx::LdStudyResult& r = sc[s].r;
            info->psd_added[s] = r.added;
            info->psd_iterations[s] = r.psd_iterations;
            info->eigen_route[s] = r.path;
            info->min_pivot_ratio[s] = r.min_pivot_ratio;
            info->spsq[s] = r.path == 0 ? r.spsq : 0.0;
            info->study_upload_ms[s] = r.upload_ms;
            info->study_psd_ms[s] = r.psd_ms;
            info->study_finish_ms[s] = r.finish_ms;
        }
    }
    const clk::time_point tc = clk::now();
    cleanup();
    e->K = -spsq / 2;
    if (psx::dmalloc(&e->dpres, e->ldg) != hipSuccess ||
        psx::dmalloc(&e->dacc, sizeof(Acc5) * ((size_t)e->ldg + 3)) != hipSuccess ||
        psx::hmalloc(&e->hstat, kStatBytes + 64) != hipSuccess)  // + the redo count (k_status_out)
        return bail(fail(PSX_EHIP, "out of device memory"));
    static_assert(sizeof(SetRec) == sizeof(Acc5), "SetRec occupies one image slot");
    e->dsacc = reinterpret_cast<SetRec*>(e->dacc + e->ldg);
    e->dtag = reinterpret_cast<PlanTag*>(e->dacc + e->ldg + 1);
    e->dflag = reinterpret_cast<int*>(e->dacc + e->ldg + 2);
    e->plans.d_flag = e->dflag;
    e->plans.own_flag = false;
    hipMemcpyAsync(e->dpres, e->pres.data(), e->ldg, hipMemcpyHostToDevice, e->stream);
    for (int s = 0; s < 2; s++) {
        dp.G[s] = e->dG[s];
        dp.Ad[s] = e->dAd[s];
        dp.y[s] = e->dy[s];
    }
    dp.pres = e->dpres;
    if (hipMemsetAsync(e->dacc, 0, sizeof(Acc5) * ((size_t)e->ldg + 3), e->stream) != hipSuccess)
        return bail(fail(PSX_EHIP, "memset"));
    if (write_tag(e)) return bail(PSX_EHIP);
    if (reset_acc(e)) return bail(PSX_EHIP);
    if (hipStreamSynchronize(e->stream) != hipSuccess) return bail(fail(PSX_EHIP, "create sync"));
    std::memset(&e->timing, 0, sizeof(e->timing));
    if (info) {
        info->setup_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tc0).count();
        info->alloc_ms = alloc_ms;
        info->studies_ms = studies_ms;
        info->tail_ms = since(tc);
    }
    *out = e;
    return 0;
}

}  // namespace

int psx_create(const psx_problem* p, int device, psx_engine** out) {
    if (!out) return fail(PSX_EINVAL, "null out");
    *out = nullptr;
    if (!p || !p->B || !p->s_prime) return fail(PSX_EINVAL, "null problem");
    return create_impl(p, nullptr, device, out, nullptr);
}

int psx_create_from_ld(const psx_ld_problem* q, int device, psx_engine** out, psx_setup_info* info) {
    if (!out) return fail(PSX_EINVAL, "null out");
    *out = nullptr;
    if (!q || !q->ld || !q->z || !q->m) return fail(PSX_EINVAL, "null problem");
    if (info) std::memset(info, 0, sizeof(*info));
    psx_problem p;
    std::memset(&p, 0, sizeof(p));
    p.n_studies = q->n_studies;
    p.m = q->m;
    p.n_union = q->n_union;
    p.union_to_local = q->union_to_local;
    p.max_causal = q->max_causal;
    p.sample_sizes = q->sample_sizes;
    p.sharing_param = q->sharing_param;
    p.gamma = q->gamma;
    p.t_squared = q->t_squared;
    p.s_squared = q->s_squared;
    return create_impl(&p, q, device, out, info);
}

namespace {
int gpu_ready(int device) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(PSX_ENODEV, "no HIP device: the engine has no CPU fallback");
    if (device < 0 || device >= ndev) return fail(PSX_EINVAL, "device index out of range");
    HIPCHK(hipSetDevice(device));
    return 0;
}
}  // namespace

int psx_warmup_for(int device, int32_t max_causal, int32_t configs_file) {
    // PSX_TIMING: the warm-up's phases on stderr (module load costs per
    // translation unit; each is its own code object, loaded on first use)
    const bool trace = getenv("PSX_TIMING") != nullptr;
    auto now = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    double t[7] = {now(), 0, 0, 0, 0, 0, 0};
    double ta = 0, tl = 0;  // engine module split: first allocation, launch enqueued
    int rc;
    if ((rc = gpu_ready(device))) return rc;
    HIPCHK(hipFree(nullptr));  // context
    t[1] = now();
    // one launch loads this translation unit's device code; on a pooled
    // stream (the setup's second study takes it next), not the null stream,
    // whose hardware queue nothing else would use
    double* d = nullptr;
    HIPCHK(psx::dmalloc(&d, 64 * sizeof(double)));
    hipStream_t ws = nullptr;
    static const char* wn = getenv("PSX_WARM_NULL");  // A/B: the null stream, as before late r06
    const bool warm_null = wn && atoi(wn);
    if (!warm_null) HIPCHK(psx::stream_get(&ws, 0));
    ta = now();
    hipLaunchKernelGGL(k_diag, dim3(1), dim3(64), 0, ws, d, 8, d + 8);
    hipError_t le = hipGetLastError();
    tl = now();
    hipError_t se = warm_null ? hipDeviceSynchronize() : hipStreamSynchronize(ws);
    if (ws) psx::stream_put(ws, 0);
    {
        psx::IdleScope idle;  // (ws synchronised)
        psx::dfree(d);
    }
    if (le != hipSuccess || se != hipSuccess)
        return fail(PSX_EHIP, std::string("warm-up: ") + hipGetErrorString(le != hipSuccess ? le : se));
    t[2] = now();
    // then the code objects the run will use, which the first create / pass
    // would otherwise load: the Model setup and the tiled sweep always, the
    // k = 3 sweep only for c >= 3, the configs-file path (hipcub's radix sort,
    // the largest) only for a -b run
    if (psx::warm_module_setup()) return fail(PSX_EHIP, "warm-up: setup device code did not load");
    t[3] = now();
    if (psx::warm_module_sweep() || psx::warm_module_plan())
        return fail(PSX_EHIP, "warm-up: sweep device code did not load");
    t[4] = now();
    if (max_causal >= 3 && psx::warm_module_sweep3()) return fail(PSX_EHIP, "warm-up: k = 3 device code did not load");
    t[5] = now();
    if (configs_file && psx::warm_module_configs()) return fail(PSX_EHIP, "warm-up: configs device code did not load");
    t[6] = now();
    if (trace)
        fprintf(stderr,
                "psx-warm {\"context_ms\": %.3f, \"engine_module_ms\": %.3f, \"setup_module_ms\": %.3f, "
                "\"sweep_module_ms\": %.3f, \"sweep3_module_ms\": %.3f, \"configs_module_ms\": %.3f, "
                "\"engine_module_split\": {\"first_alloc_ms\": %.3f, \"first_launch_enqueue_ms\": %.3f, "
                "\"first_launch_complete_ms\": %.3f}}\n",
                t[1] - t[0], t[2] - t[1], t[3] - t[2], t[4] - t[3], t[5] - t[4], t[6] - t[5], ta - t[1], tl - ta,
                t[2] - tl);
    return 0;
}

int psx_warmup(int device) { return psx_warmup_for(device, 3, 0); }

int psx_single_queue(int32_t on) {
    psx::set_single_queue(on != 0);
    return 0;
}

int psx_lu_det_gpu(const double* a, int32_t m, int device, double* det) {
    if (!a || m <= 0 || !det) return fail(PSX_EINVAL, "bad argument");
    int rc;
    if ((rc = gpu_ready(device))) return rc;
    double* dA = nullptr;
    double* dd = nullptr;
    int* ds = nullptr;
    const size_t nn = (size_t)m * m;
    if (psx::dmalloc(&dA, nn * sizeof(double)) != hipSuccess || psx::dmalloc(&dd, m * sizeof(double)) != hipSuccess ||
        psx::dmalloc(&ds, m * sizeof(int)) != hipSuccess) {
        psx::dfree(dA); psx::dfree(dd); psx::dfree(ds);
        return fail(PSX_EHIP, "out of device memory");
    }
    std::string err;
    rc = 0;
    if (hipMemcpy(dA, a, nn * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) rc = fail(PSX_EHIP, "upload");
    else if (psx::lu_det_device(dA, m, ds, dd, nullptr, det, &err)) rc = fail(PSX_EHIP, err);
    psx::dfree(dA); psx::dfree(dd); psx::dfree(ds);
    return rc;
}

int psx_elim_gpu(const double* a, int32_t m, const double* z, int32_t check, double* pivots, double* z_out,
                 int32_t* swap_needed, int device) {
    if (!a || m <= 0 || !pivots || !swap_needed || (z && !z_out)) return fail(PSX_EINVAL, "bad argument");
    int rc;
    if ((rc = gpu_ready(device))) return rc;
    std::string err;
    int sw = 0;
    if (psx::elim_device(a, m, z, check, pivots, z_out, &sw, &err)) return fail(PSX_EHIP, err);
    *swap_needed = sw;
    return 0;
}

int psx_psd_shift_gpu(double* sigma, int32_t m, double* added, int device) {
    if (!sigma || m <= 0) return fail(PSX_EINVAL, "bad argument");
    int rc;
    if ((rc = gpu_ready(device))) return rc;
    std::vector<double> t((size_t)m * m);
    double add = 0;
    for (int guard = 0;; guard++) {
        if (guard >= 100000) return fail(PSX_EINVAL, "PSD shift did not terminate");
        std::memcpy(t.data(), sigma, t.size() * sizeof(double));
        for (int i = 0; i < m; i++) t[(size_t)i * m + i] = sigma[(size_t)i * m + i] + add;
        double det = 0;
        if ((rc = psx_lu_det_gpu(t.data(), m, device, &det))) return rc;
        if (det > 0) break;
        add += 0.01;
    }
    for (int i = 0; i < m; i++) sigma[(size_t)i * m + i] += add;
    if (added) *added = add;
    return 0;
}

void psx_destroy(psx_engine* e) { delete e; }

int psx_set_shard(psx_engine* e, int rank, int world) {
    if (!e || world < 1 || rank < 0 || rank >= world) return fail(PSX_EINVAL, "bad shard");
    HIPCHK(hipSetDevice(e->dev));
    e->stat_fresh = false;  // status changes: psx_sync reads it out again
    const bool moved = rank != e->rank || world != e->world;
    e->rank = rank;
    e->world = world;
    if (moved && fused_eligible(e)) {  // this shard's plans, built ahead
        psx::plan_prefetch(e->plans, e->dev, 2, e->U, e->ldg, rank, world, false);
        if (e->maxc == 3) psx::plan_prefetch(e->plans, e->dev, 3, e->U, e->ldg, rank, world, false);
    }
    return write_tag(e);
}

int psx_plan_hash(psx_engine* e, uint64_t* hash) {
    if (!e || !hash) return fail(PSX_EINVAL, "bad argument");
    *hash = plan_hash(e);
    return 0;
}

int psx_reset(psx_engine* e) {
    HIPCHK(hipSetDevice(e->dev));
    e->stat_fresh = false;  // status changes: psx_sync reads it out again
    int rc = reset_acc(e);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(e->stream));
    return 0;
}

int psx_run_exhaustive(psx_engine* e) {
    HIPCHK(hipSetDevice(e->dev));
    e->stat_fresh = false;  // status changes: psx_sync reads it out again
    const auto t0 = std::chrono::steady_clock::now();
    int rc;
    std::memset(&e->timing, 0, sizeof(e->timing));
    e->prep_ms = 0;
    double gms = 0;
    int flag = 0;
    if (fused_eligible(e)) {
        if ((rc = fused_pass(e, &flag))) return rc;
    } else {
        if ((rc = exhaustive_pass(e, false, &gms))) return rc;
        flag = *(const int*)(e->hstat + 2 * sizeof(SetRec));
    }
    if (flag) {  // some set's notSharedLL group sits > 900 bits below its maximum: exact variant
        if ((rc = exhaustive_pass(e, true, &gms))) return rc;
        HIPCHK(hipMemsetAsync(e->dflag + 1, 0, sizeof(int), e->stream));  // handled: clear the sticky copy
    }
    e->stat_fresh = false;
    if ((rc = fill_timing(e, gms, flag))) return rc;
    e->timing.prepare_ms = e->prep_ms;
    e->timing.run_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return 0;
}

int psx_run_exhaustive_async(psx_engine* e) {
    HIPCHK(hipSetDevice(e->dev));
    if (!fused_eligible(e)) return psx_run_exhaustive(e);
    int flag = 0;
    return fused_pass(e, &flag, true);
}

int psx_sync(psx_engine* e, int32_t* exact_needed) {
    HIPCHK(hipSetDevice(e->dev));
    int rc;
    const bool fresh = e->stat_fresh;
    e->stat_fresh = false;
    if (!fresh) {
        // one launch reads the status block and the redo count out to pinned host
        // memory and re-arms the sticky EXACT flag and the plan-mismatch word
        hipLaunchKernelGGL(k_status_out, dim3(1), dim3(64), 0, e->stream, reinterpret_cast<int*>(e->dsacc),
                           (const int*)e->plans.d_redo, reinterpret_cast<int*>(e->hstat));
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(e->stream));
    const int* const words = reinterpret_cast<const int*>(e->hstat + 2 * sizeof(SetRec));
    const int sticky = words[1];
    const int redo = *reinterpret_cast<const int*>(e->hstat + kStatBytes);
    if (fresh && (sticky || words[kPlanMismatchWord])) {
        // the last merge wrote the status (no read-out launch): re-arm the words
        // the host consumes here (raised flags only: the common pass skips this)
        HIPCHK(hipMemsetAsync(e->dflag + 1, 0, sizeof(int), e->stream));
        HIPCHK(hipMemsetAsync(e->dflag + kPlanMismatchWord, 0, sizeof(int), e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
    }
    take_stamps(e);
    // a refused merge of partial images (k_merge_partials wrote nothing) is
    // reported after the pass bookkeeping below, once (k_status_out cleared it)
    const bool mismatch = words[kPlanMismatchWord] != 0;
    auto done = [&]() {
        return mismatch ? fail(PSX_EINVAL, "merged partial images are not shards 0..world-1 of one plan "
                                           "(ranks with different PSX_K3_* knobs, builds or shard settings); "
                                           "nothing was merged")
                        : 0;
    };
    if (exact_needed) *exact_needed = sticky;
    if (e->a_pending == 0 && e->a_count == 0) {
        // nothing asynchronous since the last sync: the count still follows the
        // accumulators just read (a merge of partial images folds the shards')
        SetRec st;
        std::memcpy(&st, e->hstat, sizeof(SetRec));
        e->timing.configs = (uint64_t)(st.npat + 0.5);
        return done();
    }
    while (e->a_pending > 0)
        if ((rc = consume_async(e))) return rc;
    // timing of the asynchronous passes since the last sync: the dominant
    // kernel's summed device time over its launches, per-launch work from the plan
    std::memset(&e->timing, 0, sizeof(e->timing));
    const psx::SweepArgs sa = sweep_args(e);
    psx::SweepPlan* P2 = nullptr;
    psx::SweepPlan* P3 = nullptr;
    if (psx::sweep_prepare(e->plans, 2, e->U, e->ldg, e->rank, e->world, e->stream, sa, false, &P2) ||
        (e->maxc == 3 && psx::sweep_prepare(e->plans, 3, e->U, e->ldg, e->rank, e->world, e->stream, sa, false, &P3)))
        return fail(PSX_EHIP, std::string("sweep plan: ") + psx::sweep_error());
    const psx::SweepPlan* top = P3 ? P3 : P2;
    e->timing.kernel_ms = e->a_kms;
    e->timing.span_ms = e->a_count ? (e->a_span + e->a_sspan) / e->a_count : 0.0;
    e->timing.kernel_launches = e->a_count;
    e->timing.sweep_ms = e->a_count ? e->a_kms / e->a_count : 0.0;
    e->timing.union_sets = top->union_sets;
    e->timing.alg_bytes = top->alg_bytes + top->fused_bytes;
    e->timing.flops = top->flops + top->fused_flops;
    e->timing.exact_rerun = sticky;
    e->timing.robust_units = redo;
    SetRec st;
    std::memcpy(&st, e->hstat, sizeof(SetRec));
    e->timing.configs = (uint64_t)(st.npat + 0.5);
    e->a_kms = 0;
    e->a_count = 0;
    e->a_first = -1;
    e->a_span = 0;
    e->a_sspan = 0;
    return done();
}

}  // extern "C"

namespace {
int fill_timing(psx_engine* e, double gms, int flag) {
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, e->ev[0], e->ev[1]));
    psx::SweepStats st;
    std::memset(&st, 0, sizeof(st));
    int top_tiled = 0;
    for (int k = 1; k <= e->maxc; k++)
        if (psx::sweep_supports(k, e->U)) {
            if (psx::sweep_stats(e->plans, k, e->U, e->rank, e->world, &st)) return fail(PSX_EHIP, psx::sweep_error());
            top_tiled = k;
        }
    e->timing.sweep_ms = ms;
    if (top_tiled) {
        e->timing.kernel_ms = st.kernel_ms[top_tiled];
        e->timing.kernel_launches = st.launches[top_tiled];
        e->timing.union_sets = st.union_sets[top_tiled];
        e->timing.alg_bytes = st.alg_bytes[top_tiled];
        e->timing.flops = st.flops[top_tiled];
    } else {
        e->timing.kernel_ms = gms;
        e->timing.kernel_launches = e->maxc;
    }
    e->timing.merge_ms = st.merge_ms;
    e->timing.exact_rerun = flag;
    if (psx::sweep_redo_count(e->plans, &e->timing.robust_units)) return fail(PSX_EHIP, psx::sweep_error());
    SetRec s;
    std::memcpy(&s, e->hstat, sizeof(SetRec));
    e->timing.configs = (uint64_t)(s.npat + 0.5);
    return 0;
}
}  // namespace

extern "C" {

int psx_eval_union_batch(psx_engine* e, const int32_t* sets, int32_t stride, int32_t n_sets, int accumulate,
                         double* score_out) {
    HIPCHK(hipSetDevice(e->dev));
    e->stat_fresh = false;  // status changes: psx_sync reads it out again
    const auto t0 = std::chrono::steady_clock::now();
    if (stride < 1 || stride > PSX_KMAX) return fail(PSX_ERANGE, "stride outside [1, 6]");
    if (n_sets < 0 || (n_sets > 0 && !sets)) return fail(PSX_EINVAL, "bad set batch");
    // Rows go to the device as given (one pinned copy per slice); k_eval_batch
    // validates and compacts them and evaluates the null rows.  Slices of at
    // most kBatchChunks merge chunks (an SSS neighbourhood is one slice).
    std::memset(&e->timing, 0, sizeof(e->timing));
    const size_t per = (size_t)kBatchChunks * (size_t)psx::batch_merge_sets_per_chunk(stride);
    double kms = 0, prep = 0;
    int rc;
    if ((size_t)n_sets > per) {
        // more than one slice: every slice is merged before the next one is
        // validated on the device, so the whole batch is checked here first (the
        // device rule: members >= 0 strictly ascending and < U, negatives are
        // padding) — a bad row anywhere adds nothing to the accumulators
        for (size_t r = 0; r < (size_t)n_sets; r++) {
            int prev = -1;
            for (int j = 0; j < stride; j++) {
                const int v = sets[r * stride + j];
                if (v < 0) continue;
                if (v >= e->U || v <= prev) return fail(PSX_EINVAL, "sets must be ascending union indices");
                prev = v;
            }
        }
    }
    for (size_t s0 = 0; s0 < (size_t)n_sets; s0 += per) {
        const size_t nb = std::min(per, (size_t)n_sets - s0);
        const auto ts = std::chrono::steady_clock::now();
        int* h = nullptr;
        if ((rc = stage_acquire(e, nb * stride, &h))) return rc;
        std::memcpy(h, sets + s0 * stride, nb * stride * sizeof(int));
        prep += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ts).count();
        if ((rc = eval_generic_staged(e, stride, nb, accumulate != 0, score_out ? score_out + s0 : nullptr, &kms,
                                      true)))
            return rc;
    }
    HIPCHK(hipStreamSynchronize(e->stream));
    // the batch's k_eval_batch launches (HIP events around them on e->stream)
    // and the host walls: the staging copies, the whole call
    e->timing.kernel_ms = kms;
    e->timing.kernel_launches = n_sets > 0 ? (int32_t)(((size_t)n_sets + per - 1) / per) : 0;
    e->timing.union_sets = (uint64_t)n_sets;
    e->timing.prepare_ms = prep;
    e->timing.run_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return 0;
}

int psx_run_configs(psx_engine* e, const int16_t* rows, int64_t n_rows, int32_t n_groups) {
    HIPCHK(hipSetDevice(e->dev));
    e->stat_fresh = false;  // status changes: psx_sync reads it out again
    int rc;
    if ((rc = reset_acc(e))) return rc;
    std::memset(&e->timing, 0, sizeof(e->timing));
    if (n_rows < 0 || n_groups < 0 || (n_rows > 0 && (!rows || n_groups == 0)))
        return fail(PSX_EINVAL, "bad configs rows");
    // the row walk's index maps (model.h:134-139), once per engine: global index
    // -> union position (study 1 after study 0's m0 entries), union -> local
    if (!e->d_cfg_maps) {
        std::vector<int> maps;
        maps.reserve((size_t)e->N + 2 * (size_t)e->U);
        for (int s = 0; s < 2; s++)
            for (int u = 0; u < e->U; u++)
                if (e->u2l[s * e->U + u] >= 0) maps.push_back(u);  // local order = union order (Invariant)
        if ((int)maps.size() != e->N) return fail(PSX_EINVAL, "snp map does not cover the studies");
        maps.insert(maps.end(), e->u2l.begin(), e->u2l.end());
        HIPCHK(psx::dmalloc(&e->d_cfg_maps, maps.size() * sizeof(int)));
        HIPCHK(hipMemcpy(e->d_cfg_maps, maps.data(), maps.size() * sizeof(int), hipMemcpyHostToDevice));
    }
    psx::CfgMaps C{e->d_cfg_maps, e->d_cfg_maps + e->N, e->U, e->N, e->m[0], e->m[1]};
    psx::CfgProb P;
    for (int s = 0; s < 2; s++) {
        P.G[s] = e->dp.G[s];
        P.Ad[s] = e->dp.Ad[s];
        P.y[s] = e->dp.y[s];
        P.dval[s] = e->dp.dval[s];
    }
    P.pres = e->dp.pres;
    P.ldg = e->dp.ldg;
    std::memcpy(P.Ck, e->dp.Ck, sizeof(P.Ck));
    std::memcpy(P.pit, e->dp.pit, sizeof(P.pit));
    std::memcpy(P.prior, e->dp.prior, sizeof(P.prior));
    // every rank validates every row (a bad row fails all ranks alike, before any
    // collective), and evaluates its contiguous slice (psx_set_shard)
    const int64_t r0 = n_rows * e->rank / e->world, r1 = n_rows * (e->rank + 1) / e->world;
    HIPCHK(hipEventRecord(e->ev[0], e->stream));
    psx::CfgResult res;
    const char* err = nullptr;
    if (psx::configs_pass(e->cfg, rows, n_rows, n_groups, r0, r1, C, P, e->dacc, e->dsacc, e->stream, e->ev[2],
                          e->ev[3], &res, &err))
        return fail(PSX_EHIP, std::string("configs file: ") + err);
    if (res.fail_row >= 0) {  // the first failing row in row order
        reset_acc(e);
        if (res.fail_code == 1) return fail(PSX_EINVAL, "configs row index outside the SNP range");
        if (res.fail_code == 2) return fail(PSX_ERANGE, "configs row has more than 6 union SNPs");
        return fail(PSX_EORDER, "This did not work as expected (postcal.cpp:587-590)");
    }
    if ((rc = fold_null(e, (double)res.nulls))) return rc;
    HIPCHK(hipEventRecord(e->ev[1], e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    float ms = 0, kms = 0;
    HIPCHK(hipEventElapsedTime(&ms, e->ev[0], e->ev[1]));
    if (res.nsets > 0) HIPCHK(hipEventElapsedTime(&kms, e->ev[2], e->ev[3]));
    e->timing.sweep_ms = ms;
    e->timing.kernel_ms = kms;
    e->timing.kernel_launches = res.nsets > 0 ? 1 : 0;
    e->timing.configs = (uint64_t)(r1 - r0);
    return 0;
}

// sss_postcal.cpp:102-380 with the iteration's batch work device-resident.
// The walk is serial: each iteration samples the next configuration from all
// neighbour scores with the reference's mt19937(12345) and libstdc++
// discrete_distribution, in the reference's order (sss_postcal.cpp:296-343), so
// that sampling stays on the host.  Everything else of an iteration is two
// launches and one synchronisation:
//   k_sss_eval  one wave per item: the current configuration (item 0) and the
//               neighbourhood swap ++ minus ++ plus (sss_postcal.cpp:20-99,
//               166-186) in the reference's order; each wave builds its set,
//               looks it up in a device open-addressing map (the reference's
//               unordered_map<vector<int>, double>, postcal.h:43-56, 98), and
//               evaluates it if unseen (every pattern's L, the set's score =
//               its max |L| pattern, :624-626, its records); null sets score
//               K + L0 (:463-499)
//   k_sss_post  a block per union SNP folds its records in item order (the
//               current configuration's members scan the items; any other SNP
//               i is only in the swaps (cur \ {c_v}) + {i} and the plus set
//               cur + {i}, at known item indices), one block folds the set
//               records and null configurations into the scalars, and the rest
//               insert the new scores into the map (:280-284) and write every
//               neighbour's score (the sampling weights) to pinned host memory
// With several ranks (psx_run_sss_sharded) each evaluates a contiguous slice of
// the items; the slices' scores and the ranks' normalisers are all-gathered by
// the caller's callback, then the insert runs on every rank with all scores.
extern "C" __device__ __attribute__((const)) int __ockl_wfred_add_i32(int);

namespace {
constexpr int kKeyBits = 21;  // a sorted set of <= 6 as two words of three (index + 1) fields
constexpr int kKeyMaxU = (1 << kKeyBits) - 2;

struct MapEntry {
    unsigned long long lo, hi;
    double score;
    int state, pad;
};

__host__ __device__ inline unsigned long long mix64(unsigned long long x) {
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ULL;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebULL;
    return x ^ (x >> 31);
}
__device__ inline unsigned long long map_slot(unsigned long long lo, unsigned long long hi, unsigned long long mask) {
    return mix64(lo ^ mix64(hi + 0x9e3779b97f4a7c15ULL)) & mask;
}
// Lookup of a key (linear probing) by a whole wave: 64 consecutive probe slots
// per round trip (the table stays at load <= 1/2, so the first window nearly
// always holds an empty slot); the key's slot is the first in probe order that
// is empty or matches, as a serial probe would find it.  Result in every lane.
__device__ inline bool map_find_wave(const MapEntry* T, unsigned long long mask, unsigned long long lo,
                                     unsigned long long hi, double& v) {
    const int lane = threadIdx.x & 63;
    const unsigned long long base = map_slot(lo, hi, mask);
    for (unsigned long long off = 0;; off += 64) {
        const MapEntry& e = T[(base + off + lane) & mask];
        const bool empty = e.state == 0;
        const bool match = !empty && e.lo == lo && e.hi == hi;
        const unsigned long long me = __ballot(empty), mm = __ballot(match);
        const unsigned long long before = me ? (me & (0ull - me)) - 1ull : ~0ull;  // lanes below the first empty
        if (mm & before) {
            v = __shfl(e.score, __ffsll((long long)(mm & before)) - 1);
            return true;
        }
        if (me) return false;
    }
}
// keys inserted by one launch are distinct and no lookup runs beside an insert
__device__ inline void map_insert(MapEntry* T, unsigned long long mask, unsigned long long lo, unsigned long long hi,
                                  double v) {
    for (unsigned long long i = map_slot(lo, hi, mask);; i = (i + 1) & mask)
        if (atomicCAS(&T[i].state, 0, 1) == 0) {
            T[i].lo = lo;
            T[i].hi = hi;
            T[i].score = v;
            return;
        }
}
__device__ inline void pack_key(const int* row, int n, unsigned long long& lo, unsigned long long& hi) {
    unsigned long long w[2] = {0, 0};
#pragma unroll
    for (int j = 0; j < PSX_KMAX; j++)
        if (j < n) w[j / 3] |= (unsigned long long)(row[j] + 1) << (kKeyBits * (j % 3));
    lo = w[0];
    hi = w[1];
}

// one iteration's neighbourhood geometry (sss_postcal.cpp:166-186)
struct SssIter {
    int cur[PSX_KMAX];
    int k, U, stride, num_zero, num_minus, num_plus, n_nbd, rank, world;
    double null_score;  // K + L0: a null configuration's L (postcal.cpp:797-803)
    unsigned long long* trace;  // PSX_SSS_TRACE: item 1's phase clocks (null: none)
    unsigned int seq;  // one rank: the iteration's tag in the published mark words
};

// neighbour i (0 .. n_nbd) or, for i == -1, the current configuration: its
// sorted members (-1 padded to `stride`) and size
__device__ int nbd_row(const SssIter& it, int i, int* row) {
    const int k = it.k;
    int x = -1, skip = -1, n;
    if (i < 0) {
        n = k;
    } else if (i < it.num_zero) {  // (cur \ {c_v}) + {x}
        skip = i % k;
        x = i / k;
        n = k;
    } else if (i < it.num_zero + it.num_minus) {  // cur \ {c_v}
        skip = i - it.num_zero;
        n = k - 1;
    } else {  // cur + {x}
        x = i - it.num_zero - it.num_minus;
        n = k + 1;
    }
    if (x >= 0)  // the x-th SNP not in cur
#pragma unroll
        for (int j = 0; j < PSX_KMAX; j++)
            if (j < k && it.cur[j] <= x) x++;
    int m = 0;
    bool put = x < 0;
#pragma unroll
    for (int j = 0; j < PSX_KMAX; j++) {
        if (j >= k || j == skip) continue;
        if (!put && x < it.cur[j]) {
            row[m++] = x;
            put = true;
        }
        row[m++] = it.cur[j];
    }
    if (!put) row[m++] = x;
    for (int j = m; j < it.stride; j++) row[j] = -1;
    return n;
}

// iteration counters: k_sss_eval's block 0 writes the current configuration's
// two (kCurPos: 0 if it is evaluated, else -1; kCurNull: 1 if it is an unseen
// null configuration), k_sss_post's scalar block counts the unseen neighbours
// and null configurations from mark[] (no contended atomics in the eval) and
// copies all four to pinned host memory
enum { kUnseen = 0, kNulls = 1, kCurPos = 2, kCurNull = 3, kNCnt = 4 };

// item p of the iteration: the current configuration (p = 0, always evaluated
// when unseen: sss_postcal.cpp:195-202) or neighbour i = p - 1.  mark[i]: -1
// seen (its score is the map's), -2 an unseen null set, p an unseen set.
// One rank: every neighbour's weight and mark go to pinned host memory from
// here.  The weight is stored first, then, once that store is acknowledged, the
// mark word (iteration tag << 32 | mark); both at system scope (write-through,
// no L2 write-back) into coherent pinned memory (hipHostMallocCoherent, uncached
// for the device: an acknowledged store is in host memory, so the mark cannot
// overtake the weight; a release store at system scope would add an L2
// write-back per wave, measured 13 -> 21 us per eval in r05).  The host takes
// neighbour i when its word carries this iteration's tag: no wait for the
// kernel's end (~5-8 us before its stop event completes) and no contended
// completion counter.
__device__ inline void publish_mark(double* lk_host, unsigned long long* mark_host, int i, double w, int mk,
                                    unsigned int seq) {
    __hip_atomic_store(lk_host + i, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0);  // the weight's store acknowledged
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __hip_atomic_store(mark_host + i, ((unsigned long long)seq << 32) | (unsigned int)mk, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

extern "C++" {  // (a template, inside the ABI's extern "C" block)
template <int KM>  // the most members of a set of the walk (max_causal; 5 for KM = 5)
__global__ __launch_bounds__(64) void k_sss_eval(DevProb P, SssIter it, const MapEntry* __restrict__ T,
                                                 unsigned long long mask, int lo, int hi, int* __restrict__ rows,
                                                 int* __restrict__ mark, int* __restrict__ cnt,
                                                 double* __restrict__ lk_host, SetRec* __restrict__ srec,
                                                 Acc5* __restrict__ mrec, double* __restrict__ score,
                                                 unsigned long long* __restrict__ mark_host) {
    __shared__ EvalShm shm;
    const int p = blockIdx.x, i = p - 1, lane = threadIdx.x;
    unsigned long long* const tr = (it.trace && p == 1 && lane == 0) ? it.trace : nullptr;
    if (tr) tr[0] = wall_clock64();
    int row[PSX_KMAX];
    const int n = nbd_row(it, i, row);
    // the set's operands are requested before the map probe and consumed after
    // it: one global round trip less for an unseen set (a seen one drops them)
    const EvalOps ops = eval_gather(P, row, it.stride, shm);
    double v = 0.0;
    unsigned long long klo, khi;
    pack_key(row, n, klo, khi);
    const int seen = map_find_wave(T, mask, klo, khi, v) ? 1 : 0;
    if (tr) tr[1] = wall_clock64();
    if (lane == 0) {
        if (i >= 0) {
            const int mk = seen ? -1 : (n == 0 ? -2 : p);
            mark[i] = mk;
            if (!mark_host) {
                if (seen) lk_host[i] = v;
            } else if (mk != p) {  // seen or null: published now (an unseen set after its evaluation)
                publish_mark(lk_host, mark_host, i, seen ? v : it.null_score, mk, it.seq);
            }
        } else {
            cnt[kCurPos] = (seen || n == 0) ? -1 : 0;  // a null current configuration is counted, not evaluated
            cnt[kCurNull] = (!seen && n == 0) ? 1 : 0;
        }
    }
    if (p < lo || p >= hi) return;  // another rank's item
    if (seen || n == 0) {
        // zero records (a fold of a zero record is exactly a no-op): the post folds
        // every item of the slice without looking at marks or rows
        if (lane < it.stride) mrec[(size_t)p * it.stride + lane] = psx::acc_zero();
        if (lane == 0) srec[p] = psx::set_zero();
        return;
    }
#ifdef PSX_SSS_ABLATE
    if (PSX_SSS_ABLATE == 1) {
        if (mark_host && lane == 0 && i >= 0) publish_mark(lk_host, mark_host, i, 0.0, p, it.seq);
        return;
    }
#endif
#pragma unroll
    for (int j = 0; j < PSX_KMAX; j++)
        if (j < it.stride && lane == j) rows[(size_t)p * it.stride + j] = row[j];
    eval_stage(ops, shm);
    if (tr) tr[2] = wall_clock64();
    eval_compute<KM>(P, ops, shm, nullptr, srec + p, mrec + (size_t)p * it.stride, score + p, tr);
    if (tr) tr[7] = wall_clock64();
    if (mark_host && lane == 0 && i >= 0) publish_mark(lk_host, mark_host, i, score[p], p, it.seq);  // the lane that wrote it
}
}  // extern "C++"

// blocks [0, U): per-SNP record folds; block U: the scalars; blocks > U: the
// map inserts and the sampling weights.  mode 0: folds only, 1: folds and
// inserts, 2: inserts only (after the all-gather of a sharded walk)
__global__ __launch_bounds__(256) void k_sss_post(SssIter it, int lo, int hi, const int* __restrict__ rows,
                                                  const int* __restrict__ mark, const int* __restrict__ cnt,
                                                  const Acc5* __restrict__ mrec, const SetRec* __restrict__ srec,
                                                  const double* __restrict__ score, SetRec null1,
                                                  Acc5* __restrict__ acc, SetRec* __restrict__ sacc,
                                                  SetRec* __restrict__ sacc_host, int* __restrict__ cnt_host,
                                                  MapEntry* __restrict__ T, unsigned long long mask, int mode,
                                                  double* __restrict__ lk_host) {
    const int b = blockIdx.x, t = threadIdx.x;
    if (mode == 2 && b <= it.U) return;
    // Every item p of the slice [lo, hi) has records at mrec[p * stride + j]
    // (zero records where k_sss_eval did not evaluate it), and a member's
    // position j in item p's row follows from the iteration geometry
    // (nbd_row), so the folds below issue their record loads without waiting
    // for marks or rows.
    const int k = it.k;
    if (b < it.U) {
        const int u = b;
        int ju = -1, less = 0;  // u's slot in cur (or -1); members of cur below u
        for (int j = 0; j < k; j++) {
            ju = it.cur[j] == u ? j : ju;
            less += it.cur[j] < u;
        }
        Acc5 a = psx::acc_zero();
        if (ju >= 0) {
            // in (nearly) every item: the slice's items in item order
            constexpr int kR = 8;  // record loads in flight per thread
            for (int p0 = lo + t; p0 < hi; p0 += 256 * kR) {
                Acc5 r[kR];
#pragma unroll
                for (int q = 0; q < kR; q++) {
                    const int p = p0 + 256 * q;
                    int j = -1;
                    if (p < hi) {
                        const int i = p - 1;
                        if (i < 0) {
                            j = ju;
                        } else if (i < it.num_zero + it.num_minus) {  // swap / minus: slot v dropped
                            const int v = i < it.num_zero ? i % k : i - it.num_zero;
                            if (v != ju) {
                                j = ju - (v < ju);
                                if (i < it.num_zero) {  // + the (i / k)-th SNP outside cur
                                    int x = i / k;
                                    for (int c = 0; c < k; c++) x += it.cur[c] <= x;
                                    j += x < u;
                                }
                            }
                        } else {  // plus: + the x-th SNP outside cur
                            int x = i - it.num_zero - it.num_minus;
                            for (int c = 0; c < k; c++) x += it.cur[c] <= x;
                            j = ju + (x < u);
                        }
                    }
                    r[q] = j >= 0 ? mrec[(size_t)p * it.stride + j] : psx::acc_zero();
                }
#pragma unroll
                for (int q = 0; q < kR; q++) psx::fold_acc(a, r[q]);
            }
            __shared__ Acc5 sh[4];
            psx::wave_fold_acc(a);
            if ((t & 63) == 0) sh[t >> 6] = a;
            __syncthreads();
            if (t == 0) {
                Acc5 g = acc[u];
                for (int q = 0; q < 4; q++) psx::fold_acc(g, sh[q]);
                acc[u] = g;
            }
            return;
        }
        if (t != 0) return;
        // u is the ri-th SNP outside cur: items ri * k + v (cur with slot v swapped
        // for u: u's position is `less`, one fewer when cur[v] < u), then its plus set
        const int ri = u - less;
        Acc5 r[PSX_KMAX + 1];
        const Acc5 g0 = acc[u];
#pragma unroll
        for (int v = 0; v <= PSX_KMAX; v++) {
            int i = -1, j = 0;
            if (v < k) {
                i = ri * k + v;
                j = less - (it.cur[v] < u);
            } else if (v == k && it.num_plus) {
                i = it.num_zero + it.num_minus + ri;
                j = less;
            }
            const int p = i + 1;
            const bool ok = i >= 0 && p >= lo && p < hi;
            r[v] = mrec[ok ? (size_t)p * it.stride + j : 0];  // (unconditional: one round trip, late r06)
            if (!ok) r[v] = psx::acc_zero();
        }
#pragma unroll
        for (int v = 0; v <= PSX_KMAX; v++)
            asm volatile("" : "+v"(r[v].mP), "+v"(r[v].mS), "+v"(r[v].mN), "+v"(r[v].post0), "+v"(r[v].post1),
                         "+v"(r[v].shared), "+v"(r[v].sll), "+v"(r[v].nsll));
#pragma unroll
        for (int v = 0; v <= PSX_KMAX; v++) psx::fold_acc(a, r[v]);
        if (a.post0 != 0.0 || a.post1 != 0.0 || a.shared != 0.0 || a.sll != 0.0 || a.nsll != 0.0) {
            Acc5 g = g0;
            psx::fold_acc(g, a);
            acc[u] = g;
        }
        return;
    }
    if (b == it.U) {  // the scalars: the slice's set records, then the null configurations (rank 0)
        SetRec a = psx::set_zero();
        int nu = 0, nz = 0;  // unseen neighbours, unseen null neighbours
        // the slice's set records (zero where not evaluated), eight whole records
        // in flight per thread, folded in item order (a fold of srec[p] in the
        // loop split each record into guarded field loads, one round trip per
        // field, late r06)
        for (int p0 = lo + t; p0 < hi; p0 += 256 * 8) {
            SetRec r[8];
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const int p = p0 + 256 * q;
                r[q] = srec[p < hi ? p : hi - 1];
            }
#pragma unroll
            for (int q = 0; q < 8; q++)
                asm volatile("" : "+v"(r[q].m), "+v"(r[q].m0), "+v"(r[q].m1), "+v"(r[q].tot), "+v"(r[q].nc0),
                             "+v"(r[q].nc1), "+v"(r[q].score), "+v"(r[q].npat));
#pragma unroll
            for (int q = 0; q < 8; q++)
                if (p0 + 256 * q < hi) psx::fold_set(a, r[q]);
        }
        for (int i = t; i < it.n_nbd; i += 256) {
            const int mk = mark[i];
            nu += mk != -1;
            nz += mk == -2;
        }
        __shared__ SetRec ss[4];
        __shared__ int sc[2][4];
        psx::wave_fold_set(a);
        nu = __ockl_wfred_add_i32(nu);  // DPP wave sums
        nz = __ockl_wfred_add_i32(nz);
        if ((t & 63) == 0) {
            ss[t >> 6] = a;
            sc[0][t >> 6] = nu;
            sc[1][t >> 6] = nz;
        }
        __syncthreads();
        if (t == 0) {
            SetRec g = *sacc;
            for (int q = 0; q < 4; q++) psx::fold_set(g, ss[q]);
            const int unseen = sc[0][0] + sc[0][1] + sc[0][2] + sc[0][3];
            const int nn = sc[1][0] + sc[1][1] + sc[1][2] + sc[1][3] + cnt[kCurNull];
            if (nn > 0 && it.rank == 0) {
                SetRec x = null1;  // null1 scaled to nn null configurations
                x.tot *= nn;
                x.nc0 *= nn;
                x.nc1 *= nn;
                x.npat *= nn;
                psx::fold_set(g, x);
            }
            *sacc = g;
            *sacc_host = g;
            cnt_host[kUnseen] = unseen;
            cnt_host[kNulls] = nn;
            cnt_host[kCurPos] = cnt[kCurPos];
            cnt_host[kCurNull] = cnt[kCurNull];
        }
        return;
    }
    if (mode == 0) return;
    const int i = (b - it.U - 1) * 256 + t;
    if (i >= it.n_nbd) return;
    const int mk = mark[i];
    if (mk == -1) return;  // seen: its weight was written by k_sss_eval
    const double v = mk == -2 ? it.null_score : score[mk];
    int row[PSX_KMAX];
    const int nr = nbd_row(it, i, row);
    unsigned long long klo, khi;
    pack_key(row, nr, klo, khi);
    map_insert(T, mask, klo, khi, v);
    lk_host[i] = v;
}

// the map at twice the capacity: re-insert every entry
__global__ void k_map_rehash(const MapEntry* __restrict__ old, size_t n, MapEntry* __restrict__ T,
                             unsigned long long mask) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && old[i].state) map_insert(T, mask, old[i].lo, old[i].hi, old[i].score);
}

// Sharded walk, device exchange (psx_run_sss_sharded_dev): this rank's
// all-gather send block [m, s of its running normaliser, its slice's item
// scores, zero padding to `per`], built on the device after the post ...
__global__ void k_sss_pack(const SetRec* __restrict__ sacc, const double* __restrict__ score, int lo, int n, int per,
                           double* __restrict__ snd) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) {
        snd[0] = (double)sacc->m;
        snd[1] = sacc->tot;
    }
    if (i < per) snd[2 + i] = i < n ? score[lo + i] : 0.0;
}
// ... and, after the caller's stream-ordered all-gather, every rank's scores to
// their items (full) and every rank's normaliser to pinned host memory
__global__ void k_sss_unpack(const double* __restrict__ rcv, int world, int n_items, int per,
                             double* __restrict__ full, double* __restrict__ hnorm) {
    const int r = blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x;
    const double* q = rcv + (size_t)r * (per + 2);
    const int rlo = (int)((int64_t)n_items * r / world), rn = (int)((int64_t)n_items * (r + 1) / world) - rlo;
    if (i < rn) full[rlo + i] = q[2 + i];
    if (i == 0) {
        hnorm[2 * r] = q[0];
        hnorm[2 * r + 1] = q[1];
    }
}

struct SssDev {
    MapEntry* T = nullptr;
    size_t cap = 0, used = 0;
    size_t nmax = 0, nmax_full = 0;  // item capacity of the per-item arrays (full / hscore)
    // (start, stop) event pairs around the evals, read kRingE iterations later
    // (by then complete) instead of once per iteration
    static constexpr int kRingE = 8;
    static constexpr int kEvEvery = 4;  // start events on every 4th iteration (kRingE a multiple)
    hipEvent_t ev[2 * kRingE] = {};
    int* rows = nullptr;      // per item: its set (evaluated items)
    int* mark = nullptr;      // per neighbour: -1 seen, -2 unseen null, else its item
    int* cnt = nullptr;
    double* full = nullptr;   // per item: every rank's scores (world > 1)
    double* lk = nullptr;     // pinned host: every neighbour's score
    SetRec* shost = nullptr;  // pinned host: the scalars after the iteration
    int* hcnt = nullptr;      // pinned host: the counters
    unsigned long long* hmark = nullptr;  // pinned host: per neighbour, its mark word (one rank)
    unsigned long long* trace = nullptr;  // PSX_SSS_TRACE: item 1's eval phase clocks (pinned host)
    double* hscore = nullptr; // pinned host: gathered item scores (world > 1)
    double* dx = nullptr;     // device exchange: send block | receive blocks (world > 1)
    size_t cap_dx = 0;
    double* hnorm = nullptr;  // pinned host: every rank's normaliser (m, s) (device exchange)
    int cap_hnorm = 0;
    unsigned int seq = 0;     // the last iteration tag of the mark words (never 0)
    ~SssDev() {
        psx::dfree(T);
        psx::dfree(rows);
        psx::dfree(mark);
        psx::dfree(cnt);
        psx::dfree(full);
        if (lk) psx::hfree(lk);
        if (shost) psx::hfree(shost);
        if (hcnt) psx::hfree(hcnt);
        if (hmark) psx::hfree(hmark);
        if (hscore) psx::hfree(hscore);
        if (trace) psx::hfree(trace);
        psx::dfree(dx);
        if (hnorm) psx::hfree(hnorm);
        for (int i = 0; i < 2 * kRingE; i++)
            if (ev[i]) hipEventDestroy(ev[i]);
    }
};

void sss_release(SssDev* d) { delete d; }

// the walk's workspace for up to nmax items per iteration (grown, never shrunk;
// the map is cleared for every walk)
int sss_workspace(psx_engine* e, size_t nmax, int world, hipStream_t s) {
    if (!e->sss) e->sss = new SssDev();
    SssDev& D = *e->sss;
    if (!D.cnt) {
        for (int i = 0; i < 2 * SssDev::kRingE; i++) HIPCHK(hipEventCreate(&D.ev[i]));
        HIPCHK(psx::dmalloc(&D.cnt, kNCnt * sizeof(int)));
        HIPCHK(psx::hmalloc(reinterpret_cast<void**>(&D.shost), sizeof(SetRec)));
        HIPCHK(psx::hmalloc(reinterpret_cast<void**>(&D.hcnt), kNCnt * sizeof(int)));
        if (std::getenv("PSX_SSS_TRACE")) {
            HIPCHK(psx::hmalloc(reinterpret_cast<void**>(&D.trace), 8 * sizeof(unsigned long long)));
            std::memset(D.trace, 0, 8 * sizeof(unsigned long long));
        }
    }
    if (D.nmax < nmax) {
        psx::dfree(D.rows); psx::dfree(D.mark);
        if (D.lk) psx::hfree(D.lk);
        if (D.hmark) psx::hfree(D.hmark);
        D.rows = D.mark = nullptr;
        D.hmark = nullptr;
        D.lk = nullptr;
        HIPCHK(psx::dmalloc(&D.rows, nmax * PSX_KMAX * sizeof(int)));
        HIPCHK(psx::dmalloc(&D.mark, nmax * sizeof(int)));
        // coherent: the eval's weight / mark-word hand-off (publish_mark) relies on
        // device stores reaching host memory in acknowledgement order
        HIPCHK(psx::hmalloc_coherent_raw(reinterpret_cast<void**>(&D.lk), nmax * sizeof(double)));
        HIPCHK(psx::hmalloc_coherent_raw(reinterpret_cast<void**>(&D.hmark), nmax * sizeof(unsigned long long)));
        std::memset(D.hmark, 0, nmax * sizeof(unsigned long long));  // tag 0: no iteration
        D.nmax = nmax;
    }
    if (world > 1 && D.nmax_full < nmax) {
        psx::dfree(D.full);
        if (D.hscore) psx::hfree(D.hscore);
        D.full = nullptr;
        D.hscore = nullptr;
        HIPCHK(psx::dmalloc(&D.full, nmax * sizeof(double)));
        HIPCHK(psx::hmalloc(reinterpret_cast<void**>(&D.hscore), nmax * sizeof(double)));
        D.nmax_full = nmax;
    }
    size_t cap = 1 << 16;
    while (cap < 4 * nmax) cap <<= 1;
    if (D.cap < cap) {
        psx::dfree(D.T);
        D.T = nullptr;
        HIPCHK(psx::dmalloc(&D.T, cap * sizeof(MapEntry)));
        D.cap = cap;
    }
    HIPCHK(hipMemsetAsync(D.T, 0, D.cap * sizeof(MapEntry), s));
    D.used = 0;
    return 0;
}

int run_sss(psx_engine* e, psx_allgather_fn allgather, psx_allgather_dev_fn dgather, void* ctx,
            int32_t* iterations_out) {
    HIPCHK(hipSetDevice(e->dev));
    e->stat_fresh = false;  // status changes: psx_sync reads it out again
    const bool sharded = allgather || dgather;
    const int rank = sharded ? e->rank : 0, world = sharded ? e->world : 1;
    int rc;
    if ((rc = reset_acc(e))) return rc;
    std::memset(&e->timing, 0, sizeof(e->timing));
    const int U = e->U, C = e->maxc;
    if (C > PSX_KMAX) return fail(PSX_ERANGE, "SSS max_causal > 6");
    if (U > kKeyMaxU) return fail(PSX_ERANGE, "SSS: more union SNPs than the set key holds");
    const int stride = std::max(C, 1);
    // the most items of an iteration: the current configuration + the largest
    // neighbourhood (k = C: swaps C (U - C), minus C; k < C: + U - k plus sets)
    const size_t nmax = (size_t)C * U + C + U + 2;
    const auto tw = std::chrono::steady_clock::now();
    if ((rc = sss_workspace(e, nmax, world, e->stream))) return rc;
    const double ws_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tw).count();
    SssDev& D = *e->sss;
    if ((rc = ensure(e->dsrec, e->cap_srec, nmax))) return rc;
    if ((rc = ensure(e->dmrec, e->cap_mrec, nmax * stride))) return rc;
    if ((rc = ensure(e->dscore, e->cap_score, nmax))) return rc;
    const SetRec null1 = null_rec(e, 1.0);
    std::mt19937 gen(12345);
    int cur[PSX_KMAX] = {0, 0, 0, 0, 0, 0}, k = 0;  // the current configuration, ascending
    double old_sum = 0;
    int iter;
    double kms = 0;
    int ksamples = 0;
    auto t0 = std::chrono::steady_clock::now();
    std::vector<double> pr;
    // diagnostics (PSX_SSS_PROFILE): host time per phase of the walk, on stderr
    static const bool prof = std::getenv("PSX_SSS_PROFILE") != nullptr;
    // PSX_SSS_FLAG=0 (A/B): wait for the eval's stop event before reading the mark words
    const char* fw = std::getenv("PSX_SSS_FLAG");
    const bool event_wait = fw && fw[0] == '0';
    double ph[4] = {0, 0, 0, 0};  // launch, wait for the eval, sampling, wait for the post
    double tph[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // PSX_SSS_TRACE: item 1's eval phases
    auto tick = [&](int i, std::chrono::steady_clock::time_point& t) {
        if (!prof) return;
        const auto n = std::chrono::steady_clock::now();
        ph[i] += std::chrono::duration<double, std::micro>(n - t).count();
        t = n;
    };
    for (iter = 0; iter < 1000; iter++) {
        SssIter it;
        for (int j = 0; j < PSX_KMAX; j++) it.cur[j] = j < k ? cur[j] : -1;
        it.k = k;
        it.U = U;
        it.stride = stride;
        it.num_zero = (U - k) * k;
        it.num_minus = k;
        it.num_plus = k < C ? U - k : 0;
        it.n_nbd = it.num_zero + it.num_minus + it.num_plus;
        it.rank = rank;
        it.world = world;
        it.null_score = e->K + e->L0;
        it.trace = D.trace;
        if (++D.seq == 0) D.seq = 1;  // (tag 0 is a word no iteration wrote)
        it.seq = D.seq;
        const int n_nbd = it.n_nbd, n_items = n_nbd + 1;
        // this rank's contiguous slice of the items
        const int lo = (int)((int64_t)n_items * rank / world), hi = (int)((int64_t)n_items * (rank + 1) / world);
        // the map stays at load <= 1/2 (every neighbour may be new)
        if (2 * (D.used + (size_t)n_nbd + 1) > D.cap) {
            size_t nc = D.cap;
            while (2 * (D.used + (size_t)n_nbd + 1) > nc) nc <<= 1;
            MapEntry* nt = nullptr;
            HIPCHK(psx::dmalloc(&nt, nc * sizeof(MapEntry)));
            HIPCHK(hipMemsetAsync(nt, 0, nc * sizeof(MapEntry), e->stream));
            hipLaunchKernelGGL(k_map_rehash, dim3((unsigned)((D.cap + 255) / 256)), dim3(256), 0, e->stream, D.T,
                               D.cap, nt, (unsigned long long)(nc - 1));
            HIPCHK(hipGetLastError());
            HIPCHK(hipStreamSynchronize(e->stream));
            psx::dfree(D.T);
            D.T = nt;
            D.cap = nc;
        }
        const unsigned long long mask = D.cap - 1;
        auto tp = std::chrono::steady_clock::now();
        // plain event records around the eval (the stop event is what the host
        // waits on): hipExtLaunchKernelGGL's in-packet events cost the host ~12 us
        // more per launch here (profiles/archive/r03i_sss_host_phases.txt)
        // The start event only on every kEvEvery-th iteration (an event record is
        // ~1-2 us of host time): the eval time is sampled there and scaled to all
        // iterations; the stop event (the host's wait) on every one.
        hipEvent_t* evp = D.ev + 2 * (iter % SssDev::kRingE);
        const bool timed = iter % SssDev::kEvEvery == 0;
        if (iter >= SssDev::kRingE && (iter - SssDev::kRingE) % SssDev::kEvEvery == 0) {  // kRingE iterations ago
            float ms = 0;
            HIPCHK(hipEventElapsedTime(&ms, evp[0], evp[1]));
            kms += ms;
            ksamples++;
        }
        if (timed) HIPCHK(hipEventRecord(evp[0], e->stream));
        hipLaunchKernelGGL(C <= 5 ? k_sss_eval<5> : k_sss_eval<PSX_KMAX>, dim3((unsigned)n_items), dim3(64), 0,
                           e->stream, e->dp, it, D.T, mask, lo, hi,
                           D.rows, D.mark, D.cnt, D.lk, e->dsrec, e->dmrec, e->dscore, world == 1 ? D.hmark : nullptr);
        // (the stop event: the host's wait without the completion word, else only
        // the sampled eval time)
        const bool poll = world == 1 && !event_wait;
        if (timed || !poll) HIPCHK(hipEventRecord(evp[1], e->stream));
        const unsigned post_blocks = (unsigned)(U + 1 + (world == 1 ? (n_nbd + 255) / 256 : 0));
        hipLaunchKernelGGL(k_sss_post, dim3(post_blocks), dim3(256), 0, e->stream, it, lo, hi, D.rows, D.mark, D.cnt,
                           e->dmrec, e->dsrec, e->dscore, null1, e->dacc, e->dsacc, D.shost, D.hcnt, D.T, mask,
                           world == 1 ? 1 : 0, D.lk);
        HIPCHK(hipGetLastError());
        int unseen = 0;
        double sss_sum = 0.0;
        if (world == 1) {
            // One rank: the eval wrote every neighbour's weight and mark to pinned
            // host memory, so the host samples the next configuration while the
            // GPU folds the records and inserts the new scores (k_sss_post); it
            // waits for the post only where the stop test needs the normaliser.
            tick(0, tp);
            if (!poll) HIPCHK(hipEventSynchronize(evp[1]));
            // each neighbour's mark word once it carries this iteration's tag (its
            // weight was acknowledged before it).  An idle stream (eval and post
            // done) with a word still missing is an error.
            const unsigned long long tag = (unsigned long long)it.seq << 32;
            unsigned spins = 0;
            for (int i = 0; i < n_nbd; i++) {
                unsigned long long w;
                while (((w = __atomic_load_n(D.hmark + i, __ATOMIC_ACQUIRE)) & ~0xffffffffULL) != tag) {
                    if ((++spins & 4095) == 0) {
                        const hipError_t q = hipStreamQuery(e->stream);
                        if (q == hipSuccess) {
                            w = __atomic_load_n(D.hmark + i, __ATOMIC_ACQUIRE);
                            if ((w & ~0xffffffffULL) == tag) break;
                            return fail(PSX_EHIP, "SSS: the eval finished without neighbour " + std::to_string(i) +
                                                      "'s mark word");
                        }
                        if (q != hipErrorNotReady) HIPCHK(q);
                    }
                    __builtin_ia32_pause();
                }
                unseen += (int)(unsigned int)w != -1;
            }
            tick(1, tp);
            if (D.trace) {  // item 1's eval phases (100 MHz clock), after the eval's end
                HIPCHK(hipStreamSynchronize(e->stream));
                const unsigned long long* q = D.trace;
                if (q[7]) {
                    for (int x = 0; x < 7; x++) tph[x] += (double)(q[x + 1] - q[x]) * 0.01;
                    tph[7] += 1;
                    D.trace[7] = 0;
                }
            }
        } else if (dgather) {
            // the exchange on the device: pack -> the caller's stream-ordered
            // all-gather -> unpack -> insert, then one synchronisation (no score
            // copies through the host, no host bytes for the callback)
            const int per = (n_items + world - 1) / world, wd = 2 + per;
            if ((size_t)wd * (world + 1) > D.cap_dx) {
                psx::dfree(D.dx);
                D.dx = nullptr;
                D.cap_dx = 0;
                HIPCHK(psx::dmalloc(&D.dx, sizeof(double) * (size_t)wd * (world + 1)));
                D.cap_dx = (size_t)wd * (world + 1);
            }
            if (2 * world > D.cap_hnorm) {
                if (D.hnorm) psx::hfree(D.hnorm);
                D.hnorm = nullptr;
                HIPCHK(psx::hmalloc(&D.hnorm, sizeof(double) * 2 * world));
                D.cap_hnorm = 2 * world;
            }
            double* const snd = D.dx;
            double* const rcv = D.dx + wd;
            hipLaunchKernelGGL(k_sss_pack, dim3((unsigned)((per + 255) / 256)), dim3(256), 0, e->stream, e->dsacc,
                               e->dscore, lo, hi - lo, per, snd);
            HIPCHK(hipGetLastError());
            if (dgather(ctx, snd, rcv, (int64_t)wd * (int64_t)sizeof(double), e->stream))
                return fail(PSX_EEXCHANGE, "SSS device all-gather callback failed");
            hipLaunchKernelGGL(k_sss_unpack, dim3((unsigned)((per + 255) / 256), (unsigned)world), dim3(256), 0,
                               e->stream, rcv, world, n_items, per, D.full, D.hnorm);
            hipLaunchKernelGGL(k_sss_post, dim3((unsigned)(U + 1 + (n_nbd + 255) / 256)), dim3(256), 0, e->stream, it,
                               lo, hi, D.rows, D.mark, D.cnt, e->dmrec, e->dsrec, D.full, null1, (Acc5*)nullptr,
                               (SetRec*)nullptr, (SetRec*)nullptr, (int*)nullptr, D.T, mask, 2, D.lk);
            HIPCHK(hipGetLastError());
            HIPCHK(hipStreamSynchronize(e->stream));
            unseen = D.hcnt[kUnseen];
            double mx = -INFINITY;
            std::vector<double> part(world, 0.0);
            for (int r = 0; r < world; r++) {
                part[r] = logval(e, (int32_t)D.hnorm[2 * r], D.hnorm[2 * r + 1]);
                if (part[r] != 0.0) mx = std::max(mx, part[r]);
            }
            double acc = 0.0;  // the ranks' normalisers, combined in rank order
            for (int r = 0; r < world; r++)
                if (part[r] != 0.0) acc += std::exp(part[r] - mx);
            sss_sum = acc > 0 ? mx + std::log(acc) : 0.0;
        } else {
            HIPCHK(hipStreamSynchronize(e->stream));
            unseen = D.hcnt[kUnseen];
            // one all-gather: [normaliser (m, s), the slice's item scores]; then
            // every rank inserts all scores and writes the sampling weights
            const size_t per = ((size_t)n_items + world - 1) / world, wd = 2 + per;
            std::vector<double> snd(wd, 0.0), rcv(wd * world, 0.0);
            if (hi > lo)
                HIPCHK(hipMemcpy(snd.data() + 2, e->dscore + lo, (size_t)(hi - lo) * sizeof(double),
                                 hipMemcpyDeviceToHost));
            snd[0] = (double)D.shost->m;
            snd[1] = D.shost->tot;
            if (allgather(ctx, snd.data(), rcv.data(), (int64_t)(wd * sizeof(double))))
                return fail(PSX_EEXCHANGE, "SSS all-gather callback failed");
            double mx = -INFINITY;
            std::vector<double> part(world, 0.0);
            for (int r = 0; r < world; r++) {
                const double* q = rcv.data() + (size_t)r * wd;
                const size_t rlo = (size_t)n_items * r / world, rn = (size_t)n_items * (r + 1) / world - rlo;
                std::copy(q + 2, q + 2 + rn, D.hscore + rlo);
                part[r] = logval(e, (int32_t)q[0], q[1]);
                if (part[r] != 0.0) mx = std::max(mx, part[r]);
            }
            double acc = 0.0;  // the ranks' normalisers, combined in rank order
            for (int r = 0; r < world; r++)
                if (part[r] != 0.0) acc += std::exp(part[r] - mx);
            sss_sum = acc > 0 ? mx + std::log(acc) : 0.0;
            HIPCHK(hipMemcpyAsync(D.full, D.hscore, (size_t)n_items * sizeof(double), hipMemcpyHostToDevice, e->stream));
            // the insert blocks alone (block indices past U)
            hipLaunchKernelGGL(k_sss_post, dim3((unsigned)(U + 1 + (n_nbd + 255) / 256)), dim3(256), 0, e->stream, it,
                               lo, hi, D.rows, D.mark, D.cnt, e->dmrec, e->dsrec, D.full, null1, (Acc5*)nullptr,
                               (SetRec*)nullptr, (SetRec*)nullptr, (int*)nullptr, D.T, mask, 2, D.lk);
            HIPCHK(hipGetLastError());
            HIPCHK(hipStreamSynchronize(e->stream));
        }
        D.used += (size_t)unseen;
        if (unseen == 0) break;                                                          // :260-263
        // (one rank: the sampling below runs first and is dropped when the stop
        // test of sss_postcal.cpp:265-270 ends the walk — it only advances gen)
        const double* lk = D.lk;
        double wz = 0, wm = 0, wp = 0;
        size_t zs = n_nbd, ms = n_nbd, ps = n_nbd;
        // each group: discrete_distribution(exp(lk - max))(gen) and the weights'
        // sum (accumulate), the draw restated without the distribution's vectors
        // (psx_sample.h: bit-identical partial sums, the same index)
        auto group = [&](int b, int en, double& wsum, size_t& smp) {
            pr.resize((size_t)(en - b));
            double mx = *std::max_element(lk + b, lk + en);
            // (slicing these exps over spinning host threads measured slower: the
            // serial loop takes ~5 us at 1,000 neighbours, profiles/archive/r03v_sss_threads.txt)
            double s = 0.0;
            for (int ii = b; ii < en; ii++) s += (pr[ii - b] = std::exp(lk[ii] - mx));
            smp = psx::discrete_draw(pr.data(), pr.size(), s, gen);
            wsum = s;
        };
        if (it.num_zero != 0) group(0, it.num_zero, wz, zs);                               // :296-306
        if (it.num_minus != 0) group(it.num_zero, it.num_zero + it.num_minus, wm, ms);     // :307-317
        if (it.num_plus != 0) group(it.num_zero + it.num_minus, n_nbd, wp, ps);            // :318-328
        const double w3[3] = {wz, wm, wp};                                                 // :330-343
        size_t idx = psx::discrete_draw(w3, 3, (0.0 + wz + wm) + wp, gen), fin = 0;
        switch (idx) {
            case 0: fin = zs; break;
            case 1: fin = ms + it.num_zero; break;
            case 2: fin = ps + it.num_zero + it.num_minus; break;
        }
        // the chosen neighbour becomes the current configuration (host copy of nbd_row)
        {
            const int i = (int)fin;
            int x = -1, skip = -1, n;
            if (i < it.num_zero) { skip = i % k; x = i / k; n = k; }
            else if (i < it.num_zero + it.num_minus) { skip = i - it.num_zero; n = k - 1; }
            else { x = i - it.num_zero - it.num_minus; n = k + 1; }
            if (x >= 0)
                for (int j = 0; j < k; j++)
                    if (cur[j] <= x) x++;
            int nxt[PSX_KMAX], m = 0;
            bool put = x < 0;
            for (int j = 0; j < k; j++) {
                if (j == skip) continue;
                if (!put && x < cur[j]) { nxt[m++] = x; put = true; }
                nxt[m++] = cur[j];
            }
            if (!put) nxt[m++] = x;
            std::copy(nxt, nxt + n, cur);
            k = n;
        }
        tick(2, tp);
        if (world == 1 && iter >= 99) {  // the normaliser of this iteration (k_sss_post)
            HIPCHK(hipStreamSynchronize(e->stream));
            tick(3, tp);
            sss_sum = logval(e, D.shost->m, D.shost->tot);
        }
        if (iter >= 100 && (1 - std::exp(old_sum - sss_sum)) <= 0.001) break;            // :265-270
        old_sum = sss_sum;
    }
    HIPCHK(hipStreamSynchronize(e->stream));  // the last iteration's post (one rank: not waited for in the loop)
    auto t1 = std::chrono::steady_clock::now();
    {  // the evals still in the event ring (iterations 0..iter ran; `iter` itself when it broke out)
        const int ran = std::min(iter + 1, 1000);
        for (int q = std::max(0, ran - SssDev::kRingE); q < ran; q++) {
            if (q % SssDev::kEvEvery) continue;
            float ms = 0;
            HIPCHK(hipEventElapsedTime(&ms, D.ev[2 * (q % SssDev::kRingE)], D.ev[2 * (q % SssDev::kRingE) + 1]));
            kms += ms;
            ksamples++;
        }
        if (ksamples) kms *= (double)ran / ksamples;  // the sampled evals' mean, over every iteration
    }
    if (D.trace && tph[7] > 0)
        fprintf(stderr, "[psx sss] item-1 eval us: row+probe %.2f, stage %.2f, subsets %.2f, patterns %.2f, "
                "reductions %.2f, records %.2f (%.0f evals)\n", tph[0] / tph[7], tph[1] / tph[7], tph[2] / tph[7],
                tph[3] / tph[7], tph[4] / tph[7], (tph[5] + tph[6]) / tph[7], tph[7]);
    if (prof)
        fprintf(stderr, "[psx sss] %d iterations, host us per iteration: launch %.1f, wait eval %.1f, sampling %.1f, "
                "wait post %.1f; workspace %.0f us\n", iter, ph[0] / std::max(iter, 1), ph[1] / std::max(iter, 1),
                ph[2] / std::max(iter, 1), ph[3] / std::max(iter, 1), ws_us);
    if (iterations_out) *iterations_out = iter;
    e->timing.sweep_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    e->timing.kernel_ms = kms;
    SetRec s;
    HIPCHK(hipMemcpy(&s, e->dsacc, sizeof(SetRec), hipMemcpyDeviceToHost));
    e->timing.configs = (uint64_t)(s.npat + 0.5);
    return 0;
}
}  // namespace

int psx_run_sss(psx_engine* e, int32_t* iterations_out) {
    return run_sss(e, nullptr, nullptr, nullptr, iterations_out);
}

int psx_run_sss_sharded(psx_engine* e, psx_allgather_fn allgather, void* ctx, int32_t* iterations_out) {
    if (!allgather && e->world > 1) return fail(PSX_EINVAL, "psx_run_sss_sharded: no all-gather callback");
    return run_sss(e, allgather, nullptr, ctx, iterations_out);
}

int psx_run_sss_sharded_dev(psx_engine* e, psx_allgather_dev_fn allgather, void* ctx, int32_t* iterations_out) {
    if (!allgather && e->world > 1) return fail(PSX_EINVAL, "psx_run_sss_sharded_dev: no all-gather callback");
    return run_sss(e, nullptr, allgather, ctx, iterations_out);
}

int psx_get_accum(psx_engine* e, psx_accum* out) {
    HIPCHK(hipSetDevice(e->dev));
    std::vector<Acc5> a(e->U);
    SetRec s;
    HIPCHK(hipMemcpyAsync(a.data(), e->dacc, sizeof(Acc5) * e->U, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(&s, e->dsacc, sizeof(SetRec), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    for (int u = 0; u < e->U; u++) {
        for (int st = 0; st < 2; st++) {
            int l = e->u2l[st * e->U + u];
            if (l < 0) continue;
            double v = st == 0 ? logval(e, a[u].mP, a[u].post0) : logval(e, a[u].mP, a[u].post1);
            if (out->post) out->post[(st ? e->m[0] : 0) + l] = v;
        }
        if (out->shared) out->shared[u] = logval(e, a[u].mP, a[u].shared);
        if (out->shared_ll) out->shared_ll[u] = logval(e, a[u].mS, a[u].sll);
        if (out->notshared_ll) out->notshared_ll[u] = logval(e, a[u].mN, a[u].nsll);
    }
    if (out->no_causal) {
        out->no_causal[0] = logval(e, s.m0, s.nc0);
        out->no_causal[1] = logval(e, s.m1, s.nc1);
    }
    out->total = logval(e, s.m, s.tot);
    out->n_configs = (uint64_t)(s.npat + 0.5);
    return 0;
}

int64_t psx_partials_bytes(psx_engine* e) { return (int64_t)(sizeof(Acc5) * ((size_t)e->ldg + 2)); }

int psx_export_partials(psx_engine* e, void* dst) {
    HIPCHK(hipSetDevice(e->dev));
    // per-SNP slots, the SetRec slot and the PlanTag are contiguous: the image is one copy
    // a copy kernel: it follows the merge kernels on the stream without the
    // blit path's extra dependency packets (hipMemcpyAsync D2D: +6 us gap, r06a)
    const size_t n16 = sizeof(Acc5) * ((size_t)e->ldg + 2) / 16;
    static_assert(sizeof(Acc5) % 16 == 8 || sizeof(Acc5) % 16 == 0, "image of whole 8-byte words");
    if ((reinterpret_cast<uintptr_t>(dst) & 15) || (sizeof(Acc5) * ((size_t)e->ldg + 2)) % 16) {
        HIPCHK(hipMemcpyAsync(dst, e->dacc, sizeof(Acc5) * ((size_t)e->ldg + 2), hipMemcpyDeviceToDevice, e->stream));
    } else {
        hipLaunchKernelGGL(k_copy_image, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, e->stream,
                           reinterpret_cast<const int4*>(e->dacc), n16, reinterpret_cast<int4*>(dst));
        HIPCHK(hipGetLastError());
    }
    if (!e->external_stream) HIPCHK(hipStreamSynchronize(e->stream));
    return 0;
}

int psx_partials_device_ptr(psx_engine* e, void** device_ptr) {
    if (!e || !device_ptr) return fail(PSX_EINVAL, "bad argument");
    *device_ptr = e->dacc;  // slots 0 .. ldg + 1: the exported image
    return 0;
}

int psx_set_stream(psx_engine* e, void* stream) {
    HIPCHK(hipSetDevice(e->dev));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (stream == nullptr) {
        e->stream = e->own_stream;
        e->external_stream = false;
    } else {
        e->stream = (hipStream_t)stream;
        e->external_stream = true;
    }
    return 0;
}

int psx_merge_partials(psx_engine* e, const void* src, int32_t count) {
    HIPCHK(hipSetDevice(e->dev));
    if (count < 1) return fail(PSX_EINVAL, "count < 1");
    // one-wave blocks: they take the first wave slots a running sweep frees
    hipLaunchKernelGGL(k_merge_partials, dim3((e->U + 63) / 64 + 1), dim3(64), 0, e->stream, (const Acc5*)src, e->U,
                       e->ldg, count, e->dacc, e->dsacc, e->dflag, (const int*)e->plans.d_redo,
                       reinterpret_cast<int*>(e->hstat));
    HIPCHK(hipGetLastError());
    e->stat_fresh = true;  // k_merge_partials wrote the status to hstat
    if (e->external_stream) return 0;  // a tag mismatch is reported by psx_sync
    return check_plan_mismatch(e);
}

int psx_fold_partials_host(const void* src, int32_t count, int64_t image_bytes, void* dst) {
    if (count < 1 || image_bytes < (int64_t)(3 * sizeof(Acc5)) || image_bytes % (int64_t)sizeof(Acc5) != 0)
        return fail(PSX_EINVAL, "bad partial image size");
    const size_t n = (size_t)image_bytes / sizeof(Acc5);  // ldg Acc5 slots + 1 SetRec slot + 1 PlanTag slot
    const Acc5* parts = (const Acc5*)src;
    const PlanTag& t0 = *reinterpret_cast<const PlanTag*>(parts + n - 1);
    for (int r = 0; r < count; r++) {
        const PlanTag& t = *reinterpret_cast<const PlanTag*>(parts + (size_t)r * n + n - 1);
        if (t.magic != kPlanMagic || t.hash != t0.hash || t.world != count || t.rank != r)
            return fail(PSX_EINVAL, "partial images are not shards 0.." + std::to_string(count - 1) +
                                        " of one plan (PlanTag of rank " + std::to_string(r) + ")");
    }
    std::vector<Acc5> out(n);
    std::memset(out.data(), 0, n * sizeof(Acc5));
    for (size_t u = 0; u + 2 < n; u++) {
        Acc5 a = {0, 0, 0, 0, 0.0, 0.0, 0.0, 0.0, 0.0};
        for (int r = 0; r < count; r++) psx::fold_acc(a, parts[(size_t)r * n + u]);
        out[u] = a;
    }
    SetRec s = psx::set_zero();
    for (int r = 0; r < count; r++) psx::fold_set(s, *reinterpret_cast<const SetRec*>(parts + (size_t)r * n + n - 2));
    std::memcpy(&out[n - 2], &s, sizeof(SetRec));
    PlanTag t = t0;  // the fold is a whole-plan image of world 1
    t.world = 1;
    t.rank = 0;
    std::memcpy(&out[n - 1], &t, sizeof(PlanTag));
    std::memcpy(dst, out.data(), n * sizeof(Acc5));
    return 0;
}

int psx_shard_stats(const psx_problem* p, int32_t k, int32_t rank, int32_t world, uint64_t* union_sets,
                    double* configs) {
    if (!p || p->n_studies != 2 || k < 1 || world < 1 || rank < 0 || rank >= world)
        return fail(PSX_EINVAL, "bad arguments");
    const int U = p->n_union;
    const int ldg = (U + 63) / 64 * 64;
    std::vector<unsigned char> pres(ldg, 0);
    for (int s = 0; s < 2; s++)
        for (int u = 0; u < U; u++)
            if (p->union_to_local[s * U + u] >= 0) pres[u] |= (unsigned char)(1 << s);
    double sets = 0, cfg = 0, bytes = 0;
    if (psx::sweep_supports(k, U)) {
        std::vector<psx::PlanUnit> mine;
        int ca = 0;
        if (k == 3)  // the fast kernel's decomposition (the exact rerun covers the same sets)
            psx::plan_units3c(U, ldg, rank, world, pres.data(), mine, ca, sets, cfg, bytes);
        else
            psx::plan_units(k, U, ldg, rank, world, pres.data(), mine, ca, sets, cfg, bytes);
    } else {
        uint64_t total = choose_u64(U, k);
        uint64_t lo = total * (uint64_t)rank / world, hi = total * (uint64_t)(rank + 1) / world;
        if (lo < hi) {
            std::vector<int> c(k);
            unrank_lex(lo, U, k, c.data());
            for (uint64_t r = lo; r < hi; r++) {
                double w = 1;
                for (int j = 0; j < k; j++) w *= (pres[c[j]] == 3) ? 3.0 : 1.0;
                sets += 1;
                cfg += w;
                next_lex(c.data(), U, k);
            }
        }
    }
    if (union_sets) *union_sets = (uint64_t)(sets + 0.5);
    if (configs) *configs = cfg;
    return 0;
}

int psx_plan_csr_selftest(int32_t n_union, const uint8_t* presence, int32_t k, int32_t rank, int32_t world,
                          int32_t variant, int device, int64_t* mismatches, int64_t* records) {
    if (n_union < 3 || (k != 2 && k != 3) || (variant && k != 3) || world < 1 || rank < 0 || rank >= world ||
        !mismatches || !records)
        return fail(PSX_EINVAL, "bad arguments");
    int rc;
    if ((rc = gpu_ready(device))) return rc;
    const int ldg = (n_union + 63) / 64 * 64;
    std::vector<unsigned char> pres(ldg, 0);
    for (int u = 0; u < n_union; u++) pres[u] = presence ? presence[u] : 3;
    long bad = 0, nrec = 0;
    if (psx::plan_csr_selftest(n_union, pres.data(), k, rank, world, variant, &bad, &nrec))
        return fail(PSX_EHIP, psx::sweep_error());
    *mismatches = bad;
    *records = nrec;
    return 0;
}

int psx_plan_build_ms(int32_t n_union, int32_t k, int32_t rank, int32_t world, double* ms, int32_t* n_units,
                      int64_t* n_records) {
    if (n_union < 3 || (k != 2 && k != 3) || world < 1 || rank < 0 || rank >= world || !ms || !n_units || !n_records)
        return fail(PSX_EINVAL, "bad arguments");
    long nr = 0;
    int nu = 0;
    if (psx::plan_host_ms(n_union, k, rank, world, ms, &nu, &nr)) return fail(PSX_EINVAL, psx::sweep_error());
    *n_units = nu;
    *n_records = nr;
    return 0;
}

int psx_plan_units_k3(int32_t n_union, int32_t rank, int32_t world, int32_t* units, int32_t cap) {
    if (n_union < 3 || world < 1 || rank < 0 || rank >= world || cap < 0) return fail(PSX_EINVAL, "bad arguments");
    const int U = n_union, ldg = (U + 63) / 64 * 64;
    std::vector<unsigned char> pres(ldg, 3);
    std::vector<psx::PlanUnit> mine;
    int ca = 0;
    double sets = 0, cfg = 0, bytes = 0;
    psx::plan_units3c(U, ldg, rank, world, pres.data(), mine, ca, sets, cfg, bytes);
    for (int i = 0; i < (int)mine.size() && i < cap; i++) {
        const psx::PlanUnit& u = mine[i];
        int32_t* o = units + 4 * (size_t)i;
        o[0] = u.a0;
        o[1] = u.a1;
        o[2] = u.B | (u.j0 << 16);
        o[3] = u.T | (u.j1 << 16);
    }
    return (int)mine.size();
}

int psx_get_timing(psx_engine* e, psx_timing* t) {
    *t = e->timing;
    return 0;
}

}  // extern "C"
