// psx_sweep.hip — tiled exhaustive sweep (levels k = 2, 3) and record merges.
//
// Work decomposition (DESIGN.md "Sweep kernel"): union indices are cut into
// 64-wide blocks.  A unit is (a-chunk, B, T): one wave, lane t owns
// b = 64B + t, and the wave walks the 64x64 (b, c) tile of T diagonally —
// at step j lane t takes c = 64T + ((t + j) & 63) — so at every step the 64
// lanes touch 64 distinct c and can fold their c-contributions into a per-wave
// LDS slot array with no atomics.  b-contributions stay in registers for the
// whole unit, a-contributions are wave-reduced once per a.  Every unit writes
// fixed-position records; a CSR merge folds them per SNP in a fixed order, so
// results are bitwise reproducible and independent of scheduling.
//
// Per (a, b, c) the kernel forms the LDL^T of every per-study subset of
// {a, b, c} incrementally (the (a, b) prefix once per a, the c-row once per
// step), turns each into a split weight 2^n * mu (psx_math.h), and folds the
// 3^k study assignments (postcal.cpp:907-1030 for the masks passing checkOR).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "psx_sweep.h"

namespace psx {

static thread_local std::string g_sweep_err;
const char* sweep_error() { return g_sweep_err.c_str(); }

#define SWCHK(expr)                                                                                 \
    do {                                                                                            \
        hipError_t _e = (expr);                                                                     \
        if (_e != hipSuccess) {                                                                     \
            g_sweep_err = std::string(hipGetErrorString(_e)) + " at " + __FILE__ + ":" +            \
                          std::to_string(__LINE__);                                                 \
            return -1;                                                                              \
        }                                                                                           \
    } while (0)

struct TileArgs {
    const double* G[2];
    const double* Ad[2];
    const double* y[2];
    const double* skew[2];
    const unsigned char* pres;
    double d[2];
    int U, ldg, Ck;
    double pit[4];
};

__device__ inline Acc5 acc_zero() {
    Acc5 a;
    a.mP = a.mS = a.mN = a.pad = 0;
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

// Fold the 3^K study assignments of one union set given per-study subset
// weights (mu, n) indexed by member bitmask; member j has bit (1 << j).
// Outputs per-member Acc5 contributions and the set's scalar record.
template <int K>
__device__ __forceinline__ void fold_patterns(const double (&mu0)[1 << K], const int (&n0)[1 << K],
                                              const double (&mu1)[1 << K], const int (&n1)[1 << K], int Sm0,
                                              int Sm1, const TileArgs& A, Acc5 (&mem)[K], SetRec& sr) {
    constexpr int NS = 1 << K;
    constexpr int FULL = NS - 1;
    constexpr int NP = (K == 1) ? 3 : (K == 2) ? 9 : 27;
    const int Gll = n0[FULL] + n1[FULL] + 2;
    int GN[K];
#pragma unroll
    for (int j = 0; j < K; j++) {
        const int bj = 1 << j;
        GN[j] = imax(n0[FULL] + n1[FULL ^ bj], n0[FULL ^ bj] + n1[FULL]) + 2;
    }
    const int GS = Gll + A.Ck;
    double tot = 0, nc0 = 0, nc1 = 0, npat = 0;
    double p0[K], p1[K], sh[K], sl[K], ns[K];
#pragma unroll
    for (int j = 0; j < K; j++) p0[j] = p1[j] = sh[j] = sl[j] = ns[j] = 0.0;
#pragma unroll
    for (int p = 0; p < NP; p++) {
        int c0 = 0, c1 = 0, nsh = 0, r = p;
        int x[K];
#pragma unroll
        for (int j = 0; j < K; j++) {
            x[j] = r % 3 + 1;
            r /= 3;
            if (x[j] & 1) c0 |= 1 << j;
            if (x[j] & 2) c1 |= 1 << j;
            if (x[j] == 3) nsh++;
        }
        const bool valid = ((c0 & ~Sm0) == 0) && ((c1 & ~Sm1) == 0);
        const double mup = mu0[c0] * mu1[c1];
        const int np = n0[c0] + n1[c1];
        const double wll = valid ? ldexp(mup, np - Gll) : 0.0;
        const double w = wll * A.pit[nsh];
        tot += w;
        npat += valid ? 1.0 : 0.0;
        // noCausal[s]: the single assignment with C_s empty, on its own shift
        if (c0 == 0) nc0 = valid ? mu1[c1] * A.pit[0] : 0.0;
        if (c1 == 0) nc1 = valid ? mu0[c0] * A.pit[0] : 0.0;
#pragma unroll
        for (int j = 0; j < K; j++) {
            if (x[j] & 1) p0[j] += w;
            if (x[j] & 2) p1[j] += w;
            if (x[j] == 3) {
                sh[j] += w;
                sl[j] += wll;
            } else {
                ns[j] += valid ? ldexp(mup, np - GN[j]) : 0.0;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < K; j++) {
        mem[j].mP = GS;
        mem[j].mS = Gll;
        mem[j].mN = GN[j];
        mem[j].pad = 0;
        mem[j].post0 = p0[j];
        mem[j].post1 = p1[j];
        mem[j].shared = sh[j];
        mem[j].sll = sl[j];
        mem[j].nsll = ns[j];
    }
    sr.m = GS;
    sr.m0 = n1[FULL] + A.Ck;  // C0 empty => C1 = FULL: 2^{n1[FULL]} mu1[FULL] 2^{prior}
    sr.m1 = n0[FULL] + A.Ck;
    sr.pad = 0;
    sr.tot = tot;
    sr.nc0 = nc0;
    sr.nc1 = nc1;
    sr.score = 1e300;
    sr.npat = npat;
}

__device__ __forceinline__ void split(double q, double P, int& n, double& mu) {
    split_exp(0.5 * q * PSX_LOG2E, 1.0 / sqrt(P), n, mu);
}

template <int K>
__global__ __launch_bounds__(64) void k_sweep(TileArgs A, const int4* __restrict__ units, Acc5* __restrict__ rec,
                                              SetRec* __restrict__ srec, int rec_stride) {
    __shared__ Acc5 slot[64];
    const int unit = blockIdx.x;
    const int t = threadIdx.x;
    const int4 un = units[unit];
    const int a0 = un.x, a1 = un.y, B = un.z, T = un.w;
    const int b = 64 * B + t;
    const bool bvalid = b < A.U;
    const int tile = T * (T + 1) / 2 + B;
    const int ldg = A.ldg;
    slot[t] = acc_zero();
    Acc5 accb = acc_zero();
    SetRec accs = set_zero();
    const unsigned pb = bvalid ? A.pres[b] : 0u;
    double Abb[2], yb[2], iAbb[2], qb[2], Pb[2];
#pragma unroll
    for (int s = 0; s < 2; s++) {
        Abb[s] = A.Ad[s][b];
        yb[s] = A.y[s][b];
        iAbb[s] = 1.0 / Abb[s];
        qb[s] = yb[s] * yb[s] * iAbb[s];
        Pb[s] = A.d[s] * Abb[s];
    }
    const int na = (K == 3) ? (a1 - a0) : 1;
    for (int ai = 0; ai < na; ai++) {
        const int a = a0 + ai;
        Acc5 acca = acc_zero();
        // ---- (a, b) prefix, per study -------------------------------------------------
        double iAaa[2], ya[2], Gab[2], qa[2], Pa[2], Dab[2], iDab[2], wab[2], qab[2], Pab[2];
        unsigned pa = 0;
        if (K == 3) {
            pa = A.pres[a];
#pragma unroll
            for (int s = 0; s < 2; s++) {
                const double Aaa = A.Ad[s][a];
                iAaa[s] = 1.0 / Aaa;
                ya[s] = A.y[s][a];
                Gab[s] = A.G[s][(size_t)a * ldg + b];
                qa[s] = ya[s] * ya[s] * iAaa[s];
                Pa[s] = A.d[s] * Aaa;
                const double l = Gab[s] * iAaa[s];
                Dab[s] = Abb[s] - l * Gab[s];
                iDab[s] = 1.0 / Dab[s];
                wab[s] = yb[s] - l * ya[s];
                qab[s] = qa[s] + wab[s] * wab[s] * iDab[s];
                Pab[s] = Pa[s] * A.d[s] * Dab[s];
            }
        }
        // subset weights not involving c (hoisted out of the c loop)
        constexpr int NS = 1 << K;
        double mu[2][NS];
        int nn[2][NS];
#pragma unroll
        for (int s = 0; s < 2; s++) {
            mu[s][0] = 1.0;
            nn[s][0] = 0;
            if (K == 3) {
                split(qa[s], Pa[s], nn[s][1], mu[s][1]);   // {a}
                split(qb[s], Pb[s], nn[s][2], mu[s][2]);   // {b}
                split(qab[s], Pab[s], nn[s][3], mu[s][3]); // {a,b}
            } else {
                split(qb[s], Pb[s], nn[s][1], mu[s][1]);   // {b}
            }
        }
        const bool abvalid = bvalid && (K == 2 || a < b);
        for (int j = 0; j < 64; j++) {
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
                    const double ds = A.d[s];
                    // {c}
                    const double qc = yc * yc / Acc_;
                    // {b, c}
                    const double l2 = Gbc * iAbb[s];
                    const double D2 = Acc_ - l2 * Gbc;
                    const double w2 = yc - l2 * yb[s];
                    const double qbc = qb[s] + w2 * w2 / D2;
                    if (K == 3) {
                        const double Gac = A.G[s][(size_t)a * ldg + c];
                        // {a, c}
                        const double l1 = Gac * iAaa[s];
                        const double D1 = Acc_ - l1 * Gac;
                        const double w1 = yc - l1 * ya[s];
                        const double qac = qa[s] + w1 * w1 / D1;
                        // {a, b, c}: extend the (a, b) factor by the c row
                        const double lcb = (Gbc - l1 * Gab[s]) * iDab[s];
                        const double D3 = D1 - lcb * lcb * Dab[s];
                        const double w3 = w1 - lcb * wab[s];
                        const double qabc = qab[s] + w3 * w3 / D3;
                        split(qc, ds * Acc_, nn[s][4], mu[s][4]);
                        split(qac, Pa[s] * ds * D1, nn[s][5], mu[s][5]);
                        split(qbc, Pb[s] * ds * D2, nn[s][6], mu[s][6]);
                        split(qabc, Pab[s] * ds * D3, nn[s][7], mu[s][7]);
                    } else {
                        split(qc, ds * Acc_, nn[s][2], mu[s][2]);
                        split(qbc, Pb[s] * ds * D2, nn[s][3], mu[s][3]);
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
                Acc5 mem[K];
                SetRec sr;
                fold_patterns<K>(mu[0], nn[0], mu[1], nn[1], Sm0, Sm1, A, mem, sr);
                fold_set(accs, sr);
                if (K == 3) {
                    fold_acc(acca, mem[0]);
                    fold_acc(accb, mem[1]);
                    Acc5 sl = slot[cc];
                    fold_acc(sl, mem[2]);
                    slot[cc] = sl;
                } else {
                    fold_acc(accb, mem[0]);
                    Acc5 sl = slot[cc];
                    fold_acc(sl, mem[1]);
                    slot[cc] = sl;
                }
            }
            __syncthreads();  // slot[] ownership rotates across lanes every step
        }
        if (K == 3) {
            wave_fold_acc(acca);
            if (t == 0) rec[(size_t)unit * rec_stride + 128 + ai] = acca;
        }
    }
    __syncthreads();
    rec[(size_t)unit * rec_stride + t] = slot[t];
    rec[(size_t)unit * rec_stride + 64 + t] = accb;
    wave_fold_set(accs);
    if (t == 0) srec[unit] = accs;
}

// skew[tile(B,T)][j][t] = G[64B + t][64T + ((t + j) & 63)]  for B <= T
__global__ void k_build_skew(const double* __restrict__ G, int ldg, int nblk, double* __restrict__ skew) {
    const int tile = blockIdx.x;
    const int j = blockIdx.y;
    const int t = threadIdx.x;
    int T = 0;
    while ((T + 1) * (T + 2) / 2 <= tile) T++;
    const int B = tile - T * (T + 1) / 2;
    const int r = 64 * B + t;
    const int c = 64 * T + ((t + j) & 63);
    skew[(size_t)tile * 4096 + j * 64 + t] = G[(size_t)r * ldg + c];
}

// ---------------------------------------------------------------------------
// Deterministic record merges (shared with the generic evaluator path)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_merge_members(const Acc5* __restrict__ rec, const int* __restrict__ ptr,
                                                      const int* __restrict__ idx, const int* __restrict__ row_snp,
                                                      Acc5* __restrict__ acc) {
    const int row = blockIdx.x;
    const int lane = threadIdx.x;
    Acc5 a = acc_zero();
    for (int i = ptr[row] + lane; i < ptr[row + 1]; i += 64) fold_acc(a, rec[idx[i]]);
    wave_fold_acc(a);
    if (lane == 0) {
        const int u = row_snp[row];
        Acc5 g = acc[u];
        fold_acc(g, a);
        acc[u] = g;
    }
}

__global__ __launch_bounds__(256) void k_merge_sets(const SetRec* __restrict__ rec, long n, SetRec extra,
                                                    SetRec* __restrict__ acc) {
    __shared__ SetRec sh[256];
    SetRec a = set_zero();
    for (long i = threadIdx.x; i < n; i += 256) fold_set(a, rec[i]);
    sh[threadIdx.x] = a;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) fold_set(sh[threadIdx.x], sh[threadIdx.x + s]);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        SetRec g = *acc;
        fold_set(g, extra);
        fold_set(g, sh[0]);
        *acc = g;
    }
}

int launch_merge_members(const Acc5* rec, const int* ptr, const int* idx, const int* rows, int n_rows, Acc5* acc,
                         hipStream_t st) {
    if (n_rows <= 0) return 0;
    hipLaunchKernelGGL(k_merge_members, dim3(n_rows), dim3(64), 0, st, rec, ptr, idx, rows, acc);
    SWCHK(hipGetLastError());
    return 0;
}

int launch_merge_sets(const SetRec* rec, long n, const SetRec& extra, SetRec* acc, hipStream_t st) {
    hipLaunchKernelGGL(k_merge_sets, dim3(1), dim3(256), 0, st, rec, n, extra, acc);
    SWCHK(hipGetLastError());
    return 0;
}

// ---------------------------------------------------------------------------
// Host planning
// ---------------------------------------------------------------------------
bool sweep_supports(int k, int U) { return (k == 2 || k == 3) && U >= 3; }

// algorithmic bytes of one union set's configurations:
// 8 * sum over assignments of sum_s (|C_s|^2 + |C_s|)
static double set_alg_bytes(int k, const int* memb /*bit0 study0, bit1 study1*/) {
    int np = 1;
    for (int j = 0; j < k; j++) np *= 3;
    double tot = 0;
    for (int p = 0; p < np; p++) {
        int r = p, n0 = 0, n1 = 0;
        bool ok = true;
        for (int j = 0; j < k; j++) {
            int x = r % 3 + 1;
            r /= 3;
            if ((x & ~memb[j]) != 0) { ok = false; break; }
            n0 += x & 1;
            n1 += (x >> 1) & 1;
        }
        if (ok) tot += 8.0 * (n0 * n0 + n0 + n1 * n1 + n1);
    }
    return tot;
}

// Host-only decomposition of level k into wave units for shard (rank, world),
// plus exact union-set / configuration counts and algorithmic bytes.
int plan_units(int k, int U, int ldg, int rank, int world, const unsigned char* pres_host,
               std::vector<PlanUnit>& mine, int& ca, double& sets, double& configs, double& bytes) {
    const int nblk = ldg / 64;
    std::vector<PlanUnit> all;
    if (k == 3) {
        double total_a = 0;
        for (int T = 0; T < nblk; T++)
            for (int B = 0; B <= T; B++) total_a += std::min(64 * B + 63, U);
        ca = (int)std::floor(total_a / (4096.0 * world));
        ca = std::max(1, std::min(64, ca));
        for (int T = 0; T < nblk; T++) {
            if (64 * T >= U) break;
            for (int B = 0; B <= T; B++) {
                if (64 * B >= U) break;
                int amax = std::min(64 * B + 63, U);
                for (int a0 = 0; a0 < amax; a0 += ca) {
                    int a1 = std::min(a0 + ca, amax);
                    all.push_back({a0, a1, B, T, (double)(a1 - a0)});
                }
            }
        }
    } else if (k == 2) {
        ca = 0;
        for (int T = 0; T < nblk; T++) {
            if (64 * T >= U) break;
            for (int B = 0; B <= T; B++) {
                if (64 * B >= U) break;
                all.push_back({0, 1, B, T, 1.0});
            }
        }
    } else {
        return -1;
    }
    // contiguous shard with ~equal work
    double wsum = 0;
    for (auto& u : all) wsum += u.work;
    double lo = wsum * rank / world, hi = wsum * (rank + 1) / world, run = 0;
    mine.clear();
    for (auto& u : all) {
        double mid = run + 0.5 * u.work;
        if (mid >= lo && mid < hi) mine.push_back(u);
        run += u.work;
    }
    // exact counts: membership classes (1 study0, 2 study1, 3 both) with prefix counts
    double bytes_cls[4][4][4];
    for (int x = 1; x < 4; x++)
        for (int y = 1; y < 4; y++)
            for (int z = 1; z < 4; z++) {
                int m3[3] = {x, y, z};
                bytes_cls[x][y][z] = (k == 3) ? set_alg_bytes(3, m3) : set_alg_bytes(2, m3 + 1);
            }
    const double wcls[4] = {0, 1, 1, 3};
    std::vector<int> pref[4];
    for (int x = 1; x < 4; x++) {
        pref[x].assign(U + 1, 0);
        for (int i = 0; i < U; i++) pref[x][i + 1] = pref[x][i] + (pres_host[i] == x);
    }
    sets = 0; bytes = 0; configs = 0;
    for (auto& u : mine) {
        for (int t = 0; t < 64; t++) {
            int b = 64 * u.B + t;
            if (b >= U) break;
            int c_lo = (u.B < u.T) ? 64 * u.T : b + 1;
            int c_hi = std::min(64 * u.T + 64, U);
            if (c_hi <= c_lo) continue;
            int mb = pres_host[b];
            if (mb == 0) continue;
            if (k == 3) {
                int ahi = std::min(u.a1, b);
                if (ahi <= u.a0) continue;
                for (int x = 1; x < 4; x++) {
                    double na = pref[x][ahi] - pref[x][u.a0];
                    if (na == 0) continue;
                    for (int z = 1; z < 4; z++) {
                        double ncz = pref[z][c_hi] - pref[z][c_lo];
                        sets += na * ncz;
                        bytes += na * ncz * bytes_cls[x][mb][z];
                        configs += na * ncz * wcls[x] * wcls[mb] * wcls[z];
                    }
                }
            } else {
                for (int z = 1; z < 4; z++) {
                    double ncz = pref[z][c_hi] - pref[z][c_lo];
                    sets += ncz;
                    bytes += ncz * bytes_cls[1][mb][z];
                    configs += ncz * wcls[mb] * wcls[z];
                }
            }
        }
    }
    return 0;
}

static int build_plan(SweepPlan& P, int k, int U, int ldg, int rank, int world, const unsigned char* pres_host) {
    P.k = k; P.U = U; P.ldg = ldg; P.rank = rank; P.world = world;
    std::vector<PlanUnit> mine;
    int ca = 0;
    double sets = 0, configs = 0, bytes = 0;
    if (plan_units(k, U, ldg, rank, world, pres_host, mine, ca, sets, configs, bytes)) {
        g_sweep_err = "unsupported sweep level";
        return -1;
    }
    P.ca = ca;
    P.rec_stride = (k == 3) ? 128 + ca : 128;
    P.n_units = (int)mine.size();
    P.union_sets = (uint64_t)sets;
    P.alg_bytes = bytes;
    // FP64 operation estimate per union set (prefix, c-row
    // extension, split-exps, 3^k assignment folds and record folds)
    P.flops = sets * (k == 3 ? 900.0 : 260.0);
    // device buffers
    std::vector<int4> hu(P.n_units);
    for (int i = 0; i < P.n_units; i++) hu[i] = make_int4(mine[i].a0, mine[i].a1, mine[i].B, mine[i].T);
    if (P.n_units > 0) {
        SWCHK(hipMalloc(&P.d_units, sizeof(int4) * P.n_units));
        SWCHK(hipMemcpy(P.d_units, hu.data(), sizeof(int4) * P.n_units, hipMemcpyHostToDevice));
        SWCHK(hipMalloc(&P.d_rec, sizeof(Acc5) * (size_t)P.n_units * P.rec_stride));
        SWCHK(hipMalloc(&P.d_srec, sizeof(SetRec) * (size_t)P.n_units));
    }
    // CSR: record -> SNP, grouped by SNP in record order (deterministic folds)
    std::vector<int> key((size_t)P.n_units * P.rec_stride, -1);
    for (int i = 0; i < P.n_units; i++) {
        const PlanUnit& u = mine[i];
        int* kk = key.data() + (size_t)i * P.rec_stride;
        for (int t = 0; t < 64; t++) {
            int c = 64 * u.T + t;
            if (c < U) kk[t] = c;
            int b = 64 * u.B + t;
            if (b < U) kk[64 + t] = b;
        }
        if (k == 3)
            for (int a = u.a0; a < u.a1; a++) kk[128 + (a - u.a0)] = a;
    }
    std::vector<int> cnt(U, 0);
    for (int v : key) if (v >= 0) cnt[v]++;
    std::vector<int> ptr(1, 0), rows, start(U, -1);
    int acc = 0;
    for (int u = 0; u < U; u++)
        if (cnt[u]) { start[u] = acc; rows.push_back(u); acc += cnt[u]; ptr.push_back(acc); }
    std::vector<int> idx(acc), fill(U, 0);
    for (size_t i = 0; i < key.size(); i++)
        if (key[i] >= 0) idx[start[key[i]] + fill[key[i]]++] = (int)i;
    P.n_rows = (int)rows.size();
    P.csr_ptr_len = (int)ptr.size();
    P.csr_idx_len = (int)idx.size();
    std::vector<int> packed;
    packed.insert(packed.end(), ptr.begin(), ptr.end());
    packed.insert(packed.end(), idx.begin(), idx.end());
    packed.insert(packed.end(), rows.begin(), rows.end());
    if (!packed.empty()) {
        SWCHK(hipMalloc(&P.d_csr, sizeof(int) * packed.size()));
        SWCHK(hipMemcpy(P.d_csr, packed.data(), sizeof(int) * packed.size(), hipMemcpyHostToDevice));
    }
    return 0;
}

static int ensure_skew(SweepPlanCache& C, const SweepArgs& a, int ldg, hipStream_t st) {
    if (C.d_skew[0] && C.skew_ldg == ldg && C.skew_src[0] == a.G0 && C.skew_src[1] == a.G1) return 0;
    for (int s = 0; s < 2; s++) { hipFree(C.d_skew[s]); C.d_skew[s] = nullptr; }
    const int nblk = ldg / 64;
    const int ntile = nblk * (nblk + 1) / 2;
    for (int s = 0; s < 2; s++) {
        SWCHK(hipMalloc(&C.d_skew[s], sizeof(double) * (size_t)ntile * 4096));
        hipLaunchKernelGGL(k_build_skew, dim3(ntile, 64), dim3(64), 0, st, s ? a.G1 : a.G0, ldg, nblk, C.d_skew[s]);
        SWCHK(hipGetLastError());
    }
    C.skew_ldg = ldg;
    C.skew_src[0] = a.G0;
    C.skew_src[1] = a.G1;
    return 0;
}

int sweep_level(SweepPlanCache& C, int k, int U, int ldg, int rank, int world, hipStream_t st, const SweepArgs& a,
                Acc5* acc, SetRec* sacc, SweepStats* stats) {
    if (!C.ev[0])
        for (int i = 0; i < 4; i++) SWCHK(hipEventCreate(&C.ev[i]));
    if (ensure_skew(C, a, ldg, st)) return -1;
    auto key = std::make_tuple(k, U, rank, world);
    auto it = C.plans.find(key);
    if (it == C.plans.end()) {
        std::vector<unsigned char> pres(ldg);
        SWCHK(hipMemcpy(pres.data(), a.pres, ldg, hipMemcpyDeviceToHost));
        SweepPlan P;
        if (build_plan(P, k, U, ldg, rank, world, pres.data())) return -1;
        it = C.plans.emplace(key, P).first;
    }
    SweepPlan& P = it->second;
    if (P.n_units == 0) return 0;
    TileArgs A;
    A.G[0] = a.G0; A.G[1] = a.G1;
    A.Ad[0] = a.Ad0; A.Ad[1] = a.Ad1;
    A.y[0] = a.y0; A.y[1] = a.y1;
    A.skew[0] = C.d_skew[0]; A.skew[1] = C.d_skew[1];
    A.pres = a.pres;
    A.d[0] = a.d0; A.d[1] = a.d1;
    A.U = U; A.ldg = ldg;
    A.Ck = a.Ck[k];
    for (int n = 0; n < 4; n++) A.pit[n] = (n <= k) ? a.pit[k * a.pit_ld + n] : 0.0;
    SWCHK(hipEventRecord(C.ev[0], st));
    if (k == 3)
        hipLaunchKernelGGL(k_sweep<3>, dim3(P.n_units), dim3(64), 0, st, A, P.d_units, P.d_rec, P.d_srec, P.rec_stride);
    else
        hipLaunchKernelGGL(k_sweep<2>, dim3(P.n_units), dim3(64), 0, st, A, P.d_units, P.d_rec, P.d_srec, P.rec_stride);
    SWCHK(hipGetLastError());
    SWCHK(hipEventRecord(C.ev[1], st));
    const int* ptr = P.d_csr;
    const int* idx = P.d_csr + P.csr_ptr_len;
    const int* rows = P.d_csr + P.csr_ptr_len + P.csr_idx_len;
    if (launch_merge_members(P.d_rec, ptr, idx, rows, P.n_rows, acc, st)) return -1;
    SetRec none = set_zero();
    if (launch_merge_sets(P.d_srec, P.n_units, none, sacc, st)) return -1;
    SWCHK(hipEventRecord(C.ev[2], st));
    SWCHK(hipEventSynchronize(C.ev[2]));
    float k_ms = 0, m_ms = 0;
    SWCHK(hipEventElapsedTime(&k_ms, C.ev[0], C.ev[1]));
    SWCHK(hipEventElapsedTime(&m_ms, C.ev[1], C.ev[2]));
    if (stats) {
        stats->kernel_ms[k] += k_ms;
        stats->launches[k] += 1;
        stats->union_sets[k] += P.union_sets;
        stats->alg_bytes[k] += P.alg_bytes;
        stats->flops[k] += P.flops;
        stats->merge_ms += m_ms;
    }
    return 0;
}

void sweep_free(SweepPlanCache& C) {
    for (auto& kv : C.plans) {
        SweepPlan& P = kv.second;
        hipFree(P.d_units); hipFree(P.d_rec); hipFree(P.d_srec); hipFree(P.d_csr);
    }
    C.plans.clear();
    for (int s = 0; s < 2; s++) { hipFree(C.d_skew[s]); C.d_skew[s] = nullptr; }
    for (int i = 0; i < 4; i++) if (C.ev[i]) { hipEventDestroy(C.ev[i]); C.ev[i] = nullptr; }
}

}  // namespace psx
