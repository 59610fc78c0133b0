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
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>

#include <algorithm>
#include <chrono>
#include <array>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "psx_sweep.h"
#include "psx_sweep_dev.h"
#include "psx_sweep_unit.h"
#include "psx_mem.h"

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

template <int K, bool EXACT>
__global__ __launch_bounds__(64, (K == 3 ? 2 : 4)) void k_sweep(TileArgs A, const int4* __restrict__ units, Acc5* __restrict__ rec,
                                              SetRec* __restrict__ srec, int rec_stride, int* __restrict__ flag,
                                              const int* __restrict__ pos) {
    __shared__ SweepUnitSmem sm;
    sweep_unit<K, EXACT>(A, blockIdx.x, units, rec, srec, rec_stride, flag, pos, sm);
}

// singleton subset weights per union SNP: h = y^2 / (2 A) log2(e), rP = (d A)^{-1/2}
__global__ void k_build_singles(const double* __restrict__ Ad, const double* __restrict__ y, double rsd, int ldg,
                                double* __restrict__ muS, int* __restrict__ nS) {
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= ldg) return;
    const double r = rsqrt_nr(Ad[u]);
    const double q = y[u] * y[u] * r * r;
    int n;
    double mu;
    split2(0.5 * q * PSX_LOG2E, r * rsd, n, mu);
    muS[u] = mu;
    nS[u] = n;
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
// Gathered records (generic evaluator: SSS batches, configs rows, levels >= 4).
// A row can hold thousands of records (an SSS neighbourhood repeats the current
// configuration's members in every swap set), so 256 threads fold it and each
// thread issues MERGE_R index loads, then MERGE_R record loads, before folding:
// two dependent round trips per MERGE_R * 256 records instead of per 64.
constexpr int MERGE_R = 8;
__global__ __launch_bounds__(256) void k_merge_members(const Acc5* __restrict__ rec, const int* __restrict__ ptr,
                                                       const int* __restrict__ idx, const int* __restrict__ row_snp,
                                                       Acc5* __restrict__ acc) {
    __shared__ Acc5 sh[4];
    const int row = blockIdx.x;
    const int b = ptr[row], e = ptr[row + 1];
    Acc5 a = acc_zero();
    for (int i0 = b + (int)threadIdx.x; i0 < e; i0 += 256 * MERGE_R) {
        int ix[MERGE_R];
#pragma unroll
        for (int r = 0; r < MERGE_R; r++) ix[r] = i0 + 256 * r < e ? idx[i0 + 256 * r] : -1;
        Acc5 v[MERGE_R];
#pragma unroll
        for (int r = 0; r < MERGE_R; r++) v[r] = ix[r] >= 0 ? rec[ix[r]] : acc_zero();
#pragma unroll
        for (int r = 0; r < MERGE_R; r++) fold_acc(a, v[r]);
    }
    wave_fold_acc(a);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = a;
    __syncthreads();
    if (threadIdx.x == 0) {
        const int u = row_snp[row];
        Acc5 g = acc[u];
        for (int w = 0; w < 4; w++) fold_acc(g, sh[w]);
        acc[u] = g;
    }
}

// SNP u's records are CSR positions [dptr[u], dptr[u+1]) (none: the block
// returns), each gathered from record slot gidx[q] (unit-major record
// buffers); 256 threads fold them in a fixed order.
__global__ __launch_bounds__(256) void k_merge_rows(const Acc5* __restrict__ rec, const int* __restrict__ dptr,
                                                   const int* __restrict__ gidx, Acc5* __restrict__ acc) {
    __shared__ Acc5 sh[4];
    const int u = blockIdx.x;
    const int q0 = dptr[u], q1 = dptr[u + 1];
    if (q0 == q1) return;  // uniform
    Acc5 a = acc_zero();
    for (int i = q0 + (int)threadIdx.x; i < q1; i += 256) fold_acc(a, rec[gidx[i]]);
    wave_fold_acc(a);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = a;
    __syncthreads();
    if (threadIdx.x == 0) {
        Acc5 g = acc[u];
        for (int w = 0; w < 4; w++) fold_acc(g, sh[w]);
        acc[u] = g;
    }
}

// Fold n set records (+ extra) into *acc; init: overwrite *acc instead of
// folding into it and zero *zero_flag (start of an exhaustive pass).
// Fixed fold order (thread-strided, then wave and block trees): deterministic.
__global__ __launch_bounds__(512) void k_merge_sets(const SetRec* __restrict__ rec, long n, SetRec extra,
                                                    SetRec* __restrict__ acc, int init, int* __restrict__ zero_flag) {
    __shared__ SetRec sh[8];
    SetRec a = set_zero();
    // MERGE_R loads in flight per thread before folding them (fold order fixed)
    for (long i0 = threadIdx.x; i0 < n; i0 += 512 * MERGE_R) {
        SetRec v[MERGE_R];
#pragma unroll
        for (int r = 0; r < MERGE_R; r++) v[r] = i0 + 512 * r < n ? rec[i0 + 512 * r] : set_zero();
#pragma unroll
        for (int r = 0; r < MERGE_R; r++) fold_set(a, v[r]);
    }
    wave_fold_set(a);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = a;
    __syncthreads();
    if (threadIdx.x == 0) {
        SetRec g = init ? set_zero() : *acc;
        fold_set(g, extra);
        for (int w = 0; w < 8; w++) fold_set(g, sh[w]);
        *acc = g;
        if (zero_flag) *zero_flag = 0;
    }
}

int launch_merge_members(const Acc5* rec, const int* ptr, const int* idx, const int* rows, int n_rows, Acc5* acc,
                         hipStream_t st) {
    if (n_rows <= 0) return 0;
    hipLaunchKernelGGL(k_merge_members, dim3(n_rows), dim3(256), 0, st, rec, ptr, idx, rows, acc);
    SWCHK(hipGetLastError());
    return 0;
}

// k_merge_members over a dptr CSR: block u folds SNP u's records (8 loads in
// flight per thread), the fold order of k_merge_members
__global__ __launch_bounds__(256) void k_merge_dptr(const Acc5* __restrict__ rec, const int* __restrict__ dptr,
                                                    const int* __restrict__ gidx, Acc5* __restrict__ acc) {
    __shared__ Acc5 sh[4];
    const int u = blockIdx.x;
    const int b = dptr[u], e = dptr[u + 1];
    if (b == e) return;  // uniform
    Acc5 a = acc_zero();
    for (int i0 = b + (int)threadIdx.x; i0 < e; i0 += 256 * MERGE_R) {
        int ix[MERGE_R];
#pragma unroll
        for (int r = 0; r < MERGE_R; r++) ix[r] = i0 + 256 * r < e ? gidx[i0 + 256 * r] : -1;
        Acc5 v[MERGE_R];
#pragma unroll
        for (int r = 0; r < MERGE_R; r++) v[r] = ix[r] >= 0 ? rec[ix[r]] : acc_zero();
#pragma unroll
        for (int r = 0; r < MERGE_R; r++) fold_acc(a, v[r]);
    }
    wave_fold_acc(a);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = a;
    __syncthreads();
    if (threadIdx.x == 0) {
        Acc5 g = acc[u];
        for (int w = 0; w < 4; w++) fold_acc(g, sh[w]);
        acc[u] = g;
    }
}

int launch_merge_dptr(const Acc5* rec, const int* dptr, const int* gidx, int U, Acc5* acc, hipStream_t st) {
    if (U <= 0) return 0;
    hipLaunchKernelGGL(k_merge_dptr, dim3(U), dim3(256), 0, st, rec, dptr, gidx, acc);
    SWCHK(hipGetLastError());
    return 0;
}

int launch_merge_sets(const SetRec* rec, long n, const SetRec& extra, SetRec* acc, hipStream_t st, bool init,
                      int* zero_flag) {
    hipLaunchKernelGGL(k_merge_sets, dim3(1), dim3(512), 0, st, rec, n, extra, acc, init ? 1 : 0, zero_flag);
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
        ca = (int)std::floor(total_a / (4096.0 * world));  // exact-variant kernel (k_sweep<3, true>)
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
        // one wave per (B, T) tile would leave most of the 1024 SIMDs idle:
        // split the 64-step diagonal walk into S j-ranges (a0, a1 = j0, j1)
        int tiles = 0;
        for (int T = 0; T < nblk && 64 * T < U; T++) tiles += std::min(T + 1, (U + 63) / 64);
        const int S = std::max(1, std::min(8, (1024 * world + tiles - 1) / std::max(1, tiles)));
        ca = 0;
        for (int T = 0; T < nblk; T++) {
            if (64 * T >= U) break;
            for (int B = 0; B <= T; B++) {
                if (64 * B >= U) break;
                for (int i = 0; i < S; i++) all.push_back({64 * i / S, 64 * (i + 1) / S, B, T, 1.0 / S});
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
                for (int j = u.a0; j < u.a1; j++) {  // this unit's part of the diagonal walk
                    const int cc = (t + j) & 63, c = 64 * u.T + cc;
                    if (c >= U || (u.B == u.T && cc <= t) || pres_host[c] == 0) continue;
                    sets += 1;
                    bytes += bytes_cls[1][mb][pres_host[c]];
                    configs += wcls[mb] * wcls[pres_host[c]];
                }
            }
        }
    }
    return 0;
}

// k = 3 fast-kernel decomposition (k_sweep3): units (a0, a1, K, C), K <= C, in
// the padded space v = u + pad.  Lane t owns c = 64C + t; b runs over block K;
// a over [a0, a1) with a < b.  Exact per-shard set / configuration / byte counts
// in O(64 * 9) per unit from per-class prefix counts over v.
constexpr double kTailFrac = 0.05;  // share of a shard's work cut into single-a units at the end (PSX_K3_TAIL)
constexpr double kDiagW = 0.65;   // per-a cost of a pipelined diagonal walk (PSX_K3_DIAGW; 0.59 before r04ae)
constexpr double kUnitW = 0.04;   // fixed cost of a unit (PSX_K3_UNITW)
constexpr int kPlanVersion = 2;  // the shard split's rules (r05: per-class bands), in the plan hash
constexpr double kMaskedDiagW = 0.65;  // per-a cost of a masked diagonal walk (PSX_K3_MASKW; 1.0 / 1.3 worse, r04aa; 0.65 with DIAGW 0.65 balances world 8 best, r04ae)

// The plan-shaping knobs, read once per process.  PSX_K3_ROUNDS / PSX_K3_DIAG_DIV
// (environment, tuning experiments) override the dispatch rounds the a-chunk is
// sized for and divide the diagonal units' a-chunk; PSX_K3_MASKW / DIAGW /
// UNITW the cost model of the shard split; PSX_K3_TAIL / TAIL2 the tail cuts.
// Every rank of a job must cut the same plan: plan_knobs_hash() goes into each
// rank's partial image (PlanTag) and the merge refuses images whose hashes differ.
const K3Knobs& k3_knobs() {
    static const K3Knobs k = [] {
        K3Knobs r;
        auto num = [](const char* name, double dflt, bool zero_ok) {
            const char* e = std::getenv(name);
            if (!e) return dflt;
            const double v = std::atof(e);
            return (zero_ok ? v >= 0 : v > 0) ? v : dflt;
        };
        r.rounds = num("PSX_K3_ROUNDS", (double)PSX_K3_ROUNDS, false);
        r.diag_div = (int)num("PSX_K3_DIAG_DIV", 1.0, false);
        r.maskw = num("PSX_K3_MASKW", kMaskedDiagW, false);
        r.diagw = num("PSX_K3_DIAGW", kDiagW, false);
        r.unitw = num("PSX_K3_UNITW", kUnitW, true);
        const char* t = std::getenv("PSX_K3_TAIL");
        r.tail_frac = t ? std::atof(t) : kTailFrac;
        const char* t2 = std::getenv("PSX_K3_TAIL2");
        r.tail2 = t2 ? std::atof(t2) : 0.0;
        return r;
    }();
    return k;
}

uint64_t plan_knobs_hash() {
    const K3Knobs& k = k3_knobs();
    const double v[7] = {k.rounds, (double)k.diag_div, k.maskw, k.diagw, k.unitw, k.tail_frac, k.tail2};
    uint64_t h = 1469598103934665603ull;  // FNV-1a over the values' bytes and the compiled constants
    auto mix = [&](const void* p, size_t n) {
        for (size_t i = 0; i < n; i++) h = (h ^ ((const unsigned char*)p)[i]) * 1099511628211ull;
    };
    mix(v, sizeof(v));
    const int c[4] = {PSX_K3_WAVES, kMaxChunkA3, PSX_KMAX, kPlanVersion};
    mix(c, sizeof(c));
    return h;
}

int plan_units3c(int U, int ldg, int rank, int world, const unsigned char* pres_host, std::vector<PlanUnit>& mine,
                 int& ca, double& sets, double& configs, double& bytes) {
    const int nblk = ldg / 64, pad = ldg - U;
    auto cls = [&](int v) { return v >= pad ? (int)pres_host[v - pad] : 0; };
    double total_a = 0;
    for (int C = 0; C < nblk; C++)
        for (int K = 0; K <= C; K++) total_a += (K < C) ? std::max(0, 64 * K - pad) : U;  // a-range per tile
    // a-chunk size: k_sweep3 holds 2 waves per SIMD (~245 VGPRs), i.e. 8 unit
    // slots per CU.  Larger chunks amortise the per-unit prologue / records,
    // smaller ones shorten the last dispatch round (the longest-first order
    // below leaves the short folded-diagonal units for it): about 3.5 rounds of
    // the wave slots per shard, at most 4 a per unit (measured on MI355X,
    // syn1000c3, tools/ca_sweep.sh: ca = 4 at world 1, 2 at worlds 2 and 4, 1 at
    // world 8).
    // Units per shard the a-chunk is sized for, from MI355X's 256 CUs as a fixed
    // constant, not a device query: every rank (in any process, on any device)
    // must cut the same unit list, or the union of the ranks' work bands would not
    // cover every walk step exactly once.  (On a device with another CU count the
    // plan stays exact, only its dispatch rounds differ.)
    // PSX_K3_ROUNDS / PSX_K3_DIAG_DIV (environment, tuning experiments; the same
    // for every rank of a job) override the dispatch rounds the a-chunk is sized
    // for and divide the diagonal units' a-chunk (shorter units for the last
    // dispatch rounds).
    constexpr double kPlanCUs = 256.0;
    const K3Knobs& kn = k3_knobs();
    const double rounds = kn.rounds, maskw = kn.maskw, diagw = kn.diagw, unitw = kn.unitw;
    const int diag_div = kn.diag_div;
    const double kTarget = rounds * (4.0 * PSX_K3_WAVES * kPlanCUs);
    ca = (int)std::lround(total_a / (kTarget * world));
    ca = std::min(ca, kMaxChunkA3);  // (caps 6 / 8 with the tail split: +0.4 / +1.5 % at world 1, r04w)
    ca = std::max(1, std::min(64, ca));
    const int cad = std::max(1, ca / diag_div);
    // Every union triple x < y < z belongs to exactly one unit family, by which
    // of its members share a 64-block:
    //   all in different blocks      -> off-diagonal tile (K = blk y, C = blk z), a = x
    //   x, y in one block, z later   -> diagonal tile (K = C = blk x), a = z (after the block)
    //   y, z in one block, x earlier -> diagonal tile (K = C = blk y), a = x (before the block)
    //   all three in one block       -> diagonal tile, a = x (in the block, below the pair)
    // so off-diagonal tiles only see a < 64K (every lane active every step) and
    // the triangular pair structure only occurs in diagonal tiles, which walk
    // it folded (psx_sweep3.hip): no in-block masking waste.
    // a diagonal tile's walk of a is masked when a lies inside the block, or in
    // every walk of block 0 when it holds padding
    auto masked = [&](int K, int a) { return (a >= 64 * K && a < 64 * K + 64) || 64 * K < pad; };
    auto a_work = [&](int K, int C, int a) { return K < C ? 1.0 : masked(K, a) ? maskw : diagw; };
    std::vector<PlanUnit> all;
    for (int C = 0; C < nblk; C++) {
        if (64 * C + 64 <= pad) continue;
        for (int K = 0; K <= C; K++) {
            const int amax = (K < C) ? 64 * K : ldg;
            const int cu = K < C ? ca : cad;
            for (int a0 = pad; a0 < amax; a0 += cu) {
                const int a1 = std::min(a0 + cu, amax);
                // unit cost in off-diagonal-a units: a fixed per-unit part and a
                // per-a part; a diagonal tile's folded walk has half the steps (first
                // fitted to unit durations, tools/unit_trace.py: off-diagonal 3.3 +
                // 81.8 ca us, diagonal 3.0 + 48.4 ca us; the diagonal weight then
                // raised to 0.65 where it balanced the world-8 shards best, r04ae).
                // (the diagonal walks of a inside the block, and every walk of block 0
                // when it holds padding, take the masked step loop: maskw per a)
                double w = unitw;
                for (int a = a0; a < a1; a++) w += a_work(K, C, a);
                all.push_back({a0, a1, K, C, w});
            }
        }
    }
    // Contiguous work bands in enumeration order (C, K, a), cut per unit class:
    // off-diagonal units, diagonal units whose a all walk pipelined, and diagonal
    // units with a masked walk (a inside the block, or block 0 holding padding).
    // Each rank takes 1/world of every class, so the split does not depend on the
    // relative weights of the classes (a single band over all units put most
    // diagonal tiles, i.e. the low C, on the low ranks: the r04 rehearsal's 5-7 %
    // per-rank spread at worlds 2 / 4 / 8 came from the diagonal weight).  (Dealing
    // the units cyclically instead was measured box-dependent, -4 % .. +5 % at world 8.)
    auto ucls = [&](const PlanUnit& u) {
        if (u.B < u.T) return 0;
        for (int a = u.a0; a < u.a1; a++)
            if (masked(u.B, a)) return 2;
        return 1;
    };
    mine.clear();
    for (int c = 0; c < 3; c++) {
        double wsum = 0;
        for (auto& u : all)
            if (ucls(u) == c) wsum += u.work;
        const double lo = wsum * rank / world, hi = wsum * (rank + 1) / world;
        double run = 0;
        for (auto& u : all) {
            if (ucls(u) != c) continue;
            const double mid = run + 0.5 * u.work;
            if (mid >= lo && mid < hi) mine.push_back(u);
            run += u.work;
        }
    }
    // (back to enumeration order: the LPT sort below is stable within a weight)
    std::stable_sort(mine.begin(), mine.end(), [](const PlanUnit& x, const PlanUnit& y) {
        return x.T != y.T ? x.T < y.T : x.B != y.B ? x.B < y.B : x.a0 < y.a0;
    });
    double bytes_cls[4][4][4];
    for (int x = 1; x < 4; x++)
        for (int y = 1; y < 4; y++)
            for (int z = 1; z < 4; z++) {
                int m3[3] = {x, y, z};
                bytes_cls[x][y][z] = set_alg_bytes(3, m3);
            }
    const double wcls[4] = {0, 1, 1, 3};
    std::vector<int> pref[4];  // pref[x][v]: class-x SNPs with index < v (v space)
    for (int x = 1; x < 4; x++) {
        pref[x].assign(ldg + 1, 0);
        for (int v = 0; v < ldg; v++) pref[x][v + 1] = pref[x][v] + (cls(v) == x);
    }
    auto cnt = [&](int x, int v0, int v1) { return (double)(pref[x][v1] - pref[x][v0]); };
    sets = 0; bytes = 0; configs = 0;
    auto add = [&](double n, int x, int y, int z) {
        if (n == 0) return;
        sets += n;
        bytes += n * bytes_cls[x][y][z];
        configs += n * wcls[x] * wcls[y] * wcls[z];
    };
    for (auto& u : mine) {
        const int b0 = 64 * u.B, c0 = 64 * u.T;
        if (u.B < u.T) {  // a < block K < block C: every (a, b, c) of the tile
            for (int x = 1; x < 4; x++) {
                const double na = cnt(x, u.a0, u.a1);
                if (na == 0) continue;
                for (int y = 1; y < 4; y++)
                    for (int z = 1; z < 4; z++) add(na * cnt(y, b0, b0 + 64) * cnt(z, c0, c0 + 64), x, y, z);
            }
            continue;
        }
        for (int a = u.a0; a < u.a1; a++) {  // diagonal tile: pairs of the block (above a if a is in it)
            const int x = cls(a);
            if (x == 0) continue;
            const int lo_v = (a >= b0 && a < b0 + 64) ? a + 1 : b0;
            double n[4] = {0, cnt(1, lo_v, b0 + 64), cnt(2, lo_v, b0 + 64), cnt(3, lo_v, b0 + 64)};
            for (int y = 1; y < 4; y++)
                for (int z = y; z < 4; z++) add(y == z ? n[y] * (n[y] - 1) / 2 : n[y] * n[z], x, y, z);
        }
    }
    // Longest units first (LPT): the off-diagonal units, then the folded
    // diagonal ones (0.71), so the launch's last dispatch round is made of the
    // shorter units (the in-launch level-2 units follow them).  The unit
    // timeline (tools/unit_trace.py) showed a ~60 us tail of full-length units
    // on a world-8 shard in tile order.  Stable: tile order kept within a class.
    std::stable_sort(mine.begin(), mine.end(), [](const PlanUnit& x, const PlanUnit& y) { return x.work > y.work; });
    // The last dispatch round drains while its units finish: PSX_K3_TAIL (a
    // fraction of the shard's work, default kTailFrac) cuts the units at the end
    // of the order into single-a units, so the drain is made of the shortest
    // units.  Each (a, b, c) stays in the same shard, so the counts above hold.
    const double tail_frac = kn.tail_frac;
    if (tail_frac > 0 && ca > 1) {
        double wtot = 0, wacc = 0;
        for (auto& u : mine) wtot += u.work;
        size_t cut = mine.size();
        while (cut > 0 && wacc + mine[cut - 1].work <= tail_frac * wtot) wacc += mine[--cut].work;
        std::vector<PlanUnit> tail;
        for (size_t i = cut; i < mine.size(); i++) {
            const PlanUnit& u = mine[i];
            for (int a = u.a0; a < u.a1; a++) {
                PlanUnit v = u;
                v.a0 = a;
                v.a1 = a + 1;
                v.work = unitw + a_work(u.B, u.T, a);
                tail.push_back(v);
            }
        }
        mine.resize(cut);
        std::stable_sort(tail.begin(), tail.end(), [](const PlanUnit& x, const PlanUnit& y) { return x.work > y.work; });
        // PSX_K3_TAIL2 (a fraction of the shard's work, default 0): the very last
        // diagonal single-a units walk half their (folded) steps each, so the
        // final drain is made of half-length pieces; each pair of the block is
        // still visited once (steps 1..16 | 17..32)
        const double tail2 = kn.tail2;
        if (tail2 > 0) {
            double w2 = 0;
            size_t c2 = tail.size();
            while (c2 > 0 && tail[c2 - 1].B == tail[c2 - 1].T && tail[c2 - 1].j0 == 0 && tail[c2 - 1].j1 == 64 &&
                   w2 + tail[c2 - 1].work <= tail2 * wtot)
                w2 += tail[--c2].work;
            std::vector<PlanUnit> halves;
            for (size_t i = c2; i < tail.size(); i++) {
                PlanUnit h = tail[i];
                h.work *= 0.5;
                h.j0 = 0;
                h.j1 = 32;
                halves.push_back(h);
                h.j0 = 32;
                h.j1 = 64;
                halves.push_back(h);
            }
            tail.resize(c2);
            tail.insert(tail.end(), halves.begin(), halves.end());
        }
        mine.insert(mine.end(), tail.begin(), tail.end());
    }
    // (An XCD-aware order — runs of one tile's units packed onto the 8 XCDs,
    // workgroup i running on XCD (i + launch offset) % 8, so each 4 MB L2 serves
    // ~1/8 of the tile rows — measured neutral (r01y, worlds 1-8) once the next
    // step's tile row is prefetched, and 10 % slower in r05 with tiles dealt to
    // 8 interleaved groups, profiles/r05zo_xcd_order_ab.txt; not used.)
    // (Splitting the last dispatch rounds into shorter b-walk pieces was
    // measured +1-6 % slower: a unit's fixed cost is ~11 us, EXPERIMENTS.md A.)
    return 0;
}

// a plan's unit list to the device and its record CSR built there
// (psx_plan.hip: pos | dptr | gidx in one block); the host unit list is dropped
static int upload_plan(SweepPlan& P, SweepPlanCache& C, hipStream_t st) {
    if (P.uploaded) return 0;
    const size_t n = P.rec_len;
    if (P.n_units > 0) {
        SWCHK(psx::dmalloc(&P.d_units, sizeof(int4) * P.n_units));
        SWCHK(hipMemcpyAsync(P.d_units, P.h_units.data(), sizeof(int4) * P.n_units, hipMemcpyHostToDevice, st));
        SWCHK(psx::dmalloc(&P.d_srec, sizeof(SetRec) * (size_t)P.n_units));
    }
    SWCHK(psx::dmalloc(&P.d_csr, sizeof(int) * (2 * n + P.U + 1)));
    P.d_pos = P.d_csr;
    P.d_dptr = P.d_csr + n;
    P.d_gidx = P.d_csr + n + P.U + 1;
    P.csr_pos = records_at_csr_positions(P.world);
    if (plan_csr_device(P.d_units, P.n_units, P.rec_stride, P.k, P.variant, P.pad, P.U, const_cast<int*>(P.d_pos),
                        const_cast<int*>(P.d_dptr), const_cast<int*>(P.d_gidx), C.csr_scratch, st, P.csr_pos)) {
        g_sweep_err = "plan CSR on the device failed";
        return -1;
    }
    SWCHK(hipStreamSynchronize(st));  // the host unit list is released below
    std::vector<int4>().swap(P.h_units);
    P.uploaded = true;
    return 0;
}

// The record CSR restated on the host (the pre-r05 builder): tests compare the
// device build against it (plan_csr_selftest).
static void host_plan_csr(const SweepPlan& P, const std::vector<int4>& hu, std::vector<int>& pos,
                          std::vector<int>& dptr, std::vector<int>& gidx) {
    const int U = P.U, pad = P.pad;
    std::vector<int> key((size_t)P.n_units * P.rec_stride, -1);
    for (int i = 0; i < P.n_units; i++) {
        const int B = hu[i].z & 0xffff, T = hu[i].w & 0xffff;
        int* kk = key.data() + (size_t)i * P.rec_stride;
        const bool one = P.variant && P.k == 3 && B == T;
        for (int t = 0; t < 64; t++) {
            int c = 64 * T + t - pad;
            if (c >= 0 && c < U) kk[t] = c;
            int b = 64 * B + t - pad;
            if (!one && b >= 0 && b < U) kk[64 + t] = b;
        }
        if (P.k == 3)
            for (int a = hu[i].x; a < hu[i].y; a++) kk[128 + (a - hu[i].x)] = a - pad;
    }
    std::vector<int> cnt(U + 1, 0);
    for (int v : key) if (v >= 0) cnt[v]++;
    dptr.assign(U + 1, 0);
    for (int u = 0; u < U; u++) dptr[u + 1] = dptr[u] + cnt[u];
    gidx.assign(dptr[U], 0);
    std::vector<int> fill(dptr.begin(), dptr.end() - 1);
    pos.assign(key.size(), -1);
    for (size_t i = 0; i < key.size(); i++)
        if (key[i] >= 0) {  // slot i's record at its CSR position (stable in slot order)
            const int q = fill[key[i]]++;
            const bool csr = records_at_csr_positions(P.world);
            gidx[q] = csr ? q : (int)i;
            pos[i] = csr ? q : (int)i;
        }
}

// variant 1: the k = 3 fast kernel's decomposition (plan_units3c, v space);
// variant 0: plan_units (k = 2, and the exact k = 3 rerun).  Host only: the unit
// list and the plan's counts (upload_plan puts it on the device).
static int build_plan(SweepPlan& P, int k, int U, int ldg, int rank, int world, const unsigned char* pres_host,
                      int variant) {
    P.k = k; P.U = U; P.ldg = ldg; P.rank = rank; P.world = world;
    P.variant = variant;
    std::vector<PlanUnit> mine;
    int ca = 0;
    double sets = 0, configs = 0, bytes = 0;
    const int rc = variant ? plan_units3c(U, ldg, rank, world, pres_host, mine, ca, sets, configs, bytes)
                           : plan_units(k, U, ldg, rank, world, pres_host, mine, ca, sets, configs, bytes);
    if (rc) {
        g_sweep_err = "unsupported sweep level";
        return -1;
    }
    P.ca = ca;
    if (variant)  // the fast kernel stages a unit's a scalars in LDS arrays of kMaxChunkA3
        for (const PlanUnit& u : mine)
            if (u.a1 - u.a0 > kMaxChunkA3 || u.a1 <= u.a0) {
                g_sweep_err = "k = 3 unit a-range outside 1.." + std::to_string(kMaxChunkA3);
                return -1;
            }
    P.rec_stride = (k == 3) ? 128 + ca : 128;
    P.n_units = (int)mine.size();
    P.union_sets = (uint64_t)sets;
    P.alg_bytes = bytes;
    // FP64 operations per union set (FMA = 2), fitted to the PMC FP64 counts of
    // the k = 3 fast kernel (64 x SQ_INSTS_VALU_FLOPS_FP64 / sets: 281 before the
    // deferred fold, 159 after it (r02zd), 141.8 in r03zb, 139.2 in r04h, 132.5 in
    // r04t, 131.8 in r04ag): kept at or below the last count, so a bench line without PMC
    // counters of its own build cannot overstate the FP64 rate; k = 2 by the
    // round-1 ratio of VALU work per set.  bench.py reports it only as a model.
    P.flops = sets * (k == 3 ? 131.0 : 110.0);
    P.pad = variant ? ldg - U : 0;  // record keys of variant 1 are in v space
    // variant 1 packs the b-walk step range of (half) units into the high bits
    P.h_units.resize(P.n_units);
    for (int i = 0; i < P.n_units; i++)
        P.h_units[i] = variant ? make_int4(mine[i].a0, mine[i].a1, mine[i].B | (mine[i].j0 << 16),
                                           mine[i].T | (mine[i].j1 << 16))
                               : make_int4(mine[i].a0, mine[i].a1, mine[i].B, mine[i].T);
    // Records at their CSR positions (since r06): the kernels write record slot
    // i at pos[i] (-1: no SNP), each SNP's run contiguous in slot order, so the
    // pass merge reads it coalesced (r01-r05 wrote slot i at i, unit-major, and
    // the merges gathered through gidx: the single-pass merge then ran at ~2.6
    // TB/s of records; the sweeps' scattered stores measured neutral at world 1
    // and 0-2 % slower at world 8 in r04al, when the merge was hidden anyway)
    P.rec_len = (size_t)P.n_units * P.rec_stride;
    return 0;
}

int plan_csr_selftest(int U, const unsigned char* pres, int k, int rank, int world, int variant, long* mismatches,
                      long* records) {
    const int ldg = (U + 63) / 64 * 64;
    SweepPlan P;
    SweepPlanCache C;
    if (build_plan(P, k, U, ldg, rank, world, pres, variant)) return -1;
    const std::vector<int4> hu = P.h_units;
    std::vector<int> pos, dptr, gidx;
    host_plan_csr(P, hu, pos, dptr, gidx);
    hipStream_t st = nullptr;
    if (upload_plan(P, C, st)) return -1;
    std::vector<int> dpos(P.rec_len), ddptr(U + 1), dgidx(P.rec_len);
    SWCHK(hipMemcpy(dpos.data(), P.d_pos, sizeof(int) * P.rec_len, hipMemcpyDeviceToHost));
    SWCHK(hipMemcpy(ddptr.data(), P.d_dptr, sizeof(int) * (U + 1), hipMemcpyDeviceToHost));
    SWCHK(hipMemcpy(dgidx.data(), P.d_gidx, sizeof(int) * P.rec_len, hipMemcpyDeviceToHost));
    long bad = 0;
    for (size_t i = 0; i < P.rec_len; i++) bad += dpos[i] != pos[i];
    for (int u = 0; u <= U; u++) bad += ddptr[u] != dptr[u];
    for (size_t q = 0; q < gidx.size(); q++) bad += dgidx[q] != gidx[q];
    *mismatches = bad;
    *records = (long)gidx.size();
    psx::dfree(P.d_units); psx::dfree(P.d_srec); psx::dfree(P.d_csr); psx::dfree(C.csr_scratch.p);
    return 0;
}

static TileArgs tile_args(const SweepPlanCache& C, const SweepArgs& a, int k, int U, int ldg);

// arguments of the k = 3 fast kernel (and of its {b, c} precompute)
static Sweep3Args sweep3_args(const SweepPlanCache& C, const SweepArgs& a, int U, int ldg) {
    const TileArgs A = tile_args(C, a, 3, U, ldg);
    Sweep3Args S3;
    for (int s = 0; s < 2; s++) {
        S3.G[s] = A.G[s]; S3.Ad[s] = A.Ad[s]; S3.ys[s] = C.d_ys[s]; S3.skewT[s] = C.d_skewT[s];
        S3.muS[s] = A.muS[s]; S3.nS[s] = A.nS[s]; S3.rsd[s] = A.rsd[s];
    }
    S3.bcn = C.d_bcn;
    S3.bcsm = C.d_bcsm;
    S3.bcsn = C.d_bcsn;
    S3.bccm = C.d_bccm;
    S3.bccn = C.d_bccn;
    S3.g01 = C.d_g01;
    S3.mu01 = C.d_mu01;
    S3.pad = ldg - U;
    S3.pres = A.pres;
    S3.tab = C.d_tab;
    S3.pit0 = A.pit[0];
    S3.rho = A.pit[0] > 0 ? A.pit[1] / A.pit[0] : 0.0;
    S3.U = U; S3.ldg = ldg; S3.Ck = A.Ck;
    S3.redo_count = C.d_redo;
    return S3;
}

static void free_k3(SweepPlanCache& C) {
    for (int s = 0; s < 2; s++) {
        psx::dfree(C.d_skewT[s]); C.d_skewT[s] = nullptr;
        psx::dfree(C.d_ys[s]); C.d_ys[s] = nullptr;
    }
    psx::dfree(C.d_bcn); C.d_bcn = nullptr;
    psx::dfree(C.d_bcsm); C.d_bcsm = nullptr;
    psx::dfree(C.d_bcsn); C.d_bcsn = nullptr;
    psx::dfree(C.d_bccm); C.d_bccm = nullptr;
    psx::dfree(C.d_bccn); C.d_bccn = nullptr;
    psx::dfree(C.d_g01); C.d_g01 = nullptr;
    psx::dfree(C.d_mu01); C.d_mu01 = nullptr;
}

// the layouts every tiled level reads (skewed Sigma~ tiles, singleton weights,
// the exp2 table), built once per locus
static int ensure_skew(SweepPlanCache& C, const SweepArgs& a, int ldg, int U, hipStream_t st) {
    if (C.d_skew[0] && C.skew_ldg == ldg && C.skew_src[0] == a.G0 && C.skew_src[1] == a.G1) return 0;
    free_k3(C);
    for (int s = 0; s < 2; s++) {
        psx::dfree(C.d_skew[s]); C.d_skew[s] = nullptr;
        psx::dfree(C.d_muS[s]); C.d_muS[s] = nullptr;
        psx::dfree(C.d_nS[s]); C.d_nS[s] = nullptr;
    }
    psx::dfree(C.d_tab); C.d_tab = nullptr;
    {
        // 2^(i/256) correctly rounded (long double on the host)
        double tab[256];
        for (int i = 0; i < 256; i++) tab[i] = (double)exp2l((long double)i / 256.0L);
        SWCHK(psx::dmalloc(&C.d_tab, sizeof(tab)));
        SWCHK(hipMemcpyAsync(C.d_tab, tab, sizeof(tab), hipMemcpyHostToDevice, st));
        std::vector<unsigned char> pres(ldg);
        SWCHK(hipMemcpyAsync(pres.data(), a.pres, ldg, hipMemcpyDeviceToHost, st));
        SWCHK(hipStreamSynchronize(st));
        C.allpres = true;
        for (int u = 0; u < U; u++) C.allpres = C.allpres && pres[u] == 3;
    }
    for (int s = 0; s < 2; s++) {
        SWCHK(psx::dmalloc(&C.d_muS[s], sizeof(double) * ldg));
        SWCHK(psx::dmalloc(&C.d_nS[s], sizeof(int) * ldg));
        hipLaunchKernelGGL(k_build_singles, dim3((ldg + 255) / 256), dim3(256), 0, st, s ? a.Ad1 : a.Ad0,
                           s ? a.y1 : a.y0, 1.0 / std::sqrt(s ? a.d1 : a.d0), ldg, C.d_muS[s], C.d_nS[s]);
        SWCHK(hipGetLastError());
    }
    const int nblk = ldg / 64;
    const int ntile = nblk * (nblk + 1) / 2;
    for (int s = 0; s < 2; s++) {
        SWCHK(psx::dmalloc(&C.d_skew[s], sizeof(double) * (size_t)ntile * 4096));
        hipLaunchKernelGGL(k_build_skew, dim3(ntile, 64), dim3(64), 0, st, s ? a.G1 : a.G0, ldg, nblk, C.d_skew[s]);
        SWCHK(hipGetLastError());
    }
    if (!C.d_redo) {
        SWCHK(psx::dmalloc(&C.d_redo, sizeof(int)));
        SWCHK(hipMemsetAsync(C.d_redo, 0, sizeof(int), st));
    }
    C.skew_ldg = ldg;
    C.skew_src[0] = a.G0;
    C.skew_src[1] = a.G1;
    return 0;
}

// what only the fast k = 3 kernel reads (scaled y, transposed tiles, the
// a-independent {b, c} weights and their sums), built on the first k = 3 pass
// of a locus: a c <= 2 run never loads the k = 3 code object
static int ensure_k3_build(SweepPlanCache& C, const SweepArgs& a, int ldg, int U, hipStream_t st);

// d_g01 marks a complete build: a build that failed part way is released
// (d_g01 back to null), so a retry starts from nothing (no orphaned buffers)
static int ensure_k3(SweepPlanCache& C, const SweepArgs& a, int ldg, int U, hipStream_t st) {
    if (C.d_g01) return 0;
    free_k3(C);
    if (ensure_k3_build(C, a, ldg, U, st)) {
        const std::string err = g_sweep_err;
        free_k3(C);
        g_sweep_err = err;
        return -1;
    }
    return 0;
}

static int ensure_k3_build(SweepPlanCache& C, const SweepArgs& a, int ldg, int U, hipStream_t st) {
    const int nblk = ldg / 64;
    const int ntile = nblk * (nblk + 1) / 2;
    for (int s = 0; s < 2; s++) {
        SWCHK(psx::dmalloc(&C.d_ys[s], sizeof(double) * ldg));
        if (launch_scale_y(s ? a.y1 : a.y0, ldg, C.d_ys[s], st)) SWCHK(hipGetLastError());
        SWCHK(psx::dmalloc(&C.d_skewT[s], sizeof(double) * (size_t)ntile * 4096));
        if (launch_build_skewT(s ? a.G1 : a.G0, ldg, ldg - U, C.d_skewT[s], st)) SWCHK(hipGetLastError());
    }
    {  // the a-independent {b, c} weights of every k = 3 step
        Sweep3Args S3 = sweep3_args(C, a, U, ldg);
        // kTileRowPad rows past the last tile: the pipelined b-walk loads up to
        // three steps ahead without clamping (rows it never uses)
        const size_t nrow = (size_t)ntile * 4096, npad = (size_t)kTileRowPad * 64;
        SWCHK(psx::dmalloc(&C.d_mu01, sizeof(double2) * (nrow + npad)));
        SWCHK(psx::dmalloc(&C.d_bcn, sizeof(int2) * (nrow + npad)));
        SWCHK(psx::dmalloc(&C.d_g01, sizeof(double2) * (nrow + npad)));
        SWCHK(hipMemsetAsync(C.d_mu01 + nrow, 0, sizeof(double2) * npad, st));
        SWCHK(hipMemsetAsync(C.d_bcn + nrow, 0, sizeof(int2) * npad, st));
        SWCHK(hipMemsetAsync(C.d_g01 + nrow, 0, sizeof(double2) * npad, st));
        if (launch_build_bc3(S3, ntile, C.d_mu01, C.d_bcn, st)) SWCHK(hipGetLastError());
        SWCHK(psx::dmalloc(&C.d_bcsm, sizeof(double2) * (size_t)ntile * 64));
        SWCHK(psx::dmalloc(&C.d_bcsn, sizeof(int2) * (size_t)ntile * 64));
        if (launch_bc3_rowsum(ntile, C.d_mu01, C.d_bcn, C.d_bcsm, C.d_bcsn, st)) SWCHK(hipGetLastError());
        SWCHK(psx::dmalloc(&C.d_bccm, sizeof(double2) * (size_t)ntile * 64));
        SWCHK(psx::dmalloc(&C.d_bccn, sizeof(int2) * (size_t)ntile * 64));
        if (launch_bc3_colsum(ntile, C.d_mu01, C.d_bcn, C.d_bccm, C.d_bccn, st)) SWCHK(hipGetLastError());
        if (launch_interleave2(C.d_skewT[0], C.d_skewT[1], (size_t)ntile * 4096, C.d_g01, st)) SWCHK(hipGetLastError());
    }
    return 0;
}

int plan_host_ms(int U, int k, int rank, int world, double* ms, int* n_units, long* n_records) {
    const int ldg = (U + 63) / 64 * 64;
    std::vector<unsigned char> pres(ldg, 0);
    for (int u = 0; u < U; u++) pres[u] = 3;
    SweepPlan P;
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = build_plan(P, k, U, ldg, rank, world, pres.data(), k == 3 ? 1 : 0);
    *ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    *n_units = P.n_units;
    *n_records = (long)P.rec_len;
    return rc;
}

void plan_prefetch(SweepPlanCache& C, int device, int k, int U, int ldg, int rank, int world, bool exact) {
    const int variant = (k == 3 && !exact) ? 1 : 0;
    auto key = std::make_tuple(k, U, rank, world, variant);
    if ((int)C.pres_host.size() != ldg || C.plans.count(key) || C.pending.count(key)) return;
    std::unique_ptr<PlanJob> job(new PlanJob());
    PlanJob* J = job.get();
    std::vector<unsigned char> pres(C.pres_host);
    J->done = std::async(std::launch::async, [=]() {
        (void)device;  // host work only: the device part runs at the first pass
        const int rc = build_plan(J->P, k, U, ldg, rank, world, pres.data(), variant);
        if (rc) J->err = g_sweep_err;
        return rc;
    });
    C.pending.emplace(key, std::move(job));
}

int sweep_begin(SweepPlanCache& C, hipStream_t st) {
    if (!C.d_flag) SWCHK(psx::dmalloc(&C.d_flag, sizeof(int)));
    SWCHK(hipMemsetAsync(C.d_flag, 0, sizeof(int), st));
    return 0;
}

int sweep_redo_count(SweepPlanCache& C, int* count) {
    *count = 0;
    if (C.d_redo) SWCHK(hipMemcpy(count, C.d_redo, sizeof(int), hipMemcpyDeviceToHost));
    return 0;
}

int sweep_flag(SweepPlanCache& C, int* flag) {
    *flag = 0;
    if (C.d_flag) SWCHK(hipMemcpy(flag, C.d_flag, sizeof(int), hipMemcpyDeviceToHost));
    return 0;
}

// The level's plan for (rank, world), built (host decomposition + CSR upload)
// on first use; also builds the shared skewed layouts.
int sweep_prepare(SweepPlanCache& C, int k, int U, int ldg, int rank, int world, hipStream_t st, const SweepArgs& a,
                  bool exact, SweepPlan** out) {
    if (ensure_skew(C, a, ldg, U, st)) return -1;
    const int variant = (k == 3 && !exact) ? 1 : 0;
    if (variant && ensure_k3(C, a, ldg, U, st)) return -1;
    auto key = std::make_tuple(k, U, rank, world, variant);
    auto it = C.plans.find(key);
    if (it == C.plans.end()) {
        SweepPlan P;
        auto pj = C.pending.find(key);
        if (pj != C.pending.end()) {  // built ahead (plan_prefetch)
            const int rc = pj->second->done.get();
            P = pj->second->P;
            const std::string err = pj->second->err;
            C.pending.erase(pj);
            if (rc) {
                g_sweep_err = err;
                return -1;
            }
        } else {
            std::vector<unsigned char> pres(C.pres_host);
            if ((int)pres.size() != ldg) {
                pres.assign(ldg, 0);
                SWCHK(hipStreamSynchronize(st));
                SWCHK(hipMemcpy(pres.data(), a.pres, ldg, hipMemcpyDeviceToHost));
            }
            if (build_plan(P, k, U, ldg, rank, world, pres.data(), variant)) return -1;
        }
        if (upload_plan(P, C, st)) return -1;
        if (P.rec_len && !P.d_rec) SWCHK(psx::dmalloc(&P.d_rec, sizeof(Acc5) * P.rec_len));
        P.variant = variant;
        for (int i = 0; i < 3; i++) SWCHK(hipEventCreate(&P.ev[i]));
        it = C.plans.emplace(key, P).first;
    }
    *out = &it->second;
    return 0;
}

// Enqueue one level (kernel + record merges) on `st`; no host synchronisation.
int sweep_level(SweepPlanCache& C, int k, int U, int ldg, int rank, int world, hipStream_t st, const SweepArgs& a,
                Acc5* acc, SetRec* sacc, bool exact) {
    SweepPlan* PP = nullptr;
    if (sweep_prepare(C, k, U, ldg, rank, world, st, a, exact, &PP)) return -1;
    if (sweep_kernel(C, *PP, st, a, nullptr, exact, nullptr, nullptr)) return -1;
    SweepPlan& P = *PP;
    if (P.n_units == 0) return 0;
    hipLaunchKernelGGL(k_merge_rows, dim3(P.U), dim3(256), 0, st, P.d_rec, P.d_dptr, P.d_gidx, acc);
    SWCHK(hipGetLastError());
    SetRec none = set_zero();
    if (launch_merge_sets(P.d_srec, P.n_units, none, sacc, st)) return -1;
    SWCHK(hipEventRecord(P.ev[2], st));
    return 0;
}

// Launch only the level's kernel: per-SNP records into the plan's CSR buffer,
// set records into srec_out (the plan's own buffer when null).
static TileArgs tile_args(const SweepPlanCache& C, const SweepArgs& a, int k, int U, int ldg) {
    TileArgs A;
    A.G[0] = a.G0; A.G[1] = a.G1;
    A.Ad[0] = a.Ad0; A.Ad[1] = a.Ad1;
    A.y[0] = a.y0; A.y[1] = a.y1;
    A.skew[0] = C.d_skew[0]; A.skew[1] = C.d_skew[1];
    A.pres = a.pres;
    A.muS[0] = C.d_muS[0]; A.muS[1] = C.d_muS[1];
    A.nS[0] = C.d_nS[0]; A.nS[1] = C.d_nS[1];
    A.d[0] = a.d0; A.d[1] = a.d1;
    A.rsd[0] = 1.0 / std::sqrt(a.d0); A.rsd[1] = 1.0 / std::sqrt(a.d1);
    A.U = U; A.ldg = ldg;
    A.Ck = a.Ck[k];
    for (int n = 0; n < 4; n++) A.pit[n] = (n <= k) ? a.pit[k * a.pit_ld + n] : 0.0;
    return A;
}

static void mark_last(SweepPlanCache& C, SweepPlan& P) {
    P.ran = false;
    auto other = C.plans.find(std::make_tuple(P.k, P.U, P.rank, P.world, 1 - P.variant));
    if (other != C.plans.end()) other->second.ran = false;  // stats: the last pass only
}

Acc5* plan_records(SweepPlan& P, int parity) {
    if (!parity) return P.d_rec;
    if (parity < 0 || parity >= kRecBufs) {
        g_sweep_err = "bad record buffer index";
        return nullptr;
    }
    Acc5*& r = P.d_rec_alt[parity - 1];
    if (!r && P.rec_len > 0 && psx::dmalloc(&r, sizeof(Acc5) * P.rec_len) != hipSuccess) {
        r = nullptr;
        g_sweep_err = "out of device memory (record buffer)";
    }
    return r;
}

int sweep_kernel(SweepPlanCache& C, SweepPlan& P, hipStream_t st, const SweepArgs& a, SetRec* srec_out, bool exact,
                 SweepPlan* l2, SetRec* srec2, int parity, int* flag_in, bool timed, hipEvent_t ev0,
                 hipEvent_t ev1) {
    const int k = P.k, U = P.U, ldg = P.ldg;
    mark_last(C, P);
    P.fused_bytes = P.fused_flops = 0;
    const bool ride = l2 && k == 3 && !exact && l2->k == 2 && l2->n_units > 0;
    if (l2) mark_last(C, *l2);
    if (P.n_units == 0 && !ride) {
        if (l2 && sweep_kernel(C, *l2, st, a, srec2, exact, nullptr, nullptr, parity, flag_in, timed)) return -1;
        return 0;
    }
    SetRec* srec = srec_out ? srec_out : P.d_srec;
    const TileArgs A = tile_args(C, a, k, U, ldg);
    if (!C.d_flag && sweep_begin(C, st)) return -1;
    int* const flag = flag_in ? flag_in : C.d_flag;
    Acc5* const rec = plan_records(P, parity);
    if (!rec && P.rec_len > 0) return -1;
    if (timed) SWCHK(hipEventRecord(P.ev[0], st));
    const dim3 g(P.n_units), blk(64);
    if (k == 3 && !exact) {
        Sweep3Args S3 = sweep3_args(C, a, U, ldg);
        S3.tstamp = C.stamp;
        Level2Blocks b{0, TileArgs{}, nullptr, nullptr, nullptr, nullptr};
        if (ride) {  // level 2 in the same launch: its units are the first blocks of the grid
            Acc5* rec2 = plan_records(*l2, parity);
            if (!rec2 && l2->rec_len > 0) return -1;
            b = Level2Blocks{l2->n_units, tile_args(C, a, 2, U, ldg), l2->d_units, rec2,
                             srec2 ? srec2 : l2->d_srec, l2->d_pos};
            P.fused_bytes = l2->alg_bytes;
            P.fused_flops = l2->flops;
        }
        static const char* trace_path = std::getenv("PSX_UNIT_TRACE");  // diagnostics: unit timeline dump
        if (trace_path) SWCHK(psx::dmalloc(&S3.trace, sizeof(unsigned long long) * kTraceWords * (size_t)P.n_units));
        if (trace_path) SWCHK(hipMemsetAsync(S3.trace, 0, sizeof(unsigned long long) * kTraceWords * (size_t)P.n_units, st));
        if (launch_sweep3(C.allpres, S3, P.n_units, P.d_units, rec, srec, P.rec_stride, flag, P.d_pos, st,
                          ride ? &b : nullptr, ev0, ev1))
            SWCHK(hipGetLastError());
        if (trace_path) {
            std::vector<unsigned long long> h(kTraceWords * (size_t)P.n_units);
            SWCHK(hipStreamSynchronize(st));
            SWCHK(hipMemcpy(h.data(), S3.trace, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
            SWCHK(psx::dfree(S3.trace));
            if (FILE* f = std::fopen(trace_path, "wb")) {
                std::fwrite(h.data(), sizeof(unsigned long long), h.size(), f);
                std::fclose(f);
            }
        }
    } else if (k == 3)
        hipLaunchKernelGGL((k_sweep<3, true>), g, blk, 0, st, A, P.d_units, rec, srec, P.rec_stride, flag, P.d_pos);
    else if (!exact)
        hipExtLaunchKernelGGL((k_sweep<2, false>), g, blk, 0, st, ev0, ev1, 0, A, P.d_units, rec, srec, P.rec_stride,
                              flag, P.d_pos);
    else
        hipLaunchKernelGGL((k_sweep<2, true>), g, blk, 0, st, A, P.d_units, rec, srec, P.rec_stride, flag, P.d_pos);
    SWCHK(hipGetLastError());
    if (timed) {
        SWCHK(hipEventRecord(P.ev[1], st));
        SWCHK(hipEventRecord(P.ev[2], st));  // merges (if any) re-record ev[2]
        P.ran = true;
    }
    if (l2 && !ride && sweep_kernel(C, *l2, st, a, srec2, exact, nullptr, nullptr, parity, flag_in, timed)) return -1;
    return 0;
}

// After the stream has been synchronised: per-level statistics of the last run.
int sweep_stats_plan(SweepPlan& P, int k, SweepStats* stats);

int sweep_stats(SweepPlanCache& C, int k, int U, int rank, int world, SweepStats* stats) {
    for (int variant = 0; variant < 2; variant++) {
        auto it = C.plans.find(std::make_tuple(k, U, rank, world, variant));
        if (it == C.plans.end() || !it->second.ran) continue;
        if (sweep_stats_plan(it->second, k, stats)) return -1;
    }
    return 0;
}

int sweep_stats_plan(SweepPlan& P, int k, SweepStats* stats) {
    float k_ms = 0, m_ms = 0;
    SWCHK(hipEventElapsedTime(&k_ms, P.ev[0], P.ev[1]));
    SWCHK(hipEventElapsedTime(&m_ms, P.ev[1], P.ev[2]));
    stats->kernel_ms[k] += k_ms;
    stats->launches[k] += 1;
    stats->union_sets[k] += P.union_sets;
    stats->alg_bytes[k] += P.alg_bytes + P.fused_bytes;  // per launch: in-launch level-2 work included
    stats->flops[k] += P.flops + P.fused_flops;
    stats->merge_ms += m_ms;
    return 0;
}

void sweep_free(SweepPlanCache& C) {
    psx::dfree(C.csr_scratch.p);
    C.csr_scratch = PlanScratch();
    for (auto& kv : C.pending) {  // plans built ahead and never used
        kv.second->done.wait();
        SweepPlan& P = kv.second->P;
        psx::dfree(P.d_units); psx::dfree(P.d_srec); psx::dfree(P.d_csr);
    }
    C.pending.clear();
    for (auto& kv : C.plans) {
        SweepPlan& P = kv.second;
        psx::dfree(P.d_units); psx::dfree(P.d_rec); psx::dfree(P.d_srec);
        psx::dfree(P.d_csr);
        for (Acc5* r : P.d_rec_alt) psx::dfree(r);
        for (int i = 0; i < 3; i++) if (P.ev[i]) hipEventDestroy(P.ev[i]);
    }
    C.plans.clear();
    free_k3(C);
    for (int s = 0; s < 2; s++) {
        psx::dfree(C.d_skew[s]); C.d_skew[s] = nullptr;
        psx::dfree(C.d_muS[s]); C.d_muS[s] = nullptr;
        psx::dfree(C.d_nS[s]); C.d_nS[s] = nullptr;
    }
    psx::dfree(C.d_tab); C.d_tab = nullptr;
    psx::dfree(C.d_redo); C.d_redo = nullptr;
    if (C.own_flag) psx::dfree(C.d_flag);
    C.d_flag = nullptr;
}

// load this translation unit's device code on the current device (psx_warmup)
int warm_module_sweep() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, (const void*)k_merge_sets) == hipSuccess ? 0 : -1;
}

}  // namespace psx
