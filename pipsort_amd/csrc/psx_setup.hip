// psx_setup.hip — the Model setup that feeds PostCal (model.h:171-264,
// util.cpp:195-263) on the GPU, behind psx_create_from_ld.
//
// Per study the reference
//   1. shifts the LD diagonal by 0.01 until the GSL partial-pivot LU
//      determinant is > 0 (util.cpp:195-226),
//   2. eigendecomposes Sigma' = Q W Q^T (util.cpp:228-263) and builds
//      B = |W|^1/2 Q^T, S' = |W|^-1/2 Q^T z (model.h:213-259).
// The engine only consumes Sigma~ = B^T B, y = B^T S' and ||S'||^2.  These are
// Q|W|Q^T, z and z^T Q|W|^-1 Q^T z, so whenever Sigma' is positive definite
// they are exactly Sigma', z and z^T Sigma'^-1 z: no eigendecomposition.
//
//  * Step 1 runs here as a right-looking elimination with the reference's
//    operation order and IEEE rounding (division correctly rounded, multiply
//    and subtract not fused), so the per-element update sequence — and hence
//    every U_ii and the index-order determinant product — is bit-identical to
//    the host restatement psx_psd_shift (model.cpp), the oracle of this step.
//    Swap-free LDs (every SYN-v1 locus) take the tiled kernels: one launch
//    per 16-column panel, each block factoring the panel's diagonal block with
//    its tile's rows and applying the delayed updates to its tile (k_lu_step,
//    ~5-12 us per panel; M = 2000 in 2.7 ms).  An LD that needs a row swap
//    takes GSL's pivot search in LDS panels (k_lu_panel_piv + k_lu_trail).
//  * Positive definiteness and z^T Sigma'^-1 z come from one elimination
//    without pivoting of the symmetrised Sigma' (its pivots are the D of
//    L D L^T) with the forward solve of z fused in.  When some pivot is not
//    comfortably positive (ratio to the largest diagonal < kPdRatio) the
//    caller falls back to the reference's eigen route (rocSOLVER, psx_eigen.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "psx_setup.h"
#include "psx_mem.h"

namespace psx {

namespace {

constexpr int kElimCols = 256;  // threads (columns) per elimination block
constexpr int kElimRows = 16;   // rows per elimination block
constexpr double kPdRatio = 1e-8;

// A = L + add * I (row-major n x n).  Off-diagonal entries are copied, not
// added to, exactly as util.cpp:206-211 sets them.
__global__ void k_psd_copy(const double* __restrict__ L, int n, double add, double* __restrict__ A) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)n * n) return;
    const int i = (int)(idx / n), k = (int)(idx % n);
    A[idx] = (i == k) ? L[idx] + add : L[idx];
}

// S[i][k] = S'[max(i,k)][min(i,k)] + add [i == k]: the lower triangle the
// reference's gsl_eigen_symmv reads (util.cpp:242), mirrored.
__global__ void k_sym_lower(const double* __restrict__ L, int n, double add, double* __restrict__ S) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)n * n) return;
    const int i = (int)(idx / n), k = (int)(idx % n);
    const double v = (i >= k) ? L[(size_t)i * n + k] : L[(size_t)k * n + i];
    S[idx] = (i == k) ? v + add : v;
}

// Partial pivoting of column j (GSL 2.5 gsl_linalg_LU_decomp): the first row
// i >= j of maximal |a_ij| (strict > scanning upwards from a_jj), then swap
// rows j and ip from column j on (columns < j hold L, irrelevant to det).
__global__ __launch_bounds__(1024) void k_lu_pivot(double* __restrict__ A, int n, int j, int* __restrict__ swp) {
    __shared__ double sv[1024];
    __shared__ int si[1024];
    const int t = threadIdx.x;
    double mx = -1.0;  // below every |a|, above no NaN: NaNs are never chosen, as with `>`
    int ip = n;
    for (int i = j + t; i < n; i += 1024) {
        const double v = fabs(A[(size_t)i * n + j]);
        if (v > mx) { mx = v; ip = i; }
    }
    sv[t] = mx;
    si[t] = ip;
    __syncthreads();
    for (int w = 512; w > 0; w >>= 1) {
        if (t < w) {
            const double v2 = sv[t + w];
            const int i2 = si[t + w];
            if (v2 > sv[t] || (v2 == sv[t] && i2 < si[t])) { sv[t] = v2; si[t] = i2; }
        }
        __syncthreads();
    }
    const double ajj = A[(size_t)j * n + j];
    const int p = (ajj != ajj || si[0] >= n) ? j : si[0];  // a NaN a_jj keeps row j (nothing is > NaN)
    if (t == 0) swp[j] = (p != j) ? 1 : 0;
    if (p == j) return;
    for (int k = j + t; k < n; k += 1024) {
        const double a = A[(size_t)j * n + k];
        A[(size_t)j * n + k] = A[(size_t)p * n + k];
        A[(size_t)p * n + k] = a;
    }
}

// One elimination step at column j: for rows i > j, l_i = a_ij / a_jj and
// a_ik = a_ik - l_i * a_jk for k > j (not fused; skipped when a_jj == 0, as
// GSL does).  With z: the unit-lower forward solve z_i -= l_i z_j.
__global__ __launch_bounds__(kElimCols) void k_elim(double* __restrict__ A, int n, int j, double* __restrict__ z) {
#pragma clang fp contract(off)
    __shared__ double sl[kElimRows];
    const double ajj = A[(size_t)j * n + j];
    if (ajj == 0.0) return;
    const int t = threadIdx.x;
    const int i0 = j + 1 + blockIdx.y * kElimRows;
    const int nr = min(kElimRows, n - i0);
    if (t < nr) sl[t] = A[(size_t)(i0 + t) * n + j] / ajj;
    __syncthreads();
    if (z && blockIdx.x == 0 && t < nr) {
        const double zj = z[j];
        z[i0 + t] = z[i0 + t] - sl[t] * zj;
    }
    const int k = j + 1 + blockIdx.x * kElimCols + t;
    if (k >= n) return;
    const double ujk = A[(size_t)j * n + k];
    for (int r = 0; r < nr; r++) {
        double* p = A + (size_t)(i0 + r) * n + k;
        const double prod = sl[r] * ujk;
        *p = *p - prod;
    }
}

// Swap-free elimination, tiled with delayed updates (LD matrices: the
// diagonal stays the column maximum, so no row is ever swapped).  Element
// (i, k) of the right-looking elimination receives, for every step q <
// min(i, k), a_ik <- a_ik - l_iq * u_qk (multiply and subtract not fused), in
// increasing q.  Any schedule that applies those updates in increasing q with
// the same l_iq and u_qk gives every element — U_ii, z~ — bit for bit what the
// per-column elimination gives.  Without pivoting a panel's factorisation is
// row-local once its 16 x 16 diagonal block D is factored: row i's panel
// entries take l_iq = a_iq / u_qq and a_ic -= l_iq u_qc (c > q in the panel),
// column k's U entries take u_rk -= l_rq u_qk (q < r, l from D).  So one
// launch per panel (k_lu_step, below) does a panel: every block factors D and
// its tile rows' L chains in one pass, solves its tile columns' U rows and
// applies the delayed updates to its tile; L and U are recomputed per tile
// (identically), never stored — the setup consumes U_ii and z~ only.  The
// swap check (GSL's pivot: the first row of maximal |a_iq|, NaNs never chosen,
// so a swap is needed iff some |a_iq| > |u_qq|, i > q) raises *flag, and the
// caller reruns the pivoting path from a fresh copy.  A zero u_qq skips step q
// (GSL).
constexpr int kPanel = 16;     // panel width (k_lu_step, k_lu_panel_piv)
constexpr int kPanelThreads = 1024;
constexpr int kTrCols = 64;
constexpr int kTrRows = 32;
constexpr int kTrGroups = 4;  // row groups per trailing block (kTrRows / kTrGroups rows per thread)
constexpr int kPanelLds = 152 * 1024;  // dynamic LDS budget of k_lu_panel_piv (160 KB per CU; 158 KB is refused)

__device__ inline double rdlane(double v, int l) {
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_readlane((int)b, l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}

// Factor the nb x nb diagonal block at (j, j) held in one wave's registers
// (lane r < nb: row j + r, v[c] = a_{j+r, j+c} after every earlier panel's
// updates, zr = z_{j+r} likewise) with the per-column elimination's operations;
// rows of the block below q are checked for a needed swap.  Writes the block
// back to A (in place) and z to z.
__device__ void factor_diag(double (&v)[kPanel], double zr, int j, int nb, double* __restrict__ A, int n,
                            double* __restrict__ z, int check, int* __restrict__ flag) {
#pragma clang fp contract(off)
    const int r = threadIdx.x & 63;
    const bool row = r < nb;
    bool sw = false;
#pragma unroll
    for (int q = 0; q < kPanel; q++) {
        const double uqq = rdlane(v[q], q);
        const bool step = q < nb;  // uniform (nb < kPanel only for the last block)
        if (check && step && uqq == uqq && row && r > q && fabs(v[q]) > fabs(uqq)) sw = true;
        // u_qq == 0 skips step q (GSL): a lane predicate below, no branch
        const double zq = rdlane(zr, q);
        double uq[kPanel];
#pragma unroll
        for (int c = q + 1; c < kPanel; c++) uq[c] = rdlane(v[c], q);
        if (step && row && r > q && uqq != 0.0) {
            const double l = v[q] / uqq;
            v[q] = l;
            const double pz = l * zq;
            zr = zr - pz;
#pragma unroll
            for (int c = q + 1; c < kPanel; c++) {
                const double p = l * uq[c];
                v[c] = v[c] - p;
            }
        }
    }
    if (check && __any(sw) && r == 0) *flag = 1;
    if (row) {
#pragma unroll
        for (int c = 0; c < kPanel; c++)
            if (c < nb) A[(size_t)(j + r) * n + j + c] = v[c];
        if (z) z[j + r] = zr;
    }
}

// the diagonal block at (j, j) of n - j <= kPanel rows, factored in place (the
// last one, after k_lu_step's panels); then the earlier panels' U_ii and final
// z (dg / zf, kept aside by k_lu_step) go to A's diagonal and z
__global__ __launch_bounds__(64) void k_lu_diag_at(double* __restrict__ A, int n, int j, double* __restrict__ z,
                                                   int check, int* __restrict__ flag, const double* __restrict__ dg,
                                                   const double* __restrict__ zf) {
    const int r = threadIdx.x, nb = n - j;
    double v[kPanel];
#pragma unroll
    for (int c = 0; c < kPanel; c++) v[c] = (r < nb && c < nb) ? A[(size_t)(j + r) * n + j + c] : 0.0;
    const double zr = (z && r < nb) ? z[j + r] : 0.0;
    factor_diag(v, zr, j, nb, A, n, z, check, flag);
    for (int i = r; i < j; i += 64) {
        A[(size_t)i * n + i] = dg[i];
        if (z) z[i] = zf[i];
    }
}

// One launch per panel, v2 (k_lu_step): no published diagonal block.  Every
// block factors the panel's diagonal block D itself, merged with its tile rows'
// L chains into one right-looking pass over a 64-row panel per "row wave"
// (lanes 0 .. 15: D's rows j0 .. j0 + 15, lanes 16 .. 63: 48 tile rows): at
// step q lane q holds the pivot row, broadcast by readlane, and every lane
// below it takes l = a_q / u_qq and its updates — the per-column elimination's
// operations on these elements, in its order.  Then CW "column waves" solve the
// tile's 64 CW columns' U rows with D's l (LDS), and all 16 waves apply the
// panel's delayed updates to the (48 RW) x (64 CW) tile.  The tile shape is
// picked per panel so that one round of blocks (one 1024-thread block per CU)
// covers the trailing matrix.  Block (0, 0) keeps D's U_ii and final z aside
// (every block of the launch reads D's rows from A), and k_lu_diag_at factors
// the last diagonal block and writes them all back.
constexpr int kStepRows = 48;   // tile rows per row wave (it holds them with D's 16)
constexpr int kStepWaves = 16;  // waves per block
static_assert(kStepRows + kPanel == 64, "a row wave holds D and its tile rows");

// One matrix of a k_lu_step launch.  A launch carries up to two (the setup's
// two studies, late r06): blockIdx.z picks the matrix, so both studies' panels take
// one launch each instead of two launches contending for the CUs; a block
// outside its matrix's trailing part returns at once.
struct LuSet {
    double* A;    // n x n row-major, eliminated in place
    double* z;    // forward-solved in place (may be null)
    int* flag;    // raised when a row swap is needed (check)
    double* dg;   // U_ii of the panels' diagonal blocks, kept aside
    double* zf;   // their final z, kept aside
    int n, check;
};
struct LuSets {
    LuSet s[2];
};

template <int RW, int CW>
__global__ __launch_bounds__(64 * kStepWaves) void k_lu_step(const LuSets P, int j0,
                                                               unsigned long long* __restrict__ tr) {
#pragma clang fp contract(off)
    constexpr int nb = kPanel;
    constexpr int TR = kStepRows * RW, TC = 64 * CW;
    constexpr int kSets = kStepWaves / CW;     // row sets in the update (wave w: column group w % CW)
    constexpr int kRows = TR / kSets;          // rows per wave in the update
    static_assert(RW + CW <= kStepWaves && TR % kSets == 0, "tile shape");
    __shared__ double sD[kPanel][kPanel + 1];  // D factored: l below, u on and above
    __shared__ double sL[TR][kPanel + 1];      // l of the tile's rows
    __shared__ double sU[kPanel][TC];          // u of the tile's columns
    __shared__ unsigned long long sSkip;
    const LuSet& S = blockIdx.z ? P.s[1] : P.s[0];
    double* __restrict__ A = S.A;
    double* __restrict__ z = S.z;
    int* __restrict__ flag = S.flag;
    const int n = S.n, check = S.check;
    const int tb = blockIdx.z ? -1
                              : (blockIdx.x == 0 && blockIdx.y == 0) ? 0 : (blockIdx.x == 1 && blockIdx.y == 1) ? 1 : -1;
    auto stamp = [&](int i) {
        if (tr && tb >= 0 && threadIdx.x == 0) tr[tb * 8 + i] = wall_clock64();
    };
    stamp(0);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int j1 = j0 + nb;
    const int i0 = j1 + blockIdx.y * TR, k0 = j1 + blockIdx.x * TC;
    // outside this matrix's trailing part (the grid covers the larger of a
    // launch's matrices): no rows or columns to update, and the D rows' swap
    // check is block (0, 0)'s as well
    if (i0 >= n || k0 >= n) return;
    if (check && *flag) return;
    double* __restrict__ dg = S.dg;
    double* __restrict__ zf = S.zf;
    const bool corner = blockIdx.x == 0 && blockIdx.y == 0;
    // the update's operands first (its first chunk of rows): their latency hides
    // behind the panel pass
    const int cg = w % CW, rs = w / CW;  // this wave's column group and row set
    const int k = k0 + 64 * cg + lane;
    constexpr int kChunk = kRows < 6 ? kRows : 6;  // rows in registers at a time (more spill)
    static_assert(kRows % kChunk == 0, "update chunks");
    double t[kChunk];
    auto load_chunk = [&](int c0) {
#pragma unroll
        for (int m = 0; m < kChunk; m++) {
            const int i = i0 + rs * kRows + c0 + m;
            t[m] = (i < n && k < n) ? A[(size_t)i * n + k] : 0.0;
        }
    };
    load_chunk(0);
    double v[kPanel];
    if (w < RW) {
        // lane r < 16: D's row j0 + r; lane r >= 16: tile row i0 + 48 w + r - 16
        const int row = lane < nb ? j0 + lane : i0 + kStepRows * w + lane - nb;
        const bool live = row < n;
#pragma unroll
        for (int c = 0; c < kPanel; c++) v[c] = live ? A[(size_t)row * n + j0 + c] : 0.0;
        double zr = (z && live && (lane < nb || blockIdx.x == 0)) ? z[row] : 0.0;
        unsigned long long skip = 0;
        bool sw = false;
#pragma unroll
        for (int q = 0; q < kPanel; q++) {
            const double uqq = rdlane(v[q], q);
            const bool below = lane > q && live;  // D rows below the pivot, every tile row
            if (check && uqq == uqq && below && fabs(v[q]) > fabs(uqq)) sw = true;
            // u_qq == 0 skips step q (GSL): folded into the lane predicate, no
            // uniform branch (one made the compiler copy the whole row per step)
            if (uqq == 0.0) skip |= 1ull << q;
            const double zq = rdlane(zr, q);
            double uq[kPanel];
#pragma unroll
            for (int c = q + 1; c < kPanel; c++) uq[c] = rdlane(v[c], q);
            if (below && uqq != 0.0) {
                const double l = v[q] / uqq;
                v[q] = l;
                const double pz = l * zq;
                zr = zr - pz;
#pragma unroll
                for (int c = q + 1; c < kPanel; c++) {
                    const double p = l * uq[c];
                    v[c] = v[c] - p;
                }
            }
        }
        if (check && __any(sw) && lane == 0) *flag = 1;
        if (lane < nb) {
            if (w == 0) {
#pragma unroll
                for (int c = 0; c < kPanel; c++) sD[lane][c] = v[c];
                // D's U_ii and final z to the side arrays: every block of this launch
                // reads D's rows and z from A / z, so nothing is written back there
                if (corner) {
#pragma unroll
                    for (int c = 0; c < kPanel; c++)
                        if (c == lane) dg[j0 + lane] = v[c];
                    zf[j0 + lane] = zr;
                }
            }
        } else {
#pragma unroll
            for (int c = 0; c < kPanel; c++) sL[kStepRows * w + lane - nb][c] = v[c];
            if (z && blockIdx.x == 0 && live) z[row] = zr;
        }
        if (w == 0 && lane == 0) sSkip = skip;
    } else if (w < RW + CW) {
        const int kc = k0 + 64 * (w - RW) + lane;
#pragma unroll
        for (int c = 0; c < kPanel; c++) v[c] = (kc < n) ? A[(size_t)(j0 + c) * n + kc] : 0.0;
    }
    __syncthreads();
    stamp(1);
    const unsigned long long skip = sSkip;
    if (w >= RW && w < RW + CW) {  // U-row solve of column k0 + 64 (w - RW) + lane with D's l
#pragma unroll
        for (int r = 1; r < kPanel; r++) {
#pragma unroll
            for (int q = 0; q < r; q++) {
                if ((skip >> q) & 1) continue;
                const double p = sD[r][q] * v[q];
                v[r] = v[r] - p;
            }
        }
#pragma unroll
        for (int q = 0; q < kPanel; q++) sU[q][64 * (w - RW) + lane] = v[q];
    }
    __syncthreads();
    stamp(2);
    double uc[kPanel];  // this lane's column of the panel's U rows
#pragma unroll
    for (int q = 0; q < kPanel; q++) uc[q] = sU[q][64 * cg + lane];
    // the chunks' loads run one chunk ahead of their updates (r06: the update
    // waited a full load round trip per chunk, ~4 of them per panel at M = 2000)
    double tn[kChunk];
#pragma unroll
    for (int c0 = 0; c0 < kRows; c0 += kChunk) {
        if (c0 + kChunk < kRows) {
#pragma unroll
            for (int m = 0; m < kChunk; m++) {
                const int i = i0 + rs * kRows + c0 + kChunk + m;
                tn[m] = (i < n && k < n) ? A[(size_t)i * n + k] : 0.0;
            }
        }
#pragma unroll
        for (int q = 0; q < kPanel; q++) {
            if ((skip >> q) & 1) continue;
#pragma unroll
            for (int m = 0; m < kChunk; m++) {
                const double p = sL[rs * kRows + c0 + m][q] * uc[q];
                t[m] = t[m] - p;
            }
        }
#pragma unroll
        for (int m = 0; m < kChunk; m++) {
            const int ii = i0 + rs * kRows + c0 + m;
            if (ii < n && k < n) A[(size_t)ii * n + k] = t[m];
        }
#pragma unroll
        for (int m = 0; m < kChunk; m++) t[m] = tn[m];
    }
    stamp(3);
}

// one panel's k_lu_step over the matrices of P that still have a trailing part
// at j0: the smallest tile whose blocks (summed over the matrices) fit one
// round (one 1024-thread block per CU), else the largest
void launch_lu_step(const LuSets& P, int ns, int j0, unsigned long long* tr, hipStream_t st) {
    int rest = 0;  // the grid's extent: the largest trailing part
    for (int s = 0; s < ns; s++) rest = std::max(rest, P.s[s].n - j0 - kPanel);
    auto blocks = [&](int rw, int cw) {
        long b = 0;
        for (int s = 0; s < ns; s++) {
            const int r = P.s[s].n - j0 - kPanel;
            if (r > 0) b += (long)((r + kStepRows * rw - 1) / (kStepRows * rw)) * ((r + 64 * cw - 1) / (64 * cw));
        }
        return b;
    };
    constexpr long kRound = 256;
    const dim3 b(64 * kStepWaves);
#define PSX_LU_STEP(RW, CW)                                                                                         \
    hipLaunchKernelGGL((k_lu_step<RW, CW>),                                                                         \
                       dim3((rest + 64 * CW - 1) / (64 * CW), (rest + kStepRows * RW - 1) / (kStepRows * RW), ns), \
                       b, 0, st, P, j0, tr)
    if (blocks(1, 1) <= kRound) PSX_LU_STEP(1, 1);
    else if (blocks(1, 2) <= kRound) PSX_LU_STEP(1, 2);
    else if (blocks(2, 2) <= kRound) PSX_LU_STEP(2, 2);
    else if (blocks(2, 4) <= kRound) PSX_LU_STEP(2, 4);
    else PSX_LU_STEP(3, 4);
#undef PSX_LU_STEP
}

// The partial-pivot elimination (GSL 2.5 gsl_linalg_LU_decomp), blocked the
// LAPACK getrf way: the panel (rows j0 .. n - 1, LDS, odd row stride) takes
// each step's pivot (first row of maximal |a_iq|, NaNs never chosen, a NaN
// a_qq keeps row q), swaps whole panel rows, stores l in place of a_iq and
// updates the panel columns; then the trailing columns take the panel's swaps
// in step order, the U-row solve, and k_lu_trail's delayed updates.  Swaps
// only move data, and a row at position q is never moved after step q, so
// every element of U sees the unblocked elimination's operations on the same
// values: U_ii and the swap count are bit-identical.
__global__ __launch_bounds__(kPanelThreads) void k_lu_panel_piv(double* __restrict__ A, int n, int j0, int nb,
                                                                double* __restrict__ Lp, double* __restrict__ sk,
                                                                int* __restrict__ swp) {
#pragma clang fp contract(off)
    __shared__ double sT[kPanel][kPanel];
    __shared__ double sSk[kPanel];
    __shared__ int sPiv[kPanel];
    __shared__ double wv[kPanelThreads / 64];
    __shared__ int wi[kPanelThreads / 64];
    extern __shared__ double sP[];
    const int t = threadIdx.x;
    const int R = n - j0;
    const int ls = nb + 1;
    for (int e = t; e < R * nb; e += kPanelThreads) sP[(e / nb) * ls + e % nb] = A[(size_t)(j0 + e / nb) * n + j0 + e % nb];
    __syncthreads();
    for (int qq = 0; qq < nb; qq++) {
        double mx = -1.0;
        int ip = R;
        for (int r = qq + t; r < R; r += kPanelThreads) {
            const double v = fabs(sP[r * ls + qq]);
            if (v > mx) { mx = v; ip = r; }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const double v2 = __shfl_xor(mx, o);
            const int i2 = __shfl_xor(ip, o);
            if (v2 > mx || (v2 == mx && i2 < ip)) { mx = v2; ip = i2; }
        }
        if ((t & 63) == 0) { wv[t >> 6] = mx; wi[t >> 6] = ip; }
        __syncthreads();
        mx = wv[0];
        ip = wi[0];
        for (int w = 1; w < kPanelThreads / 64; w++)
            if (wv[w] > mx || (wv[w] == mx && wi[w] < ip)) { mx = wv[w]; ip = wi[w]; }
        const double a0 = sP[qq * ls + qq];
        const int p = (a0 != a0 || ip >= R) ? qq : ip;
        if (t == 0) {
            sPiv[qq] = p;
            swp[j0 + qq] = (p != qq) ? 1 : 0;
        }
        __syncthreads();  // every thread has read wv / wi and row qq's old a_qq
        if (p != qq) {
            if (t < nb) {
                const double x = sP[qq * ls + t];
                sP[qq * ls + t] = sP[p * ls + t];
                sP[p * ls + t] = x;
            }
            __syncthreads();
        }
        const double aqq = sP[qq * ls + qq];
        if (t == 0) sk[qq] = sSk[qq] = (aqq == 0.0) ? 1.0 : 0.0;
        if (aqq == 0.0) continue;  // uniform
        for (int r = qq + 1 + t; r < R; r += kPanelThreads) {
            const double l = sP[r * ls + qq] / aqq;
            sP[r * ls + qq] = l;
            for (int c = qq + 1; c < nb; c++) {
                const double pc = l * sP[qq * ls + c];
                sP[r * ls + c] = sP[r * ls + c] - pc;
            }
        }
        __syncthreads();
    }
    __syncthreads();
    for (int e = t; e < R * nb; e += kPanelThreads) {
        const int r = e / nb, c = e % nb;
        const double v = sP[r * ls + c];
        if (r > c) Lp[(size_t)c * n + j0 + r] = v;  // l, at the row's final position
        A[(size_t)(j0 + r) * n + j0 + c] = v;
    }
    for (int e = t; e < kPanel * kPanel; e += kPanelThreads) {
        const int q = e / kPanel, r = e % kPanel;
        sT[q][r] = (q < r && r < nb) ? sP[r * ls + q] : 0.0;
    }
    __syncthreads();
    for (int k = j0 + nb + t; k < n; k += kPanelThreads) {
        for (int q = 0; q < nb; q++) {  // the panel's swaps, in step order
            const int p = sPiv[q];
            if (p != q) {
                double* const x = A + (size_t)(j0 + q) * n + k;
                double* const y = A + (size_t)(j0 + p) * n + k;
                const double tq = *x;
                *x = *y;
                *y = tq;
            }
        }
        double u[kPanel];
#pragma unroll
        for (int r = 0; r < kPanel; r++) u[r] = r < nb ? A[(size_t)(j0 + r) * n + k] : 0.0;
#pragma unroll
        for (int r = 1; r < kPanel; r++) {
            if (r >= nb) break;
#pragma unroll
            for (int q = 0; q < r; q++) {
                if (sSk[q] != 0.0) continue;
                const double prod = sT[q][r] * u[q];
                u[r] = u[r] - prod;
            }
            A[(size_t)(j0 + r) * n + k] = u[r];
        }
    }
}

__global__ __launch_bounds__(kTrCols * kTrGroups) void k_lu_trail(double* __restrict__ A, int n, int j0, int nb,
                                                                  const double* __restrict__ Lp,
                                                                  const double* __restrict__ sk,
                                                                  const int* __restrict__ flag) {
#pragma clang fp contract(off)
    constexpr int kPer = kTrRows / kTrGroups;  // rows per thread, independent chains
    __shared__ double sL[kPanel][kTrRows];
    __shared__ double sS[kPanel];
    if (*flag) return;
    const int tx = threadIdx.x, ty = threadIdx.y, t = ty * kTrCols + tx;
    const int c0 = j0 + nb;  // first trailing column / row
    const int i0 = c0 + blockIdx.y * kTrRows;
    const int nr = max(0, min(kTrRows, n - i0));
    for (int e = t; e < kPanel * kTrRows; e += kTrCols * kTrGroups) {
        const int q = e / kTrRows, r = e % kTrRows;
        sL[q][r] = (q < nb && r < nr) ? Lp[(size_t)q * n + i0 + r] : 0.0;
    }
    if (t < kPanel) sS[t] = t < nb ? sk[t] : 1.0;
    __syncthreads();
    const int k = c0 + blockIdx.x * kTrCols + tx;
    if (k >= n) return;
    double u[kPanel];  // the panel's U rows, final (k_lu_panel)
#pragma unroll
    for (int q = 0; q < kPanel; q++) u[q] = q < nb ? A[(size_t)(j0 + q) * n + k] : 0.0;
    double v[kPer];
#pragma unroll
    for (int m = 0; m < kPer; m++) {
        const int r = ty + kTrGroups * m;
        v[m] = r < nr ? A[(size_t)(i0 + r) * n + k] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < kPanel; q++) {
        if (q >= nb) break;
        if (sS[q] != 0.0) continue;
#pragma unroll
        for (int m = 0; m < kPer; m++) {
            const double prod = sL[q][ty + kTrGroups * m] * u[q];
            v[m] = v[m] - prod;
        }
    }
#pragma unroll
    for (int m = 0; m < kPer; m++) {
        const int r = ty + kTrGroups * m;
        if (r < nr) A[(size_t)(i0 + r) * n + k] = v[m];
    }
}

// *asym = 1 when L is not exactly symmetric (any L_ik != L_ki, NaNs included)
__global__ void k_sym_check(const double* __restrict__ L, int n, int* __restrict__ asym) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)n * n) return;
    const int i = (int)(idx / n), k = (int)(idx % n);
    if (k > i && !(L[idx] == L[(size_t)k * n + i])) *asym = 1;
}

__global__ void k_get_diag(const double* __restrict__ A, int n, double* __restrict__ d) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) d[i] = A[(size_t)i * n + i];
}

int chk(hipError_t e, const char* what, std::string* err) {
    if (e == hipSuccess) return 0;
    if (err) *err = std::string(what) + ": " + hipGetErrorString(e);
    return -1;
}

// enqueue the partial-pivot elimination of A (n x n, device) on st
// (returns -1 with *err set when a launch failed; the HIP error is read once, here)
int enqueue_lu(double* A, int n, int* dswp, hipStream_t st, std::string* err) {
    for (int j = 0; j < n - 1; j++) {
        hipLaunchKernelGGL(k_lu_pivot, dim3(1), dim3(1024), 0, st, A, n, j, dswp);
        const int r = n - j - 1;
        hipLaunchKernelGGL(k_elim, dim3((r + kElimCols - 1) / kElimCols, (r + kElimRows - 1) / kElimRows),
                           dim3(kElimCols), 0, st, A, n, j, (double*)nullptr);
    }
    return chk(hipGetLastError(), "LU launch", err);
}

// enqueue the tiled swap-free elimination (one k_lu_step per panel, then
// k_lu_diag_at); with check, *flag != 0 afterwards when some column needed a
// row swap (A is then partly eliminated: recopy and pivot).  Afterwards A's
// diagonal holds U_ii and z holds z~.  work: 2 n doubles (U_ii / z kept aside).  Returns -1 with *err set when a
// launch failed (the HIP error is read once, here).
// The matrices of P (ns of them, each with work = 2 n doubles) in joint
// launches: every panel of every matrix in one k_lu_step per panel index.
int enqueue_lu_sets(const LuSets& P, int ns, hipStream_t st, std::string* err) {
    int nmax = 0;
    for (int s = 0; s < ns; s++) {
        if (chk(hipMemsetAsync(P.s[s].flag, 0, sizeof(int), st), "memset", err)) return -1;
        nmax = std::max(nmax, P.s[s].n);
    }
    // PSX_LU_TRACE (diagnostics): per-panel phase clocks of two tiles of the
    // first matrix, averaged on stderr
    static const bool trace = std::getenv("PSX_LU_TRACE") != nullptr;
    const int n = P.s[0].n;
    const int npan = std::max(0, (n - 1) / kPanel);
    unsigned long long* tr = nullptr;
    if (trace && npan > 0) {
        if (chk(psx::dmalloc(&tr, sizeof(unsigned long long) * 16 * npan), "trace", err)) return -1;
        (void)hipMemsetAsync(tr, 0, sizeof(unsigned long long) * 16 * npan, st);
    }
    int p = 0, j0 = 0;
    for (; j0 + kPanel < nmax; j0 += kPanel, p++)
        launch_lu_step(P, ns, j0, tr && p < npan ? tr + 16 * p : nullptr, st);
    // per matrix: the last diagonal block (n - j0 <= kPanel rows), then U_ii / z
    // of the others
    for (int s = 0; s < ns; s++) {
        const LuSet& S = P.s[s];
        int js = 0;
        while (js + kPanel < S.n) js += kPanel;
        hipLaunchKernelGGL(k_lu_diag_at, dim3(1), dim3(64), 0, st, S.A, S.n, js, S.z, S.check, S.flag,
                           (const double*)S.dg, (const double*)S.zf);
    }
    if (tr) {
        std::vector<unsigned long long> h(16 * (size_t)npan);
        (void)hipMemcpyAsync(h.data(), tr, h.size() * 8, hipMemcpyDeviceToHost, st);
        (void)hipStreamSynchronize(st);
        double ph[2][4] = {{0}}, cnt[2] = {0, 0};
        for (int q = 0; q < npan; q++)
            for (int b = 0; b < 2; b++) {
                const unsigned long long* t = h.data() + 16 * q + 8 * b;
                if (!t[0] || !t[3]) continue;
                cnt[b]++;
                for (int i = 0; i < 3; i++) ph[b][i] += (double)(t[i + 1] - t[i]) * 0.01;  // 100 MHz -> us
                if (b == 0 && t[4]) ph[b][3] += (double)(t[4] - t[3]) * 0.01;
            }
        // panel to panel: block (0, 0)'s start of panel q + 1 after its end of panel q
        double gap = 0, per = 0;
        int ng = 0;
        for (int q = 0; q + 1 < npan; q++) {
            const unsigned long long* a = h.data() + 16 * q;
            const unsigned long long* b = h.data() + 16 * (q + 1);
            if (!a[0] || !a[3] || !b[0]) continue;
            gap += (double)(b[0] - a[3]) * 0.01;
            per += (double)(b[0] - a[0]) * 0.01;
            ng++;
        }
        fprintf(stderr, "psx-lu-trace n=%d panels=%d block(0,0): %.2f %.2f %.2f us; block(1,1): %.2f %.2f %.2f us "
                        "(loads + D + L pass | U solve | update); block (0,0) end -> next panel's start %.2f us, "
                        "panel to panel %.2f us\n",
                n, npan, ph[0][0] / std::max(1.0, cnt[0]), ph[0][1] / std::max(1.0, cnt[0]),
                ph[0][2] / std::max(1.0, cnt[0]), ph[1][0] / std::max(1.0, cnt[1]),
                ph[1][1] / std::max(1.0, cnt[1]), ph[1][2] / std::max(1.0, cnt[1]), gap / std::max(1, ng),
                per / std::max(1, ng));
        psx::dfree(tr);
    }
    return chk(hipGetLastError(), "LU launch", err);
}

LuSet lu_set(double* A, int n, double* work, int* flag, double* z, bool check) {
    return LuSet{A, z, flag, work, work + n, n, check ? 1 : 0};
}

int enqueue_lu_fused(double* A, int n, double* work, int* flag, double* z, hipStream_t st, std::string* err,
                     bool check = true) {
    LuSets P{};
    P.s[0] = lu_set(A, n, work, flag, z, check);
    return enqueue_lu_sets(P, 1, st, err);
}

// Study s arrives at its first elimination (LuJoin).  Returns 1 when the joint
// launches cover this matrix (enqueued on study 0's stream; st ordered after
// them), 0 when the study eliminates on its own, -1 on a launch error.
int lu_join_run(LuJoin* J, int s, double* A, int n, double* work, int* flag, double* z, hipStream_t st,
                std::string* err) {
    std::unique_lock<std::mutex> lk(J->m);
    if (s == 1 && (chk(hipEventCreateWithFlags(&J->ready, hipEventDisableTiming), "event", err) ||
                   chk(hipEventRecord(J->ready, st), "event", err))) {
        J->in[s] = true;  // arrives without a matrix: the other study goes alone
        J->cv.notify_all();
        return -1;
    }
    J->A[s] = A;
    J->n[s] = n;
    J->work[s] = work;
    J->flag[s] = flag;
    J->z[s] = z;
    J->st[s] = st;
    J->in[s] = J->mat[s] = true;
    J->cv.notify_all();
    J->cv.wait(lk, [&] { return J->in[0] && J->in[1]; });
    if (!(J->mat[0] && J->mat[1])) return 0;
    if (s == 1) {
        J->cv.wait(lk, [&] { return J->state != 0; });
        if (J->state != 1) {
            if (err) *err = J->err;
            return -1;
        }
        return chk(hipStreamWaitEvent(st, J->done, 0), "event wait", err) ? -1 : 1;
    }
    lk.unlock();
    std::string e;
    LuSets P{};
    for (int q = 0; q < 2; q++) P.s[q] = lu_set(J->A[q], J->n[q], J->work[q], J->flag[q], J->z[q], true);
    int rc = chk(hipStreamWaitEvent(st, J->ready, 0), "event wait", &e);
    if (!rc) rc = enqueue_lu_sets(P, 2, st, &e);
    if (!rc) rc = chk(hipEventCreateWithFlags(&J->done, hipEventDisableTiming), "event", &e);
    if (!rc) rc = chk(hipEventRecord(J->done, st), "event", &e);
    lk.lock();
    J->state = rc ? 2 : 1;
    J->err = e;
    J->cv.notify_all();
    if (rc && err) *err = e;
    return rc ? -1 : 1;
}

}  // namespace

void LuJoin::leave(int s) {
    std::lock_guard<std::mutex> g(m);
    if (!in[s]) {
        in[s] = true;
        cv.notify_all();
    }
}

LuJoin::~LuJoin() {
    if (ready) (void)hipEventDestroy(ready);
    if (done) (void)hipEventDestroy(done);
}

int lu_det_device(double* dA, int n, int* dswp, double* ddiag, hipStream_t st, double* det, std::string* err) {
    if (n <= 0) return -1;
    // blocked when the panel fits the LDS budget (PSX_LU_UNBLOCKED=1: per-column launches)
    int pw = kPanel;
    while (pw > 1 && (size_t)n * (pw + 1) * sizeof(double) > (size_t)(64 * 1024)) pw--;
    // per call: the attribute is per device, and a process may drive several
    const bool attr = hipFuncSetAttribute((const void*)k_lu_panel_piv, hipFuncAttributeMaxDynamicSharedMemorySize,
                                          kPanelLds) == hipSuccess;
    (void)hipGetLastError();
    if (attr) {
        pw = kPanel;
        while (pw > 1 && (size_t)n * (pw + 1) * sizeof(double) > (size_t)kPanelLds) pw--;
    }
    const size_t need = (size_t)n * (pw + 1) * sizeof(double);
    if (need <= (size_t)(attr ? kPanelLds : 64 * 1024) && !std::getenv("PSX_LU_UNBLOCKED")) {
        double* work = nullptr;
        if (chk(psx::dmalloc(&work, ((size_t)kPanel * n + kPanel) * sizeof(double) + sizeof(int)), "LU work", err))
            return -1;
        double* const sk = work + (size_t)kPanel * n;
        int* const zflag = (int*)(sk + kPanel);
        int rc = chk(hipMemsetAsync(zflag, 0, sizeof(int), st), "memset", err);
        for (int j0 = 0; !rc && j0 < n - 1; j0 += pw) {
            const int nb = std::min(pw, n - 1 - j0);
            const int rest = n - j0 - nb;
            hipLaunchKernelGGL(k_lu_panel_piv, dim3(1), dim3(kPanelThreads), (size_t)(n - j0) * (nb + 1) * sizeof(double),
                               st, dA, n, j0, nb, work, sk, dswp);
            hipLaunchKernelGGL(k_lu_trail, dim3((rest + kTrCols - 1) / kTrCols, (rest + kTrRows - 1) / kTrRows),
                               dim3(kTrCols, kTrGroups), 0, st, dA, n, j0, nb, (const double*)work, (const double*)sk,
                               (const int*)zflag);
        }
        if (!rc) rc = chk(hipGetLastError(), "LU launch", err);
        if (!rc) rc = chk(hipStreamSynchronize(st), "LU sync", err);
        psx::dfree(work);
        if (rc) return rc;
    } else if (enqueue_lu(dA, n, dswp, st, err)) {
        return -1;
    }
    hipLaunchKernelGGL(k_get_diag, dim3((n + 255) / 256), dim3(256), 0, st, dA, n, ddiag);
    std::vector<double> diag(n);
    std::vector<int> swp(std::max(n - 1, 1), 0);
    if (chk(hipMemcpyAsync(diag.data(), ddiag, n * sizeof(double), hipMemcpyDeviceToHost, st), "copy", err)) return -1;
    if (n > 1 && chk(hipMemcpyAsync(swp.data(), dswp, (n - 1) * sizeof(int), hipMemcpyDeviceToHost, st), "copy", err))
        return -1;
    if (chk(hipStreamSynchronize(st), "LU sync", err)) return -1;
    // gsl_linalg_LU_det: signum, then the U_ii multiplied in index order
    int signum = 1;
    for (int j = 0; j < n - 1; j++)
        if (swp[j]) signum = -signum;
    double d = signum;
    for (int i = 0; i < n; i++) d *= diag[i];
    *det = d;
    return 0;
}

int elim_device(const double* a, int n, const double* z, int check, double* piv, double* zt, int* swap,
                std::string* err) {
    if (n <= 0) return -1;
    const size_t nn = (size_t)n * n;
    double *dA = nullptr, *dz = nullptr, *dw = nullptr, *dd = nullptr;
    int* dflag = nullptr;
    int rc = 0;
    if (chk(psx::dmalloc(&dA, nn * sizeof(double)), "alloc", err) || chk(psx::dmalloc(&dz, n * sizeof(double)), "alloc", err) ||
        chk(psx::dmalloc(&dw, 2 * (size_t)n * sizeof(double)), "alloc", err) ||
        chk(psx::dmalloc(&dd, n * sizeof(double)), "alloc", err) || chk(psx::dmalloc(&dflag, sizeof(int)), "alloc", err))
        rc = -1;
    if (!rc) rc = chk(hipMemcpy(dA, a, nn * sizeof(double), hipMemcpyHostToDevice), "upload", err);
    if (!rc && z) rc = chk(hipMemcpy(dz, z, n * sizeof(double), hipMemcpyHostToDevice), "upload", err);
    if (!rc) rc = enqueue_lu_fused(dA, n, dw, dflag, z ? dz : nullptr, nullptr, err, check != 0);
    if (!rc) {
        hipLaunchKernelGGL(k_get_diag, dim3((n + 255) / 256), dim3(256), 0, nullptr, dA, n, dd);
        rc = chk(hipGetLastError(), "launch", err);
    }
    if (!rc) rc = chk(hipMemcpy(piv, dd, n * sizeof(double), hipMemcpyDeviceToHost), "copy", err);
    if (!rc && z) rc = chk(hipMemcpy(zt, dz, n * sizeof(double), hipMemcpyDeviceToHost), "copy", err);
    if (!rc) rc = chk(hipMemcpy(swap, dflag, sizeof(int), hipMemcpyDeviceToHost), "copy", err);
    psx::dfree(dA); psx::dfree(dz); psx::dfree(dw); psx::dfree(dd); psx::dfree(dflag);
    return rc;
}

int ld_study_setup(const double* ld, const double* z, int M, hipStream_t st, double* dS, double* dy,
                   LdStudyResult* res, std::string* err, LuJoin* join, int s) {
    std::memset(res, 0, sizeof(*res));
    using clk = std::chrono::steady_clock;
    auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    const clk::time_point t0 = clk::now();
    clk::time_point t1 = t0, t2 = t0;
    const size_t nn = (size_t)M * M;
    double *dL = nullptr, *dA = nullptr, *dz = nullptr, *ddiag = nullptr, *dcol = nullptr;
    int* dswp = nullptr;
    auto cleanup = [&]() {
        (void)hipStreamSynchronize(st);
        psx::IdleScope idle;  // the scratch is used on st only
        psx::dfree(dL); psx::dfree(dA); psx::dfree(dz); psx::dfree(ddiag); psx::dfree(dcol); psx::dfree(dswp);
    };
    if (psx::dmalloc(&dL, nn * sizeof(double)) != hipSuccess || psx::dmalloc(&dA, nn * sizeof(double)) != hipSuccess ||
        psx::dmalloc(&dz, M * sizeof(double)) != hipSuccess || psx::dmalloc(&ddiag, M * sizeof(double)) != hipSuccess ||
        psx::dmalloc(&dcol, ((size_t)kPanel * M + kPanel) * sizeof(double)) != hipSuccess ||
        psx::dmalloc(&dswp, (std::max(M, 1) + 2) * sizeof(int)) != hipSuccess) {
        cleanup();
        if (err) *err = "out of device memory (LD setup)";
        return -1;
    }
    int* const dflag = dswp + std::max(M, 1);
    // an exactly symmetric LD whose elimination needs no row swap gives step 2's
    // unpivoted elimination of Sigma' bit for bit (same matrix, same operations):
    // z's forward solve then rides in step 1 and step 2 is not run again
    int* const dasym = dflag + 1;
    int hasym = 1;
    const int cb = 256;
    const unsigned gb = (unsigned)((nn + cb - 1) / cb);
    int rc = 0;
    do {
        if ((rc = chk(hipMemcpyAsync(dL, ld, nn * sizeof(double), hipMemcpyHostToDevice, st), "LD upload", err))) break;
        t1 = clk::now();
        if ((rc = chk(hipMemsetAsync(dasym, 0, sizeof(int), st), "memset", err))) break;
        hipLaunchKernelGGL(k_sym_check, dim3(gb), dim3(cb), 0, st, dL, M, dasym);
        if ((rc = chk(hipMemcpyAsync(&hasym, dasym, sizeof(int), hipMemcpyDeviceToHost, st), "copy", err))) break;
        // 1. util.cpp:195-226: add 0.01 until det(LU) > 0
        double add = 0.0;
        int it = 0;
        bool fused = false;      // the last LU ran swap-free with z's forward solve
        bool try_fused = true;   // until some shift of this LD needed a row swap
        std::vector<double> udiag(M);
        for (;; it++) {
            if (it >= 100000) { rc = -1; if (err) *err = "PSD shift did not terminate"; break; }
            hipLaunchKernelGGL(k_psd_copy, dim3(gb), dim3(cb), 0, st, dL, M, add, dA);
            double det = 0;
            int hflag = 1;
            if (try_fused) {
                if ((rc = chk(hipMemcpyAsync(dz, z, M * sizeof(double), hipMemcpyHostToDevice, st), "z upload", err)))
                    break;
                // the first elimination in joint launches with the other study (LuJoin)
                const int jr = (join && it == 0) ? lu_join_run(join, s, dA, M, dcol, dflag, dz, st, err) : 0;
                if (jr < 0) { rc = -1; break; }
                if (jr == 0 && enqueue_lu_fused(dA, M, dcol, dflag, dz, st, err)) { rc = -1; break; }
                hipLaunchKernelGGL(k_get_diag, dim3((M + 255) / 256), dim3(256), 0, st, dA, M, ddiag);
                if ((rc = chk(hipMemcpyAsync(udiag.data(), ddiag, M * sizeof(double), hipMemcpyDeviceToHost, st),
                              "copy", err)) ||
                    (rc = chk(hipMemcpyAsync(&hflag, dflag, sizeof(int), hipMemcpyDeviceToHost, st), "copy", err)) ||
                    (rc = chk(hipStreamSynchronize(st), "LU sync", err)))
                    break;
                if (hflag) {  // a row swap is needed: the pivoting elimination from a fresh copy
                    try_fused = false;
                    hipLaunchKernelGGL(k_psd_copy, dim3(gb), dim3(cb), 0, st, dL, M, add, dA);
                }
            }
            if (!hflag) {
                // gsl_linalg_LU_det with signum +1: the U_ii multiplied in index order
                det = 1.0;
                for (int i = 0; i < M; i++) det *= udiag[i];
                fused = true;
            } else {
                if ((rc = lu_det_device(dA, M, dswp, ddiag, st, &det, err))) break;
                fused = false;
            }
            if (det > 0) break;
            add += 0.01;
        }
        if (rc) break;
        t2 = clk::now();
        res->added = add;
        res->psd_iterations = it + 1;
        // 2. Sigma' (lower triangle, symmetrised) -> dS; elimination without pivoting
        //    of a copy with z's forward solve: pivots D, z~ = L^-1 z
        hipLaunchKernelGGL(k_sym_lower, dim3(gb), dim3(cb), 0, st, dL, M, add, dS);
        std::vector<double> piv(M), zt(M), dg(M);
        const bool sym = hasym == 0;  // read back with the first LU sync
        if (fused && sym) {
            piv = udiag;
            if ((rc = chk(hipMemcpyAsync(zt.data(), dz, M * sizeof(double), hipMemcpyDeviceToHost, st), "copy", err)))
                break;
            for (int i = 0; i < M; i++) dg[i] = ld[(size_t)i * M + i] + add;  // k_sym_lower's diagonal
        } else {
            if ((rc = chk(hipMemcpyAsync(dA, dS, nn * sizeof(double), hipMemcpyDeviceToDevice, st), "copy", err)))
                break;
            if ((rc = chk(hipMemcpyAsync(dz, z, M * sizeof(double), hipMemcpyHostToDevice, st), "z upload", err)))
                break;
            // elimination without pivoting: the tiled panels with the pivot check off
            if (enqueue_lu_fused(dA, M, dcol, dflag, dz, st, err, false)) { rc = -1; break; }
            hipLaunchKernelGGL(k_get_diag, dim3((M + 255) / 256), dim3(256), 0, st, dA, M, ddiag);
            if ((rc = chk(hipGetLastError(), "elimination launch", err))) break;
            hipMemcpyAsync(piv.data(), ddiag, M * sizeof(double), hipMemcpyDeviceToHost, st);
            hipMemcpyAsync(zt.data(), dz, M * sizeof(double), hipMemcpyDeviceToHost, st);
            hipLaunchKernelGGL(k_get_diag, dim3((M + 255) / 256), dim3(256), 0, st, dS, M, ddiag);
            hipMemcpyAsync(dg.data(), ddiag, M * sizeof(double), hipMemcpyDeviceToHost, st);
        }
        if ((rc = chk(hipStreamSynchronize(st), "elimination sync", err))) break;
        res->fused_route = (fused && sym) ? 1 : 0;
        double dmax = 0, pmin = INFINITY;
        for (int i = 0; i < M; i++) {
            dmax = std::max(dmax, std::fabs(dg[i]));
            pmin = std::min(pmin, piv[i]);
        }
        res->min_pivot_ratio = dmax > 0 ? pmin / dmax : 0.0;
        if (!(res->min_pivot_ratio > kPdRatio)) {
            // not (comfortably) positive definite: the caller takes the eigen route
            res->path = 1;
            res->sigma_host_needed = 1;
            break;
        }
        double q = 0;
        for (int i = 0; i < M; i++) q += zt[i] * zt[i] / piv[i];
        res->spsq = q;
        res->path = 0;
        if ((rc = chk(hipMemcpyAsync(dy, z, M * sizeof(double), hipMemcpyHostToDevice, st), "y upload", err))) break;
        if ((rc = chk(hipStreamSynchronize(st), "setup sync", err))) break;
    } while (false);
    cleanup();
    const clk::time_point t3 = clk::now();
    res->upload_ms = ms(t0, t1);
    res->psd_ms = ms(t1, t2);
    res->finish_ms = ms(t2, t3);
    return rc;
}

// load this translation unit's device code on the current device (psx_warmup)
int warm_module_setup() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, (const void*)k_get_diag) == hipSuccess ? 0 : -1;
}

}  // namespace psx
