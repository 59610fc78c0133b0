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
//  * Step 1 runs here as a right-looking elimination, blocked (an LDS panel
//    of <= kPanel columns, trailing updates delayed; swap-free LDs without
//    pivot search, others with GSL's pivot and the swaps replayed on the
//    trailing columns; per-column launches past the LDS budget), with the
//    reference's operation
//    order and IEEE rounding (division correctly rounded, multiply and
//    subtract not fused), so the per-element update sequence — and hence
//    every U_ii and the index-order determinant product — is bit-identical to
//    the host restatement psx_psd_shift (model.cpp), the oracle of this step.
//  * Positive definiteness and z^T Sigma'^-1 z come from one elimination
//    without pivoting of the symmetrised Sigma' (its pivots are the D of
//    L D L^T) with the forward solve of z fused in.  When some pivot is not
//    comfortably positive (ratio to the largest diagonal < kPdRatio) the
//    caller falls back to the reference's eigen route (host restatement).
//
// The trailing update is an HBM/L2 streaming kernel (one read-modify-write of
// the trailing matrix per panel); the matrix (32 MB at M = 2000) stays
// L2/MALL resident.  The panel kernel is one workgroup on one CU (its LDS
// throughput bounds it); launch latency dominates below a few hundred rows.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "psx_setup.h"

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

// Swap-free elimination, blocked with delayed updates (LD matrices: the
// diagonal stays the column maximum, so no row is ever swapped).  Element
// (i, k) of the right-looking elimination receives, for every step q <
// min(i, k), a_ik <- a_ik - l_iq * u_qk (multiply and subtract not fused), in
// increasing q.  Delaying the updates of columns beyond a kPanel-wide panel
// and applying them later, still in increasing q and with the same l_iq and
// u_qk, gives every element — U_ii, z~ — bit for bit what the per-column
// elimination gives, at one read-modify-write of the trailing matrix per
// panel instead of per column.
//   k_lu_panel  (one workgroup): steps j0 .. j0 + nb - 1 on the panel columns
//               and z; l_iq kept in Lp[q - j0][i]; a row swap (GSL's pivot, the
//               first row of maximal |a_iq| with NaNs never chosen, would not be
//               row q) raises *flag and every later launch returns at once (the
//               caller reruns the pivoting path from a fresh copy); a_qq == 0
//               skips the step (GSL), marked in sk[q - j0].
//               Then the panel's U rows on the trailing columns (row j0 + r
//               takes steps j0 .. j0 + r - 1, one column per thread).
//   k_lu_trail  the panel's nb updates on rows and columns >= j0 + nb,
//               kTrRows rows per block (kTrRows / kTrGroups independent rows
//               per thread), l from LDS.
constexpr int kPanel = 16;
constexpr int kPanelThreads = 1024;
constexpr int kTrCols = 64;
constexpr int kTrRows = 32;
constexpr int kTrGroups = 4;  // row groups per trailing block (kTrRows / kTrGroups rows per thread)
constexpr int kPanelLds = 152 * 1024;  // dynamic LDS budget of k_lu_panel_lds (160 KB per CU; 158 KB is refused)

__global__ __launch_bounds__(kPanelThreads) void k_lu_panel(double* __restrict__ A, int n, int j0, int nb,
                                                            double* __restrict__ Lp, double* __restrict__ sk,
                                                            int* __restrict__ flag, double* __restrict__ z) {
#pragma clang fp contract(off)
    if (*flag) return;
    const int t = threadIdx.x;
    for (int q = j0; q < j0 + nb; q++) {
        const double aqq = A[(size_t)q * n + q];
        const double mq = fabs(aqq);
        bool swap = false;
        if (aqq == aqq)
            for (int i = q + 1 + t; i < n; i += kPanelThreads) swap |= fabs(A[(size_t)i * n + q]) > mq;
        if (__syncthreads_or(swap)) {
            if (t == 0) *flag = 1;
            return;
        }
        if (t == 0) sk[q - j0] = (aqq == 0.0) ? 1.0 : 0.0;
        if (aqq == 0.0) continue;  // uniform
        const double zq = z[q];
        double* const lq = Lp + (size_t)(q - j0) * n;
        for (int i = q + 1 + t; i < n; i += kPanelThreads) {  // one row per thread
            const double l = A[(size_t)i * n + q] / aqq;
            lq[i] = l;
            const double prod = l * zq;
            z[i] = z[i] - prod;
            for (int k = q + 1; k < j0 + nb; k++) {  // panel columns right of q
                const double pk = l * A[(size_t)q * n + k];
                double* const p = A + (size_t)i * n + k;
                *p = *p - pk;
            }
        }
        __syncthreads();
    }
    __syncthreads();
    // the panel's U rows on the trailing columns: row j0 + r takes steps j0 .. j0 + r - 1
    for (int k = j0 + nb + t; k < n; k += kPanelThreads) {
        double u[kPanel];
#pragma unroll
        for (int r = 0; r < kPanel; r++) {
            if (r >= nb) break;
            double v = A[(size_t)(j0 + r) * n + k];
#pragma unroll
            for (int q = 0; q < r; q++) {
                if (sk[q] != 0.0) continue;
                const double prod = Lp[(size_t)q * n + j0 + r] * u[q];
                v = v - prod;
            }
            u[r] = v;
            if (r > 0) A[(size_t)(j0 + r) * n + k] = v;
        }
    }
}

// k_lu_panel with the panel rows j0 .. n - 1 and z[j0 .. n - 1] held in LDS
// (dynamic, (n - j0) x (nb + 2) doubles: rows padded to nb + 1, then z): the same operations on the same
// values, one global round trip in and out instead of several per step.
__global__ __launch_bounds__(kPanelThreads) void k_lu_panel_lds(double* __restrict__ A, int n, int j0, int nb,
                                                                double* __restrict__ Lp, double* __restrict__ sk,
                                                                int* __restrict__ flag, double* __restrict__ z,
                                                                int check) {
#pragma clang fp contract(off)
    __shared__ double sT[kPanel][kPanel];  // l of the panel's own rows (the U-row solve)
    __shared__ double sSk[kPanel];
    extern __shared__ double sP[];
    if (*flag) return;
    const int t = threadIdx.x;
    const int R = n - j0;
    const int ls = nb + 1;  // LDS row stride: odd in doubles, so a wave's rows spread over the banks
    double* const sZ = sP + (size_t)R * ls;  // z[j0 .. n - 1]
    for (int e = t; e < R * nb; e += kPanelThreads) sP[(e / nb) * ls + e % nb] = A[(size_t)(j0 + e / nb) * n + j0 + e % nb];
    for (int r = t; r < R; r += kPanelThreads) sZ[r] = z[j0 + r];
    __syncthreads();
    for (int qq = 0; qq < nb; qq++) {
        const double aqq = sP[qq * ls + qq];
        const double mq = fabs(aqq);
        bool swap = false;
        if (check && aqq == aqq)
            for (int r = qq + 1 + t; r < R; r += kPanelThreads) swap |= fabs(sP[r * ls + qq]) > mq;
        if (__syncthreads_or(swap)) {
            if (t == 0) *flag = 1;
            return;
        }
        if (t == 0) sk[qq] = sSk[qq] = (aqq == 0.0) ? 1.0 : 0.0;
        if (aqq == 0.0) continue;  // uniform
        const double zq = sZ[qq];
        double* const lq = Lp + (size_t)qq * n + j0;
        for (int r = qq + 1 + t; r < R; r += kPanelThreads) {  // one row per thread
            const double l = sP[r * ls + qq] / aqq;
            lq[r] = l;
            if (r < nb) sT[qq][r] = l;
            const double prod = l * zq;
            sZ[r] = sZ[r] - prod;
            for (int c = qq + 1; c < nb; c++) {
                const double pc = l * sP[qq * ls + c];
                sP[r * ls + c] = sP[r * ls + c] - pc;
            }
        }
        __syncthreads();
    }
    __syncthreads();
    for (int e = t; e < R * nb; e += kPanelThreads) A[(size_t)(j0 + e / nb) * n + j0 + e % nb] = sP[(e / nb) * ls + e % nb];
    for (int r = t; r < R; r += kPanelThreads) z[j0 + r] = sZ[r];
    // the panel's U rows on the trailing columns (l and skip marks from LDS,
    // the column's nb entries loaded before the triangular solve)
    for (int k = j0 + nb + t; k < n; k += kPanelThreads) {
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

// enqueue the blocked swap-free elimination; *flag != 0 afterwards when some
// column needed a row swap (A is then partly eliminated: recopy and pivot).
// work: kPanel * n + kPanel doubles (panel multipliers, skipped-step marks)
// Returns -1 with *err set when a launch failed (the HIP error is read once,
// here), 1 when !check and the panel does not fit LDS (nothing enqueued).
int enqueue_lu_fused(double* A, int n, double* work, int* flag, double* z, hipStream_t st, std::string* err,
                     bool check = true) {
    if (chk(hipMemsetAsync(flag, 0, sizeof(int), st), "memset", err)) return -1;
    double* const sk = work + (size_t)kPanel * n;
    // panel width: the widest (<= kPanel) whose n rows fit in LDS; the global-
    // memory panel kernel beyond that.  The attribute is set on every call: it is
    // per device (a process may drive several) and cheap.
    int lds_cap = kPanelLds;
    if (hipFuncSetAttribute((const void*)k_lu_panel_lds, hipFuncAttributeMaxDynamicSharedMemorySize, kPanelLds) !=
        hipSuccess) {
        (void)hipGetLastError();
        lds_cap = 64 * 1024;
    }
    int pw = kPanel;
    while (pw > 1 && (size_t)n * (pw + 2) * sizeof(double) > (size_t)lds_cap) pw--;
    // PSX_LU_GLOBAL: the global-memory panel kernel at any size (tests)
    const bool lds = (size_t)n * (pw + 2) * sizeof(double) <= (size_t)lds_cap && !std::getenv("PSX_LU_GLOBAL");
    if (!check && !lds) return 1;  // no unchecked global-memory panel: the caller eliminates per column
    if (!lds) pw = kPanel;
    for (int j0 = 0; j0 < n - 1; j0 += pw) {
        const int nb = std::min(pw, n - 1 - j0);
        const int rest = n - j0 - nb;  // trailing columns (and rows), >= 1
        if (lds)
            hipLaunchKernelGGL(k_lu_panel_lds, dim3(1), dim3(kPanelThreads), (size_t)(n - j0) * (nb + 2) * sizeof(double), st,
                               A, n, j0, nb, work, sk, flag, z, check ? 1 : 0);
        else
            hipLaunchKernelGGL(k_lu_panel, dim3(1), dim3(kPanelThreads), 0, st, A, n, j0, nb, work, sk, flag, z);
        hipLaunchKernelGGL(k_lu_trail, dim3((rest + kTrCols - 1) / kTrCols, (rest + kTrRows - 1) / kTrRows),
                           dim3(kTrCols, kTrGroups), 0, st, A, n, j0, nb, (const double*)work, (const double*)sk,
                           (const int*)flag);
    }
    return chk(hipGetLastError(), "LU launch", err);
}

}  // namespace

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
        if (chk(hipMalloc(&work, ((size_t)kPanel * n + kPanel) * sizeof(double) + sizeof(int)), "LU work", err))
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
        hipFree(work);
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

int ld_study_setup(const double* ld, const double* z, int M, hipStream_t st, double* dS, double* dy,
                   LdStudyResult* res, std::string* err) {
    std::memset(res, 0, sizeof(*res));
    const size_t nn = (size_t)M * M;
    double *dL = nullptr, *dA = nullptr, *dz = nullptr, *ddiag = nullptr, *dcol = nullptr;
    int* dswp = nullptr;
    auto cleanup = [&]() { hipFree(dL); hipFree(dA); hipFree(dz); hipFree(ddiag); hipFree(dcol); hipFree(dswp); };
    if (hipMalloc(&dL, nn * sizeof(double)) != hipSuccess || hipMalloc(&dA, nn * sizeof(double)) != hipSuccess ||
        hipMalloc(&dz, M * sizeof(double)) != hipSuccess || hipMalloc(&ddiag, M * sizeof(double)) != hipSuccess ||
        hipMalloc(&dcol, ((size_t)kPanel * M + kPanel) * sizeof(double)) != hipSuccess ||
        hipMalloc(&dswp, (std::max(M, 1) + 2) * sizeof(int)) != hipSuccess) {
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
                if (enqueue_lu_fused(dA, M, dcol, dflag, dz, st, err)) { rc = -1; break; }
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
            // elimination without pivoting: the blocked panels with the pivot check off
            // (per-column launches when the panel does not fit LDS)
            const int lrc = enqueue_lu_fused(dA, M, dcol, dflag, dz, st, err, false);
            if (lrc < 0) { rc = -1; break; }
            if (lrc > 0)
                for (int j = 0; j < M - 1; j++) {
                    const int r = M - j - 1;
                    hipLaunchKernelGGL(k_elim, dim3((r + kElimCols - 1) / kElimCols, (r + kElimRows - 1) / kElimRows),
                                       dim3(kElimCols), 0, st, dA, M, j, dz);
                }
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
    return rc;
}

// load this translation unit's device code on the current device (psx_warmup)
int warm_module_setup() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, (const void*)k_get_diag) == hipSuccess ? 0 : -1;
}

}  // namespace psx
