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
//  * Step 1 runs here as an unblocked right-looking elimination, one pivot
//    launch + one update launch per column, with the reference's operation
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
// The elimination kernels are HBM/L2 streaming kernels (one read-modify-write
// of the trailing matrix per column, 2/3 M^3 * 16 B over a setup); the matrix
// (32 MB at M = 2000) stays L2/MALL resident.  Launch latency dominates below
// a few hundred trailing rows.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
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

// Fused step j of the partial-pivot elimination for matrices that need no row
// swap (LD matrices: the diagonal stays the column maximum).  Column j sits
// contiguous in col[j & 1] (written by step j - 1's owners of column j), so
// every block reduces it to GSL's pivot (first row of maximal |a_ij|, NaNs never
// chosen; the same decision k_lu_pivot makes).  If that pivot is row j the
// block eliminates exactly as k_elim (same operations, same rounding) and the
// owners of column j + 1 publish its new entries to col[(j + 1) & 1]; else the
// step raises *flag and this and every later step do nothing (the caller then
// reruns the pivoting path from a fresh copy).  One launch per column instead
// of a pivot launch plus an update launch.
__global__ __launch_bounds__(kElimCols) void k_lu_step(double* __restrict__ A, int n, int j,
                                                       double* __restrict__ col, int* __restrict__ flag,
                                                       double* __restrict__ z) {
#pragma clang fp contract(off)
    __shared__ double sv[kElimCols];
    __shared__ int si[kElimCols];
    __shared__ double sl[kElimRows];
    if (*flag) return;
    const int t = threadIdx.x;
    const double* cj = col + (size_t)(j & 1) * n;
    double mx = -1.0;
    int ip = n;
    for (int i = j + t; i < n; i += kElimCols) {
        const double v = fabs(cj[i]);
        if (v > mx) { mx = v; ip = i; }
    }
    sv[t] = mx;
    si[t] = ip;
    __syncthreads();
    for (int w = kElimCols / 2; w > 0; w >>= 1) {
        if (t < w) {
            const double v2 = sv[t + w];
            const int i2 = si[t + w];
            if (v2 > sv[t] || (v2 == sv[t] && i2 < si[t])) { sv[t] = v2; si[t] = i2; }
        }
        __syncthreads();
    }
    const double ajj = cj[j];
    const int p = (ajj != ajj || si[0] >= n) ? j : si[0];
    if (p != j) {
        if (t == 0) *flag = 1;
        return;
    }
    const int i0 = j + 1 + blockIdx.y * kElimRows;
    const int nr = min(kElimRows, n - i0);
    const int k = j + 1 + blockIdx.x * kElimCols + t;
    double* cn = col + (size_t)((j + 1) & 1) * n;
    if (ajj == 0.0) {  // GSL skips the column: column j + 1 is published unchanged
        if (k == j + 1)
            for (int r = 0; r < nr; r++) cn[i0 + r] = A[(size_t)(i0 + r) * n + k];
        return;
    }
    if (t < nr) sl[t] = A[(size_t)(i0 + t) * n + j] / ajj;
    __syncthreads();
    if (z && blockIdx.x == 0 && t < nr) {
        const double zj = z[j];
        z[i0 + t] = z[i0 + t] - sl[t] * zj;
    }
    if (k >= n) return;
    const double ujk = A[(size_t)j * n + k];
    for (int r = 0; r < nr; r++) {
        double* q = A + (size_t)(i0 + r) * n + k;
        const double prod = sl[r] * ujk;
        const double v = *q - prod;
        *q = v;
        if (k == j + 1) cn[i0 + r] = v;
    }
}

// *asym = 1 when L is not exactly symmetric (any L_ik != L_ki, NaNs included)
__global__ void k_sym_check(const double* __restrict__ L, int n, int* __restrict__ asym) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)n * n) return;
    const int i = (int)(idx / n), k = (int)(idx % n);
    if (k > i && !(L[idx] == L[(size_t)k * n + i])) *asym = 1;
}

// col[0][i] = A[i][0]: column 0 for the first fused step; flag re-armed
__global__ void k_lu_begin(const double* __restrict__ A, int n, double* __restrict__ col, int* __restrict__ flag) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) col[i] = A[(size_t)i * n];
    if (i == 0) *flag = 0;
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
int enqueue_lu(double* A, int n, int* dswp, hipStream_t st) {
    for (int j = 0; j < n - 1; j++) {
        hipLaunchKernelGGL(k_lu_pivot, dim3(1), dim3(1024), 0, st, A, n, j, dswp);
        const int r = n - j - 1;
        hipLaunchKernelGGL(k_elim, dim3((r + kElimCols - 1) / kElimCols, (r + kElimRows - 1) / kElimRows),
                           dim3(kElimCols), 0, st, A, n, j, (double*)nullptr);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// enqueue the fused (swap-free) elimination; *flag != 0 afterwards when some
// column needed a row swap (A is then partly eliminated: recopy and pivot)
int enqueue_lu_fused(double* A, int n, double* col, int* flag, double* z, hipStream_t st) {
    hipLaunchKernelGGL(k_lu_begin, dim3((n + 255) / 256), dim3(256), 0, st, A, n, col, flag);
    for (int j = 0; j < n - 1; j++) {
        const int r = n - j - 1;
        hipLaunchKernelGGL(k_lu_step, dim3((r + kElimCols - 1) / kElimCols, (r + kElimRows - 1) / kElimRows),
                           dim3(kElimCols), 0, st, A, n, j, col, flag, z);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace

int lu_det_device(double* dA, int n, int* dswp, double* ddiag, hipStream_t st, double* det, std::string* err) {
    if (n <= 0) return -1;
    if (enqueue_lu(dA, n, dswp, st)) return chk(hipGetLastError(), "LU launch", err);
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
        hipMalloc(&dcol, 2 * (size_t)M * sizeof(double)) != hipSuccess ||
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
                if (enqueue_lu_fused(dA, M, dcol, dflag, dz, st)) { rc = chk(hipGetLastError(), "LU launch", err); break; }
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

}  // namespace psx
