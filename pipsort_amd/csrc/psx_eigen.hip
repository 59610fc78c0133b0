// psx_eigen.hip — the reference's eigen route of the Model setup on the GPU
// (util.cpp:228-263 eigen_decomp, model.h:213-259), for a study whose shifted
// LD Sigma' is not positive definite (psx_setup.hip's LDL^T pivots tell).
//
//   Sigma' = Q W Q^T  (rocSOLVER dsyevd: blocked Householder tridiagonalisation
//                      + divide and conquer, reading the triangle GSL's symmv
//                      reads, util.cpp:242)
//   B  = |W|^1/2 Q^T,  S' = |W|^-1/2 Q^T z          (model.h:227-251)
//
// B and S' are then PostCal's own inputs (postcal.h:118): the engine forms
// Sigma~ = B^T B and y = B^T S' from them exactly as for psx_create.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>  // types only: the libraries are opened on first use
#include <rocsolver/rocsolver.h>

#include <cmath>
#include <mutex>
#include <string>
#include <vector>

#include "psx_setup.h"
#include "psx_mem.h"

namespace psx {

namespace {

__device__ inline double wave_sum64(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// one eigenpair r per block: B(r, c) = sqrt|w_r| Q(c, r) (B column-major, as
// Armadillo stores BIG_SIGMA), S'_r = (Q(:, r) . z) / sqrt|w_r|
__global__ __launch_bounds__(64) void k_eig_lowrank(const double* __restrict__ Q, const double* __restrict__ w,
                                                    const double* __restrict__ z, int M, double* __restrict__ B,
                                                    double* __restrict__ sp) {
    const int r = blockIdx.x;
    const double so = sqrt(fabs(w[r]));
    double acc = 0.0;
    for (int c = threadIdx.x; c < M; c += 64) {
        const double q = Q[(size_t)r * M + c];
        B[(size_t)c * M + r] = so * q;
        acc = fma(q, z[c], acc);
    }
    acc = wave_sum64(acc);
    if (threadIdx.x == 0) sp[r] = acc / so;
}

// rocSOLVER (and the rocBLAS it depends on) opened on the first eigen route of
// the process, not linked: loading rocBLAS costs every process ~10 ms at start,
// and the route only runs for a study whose Sigma' is not positive definite
struct Solver {
    rocblas_status (*create)(rocblas_handle*) = nullptr;
    rocblas_status (*set_stream)(rocblas_handle, hipStream_t) = nullptr;
    rocblas_status (*destroy)(rocblas_handle) = nullptr;
    rocblas_status (*dsyevd)(rocblas_handle, const rocblas_evect, const rocblas_fill, const rocblas_int, double*,
                             const rocblas_int, double*, double*, rocblas_int*) = nullptr;
    bool ok = false;
};

const Solver& solver() {
    static Solver S;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librocsolver.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librocsolver.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        S.create = reinterpret_cast<decltype(S.create)>(dlsym(h, "rocblas_create_handle"));
        S.set_stream = reinterpret_cast<decltype(S.set_stream)>(dlsym(h, "rocblas_set_stream"));
        S.destroy = reinterpret_cast<decltype(S.destroy)>(dlsym(h, "rocblas_destroy_handle"));
        S.dsyevd = reinterpret_cast<decltype(S.dsyevd)>(dlsym(h, "rocsolver_dsyevd"));
        S.ok = S.create && S.set_stream && S.destroy && S.dsyevd;
    });
    return S;
}

}  // namespace

int eigen_lowrank_device(const double* sig, const double* z, int M, hipStream_t st, double* dQ, double* dB,
                         double* dsp, double* spsq, std::string* err) {
    auto bad = [&](const std::string& m) {
        *err = m;
        return -1;
    };
    const Solver& L = solver();
    if (!L.ok) return bad("rocSOLVER not found (librocsolver.so.0)");
    double* dw = nullptr;
    double* dz = nullptr;
    rocblas_int* dinfo = nullptr;
    rocblas_handle h = nullptr;
    auto done = [&]() {
        if (h) L.destroy(h);
        psx::dfree(dw);
        psx::dfree(dz);
        psx::dfree(dinfo);
    };
    if (psx::dmalloc(&dw, 2 * (size_t)M * sizeof(double)) != hipSuccess ||
        psx::dmalloc(&dz, (size_t)M * sizeof(double)) != hipSuccess || psx::dmalloc(&dinfo, sizeof(rocblas_int)) != hipSuccess) {
        done();
        return bad("out of device memory (eigen route)");
    }
    // Sigma' row-major: its lower triangle (what gsl_eigen_symmv reads) is the
    // upper triangle of the same buffer read column-major
    if (hipMemcpyAsync(dQ, sig, (size_t)M * M * sizeof(double), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(dz, z, (size_t)M * sizeof(double), hipMemcpyHostToDevice, st) != hipSuccess) {
        done();
        return bad("eigen route upload");
    }
    if (L.create(&h) != rocblas_status_success || L.set_stream(h, st) != rocblas_status_success) {
        done();
        return bad("rocblas handle");
    }
    if (L.dsyevd(h, rocblas_evect_original, rocblas_fill_upper, M, dQ, M, dw, dw + M, dinfo) !=
        rocblas_status_success) {
        done();
        return bad("rocsolver_dsyevd");
    }
    hipLaunchKernelGGL(k_eig_lowrank, dim3(M), dim3(64), 0, st, dQ, dw, dz, M, dB, dsp);
    rocblas_int info = 0;
    std::vector<double> sp(M);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(&info, dinfo, sizeof(info), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(sp.data(), dsp, (size_t)M * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {
        done();
        return bad("eigen route kernels");
    }
    done();
    if (info != 0) return bad("dsyevd did not converge (info " + std::to_string(info) + ")");
    double s = 0.0;
    for (int i = 0; i < M; i++) s += sp[i] * sp[i];  // model.h:249-251 then ||S'||^2
    *spsq = s;
    return 0;
}

}  // namespace psx
