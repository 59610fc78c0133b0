// psx_setup.h — GPU Model setup (model.h:171-264, util.cpp:195-263); see psx_setup.hip.
#ifndef PSX_SETUP_H
#define PSX_SETUP_H

#include <hip/hip_runtime.h>

#include <string>

namespace psx {

struct LdStudyResult {
    double added;             // diagonal shift of util.cpp:195-226
    int psd_iterations;       // LU determinants evaluated
    int path;                 // 0: Sigma' positive definite (identity route), 1: eigen route needed
    int sigma_host_needed;    // path 1: the caller rebuilds Sigma' = LD + added I on the host
    double min_pivot_ratio;   // min L D L^T pivot / max |diag|
    double spsq;              // path 0: ||S'_s||^2 = z^T Sigma'^-1 z
    int fused_route;          // 1: swap-free LU of a symmetric LD carried step 2 (one elimination)
    double upload_ms, psd_ms, finish_ms;  // wall time of the phases (LD upload, PSD loop, step 2 + readback)
};

// Partial-pivot LU determinant of the device matrix dA (n x n row-major,
// destroyed), bit-identical to the host restatement (model.cpp lu_det).
// dswp: n ints, ddiag: n doubles of device scratch.
int lu_det_device(double* dA, int n, int* dswp, double* ddiag, hipStream_t st, double* det, std::string* err);

// The setup's swap-free elimination (k_lu_diag + k_lu_tile) of the host matrix
// a (n x n row-major) with z's forward solve (z may be null): pivots U_ii ->
// piv, z~ -> zt (when z), *swap = 1 when check and some column needed a row
// swap (piv / zt are then meaningless).  For parity tests (psx_elim_gpu).
int elim_device(const double* a, int n, const double* z, int check, double* piv, double* zt, int* swap,
                std::string* err);

// One study: LD (host, row-major M x M as parsed, util.cpp:86-96) and z (host,
// M) -> dS = Sigma~_s (device, row-major M x M) and dy = y_s (device, M).
int ld_study_setup(const double* ld, const double* z, int M, hipStream_t st, double* dS, double* dy,
                   LdStudyResult* res, std::string* err);

// The reference's eigen route for a study whose Sigma' is not positive
// definite (util.cpp:228-263, model.h:213-259), on the GPU (psx_eigen.hip): sig
// (host, row-major M x M, Sigma' = LD + shift I) and z (host) -> dB = B =
// |W|^1/2 Q^T (device, column-major) and dsp = S' = |W|^-1/2 Q^T z (device),
// *spsq = ||S'||^2.  dQ: M x M device scratch.
int eigen_lowrank_device(const double* sig, const double* z, int M, hipStream_t st, double* dQ, double* dB,
                         double* dsp, double* spsq, std::string* err);

// this translation unit's device code, loaded ahead of first use (psx_warmup)
int warm_module_setup();

}  // namespace psx

#endif
