// psx_setup.h — GPU Model setup (model.h:171-264, util.cpp:195-263); see psx_setup.hip.
#ifndef PSX_SETUP_H
#define PSX_SETUP_H

#include <hip/hip_runtime.h>

#include <condition_variable>
#include <mutex>
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

// The two studies' first PSD-shift elimination in joint launches (late r06): each
// study's thread arrives in ld_study_setup with its shifted copy and z staged
// on its stream; study 0's thread then enqueues both matrices' panels, one
// k_lu_step per panel index, on its stream, and study 1's stream waits for
// them.  The two studies' separate panel launches contended for the CUs (a
// panel every 18-21 us per study instead of 16 alone, profiles/r06/r06late_a_*).  A study
// that arrives without a matrix (an early failure; the caller's guard calls
// leave() when the study's setup returns) leaves the other to its own
// launches.  Later shift iterations and the pivoting path stay per study.
struct LuJoin {
    std::mutex m;
    std::condition_variable cv;
    bool in[2] = {false, false};   // arrived (with or without a matrix)
    bool mat[2] = {false, false};  // arrived with a matrix
    double* A[2] = {nullptr, nullptr};
    double* z[2] = {nullptr, nullptr};
    double* work[2] = {nullptr, nullptr};
    int* flag[2] = {nullptr, nullptr};
    int n[2] = {0, 0};
    hipStream_t st[2] = {nullptr, nullptr};
    hipEvent_t ready = nullptr;  // study 1's matrix staged on its stream
    hipEvent_t done = nullptr;   // the joint panels, on study 0's stream
    int state = 0;               // 0: pending, 1: enqueued, 2: the enqueue failed
    std::string err;
    void leave(int s);
    ~LuJoin();
};

// One study: LD (host, row-major M x M as parsed, util.cpp:86-96) and z (host,
// M) -> dS = Sigma~_s (device, row-major M x M) and dy = y_s (device, M).
// join / s: the first elimination joint with the other study (see LuJoin).
int ld_study_setup(const double* ld, const double* z, int M, hipStream_t st, double* dS, double* dy,
                   LdStudyResult* res, std::string* err, LuJoin* join = nullptr, int s = 0);

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
