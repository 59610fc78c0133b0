/*
 * pipsort_model.h — host-side Model setup that feeds the PostCal seam.
 *
 * These restate the reference driver's per-study setup (model.h:171-264,
 * util.cpp:195-263) without GSL/Armadillo/LAPACK, so the PIPSORT executable
 * can build psx_problem from the CLI inputs.  Host C++ (OpenMP), not GPU.
 */
#ifndef PIPSORT_MODEL_H
#define PIPSORT_MODEL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* util.cpp:195-226 makeSigmaPositiveSemiDefinite: add 0.01 to the diagonal until
 * the partial-pivot LU determinant (GSL-2.5 elimination, det = sign * prod U_ii
 * in index order, strict IEEE) is > 0.  sigma is row-major m x m, updated in
 * place; *added receives the total diagonal shift. */
int psx_psd_shift(double *sigma, int32_t m, double *added);

/* The determinant psx_psd_shift tests (a row-major m x m, not modified). */
int psx_lu_det(const double *a, int32_t m, double *det);

/* model.h:213-259 with util.cpp:228-263: Sigma' = Q W Q^T, B = |W|^(1/2) Q^T
 * (column-major m x m, Armadillo layout) and S' = |W|^(-1/2) Q^T z. */
int psx_lowrank_study(const double *sigma, const double *z, int32_t m, double *B_out, double *sprime_out);

/* Symmetric eigendecomposition used above (Householder tridiagonalisation +
 * implicit QL).  a row-major m x m; w[m] eigenvalues; q row-major, column j is
 * the eigenvector of w[j]. */
int psx_sym_eigen(const double *a, int32_t m, double *w, double *q);

#ifdef __cplusplus
}
#endif
#endif
