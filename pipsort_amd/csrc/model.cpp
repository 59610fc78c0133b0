// model.cpp — host restatement of the reference Model setup (model.h:171-264,
// util.cpp:195-263).  Compiled with -ffp-contract=off: the PSD decision depends
// on the exact rounding of the LU elimination (hard parts).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/pipsort_model.h"

extern "C" {

// util.cpp:195-226 with gsl_linalg_LU_decomp / gsl_linalg_LU_det (GSL 2.5):
// right-looking elimination, partial pivoting on the first maximal |a_ij|,
// det = signum * prod_i U_ii multiplied in index order.
static double lu_det(std::vector<double>& a, int n) {
    int signum = 1;
    for (int j = 0; j < n - 1; j++) {
        double mx = std::fabs(a[(size_t)j * n + j]);
        int ip = j;
        for (int i = j + 1; i < n; i++) {
            double v = std::fabs(a[(size_t)i * n + j]);
            if (v > mx) { mx = v; ip = i; }
        }
        if (ip != j) {
            std::swap_ranges(a.begin() + (size_t)j * n, a.begin() + (size_t)j * n + n, a.begin() + (size_t)ip * n);
            signum = -signum;
        }
        const double ajj = a[(size_t)j * n + j];
        if (ajj != 0.0) {
            const double* rj = &a[(size_t)j * n];
#pragma omp parallel for schedule(static) if (n - j > 256)
            for (int i = j + 1; i < n; i++) {
                double* ri = &a[(size_t)i * n];
                const double aij = ri[j] / ajj;
                ri[j] = aij;
                for (int k = j + 1; k < n; k++) ri[k] = ri[k] - aij * rj[k];
            }
        }
    }
    double det = signum;
    for (int i = 0; i < n; i++) det *= a[(size_t)i * n + i];
    return det;
}

int psx_lu_det(const double* a, int32_t m, double* det) {
    if (m <= 0 || !det) return -1;
    std::vector<double> t(a, a + (size_t)m * m);
    *det = lu_det(t, m);
    return 0;
}

int psx_psd_shift(double* sigma, int32_t m, double* added) {
    if (m <= 0) return -1;
    double add = 0;
    std::vector<double> t((size_t)m * m);
    for (int guard = 0; guard < 1000000; guard++) {
        std::memcpy(t.data(), sigma, sizeof(double) * (size_t)m * m);
        for (int i = 0; i < m; i++) t[(size_t)i * m + i] = sigma[(size_t)i * m + i] + add;
        if (lu_det(t, m) > 0) break;
        add += 0.01;
    }
    for (int i = 0; i < m; i++) sigma[(size_t)i * m + i] += add;
    if (added) *added = add;
    return 0;
}

// Householder reduction of a symmetric matrix to tridiagonal form with the
// transformations accumulated, then implicit QL with Wilkinson-style shifts
// (the classical EISPACK tred2/tql2 pair).  V is row-major n x n; on exit
// column j of V is the eigenvector of d[j].
static void tred2(int n, std::vector<double>& V, std::vector<double>& d, std::vector<double>& e) {
    for (int j = 0; j < n; j++) d[j] = V[(size_t)(n - 1) * n + j];
    for (int i = n - 1; i > 0; i--) {
        double scale = 0.0, h = 0.0;
        for (int k = 0; k < i; k++) scale += std::fabs(d[k]);
        if (scale == 0.0) {
            e[i] = d[i - 1];
            for (int j = 0; j < i; j++) {
                d[j] = V[(size_t)(i - 1) * n + j];
                V[(size_t)i * n + j] = 0.0;
                V[(size_t)j * n + i] = 0.0;
            }
        } else {
            for (int k = 0; k < i; k++) {
                d[k] /= scale;
                h += d[k] * d[k];
            }
            double f = d[i - 1];
            double g = std::sqrt(h);
            if (f > 0) g = -g;
            e[i] = scale * g;
            h = h - f * g;
            d[i - 1] = f - g;
            for (int j = 0; j < i; j++) e[j] = 0.0;
            for (int j = 0; j < i; j++) {
                f = d[j];
                V[(size_t)j * n + i] = f;
                g = e[j] + V[(size_t)j * n + j] * f;
                for (int k = j + 1; k <= i - 1; k++) {
                    g += V[(size_t)k * n + j] * d[k];
                    e[k] += V[(size_t)k * n + j] * f;
                }
                e[j] = g;
            }
            f = 0.0;
            for (int j = 0; j < i; j++) {
                e[j] /= h;
                f += e[j] * d[j];
            }
            double hh = f / (h + h);
            for (int j = 0; j < i; j++) e[j] -= hh * d[j];
#pragma omp parallel for schedule(static) if (i > 256)
            for (int j = 0; j < i; j++) {
                double fj = d[j], gj = e[j];
                for (int k = j; k <= i - 1; k++) V[(size_t)k * n + j] -= (fj * e[k] + gj * d[k]);
            }
            for (int j = 0; j < i; j++) {
                d[j] = V[(size_t)(i - 1) * n + j];
                V[(size_t)i * n + j] = 0.0;
            }
        }
        d[i] = h;
    }
    // accumulate transformations
    for (int i = 0; i < n - 1; i++) {
        V[(size_t)(n - 1) * n + i] = V[(size_t)i * n + i];
        V[(size_t)i * n + i] = 1.0;
        double h = d[i + 1];
        if (h != 0.0) {
            for (int k = 0; k <= i; k++) d[k] = V[(size_t)k * n + i + 1] / h;
#pragma omp parallel for schedule(static) if (i > 256)
            for (int j = 0; j <= i; j++) {
                double g = 0.0;
                for (int k = 0; k <= i; k++) g += V[(size_t)k * n + i + 1] * V[(size_t)k * n + j];
                for (int k = 0; k <= i; k++) V[(size_t)k * n + j] -= g * d[k];
            }
        }
        for (int k = 0; k <= i; k++) V[(size_t)k * n + i + 1] = 0.0;
    }
    for (int j = 0; j < n; j++) {
        d[j] = V[(size_t)(n - 1) * n + j];
        V[(size_t)(n - 1) * n + j] = 0.0;
    }
    V[(size_t)(n - 1) * n + n - 1] = 1.0;
    e[0] = 0.0;
}

static void tql2(int n, std::vector<double>& V, std::vector<double>& d, std::vector<double>& e) {
    for (int i = 1; i < n; i++) e[i - 1] = e[i];
    e[n - 1] = 0.0;
    double f = 0.0, tst1 = 0.0;
    const double eps = std::ldexp(1.0, -52);
    for (int l = 0; l < n; l++) {
        tst1 = std::max(tst1, std::fabs(d[l]) + std::fabs(e[l]));
        int m = l;
        while (m < n) {
            if (std::fabs(e[m]) <= eps * tst1) break;
            m++;
        }
        if (m > l) {
            int iter = 0;
            do {
                iter++;
                double g = d[l];
                double p = (d[l + 1] - g) / (2.0 * e[l]);
                double r = std::hypot(p, 1.0);
                if (p < 0) r = -r;
                d[l] = e[l] / (p + r);
                d[l + 1] = e[l] * (p + r);
                double dl1 = d[l + 1];
                double h = g - d[l];
                for (int i = l + 2; i < n; i++) d[i] -= h;
                f += h;
                p = d[m];
                double c = 1.0, c2 = c, c3 = c;
                double el1 = e[l + 1];
                double s = 0.0, s2 = 0.0;
                for (int i = m - 1; i >= l; i--) {
                    c3 = c2;
                    c2 = c;
                    s2 = s;
                    g = c * e[i];
                    h = c * p;
                    r = std::hypot(p, e[i]);
                    e[i + 1] = s * r;
                    s = e[i] / r;
                    c = p / r;
                    p = c * d[i] - s * g;
                    d[i + 1] = h + s * (c * g + s * d[i]);
                    for (int k = 0; k < n; k++) {
                        h = V[(size_t)k * n + i + 1];
                        V[(size_t)k * n + i + 1] = s * V[(size_t)k * n + i] + c * h;
                        V[(size_t)k * n + i] = c * V[(size_t)k * n + i] - s * h;
                    }
                }
                p = -s * s2 * c3 * el1 * e[l] / dl1;
                e[l] = s * p;
                d[l] = c * p;
            } while (std::fabs(e[l]) > eps * tst1 && iter < 300);
        }
        d[l] = d[l] + f;
        e[l] = 0.0;
    }
}

int psx_sym_eigen(const double* a, int32_t m, double* w, double* q) {
    if (m <= 0) return -1;
    std::vector<double> V(a, a + (size_t)m * m), d(m), e(m);
    if (m == 1) {
        w[0] = a[0];
        q[0] = 1.0;
        return 0;
    }
    tred2(m, V, d, e);
    tql2(m, V, d, e);
    std::copy(d.begin(), d.end(), w);
    std::copy(V.begin(), V.end(), q);
    return 0;
}

int psx_lowrank_study(const double* sigma, const double* z, int32_t m, double* B_out, double* sprime_out) {
    std::vector<double> w(m), q((size_t)m * m);
    if (psx_sym_eigen(sigma, m, w.data(), q.data())) return -1;
    // model.h:227 |Omega|; model.h:232 B = sqrt(Omega) Q^T; model.h:249-251 S' = inv(sqrt(Omega)) Q^T z
    for (int r = 0; r < m; r++) {
        const double so = std::sqrt(std::fabs(w[r]));
        double acc = 0.0;
        for (int c = 0; c < m; c++) {
            const double qcr = q[(size_t)c * m + r];
            B_out[(size_t)c * m + r] = so * qcr;  // column-major B(r, c) = so * Q(c, r)
            acc += qcr * z[c];
        }
        sprime_out[r] = acc / so;
    }
    return 0;
}

}  // extern "C"
