// Accuracy of v_rsq_f64 (+0/1/2 Newton steps) and of the table exp2 on gfx950.
//   hipcc -O3 --offload-arch=gfx950 tools/rsq_acc.hip -o /tmp/rsq_acc && /tmp/rsq_acc
// Reports the max relative error against long-double references computed on
// the host; used to size the Newton count in psx_sweep.hip.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

__global__ void k_rsq(const double* x, double* r0, double* r1, double* r2, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double v = x[i];
    double y = __builtin_amdgcn_rsq(v);
    r0[i] = y;
    double e = fma(-v * y, y, 1.0);
    y = fma(0.5 * y, e, y);
    r1[i] = y;
    e = fma(-v * y, y, 1.0);
    r2[i] = fma(0.5 * y, e, y);
}

int main() {
    const int n = 1 << 22;
    std::mt19937_64 g(1);
    std::uniform_real_distribution<double> u(-40.0, 40.0);
    std::vector<double> x(n);
    for (auto& v : x) v = std::exp2(u(g));
    double *dx, *d0, *d1, *d2;
    hipMalloc(&dx, n * 8);
    hipMalloc(&d0, n * 8);
    hipMalloc(&d1, n * 8);
    hipMalloc(&d2, n * 8);
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_rsq, dim3(n / 256), dim3(256), 0, 0, dx, d0, d1, d2, n);
    std::vector<double> r[3];
    double* dd[3] = {d0, d1, d2};
    for (int k = 0; k < 3; k++) {
        r[k].resize(n);
        hipMemcpy(r[k].data(), dd[k], n * 8, hipMemcpyDeviceToHost);
    }
    for (int k = 0; k < 3; k++) {
        long double mx = 0;
        for (int i = 0; i < n; i++) {
            long double ref = 1.0L / sqrtl((long double)x[i]);
            long double e = fabsl((long double)r[k][i] - ref) / ref;
            if (e > mx) mx = e;
        }
        printf("rsq newton=%d max_rel_err=%.3Le (%.2f ulp)\n", k, mx, (double)(mx / 1.1102230246251565e-16L));
    }
    return 0;
}
