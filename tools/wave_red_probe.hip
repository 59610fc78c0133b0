// wave_red_probe.hip — checks the transposed wave reductions of psx_wave.h
// (v_permlane32_swap / v_permlane16_swap + row DPP) against host sums / maxima
// on one wave, before the k = 3 kernel relies on them (developer tool).
//   hipcc -O3 --offload-arch=gfx950 -I pipsort_amd/csrc tools/wave_red_probe.hip -o tools/wave_red_probe.bin
// Exit status 0 when every case matches (integer-valued doubles: exact sums).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "psx_wave.h"

template <int K>
__global__ void k_sum(const double* in, double* out_t, double* out_k) {
    const int t = threadIdx.x;
    double v[K], w[K];
#pragma unroll
    for (int k = 0; k < K; k++) v[k] = w[k] = in[k * 64 + t];
    psx::wave_sum_t(v);
    psx::wave_sum_k(w);
    if (t == 0)
        for (int k = 0; k < K; k++) {
            out_t[k] = v[k];
            out_k[k] = w[k];
        }
}

template <int K>
__global__ void k_max(const int* in, int* out) {
    const int t = threadIdx.x;
    int v[K];
#pragma unroll
    for (int k = 0; k < K; k++) v[k] = in[k * 64 + t];
    psx::wave_max_t(v);
    if (t == 5)  // a uniform: any lane
        for (int k = 0; k < K; k++) out[k] = v[k];
}

template <int K>
int check_sum(std::mt19937& g) {
    std::vector<double> h(K * 64);
    std::uniform_int_distribution<int> d(-1000000, 1000000);
    for (auto& x : h) x = (double)d(g) * 0.25;  // exact in any order
    double *din, *dt, *dk;
    hipMalloc(&din, h.size() * 8);
    hipMalloc(&dt, K * 8);
    hipMalloc(&dk, K * 8);
    hipMemcpy(din, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_sum<K>, dim3(1), dim3(64), 0, 0, din, dt, dk);
    std::vector<double> rt(K), rk(K);
    hipMemcpy(rt.data(), dt, K * 8, hipMemcpyDeviceToHost);
    hipMemcpy(rk.data(), dk, K * 8, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int k = 0; k < K; k++) {
        double s = 0;
        for (int t = 0; t < 64; t++) s += h[k * 64 + t];
        if (rt[k] != s || rk[k] != s) {
            if (bad < 4) printf("sum K=%d value %d: transposed %.17g dpp %.17g host %.17g\n", K, k, rt[k], rk[k], s);
            bad++;
        }
    }
    hipFree(din);
    hipFree(dt);
    hipFree(dk);
    return bad;
}

template <int K>
int check_max(std::mt19937& g) {
    std::vector<int> h(K * 64);
    std::uniform_int_distribution<int> d(-5000, 5000);
    for (auto& x : h) x = d(g);
    for (int t = 0; t < 64; t++) h[0 * 64 + t] = psx::EMPTY;  // an all-empty value
    int *din, *dout;
    hipMalloc(&din, h.size() * 4);
    hipMalloc(&dout, K * 4);
    hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_max<K>, dim3(1), dim3(64), 0, 0, din, dout);
    std::vector<int> r(K);
    hipMemcpy(r.data(), dout, K * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int k = 0; k < K; k++) {
        int m = h[k * 64];
        for (int t = 1; t < 64; t++) m = std::max(m, h[k * 64 + t]);
        if (r[k] != m) {
            if (bad < 4) printf("max K=%d value %d: %d host %d\n", K, k, r[k], m);
            bad++;
        }
    }
    hipFree(din);
    hipFree(dout);
    return bad;
}

int main() {
    std::mt19937 g(7);
    int bad = 0;
    for (int rep = 0; rep < 20; rep++) {
        bad += check_sum<4>(g) + check_sum<8>(g) + check_sum<12>(g) + check_sum<16>(g);
        bad += check_max<4>(g) + check_max<8>(g);
    }
    printf("wave_red_probe: %s (%d mismatches)\n", bad ? "FAIL" : "ok", bad);
    return bad ? 1 : 0;
}
