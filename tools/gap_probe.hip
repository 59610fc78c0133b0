// Gap between back-to-back kernels on one stream (diagnostics): the same
// busy-loop kernel launched 20 times with start / stop events in its dispatch,
// for a few grid / LDS shapes; prints the mean kernel time and the mean gap
// (next start - previous stop).  hipcc --offload-arch=gfx950 -O3 gap_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>

template <int LDS>
__global__ __launch_bounds__(64) void k_busy(double* out, int iters, double* rec) {
    __shared__ double sh[LDS / 8 > 0 ? LDS / 8 : 1];
    double x = threadIdx.x * 1e-3 + blockIdx.x;
    for (int i = 0; i < iters; i++) x = fma(x, 0.999999, 1e-7);
    if (LDS > 8) { sh[threadIdx.x % (LDS / 8)] = x; __syncthreads(); x += sh[(threadIdx.x + 1) % (LDS / 8)]; }
    if (x == 12345.0) out[blockIdx.x] = x;
    if (rec) {  // 128 records of 56 B per block at its end, like a sweep unit
        double* r = rec + (size_t)blockIdx.x * 128 * 7;
        for (int q = 0; q < 14; q++) r[q * 64 + threadIdx.x] = x + q;
    }
}

// follower: a short one-wave-block kernel on a second (high-priority) stream
// after each big kernel's stop event, like the record merge of a pass
__global__ __launch_bounds__(64) void k_follow(double* out) {
    double x = threadIdx.x;
    for (int i = 0; i < 200; i++) x = fma(x, 0.999, 1e-3);
    if (x == 12345.0) out[blockIdx.x] = x;
}

template <int LDS>
void probe(const char* name, int grid, int iters, double* out, bool follow = false, double* rec = nullptr) {
    const int n = 20;
    hipEvent_t ev[2 * n];
    for (auto& e : ev) hipEventCreate(&e);
    hipStream_t S, X;
    int lo = 0, hi = 0;
    hipDeviceGetStreamPriorityRange(&lo, &hi);
    hipStreamCreateWithPriority(&S, hipStreamNonBlocking, (lo + hi) / 2);
    hipStreamCreateWithPriority(&X, hipStreamNonBlocking, hi);
    for (int w = 0; w < 3; w++) hipLaunchKernelGGL(k_busy<LDS>, dim3(grid), dim3(64), 0, S, out, iters, rec);
    hipDeviceSynchronize();
    for (int i = 0; i < n; i++) {
        hipExtLaunchKernelGGL(k_busy<LDS>, dim3(grid), dim3(64), 0, S, ev[2 * i], ev[2 * i + 1], 0, out, iters, rec);
        if (follow) {
            hipStreamWaitEvent(X, ev[2 * i + 1], 0);
            hipLaunchKernelGGL(k_follow, dim3(1001), dim3(64), 0, X, out);
        }
    }
    hipDeviceSynchronize();
    hipStreamDestroy(S);
    hipStreamDestroy(X);
    double kt = 0, gap = 0;
    for (int i = 0; i < n; i++) {
        float ms;
        hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]);
        kt += ms;
        if (i) {
            hipEventElapsedTime(&ms, ev[2 * i - 1], ev[2 * i]);
            gap += ms;
        }
    }
    printf("%-30s grid %6d: kernel %.3f ms, gap %.1f us\n", name, grid, kt / n, gap / (n - 1) * 1e3);
    for (auto& e : ev) hipEventDestroy(e);
}

int main() {
    double* out;
    hipMalloc(&out, sizeof(double) * 100000);
    probe<8>("no LDS, short", 2048, 2000, out);
    probe<8>("no LDS, 8k blocks", 8192, 20000, out);
    probe<20480>("20 KB LDS, 8k blocks", 8192, 20000, out);
    probe<20480>("20 KB LDS, 12k blocks", 12330, 40000, out);
    probe<20480>("20 KB LDS, 8k + follower", 8192, 20000, out, true);
    probe<20480>("20 KB LDS, 12k + follower", 12330, 40000, out, true);
    double* rec;
    hipMalloc(&rec, sizeof(double) * 12330 * 128 * 7);
    probe<20480>("8k, 7 KB of records per block", 8192, 20000, out, true, rec);
    probe<20480>("12k, 7 KB of records per block", 12330, 40000, out, true, rec);
    hipFree(rec);
    hipFree(out);
    return 0;
}
