// Cold-start split of a one-locus process (tests/example wall):
// hsa_init alone, then the HIP runtime (hipGetDeviceCount), context
// (hipFree(0)), first launch.  Prints one JSON line, with the monotonic clock
// at _exit (end_ms: the parent times the exit, tools/exit_probe.py).  Optional
// argv[2] / argv[3]: MiB of device / pinned host memory held at exit; argv[4]:
// streams created (hipStreamCreate, one launch each) and held at exit.
// Developer tool:
//   hipcc --offload-arch=gfx950 -O2 -o tools/init_probe tools/init_probe.cpp -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <unistd.h>

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__global__ void k_noop(int* p) {
    if (p && threadIdx.x == 0) p[0] = 1;
}

int main(int argc, char** argv) {
    const bool hsa_first = argc > 1 && atoi(argv[1]) == 1;
    const double t0 = now_ms();
    if (hsa_first) hsa_init();
    const double t1 = now_ms();
    int n = 0;
    (void)hipGetDeviceCount(&n);
    const double t2 = now_ms();
    (void)hipSetDevice(0);
    (void)hipFree(nullptr);
    const double t3 = now_ms();
    int* d = nullptr;
    (void)hipMalloc(&d, 256);
    const double t4 = now_ms();
    hipLaunchKernelGGL(k_noop, dim3(1), dim3(64), 0, nullptr, d);
    (void)hipDeviceSynchronize();
    const double t5 = now_ms();
    const size_t dmb = argc > 2 ? (size_t)atol(argv[2]) : 0, hmb = argc > 3 ? (size_t)atol(argv[3]) : 0;
    void *big = nullptr, *pin = nullptr;
    if (dmb) (void)hipMalloc(&big, dmb << 20);
    if (hmb) (void)hipHostMalloc(&pin, hmb << 20);
    const int nst = argc > 4 ? atoi(argv[4]) : 0;
    for (int i = 0; i < nst; i++) {
        hipStream_t st;
        (void)hipStreamCreate(&st);
        hipLaunchKernelGGL(k_noop, dim3(1), dim3(64), 0, st, d);
        (void)hipStreamSynchronize(st);
    }
    const double t6 = now_ms();
    printf("{\"hsa_init_ms\": %.2f, \"hip_device_count_ms\": %.2f, \"context_ms\": %.2f, \"malloc_ms\": %.2f, "
           "\"first_launch_ms\": %.2f, \"held_alloc_ms\": %.2f, \"devices\": %d, \"end_ms\": %.3f}\n",
           t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5, n, now_ms());
    fflush(stdout);
    _exit(0);
}
