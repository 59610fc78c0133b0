// valu_lat.hip — gfx950 FP64 VALU issue/latency probe (developer tool).
// One workgroup of W waves on one CU (W <= 4 waves land on different SIMDs, so
// launch 4*k waves to put k waves per SIMD); each wave runs CH independent
// dependent-chains of N ops; prints cycles per wave-instruction of wave 0 (the
// oldest wave has issue priority, so with 2 waves per SIMD it still shows the
// single-wave latency).  Measured on MI355X (r01y): dependent v_fma_f64 5.75
// cycles, v_add_f64 7.5, v_rsq_f64 ~18; independent FP64 ops 4.3 (the wave64
// issue rate of a 16-lane SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CH, int OP>
__global__ void k_chain(double* out, long long* cyc, int n, double y, double z) {
    double x[CH];
    const int e = (int)(threadIdx.x & 1) - 1;
#pragma unroll
    for (int c = 0; c < CH; c++) x[c] = threadIdx.x * 1e-3 + c;
    __syncthreads();
    const long long t0 = wall_clock64();
    const long long c0 = clock64();
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int r = 0; r < 16; r++) {
#pragma unroll
            for (int c = 0; c < CH; c++) {
                if (OP == 0) x[c] = fma(x[c], y, z);
                else if (OP == 1) x[c] = x[c] + z;
                else if (OP == 2) asm volatile("v_ldexp_f64 %0, %1, %2" : "=v"(x[c]) : "v"(x[c]), "v"(e));  // no folding
                else if (OP == 3) x[c] = __builtin_amdgcn_rsq(x[c]);
            }
        }
    }
    const long long c1 = clock64();
    double s = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x * 16 + threadIdx.y] = c1 - c0;
    (void)t0;
}

template <int CH, int OP>
void run(const char* name, int waves_per_simd) {
    double* out; long long* cyc;
    hipMalloc(&out, 1 << 20); hipMalloc(&cyc, 1 << 12);
    const int n = 4096;
    dim3 blk(64, 4 * waves_per_simd);
    hipLaunchKernelGGL((k_chain<CH, OP>), dim3(1), blk, 0, 0, out, cyc, n, 1.0000001, 1e-9);
    hipLaunchKernelGGL((k_chain<CH, OP>), dim3(1), blk, 0, 0, out, cyc, n, 1.0000001, 1e-9);
    hipDeviceSynchronize();
    long long h[16];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double insts = (double)n * 16 * CH;
    // clock64 = s_memtime (shader clock)
    printf("%-8s chains=%d waves/SIMD=%d: %.2f cycles per wave-instruction per wave\n", name, CH, waves_per_simd,
           h[0] / insts);
    hipFree(out); hipFree(cyc);
}

int main() {
    for (int w = 1; w <= 2; w++) {
        run<1, 0>("fma", w); run<2, 0>("fma", w); run<4, 0>("fma", w); run<8, 0>("fma", w);
        run<1, 1>("add", w); run<4, 1>("add", w);
        run<1, 2>("ldexp", w); run<4, 2>("ldexp", w);
        run<1, 3>("rsq", w); run<4, 3>("rsq", w);
    }
    return 0;
}
