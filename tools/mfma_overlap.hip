// mfma_overlap.hip — does gfx950's FP64 matrix pipe issue beside FP64 VALU work
// on one SIMD?  (developer tool; VERDICT r03 "next round" 3(a))
//
// One workgroup on one CU.  Waves land round-robin on the 4 SIMDs (wave w on
// SIMD w % 4), so a block of 4 waves puts one wave on every SIMD and a block of
// 8 puts two.  Each wave runs a stream of independent chains:
//   VALU  8 chains of v_fma_f64 (inline asm, nothing folds)
//   MFMA  4 accumulators of v_mfma_f64_16x16x4_f64 (2,048 flops per instruction)
//   MIXk  per step one MFMA and k v_fma_f64 of other chains, in one wave
// and records its s_memtime span.  Cases:
//   solo VALU / solo MFMA (1 wave per SIMD), VALU+VALU and MFMA+MFMA (2 per
//   SIMD), VALU+MFMA (one of each per SIMD), and the in-wave mixes.
// If VALU+MFMA finishes in ~max(solo VALU, solo MFMA) rather than their sum,
// the pipes overlap and FP64 contractions could move to the matrix core.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double v4d __attribute__((ext_vector_type(4)));

enum Mode { VALU = 0, MFMA = 1, SPLIT = 2, MIX2 = 3, MIX4 = 4, MIX8 = 5, MIX16 = 6 };

template <int MODE>
__device__ __forceinline__ void run_stream(int role, int n, double y, double z, double& xs, v4d& as) {
    double x[8];
    v4d acc[4];
#pragma unroll
    for (int c = 0; c < 8; c++) x[c] = threadIdx.x * 1e-3 + c + 1.0;
#pragma unroll
    for (int c = 0; c < 4; c++) acc[c] = v4d{1.0 * c, 0.5, 0.25, 0.125};
    const double a = y + threadIdx.x * 1e-6, b = z + threadIdx.x * 1e-7;
    const int kv = MODE == MIX2 ? 2 : MODE == MIX4 ? 4 : MODE == MIX8 ? 8 : MODE == MIX16 ? 16 : 0;
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            if (MODE == VALU || (MODE == SPLIT && role == 0)) {
#pragma unroll
                for (int c = 0; c < 8; c++) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z));
            } else if (MODE == MFMA || (MODE == SPLIT && role == 1)) {
#pragma unroll
                for (int c = 0; c < 4; c++) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
            } else {
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
#pragma unroll
                    for (int v = 0; v < kv; v++)
                        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x[(c * kv + v) & 7]) : "v"(y), "v"(z));
                }
            }
        }
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < 8; c++) s += x[c];
    xs = s;
    as = acc[0] + acc[1] + acc[2] + acc[3];
}

template <int MODE>
__global__ void k_probe(double* out, long long* cyc, int n, double y, double z) {
    const int w = threadIdx.y;
    const int role = MODE == SPLIT ? (w >= 4 ? 1 : 0) : 0;
    double xs;
    v4d as;
    __syncthreads();
    const long long c0 = clock64();
    run_stream<MODE>(role, n, y, z, xs, as);
    const long long c1 = clock64();
    out[w * 64 + threadIdx.x] = xs + as.x + as.y + as.z + as.w;
    if (threadIdx.x == 0) cyc[w] = c1 - c0;
}

// per wave: VALU instructions and MFMA instructions it issued
static void counts(int mode, int role, int n, double& nv, double& nm) {
    const double steps = (double)n * 4;
    nv = nm = 0;
    if (mode == VALU || (mode == SPLIT && role == 0)) nv = steps * 8;
    else if (mode == MFMA || (mode == SPLIT && role == 1)) nm = steps * 4;
    else {
        const int kv = mode == MIX2 ? 2 : mode == MIX4 ? 4 : mode == MIX8 ? 8 : 16;
        nm = steps * 4;
        nv = steps * 4 * kv;
    }
}

template <int MODE>
void run(const char* name, int waves) {
    double* out;
    long long* cyc;
    hipMalloc(&out, 64 * 16 * sizeof(double));
    hipMalloc(&cyc, 16 * sizeof(long long));
    const int n = 4096;
    for (int rep = 0; rep < 3; rep++)
        hipLaunchKernelGGL(k_probe<MODE>, dim3(1), dim3(64, waves), 0, 0, out, cyc, n, 1.0000001, 1e-9);
    hipDeviceSynchronize();
    long long h[16];
    hipMemcpy(h, cyc, sizeof(long long) * waves, hipMemcpyDeviceToHost);
    printf("%-10s waves/SIMD=%d:", name, waves / 4);
    for (int w = 0; w < waves; w++) {
        double nv, nm;
        counts(MODE, MODE == SPLIT && w >= 4 ? 1 : 0, n, nv, nm);
        printf(" w%d %.0fk cyc (%s%.2f cyc/inst)", w, h[w] / 1e3, nm > 0 && nv == 0 ? "mfma " : nv > 0 && nm == 0 ? "fma " : "mix ",
               h[w] / (nv + nm));
    }
    printf("\n");
    hipFree(out);
    hipFree(cyc);
}

int main() {
    run<VALU>("valu", 4);
    run<MFMA>("mfma", 4);
    run<VALU>("valu2", 8);
    run<MFMA>("mfma2", 8);
    run<SPLIT>("valu+mfma", 8);
    run<MIX2>("mix1:2", 4);
    run<MIX4>("mix1:4", 4);
    run<MIX8>("mix1:8", 4);
    run<MIX16>("mix1:16", 4);
    run<MIX4>("mix1:4x2", 8);
    return 0;
}
