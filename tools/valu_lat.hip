// valu_lat.hip — gfx950 VALU issue-cost / latency probe (developer tool).
//
// One workgroup of 4*W waves on one CU: waves land round-robin on the 4 SIMDs,
// so every SIMD holds W waves.  Each wave runs CH independent chains of one
// instruction (inline asm, so nothing folds); every wave's s_memtime span is
// recorded and the SIMD's issue cost is
//     cycles per wave-instruction = max span / (W * instructions per wave)
// (throughput of the SIMD, all W waves' streams together), next to the oldest
// wave's own span (its latency-bound rate when CH = 1).
//
// Mixed streams ("mix"): per chain step one FP64 FMA plus K non-FP64 ops of
// independent chains, to see whether non-FP64 work issues inside the FP64 FMA's
// 4-cycle pipe occupancy (the cost model of bench.py's roofline.valu_issue).
//
// Round-1 numbers (r01y): dependent v_fma_f64 5.75 cycles, v_add_f64 7.5,
// v_rsq_f64 ~18; independent FP64 4.3.  Round-3 table: profiles/archive/r03*_valu_issue.txt.
#include <hip/hip_runtime.h>
#include <cstdio>

enum Op {
    FMA_F64, ADD_F64, MUL_F64, LDEXP_F64, RSQ_F64, FMA_F32, MUL_F32, ADD_U32, CNDMASK, BFE_U32, LSHR_B32, AND_B32,
    MOV_B32, CVT_F64_I32, MIX1, MIX2, MIX4, NOP
};
static const char* kName[] = {"v_fma_f64", "v_add_f64", "v_mul_f64", "v_ldexp_f64", "v_rsq_f64", "v_fma_f32",
                              "v_mul_f32", "v_add_u32", "v_cndmask_b32", "v_bfe_u32", "v_lshrrev_b32", "v_and_b32",
                              "v_mov_b32", "v_cvt_f64_i32", "fma_f64+1 int", "fma_f64+2 int", "fma_f64+4 int", ""};
static const int kPerStep[] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 3, 5, 0};

template <int CH, int OP>
__global__ void k_chain(double* out, long long* cyc, int n, double y, double z) {
    double x[CH];
    float f[CH];
    int k[CH], k2[CH];
    const int e = (int)(threadIdx.x & 1) - 1;
#pragma unroll
    for (int c = 0; c < CH; c++) {
        x[c] = threadIdx.x * 1e-3 + c + 1.0;
        f[c] = (float)x[c];
        k[c] = threadIdx.x + c;
        k2[c] = threadIdx.x * 3 + c;
    }
    const float fy = (float)y, fz = (float)z;
    const int iz = 7;
    __syncthreads();
    const long long c0 = clock64();
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int r = 0; r < 16; r++) {
#pragma unroll
            for (int c = 0; c < CH; c++) {
                if (OP == FMA_F64) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z));
                else if (OP == ADD_F64) asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[c]) : "v"(z));
                else if (OP == MUL_F64) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(x[c]) : "v"(y));
                else if (OP == LDEXP_F64) asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(x[c]) : "v"(e));
                else if (OP == RSQ_F64) asm volatile("v_rsq_f64 %0, %0" : "+v"(x[c]));
                else if (OP == FMA_F32) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f[c]) : "v"(fy), "v"(fz));
                else if (OP == MUL_F32) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(f[c]) : "v"(fy));
                else if (OP == ADD_U32) asm volatile("v_add_u32 %0, %0, %1" : "+v"(k[c]) : "v"(iz));
                else if (OP == CNDMASK) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(k[c]) : "v"(iz));
                else if (OP == BFE_U32) asm volatile("v_bfe_u32 %0, %0, 3, 8" : "+v"(k[c]));
                else if (OP == LSHR_B32) asm volatile("v_lshrrev_b32 %0, 1, %0" : "+v"(k[c]));
                else if (OP == AND_B32) asm volatile("v_and_b32 %0, 0x7fff, %0" : "+v"(k[c]));
                else if (OP == MOV_B32) asm volatile("v_mov_b32 %0, %1" : "=v"(k[c]) : "v"(k2[c]));
                else if (OP == CVT_F64_I32) asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(x[c]) : "v"(k[c]));
                else if (OP == MIX1 || OP == MIX2 || OP == MIX4) {
                    asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z));
                    asm volatile("v_add_u32 %0, %0, %1" : "+v"(k[c]) : "v"(iz));
                    if (OP != MIX1) asm volatile("v_and_b32 %0, 0x7fff, %0" : "+v"(k2[c]));
                    if (OP == MIX4) {
                        asm volatile("v_lshrrev_b32 %0, 1, %0" : "+v"(k[c]));
                        asm volatile("v_mul_f32 %0, %0, %1" : "+v"(f[c]) : "v"(fy));
                    }
                }
            }
        }
    }
    const long long c1 = clock64();
    double s = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) s += x[c] + f[c] + k[c] + k2[c];
    out[blockIdx.x * blockDim.x * blockDim.y + threadIdx.y * 64 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[threadIdx.y] = c1 - c0;
}

template <int CH, int OP>
void run(int w) {
    double* out;
    long long* cyc;
    hipMalloc(&out, 1 << 20);
    hipMalloc(&cyc, 64 * sizeof(long long));
    const int n = 2048;
    dim3 blk(64, 4 * w);
    for (int rep = 0; rep < 2; rep++)
        hipLaunchKernelGGL((k_chain<CH, OP>), dim3(1), blk, 0, 0, out, cyc, n, 1.0000001, 1e-9);
    hipDeviceSynchronize();
    long long h[64];
    hipMemcpy(h, cyc, sizeof(long long) * 4 * w, hipMemcpyDeviceToHost);
    long long mx = 0;
    for (int i = 0; i < 4 * w; i++) mx = h[i] > mx ? h[i] : mx;
    const double insts = (double)n * 16 * CH * kPerStep[OP];  // per wave
    printf("%-16s chains=%d waves/SIMD=%d: SIMD %.2f cyc/wave-inst (all waves), oldest wave alone %.2f\n", kName[OP],
           CH, w, mx / (insts * w), h[0] / insts);
    hipFree(out);
    hipFree(cyc);
}

template <int OP>
void sweep() {
    run<1, OP>(1);
    for (int w = 1; w <= 4; w *= 2) run<8, OP>(w);
}

int main() {
    sweep<FMA_F64>(); sweep<ADD_F64>(); sweep<MUL_F64>(); sweep<LDEXP_F64>(); sweep<RSQ_F64>();
    sweep<FMA_F32>(); sweep<MUL_F32>(); sweep<ADD_U32>(); sweep<CNDMASK>(); sweep<BFE_U32>();
    sweep<LSHR_B32>(); sweep<AND_B32>(); sweep<MOV_B32>(); sweep<CVT_F64_I32>();
    sweep<MIX1>(); sweep<MIX2>(); sweep<MIX4>();
    run<4, FMA_F64>(3); run<4, MIX2>(3); run<8, MIX2>(3);
    return 0;
}
