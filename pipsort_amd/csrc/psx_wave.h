// psx_wave.h — one-wave (64-lane) batched reductions of the k = 3 sweep
// (k_sweep3) on gfx950: DPP row reductions, and transposed batches through
// v_permlane32_swap / v_permlane16_swap.  Device code only; every lane of the
// wave must be active.
#pragma once

#include <hip/hip_runtime.h>

#include "psx_sweep_dev.h"

namespace psx {

// Batched wave reductions: K independent values reduced together, so the K
// dependency chains interleave (one chain of DPP steps is ~100 cycles of
// latency; eight of them back to back were ~1.8 us of the a prologue at two
// waves per SIMD, tools/unit_trace.py).  Within each row of 16 lanes four
// row_shr steps leave the row's sum / max in its lane 15; row_bcast:15 (into
// rows 1 and 3) and row_bcast:31 (into rows 2 and 3) then carry the rows into
// lane 63, whose value (a fixed summation order) is read as a uniform.  Every
// lane must be active.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double x) {  // lanes without a source read 0 (bound_ctrl)
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), CTRL, 0xf, 0xf, true);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double readlane_f64(double x, int lane) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), lane),
                            __builtin_amdgcn_readlane(__double2loint(x), lane));
}
// (row_bcast:15 adds lane 16r - 1 into row r, row_bcast:31 lane 31 into rows 2
// and 3; rows without a source add 0: lane 63 ends with (S3 + S2) + (S1 + S0))
template <int K>
__device__ __forceinline__ void wave_sum_k(double (&v)[K]) {
#pragma unroll
    for (int k = 0; k < K; k++) v[k] += dpp_f64<0x111>(v[k]);  // row_shr:1
#pragma unroll
    for (int k = 0; k < K; k++) v[k] += dpp_f64<0x112>(v[k]);  // row_shr:2
#pragma unroll
    for (int k = 0; k < K; k++) v[k] += dpp_f64<0x114>(v[k]);  // row_shr:4
#pragma unroll
    for (int k = 0; k < K; k++) v[k] += dpp_f64<0x118>(v[k]);  // row_shr:8
#pragma unroll
    for (int k = 0; k < K; k++) v[k] += dpp_f64<0x142>(v[k]);  // row_bcast:15
#pragma unroll
    for (int k = 0; k < K; k++) v[k] += dpp_f64<0x143>(v[k]);  // row_bcast:31
#pragma unroll
    for (int k = 0; k < K; k++) v[k] = readlane_f64(v[k], 63);
}
// maxima of values >= EMPTY, reduced as x - EMPTY >= 0 so that a lane without a
// DPP source (reading 0) is neutral
template <int CTRL>
__device__ __forceinline__ int dpp_max_b(int y) {
    return max(y, __builtin_amdgcn_mov_dpp(y, CTRL, 0xf, 0xf, true));
}
template <int K>
__device__ __forceinline__ void wave_max_k(int (&v)[K]) {
    int y[K];
#pragma unroll
    for (int k = 0; k < K; k++) y[k] = v[k] - EMPTY;
#pragma unroll
    for (int k = 0; k < K; k++) y[k] = dpp_max_b<0x111>(y[k]);
#pragma unroll
    for (int k = 0; k < K; k++) y[k] = dpp_max_b<0x112>(y[k]);
#pragma unroll
    for (int k = 0; k < K; k++) y[k] = dpp_max_b<0x114>(y[k]);
#pragma unroll
    for (int k = 0; k < K; k++) y[k] = dpp_max_b<0x118>(y[k]);
#pragma unroll
    for (int k = 0; k < K; k++) y[k] = dpp_max_b<0x142>(y[k]);
#pragma unroll
    for (int k = 0; k < K; k++) y[k] = dpp_max_b<0x143>(y[k]);
#pragma unroll
    for (int k = 0; k < K; k++) v[k] = __builtin_amdgcn_readlane(y[k], 63) + EMPTY;
}

// K (shift, sum) pairs at once, as wave_pair_dpp
template <int K>
__device__ __forceinline__ void wave_pair_k(int (&m)[K], double (&x)[K]) {
    int M[K];
#pragma unroll
    for (int k = 0; k < K; k++) M[k] = x[k] != 0.0 ? m[k] : EMPTY;
    wave_max_k(M);
#pragma unroll
    for (int k = 0; k < K; k++) x[k] = x[k] != 0.0 ? ldexp(x[k], m[k] - M[k]) : 0.0;
    wave_sum_k(x);
#pragma unroll
    for (int k = 0; k < K; k++) m[k] = x[k] != 0.0 ? M[k] : EMPTY;
}

// Transposed batches (gfx950 v_permlane32_swap / v_permlane16_swap): K values,
// K a multiple of 4, reduced in halves.  The swap of (v[i], v[i + K/2]) leaves
// lanes 0-31 with v[i] of both wave halves and lanes 32-63 with v[i + K/2] of
// both, so one add per pair halves the batch; the 16-lane swap does the same
// across rows.  The K/4 values left per lane then reduce within their rows
// (row_shr 1, 2, 4, 8 into lane 15): value i + (r & 1) K/4 + (r >> 1) K/2 ends in
// lane 16 r + 15.  ~7 instructions per value instead of ~20.
__device__ __forceinline__ void swap32_f64(double& x, double& y) {
    const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(x), __double2loint(y), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(x), __double2hiint(y), false, false);
    x = __hiloint2double(hi[0], lo[0]);
    y = __hiloint2double(hi[1], lo[1]);
}
__device__ __forceinline__ void swap16_f64(double& x, double& y) {
    const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(x), __double2loint(y), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(x), __double2hiint(y), false, false);
    x = __hiloint2double(hi[0], lo[0]);
    y = __hiloint2double(hi[1], lo[1]);
}
template <int K>
__device__ __forceinline__ void wave_sum_t(double (&v)[K]) {
    static_assert(K % 4 == 0, "transposed batch: K multiple of 4");
    constexpr int H = K / 2, Q = K / 4;
    double a[H], b[Q];
#pragma unroll
    for (int i = 0; i < H; i++) {
        double x = v[i], y = v[i + H];
        swap32_f64(x, y);
        a[i] = x + y;
    }
#pragma unroll
    for (int i = 0; i < Q; i++) {
        double x = a[i], y = a[i + Q];
        swap16_f64(x, y);
        b[i] = x + y;
    }
#pragma unroll
    for (int i = 0; i < Q; i++) b[i] += dpp_f64<0x111>(b[i]);
#pragma unroll
    for (int i = 0; i < Q; i++) b[i] += dpp_f64<0x112>(b[i]);
#pragma unroll
    for (int i = 0; i < Q; i++) b[i] += dpp_f64<0x114>(b[i]);
#pragma unroll
    for (int i = 0; i < Q; i++) b[i] += dpp_f64<0x118>(b[i]);
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
        for (int i = 0; i < Q; i++) v[i + (r & 1) * Q + (r >> 1) * H] = readlane_f64(b[i], 16 * r + 15);
}
// maxima of values >= EMPTY, transposed as wave_sum_t (the biased values are >= 0)
template <int K>
__device__ __forceinline__ void wave_max_t(int (&v)[K]) {
    static_assert(K % 4 == 0, "transposed batch: K multiple of 4");
    constexpr int H = K / 2, Q = K / 4;
    int a[H], b[Q];
#pragma unroll
    for (int i = 0; i < H; i++) {
        const auto r = __builtin_amdgcn_permlane32_swap(v[i] - EMPTY, v[i + H] - EMPTY, false, false);
        a[i] = max((int)r[0], (int)r[1]);
    }
#pragma unroll
    for (int i = 0; i < Q; i++) {
        const auto r = __builtin_amdgcn_permlane16_swap(a[i], a[i + Q], false, false);
        b[i] = max((int)r[0], (int)r[1]);
    }
#pragma unroll
    for (int i = 0; i < Q; i++) b[i] = dpp_max_b<0x111>(b[i]);
#pragma unroll
    for (int i = 0; i < Q; i++) b[i] = dpp_max_b<0x112>(b[i]);
#pragma unroll
    for (int i = 0; i < Q; i++) b[i] = dpp_max_b<0x114>(b[i]);
#pragma unroll
    for (int i = 0; i < Q; i++) b[i] = dpp_max_b<0x118>(b[i]);
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
        for (int i = 0; i < Q; i++) v[i + (r & 1) * Q + (r >> 1) * H] = __builtin_amdgcn_readlane(b[i], 16 * r + 15) + EMPTY;
}

}  // namespace psx
