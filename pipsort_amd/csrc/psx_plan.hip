// psx_plan.hip — a sweep plan's record CSR built on the device.
//
// A plan's records are unit-major (slot i = unit * rec_stride + t): the c
// records (t < 64), the b records (64 <= t < 128) and, for k = 3, the a
// records (t >= 128) of each unit.  The merges need, per union SNP u, the
// record slots that hold u in increasing slot order (a stable grouping by SNP):
//   pos[i]   = i when slot i holds a SNP, else -1 (the sweep kernels skip it)
//   gidx[q]  = the q-th record slot in (SNP, slot) order
//   dptr[u]  = first q of SNP u (dptr[U] = records in all): u's run is
//              [dptr[u], dptr[u + 1])
// Built on the host this was ~2M-element passes (8 ms per locus on the
// MI355X host at M = 1000, c = 3); here: one key kernel, hipcub's stable radix
// sort of (SNP, slot) pairs, one binary-search kernel for dptr.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include "psx_mem.h"
#include "psx_sweep.h"

namespace psx {

namespace {

// The SNP (union index, -1: none) of record slot i, as the sweep kernels write
// them (psx_sweep3.hip / psx_sweep.hip; the host restatement was build_plan's
// key loop): variant 1 packs each unit's b-walk step range in the high bits
// of B / T and keeps v = u + pad indices; a diagonal tile of the k = 3 fast
// kernel writes its c and b-slot records of one SNP as one (c) record.
__global__ void k_plan_keys(const int4* __restrict__ units, long n, int rec_stride, int k, int variant, int pad, int U,
                            int* __restrict__ keys, int* __restrict__ vals, int* __restrict__ pos) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int unit = (int)(i / rec_stride), t = (int)(i % rec_stride);
    const int4 u = units[unit];
    const int B = u.z & 0xffff, T = u.w & 0xffff;
    int key = -1;
    if (t < 64) {
        const int c = 64 * T + t - pad;
        if (c >= 0 && c < U) key = c;
    } else if (t < 128) {
        const bool one = variant && k == 3 && B == T;
        const int b = 64 * B + (t - 64) - pad;
        if (!one && b >= 0 && b < U) key = b;
    } else if (k == 3) {
        const int a = u.x + (t - 128);
        if (a < u.y) key = a - pad;
    }
    keys[i] = key >= 0 ? key : U;  // no SNP: sorted behind every SNP
    vals[i] = (int)i;
    pos[i] = key >= 0 ? (int)i : -1;
}

// dptr[u] = lower_bound(sorted keys, u), u = 0 .. U
__global__ void k_plan_dptr(const int* __restrict__ skeys, long n, int U, int* __restrict__ dptr) {
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u > U) return;
    long lo = 0, hi = n;
    while (lo < hi) {
        const long mid = (lo + hi) >> 1;
        if (skeys[mid] < u) lo = mid + 1; else hi = mid;
    }
    dptr[u] = (int)lo;
}

int chk(hipError_t e) { return e == hipSuccess ? 0 : -1; }

}  // namespace

int plan_csr_device(const int4* d_units, int n_units, int rec_stride, int k, int variant, int pad, int U, int* d_pos,
                    int* d_dptr, int* d_gidx, PlanScratch& S, hipStream_t st) {
    const long n = (long)n_units * rec_stride;
    if (n == 0) return chk(hipMemsetAsync(d_dptr, 0, sizeof(int) * (U + 1), st));
    int end_bit = 1;
    while ((1 << end_bit) <= U) end_bit++;
    size_t tmp = 0;
    if (chk(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (const int*)nullptr, (int*)nullptr, (const int*)nullptr,
                                               (int*)nullptr, (int)n, 0, end_bit, st)))
        return -1;
    // scratch: keys, sorted keys, slots (the sorted slots go straight to gidx), sort temp
    const size_t need = sizeof(int) * 3 * (size_t)n + tmp + 256;
    if (need > S.bytes) {
        if (S.p) psx::dfree(S.p);
        S.p = nullptr;
        S.bytes = 0;
        if (chk(psx::dmalloc(&S.p, need))) return -1;
        S.bytes = need;
    }
    int* keys = (int*)S.p;
    int* skeys = keys + n;
    int* vals = skeys + n;
    void* sort_tmp = (void*)(((uintptr_t)(vals + n) + 255) & ~(uintptr_t)255);
    hipLaunchKernelGGL(k_plan_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, d_units, n, rec_stride, k,
                       variant, pad, U, keys, vals, d_pos);
    if (chk(hipGetLastError())) return -1;
    // stable: equal SNPs keep increasing slot order (the fold order of the merges)
    if (chk(hipcub::DeviceRadixSort::SortPairs(sort_tmp, tmp, keys, skeys, vals, d_gidx, (int)n, 0, end_bit, st)))
        return -1;
    hipLaunchKernelGGL(k_plan_dptr, dim3((U + 1 + 255) / 256), dim3(256), 0, st, skeys, n, U, d_dptr);
    return chk(hipGetLastError());
}

// load this translation unit's device code on the current device (psx_warmup)
int warm_module_plan() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, (const void*)k_plan_keys) == hipSuccess ? 0 : -1;
}

}  // namespace psx
