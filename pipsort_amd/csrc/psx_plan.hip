// psx_plan.hip — a sweep plan's record CSR built on the device, and the
// merge of a batch of generic set records (k_batch_part / k_batch_fold below).
//
// A plan's records are unit-major (slot i = unit * rec_stride + t): the c
// records (t < 64), the b records (64 <= t < 128) and, for k = 3, the a
// records (t >= 128) of each unit.  The merges need, per union SNP u, the
// record slots that hold u in increasing slot order (a stable grouping by SNP):
//   pos[i]   = the buffer position of slot i's record, -1: no SNP (the sweep
//              kernels skip it): i (unit-major), or, for world > 1 since r06,
//              its CSR position q (below), so each SNP's records are contiguous
//   gidx[q]  = the buffer position of the q-th record in (SNP, slot) order
//              (the slot, or the identity with CSR positions)
//   dptr[u]  = first q of SNP u (dptr[U] = records in all): u's run is
//              [dptr[u], dptr[u + 1])
// Built on the host this was ~2M-element passes (8 ms per locus on the
// MI355X host at M = 1000, c = 3); here: one key kernel, hipcub's stable radix
// sort of (SNP, slot) pairs, one binary-search kernel for dptr.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include <cstdlib>

#include "psx_mem.h"
#include "psx_sweep.h"
#include "psx_sweep_dev.h"

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

// Records at their CSR positions (r06): slot gidx[q] is written at position q,
// so each SNP's run is contiguous in the record buffer (the pass merge reads it
// coalesced instead of gathering 56-byte records across units; the sweeps'
// stores scatter instead: measured neutral at world 1 in r04al), and gidx
// becomes the identity for every other merge of the plan's records.
__global__ void k_plan_csr_pos(const int* __restrict__ dptr, int U, long n, int* __restrict__ gidx,
                               int* __restrict__ pos) {
    const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n || q >= dptr[U]) return;
    const int slot = gidx[q];
    pos[slot] = (int)q;
    gidx[q] = (int)q;
}

// keys of a flat record array (record i's SNP, -1: none)
__global__ void k_keys_flat(const int* __restrict__ src, long n, int U, int* __restrict__ keys, int* __restrict__ vals) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int v = src[i];
    keys[i] = v >= 0 ? v : U;
    vals[i] = (int)i;
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

// keys / slots of n records -> stable radix sort by SNP -> gidx, dptr
template <typename FillKeys>
int sort_to_csr(long n, int U, int* d_dptr, int* d_gidx, PlanScratch& S, hipStream_t st, FillKeys fill) {
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
    fill(keys, vals);
    if (chk(hipGetLastError())) return -1;
    // stable: equal SNPs keep increasing slot order (the fold order of the merges)
    if (chk(hipcub::DeviceRadixSort::SortPairs(sort_tmp, tmp, keys, skeys, vals, d_gidx, (int)n, 0, end_bit, st)))
        return -1;
    hipLaunchKernelGGL(k_plan_dptr, dim3((U + 1 + 255) / 256), dim3(256), 0, st, skeys, n, U, d_dptr);
    return chk(hipGetLastError());
}

int plan_csr_device(const int4* d_units, int n_units, int rec_stride, int k, int variant, int pad, int U, int* d_pos,
                    int* d_dptr, int* d_gidx, PlanScratch& S, hipStream_t st, bool csr_pos) {
    const long n = (long)n_units * rec_stride;
    if (sort_to_csr(n, U, d_dptr, d_gidx, S, st, [&](int* keys, int* vals) {
            hipLaunchKernelGGL(k_plan_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, d_units, n,
                               rec_stride, k, variant, pad, U, keys, vals, d_pos);
        }))
        return -1;
    if (n == 0 || !csr_pos) return 0;
    hipLaunchKernelGGL(k_plan_csr_pos, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, d_dptr, U, n, d_gidx, d_pos);
    return chk(hipGetLastError());
}

// Where a shard's records go (the fold order, hence every result, is the same
// either way): at their CSR positions for world > 1, where the merge is a large
// share of a single pass (world 8 0.165 -> 0.162 ms); unit-major (slot i at i,
// the merges gather through gidx) at world 1, where the sweep's coalesced record
// stores win (kernel 0.758 vs 0.771 ms, bench step 0.798 vs 0.806 ms, same-box
// A/B, profiles/r06/r06q_*).  PSX_REC_CSR = 0 / 1 forces either.
bool records_at_csr_positions(int world) {
    static const int force = [] {
        const char* e = std::getenv("PSX_REC_CSR");
        return e ? (e[0] == '0' ? 0 : 1) : -1;
    }();
    return force >= 0 ? force == 1 : world > 1;
}

// the CSR of records laid out flat with SNP keys[i] (-1: none): dptr[U + 1],
// gidx[n] (records of SNP u in increasing index order at [dptr[u], dptr[u + 1]))
int csr_from_keys_device(const int* d_keys, long n, int U, int* d_dptr, int* d_gidx, PlanScratch& S, hipStream_t st) {
    return sort_to_csr(n, U, d_dptr, d_gidx, S, st, [&](int* keys, int* vals) {
        hipLaunchKernelGGL(k_keys_flat, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, d_keys, n, U, keys,
                           vals);
    });
}

// ---------------------------------------------------------------------------
// Set-batch merge (psx_eval_union_batch, the generic levels): fold the member
// records of n union sets ([set][stride], record j of a set = its j-th member)
// into the per-SNP accumulators and the set records into the scalars, in two
// launches and a fixed order, without a device-wide sort.
//   k_batch_part  chunk c = 256 records of whole sets: a wave radix-sorts the
//                 chunk's (SNP, record) pairs in LDS; each thread folds the runs
//                 of its 4 sorted positions, a fixed binary tree over the
//                 threads joins the runs that cross threads; every SNP's chunk
//                 total goes to part[c][u] + a presence bit, the chunk's set
//                 records to spart[c]
//   k_batch_fold  a wave per SNP u folds part[0..nc)[u] (present ones, nc <= 256)
//                 by a fixed shuffle tree into acc[u]; one wave folds
//                 spart[0..nc) into the scalars
// ---------------------------------------------------------------------------
namespace {

constexpr int kBT = 64, kBI = 4;  // a chunk: one wave, 256 records (more chunks in flight, no cross-wave sort)
constexpr int kBWords = 4096;  // presence bitmap words in LDS: U <= 131072

// A run of equal SNPs over a range of sorted positions: the first and last runs
// (possibly the same: full) of the range, and its first / last SNPs; the runs
// strictly inside have been emitted.
struct BRange {
    int fk, lk, full, pad;
    Acc5 F, L;
};

__global__ __launch_bounds__(kBT) void k_batch_part(const int* __restrict__ sets, int stride, long nsets, int spc,
                                                   int U, int end_bit, const Acc5* __restrict__ rec,
                                                   const SetRec* __restrict__ srec, Acc5* __restrict__ part,
                                                   unsigned* __restrict__ bits, int words, SetRec* __restrict__ spart,
                                                   const unsigned long long* __restrict__ bad,
                                                   unsigned long long badv, unsigned long long* __restrict__ tstamp) {
    if (tstamp && blockIdx.x == 0 && threadIdx.x == 0) *tstamp = wall_clock64();  // (the batch's kernel clock)
    if (bad && *bad == badv) return;  // an invalid row: the batch adds nothing (uniform)
    using Sort = hipcub::BlockRadixSort<int, kBT, kBI, int>;
    __shared__ union {
        typename Sort::TempStorage sort;
        BRange node[kBT];
    } sh;
    __shared__ SetRec sw[kBT / 64];
    __shared__ unsigned sbits[kBWords];
    const int t = threadIdx.x, c = blockIdx.x;
    const long s0 = (long)c * spc, s1 = s0 + spc < nsets ? s0 + spc : nsets;
    const int n = (int)((s1 - s0) * stride);
    const int* ks = sets + s0 * stride;
    const Acc5* rc = rec + s0 * stride;
    for (int w = t; w < words; w += kBT) sbits[w] = 0u;
    int key[kBI], val[kBI];
#pragma unroll
    for (int j = 0; j < kBI; j++) {
        const int i = t * kBI + j;
        const int v = i < n ? ks[i] : -1;
        key[j] = v >= 0 ? v : U;  // no SNP: sorted behind every SNP
        val[j] = i;
    }
    // the chunk's set records, thread-strided (spc <= kBT kBI: at most kBI per
    // thread), loaded whole from clamped indices before the sort and folded
    // after it in the same order.  (A fold of srec[i] in the loop let the
    // compiler split each record into guarded field loads, one round trip per
    // field, late r06.)
    SetRec sv[kBI];
#pragma unroll
    for (int q = 0; q < kBI; q++) {
        const long i = s0 + t + (long)q * kBT;
        sv[q] = srec[i < s1 ? i : s1 - 1];
    }
#pragma unroll
    for (int q = 0; q < kBI; q++)  // (every field materialised: no guarded field loads)
        asm volatile("" : "+v"(sv[q].m), "+v"(sv[q].m0), "+v"(sv[q].m1), "+v"(sv[q].tot), "+v"(sv[q].nc0),
                     "+v"(sv[q].nc1), "+v"(sv[q].score), "+v"(sv[q].npat));
    Sort(sh.sort).Sort(key, val, 0, end_bit);  // blocked: thread t holds sorted positions kBI t .. kBI t + kBI - 1
    SetRec a = set_zero();
#pragma unroll
    for (int q = 0; q < kBI; q++)
        if (s0 + t + (long)q * kBT < s1) fold_set(a, sv[q]);
    Acc5 r[kBI];
#pragma unroll
    for (int j = 0; j < kBI; j++) r[j] = key[j] < U ? rc[val[j]] : acc_zero();
    auto emit = [&](int u, const Acc5& g) {
        if (u >= U) return;
        part[(size_t)c * U + u] = g;
        atomicOr(&sbits[u >> 5], 1u << (u & 31));
    };
    // the thread's 8 positions: runs inside are complete, the first and last stay open
    BRange A;
    A.fk = key[0];
    A.full = 1;
    A.F = acc_zero();
    Acc5 cur = acc_zero();
    int ck = key[0];
#pragma unroll
    for (int j = 0; j < kBI; j++) {
        if (key[j] != ck) {
            if (A.full) A.F = cur;
            else emit(ck, cur);
            A.full = 0;
            cur = acc_zero();
            ck = key[j];
        }
        fold_acc(cur, r[j]);
    }
    A.lk = ck;
    A.L = cur;
    if (A.full) A.F = cur;
    __syncthreads();  // the sort's LDS is reused for the ranges
    // Fixed binary tree over the 256 ranges (left folds right): a run is
    // emitted once it is closed on both sides, so each SNP of the chunk once.
    for (int h = 1; h < kBT; h <<= 1) {
        if ((t & (h - 1)) == 0 && (t & h)) sh.node[t] = A;
        __syncthreads();
        if ((t & (2 * h - 1)) == 0) {
            const BRange& B = sh.node[t + h];
            if (A.lk == B.fk) {
                Acc5 mid = A.L;
                fold_acc(mid, B.F);
                if (A.full && B.full) {
                    A.F = A.L = mid;
                } else if (A.full) {
                    A.F = mid;
                    A.L = B.L;
                    A.lk = B.lk;
                    A.full = 0;
                } else if (B.full) {
                    A.L = mid;
                } else {
                    emit(A.lk, mid);
                    A.L = B.L;
                    A.lk = B.lk;
                }
            } else {
                if (!A.full) emit(A.lk, A.L);
                if (!B.full) emit(B.fk, B.F);
                A.L = B.L;
                A.lk = B.lk;
                A.full = 0;
            }
        }
        __syncthreads();
    }
    if (t == 0) {
        emit(A.fk, A.F);
        if (!A.full) emit(A.lk, A.L);
    }
    // the chunk's set records: wave and block trees
    wave_fold_set(a);
    if ((t & 63) == 0) sw[t >> 6] = a;
    __syncthreads();
    for (int w = t; w < words; w += kBT) bits[(size_t)c * words + w] = sbits[w];
    if (t == 0) {
        SetRec g = sw[0];
        for (int w = 1; w < kBT / 64; w++) fold_set(g, sw[w]);
        spart[c] = g;
    }
}

// a wave per SNP: lane l folds chunks l, l + 64, l + 128, l + 192 (the present
// ones, nc <= 256) in that order, a fixed shuffle tree folds the lanes, lane 0
// folds the result into acc[u]
__global__ __launch_bounds__(256) void k_batch_fold(const Acc5* __restrict__ part, const unsigned* __restrict__ bits,
                                                   int words, int nc, int U, const SetRec* __restrict__ spart,
                                                   Acc5* __restrict__ acc, SetRec* __restrict__ sacc,
                                                   const unsigned long long* __restrict__ bad,
                                                   unsigned long long badv) {
    if (bad && *bad == badv) return;
    const int lane = threadIdx.x & 63;
    const int u = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (u < U) {
        // every load up front (the accumulator, the presence words and the
        // partials of all the lane's chunks, absent ones discarded): one round
        // trip instead of three dependent ones
        Acc5 a0 = acc_zero();
        if (lane == 0) a0 = acc[u];
        unsigned w[4];
        Acc5 q[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int c = lane + 64 * r;
            w[r] = c < nc ? bits[(size_t)c * words + (u >> 5)] : 0u;
            q[r] = c < nc ? part[(size_t)c * U + u] : acc_zero();
        }
        Acc5 g = acc_zero();
        bool have = false;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            if ((w[r] >> (u & 31)) & 1u) {
                fold_acc(g, q[r]);
                have = true;
            }
        }
        if (__ballot(have)) {
            wave_fold_acc(g);
            if (lane == 0) {
                fold_acc(a0, g);
                acc[u] = a0;
            }
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < 64) {
        SetRec s = set_zero();
        for (int c = threadIdx.x; c < nc; c += 64) fold_set(s, spart[c]);
        wave_fold_set(s);
        if (threadIdx.x == 0) {
            SetRec g = *sacc;
            fold_set(g, s);
            *sacc = g;
        }
    }
}

}  // namespace

int batch_merge_sets_per_chunk(int stride) { return (kBT * kBI) / stride; }

int batch_merge_chunks(long nsets, int stride) {
    const long spc = (kBT * kBI) / stride;
    return (int)((nsets + spc - 1) / spc);
}

size_t batch_merge_bytes(long nsets, int stride, int U) {
    const size_t nc = (size_t)batch_merge_chunks(nsets, stride), words = ((size_t)U + 31) / 32;
    return nc * ((size_t)U * sizeof(Acc5) + words * sizeof(unsigned) + sizeof(SetRec)) + 256;
}

int launch_merge_batch(const int* d_sets, int stride, long nsets, int U, const Acc5* rec, const SetRec* srec,
                       void* scratch, Acc5* acc, SetRec* sacc, hipStream_t st, const unsigned long long* bad,
                       unsigned long long badv, unsigned long long* tstamp) {
    if (nsets <= 0) return 0;
    const int words = (U + 31) / 32;
    if (words > kBWords || stride < 1 || stride > kBT * kBI) return -1;
    const int spc = (kBT * kBI) / stride, nc = batch_merge_chunks(nsets, stride);
    int end_bit = 1;
    while ((1 << end_bit) <= U) end_bit++;
    Acc5* part = (Acc5*)scratch;
    SetRec* spart = (SetRec*)(part + (size_t)nc * U);
    unsigned* bits = (unsigned*)(spart + nc);
    hipLaunchKernelGGL(k_batch_part, dim3(nc), dim3(kBT), 0, st, d_sets, stride, nsets, spc, U, end_bit, rec, srec,
                       part, bits, words, spart, bad, badv, tstamp);
    if (chk(hipGetLastError())) return -1;
    hipLaunchKernelGGL(k_batch_fold, dim3((U + 3) / 4), dim3(256), 0, st, part, bits, words, nc, U, spart, acc,
                       sacc, bad, badv);
    return chk(hipGetLastError());
}

// load this translation unit's device code on the current device (psx_warmup)
int warm_module_plan() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, (const void*)k_plan_keys) == hipSuccess ? 0 : -1;
}

}  // namespace psx
