// psx_configs.hip — the -b configs-file enumerator on the device
// (PostCal::computeTotalLikelihoodGivenConfigs, postcal.cpp:400-714).
//
// The reference walks the mmapped int16 rows one by one (postcal.cpp:441-590):
// global SNP indices -> union positions (sorted, unique), then a study-major walk
// that assigns every entry to a (study, member) pair and exits on a row out of
// order; every row is then one forced causal assignment evaluated by the
// low-rank likelihood and folded into the accumulators (postcal.cpp:611-681).
// Here the raw rows go to the device once and five launches do the rest:
//
//   k_cfg_count  a thread per row, ALL rows: the walk, the first failing row
//                (atomic min, so every rank of a sharded run rejects the same
//                file), and for this rank's slice per-block counts of evaluated
//                rows / member records and per-SNP record counts
//   k_cfg_scan   one block: exclusive scans -> per-block output offsets (row
//                order) and the per-SNP record CSR pointer
//   (host)       one status read: the failing row, the counts
//   k_cfg_eval   a thread per row of the slice: the walk again, the row's two
//                forced subsets factored (ldlt_terms), its set record, its
//                assignment's weights and its member records' sort keys, all
//                at offsets fixed by row order
//   radix sort   (hipcub, stable) member records by union SNP: the CSR's record
//                order within an SNP is row order, as the host pass built it
//   k_cfg_merge  per union SNP, its records in that order, folded in two levels:
//                S contiguous slices of the SNP's run by one block each, then
//                the S partials in slice order (a file's records concentrate on
//                the few SNPs its groups name: one block per SNP left the GPU
//                idle for ~3 ms on 29M records, r03e); the records themselves
//                are rebuilt from the row's weights and its assignment masks
//                (no 56-byte record per member in HBM)
//   k_cfg_sets   the set records folded the same way: contiguous chunks, then
//                the chunk partials in order (the one-block fold took 6 ms on
//                4.8M rows)
//
// Every fold order is fixed by the row order and the launch shapes, so the
// results are deterministic (and within rounding of the host pre-pass this
// replaced).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

#include "psx_configs.h"
#include "psx_sweep.h"
#include "psx_sweep_dev.h"
#include "psx_mem.h"

namespace psx {

namespace {

constexpr int kRowsPerBlock = 256;
constexpr int kLdsHistMax = 16384;  // union SNPs whose per-block counts fit in LDS (64 KB)

// the one forced assignment of an evaluated row (the weights k_eval_rows gives
// every member record of the row); valid == 0: the assignment adds nothing
struct CfgRow {
    double w, wll;
    int G, Ck, valid, pad;
};

// postcal.cpp:441-590 for one row, as the host pass restated it: returns k
// (0: null row), -1 an index outside [0, N), -2 more than PSX_KMAX union SNPs,
// -3 the study-major walk failed (postcal.cpp:587-590).  locs: the sorted union
// positions; b0 / b1: the members causal in study 0 / 1.  Register-only (every
// array index is a compile-time constant after unrolling).
__device__ int cfg_row(const int16_t* in, int ng, const CfgMaps& C, int (&locs)[PSX_KMAX], int& b0, int& b1) {
    int n = 0;
    bool over = false;
    for (int i = 0; i < ng; i++) {
        const int g = in[i];
        if (g < 0) continue;
        if (g >= C.N) return -1;
        const int u = C.l2u[g];  // study (g >= m0) and local index fold into the concatenated map
        bool dup = false;
        int p = 0;  // insertion position: members below u
#pragma unroll
        for (int q = 0; q < PSX_KMAX; q++)
            if (q < n) {
                dup |= locs[q] == u;
                p += locs[q] < u;
            }
        if (dup) continue;
        if (n == PSX_KMAX) {
            over = true;
            continue;
        }
#pragma unroll
        for (int q = PSX_KMAX - 1; q > 0; q--)
            if (q > p && q <= n) locs[q] = locs[q - 1];
#pragma unroll
        for (int q = 0; q < PSX_KMAX; q++)
            if (q == p) locs[q] = u;
        n++;
    }
    if (over) return -2;
    if (n == 0) return 0;  // postcal.cpp:459-488
    b0 = b1 = 0;
    int aux = 0;
    while (aux < ng && in[aux] < 0) aux++;
    int cum = 0;
    for (int i = 0; i < 2; i++) {
        cum += i ? C.m1 : C.m0;
        const int offi = i ? C.m0 : 0;
        bool stop = false;
#pragma unroll
        for (int j = 0; j < PSX_KMAX; j++) {
            if (j >= n || stop) continue;
            const int loc = C.u2l[i * C.U + locs[j]];
            if (loc < 0) continue;
            const int gidx = offi + loc;
            if (gidx >= cum) {
                stop = true;
                continue;
            }
            if (aux < ng && in[aux] == gidx) {
                aux++;
                if (i) b1 |= 1 << j;
                else b0 |= 1 << j;
                while (aux < ng && in[aux] < 0) aux++;
            }
        }
        if (aux == ng) break;
    }
    return aux == ng ? n : -3;
}

// exclusive prefix (row order) of two per-thread counts over the block, and totals
__device__ void block_exscan2(int a, int b, int& pa, int& pb, int& ta, int& tb) {
    __shared__ int sa[kRowsPerBlock / 64], sb[kRowsPerBlock / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int xa = a, xb = b;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int ya = __shfl_up(xa, o), yb = __shfl_up(xb, o);
        if (lane >= o) {
            xa += ya;
            xb += yb;
        }
    }
    if (lane == 63) {
        sa[w] = xa;
        sb[w] = xb;
    }
    __syncthreads();
    int oa = 0, ob = 0;
    ta = tb = 0;
#pragma unroll
    for (int i = 0; i < kRowsPerBlock / 64; i++) {
        if (i < w) {
            oa += sa[i];
            ob += sb[i];
        }
        ta += sa[i];
        tb += sb[i];
    }
    pa = oa + xa - a;
    pb = ob + xb - b;
    __syncthreads();  // sa / sb are reused by the next call
}

__global__ __launch_bounds__(kRowsPerBlock) void k_cfg_count(const int16_t* __restrict__ rows, long n_rows, int ng,
                                                            CfgMaps C, long r0, long r1,
                                                            unsigned long long* __restrict__ status,
                                                            int* __restrict__ blk, int nblk, int* __restrict__ hist,
                                                            int lds_hist) {
    extern __shared__ int sh_hist[];
    if (lds_hist)
        for (int u = threadIdx.x; u < C.U; u += kRowsPerBlock) sh_hist[u] = 0;
    __syncthreads();
    const long r = (long)blockIdx.x * kRowsPerBlock + threadIdx.x;
    int locs[PSX_KMAX] = {0, 0, 0, 0, 0, 0}, b0 = 0, b1 = 0, code = 0;
    if (r < n_rows) {
        code = cfg_row(rows + r * ng, ng, C, locs, b0, b1);
        if (code < 0) atomicMin(&status[0], ((unsigned long long)r << 3) | (unsigned long long)(-code));
    }
    const bool mine = r >= r0 && r < r1;
    const int k = (mine && code > 0) ? code : 0;
#pragma unroll
    for (int j = 0; j < PSX_KMAX; j++)
        if (j < k) {
            if (lds_hist) atomicAdd(&sh_hist[locs[j]], 1);
            else atomicAdd(&hist[locs[j]], 1);
        }
    int ps, pr, ts, tr;
    block_exscan2(k > 0, k, ps, pr, ts, tr);
    int pn, pz, tn, tz;
    block_exscan2((mine && code == 0) ? 1 : 0, 0, pn, pz, tn, tz);
    if (threadIdx.x == 0) {
        blk[blockIdx.x] = ts;
        blk[nblk + blockIdx.x] = tr;
        if (tn) atomicAdd(&status[1], (unsigned long long)tn);
    }
    if (lds_hist) {
        __syncthreads();
        for (int u = threadIdx.x; u < C.U; u += kRowsPerBlock)
            if (sh_hist[u]) atomicAdd(&hist[u], sh_hist[u]);
    }
}

// exclusive scan of n ints in place (out may alias in) by one 1024-thread block;
// returns the total in thread 0
__device__ long block_scan_inplace(int* a, int n) {
    __shared__ long part[1024];
    const int t = threadIdx.x;
    const int chunk = (n + 1023) / 1024;
    const int lo = t * chunk < n ? t * chunk : n, hi = lo + chunk < n ? lo + chunk : n;
    long s = 0;
    for (int i = lo; i < hi; i++) s += a[i];
    part[t] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan of the partials
        const long v = t >= o ? part[t - o] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    long run = part[t] - s;
    const long total = part[1023];
    for (int i = lo; i < hi; i++) {
        const int x = a[i];
        a[i] = (int)run;
        run += x;
    }
    __syncthreads();
    return total;
}

__global__ __launch_bounds__(1024) void k_cfg_scan(int* __restrict__ blk, int nblk, int* __restrict__ ptr, int U,
                                                   unsigned long long* __restrict__ status) {
    unsigned long long mx = 0;  // the most records of one union SNP (sizes the member fold's slices)
    for (int u = threadIdx.x; u < U; u += 1024) mx = max(mx, (unsigned long long)ptr[u]);
    if (mx) atomicMax(&status[4], mx);
    const long sets = block_scan_inplace(blk, nblk);
    const long recs = block_scan_inplace(blk + nblk, nblk);
    const long recs2 = block_scan_inplace(ptr, U);
    if (threadIdx.x == 0) {
        status[2] = (unsigned long long)sets;
        status[3] = (unsigned long long)recs;
        ptr[U] = (int)recs2;
    }
}

// A row of the slice: the walk, the forced assignment (c0 = b0, c1 = b1) of its
// k union SNPs evaluated exactly as k_eval_rows does it (psx_engine.hip), and
// its outputs at its row-order offsets.
__global__ __launch_bounds__(kRowsPerBlock) void k_cfg_eval(const int16_t* __restrict__ rows, int ng, CfgMaps C,
                                                           long r0, long r1, CfgProb P, const int* __restrict__ blk,
                                                           int nblk, SetRec* __restrict__ srec,
                                                           CfgRow* __restrict__ rrec, int* __restrict__ masks,
                                                           unsigned* __restrict__ keys, int* __restrict__ vals) {
    constexpr int KM = PSX_KMAX;
    const long r = (long)blockIdx.x * kRowsPerBlock + threadIdx.x;
    int mem[KM] = {0, 0, 0, 0, 0, 0}, c0 = 0, c1 = 0, k = 0;
    if (r >= r0 && r < r1) {
        const int code = cfg_row(rows + r * ng, ng, C, mem, c0, c1);
        k = code > 0 ? code : 0;  // failing rows were rejected before this launch
    }
    int ps, pr, ts, tr;
    block_exscan2(k > 0, k, ps, pr, ts, tr);
    if (k == 0) return;
    const long si = (long)blk[blockIdx.x] + ps;
    const long ri = (long)blk[nblk + blockIdx.x] + pr;
    int S0 = 0, S1 = 0;
#pragma unroll
    for (int j = 0; j < KM; j++)
        if (j < k) {
            const unsigned pr_ = P.pres[mem[j]];
            if (pr_ & 1u) S0 |= 1 << j;
            if (pr_ & 2u) S1 |= 1 << j;
        }
    const int Ck = P.Ck[k];
    SetRec rr = set_zero();
    CfgRow row{0.0, 0.0, 0, 0, 0, 0};
    const bool valid = ((c0 | c1) == (1 << k) - 1) && !(c0 & ~S0) && !(c1 & ~S1);
    if (valid) {
        double mu[2], f[2];
        int n[2];
        for (int s = 0; s < 2; s++) {
            const int cs = s ? c1 : c0;
            int idx[KM];
            int t = 0;
            for (int j = 0; j < k; j++)
                if ((cs >> j) & 1) idx[t++] = mem[j];
            double q, Pd;
            ldlt_terms(P.G[s], P.ldg, P.Ad[s], P.y[s], P.dval[s], idx, t, q, Pd);
            split_exp(0.5 * q * PSX_LOG2E, 1.0 / sqrt(Pd), n[s], mu[s]);
            f[s] = 0.5 * q - 0.5 * log(Pd);
        }
        const int nsh = __popc(c0 & c1);
        const double mup = mu[0] * mu[1];
        const int np = n[0] + n[1];
        const int G = np + 2;  // k_eval_sets' "+ 2" headroom, at this assignment's exponent
        const double wll = ldexp(mup, -2);
        const double w = wll * P.pit[k][nsh];
        rr.m = G + Ck;
        rr.tot = w;
        rr.m0 = rr.m1 = np + Ck;
        rr.nc0 = c0 == 0 ? mup * P.pit[k][0] : 0.0;
        rr.nc1 = c1 == 0 ? mup * P.pit[k][0] : 0.0;
        rr.score = f[0] + f[1] + P.prior[k][nsh];
        rr.npat = 1.0;
        row = CfgRow{w, wll, G, Ck, 1, 0};
    }
    srec[si] = rr;
    rrec[si] = row;
    masks[si] = c0 | (c1 << 8);
#pragma unroll
    for (int j = 0; j < KM; j++)
        if (j < k) {
            keys[ri + j] = (unsigned)mem[j];
            vals[ri + j] = (int)(si * KM + j);
        }
}

// member j of row `set`: the record k_eval_rows writes for it
__device__ __forceinline__ Acc5 cfg_record(const CfgRow* __restrict__ rrec, const int* __restrict__ masks, int q) {
    const int set = q / PSX_KMAX, j = q - set * PSX_KMAX;
    const CfgRow row = rrec[set];
    Acc5 a = acc_zero();
    if (!row.valid) return a;
    const int m = masks[set];
    const int x = ((m >> j) & 1) | (((m >> (8 + j)) & 1) << 1);
    a.mP = row.G + row.Ck;
    a.mS = a.mN = row.G;
    a.post0 = (x & 1) ? row.w : 0.0;
    a.post1 = (x & 2) ? row.w : 0.0;
    a.shared = x == 3 ? row.w : 0.0;
    a.sll = x == 3 ? row.wll : 0.0;
    a.nsll = x == 3 ? 0.0 : row.wll;
    return a;
}

// per union SNP u, its records in CSR order (row order), folded as
// k_merge_members (psx_sweep.hip) folds gathered records: 256 threads, eight
// loads in flight per thread, then the wave / block trees.  Level 1: block
// (u, s) folds slice s of S of u's run into parts[u * S + s]; level 2 (one
// thread per SNP) folds the S partials in slice order into acc[u].
constexpr int kMergeR = 8;
constexpr int kSliceRecs = 8192;  // records per level-1 slice (S = ceil(most / kSliceRecs))
constexpr int kMaxSlices = 256;
__global__ __launch_bounds__(256) void k_cfg_merge(const CfgRow* __restrict__ rrec, const int* __restrict__ masks,
                                                   const int* __restrict__ ptr, const int* __restrict__ idx, int S,
                                                   Acc5* __restrict__ parts) {
    __shared__ Acc5 sh[4];
    const int u = blockIdx.x, sl = blockIdx.y;
    const long b0 = ptr[u], len = ptr[u + 1] - b0;
    const int b = (int)(b0 + len * sl / S), e = (int)(b0 + len * (sl + 1) / S);
    Acc5 a = acc_zero();
    for (int i0 = b + (int)threadIdx.x; i0 < e; i0 += 256 * kMergeR) {
        int ix[kMergeR];
#pragma unroll
        for (int q = 0; q < kMergeR; q++) ix[q] = i0 + 256 * q < e ? idx[i0 + 256 * q] : -1;
        Acc5 v[kMergeR];
#pragma unroll
        for (int q = 0; q < kMergeR; q++) v[q] = ix[q] >= 0 ? cfg_record(rrec, masks, ix[q]) : acc_zero();
#pragma unroll
        for (int q = 0; q < kMergeR; q++) fold_acc(a, v[q]);
    }
    wave_fold_acc(a);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = a;
    __syncthreads();
    if (threadIdx.x == 0) {
        Acc5 g = acc_zero();
        for (int w = 0; w < 4; w++) fold_acc(g, sh[w]);
        parts[(size_t)u * S + sl] = g;
    }
}

__global__ __launch_bounds__(64) void k_cfg_merge2(const Acc5* __restrict__ parts, int S, int U,
                                                   Acc5* __restrict__ acc) {
    const int u = blockIdx.x * 64 + threadIdx.x;
    if (u >= U) return;
    Acc5 g = acc[u];
    for (int sl = 0; sl < S; sl++) fold_acc(g, parts[(size_t)u * S + sl]);
    acc[u] = g;
}

// the set records: block b folds chunk b (contiguous, row order) into parts[b]
constexpr int kSetChunk = 4096;
constexpr int kMaxSetChunks = 2048;
__global__ __launch_bounds__(256) void k_cfg_sets(const SetRec* __restrict__ rec, long n, long chunk,
                                                  SetRec* __restrict__ parts) {
    __shared__ SetRec sh[4];
    const long b = (long)blockIdx.x * chunk, e = min(n, b + chunk);
    SetRec a = set_zero();
    for (long i0 = b + threadIdx.x; i0 < e; i0 += 256 * kMergeR) {
        SetRec v[kMergeR];
#pragma unroll
        for (int q = 0; q < kMergeR; q++) v[q] = i0 + 256 * q < e ? rec[i0 + 256 * q] : set_zero();
#pragma unroll
        for (int q = 0; q < kMergeR; q++) fold_set(a, v[q]);
    }
    wave_fold_set(a);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = a;
    __syncthreads();
    if (threadIdx.x == 0) {
        SetRec g = set_zero();
        for (int w = 0; w < 4; w++) fold_set(g, sh[w]);
        parts[blockIdx.x] = g;
    }
}

// Host rows -> device.  The caller's rows are pageable (an mmapped -b file, a
// numpy array), which the runtime would stage chunk by chunk on one thread;
// here T host threads copy each 8 MB chunk into one of two pinned buffers while
// the DMA engine moves the previous chunk: the upload runs at the slower of the
// parallel host copy and the PCIe transfer instead of their sum.
constexpr size_t kStageChunk = 8u << 20;
int upload_rows(CfgWork& W, const void* src, size_t bytes, void* dst, hipStream_t st) {
    if (bytes <= 2 * kStageChunk)
        return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st) == hipSuccess ? 0 : -1;
    if (!W.hpin && psx::hmalloc(reinterpret_cast<void**>(&W.hpin), 2 * kStageChunk) != hipSuccess) return -1;
    for (int b = 0; b < 2; b++)
        if (!W.dma[b] && hipEventCreateWithFlags(&W.dma[b], hipEventDisableTiming) != hipSuccess) return -1;
    const size_t nch = (bytes + kStageChunk - 1) / kStageChunk;
    cpu_set_t set;
    CPU_ZERO(&set);
    const int cores = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set) : 4;
    const int T = std::max(1, std::min(cores, 8));
    std::unique_ptr<std::atomic<int>[]> done(new std::atomic<int>[nch]);
    for (size_t c = 0; c < nch; c++) done[c].store(0);
    std::atomic<size_t> writable{2};  // chunks below this may be copied into their pinned buffer
    auto work = [&](int t) {
        for (size_t c = 0; c < nch; c++) {
            while (writable.load(std::memory_order_acquire) <= c) std::this_thread::yield();
            const size_t len = std::min(kStageChunk, bytes - c * kStageChunk);
            const size_t a = len * t / T, e = len * (t + 1) / T;
            std::memcpy(W.hpin + (c & 1) * kStageChunk + a, (const char*)src + c * kStageChunk + a, e - a);
            done[c].fetch_add(1, std::memory_order_release);
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < T; t++) th.emplace_back(work, t);
    int rc = 0;
    std::thread main_copy(work, 0);
    for (size_t c = 0; c < nch; c++) {
        while (done[c].load(std::memory_order_acquire) < T) std::this_thread::yield();
        const size_t len = std::min(kStageChunk, bytes - c * kStageChunk);
        const int b = (int)(c & 1);
        if (rc == 0 && (hipMemcpyAsync((char*)dst + c * kStageChunk, W.hpin + b * kStageChunk, len,
                                       hipMemcpyHostToDevice, st) != hipSuccess ||
                        hipEventRecord(W.dma[b], st) != hipSuccess))
            rc = -1;
        // chunk c + 2 reuses this buffer once its copy has left it
        if (c + 2 < nch) {
            if (rc == 0 && hipEventSynchronize(W.dma[b]) != hipSuccess) rc = -1;
            writable.store(c + 3, std::memory_order_release);
        }
    }
    main_copy.join();
    for (auto& x : th) x.join();
    return rc;
}

template <typename T>
bool grow(T*& p, size_t& cap, size_t n) {
    if (n <= cap) return true;
    psx::dfree(p);
    p = nullptr;
    cap = 0;
    const size_t nc = n + n / 4;
    if (psx::dmalloc(&p, nc * sizeof(T)) != hipSuccess) return false;
    cap = nc;
    return true;
}

}  // namespace

int configs_pass(CfgWork& W, const int16_t* rows, int64_t n_rows, int n_groups, int64_t r0, int64_t r1,
                 const CfgMaps& C, const CfgProb& P, Acc5* acc, SetRec* sacc, hipStream_t st, hipEvent_t k0,
                 hipEvent_t k1, CfgResult* out, const char** err) {
    *out = CfgResult{-1, 0, 0, 0, 0};
    auto bad = [&](const char* m) {
        *err = m;
        return -1;
    };
    if (n_rows == 0) return 0;
    const size_t nel = (size_t)n_rows * n_groups;
    const long nblk = (long)((n_rows + kRowsPerBlock - 1) / kRowsPerBlock);
    if (nblk > INT32_MAX / 2 || (r1 - r0) * PSX_KMAX >= (int64_t)INT32_MAX) return bad("configs file too large");
    if (!grow(W.rows, W.cap_rows, nel) || !grow(W.blk, W.cap_blk, 2 * (size_t)nblk) ||
        !grow(W.ptr, W.cap_ptr, (size_t)C.U + 1))
        return bad("out of device memory (configs rows)");
    if (!W.status && psx::dmalloc(&W.status, 5 * sizeof(unsigned long long)) != hipSuccess)
        return bad("out of device memory");
    if (!W.hstatus && psx::hmalloc(&W.hstatus, 5 * sizeof(unsigned long long)) != hipSuccess)
        return bad("out of pinned host memory");
    if (upload_rows(W, rows, nel * sizeof(int16_t), W.rows, st) ||
        hipMemsetAsync(W.status, 0xff, sizeof(unsigned long long), st) != hipSuccess ||
        hipMemsetAsync(W.status + 1, 0, 4 * sizeof(unsigned long long), st) != hipSuccess ||
        hipMemsetAsync(W.ptr, 0, ((size_t)C.U + 1) * sizeof(int), st) != hipSuccess)
        return bad("configs upload");
    const int lds = C.U <= kLdsHistMax ? 1 : 0;
    hipLaunchKernelGGL(k_cfg_count, dim3((unsigned)nblk), dim3(kRowsPerBlock), lds ? C.U * sizeof(int) : 0, st,
                       W.rows, (long)n_rows, n_groups, C, (long)r0, (long)r1, W.status, W.blk, (int)nblk, W.ptr, lds);
    hipLaunchKernelGGL(k_cfg_scan, dim3(1), dim3(1024), 0, st, W.blk, (int)nblk, W.ptr, C.U, W.status);
    if (hipGetLastError() != hipSuccess) return bad("configs count launch");
    if (hipMemcpyAsync(W.hstatus, W.status, 5 * sizeof(unsigned long long), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return bad("configs status");
    const unsigned long long f = W.hstatus[0];
    if (f != ~0ull) {  // the first failing row in row order (postcal.cpp:432-590 exits there)
        out->fail_row = (int64_t)(f >> 3);
        out->fail_code = (int)(f & 7);
        return 0;
    }
    out->nulls = (int64_t)W.hstatus[1];
    out->nsets = (int64_t)W.hstatus[2];
    out->nrec = (int64_t)W.hstatus[3];
    const size_t ns = (size_t)out->nsets, nr = (size_t)out->nrec;
    if (ns == 0) return 0;
    // level-1 shapes of the two folds and their partials buffer
    const int S = (int)std::min<unsigned long long>(kMaxSlices, std::max<unsigned long long>(1, (W.hstatus[4] + kSliceRecs - 1) / kSliceRecs));
    long chunk = kSetChunk;
    while ((long)((ns + chunk - 1) / chunk) > kMaxSetChunks) chunk *= 2;
    const int nchunk = (int)((ns + chunk - 1) / chunk);
    const size_t need = std::max((size_t)C.U * S * sizeof(Acc5), (size_t)nchunk * sizeof(SetRec));
    if (need > W.cap_parts) {
        psx::dfree(W.parts);
        W.parts = nullptr;
        W.cap_parts = 0;
        if (psx::dmalloc(&W.parts, need) != hipSuccess) return bad("out of device memory (configs folds)");
        W.cap_parts = need;
    }
    if (ns > W.cap_sets) {
        psx::dfree(W.srec);
        psx::dfree(W.rrec);
        psx::dfree(W.masks);
        W.srec = nullptr;
        W.rrec = nullptr;
        W.masks = nullptr;
        W.cap_sets = 0;
        const size_t c = ns + ns / 4;
        if (psx::dmalloc(&W.srec, c * sizeof(SetRec)) != hipSuccess || psx::dmalloc(&W.rrec, c * sizeof(CfgRow)) != hipSuccess ||
            psx::dmalloc(&W.masks, c * sizeof(int)) != hipSuccess)
            return bad("out of device memory (configs sets)");
        W.cap_sets = c;
    }
    if (nr > W.cap_rec) {  // keys and values, each sort input + output
        psx::dfree(W.keys);
        psx::dfree(W.vals);
        W.keys = nullptr;
        W.vals = nullptr;
        W.cap_rec = 0;
        const size_t c = nr + nr / 4;
        if (psx::dmalloc(&W.keys, 2 * c * sizeof(unsigned)) != hipSuccess ||
            psx::dmalloc(&W.vals, 2 * c * sizeof(int)) != hipSuccess)
            return bad("out of device memory (configs records)");
        W.cap_rec = c;
    }
    unsigned* keys_out = W.keys + W.cap_rec;
    int* vals_out = W.vals + W.cap_rec;
    int end_bit = 1;
    while ((1 << end_bit) < C.U) end_bit++;
    size_t tmp = 0;
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, W.keys, keys_out, W.vals, vals_out, (int)nr, 0, end_bit, st) !=
        hipSuccess)
        return bad("configs sort sizing");
    if (tmp > W.cap_sort) {
        psx::dfree(W.sort_tmp);
        W.sort_tmp = nullptr;
        W.cap_sort = 0;
        if (psx::dmalloc(&W.sort_tmp, tmp) != hipSuccess) return bad("out of device memory (configs sort)");
        W.cap_sort = tmp;
    }
    if (k0 && hipEventRecord(k0, st) != hipSuccess) return bad("event");
    hipLaunchKernelGGL(k_cfg_eval, dim3((unsigned)nblk), dim3(kRowsPerBlock), 0, st, W.rows, n_groups, C, (long)r0,
                       (long)r1, P, W.blk, (int)nblk, W.srec, (CfgRow*)W.rrec, W.masks, W.keys, W.vals);
    if (k1 && hipEventRecord(k1, st) != hipSuccess) return bad("event");
    if (hipGetLastError() != hipSuccess) return bad("configs eval launch");
    size_t tmp2 = W.cap_sort;
    if (hipcub::DeviceRadixSort::SortPairs(W.sort_tmp, tmp2, W.keys, keys_out, W.vals, vals_out, (int)nr, 0, end_bit,
                                           st) != hipSuccess)
        return bad("configs sort");
    hipLaunchKernelGGL(k_cfg_merge, dim3((unsigned)C.U, (unsigned)S), dim3(256), 0, st, (const CfgRow*)W.rrec,
                       W.masks, W.ptr, vals_out, S, (Acc5*)W.parts);
    hipLaunchKernelGGL(k_cfg_merge2, dim3((unsigned)((C.U + 63) / 64)), dim3(64), 0, st, (const Acc5*)W.parts, S, C.U,
                       acc);
    if (hipGetLastError() != hipSuccess) return bad("configs merge launch");
    // the set records (the partials buffer is free again: same stream)
    hipLaunchKernelGGL(k_cfg_sets, dim3((unsigned)nchunk), dim3(256), 0, st, W.srec, (long)ns, chunk, (SetRec*)W.parts);
    if (hipGetLastError() != hipSuccess) return bad("configs set fold launch");
    if (launch_merge_sets((const SetRec*)W.parts, (long)nchunk, set_zero(), sacc, st)) return bad("configs set merge");
    return 0;
}

void configs_free(CfgWork& W) {
    psx::dfree(W.rows);
    psx::dfree(W.blk);
    psx::dfree(W.ptr);
    psx::dfree(W.status);
    psx::dfree(W.srec);
    psx::dfree(W.rrec);
    psx::dfree(W.masks);
    psx::dfree(W.keys);
    psx::dfree(W.vals);
    psx::dfree(W.sort_tmp);
    psx::dfree(W.parts);
    if (W.hstatus) psx::hfree(W.hstatus);
    for (int b = 0; b < 2; b++)
        if (W.dma[b]) hipEventDestroy(W.dma[b]);
    if (W.hpin) psx::hfree(W.hpin);
    W = CfgWork{};
}

// load this translation unit's device code on the current device (psx_warmup)
int warm_module_configs() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, (const void*)k_cfg_scan) == hipSuccess ? 0 : -1;
}

}  // namespace psx
