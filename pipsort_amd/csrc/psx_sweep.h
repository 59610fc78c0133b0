// psx_sweep.h — tiled exhaustive sweep over union subsets of size k in {2, 3}
// (the dominant levels of PostCal::computeTotalLikelihood, postcal.cpp:716-1092).
#ifndef PSX_SWEEP_H
#define PSX_SWEEP_H

// waves per SIMD the k = 3 sweep is compiled for (VGPR budget 512 / waves, LDS
// 160 KiB / (4 x waves) per one-wave block); the unit planner sizes its a-chunks
// for the same number of wave slots
#ifndef PSX_K3_WAVES
#define PSX_K3_WAVES 2
#endif
// dispatch rounds of the k = 3 sweep's wave slots per shard the a-chunk is
// sized for (a build-time A/B knob, tools/build_variant.sh; the product build
// uses the default)
#ifndef PSX_K3_ROUNDS
#define PSX_K3_ROUNDS 2.0
#endif

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <future>
#include <map>
#include <memory>
#include <string>
#include <tuple>
#include <vector>

#include "psx_math.h"

namespace psx {

struct SweepArgs {
    const double* G0;
    const double* G1;
    const double* Ad0;
    const double* Ad1;
    const double* y0;
    const double* y1;
    const unsigned char* pres;
    double d0, d1;
    const int* Ck;      // host array [PSX_KMAX+1]
    const double* pit;  // host array [PSX_KMAX+1][pit_ld]
    int pit_ld;
};

struct SweepStats {           // indexed by causal-set level k
    double kernel_ms[8];      // device time of the sweep kernel
    int launches[8];
    uint64_t union_sets[8];   // union subsets covered
    double alg_bytes[8];      // 8 * sum_s (|C_s|^2 + |C_s|) over configurations
    double flops[8];          // FP64 operation estimate
    double merge_ms;          // device time of the record merges (all levels)
    int exact_reruns;         // levels re-swept with the exact notSharedLL variant
};

// Record buffer sets of the pipelined asynchronous passes: sweep i reuses the
// buffers of pass i - kRecBufs, so the host may run kRecBufs - 1 passes ahead of
// the device before it blocks.  Each set is one plan's records (~90 MB at
// M = 1000, c = 3).  12 sets (a longer lead against host stalls) measured 3 %
// slower at world 8 than 3 on the same box (profiles/archive/r02zf_ab_*): 3.
#ifndef PSX_REC_BUFS
#define PSX_REC_BUFS 3
#endif
constexpr int kRecBufs = PSX_REC_BUFS;

// One decomposition of a level into wave units, with its record CSR.
struct SweepPlan {
    int k = 0, U = 0, ldg = 0, rank = 0, world = 1, ca = 0;
    int n_units = 0, rec_stride = 0, pad = 0;  // pad: record keys in v = u + pad space (variant 1)
    uint64_t union_sets = 0;
    double alg_bytes = 0, flops = 0;
    int4* d_units = nullptr;     // {a0, a1, B, T}
    Acc5* d_rec = nullptr;       // records, unit-major: slot i of unit u at u * rec_stride + i
    Acc5* d_rec_alt[kRecBufs - 1] = {};  // more record buffers (pipelined asynchronous passes)
    size_t rec_len = 0;          // records per buffer
    SetRec* d_srec = nullptr;    // [n_units]
    int* d_csr = nullptr;        // pos[rec_len], dptr[U+1], gidx[rec_len] (psx_plan.hip)
    const int* d_pos = nullptr;  // record slot -> buffer position, -1: no SNP (inside d_csr)
    const int* d_dptr = nullptr; // [U+1] per-SNP runs of CSR positions (inside d_csr)
    const int* d_gidx = nullptr; // CSR position -> record slot (records are unit-major; the merges gather)
    int variant = 0;             // 1: the k = 3 fast kernel's decomposition
    double fused_bytes = 0, fused_flops = 0;  // in-launch level-2 work of the last launch
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};  // kernel start/end, merges end
    bool ran = false;
    // the unit list on the host until upload_plan (plans built ahead on a host thread)
    std::vector<int4> h_units;
    bool uploaded = false;
    bool csr_pos = false;        // records at their CSR positions (gidx the identity): records_at_csr_positions
};

// Arguments of the k = 3 fast kernel (psx_sweep3.hip).  Sweep indices live in
// the padded space v = u + pad, pad = ldg - U (the partial block is block 0).
struct Sweep3Args {
    const double* G[2];        // Sigma~_s in union coordinates u, [ldg][ldg]
    const double* Ad[2];       // diag(A_s) = 1/d_s + diag(Sigma~_s), by u
    const double* ys[2];       // y_s * sqrt(log2(e) / 2), by u
    const double* skewT[2];    // skewed Sigma~ tiles in v space, tile(K, C), K <= C
    const double2* g01;        // skewT of both studies interleaved (one 16-byte load per step)
    const double2* mu01;       // {b, c} subset weights mu per [tile][step][lane], both studies (a-independent)
    const int2* bcn;           // their base-2 exponents, both studies
    const double2* bcsm;       // per [tile][lane]: sum over the tile's 64 b of the {b, c} weights, both
    const int2* bcsn;          //   studies, as 2^bcsn * bcsm (the off-diagonal walk's closed-form sums)
    const double2* bccm;       // per [tile][b slot]: sum over the tile's 64 c of the {b, c} weights
    const int2* bccn;
    const double* muS[2];      // singleton weights {c}, by u
    const int* nS[2];
    const unsigned char* pres; // bit s: SNP present in study s, by u
    const double* tab;         // 2^(i/256), i < 256
    double rsd[2];             // d_s^{-1/2}
    double rho, pit0;          // pit[nsh] = pit0 * rho^nsh (prior per member is multiplicative)
    int U, ldg, pad, Ck;
    unsigned long long* trace = nullptr;  // diagnostics (PSX_UNIT_TRACE): per unit {start, end, hw id, unit}
    int* redo_count = nullptr;            // units redone by the robust variant (cumulative)
    unsigned long long* tstamp = nullptr; // single passes: block 0 stores its start clock (wall_clock64) here
};
// most a per k = 3 unit (plan_units3c): the fast kernel stages the unit's
// per-a scalars in LDS
constexpr int kMaxChunkA3 = 4;
// words per unit of the PSX_UNIT_TRACE dump (tools/unit_trace.py)
constexpr int kTraceWords = 16;
struct Level2Blocks;  // psx_sweep_dev.h
int launch_sweep3(bool allpres, const Sweep3Args& A, int n_units, const int4* units, Acc5* rec, SetRec* srec,
                  int rec_stride, int* flag, const int* pos, hipStream_t st, const Level2Blocks* l2, hipEvent_t ev0 = nullptr,
                  hipEvent_t ev1 = nullptr);
int launch_scale_y(const double* y, int n, double* ys, hipStream_t st);
int launch_build_skewT(const double* G, int ldg, int pad, double* skew, hipStream_t st);
// {b, c} subset weights of every skewT entry (the a-independent half of a k = 3
// step), computed once per locus with the sweep kernel's own arithmetic
constexpr int kTileRowPad = 4;  // zero rows after the last tile of mu01 / bcn / g01
int launch_build_bc3(const Sweep3Args& A, int ntile, double2* mu01, int2* n, hipStream_t st);
// per tile and lane c: the sum over the tile's 64 b of the {b, c} weights
int launch_bc3_rowsum(int ntile, const double2* mu01, const int2* n, double2* sm, int2* sn, hipStream_t st);
// per tile and b slot: the sum over the tile's 64 c of the {b, c} weights
int launch_bc3_colsum(int ntile, const double2* mu01, const int2* n, double2* sm, int2* sn, hipStream_t st);
// out[i] = (a[i], b[i])
int launch_interleave2(const double* a, const double* b, size_t n, double2* out, hipStream_t st);

// a level's plan built ahead on a host thread (plan_prefetch)
struct PlanJob {
    std::future<int> done;  // 0: P holds the plan (records not yet allocated)
    SweepPlan P;
    std::string err;
};

// device scratch of plan_csr_device (keys, sorted keys, slots, radix-sort temp)
struct PlanScratch {
    void* p = nullptr;
    size_t bytes = 0;
};
// a plan's record CSR (pos | dptr | gidx) built on the device from its units
// plan records written at their CSR positions (world > 1) or unit-major (world 1); PSX_REC_CSR forces
bool records_at_csr_positions(int world);
int plan_csr_device(const int4* d_units, int n_units, int rec_stride, int k, int variant, int pad, int U, int* d_pos,
                    int* d_dptr, int* d_gidx, PlanScratch& scratch, hipStream_t st, bool csr_pos);
// the CSR of flat records keyed by SNP (-1: none): dptr[U + 1], gidx[n]
int csr_from_keys_device(const int* d_keys, long n, int U, int* d_dptr, int* d_gidx, PlanScratch& scratch,
                         hipStream_t st);
// Merge n generic set evaluations ([set][stride] members, -1 after them;
// member records rec[set * stride + j], set records srec[set]) into acc / sacc
// in a fixed order (psx_plan.hip); scratch of batch_merge_bytes(); -1 when U
// or stride is outside the kernels' range (use the CSR merge).  bad (device,
// optional): the merges add nothing when *bad == badv (an invalid batch).
// tstamp (optional, host or device): the first merge's block 0 stores its start
// clock there.
size_t batch_merge_bytes(long nsets, int stride, int U);
int batch_merge_chunks(long nsets, int stride);
int batch_merge_sets_per_chunk(int stride);  // whole sets per merge chunk
int launch_merge_batch(const int* d_sets, int stride, long nsets, int U, const Acc5* rec, const SetRec* srec,
                       void* scratch, Acc5* acc, SetRec* sacc, hipStream_t st,
                       const unsigned long long* bad = nullptr, unsigned long long badv = 0,
                       unsigned long long* tstamp = nullptr);
// GPU self-check: the device CSR of a plan equals the host restatement's
int plan_csr_selftest(int U, const unsigned char* pres, int k, int rank, int world, int variant, long* mismatches,
                      long* records);
int warm_module_plan();

struct SweepPlanCache {
    std::map<std::tuple<int, int, int, int, int>, SweepPlan> plans;  // (k, U, rank, world, variant)
    std::map<std::tuple<int, int, int, int, int>, std::unique_ptr<PlanJob>> pending;  // plan_prefetch
    std::vector<unsigned char> pres_host;    // presence bits by u (ldg), set by the engine at create
    PlanScratch csr_scratch;
    double* d_skew[2] = {nullptr, nullptr};  // skewed Sigma~ tiles (B <= T), k = 2 and exact k = 3
    double* d_skewT[2] = {nullptr, nullptr}; // lane-owns-c tiles in v space (k = 3 fast kernel)
    double2* d_g01 = nullptr;                // skewT of both studies interleaved (k = 3 fast kernel)
    double2* d_mu01 = nullptr;               // {b, c} weights per skewT entry, both studies
    int2* d_bcn = nullptr;
    double2* d_bcsm = nullptr;               // row sums of the {b, c} weights per tile and lane
    int2* d_bcsn = nullptr;
    double2* d_bccm = nullptr;               // column sums of the {b, c} weights per tile and b slot
    int2* d_bccn = nullptr;
    double* d_muS[2] = {nullptr, nullptr};   // singleton subset weights
    int* d_nS[2] = {nullptr, nullptr};
    double* d_ys[2] = {nullptr, nullptr};    // scaled y (k = 3 fast kernel)
    double* d_tab = nullptr;                 // 2^(i/256) table
    bool allpres = false;                    // every union SNP is in both studies
    int skew_ldg = 0;
    const double* skew_src[2] = {nullptr, nullptr};
    int* d_redo = nullptr;  // k = 3 units redone by the robust variant since creation
    int* d_flag = nullptr;  // raised when a set needs the EXACT notSharedLL variant
    bool own_flag = true;   // false: d_flag lives in the engine's status block
    unsigned long long* stamp = nullptr;  // the next k = 3 fast launch's start clock (null: none)
};

bool sweep_supports(int k, int U);
struct PlanUnit { int a0, a1, B, T; double work; int j0 = 0, j1 = 64; };
int plan_units(int k, int U, int ldg, int rank, int world, const unsigned char* pres_host,
               std::vector<PlanUnit>& mine, int& ca, double& sets, double& configs, double& bytes);
// plan-shaping knobs of the k = 3 decomposition (environment, read once)
struct K3Knobs { double rounds, maskw, diagw, unitw, tail_frac, tail2; int diag_div; };
const K3Knobs& k3_knobs();
// hash of the knobs and the compiled plan constants (PlanTag: ranks must agree)
uint64_t plan_knobs_hash();
// k = 3 fast-kernel decomposition: units (a0, a1, K, C) in v space
int plan_units3c(int U, int ldg, int rank, int world, const unsigned char* pres_host, std::vector<PlanUnit>& mine,
                 int& ca, double& sets, double& configs, double& bytes);
// Build level k's plan for (rank, world) on a host thread (device `device`):
// the unit decomposition, counts and record CSR, uploaded; sweep_prepare takes
// it (and allocates its records) instead of building it.  Needs pres_host.
// host-only diagnostics: build level k's plan (all SNPs in both studies) without the device
int plan_host_ms(int U, int k, int rank, int world, double* ms, int* n_units, long* n_records);
void plan_prefetch(SweepPlanCache& cache, int device, int k, int U, int ldg, int rank, int world, bool exact);
int sweep_begin(SweepPlanCache& cache, hipStream_t stream);   // zero the EXACT flag
int sweep_level(SweepPlanCache& cache, int k, int U, int ldg, int rank, int world, hipStream_t stream,
                const SweepArgs& a, Acc5* acc, SetRec* sacc, bool exact);   // async enqueue
// Pieces of the fused exhaustive pass: the level's plan (built on first use)
// and its kernel alone (set records into srec_out, or the plan's own buffer).
// With l2 (a level-2 plan) the level-2 units run in the same launch as the
// k = 3 fast kernel (set records into srec2), else right after it.
int sweep_prepare(SweepPlanCache& cache, int k, int U, int ldg, int rank, int world, hipStream_t stream,
                  const SweepArgs& a, bool exact, SweepPlan** out);
// parity selects the record buffer (0: d_rec, 1 .. kRecBufs - 1: d_rec_alt,
// allocated on first use); flag overrides the cache's EXACT flag word; timed = false skips the
// plan's own timing events (asynchronous passes time the kernel themselves).
// ev0 / ev1 (optional): start / stop events recorded by the top-level kernel's
// own dispatch (hipExtLaunchKernel), used by pipelined asynchronous passes.
int sweep_kernel(SweepPlanCache& cache, SweepPlan& plan, hipStream_t stream, const SweepArgs& a, SetRec* srec_out,
                 bool exact, SweepPlan* l2, SetRec* srec2, int parity = 0, int* flag = nullptr, bool timed = true,
                 hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
// the record buffer of a parity (allocating the second one on first use)
Acc5* plan_records(SweepPlan& plan, int parity);
int sweep_flag(SweepPlanCache& cache, int* flag);                          // after sync
int sweep_redo_count(SweepPlanCache& cache, int* count);                   // after sync
int sweep_stats(SweepPlanCache& cache, int k, int U, int rank, int world, SweepStats* st);  // after sync
void sweep_free(SweepPlanCache& cache);
int launch_merge_members(const Acc5* rec, const int* ptr, const int* idx, const int* rows, int n_rows, Acc5* acc,
                         hipStream_t st);
// per-SNP folds of records through a dptr / gidx CSR (one block per SNP, empty runs return)
int launch_merge_dptr(const Acc5* rec, const int* dptr, const int* gidx, int U, Acc5* acc, hipStream_t st);
int launch_merge_sets(const SetRec* rec, long n, const SetRec& extra, SetRec* acc, hipStream_t st,
                      bool init = false, int* zero_flag = nullptr);
const char* sweep_error();

// device code of the sweep translation units, loaded ahead of first use (psx_warmup)
int warm_module_sweep();
int warm_module_sweep3();

}  // namespace psx
#endif
