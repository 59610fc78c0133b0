// psx_configs.h — the -b configs-file enumerator on the device
// (computeTotalLikelihoodGivenConfigs, postcal.cpp:400-714).
#ifndef PSX_CONFIGS_H
#define PSX_CONFIGS_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "psx_math.h"

namespace psx {

// Index maps of the row walk (model.h:134-139): l2u[off_s + j] = union position
// of study s's local SNP j (off_0 = 0, off_1 = m0); u2l[s * U + u] = local
// index or -1.
struct CfgMaps {
    const int* l2u;
    const int* u2l;
    int U, N, m0, m1;
};

// What the row evaluation reads of the device problem (psx_engine's DevProb).
struct CfgProb {
    const double* G[2];
    const double* Ad[2];
    const double* y[2];
    const unsigned char* pres;
    int ldg;
    double dval[2];
    int Ck[PSX_KMAX + 1];
    double pit[PSX_KMAX + 1][PSX_KMAX + 1];
    double prior[PSX_KMAX + 1][PSX_KMAX + 1];
};

// Device workspace of the pass, grown on demand and kept by the engine.
struct CfgWork {
    int16_t* rows = nullptr;
    size_t cap_rows = 0;           // int16 elements
    int* blk = nullptr;            // per row block: counts (sets, records), then their offsets
    size_t cap_blk = 0;            // ints
    int* ptr = nullptr;            // per union SNP: record counts, then the CSR row pointer (U + 1)
    size_t cap_ptr = 0;
    unsigned long long* status = nullptr;  // [0] first failing row << 3 | code, [1] nulls, [2] sets, [3] records,
                                           // [4] most records of one union SNP
    SetRec* srec = nullptr;        // per evaluated row: scalars
    void* rrec = nullptr;          // per evaluated row: weights of its one assignment
    int* masks = nullptr;          // per evaluated row: c0 | c1 << 8
    size_t cap_sets = 0;
    unsigned* keys = nullptr;      // per record: union SNP (sort key in / out)
    int* vals = nullptr;           // per record: set * PSX_KMAX + member (in / out)
    size_t cap_rec = 0;
    void* sort_tmp = nullptr;
    size_t cap_sort = 0;
    void* parts = nullptr;         // two-level folds: per (union SNP, slice) Acc5, then per block SetRec
    size_t cap_parts = 0;          // bytes
    unsigned long long* hstatus = nullptr;  // pinned host copy of status
    char* hpin = nullptr;                   // pinned staging of the upload: two chunks
    hipEvent_t dma[2] = {nullptr, nullptr};  // the chunks' copies out of hpin
};

struct CfgResult {
    int64_t fail_row;   // first failing row (all rows checked), -1 if none
    int fail_code;      // 1: index out of range, 2: more than PSX_KMAX union SNPs, 3: walk failed
    int64_t nulls;      // null rows of this rank's slice
    int64_t nsets;      // evaluated rows of this rank's slice
    int64_t nrec;
};

// Upload rows [0, n_rows) (host, the caller's buffer), validate every row,
// evaluate the rows of [r0, r1) and fold them into the accumulators (members
// into acc, scalars into sacc) in row order.  Returns 0, or -1 with err set.
// On a failing row the accumulators are untouched and out->fail_row >= 0.
int configs_pass(CfgWork& W, const int16_t* rows, int64_t n_rows, int n_groups, int64_t r0, int64_t r1,
                 const CfgMaps& C, const CfgProb& P, Acc5* acc, SetRec* sacc, hipStream_t st, hipEvent_t k0,
                 hipEvent_t k1, CfgResult* out, const char** err);
void configs_free(CfgWork& W);
int warm_module_configs();  // load this unit's device code (psx_warmup)

}  // namespace psx
#endif
