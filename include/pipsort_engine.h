/*
 * pipsort_engine.h — C ABI of the MI355X posterior-calculation engine.
 *
 * Drop-in boundary for the reference's PostCal class (CAST-genomics/pipsort).
 * The reference has no FFI; its seam is the PostCal object that Model builds and
 * drives (model.h:265 constructs it, model.h:274 runs it, model.h:304 prints it).
 * Each entry point below names the reference interface it replaces.  Inputs are
 * exactly PostCal's constructor inputs (postcal.h:118); outputs are PostCal's
 * accumulator arrays in the same log-space convention (0 == "empty",
 * postcal.h:102-112) plus totalLikeLihoodLOG.
 *
 * Plain C types only: host pointers and sizes; no torch/HIP types.  Every
 * function returns 0 on success and a negative PSX_E* code on failure (message
 * via psx_last_error()).  The engine is single-host-thread per handle, not
 * reentrant per handle; one handle drives one GPU.  There is no CPU fallback:
 * psx_create fails with PSX_ENODEV when no HIP device is present.
 */
#ifndef PIPSORT_ENGINE_H
#define PIPSORT_ENGINE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSX_ABI_VERSION 4

#define PSX_OK 0
#define PSX_EINVAL (-1)    /* bad argument / unsupported problem shape        */
#define PSX_ENODEV (-2)    /* no HIP device (no silent CPU fallback)          */
#define PSX_EHIP (-3)      /* HIP runtime error                               */
#define PSX_ESINGULAR (-4) /* postcal.cpp:291-294 "matrix is singular" (ref exits 0) */
#define PSX_EORDER (-5)    /* postcal.cpp:587-590 "This did not work as expected" */
#define PSX_ERANGE (-6)    /* sweep too large to index / unsupported c        */
#define PSX_EEXCHANGE (-7) /* the caller's all-gather callback failed            */

typedef struct psx_engine psx_engine;

/* PostCal constructor inputs (postcal.h:118; built by Model at model.h:213-265). */
typedef struct {
    int32_t n_studies;              /* num_of_studies; must be 2 (postcal.cpp:20-23, model.h:125) */
    const int32_t *m;               /* [n_studies] num_snps_all                                  */
    const double *B;                /* BIG_SIGMA diagonal blocks B_s, column-major M_s x M_s,
                                       concatenated (model.h:239,262)                            */
    const double *s_prime;          /* [N = sum m] S_LONG_VEC after the low-rank transform       */
    int32_t n_union;                /* unionSnpCount = rows of the snp map                       */
    const int32_t *union_to_local;  /* [n_studies][n_union] idx_to_snp_map, -1 = absent          */
    int32_t max_causal;             /* MAX_causal (-c)                                           */
    const int32_t *sample_sizes;    /* [n_studies] (-n)                                          */
    double sharing_param;           /* -p */
    double gamma;                   /* -g */
    double t_squared;               /* -t */
    double s_squared;               /* -s */
} psx_problem;

/* PostCal accumulators (postcal.h:62-78), caller-owned host arrays. */
typedef struct {
    double *post;         /* [N]          postValues                    */
    double *no_causal;    /* [n_studies]  noCausal                      */
    double *shared;       /* [n_union]    sharedPips                    */
    double *shared_ll;    /* [n_union]    sharedLL                      */
    double *notshared_ll; /* [n_union]    notSharedLL                   */
    double total;         /* totalLikeLihoodLOG (sum over all configs)  */
    uint64_t n_configs;   /* configurations evaluated (incl. null)      */
} psx_accum;

typedef struct {
    double sweep_ms;        /* wall time of the last psx_run_* (HIP events, engine stream) */
    double kernel_ms;       /* summed device time of the dominant sweep kernel             */
    int32_t kernel_launches;/* launches of that kernel in the last run                     */
    double merge_ms;        /* device time of the record-merge kernels                     */
    uint64_t configs;       /* configurations evaluated by this handle in the last run     */
    uint64_t union_sets;    /* union subsets evaluated by the dominant kernel              */
    double alg_bytes;       /* algorithmic bytes of the dominant kernel      */
    double flops;           /* FP64 operation estimate of the dominant kernel              */
    int32_t exact_rerun;    /* nonzero if the sweep was redone with the exact notSharedLL
                               variant; the checks that fired: bit 0 a set's / an a or c
                               slot's notSharedLL group (k = 3) or the k = 2 window, bit 1
                               an off-diagonal unit's b-slot notSharedLL total (k = 3) */
    int32_t robust_units;   /* k = 3 units redone by the robust variant (cumulative since create) */
    double span_ms;         /* asynchronous passes: first sweep's start to the last one's end,
                               per pass (consecutive sweeps may overlap: kernel_ms double-counts) */
    double prepare_ms;      /* psx_run_exhaustive: host wall of the plan / layout preparation
                               (first pass of a handle: k = 3 layouts, unit plans, CSR upload) */
    double run_ms;          /* psx_run_exhaustive: host wall of the whole call                */
} psx_timing;

int32_t psx_abi_version(void);
const char *psx_last_error(void);

/* CUs reserved for the merges / exchange beside overlapped asynchronous passes,
 * decided at the handle's first psx_run_exhaustive_async (-1 before it): one
 * XCD's CUs at world >= 8, 0 below; the environment variable PSX_OVERLAP = n
 * overrides.  (No reference counterpart: reported by bench.py.) */
int32_t psx_overlap_cus(const psx_engine *e);

/* Number of HIP devices visible (0 on a host without a GPU; never initialises a context). */
int psx_device_count(int *count);
/* The engine keeps freed device and pinned host blocks in a caching pool (up to
 * 4 GiB per device, 1 GiB pinned) for the next handle.  psx_pool_trim gives the
 * cached (free) blocks back to the HIP runtime — e.g. before a co-resident
 * framework needs the memory; blocks in use are untouched.
 * psx_pool_cached_bytes: bytes cached now. */
int psx_pool_trim(void);
int64_t psx_pool_cached_bytes(void);

/* Optional (no reference counterpart): bring up the HIP runtime and context of
 * `device` and load the engine's device code, so the first psx_create* does not
 * pay for it.  Thread-safe; the drop-in CLI calls it on a second thread while
 * it parses the LD / z files (model.h:86-144), overlapping the two. */
int psx_warmup(int device);
/* The same, loading only the device code a run of this shape uses: the k = 3
 * sweep's only for max_causal >= 3, the configs-file path's only when
 * configs_file != 0 (psx_warmup(d) = psx_warmup_for(d, 3, 0)).  With PSX_TIMING
 * set it prints its phases (context, each code object) on stderr. */
int psx_warmup_for(int device, int32_t max_causal, int32_t configs_file);
/* Optional (no reference counterpart), for one-locus processes: on != 0 makes
 * every handle created afterwards, and the warm-up, share one stream — one
 * hardware queue — per device.  Every queue a process holds costs ~10-13 ms
 * when the process exits; the drop-in CLI turns it on before anything else.
 * Pipelined and multi-rank passes lose their stream priorities and overlap
 * under it; results are the same.  Call before the first psx_warmup* /
 * psx_create*. */
int psx_single_queue(int32_t on);

/* PostCal::PostCal (postcal.h:118-195).  Copies the problem to device `device`,
 * forms Sigma~_s = B_s^T B_s, y_s = B_s^T S'_s and ||S'||^2 on the GPU. */
int psx_create(const psx_problem *prob, int device, psx_engine **out);
void psx_destroy(psx_engine *e);

/* Model setup + PostCal::PostCal on the GPU (model.h:171-265, util.cpp:195-263).
 * Takes what Model reads from its input files instead of the low-rank B/S':
 * per-study LD matrices (row-major M_s x M_s as util.cpp:86-96 parses them)
 * and z-scores.  The PSD shift (util.cpp:195-226) runs as a device LU whose
 * determinant is bit-identical to the reference elimination; when Sigma'_s is
 * positive definite, Sigma~_s = B_s^T B_s = Sigma'_s, y_s = B_s^T S'_s = z_s and
 * ||S'_s||^2 = z_s^T Sigma'_s^-1 z_s exactly, so no eigendecomposition is done
 * (otherwise the reference's eigen route runs for that study, on the GPU too:
 * rocSOLVER dsyevd, then B and S' from (Q, W, z); PSX_HOST_EIGEN=1 keeps a host
 * restatement). */
typedef struct {
    int32_t n_studies;              /* must be 2                                         */
    const int32_t *m;               /* [n_studies] M_s                                   */
    const double *ld;               /* LD_s, row-major M_s x M_s, concatenated           */
    const double *z;                /* [N] z-scores, study-major (S_LONG_VEC before the transform) */
    int32_t n_union;
    const int32_t *union_to_local;  /* [n_studies][n_union], -1 = absent                 */
    int32_t max_causal;
    const int32_t *sample_sizes;
    double sharing_param, gamma, t_squared, s_squared;
} psx_ld_problem;

typedef struct {
    double psd_added[2];       /* diagonal shift per study (util.cpp:195-226)            */
    int32_t psd_iterations[2]; /* LU determinants evaluated per study                    */
    int32_t eigen_route[2];    /* 1 if Sigma'_s was not positive definite (host eigen)   */
    double min_pivot_ratio[2]; /* smallest L D L^T pivot / largest |diagonal|            */
    double setup_ms;           /* wall time of the whole setup + create                  */
    double spsq[2];            /* ||S'_s||^2 = z~^T D^-1 z~ (0 on the eigen route)       */
    /* phases of setup_ms (wall, ms): device allocations, the two studies (run
     * concurrently, one host thread and stream each), accumulators + plan tag */
    double alloc_ms, studies_ms, tail_ms;
    /* per study: LD upload (H2D), PSD shift loop (LU determinants), step 2 +
     * readback, and (the rest of studies_ms) the union-coordinate layouts */
    double study_upload_ms[2], study_psd_ms[2], study_finish_ms[2];
} psx_setup_info;

int psx_create_from_ld(const psx_ld_problem *prob, int device, psx_engine **out, psx_setup_info *info);

/* The PSD shift alone on the GPU (util.cpp:195-226): same contract as the host
 * psx_psd_shift (pipsort_model.h), for parity tests and the CLI. */
int psx_psd_shift_gpu(double *sigma, int32_t m, double *added, int device);
/* One GSL-order partial-pivot LU determinant on the GPU (a row-major m x m, not
 * modified): bit-identical to the host psx_lu_det (pipsort_model.h). */
int psx_lu_det_gpu(const double *a, int32_t m, int device, double *det);
/* The setup's swap-free elimination (util.cpp:214-215's LU when no row swap
 * is needed; the forward solve of z rides along, as the setup's step 2 uses
 * it) on the GPU: a row-major m x m (not modified), z m entries or NULL.
 * pivots <- U_ii (m), z_out <- L^-1 z (m, when z), *swap_needed <- 1 when
 * check != 0 and GSL's pivot search would swap some row (pivots are then
 * meaningless).  Bit-identical to the per-column elimination; for parity
 * tests of the tiled kernels. */
int psx_elim_gpu(const double *a, int32_t m, const double *z, int32_t check, double *pivots, double *z_out,
                 int32_t *swap_needed, int device);

/* Multi-GPU sharding of the exhaustive sweep (one process per GPU): this handle
 * evaluates shard `rank` of `world` equal slices of every causal-set level; the
 * null configuration belongs to rank 0.  Default (0, 1). */
int psx_set_shard(psx_engine *e, int rank, int world);
/* The shard plan's hash (locus shape, c, world and the plan knobs PSX_K3_*):
 * every rank of one job must report the same value.  Each partial image
 * carries it with the image's rank and world; psx_merge_partials /
 * psx_fold_partials_host refuse images that are not shards 0..count-1 of one
 * plan (an error from the merge, or from psx_sync after an enqueued merge). */
int psx_plan_hash(psx_engine *e, uint64_t *hash);

/* PostCal::computeTotalLikelihood (postcal.cpp:716-1092): exhaustive sweep over
 * all union subsets of size <= max_causal and all per-study assignments passing
 * checkOR (postcal.cpp:1111-1126).  Resets and fills the accumulators. */
int psx_run_exhaustive(psx_engine *e);

/* Asynchronous exhaustive pass: enqueue one pass on the engine stream and
 * return at once (no host synchronisation), so back-to-back passes and the
 * multi-GPU exchange (psx_export_partials / collective / psx_merge_partials on
 * the same stream) pipeline on the device.  The fast kernel's EXACT flag is
 * collected in a sticky device word (and OR-ed across ranks by
 * psx_merge_partials); psx_sync waits for the stream and reports it.  Results
 * are valid only when psx_sync returns *exact_needed == 0; otherwise redo the
 * pass with psx_run_exhaustive (which reruns the exact variant where needed)
 * and repeat the exchange.  Falls back to psx_run_exhaustive for problems the
 * fused pass does not cover (c not in {2, 3}). */
int psx_run_exhaustive_async(psx_engine *e);
/* Wait for all work enqueued on the engine stream; *exact_needed = sticky EXACT
 * flag since the last psx_sync (cleared).  Timing of the asynchronous passes
 * since the last sync: kernel_ms summed over kernel_launches passes. */
int psx_sync(psx_engine *e, int32_t *exact_needed);

/* PostCal::computeTotalLikelihoodGivenConfigs (postcal.cpp:400-714): rows of
 * int16 global SNP indices (-1 = none), [n_rows][n_groups] (the -b file). */
int psx_run_configs(psx_engine *e, const int16_t *rows, int64_t n_rows, int32_t n_groups);

/* PostCal::sss_computeTotalLikelihood (sss_postcal.cpp:102-380): stochastic
 * shotgun search, host random walk (mt19937(12345)) + GPU neighbour batches. */
int psx_run_sss(psx_engine *e, int32_t *iterations_out);

/* All-gather callback of the sharded SSS walk: gather `bytes` host bytes from
 * every rank into recv (world * bytes, rank order).  Returns 0 on success.  The
 * caller binds it to its collective (torch.distributed / RCCL, MPI, ...). */
typedef int (*psx_allgather_fn)(void *ctx, const void *send, void *recv, int64_t bytes);

/* sss_computeTotalLikelihood (sss_postcal.cpp:102-380) across the ranks of
 * psx_set_shard (the reference runs it on one host, OpenMP inside).  Every
 * rank runs the same walk (same neighbourhoods, hash map and mt19937 draws);
 * each evaluates and accumulates a contiguous slice of every iteration's batch
 * (the null configuration on rank 0), and one all-gather per iteration shares
 * the slices' scores and the ranks' running normalisers (the :265-270 stop
 * test).  The accumulators are then merged like a sharded exhaustive sweep
 * (psx_export_partials / all-gather / psx_merge_partials).  With world 1 it
 * is psx_run_sss. */
int psx_run_sss_sharded(psx_engine *e, psx_allgather_fn allgather, void *ctx, int32_t *iterations_out);
/* The same walk with the per-iteration exchange kept on the device: the
 * callback gets DEVICE pointers (send: `bytes`; recv: world x `bytes`, rank
 * order) and the engine's stream (a hipStream_t), and enqueues the all-gather
 * on that stream — e.g. one RCCL all-gather — returning at once (0 = enqueued).
 * Each iteration then runs pack -> all-gather -> unpack -> insert on the stream
 * with one host synchronisation (no score copies through host memory). */
typedef int (*psx_allgather_dev_fn)(void *ctx, const void *device_send, void *device_recv, int64_t bytes,
                                    void *stream);
int psx_run_sss_sharded_dev(psx_engine *e, psx_allgather_dev_fn allgather, void *ctx, int32_t *iterations_out);

/* PostCal::expand_and_compute_lkl (sss_postcal.cpp:447-685), batched: evaluate
 * n_sets union sets (ascending union indices, -1 padded to `stride`), return the
 * SSS score (pattern L with largest |L|, sss_postcal.cpp:624-626) per set and,
 * if accumulate != 0, add every pattern into the accumulators.  Padding may sit
 * anywhere in a row; an all -1 row is the null configuration.  psx_get_timing
 * then reports the batch's evaluation kernel (kernel_ms, union_sets). */
int psx_eval_union_batch(psx_engine *e, const int32_t *sets, int32_t stride, int32_t n_sets,
                         int accumulate, double *score_out);

/* Zero the accumulators (PostCal constructor state, postcal.h:129-160). */
int psx_reset(psx_engine *e);

/* Read PostCal's accumulators (postValues, noCausal, sharedPips, sharedLL,
 * notSharedLL, totalLikeLihoodLOG) in the reference's log-space convention. */
int psx_get_accum(psx_engine *e, psx_accum *out);

/* Multi-process reduction of the accumulators (the single exchange step of the
 * sharded sweep).  Partials are opaque device bytes: export this handle's
 * partial into a caller device buffer of psx_partials_bytes() bytes, gather
 * them from all ranks (e.g. one RCCL all-gather), then merge `count`
 * concatenated partials (rank order) into this handle's accumulators. */
int64_t psx_partials_bytes(psx_engine *e);
/* Enqueue on a caller stream (a hipStream_t, e.g. the framework's current
 * stream) instead of the handle's own; NULL restores the own stream.  On a
 * caller stream psx_export_partials / psx_merge_partials only enqueue (the
 * caller orders them against its collective); psx_run_* still return with the
 * sweep complete. */
int psx_set_stream(psx_engine *e, void *stream);
int psx_export_partials(psx_engine *e, void *device_dst);
/* The handle's own partial image in device memory (psx_partials_bytes() bytes,
 * the psx_export_partials layout): a collective may read it in place instead of
 * an exported copy (one launch less per exchange).  Valid until the next pass,
 * merge or reset on the handle enqueues a write to it; read-only to the caller. */
int psx_partials_device_ptr(psx_engine *e, void **device_ptr);
int psx_merge_partials(psx_engine *e, const void *device_src, int32_t count);

/* Host-only (no GPU needed): fold `count` partial images of `image_bytes`
 * bytes each (psx_export_partials layout, rank order) into one image at dst —
 * the same fold psx_merge_partials runs on the device, for partials gathered
 * through a host collective.  PSX_EINVAL when the images' plan tags are not
 * shards 0..count-1 of one plan. */
int psx_fold_partials_host(const void *src, int32_t count, int64_t image_bytes, void *dst);

/* Host-only: union subsets and configurations of causal-set level k (1..c)
 * that shard `rank` of `world` evaluates in psx_run_exhaustive. */
int psx_shard_stats(const psx_problem *prob, int32_t k, int32_t rank, int32_t world, uint64_t *union_sets,
                    double *configs);

/* Host-side diagnostics (no device): the host time of building level k's
 * (2 or 3) unit plan and record CSR for shard rank of world, every union SNP
 * in both studies; *n_units / *n_records the plan's size. */
int psx_plan_build_ms(int32_t n_union, int32_t k, int32_t rank, int32_t world, double *ms, int32_t *n_units,
                      int64_t *n_records);
/* GPU self-check of a sweep plan's record CSR (built on the device, hipcub
 * radix sort) against the host restatement: level k, shard rank of world,
 * variant 1 = the k = 3 fast kernel's decomposition, presence bits per union
 * SNP (NULL: every SNP in both studies).  *mismatches = differing entries of
 * pos / dptr / gidx (0 expected), *records = records with a SNP. */
int psx_plan_csr_selftest(int32_t n_union, const uint8_t *presence, int32_t k, int32_t rank, int32_t world,
                          int32_t variant, int device, int64_t *mismatches, int64_t *records);
/* Host-side diagnostics (no kernel runs): the k = 3 fast sweep's work units of
 * shard `rank` of `world` for a union of n_union SNPs present in both studies,
 * in dispatch order, as int4 {a0, a1, K | j0 << 16, C | j1 << 16} (v space; a
 * diagonal tile's j counts half steps).  The a-chunk sizes are sized for
 * MI355X's 256 CUs as a fixed constant (not a device query), so every rank of a
 * sharded run, in any process, cuts the same unit list; every plan covers each
 * walk step once.  Writes at most `cap` units; returns the count (or a
 * negative error). */
int psx_plan_units_k3(int32_t n_union, int32_t rank, int32_t world, int32_t *units, int32_t cap);

/* ---- Several GPUs in one process --------------------------------------------
 * The reference runs its whole-node sweep in one process, 64 OpenMP threads
 * over the configurations (postcal.cpp:747-769).  A psx_multi holds one handle
 * per entry of devices[] (entries may repeat: several shards on one GPU); handle
 * i evaluates shard i of n (psx_set_shard), each driven by its own host thread,
 * and every run returns with the shards' accumulators folded on devices[0]
 * (peer copies of the partial images + psx_merge_partials, rank order, the
 * fold of the multi-process path).  Same semantics as the single-handle calls;
 * errors name the failing shard (psx_multi_last_error). */
typedef struct psx_multi psx_multi;
int psx_multi_create(const psx_problem *prob, const int32_t *devices, int32_t n, psx_multi **out);
int psx_multi_create_from_ld(const psx_ld_problem *prob, const int32_t *devices, int32_t n, psx_multi **out,
                             psx_setup_info *info);
int psx_multi_run_exhaustive(psx_multi *m);                                        /* computeTotalLikelihood */
int psx_multi_run_configs(psx_multi *m, const int16_t *rows, int64_t n_rows, int32_t n_groups);
int psx_multi_run_sss(psx_multi *m, int32_t *iterations_out);                     /* sharded SSS walk */
int psx_multi_get_accum(psx_multi *m, psx_accum *out);
int psx_multi_get_timing(psx_multi *m, psx_timing *t);
int32_t psx_multi_count(psx_multi *m);
const char *psx_multi_last_error(void);
void psx_multi_destroy(psx_multi *m);

/* Timing of the last psx_run_* on this handle. */
int psx_get_timing(psx_engine *e, psx_timing *t);

/* Number of configurations an exhaustive sweep evaluates (null included):
 * sum_{k<=c} e_k(w), w_u = 2^{#studies containing u} - 1. */
uint64_t psx_count_configs(const psx_problem *prob);

#ifdef __cplusplus
}
#endif
#endif /* PIPSORT_ENGINE_H */
