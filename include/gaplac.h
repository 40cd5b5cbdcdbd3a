/*
 * gaplac.h — C-ABI of libgaplac_hip.so, the MI355X (gfx950) backend for GaPLAC's
 * per-MCMC-step Gaussian-process log-marginal-likelihood.
 *
 * The reference computes, for every evaluation (AbstractGPs 0.5.12 `logpdf(::FiniteGP, v)`,
 * reached from /root/reference/CLI/src/mcmc.jl:35 and /root/reference/CLI/src/select.jl:49-50):
 *
 *     C    = sum_t K_t(X) + noise * I          (kernelmatrix of the tree built by
 *                                               GaPLAC.kernel, src/abstractgp_translations.jl:45-71)
 *     U    = chol_upper(C)                     (LAPACK dpotrf('U'))
 *     logp = -( N*log(2*pi) + 2*sum(log U_ii) + ||U^-T v||^2 ) / 2
 *
 * Each entry point below replaces one piece of that chain; all are plain C, plain
 * pointers and sizes, no device types in the signatures. Host buffers passed in are
 * copied during the call and never retained.
 *
 * Return convention (mirrors LinearAlgebra.cholesky(check=true) and the argument checks
 * of KernelFunctions constructors):
 *     0   success
 *    >0   potrf `info`: 1-based order of the first leading minor that is not positive
 *         definite (the Julia glue rethrows LinearAlgebra.PosDefException(info));
 *         *out_logpdf is NaN
 *    <0   an argument error (GAPLAC_E_*) or a HIP/RCCL runtime error; *out_logpdf is NaN
 *         and gaplac_last_error() holds the text.
 */
#ifndef GAPLAC_H
#define GAPLAC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GAPLAC_ABI_VERSION 1

/* Kernel-term kinds. Each is the KernelFunctions 0.10.38 kernel that
 * src/abstractgp_translations.jl:8-15 builds for one GaPLAC formula term. */
enum gaplac_kind {
    GAPLAC_SQEXP  = 1, /* SqExp(:x; l)  -> SqExponentialKernel ∘ ScaleTransform(1/l):
                          k = exp(-((x_i - x_j)/l)^2 / 2)       src/gp_parts.jl:21-27 */
    GAPLAC_OU     = 2, /* OU(:x; l)     -> ExponentialKernel ∘ ScaleTransform(1/l):
                          k = exp(-|x_i - x_j|/l)                src/gp_parts.jl:37-43 */
    GAPLAC_LINEAR = 3, /* Linear(:x; c) -> LinearKernel(c): k = x_i*x_j + c, c >= 0
                                                                 src/gp_parts.jl:29-35 */
    GAPLAC_CAT    = 4, /* Cat(:x)       -> CategoricalKernel: k = (x_i == x_j)
                                                                 src/gp_parts.jl:11-13,45-47 */
    GAPLAC_NOISE  = 5  /* extension (absent in the reference):
                          k = param * delta_ij by index; col ignored */
};

/* One formula term after lowering. `param` is the lengthscale l (SQEXP, OU), the
 * intercept c (LINEAR) or the variance (NOISE); ignored for CAT.
 * `group`: terms with equal group multiply, groups add. The reference lowering
 * (kernel(), abstractgp_translations.jl:45-69) only ever produces sums, so each term has
 * its own group; shared groups are the true-product extension.
 * Terms of one group must be contiguous in the array. */
typedef struct gaplac_term {
    int32_t kind;
    int32_t col;     /* 0-based column of X */
    double  param;
    int32_t group;
    int32_t reserved; /* must be 0 */
} gaplac_term;

#define GAPLAC_MAX_TERMS 16

/* error codes (<0) */
#define GAPLAC_E_ARG      (-1)  /* N < 0, D < 1 with terms reading X, ldx < N, null pointer */
#define GAPLAC_E_KIND     (-2)  /* unknown term kind / too many terms / bad group order */
#define GAPLAC_E_PARAM    (-3)  /* l <= 0 or non-finite, c < 0, noise < 0 */
#define GAPLAC_E_COL      (-4)  /* column index outside [0, D) */
#define GAPLAC_E_NODEVICE (-5)  /* no HIP device / device index out of range */
#define GAPLAC_E_HIP      (-6)  /* HIP runtime failure (text in gaplac_last_error) */
#define GAPLAC_E_OOM      (-7)  /* device allocation failed */
#define GAPLAC_E_COMM     (-8)  /* RCCL failure / communicator missing */

typedef struct gaplac_ctx gaplac_ctx;

/* Context: one device, one persistent workspace (the (N+1)-augmented covariance,
 * grown on demand and reused across MCMC steps), two HIP streams. Not re-entrant;
 * distinct contexts may be used from distinct threads.
 * Replaces: nothing in the reference (AbstractGPs allocates ~2T+3 N×N temporaries per
 * logpdf); needed so repeated MCMC evaluations do not re-allocate. */
int  gaplac_ctx_create(int device, gaplac_ctx** out);
int  gaplac_ctx_destroy(gaplac_ctx* ctx);
/* Free the context's large device workspaces (the evaluation matrix, the batched-select
 * workspace sets, the batch lanes) after waiting for its work; the next call allocates
 * again. For callers that share a device between several contexts or processes.
 * Replaces: nothing (the reference frees its temporaries per call). */
int  gaplac_ctx_release(gaplac_ctx* ctx);
const char* gaplac_last_error(const gaplac_ctx* ctx);
int  gaplac_abi_version(void);

/* The hot path. Host pointers. X is N×D column-major with leading dimension ldx (Julia
 * `Matrix(df[!, vars])` wrapped as RowVecs: observations are rows), v has N entries
 * (`y` in select.jl:49-50, the latent `fx` in mcmc.jl:35). noise is the FiniteGP
 * observation variance (0.1 at every reference call site).
 * Replaces: AbstractGPs.logpdf(FiniteGP(GP(kernel(formula)), RowVecs(X), noise), v)
 *           = kernelmatrix (KernelFunctions) + cholesky(Symmetric) (dpotrf 'U')
 *             + logdet + sum(abs2, U' \ v).
 * out_logdet / out_quad may be NULL. */
int gaplac_logpdf(gaplac_ctx* ctx, int64_t N, int32_t D, const double* X, int64_t ldx,
                  int32_t T, const gaplac_term* terms, double noise, const double* v,
                  double* out_logpdf, double* out_logdet, double* out_quad);

/* Same, with X and v already resident in device memory (HBM) on the ctx's device.
 * This is the entry the throughput benchmark times. */
int gaplac_logpdf_device(gaplac_ctx* ctx, int64_t N, int32_t D, const double* dX, int64_t ldx,
                         int32_t T, const gaplac_term* terms, double noise, const double* dv,
                         double* out_logpdf, double* out_logdet, double* out_quad);

/* Batched select (BASELINE config 5): nmodels independent formulas over the same X and
 * v; model m uses terms[term_offset[m] .. term_offset[m+1]). Replaces the two (or more)
 * `logpdf(pr_k, y_k)` calls of CLI/src/select.jl:49-50. out_logpdf / out_info have
 * nmodels entries; the return value is 0 when the batch ran (per-model PD failures are
 * reported in out_info[m] > 0 with out_logpdf[m] = NaN) and <0 on argument/runtime
 * errors. Each result is bitwise that model's gaplac_logpdf. Device memory: up to two
 * workspace sets of GAPLAC_BATCH_W (32) matrices of (N+1 rounded up to 128)^2 doubles,
 * fewer models per set when the free device memory (hipMemGetInfo, 2 GiB kept free) does
 * not hold them, and the two-lane path below two; gaplac_ctx_release frees them. */
int gaplac_logpdf_batch(gaplac_ctx* ctx, int32_t nmodels, int64_t N, int32_t D,
                        const double* X, int64_t ldx, const int32_t* term_offset,
                        const gaplac_term* terms, double noise, const double* v,
                        double* out_logpdf, int64_t* out_info);

/* Gradient of the same log-marginal-likelihood. NUTS in
 * CLI/src/mcmc.jl:31-41 differentiates logpdf(FiniteGP(GP(kernel(formula; ℓ)), RowVecs(X),
 * 0.1), fx) with ForwardDiff Duals, which cannot cross a ccall; the GaPLAC-owned method
 * returns the analytic gradient instead (a ChainRules rrule / Dual overload):
 *     out_dv[i]     = d logp / d v_i          = -(C^{-1} v)_i                  (N entries)
 *     out_dparam[t] = d logp / d param_t      = 1/2 (a' dC a - tr(C^{-1} dC)),  a = C^{-1} v,
 *                     dC = dK_t/dparam_t (times the other terms of t's product group):
 *                     l of SQEXP / OU (k u^2/l, k |u|/l with u = x_i/l - x_j/l), c of LINEAR (1),
 *                     the variance of a NOISE term (delta_ij); 0 for CAT (no parameter)
 *     out_dnoise    = d logp / d noise        (dC = I)
 * The mcmc glue sums out_dparam over the terms whose variable is in `--infer` (they share ℓ).
 * Any output pointer may be NULL. Same return convention as gaplac_logpdf (outputs NaN on
 * error / PosDefException). Replaces: ForwardDiff.gradient through AbstractGPs.logpdf. */
int gaplac_logpdf_grad(gaplac_ctx* ctx, int64_t N, int32_t D, const double* X, int64_t ldx,
                       int32_t T, const gaplac_term* terms, double noise, const double* v,
                       double* out_logpdf, double* out_dv, double* out_dparam, double* out_dnoise);
/* Same with X and v resident on the device (outputs are host pointers). */
int gaplac_logpdf_grad_device(gaplac_ctx* ctx, int64_t N, int32_t D, const double* dX, int64_t ldx,
                              int32_t T, const gaplac_term* terms, double noise, const double* dv,
                              double* out_logpdf, double* out_dv, double* out_dparam, double* out_dnoise);

/* Posterior mean and variance at M test points:
 *     mean_j = k(xs_j, X) C^{-1} y,   var_j = k(xs_j, xs_j) - k(xs_j, X) C^{-1} k(X, xs_j)
 * with C = K(X) + noise I (the FiniteGP's covariance) and the latent kernel k (no noise) for
 * the test points. Xs is M x D column-major (leading dimension ldxs) with the same columns as
 * X. Replaces: mean_and_var(posterior(FiniteGP(GP(k), X, noise), y), xs) of AbstractGPs
 * 0.5.12, reached from src/plotting.jl:8-12 (and posterior(pr, y) in CLI/src/select.jl:51-52).
 * Same return convention as gaplac_logpdf (PosDefException info > 0; outputs NaN). */
int gaplac_posterior_mean_var(gaplac_ctx* ctx, int64_t N, int32_t D, const double* X, int64_t ldx,
                              int32_t T, const gaplac_term* terms, double noise, const double* y,
                              int64_t M, const double* Xs, int64_t ldxs,
                              double* out_mean, double* out_var);

/* One draw of the FiniteGP: out = L z with C = K(X) + noise I = L L^T
 * and z the N standard-normal values the caller drew (the host keeps the RNG stream, so a
 * given z gives the same sample as the reference). Replaces: rand(rng, FiniteGP(GP(k), X,
 * noise)) = mean + cholesky(C).U' * randn(rng, N) (zero mean), reached from
 * CLI/src/sample.jl:25. */
int gaplac_rand(gaplac_ctx* ctx, int64_t N, int32_t D, const double* X, int64_t ldx,
                int32_t T, const gaplac_term* terms, double noise, const double* z, double* out);

/* Debug / parity entries (tests only; not on the timed path). */
/* Gram matrix sum_t K_t(X) + noise*I as a dense N×N column-major host matrix
 * (replaces KernelFunctions.kernelmatrix + Diagonal(Fill(noise, N))). */
int gaplac_gram(gaplac_ctx* ctx, int64_t N, int32_t D, const double* X, int64_t ldx,
                int32_t T, const gaplac_term* terms, double noise, double* out_C, int64_t ldc);
/* Measurement (bench.py extra.gram): the same Gram built from host inputs into the
 * context's workspace by one plain-grid launch, reps times, each bracketed by hipEvents on
 * the launching stream; best_ms = the fastest launch, bytes = its algorithmic HBM bytes
 * (8 Np(Np+1)/2 written + 8 N (D+1) read, Np = N+1 rounded up to 128). */
int gaplac_gram_time(gaplac_ctx* ctx, int64_t N, int32_t D, const double* X, int64_t ldx,
                     int32_t T, const gaplac_term* terms, double noise, const double* v,
                     int32_t reps, double* best_ms, double* bytes);
/* Lower Cholesky factor L = U^T of the same C (dense N×N column-major, upper part
 * zeroed) and z = L^{-1} v (replaces cholesky(Symmetric(C)).U' and U' \ v). */
int gaplac_factor(gaplac_ctx* ctx, int64_t N, int32_t D, const double* X, int64_t ldx,
                  int32_t T, const gaplac_term* terms, double noise, const double* v,
                  double* out_L, int64_t ldl, double* out_z);

/* Per-kernel timing of the evaluations run while profiling is on (off by default),
 * accumulated until gaplac_reset_stats. gaplac_set_profiling mode:
 *   0 off;
 *   1 per-launch device timestamps of every kernel (first workgroup start, last wave
 *     end; 100 MHz s_memrealtime);
 *   2 hipEvents recorded on the launching stream around every bulk trailing-update
 *     (tile_syrk_kernel) launch and every -C^{-1} tile launch of a gradient evaluation,
 *     the production schedule otherwise unchanged: fills syrk_* and cinv_* only, read
 *     back at gaplac_get_stats. */
typedef struct gaplac_stats {
    int64_t evals;
    int64_t syrk_launches;      /* bulk trailing-update launches (tile_gemm_kernel<0>) */
    double  syrk_ms;            /* summed event time of those launches */
    double  syrk_flops;         /* algorithmic flops of those launches */
    double  gram_ms;
    double  gram_bytes;         /* algorithmic bytes of the Gram launches */
    int64_t gram_launches;
    double  panel_ms;           /* diagonal-block potrf launches, summed */
    double  trsm_ms;            /* panel TRSM launches, summed */
    double  colupd_ms;          /* lookahead column-update launches, summed */
    double  total_ms;           /* whole evaluation, first kernel to result */
    double  syrk_bytes;         /* algorithmic HBM bytes of the bulk launches: C tiles read +
                                   written once, panel rows read once */
    int64_t small_launches;     /* small trailing updates (quad_bulk_kernel), not in syrk_* */
    double  small_ms;
    /* gradient evaluations (gaplac_logpdf_grad), profiling mode 1 */
    double  grad_rows_ms;       /* identity-row substitution + updates (L^{-T} rows) */
    int64_t cinv_launches;      /* -C^{-1} = -L^{-T} L^{-1} tile launches (cinv_tile_kernel) */
    double  cinv_ms;
    double  contract_ms;        /* dC/dtheta contraction (grad_contract_kernel) */
    /* persistent tail (tail_kernel: the last tile columns as one dataflow launch) */
    int64_t tail_launches;
    double  tail_ms;
    /* profiling mode 2: every bulk-type launch of the super-panel phase (triangle updates,
       bands, split heads, whole-tile lookaheads; they overlap since round 6): summed
       algorithmic flops, launches, and the union of their event intervals */
    double  bulk_flops;
    int64_t bulk_launches;
    double  bulk_union_ms;
} gaplac_stats;
int gaplac_set_profiling(gaplac_ctx* ctx, int mode);
int gaplac_get_stats(gaplac_ctx* ctx, gaplac_stats* out);
int gaplac_reset_stats(gaplac_ctx* ctx);

/* Launch-footprint check of one evaluation's schedule, on the host only (no device, no
 * context): walks every launch gaplac_logpdf (mode 0), gaplac_logpdf_grad (mode 1) or
 * gaplac_posterior_mean_var at M test points (mode 2) would enqueue for order N with
 * super-panel width spw, and checks the element range each launch's grid touches against
 * the workspace the context allocates for N. Every launcher applies the same check before
 * a real launch (a violating launch is not enqueued; the entry returns GAPLAC_E_ARG).
 * Returns 0 (the counts are valid) or GAPLAC_E_ARG for bad arguments; *out_violations is
 * the number of launches outside the workspace and msg (msglen bytes) the first one.
 * mode + 8: the same walk against a workspace one element short (the guard's negative
 * control: the last Gram tile must be reported).
 * Not in the reference (an internal guard). */
int gaplac_plan_check(int64_t N, int32_t mode, int64_t M, int32_t spw, int64_t* out_launches,
                      int64_t* out_violations, char* msg, int64_t msglen);
/* Host-only accounting of the single-GPU schedule for order N (GAPLAC_SPW = spw,
 * GAPLAC_PAIR_DEPTH = depth (0: auto), band extension pair_ext (0/1), GAPLAC_PAIR_M =
 * pair_m): every tile column gets every earlier panel column exactly once, in order, before
 * its factorisation, and every update reads factored panel columns. 0, or GAPLAC_E_ARG with
 * the first violation in msg; *out_records: launches and factorisations recorded. Not in the
 * reference (an internal guard). */
int gaplac_plan_check_schedule(int64_t N, int32_t spw, int32_t depth, int32_t pair_ext, int32_t pair_m,
                               int64_t* out_records, char* msg, int64_t msglen);

/* ------------------------------------------------------------------------------------
 * Distributed evaluation (BASELINE configs[3]: N = 65536 over the GPUs of one node; one
 * process per GPU). 1-D block-column cyclic Cholesky: super-panels of spw 128-wide
 * tile columns are dealt round-robin over the ranks; each rank builds and stores only its
 * own columns of the lower triangle (the Gram shards with no redistribution) and the only
 * data-path exchange is one broadcast per super-panel of the factored panel, which the
 * HOST enqueues with its collective library (ncclBroadcast = RCCL over xGMI) on the
 * stream gaplac_dist_comm_begin returns. Same result as gaplac_logpdf (<= 1e-9 rel).
 * Replaces, like gaplac_logpdf: AbstractGPs.logpdf(FiniteGP, v) — the GaPLAC-owned method
 * would dispatch here when the job runs on several GPUs.
 *
 * Per rank, per evaluation (every call only enqueues, except finish):
 *   gaplac_dist_begin(...)                         -> nsteps (nsp without the tail gather)
 *   if (owner(0) == rank) gaplac_dist_factor(d, 0)         (owner: gaplac_dist_owner)
 *   bcast(0)
 *   for s in 0..nsteps-1:
 *       if (s+1 < nsteps && owner(s+1) == rank) gaplac_dist_factor(d, s+1)
 *       gaplac_dist_update(d, s)
 *       if (s+1 < nsteps) bcast(s+1)
 *   [the tail gather, when set: see gaplac_dist_set_tail]
 *   gaplac_dist_finish(d, &logdet_part, &quad_part, &info_part)
 *   allreduce: logdet = sum, quad = sum, info = min over nonzero; then
 *   logpdf = -(N*log(2*pi) + logdet + quad) / 2   (NaN / PosDefException if info > 0)
 * where bcast(s) = gaplac_dist_chunks(d, s, &nc);
 *                  for c in 0..nc-1:
 *                      gaplac_dist_panel_chunk(d, s, c, &buf, &count, &root);
 *                      gaplac_dist_comm_begin_chunk(d, s, c, &stream);
 *                      ncclBroadcast(buf, buf, count, ncclDouble, root, comm, stream);
 *                      gaplac_dist_comm_end_chunk(d, s, c);
 * A chunk is a run of the panel's tile columns (gaplac_dist_configure): its owner packs it
 * as soon as its last column is final and the next owner's lookahead consumes it as it
 * arrives, so broadcasts overlap both chains. The whole panel as one
 * broadcast (gaplac_dist_panel / _comm_begin / _comm_end) is the one-chunk case.
 * ---------------------------------------------------------------------------------- */
typedef struct gaplac_dist gaplac_dist;
int gaplac_dist_create(int device, int nranks, int rank, int spw, gaplac_dist** out);
int gaplac_dist_destroy(gaplac_dist* d);
const char* gaplac_dist_last_error(const gaplac_dist* d);
/* Padded order Np = roundup(N+1, 128), tile columns nt, super-panels nsp, this rank's
 * local tile columns nloc, and the doubles one panel buffer must hold. */
int gaplac_dist_geometry(gaplac_dist* d, int64_t N, int64_t* Np, int32_t* nt, int32_t* nsp,
                         int32_t* nloc, int64_t* panel_elems);
/* Optional: two caller-owned device panel buffers (e.g. allocated by the collective
 * library's host binding), each of >= panel_elems doubles; NULLs = library-owned. */
int gaplac_dist_set_panel_buffers(gaplac_dist* d, void* buf0, void* buf1, int64_t capacity);
/* Inputs as for gaplac_logpdf (inputs_on_device: X and v are device pointers). Builds
 * this rank's Gram tiles; returns the number of super-panels in *out_nsp. */
int gaplac_dist_begin(gaplac_dist* d, int64_t N, int32_t D, const double* X, int64_t ldx,
                      int32_t T, const gaplac_term* terms, double noise, const double* v,
                      int inputs_on_device, int32_t* out_nsp);
/* Schedule options, before gaplac_dist_set_panel_buffers / begin (< 0 keeps the current
 * value; defaults from GAPLAC_DIST_DEPTH / _CHUNK / _BIG / _BIG_MIN / _ALONE): depth =
 * super-panels per deferred bulk update (1..8), chunk = tile columns per broadcast chunk
 * (1..spw), big = bulk kernel choice (0: never the large-launch kernel; 1: per rank,
 * launches of >= big_min tiles while this rank runs no chain; 2: by launch size, as on one
 * GPU — for ranks that share one device), alone = 1: a rank's bulk update waits while it
 * factors the next super-panel (the chain gets the whole GPU). Defaults with several ranks
 * (the one-GPU replay's best at N = 65536 over 8): depth 2, chunk 2, big 1,
 * alone 1; with one rank: chunk = spw, big 2, alone 0. */
int gaplac_dist_configure(gaplac_dist* d, int32_t depth, int32_t chunk, int32_t big, int32_t big_min,
                          int32_t alone);
/* Super-panel layout, before begin: snake = 1 deals the super-panels boustrophedon (rank r
 * owns super-panel u*nranks + r in even rounds u, u*nranks + nranks-1-r in odd ones), which
 * evens out the ranks' trailing-update work; 0 = round-robin. Default: 1
 * with several ranks. owner: the rank that owns super-panel s (factors it and roots its
 * broadcast). */
int gaplac_dist_set_layout(gaplac_dist* d, int32_t snake);
int gaplac_dist_owner(gaplac_dist* d, int32_t s, int32_t* out_rank);
int gaplac_dist_factor(gaplac_dist* d, int32_t s);   /* owner of super-panel s only */
int gaplac_dist_chunks(gaplac_dist* d, int32_t s, int32_t* out_chunks);
int gaplac_dist_panel_chunk(gaplac_dist* d, int32_t s, int32_t c, void** buf, int64_t* count,
                            int32_t* root);
int gaplac_dist_comm_begin_chunk(gaplac_dist* d, int32_t s, int32_t c, void** hip_stream);
int gaplac_dist_comm_end_chunk(gaplac_dist* d, int32_t s, int32_t c);
int gaplac_dist_panel(gaplac_dist* d, int32_t s, void** buf, int64_t* count, int32_t* root);
int gaplac_dist_comm_begin(gaplac_dist* d, int32_t s, void** hip_stream);
int gaplac_dist_comm_end(gaplac_dist* d, int32_t s);
int gaplac_dist_update(gaplac_dist* d, int32_t s);
/* This rank's partial logdet / quad and first failing pivot (0 = none); synchronises. */
int gaplac_dist_finish(gaplac_dist* d, double* logdet_part, double* quad_part, int64_t* info_part);
/* Debug / parity: this rank's column storage (Np x nloc*128, column-major) to host. */
int gaplac_dist_local(gaplac_dist* d, double* out, int64_t ld);
/* Host-only (no HIP calls): checks the step plan for nt tile columns — every super-panel
 * gets every earlier panel once, in order, before its chain. 0 or GAPLAC_E_ARG (msg). */
int gaplac_dist_plan_check(int32_t nt, int32_t spw, int32_t depth, int32_t pair_m, int64_t* out_ops,
                           char* msg, int64_t msglen);
/* Host-only: the plan's ops as (step, kind, sp, first panel, last panel) int32 quintuples
 * (kind 0: that super-panel, 1: every super-panel from it on, 2: the step's event after
 * super-panel step+2 is up to date); *out_n = op count, out may be NULL. */
int gaplac_dist_plan(int32_t nt, int32_t spw, int32_t depth, int32_t pair_m, int32_t* out, int64_t cap,
                     int64_t* out_n);
/* Tail gather (off by default). tail_cols > 0: the super-panels whose columns all lie in
 * the last tail_cols (<= 128) tile columns are not factored by the distributed steps. After
 * the last step's update every rank sends its columns of that trailing matrix (from each
 * super-panel's first row down) to rank `root`, which factors it with the single-GPU
 * persistent tail; begin then returns the number of distributed steps (fewer than nsp).
 * Per rank, after the step loop:
 *   gaplac_dist_tail_begin(d, &stream);      packs this rank's segments on stream
 *   for i in 0..nseg-1: gaplac_dist_tail_segment(d, i, &buf, &count, &src);
 *       src == rank != root: ncclSend(buf, count, ncclDouble, root, comm, stream)
 *       rank == root != src: ncclRecv(buf, count, ncclDouble, src, comm, stream)
 *   (all inside one ncclGroupStart / ncclGroupEnd)
 *   gaplac_dist_tail_end(d);                  the root factors the gathered matrix
 * then finish as before (the root's partial sums include the tail's). The reference's
 * logpdf is the same single evaluation (CLI/src/mcmc.jl:35); nothing in it is split. 0 = off
 * (the default with one rank). Not in the reference. */
int gaplac_dist_set_tail(gaplac_dist* d, int32_t tail_cols, int32_t root);
/* For order N, before begin: segments of the gather (0: none), the doubles this rank's
 * segment buffer needs, and the steps begin will return. */
int gaplac_dist_tail_geometry(gaplac_dist* d, int64_t N, int32_t* nseg, int64_t* buf_elems,
                              int32_t* nsteps);
/* Optional caller-owned device segment buffer of >= buf_elems doubles (NULL: library-owned). */
int gaplac_dist_set_tail_buffer(gaplac_dist* d, void* buf, int64_t capacity);
int gaplac_dist_tail_segment(gaplac_dist* d, int32_t i, void** buf, int64_t* count, int32_t* src);
int gaplac_dist_tail_begin(gaplac_dist* d, void** hip_stream);
int gaplac_dist_tail_end(gaplac_dist* d);
/* Host-only: the plan and its check with the tail gather of tail_cols tile columns. */
int gaplac_dist_plan_check_tail(int32_t nt, int32_t spw, int32_t depth, int32_t pair_m, int32_t tail_cols,
                                int64_t* out_ops, char* msg, int64_t msglen);
int gaplac_dist_plan_tail(int32_t nt, int32_t spw, int32_t depth, int32_t pair_m, int32_t tail_cols,
                          int32_t* out, int64_t cap, int64_t* out_n);
/* Replay of one rank's schedule on one GPU (diagnostics): the other ranks'
 * panels arrive as copies from their (already factored) contexts on a modelled timeline.
 * replay_enable(N) before begin turns device timestamps on (0: off); replay_chunk replaces bcast's
 * broadcast of one chunk (times in 10 ns ticks); replay_stamps copies the timestamps out;
 * replay_info: a chunk's bytes and the stamp layout. Not in the reference. */
int gaplac_dist_replay_enable(gaplac_dist* d, int64_t N);
int gaplac_dist_replay_chunk(gaplac_dist* d, const gaplac_dist* owner, int32_t s, int32_t c,
                             int64_t f_ticks, int64_t band_ticks, int64_t lat_ticks,
                             int64_t xfer_ticks, int64_t copy_ticks);
int gaplac_dist_replay_stamps(gaplac_dist* d, uint64_t* out, int64_t n);
/* The tail gather on the replayed rank (in place of tail_begin / the transfers / tail_end):
 * the root's segments from the owners' contexts of a loopback run with the same gather,
 * released at max(END(last step), Gram end + senders_end) + lat + the largest sender's
 * bytes x ticks_per_byte (senders_end: the latest sender's last update end in its own
 * replay, relative to its Gram end; 0 = this rank's own END). */
int gaplac_dist_replay_tail(gaplac_dist* d, const gaplac_dist* const* owners, int32_t nowners,
                            int64_t lat_ticks, double ticks_per_byte, int64_t copy_ticks,
                            int64_t senders_end);
int gaplac_dist_replay_info(gaplac_dist* d, int32_t s, int32_t c, int64_t* bytes, int32_t* per_step,
                            int32_t* maxc);

#ifdef __cplusplus
}
#endif
#endif /* GAPLAC_H */
