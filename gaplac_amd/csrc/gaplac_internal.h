// Internal declarations shared by the HIP kernels (gaplac_kernels.hip) and the host
// orchestration (gaplac_api.hip). Not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <vector>
#include "../../include/gaplac.h"

namespace gaplac {

// Panel width of the blocked right-looking Cholesky and edge of every square tile the
// kernels work on (Gram tiles, diagonal blocks, trailing-update tiles). 128 fp64 x 128 =
// 128 KiB: a diagonal block (plus its inverse, packed) fits one CU's 160 KiB LDS.
constexpr int NB = 128;
constexpr int DINV_PER_BLOCK = 8 * 16 * 16;  // Dinv doubles per diagonal block

// Term descriptor as the Gram kernel reads it (device memory, one small H2D copy per
// evaluation, so a captured graph replays with new hyperparameters).
struct TermPack {
    int32_t T;
    int32_t kind[GAPLAC_MAX_TERMS];
    int32_t col[GAPLAC_MAX_TERMS];
    int32_t last_in_group[GAPLAC_MAX_TERMS];
    double  p[GAPLAC_MAX_TERMS];  // 1/l for SQEXP/OU, c for LINEAR, variance for NOISE
    double  noise;                 // FiniteGP observation variance (diagonal)
};

// Device-side result record of one evaluation.
constexpr int REDUCE_BLOCKS = 64;  // workgroups of the logdet / quad reduction
struct EvalResult {
    double logpdf;
    double logdet;
    double quad;
    unsigned long long info;  // min over failing pivots of (j+1); ULLONG_MAX = none
    unsigned err;             // nonzero: a bounded in-kernel wait expired (the host returns GAPLAC_E_HIP)
    unsigned err_pad;
    double part[2][REDUCE_BLOCKS];  // per-workgroup partial sums of the reduction
    unsigned gram_ticket;           // work queue of the second Gram launch (zeroed per eval)
};

// Per-launch device timestamps (profiling): 100 MHz s_memrealtime ticks.
struct KTime {
    unsigned long long start;  // min over workgroups (init ~0)
    unsigned long long end;    // max over waves (init 0)
    // diagnostic build only (-DGAPLAC_CLOCK): per-workgroup shader cycles and 100 MHz ticks
    // of the bulk tile kernels, summed (the clock the chip held: DESIGN.md §3.8)
    unsigned long long clk_mt, clk_rt, clk_n;
};

// Where global tile column bj of the lower triangle is stored. Single-GPU layout: the
// identity (nranks = 1). 1-D block-column cyclic distribution over nranks: super-panels of
// W tile columns are dealt in rounds of nranks, one per rank, and a rank keeps its
// super-panels contiguously in order, so local tile column lj (round u = lj / W) holds
//   bj = (u * nranks + r(u)) * W + lj % W,   r(u) = rank, or with snake (boustrophedon)
// dealing nranks - 1 - rank in odd rounds (every rank then alternates
// between early and late super-panels of a round).
// Rows are never redistributed: every storage column keeps global row indices.
struct ColMap {
    int nranks, rank, W;
    int snake = 0;
    __host__ __device__ __forceinline__ int global(int lj) const {
        if (nranks == 1) return lj;
        const int u = lj / W;
        const int r = (snake && (u & 1)) ? nranks - 1 - rank : rank;
        return (u * nranks + r) * W + lj % W;
    }
};

// The kdepth panel columns a trailing update subtracts: global row r of panel column c is
// P[c * ld + (r - row0)]. Single-GPU: the factored columns inside A (row0 = 0, ld = lda);
// distributed: the broadcast panel buffer (row0 = first row of the super-panel).
struct Panel {
    const double* P;
    int64_t ld;
    int64_t row0;
};

// One bulk trailing update: tiles (bi, lj) = (bi0 + lo16, lj0 + hi16) of the list,
// C(bi, bj = cm.global(lj)) -= P_bi P_bj^T with K = kdepth.
struct BulkArgs {
    double* C;
    int64_t ldc;
    Panel pn;
    const uint32_t* tiles;  // nullptr: rectangular block of rect_rows tile rows (tile_decode)
    int ntiles, kdepth, bi0, lj0;
    ColMap cm;
    int rect_rows = 0;
    int max_r = -1, max_c = -1;  // largest lo16 / hi16 list entry (-1: an m x m triangle list)
    int whole = 0;    // 1: a band list as 128x128 tile workgroups (tile_band_kernel), never quadrants
    int tile_min = 0;  // > 0: at least this many tiles go to tile_syrk_kernel even below the quadrant limit
    // large-launch kernel (tile_syrk_big_kernel, three workgroups per CU): -1 by launch size
    // (>= BULK_BIG_TILES tiles), 0 never, 1 the caller chose it (a distributed rank with no
    // chain beside this launch); quadrant-sized launches never take it
    int big = -1;
};

// Persistent tail (gaplac_kernels.hip tail_kernel): completion counters of
// the tile tasks of the last T <= TAIL_TMAX tile columns, zeroed before every launch.
constexpr int TAIL_TMAX = 128;
struct TailCtl {
    unsigned head;  // dequeue counter
    unsigned err;   // an expired wait
    unsigned ddone[TAIL_TMAX];                // D(k) finished
    unsigned dprog[TAIL_TMAX];                // D(k): block columns (and inverses) 0 .. dprog-1 final
    unsigned sdone[TAIL_TMAX * TAIL_TMAX];    // S(i,k) finished ([i][k], relative tile indices)
    unsigned units[TAIL_TMAX * TAIL_TMAX];    // tile (i,j): update units applied per column (4; 10 on the diagonal)
    // TRSM of the sub-diagonal tile (k+1, k): per 16-row group g, the 16-column blocks of L
    // stored so far (0..8); the next diagonal tile's Q blocks consume them as they come
    unsigned sprog[TAIL_TMAX][8];
    // Gram tile (i, j) built by its task (TAIL_G, the Gram inside the tail): its first
    // column's tasks (k = 0) wait for it
    unsigned gdone[TAIL_TMAX * TAIL_TMAX];
};
struct TailArgs {
    double* A;
    int64_t lda, N;
    int ts, T;  // tile columns ts .. ts+T-1
    double* Dinv;
    EvalResult* res;
    TailCtl* ctl;
    const uint32_t* tasks;
    int ntasks;
    unsigned long long* trace;  // diagnostics (GAPLAC_TAIL_TRACE): per task dequeue / start / end times, or nullptr;
                                // single-model launches: then TAIL_DSTAMPS phase times per diagonal block at
                                // trace + 3 ntasks + TAIL_DSTAMPS k (potrf_diag2_body)
    // several models in one launch (gaplac_logpdf_batch): task bits 27.. hold the model m,
    // whose matrix is A + m a_stride, inverses Dinv + m dinv_stride, result res + m,
    // counters ctl + m (ctl[0].head is the one dequeue counter)
    int64_t a_stride = 0, dinv_stride = 0;
    int nmodels = 1;
    // debug (GAPLAC_TAIL_FAULT, tests only): the diagonal-block task of relative tile column
    // fault is skipped, never publishing, so every wait behind it expires and the evaluation
    // must come back as GAPLAC_E_HIP; -1 = off
    int fault = -1;
    int xrows = 0;  // extra tile rows below the matrix factored along (tile rows ts+T .. ts+T+xrows-1)
    // The Gram inside the tail (single evaluations whose matrix lies whole in it, ts = 0):
    // the list holds one TAIL_G task per lower tile, built from gX (ld gldx), gv and gtp as
    // gram_kernel builds it; nullptr: the Gram is built before the launch
    const double* gX = nullptr;
    int64_t gldx = 0;
    const double* gv = nullptr;
    const TermPack* gtp = nullptr;
};
constexpr int TAIL_DSTAMPS = 20;  // start, load in LDS, per panel s: phase 2 start / end, done
constexpr int TAIL_MODEL_SHIFT = 27;
constexpr int TAIL_MAX_MODELS = 32;
// colstart (optional): index in out where the tasks of tile column g = 0 .. T-2 begin.
// gw (4 or 8): panel columns per deep update of a far tile; near: tile columns beyond the
// current block of gw that still get per-column updates; quad_last: the last quad_last
// columns take latency-shaped tasks (the next tile column's tiles updated as four 64x64
// quadrant tasks), the columns before them whole tiles; whole_trsm: before the last
// quad_last columns the TRSMs are whole-tile tasks after the diagonal block, not two row
// halves pipelined behind it; group (1, 2 or 4): near tiles take that many columns per
// task (K = 128 group) where the chain allows.
// xrows > 0: xrows extra tile rows below the matrix (relative rows T .. T+xrows-1, the
// posterior's cross-covariance rows) factored along: whole-tile TRSMs and updates only.
// crit_quads > 0: column g's updates of tiles (g+1+d, g+1), 1 <= d <= crit_quads, are
// quadrant tasks in every column (not only the last quad_last).
void build_tail_tasks(int T, std::vector<uint32_t>& out, std::vector<size_t>* colstart = nullptr, int gw = 4,
                      int near = 4, int quad_last = TAIL_TMAX, bool whole_trsm = false, int group = 1,
                      int xrows = 0, int crit_quads = 0);
// The list (no extra rows) reordered by a simulated schedule on `workers` workgroups
// (longest path to the end first, measured task durations); kept as built if the result
// fails check_tail_tasks. Returns 0 when reordered, 1 if the simulation stalled, 2 if the
// order failed the check (both: list unchanged).
int sim_order_tail_tasks(int T, std::vector<uint32_t>& list, int workers);
// B models' task lists interleaved (each model's own order kept, so the result is a
// topological order per model). lag = 0: task by task, all models in step. lag > 0: a
// software pipeline: model m runs lag * m tile columns behind model 0, and the tasks of the
// models' current columns are interleaved task by task (colstart from build_tail_tasks).
void interleave_tail_tasks(const std::vector<uint32_t>& one, const std::vector<size_t>& colstart, int B, int lag,
                           std::vector<uint32_t>& out);
// The list is a topological order of the tail's dataflow that applies every update once
// (gram: it also builds every lower tile once, before the tile's first task).
bool check_tail_tasks(int T, const std::vector<uint32_t>& list, std::string* why, int xrows = 0, bool gram = false);
// The Gram inside the tail: one TAIL_G task per lower tile of the T x T tile triangle
// prepended to a list (tile (0,0) first, then D(0), then the rest column by column).
void add_gram_tasks(int T, std::vector<uint32_t>& list);
void launch_tail(hipStream_t s, const TailArgs& a, int grid, KTime* kt);
// init_result_kernel's reset of res plus every word of the tail's counters ctl, one launch;
// it also stores tp (by value) into dtp
void launch_init_result_ctl(hipStream_t s, EvalResult* res, TailCtl* ctl, const TermPack& tp, TermPack* dtp);
// The single-evaluation tail list (gaplac_api.hip): T tile columns, X extra tile rows, the
// simulated order per tail_sim (-1 auto: T < 80) planned for `workers` workgroups.
void build_single_tail_list(int T, int X, int tail_sim, int workers, std::vector<uint32_t>& out, bool gram = false);

// Host-side footprint guard. Before launching, every launcher computes the
// element range [p + lo, p + hi) its grid will touch in the column storage it is given
// and checks it against the guarded allocation; a launch outside it is skipped and
// recorded (the API then returns GAPLAC_E_ARG). In dry mode nothing is launched at all:
// the host walks the real schedule (gaplac_plan_check), so the footprints of every launch
// of an evaluation can be checked without a GPU.
struct LaunchGuard {
    const double* base = nullptr;  // the guarded allocation (a context's column storage)
    int64_t elems = 0;
    bool dry = false;
    int64_t launches = 0;
    int64_t violations = 0;
    std::string first;  // the first violation
    // optional schedule accounting of a dry single-GPU walk (gaplac_plan_check_schedule):
    // 5 ints per record {kind, j0, j1, k0, k1}: kind 0 = tile columns [j0, j1) updated
    // (rows from their diagonal down) with panel columns [k0, k1); 1 = column j0 factored
    // (diagonal block / TRSM); 2 = the persistent tail factors columns >= j0
    std::vector<int>* acct = nullptr;
};
// record into the current guard's accounting (no-op without one)
void acct_record(int kind, int j0, int j1, int k0, int k1);
// panel column of a single-GPU panel pointer (its offset from the guard's base / (ld NB))
int acct_panel_col(const double* P, int64_t ld);
LaunchGuard*& current_guard();  // this thread's guard (nullptr: unchecked)
struct GuardScope {
    LaunchGuard* prev;
    explicit GuardScope(LaunchGuard* g) : prev(current_guard()) { current_guard() = g; }
    ~GuardScope() { current_guard() = prev; }
};
// true if the launch may proceed: [p + lo, p + hi) inside the guard (when p is guarded,
// i.e. derived from its base) and not a dry run
bool guard_launch(const char* what, const double* p, int64_t lo, int64_t hi);
// launches that touch no guarded storage: counted, skipped in a dry run
bool guard_launch(const char* what);

// Term validation + kernel-argument pack (gaplac_api.hip); on error returns GAPLAC_E_*
// and sets *err.
int pack_terms(int32_t D, int32_t T, const gaplac_term* terms, TermPack* tp, std::string* err);

// Launchers (gaplac_kernels.hip). Every launcher takes a KTime slot (nullptr = off).
// Single-GPU layout: A is the Np x Np column-major augmented matrix (lda = Np, Np =
// roundup(N+1, NB)): rows/cols 0..N-1 hold C, row N holds v^T.
// part 0: all lower tiles; part 1: the first w tile columns; part 2: tiles with both
// block indices >= w (parts 1 + 2 = part 0).
// Tiles of part 2 as a work queue with per_cu workgroups per CU (room for the panel
// chain beside them); res->gram_ticket must be zero (init_result_kernel) on the same stream.
// Tiles of tile columns w .. w1-1 only when w1 < nt.
void launch_gram_queue(hipStream_t s, double* A, int64_t lda, int64_t N, int nt, const double* X, int64_t ldx,
                       const double* v, const TermPack* dtp, int w, int w1, int per_cu, EvalResult* res, KTime* kt);
void launch_gram(hipStream_t s, double* A, int64_t lda, int64_t N, int nt,
                 const double* X, int64_t ldx, const double* v, const TermPack* dtp, int part, int w,
                 KTime* kt);
// Gram tiles of a list (entry bi | lj << 16, absolute, bi <= max_bi, lj <= max_lj) into
// column storage C.
void launch_gram_list(hipStream_t s, double* C, int64_t ldc, int64_t N, const double* X, int64_t ldx,
                      const double* v, const TermPack* dtp, const uint32_t* tiles, int ntiles, ColMap cm,
                      int max_bi, int max_lj, KTime* kt);
// Diagonal block at Ablk (global rows/cols g0..g0+127): L in place + Dinv (DINV_PER_BLOCK
// doubles: 8 column-major 16x16 inverses of its diagonal sub-blocks).
void launch_potrf_diag(hipStream_t s, double* Ablk, int64_t lda, int64_t N, int64_t g0,
                       double* Dinv, EvalResult* res, KTime* kt);
// TRSM of the panel rows below diagonal block k: Acol is the storage of global column
// k*NB; rows bi*NB.. for bi = k+1..nt-1 become A[bi,k] L_kk^{-T}.
void launch_trsm(hipStream_t s, double* Acol, int64_t lda, int nt, int k, const double* Dinv, KTime* kt);
// Same substitution for an arbitrary run of row tiles bi0 .. bi0+nrows-1 of column k
// (the gradient's identity rows below the matrix).
void launch_trsm_rows(hipStream_t s, double* Acol, int64_t lda, int k, int bi0, int nrows, const double* Dinv,
                      KTime* kt);
// Bulk trailing update (tile kernel, or quadrant kernel for small tile counts).
void launch_bulk(hipStream_t s, const BulkArgs& a, KTime* kt);
// True when launch_bulk over ntiles tiles runs the small (quadrant) kernel.
bool syrk_is_small(int ntiles);
// Update of global tile columns jb .. jb+ncols-1 (rows >= their diagonal), stored in local
// tile columns lj0.., with the kdepth panel columns of pn.
void launch_col_update(hipStream_t s, double* C, int64_t ldc, const Panel& pn, int nt, int jb, int lj0,
                       int ncols, int kdepth, KTime* kt);
void build_tile_list(int m, uint32_t* out);
// logdet / quad over storage columns 0..ncols-1 (global columns via cm, those < N).
void launch_reduce(hipStream_t s, const double* C, int64_t ldc, int64_t N, int64_t ncols, ColMap cm,
                   EvalResult* res);
void launch_kt_reset(hipStream_t s, KTime* kt, int n);
void launch_init_result(hipStream_t s, EvalResult* res);

// ---- gradient of logpdf ----
// Rows Np .. 2Np-1 of the column storage (lda = 2 Np) hold the identity rows E = [I 0]
// whose factorisation leaves Y = L^{-T} (upper triangular). Y tile (E, J) is stored at
// A + J*NB*lda + Np + E*NB.
// Reset the identity rows: tiles E <= J get identity / zero, tiles below the diagonal
// within a super-panel of W tile columns get zero (read as panel rows by its update).
void launch_init_identity_rows(hipStream_t s, double* A, int64_t lda, int64_t Np, int nt, int W);
// Zero Y[:, N .. Np) (the columns of the padding / v row).
void launch_zero_tail_cols(hipStream_t s, double* A, int64_t lda, int64_t Np, int64_t N);
// z = row N of the factor into a contiguous buffer (N doubles).
void launch_copy_z(hipStream_t s, const double* A, int64_t lda, int64_t N, double* z);
// alpha = Y z (= C^{-1} v), z from launch_copy_z: partial sums per 512-column chunk, then a
// fixed-order sum; also writes dv = -alpha. Reads only the identity rows and z, so it runs
// beside cinv_tile_kernel (which overwrites the factor storage).
void launch_alpha(hipStream_t s, const double* A, int64_t lda, int64_t Np, int64_t N, const double* z,
                  double* partial, double* alpha, double* dv);
// Product-group bounds per term (the gradient of a term inside a product group carries
// the group's other terms).
struct GradTermPack {
    int32_t gstart[GAPLAC_MAX_TERMS];  // first term of t's product group
    int32_t gend[GAPLAC_MAX_TERMS];    // one past its last term
};
// M = -C^{-1} = -Y Y^T over the lower tiles I >= J (I, J < m) into the factor storage
// (rows / columns < Np of A): tile (I, J) = -sum_{k >= I NB} Y_Ik Y_Jk^T. list[b] = I | J << 16
// for workgroup b, 0xffffffff = idle (build_grad_list).
void launch_cinv_tiles(hipStream_t s, double* A, int64_t lda, int64_t Np, const uint32_t* list, int nblocks, int m,
                       KTime* kt);
// Per lower tile of M: its share of sum_ij (alpha_i alpha_j - Cinv_ij) dC_ij/dtheta for every
// term parameter (t < T) and the observation variance (t = T): partial[tile * (T+1) + t].
void launch_grad_contract(hipStream_t s, const double* A, int64_t lda, int64_t N, const double* X, int64_t ldx,
                          const double* alpha, const TermPack* dtp, const GradTermPack* dgp, double* partial,
                          KTime* kt);
// ---- posterior mean / variance ----
// Extra rows Np .. Np + 128 mt - 1 (lda = Np + 128 mt) = K(xs, X): mt x nt tiles, zero
// outside test point j < M and training point i < N.
void launch_cross_gram(hipStream_t s, double* A, int64_t lda, int64_t Np, int nt, int64_t N, int64_t M, int mt,
                       const double* X, int64_t ldx, const double* Xs, int64_t ldxs, const TermPack* dtp);
// After the factorisation: mean_j = sum_k V^T[j,k] z_k, var_j = kdiag(xs_j) - sum_k V^T[j,k]^2
// (partial: 2 * ceil(N/512) * M doubles).
void launch_posterior(hipStream_t s, const double* A, int64_t lda, int64_t Np, int64_t N, int64_t M,
                      const double* Xs, int64_t ldxs, const TermPack* dtp, double* partial, double* mean,
                      double* var);
// ---- rand(FiniteGP): out = L z over the factor's lower triangle (partial: ceil(N/512) * N) ----
void launch_lower_mv(hipStream_t s, const double* A, int64_t lda, int64_t N, const double* z, double* partial,
                     double* out);
// The same tiles of M = -C^{-1} contracted in place (never stored) with every dC/dtheta:
// partial as launch_grad_contract's; alpha must be final before the launch; formulas whose
// groups are all single terms only.
void launch_cinv_contract(hipStream_t s, const double* A, int64_t lda, int64_t Np, int64_t N, const double* X,
                          int64_t ldx, const double* alpha, const TermPack* dtp, const uint32_t* list, int nblocks,
                          double* partial, KTime* kt);
// dparam[t] = 0.5 * sum over tiles (fixed order), t = 0..T (T = observation variance).
void launch_grad_reduce(hipStream_t s, const double* partial, int ntiles, int T, double* out);
// Workgroup -> tile list for launch_grad_tiles over the m x m triangle (XCD-balanced).
void build_grad_list(int m, std::vector<uint32_t>& out);

}  // namespace gaplac
