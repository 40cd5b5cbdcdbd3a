// Host side of libgaplac_hip.so: the C-ABI declared in include/gaplac.h.
//
// One evaluation = Gram build + blocked right-looking Cholesky of the (N+1)-augmented
// matrix with one-panel lookahead + logdet/quad reduction:
//
//   s_main : gram | wait(P0) syrk_tri(2..) rec(R0) | wait(P1) syrk_tri(3..) rec(R1) | ...
//   s_panel:        potrf(0) trsm(0) rec(P0) | syrk_col(1) potrf(1) trsm(1) rec(P1) |
//                   wait(R0) syrk_col(2) potrf(2) trsm(2) rec(P2) | ...
// (details at factor_and_reduce)
#include "gaplac_internal.h"

#include <cstddef>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

using namespace gaplac;

struct gaplac_ctx {
    int device = 0;
    hipStream_t s_main = nullptr, s_panel = nullptr;
    hipStream_t s_extra = nullptr;  // extra rows (gradient / posterior), beside the bulk updates
    hipStream_t s_xrest = nullptr;  // extra rows: their updates beyond the next SP
    hipEvent_t ev_xinit = nullptr, ev_xdone = nullptr;
    hipEvent_t ev_xc[2] = {}, ev_xr[2] = {};  // extra rows: SP chain done (s_extra), SP rest done (s_xrest)
    hipEvent_t ev_P[2] = {}, ev_R[2] = {}, ev_gram = nullptr, ev_gram2 = nullptr;
    hipEvent_t ev_split[2] = {}, ev_rest[2] = {};  // split bulk updates (factor_and_reduce), ping-pong
    double* A = nullptr;
    size_t A_elems = 0;
    double* Dinv = nullptr;  // per diagonal block: 8 inverses of its 16x16 sub-blocks
    size_t Dinv_elems = 0;
    // Tile lists for the bulk trailing updates: the list for an m x m triangle is a
    // prefix-independent array, so one list per m, all packed: offset[m] into tiles.
    uint32_t* tiles = nullptr;
    size_t tiles_elems = 0;
    int tiles_nt = 0;
    std::vector<size_t> tile_off;
    // band lists (paired updates): tile columns 0 .. spw-1 of an m-row trailing matrix, rows
    // r >= c, rows outer; packed after the triangle lists, band_off[m] into tiles
    std::vector<size_t> band_off;
    double* dX = nullptr;
    size_t dX_elems = 0;
    double* dv = nullptr;
    size_t dv_elems = 0;
    EvalResult* dres = nullptr;
    EvalResult* hres = nullptr;  // pinned
    TermPack* dtp = nullptr;     // device copy of the term descriptor (read by gram_kernel)
    TermPack* htp = nullptr;     // pinned staging for it
    std::string err;
    // profiling: 1 = per-launch device timestamps (KTime slots, see kt_begin/kt_end);
    // 2 = hipEvents recorded on s_main around every bulk tile_syrk launch (eager launches),
    //     read back by gaplac_get_stats
    int prof_mode = 0;
    bool profiling = false;  // prof_mode == 1
    std::vector<hipEvent_t> evpool;
    struct EvPair {
        size_t i0;
        double flops, bytes;
        int kind;  // 0 bulk tile_syrk launch, 8 cinv_tile launch
    };
    std::vector<EvPair> evpairs;
    // Schedule switches, read once in gaplac_ctx_create; the defaults are
    // the measured best at N = 16384.
    bool serial = false;  // GAPLAC_SERIAL=1: one stream, no overlap (per-kernel timing)
    bool dry = false;     // host-only walk of the schedule (gaplac_plan_check): no HIP calls
    int spw = 4;          // GAPLAC_SPW: super-panel width in 128-column tiles (bulk K = 128 spw)
    int tail_s = 32;      // GAPLAC_TAIL_S: the last ~tail_s tile columns run serially on one stream
                          //   (default 48 with the persistent tail, 32 without)
    int pair_ext = 1;     // 1 = a deferring step also updates the band after next (§3.2)
    int band_tiles_m = 64;  // GAPLAC_BAND_TILES_M: bands of >= this many tile rows as whole tiles
    int grad_fused = 1;     // GAPLAC_GRAD_FUSED: -C^{-1} contracted inside cinv_contract_kernel (0: stored, then contracted)
    bool grad_singletons = true;  // the gradient's formula has single-term groups only (the fused path's case)
    int la_tiles_m = 120;   // the lookahead of >= this many tile rows as whole tiles (0: never)
    // GAPLAC_TAIL_SIM: the single-evaluation tail list ordered by a simulated schedule
    // (sim_order_tail_tasks); -1 = for tails of fewer than 80 tile columns (measured: T = 33
    // -4.4%, T = 65 -1.3%, T = 80 +0.3%), 0 never, 1 always
    int tail_sim = -1;
    int pair_m = 40;      // GAPLAC_PAIR_M: paired bulk updates while >= this many tile rows follow the band
    int pair_depth = 0;   // (plan checks only) super-panels per deferred bulk update (0: 4 from 256 tile
                          //   columns on, else 2; N = 65536 1439 -> 1427 ms, 16k 26.97 -> 27.14 ms at 3-4)
    int ncu = 256;        // compute units of the device
    bool tailk = true;    // GAPLAC_TAILK: the serial tail as one persistent dataflow launch (tail_kernel)
    TailCtl* tctl = nullptr;     // its completion counters (zeroed per launch)
    uint32_t* ttasks = nullptr;  // its task list for ttasks_T tile columns
    size_t ttasks_elems = 0;
    int ttasks_T = -1, ttasks_X = 0, ttasks_n = 0;
    bool ttasks_G = false;  // the list holds the Gram's tile tasks (gram_in_tail)
    std::string ttrace_path;     // GAPLAC_TAIL_TRACE: append per-task times of every tail launch here
    int tail_fault = -1;         // GAPLAC_TAIL_FAULT (tests only): skip this tail column's diagonal block
    unsigned long long* ttrace = nullptr;
    size_t ttrace_elems = 0;
    gaplac_stats stats{};
    struct Slot {
        int kind;  // 0 bulk syrk, 1 gram, 2 diag, 4 trsm, 5 column update, 6 small bulk
        double work;
        double bytes;  // kind 0: algorithmic HBM bytes
    };
    std::vector<Slot> slots;     // slots of the launches being enqueued
    KTime* dkt = nullptr;        // device slot array
    KTime* hkt = nullptr;        // pinned copy
    size_t kt_cap = 0;
    bool recording = false;      // assign slots while enqueuing
    // Batched select: models in flight on independent lanes (child contexts with their
    // own workspace and streams; they read the parent's uploaded X and v).
    std::vector<gaplac_ctx*> lanes;
    int batch_lanes = 2;           // GAPLAC_BATCH_LANES (measured at N=8192: 1 lane 138, 2 lanes 191, 3-6 lanes 161-187 evals/s)
    int tail_share = 1;            // lanes sharing the GPU (gaplac_logpdf_batch): tail grid = CUs / share
    int batch_w = 32;              // GAPLAC_BATCH_W: models per tail launch when the whole matrix is in the tail
    int batch_lag = -1;            // GAPLAC_BATCH_LAG: tile columns between consecutive models of a tail launch
                                   // (-1: 3/8 of the matrix's tile columns)
#ifndef GAPLAC_SINGLE_GROUP
#define GAPLAC_SINGLE_GROUP 2
#endif
#ifndef GAPLAC_BATCH_GROUP
#define GAPLAC_BATCH_GROUP 2
#endif
#ifndef GAPLAC_QUAD_LAST
#define GAPLAC_QUAD_LAST 24
#endif
    int batch_gw = 8, batch_near = 2;  // the batched tail's deep-task width and near distance (A/B: §3.4)
    // single evaluations: quadrant next-column updates in the last 24 tail columns (the
    // latency-bound end) and pipelined half-tile TRSMs; batched lists: whole tiles and
    // whole-tile TRSMs throughout (select: 258 -> 267 evals/s)
    // the batched-tail workspace (gaplac_logpdf_batch): batch_w matrices
    struct BatchWs {
        double* A = nullptr;
        size_t A_elems = 0;
        double* Dinv = nullptr;
        size_t Dinv_elems = 0;
        EvalResult* dres = nullptr;
        size_t dres_elems = 0;
        EvalResult* hres = nullptr;  // pinned
        TermPack* dtp = nullptr;
        size_t dtp_elems = 0;
        TermPack* htp = nullptr;  // pinned
        int host_cap = 0;
        TailCtl* ctl = nullptr;
        size_t ctl_elems = 0;
        uint32_t* tasks = nullptr;
        size_t tasks_elems = 0;
        int tasks_T = -1, tasks_B = 0, tasks_n = 0, tasks_lag = -1;
        hipEvent_t ev_gram = nullptr, ev_done = nullptr;  // Grams written (s_panel); launch retired (s_main)
        bool busy = false;                                // a launch on this set is in flight
        int m0 = 0, B = 0;                                // its models
    } bw[2];  // two sets: one launch's Grams overlap the previous launch's tail
    bool borrowed_inputs = false;  // dX / dv belong to the parent
    // Extra rows below the matrix, factored along (lda = Np + 128 xr_tiles):
    //   1 = identity rows E = [I 0] -> L^{-T} (gradient, gaplac_logpdf_grad)
    //   2 = K(xs, X) -> (L^{-1} K(X, xs))^T (posterior, gaplac_posterior_mean_var, §10)
    int xr_mode = 0;
    int xr_tiles = 0;
    int64_t xr_M = 0;       // mode 2: test points
    double* dXs = nullptr;  // mode 2: test inputs (ld M)
    size_t dXs_elems = 0;
    double* pmean = nullptr;
    double* pvar = nullptr;
    size_t pmv_elems = 0;
    // gradient: alpha, partial sums, the XCD-balanced C^{-1} tile list
    double* galpha = nullptr;
    size_t galpha_elems = 0;
    double* gdv = nullptr;
    size_t gdv_elems = 0;
    double* gz = nullptr;  // z (row N of the factor), contiguous: alpha's input beside cinv
    size_t gz_elems = 0;
    double* gpart = nullptr;
    size_t gpart_elems = 0;
    double* gout = nullptr;   // device: T+1 results
    double* hgout = nullptr;  // pinned copy
    GradTermPack* dgp = nullptr;
    GradTermPack* hgp = nullptr;  // pinned staging
    uint32_t* glist = nullptr;
    size_t glist_elems = 0;
    int glist_m = -1, glist_blocks = 0;
};

namespace {

int set_err(gaplac_ctx* ctx, int code, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
int set_err(gaplac_ctx* ctx, int code, const char* fmt, ...) {
    if (ctx) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        ctx->err = buf;
    }
    return code;
}

#define HIPCK(ctx, call)                                                                   \
    do {                                                                                   \
        hipError_t e_ = (call);                                                            \
        if (e_ != hipSuccess)                                                              \
            return set_err(ctx, GAPLAC_E_HIP, "%s failed: %s", #call, hipGetErrorString(e_)); \
    } while (0)

// HIP runtime calls of the schedule itself (events, waits, copies): skipped in a dry run.
#define HIPQ(ctx, call)                    \
    do {                                   \
        if (!(ctx)->dry) HIPCK(ctx, call); \
    } while (0)

int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

}  // namespace

// Validate terms and build the kernel-argument pack. Mirrors the argument checks of the
// KernelFunctions constructors GaPLAC calls (src/abstractgp_translations.jl:8-15):
// LinearKernel requires c >= 0; ScaleTransform(1/l) requires a positive finite scale.
static int pfail(std::string* err, int code, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
static int pfail(std::string* err, int code, const char* fmt, ...) {
    if (err) {
        char buf[256];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        *err = buf;
    }
    return code;
}

int gaplac::pack_terms(int32_t D, int32_t T, const gaplac_term* terms, TermPack* tp, std::string* err) {
#define fail(...) pfail(err, __VA_ARGS__)
    if (T < 0 || T > GAPLAC_MAX_TERMS) return fail(GAPLAC_E_KIND, "term count %d outside [0, %d]", T, GAPLAC_MAX_TERMS);
    if (T > 0 && !terms) return fail(GAPLAC_E_ARG, "terms is NULL");
    std::memset(tp, 0, sizeof *tp);
    tp->T = T;
    for (int t = 0; t < T; ++t) {
        const gaplac_term& x = terms[t];
        if (x.reserved != 0) return fail(GAPLAC_E_ARG, "term %d: reserved field not 0", t);
        // groups must be contiguous: a group id seen before must be the previous term's
        for (int u = 0; u + 1 < t; ++u)
            if (terms[u].group == x.group && terms[t - 1].group != x.group)
                return fail(GAPLAC_E_KIND, "term %d: product group %d not contiguous", t, x.group);
        tp->kind[t] = x.kind;
        tp->col[t] = x.col;
        switch (x.kind) {
            case GAPLAC_SQEXP:
            case GAPLAC_OU:
                if (!(x.param > 0.0) || !std::isfinite(x.param))
                    return fail(GAPLAC_E_PARAM, "term %d: lengthscale %g must be > 0", t, x.param);
                tp->p[t] = 1.0 / x.param;  // ScaleTransform(inv(l))
                if (!(tp->p[t] > 0.0)) return fail(GAPLAC_E_PARAM, "term %d: scale 1/l underflows", t);
                break;
            case GAPLAC_LINEAR:
                if (!(x.param >= 0.0) || !std::isfinite(x.param))
                    return fail(GAPLAC_E_PARAM, "term %d: c = %g must be >= 0", t, x.param);
                tp->p[t] = x.param;
                break;
            case GAPLAC_CAT:
                tp->p[t] = 0.0;
                break;
            case GAPLAC_NOISE:
                if (!(x.param >= 0.0) || !std::isfinite(x.param))
                    return fail(GAPLAC_E_PARAM, "term %d: noise variance %g must be >= 0", t, x.param);
                tp->p[t] = x.param;
                tp->col[t] = 0;
                break;
            default:
                return fail(GAPLAC_E_KIND, "term %d: unknown kind %d", t, x.kind);
        }
        if (x.kind != GAPLAC_NOISE && (x.col < 0 || x.col >= D))
            return fail(GAPLAC_E_COL, "term %d: column %d outside [0, %d)", t, x.col, D);
        tp->last_in_group[t] = (t == T - 1 || terms[t + 1].group != x.group) ? 1 : 0;
    }
#undef fail
    return 0;
}

namespace {

int pack_terms(gaplac_ctx* ctx, int32_t D, int32_t T, const gaplac_term* terms, TermPack* tp) {
    return gaplac::pack_terms(D, T, terms, tp, ctx ? &ctx->err : nullptr);
}

int check_common(gaplac_ctx* ctx, int64_t N, int32_t D, const void* X, int64_t ldx, double noise,
                 const void* v) {
    if (!ctx) return GAPLAC_E_ARG;
    if (N < 0) return set_err(ctx, GAPLAC_E_ARG, "N = %lld < 0", (long long)N);
    if (N > 0 && D > 0 && (!X || ldx < N))
        return set_err(ctx, GAPLAC_E_ARG, "X NULL or ldx %lld < N %lld", (long long)ldx,
                       (long long)N);
    if (N > 0 && !v) return set_err(ctx, GAPLAC_E_ARG, "v is NULL");
    if (D < 0) return set_err(ctx, GAPLAC_E_ARG, "D = %d < 0", D);
    if (!(noise >= 0.0) || !std::isfinite(noise))
        return set_err(ctx, GAPLAC_E_PARAM, "noise %g must be finite and >= 0", noise);
    return 0;
}

template <typename T>
int ensure(gaplac_ctx* ctx, T** p, size_t* cap, size_t n) {
    if (*cap >= n) return 0;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc(reinterpret_cast<void**>(p), n * sizeof(T)) != hipSuccess)
        return set_err(ctx, GAPLAC_E_OOM, "hipMalloc of %zu bytes failed", n * sizeof(T));
    *cap = n;
    return 0;
}

// Profiling slot for the next launch (nullptr when profiling is off).
KTime* slot(gaplac_ctx* ctx, int kind, double work, double bytes = 0.0) {
    if (!ctx->recording) return nullptr;
    const size_t i = ctx->slots.size();
    if (i >= ctx->kt_cap) return nullptr;
    ctx->slots.push_back({kind, work, bytes});
    return ctx->dkt + i;
}

// Algorithmic flops of one bulk trailing-update launch per 128 of K: lower triangle
// (incl. diagonal) of the m x m tile triangle, 2 flops per multiply-add.
double syrk_flops(int m) {
    const double nbd = NB;
    const double rows = (double)m * nbd;
    return 2.0 * nbd * rows * (rows + 1) / 2.0;
}

// Algorithmic HBM bytes of one bulk trailing-update launch over the m x m tile triangle
// with K = kd: every C tile read and written once, the m*NB panel rows read once.
double syrk_bytes(int m, int kd) {
    const double tiles = (double)m * (m + 1) / 2.0;
    return tiles * NB * NB * 8.0 * 2.0 + (double)m * NB * kd * 8.0;
}

// Algorithmic flops of a band launch: the W tile columns of an mbd-row trailing matrix
// (rows r >= c), K = kd: W diagonal tiles (lower triangle incl. diagonal), the rest whole.
double band_flops(int mbd, int W, int kd) {
    const int w = std::min(W, mbd);
    const double tiles = (double)w * mbd - (double)w * (w - 1) / 2.0;
    return (tiles - w) * 2.0 * NB * NB * kd + (double)w * NB * (NB + 1) * kd;
}

// Fold the device timestamps of the given slots into ctx->stats (ticks: 100 MHz).
int accumulate_slots(gaplac_ctx* ctx, const std::vector<gaplac_ctx::Slot>& slots) {
    if (slots.empty()) return 0;
    HIPCK(ctx, hipMemcpy(ctx->hkt, ctx->dkt, slots.size() * sizeof(KTime), hipMemcpyDeviceToHost));
    unsigned long long t0 = ~0ull, t1 = 0;
    for (size_t i = 0; i < slots.size(); ++i) {
        const KTime& t = ctx->hkt[i];
        if (t.end < t.start || t.start == ~0ull) continue;
        const double ms = (double)(t.end - t.start) * 1e-5;
#if defined(GAPLAC_CLOCK) && GAPLAC_CLOCK
        if (t.clk_rt > 0)  // diagnostic build: the clock each bulk launch held
            std::fprintf(stderr, "clk slot %zu kind %d %.3f ms %.3f GHz, %llu workgroups, %.0f cycles each\n", i,
                         slots[i].kind, ms, (double)t.clk_mt / (double)t.clk_rt * 0.1, t.clk_n,
                         (double)t.clk_mt / (double)std::max(1ull, t.clk_n));
#endif
        t0 = std::min(t0, t.start);
        t1 = std::max(t1, t.end);
        switch (slots[i].kind) {
            case 0:
                ctx->stats.syrk_ms += ms;
                ctx->stats.syrk_flops += slots[i].work;
                ctx->stats.syrk_launches += 1;
                ctx->stats.syrk_bytes += slots[i].bytes;
                break;
            case 6:
                ctx->stats.small_ms += ms;
                ctx->stats.small_launches += 1;
                break;
            case 7:
                ctx->stats.grad_rows_ms += ms;
                break;
            case 8:
                ctx->stats.cinv_ms += ms;
                ctx->stats.cinv_launches += 1;
                break;
            case 9:
                ctx->stats.contract_ms += ms;
                break;
            case 10:
                ctx->stats.tail_ms += ms;
                ctx->stats.tail_launches += 1;
                break;
            case 1:
                ctx->stats.gram_ms += ms;
                ctx->stats.gram_bytes += slots[i].work;
                ctx->stats.gram_launches += 1;
                break;
            case 2:
                ctx->stats.panel_ms += ms;
                break;
            case 4:
                ctx->stats.trsm_ms += ms;
                break;
            default:
                ctx->stats.colupd_ms += ms;
                break;
        }
    }
    if (t1 > t0) ctx->stats.total_ms += (double)(t1 - t0) * 1e-5;
    ctx->stats.evals += 1;
    return 0;
}

// Factor the augmented matrix already built in ctx->A (Gram launched on s_main).
//
// Super-panels of W 128-wide tile columns (SP p covers tile columns pW .. pW+W-1,
// GAPLAC_SPW, default 4): the panel chain factors 128-wide blocks, the bulk trailing
// update applies a whole super-panel at once (K = 128 W). Measured per 128x128 tile:
// ~10 us fixed (C load, first staging, epilogue) + K at the MFMA ceiling, so larger K
// amortises the fixed part (and cuts C-tile HBM traffic per flop by W).
//
// Two streams, eager launches. s_panel (highest priority, all CUs) runs the critical path
// in order; s_main (lowest priority) runs the Gram and the bulk updates. Super-panel
// boundaries come from superpanel_starts() (width spw; the last ~tail_s tile columns are
// factored by serial_tail() on s_main alone).
//   s_panel: wait R(p-1) | col_update(columns of SP p+1, with SP p, K=128W)
//            | for each column c of SP p+1: [col_update(c with c-1..first, K=128)] potrf(c) trsm(c)
//            | rec P(p+1)
//   s_main : wait P(p)   | syrk_tri(tile columns >= (p+2)W, with SP p, K=128W) | rec R(p)
// Within SP p+1 the chain is right-looking with K=128 column updates (each column gets
// the previous columns of its own super-panel). Columns of SP p+1 receive SP p-1 in
// R(p-1) and SP p in the lookahead col_update; within a step the streams touch disjoint
// tile columns. Events ping-pong (p & 1).
// GAPLAC_CHAIN_SKIP (-D, timing diagnostics only: the result is void): 1 = the super-panel
// chain's column updates, diagonal blocks and TRSMs are not launched, 2 = nor the
// lookahead; what the evaluation costs without the chain's CU share and latency.
#ifndef GAPLAC_CHAIN_SKIP
#define GAPLAC_CHAIN_SKIP 0
#endif
int factor_superpanel(gaplac_ctx* ctx, hipStream_t sp, int64_t N, int64_t lda, int nt, int c0, int c1) {
    if (GAPLAC_CHAIN_SKIP >= 1 && !ctx->dry) return 0;
    for (int c = c0; c < c1; ++c) {
        double* Acol = ctx->A + (int64_t)c * NB * lda;
        if (c > c0)
            launch_col_update(sp, ctx->A, lda, Panel{Acol - NB * lda, lda, 0}, nt, c, c, c1 - c, NB,
                              slot(ctx, 5, 0));
        double* Dk = ctx->Dinv + (size_t)c * DINV_PER_BLOCK;
        if ((int64_t)c * NB < N)
            launch_potrf_diag(sp, Acol + (int64_t)c * NB, lda, N, (int64_t)c * NB, Dk, ctx->dres, slot(ctx, 2, 0));
        launch_trsm(sp, Acol, lda, nt, c, Dk, slot(ctx, 4, 0));
    }
    return 0;
}

// Extra rows, tile rows nt .. nt + xr_tiles - 1 of the column storage,
// factored along on s_main, off the critical path: once SP p's columns are final (P(p)),
// its extra-row tiles get the column-by-column substitution (the earlier columns of the SP
// applied first, K = 128), then SP p is applied to every later column (K = 128 W).
// Identity rows (gradient): only rows E <= c of column c are nonzero (Y = L^{-T} is upper
// triangular), so each step touches rows [0, c] / [0, end of SP); tiles below Y's diagonal
// stay exactly zero and are never written. Cross-covariance rows (posterior): all rows.
// extra-row updates of at least this many tiles run as whole 128x128 tiles (tile_syrk_kernel),
// not quadrants: gradient 79.4 -> 78.0 ms with the split below (profiles/r04r_xr_ab.txt)
constexpr int XR_TILE_MIN = 128;

static void extra_rows_chain(gaplac_ctx* ctx, hipStream_t sm, int64_t lda, int nt, int c0, int c1) {
    const int W = ctx->spw;
    const bool tri = ctx->xr_mode == 1;
    const int mt = ctx->xr_tiles;
    for (int c = c0; c < c1; ++c) {
        double* Acol = ctx->A + (int64_t)c * NB * lda;
        if (c > c0) {
            const int rows = tri ? c : mt;
            BulkArgs ba{ctx->A, lda, Panel{Acol - NB * lda, lda, 0}, nullptr, rows * (c1 - c), NB, nt, c,
                        ColMap{1, 0, W}};
            ba.rect_rows = rows;
            ba.tile_min = XR_TILE_MIN;
            launch_bulk(sm, ba, slot(ctx, 7, 0));
        }
        launch_trsm_rows(sm, Acol, lda, c, nt, tri ? c + 1 : mt, ctx->Dinv + (size_t)c * DINV_PER_BLOCK,
                         slot(ctx, 7, 0));
    }
}

// SP [c0, c1)'s extra-row tiles applied to tile columns [jb, je) of the extra rows (K = 128 W)
static void extra_rows_update(gaplac_ctx* ctx, hipStream_t sm, int64_t lda, int nt, int c0, int c1, int jb,
                              int je) {
    if (je <= jb) return;
    const int rows = ctx->xr_mode == 1 ? c1 : ctx->xr_tiles;
    BulkArgs ba{ctx->A, lda, Panel{ctx->A + (int64_t)c0 * NB * lda, lda, 0}, nullptr, rows * (je - jb),
                (c1 - c0) * NB, nt, jb, ColMap{1, 0, ctx->spw}};
    ba.rect_rows = rows;
    ba.tile_min = XR_TILE_MIN;
    launch_bulk(sm, ba, slot(ctx, 7, 0));
}

// Super-panel boundaries: tile columns sp[p] .. sp[p+1]-1 form SP p, width spw. With a
// serial tail (tail_s > 0, plain logpdf) the list stops at the first boundary with at
// most tail_s tile columns after it; those columns are factored by serial_tail().
// The whole matrix in the persistent tail (no super-panels): plain logpdf with at most
// tail_s (and TAIL_TMAX) tile columns.
// Which evaluations take a tail: plain logpdf, and the posterior when its cross-covariance
// rows fit beside the tail's columns (the persistent tail factors them along, §10); the
// gradient's identity rows (one per column) never do.
static bool tail_allowed(const gaplac_ctx* ctx) {
    return ctx->xr_mode == 0 || (ctx->xr_mode == 2 && ctx->tailk && ctx->tail_s > 0 &&
                                 ctx->xr_tiles + std::min(ctx->tail_s, TAIL_TMAX) <= TAIL_TMAX);
}

static bool whole_in_tail(const gaplac_ctx* ctx, int nt) {
    return tail_allowed(ctx) && ctx->tailk && ctx->tail_s > 0 && nt <= TAIL_TMAX && nt <= ctx->tail_s;
}

// The Gram inside the tail (TAIL_G tasks, -D GAPLAC_TAIL_GRAM=0 turns it off): a plain
// single evaluation whose matrix lies whole in the tail builds its Gram tiles as the tail's
// first tasks instead of in two launches before it (N = 4096: the Gram launches, their gaps
// and the tail's start behind them were ~50 us of the 1.15 ms evaluation).
// Needs the tile stores' buffer offsets (< 2^31 bytes per tile column span).
#ifndef GAPLAC_TAIL_GRAM
#define GAPLAC_TAIL_GRAM 1
#endif
static bool gram_in_tail(const gaplac_ctx* ctx, int nt, int64_t lda) {
    return GAPLAC_TAIL_GRAM && ctx->xr_mode == 0 && whole_in_tail(ctx, nt) &&
           ((int64_t)(NB - 1) * lda + NB) * 8 < ((int64_t)1 << 31);
}

// The term descriptor reaches ctx->dtp through the evaluation's first launch
// (init_result_ctl_kernel, when the Gram is inside the tail) instead of a copy.
static bool tp_by_init(const gaplac_ctx* ctx, int64_t N) {
    const int64_t Np = round_up(N + 1, NB);
    return gram_in_tail(ctx, (int)(Np / NB), Np + (int64_t)NB * ctx->xr_tiles);
}

static std::vector<int> superpanel_starts(const gaplac_ctx* ctx, int nt) {
    std::vector<int> sp{0};
    // a matrix the persistent tail covers whole (plain logpdf, at most TAIL_TMAX tile
    // columns, within tail_s): no super-panel at all, every column in the tail kernel
    if (whole_in_tail(ctx, nt)) return sp;
    int c = 0;
    while (c < nt) {
        if (tail_allowed(ctx) && ctx->tail_s > 0 && c > 0 && nt - c <= ctx->tail_s) break;
        c = std::min(c + ctx->spw, nt);
        sp.push_back(c);
    }
    return sp;
}

// Serial tail: tile columns ts .. nt-1 factored right-looking on one stream,
// after the bulk update that applied the last super-panel to them: per column the whole
// remaining triangle gets the previous column (K = 128), then the diagonal block and the
// TRSM. No events: in the chain-bound tail every event record or cross-stream wait costs
// ~6-12 us of dispatch latency on the critical path, more than the small updates save by
// overlapping.
static void serial_tail(gaplac_ctx* ctx, hipStream_t sm, int64_t N, int64_t lda, int nt, int ts) {
    for (int c = ts; c < nt; ++c) {
        double* Acol = ctx->A + (int64_t)c * NB * lda;
        if (c > ts) {
            const int m = nt - c;
            BulkArgs ba{ctx->A, lda, Panel{Acol - NB * lda, lda, 0}, ctx->tiles + ctx->tile_off[(size_t)m],
                        m * (m + 1) / 2, NB, c, c, ColMap{1, 0, ctx->spw}};
            launch_bulk(sm, ba, slot(ctx, 6, 0));
        }
        double* Dk = ctx->Dinv + (size_t)c * DINV_PER_BLOCK;
        if ((int64_t)c * NB < N)
            launch_potrf_diag(sm, Acol + (int64_t)c * NB, lda, N, (int64_t)c * NB, Dk, ctx->dres, slot(ctx, 2, 0));
        launch_trsm(sm, Acol, lda, nt, c, Dk, slot(ctx, 4, 0));
    }
}

// Paired bulk updates (GAPLAC_PAIR_M): does step p defer its bulk update
// (only the next-needed bands get SP p; the columns after them get SPs p and p+1 together
// at step p+1)? pend: the super-panel still pending (-1: none).
static bool pair_defer(const gaplac_ctx* ctx, const std::vector<int>& spc, int nt, int p, int pend) {
    const int nsp = (int)spc.size() - 1;
    const int jb = p + 2 <= nsp ? spc[(size_t)p + 2] : spc[(size_t)nsp];
    const int je = p + 3 <= nsp ? spc[(size_t)p + 3] : spc[(size_t)nsp];
    const int depth = ctx->pair_depth > 0 ? ctx->pair_depth : nt >= 256 ? 4 : 2;
    return ctx->pair_m > 0 && (pend < 0 || p - pend + 1 < depth) && !ctx->serial && !ctx->xr_mode && je > jb &&
           p + 1 + ctx->pair_ext < nsp &&
           p + 3 + ctx->pair_ext <= nsp && nt - spc[(size_t)p + 3 + ctx->pair_ext] >= ctx->pair_m;
}

// Latency-shaped (quadrant) columns of a single evaluation's tail: with the simulated
// order a tail of at most 40 tile columns takes them in every column (N = 4096: -2%; at T =
// 65 all columns cost +4%, 40 of them +1.5%), else the last GAPLAC_QUAD_LAST.
static int tail_quad_last(bool sim, int T) { return sim && T <= 40 ? TAIL_TMAX : GAPLAC_QUAD_LAST; }

// Deep-task width of a single evaluation's tail: 4 columns (K = 512), or 8 (K = 1024) for
// tails of at least GAPLAC_GW8_T tile columns (-D; A/B switch).
#ifndef GAPLAC_GW8_T
#define GAPLAC_GW8_T 1000
#endif
static int tail_gw(int T) { return T >= GAPLAC_GW8_T ? 8 : 4; }

}  // namespace
namespace gaplac {
// The single-evaluation tail list of T tile columns (X extra tile rows), as eval_device
// launches it; also the distributed root's gathered tail (gaplac_dist.hip). tail_sim as
// gaplac_ctx::tail_sim; workers: the persistent grid the simulated order plans for.
void build_single_tail_list(int T, int X, int tail_sim, int workers, std::vector<uint32_t>& out, bool gram) {
    const bool sim = (tail_sim > 0 || (tail_sim < 0 && T < 80)) && X == 0;
    out.clear();
    build_tail_tasks(T, out, nullptr, tail_gw(T), 4, tail_quad_last(sim, T), false, GAPLAC_SINGLE_GROUP, X, sim ? 1 : 0);
    if (sim && workers > 0) sim_order_tail_tasks(T, out, workers);
    if (gram && X == 0) add_gram_tasks(T, out);
}
}  // namespace gaplac
namespace {

// Split bulk updates (GAPLAC_SPLIT, -D): plain evaluations whose
// super-panel phase defers in pairs (depth 2); a triangle launch is split only when its
// rest keeps at least SPLIT_REST_MIN tile columns.
#ifndef GAPLAC_SPLIT
#define GAPLAC_SPLIT 1
#endif
constexpr int SPLIT_REST_MIN = 16;
#ifndef GAPLAC_SPLIT_MINCOLS
#define GAPLAC_SPLIT_MINCOLS 32
#endif
#ifndef GAPLAC_SPLIT_DEPTH
#define GAPLAC_SPLIT_DEPTH 2  // deferral depths the split applies to (the head is depth x W columns)
#endif
static bool split_wanted(const gaplac_ctx* ctx, int nt) {
    const int depth = ctx->pair_depth > 0 ? ctx->pair_depth : nt >= 256 ? 4 : 2;
    const std::vector<int> spc = superpanel_starts(ctx, nt);  // (a short super-panel phase: not worth it)
    return GAPLAC_SPLIT && ctx->xr_mode == 0 && !ctx->serial && depth <= GAPLAC_SPLIT_DEPTH &&
           !whole_in_tail(ctx, nt) && spc.back() >= GAPLAC_SPLIT_MINCOLS;
}
static bool split_bulk(const gaplac_ctx* ctx, int nt) {
    return split_wanted(ctx, nt) && (ctx->s_xrest != nullptr || ctx->dry);
}

int factor_and_reduce(gaplac_ctx* ctx, int64_t N, int64_t lda, int nt) {
    hipStream_t sm = ctx->s_main;
    hipStream_t sp = ctx->serial ? sm : ctx->s_panel;
    const int W = ctx->spw;
    const std::vector<int> spc = superpanel_starts(ctx, nt);
    const int nsp = (int)spc.size() - 1;
    int frc;
    // Split bulk updates (split_bulk): a bulk update's first 2W tile columns
    // (what the next steps' bands read) stay on s_main, the rest goes to s_xrest, so the
    // next steps' small band launches run beside it instead of after it. rest_from: first
    // tile column of the rest still in flight there; every later launch that reaches it
    // waits for ev_rest first (on its own stream).
    const bool split = split_bulk(ctx, nt);
    hipStream_t sr = ctx->s_xrest;
    int rest_from = nt + 1, nsplit = 0;
    auto wait_rest = [&](hipStream_t st, int col_end) {
        if (col_end <= rest_from) return 0;
        HIPQ(ctx, hipStreamWaitEvent(st, ctx->ev_rest[(nsplit - 1) & 1], 0));
        if (st == sm) rest_from = nt + 1;  // s_main is past it for good (s_panel waits behind s_main's marks)
        return 0;
    };
    if (nsp > 0) {
        HIPQ(ctx, hipStreamWaitEvent(sp, ctx->ev_gram, 0));  // first W tile columns built
        if ((frc = factor_superpanel(ctx, sp, N, lda, nt, spc[0], spc[1]))) return frc;
        HIPQ(ctx, hipEventRecord(ctx->ev_P[0], sp));
    }
    // profiling mode 2: hipEvents around a band-type bulk launch (whole-tile bands, heads and
    // lookaheads: kind 5) on its stream, for the bulk phase's union of launch intervals
    auto band_launch = [&](hipStream_t st, const BulkArgs& bb, int mbd) {
        const bool ev = ctx->prof_mode == 2 && bb.whole && !ctx->xr_mode;
        size_t e0 = 0;
        if (ev) {
            e0 = 2 * ctx->evpairs.size();
            while (ctx->evpool.size() < e0 + 2) {
                hipEvent_t e;
                HIPQ(ctx, hipEventCreate(&e));
                ctx->evpool.push_back(e);
            }
            HIPQ(ctx, hipEventRecord(ctx->evpool[e0], st));
        }
        launch_bulk(st, bb, slot(ctx, 5, 0));
        if (ev) {
            HIPQ(ctx, hipEventRecord(ctx->evpool[e0 + 1], st));
            ctx->evpairs.push_back({e0, band_flops(mbd, W, bb.kdepth), 0.0, 5});
        }
        return 0;
    };
    // bulk trailing update of the triangle of tile columns >= j0 with the panel pn (K = kd)
    auto bulk_tri = [&](int j0, const Panel& pn, int kdep) -> int {
        if (j0 >= nt) return 0;
        wait_rest(sm, nt);
        int jr = j0;  // first tile column of the triangle launch (after the head)
        hipStream_t st = sm;
        const int hw = (ctx->pair_depth > 0 ? ctx->pair_depth : nt >= 256 ? 4 : 2) * W;  // head width
        if (split && nt - j0 >= hw + SPLIT_REST_MIN && ctx->band_off.size() > (size_t)(nt - j0)) {
            // what s_main holds so far (this step's panel wait, earlier updates) before the rest
            HIPQ(ctx, hipEventRecord(ctx->ev_split[nsplit & 1], sm));
            // head: tile columns [j0, j0 + hw) as band launches (whole tiles) on s_main
            for (int b0 = j0; b0 < j0 + hw; b0 += W) {
                const int mbd = nt - b0;
                BulkArgs bb{ctx->A, lda, pn, ctx->tiles + ctx->band_off[(size_t)mbd], W * mbd - W * (W - 1) / 2, kdep,
                            b0, b0, ColMap{1, 0, W}};
                bb.max_r = mbd - 1;
                bb.max_c = W - 1;
                bb.whole = 1;
                band_launch(sm, bb, mbd);
            }
            jr = j0 + hw;
            st = sr;
            HIPQ(ctx, hipStreamWaitEvent(sr, ctx->ev_split[nsplit & 1], 0));
        }
        const int m = nt - jr;
        BulkArgs ba{ctx->A, lda, pn, ctx->tiles + ctx->tile_off[(size_t)m], m * (m + 1) / 2, kdep, jr, jr,
                    ColMap{1, 0, W}};
        const bool small = syrk_is_small(ba.ntiles);
        const double fl = syrk_flops(m) * (kdep / NB), by = syrk_bytes(m, kdep);
        KTime* kt = small ? slot(ctx, 6, 0) : slot(ctx, 0, fl, by);
        const bool ev = ctx->prof_mode == 2 && !small;
        size_t e0 = 0;
        if (ev) {
            e0 = 2 * ctx->evpairs.size();
            while (ctx->evpool.size() < e0 + 2) {
                hipEvent_t e;
                HIPQ(ctx, hipEventCreate(&e));
                ctx->evpool.push_back(e);
            }
            HIPQ(ctx, hipEventRecord(ctx->evpool[e0], st));
        }
        launch_bulk(st, ba, kt);
        if (ev) {
            HIPQ(ctx, hipEventRecord(ctx->evpool[e0 + 1], st));
            ctx->evpairs.push_back({e0, fl, by, 0});
        }
        if (st == sr) {
            HIPQ(ctx, hipEventRecord(ctx->ev_rest[nsplit & 1], sr));
            ++nsplit;
            rest_from = jr;
        }
        return 0;
    };
    int pend = -1;  // the super-panel not yet applied to the columns >= dcol (paired updates)
    int dcol = nt;
    for (int p = 0; p < nsp; ++p) {
        const int c0 = spc[(size_t)p], c1 = spc[(size_t)p + 1];
        const int kd = (c1 - c0) * NB;  // depth of super-panel p
        if (p + 1 < nsp) {
            if (p >= 1)
                HIPQ(ctx, hipStreamWaitEvent(sp, ctx->ev_R[(p - 1) & 1], 0));
            else
                HIPQ(ctx, hipStreamWaitEvent(sp, ctx->ev_gram2, 0));  // rest of the Gram built
            const int c2 = spc[(size_t)p + 2];
            wait_rest(sp, c2);  // (SP p+1's columns in a split update's rest still in flight)
            const int mla = nt - c1;
            if (GAPLAC_CHAIN_SKIP >= 2 && !ctx->dry) {
            } else if (ctx->la_tiles_m > 0 && mla >= ctx->la_tiles_m && c2 - c1 == W && ctx->band_off.size() > (size_t)mla &&
                       !ctx->xr_mode) {
                // the lookahead as whole 128x128 tiles (the band list of SP p+1's columns):
                // less CU time than the quadrant kernel while the trailing matrix is large
                BulkArgs ba{ctx->A, lda, Panel{ctx->A + (int64_t)c0 * NB * lda, lda, 0},
                            ctx->tiles + ctx->band_off[(size_t)mla], W * mla - W * (W - 1) / 2, kd, c1, c1,
                            ColMap{1, 0, W}};
                ba.max_r = mla - 1;
                ba.max_c = W - 1;
                ba.whole = 1;
                band_launch(sp, ba, mla);
            } else {
                launch_col_update(sp, ctx->A, lda, Panel{ctx->A + (int64_t)c0 * NB * lda, lda, 0}, nt, c1, c1,
                                  c2 - c1, kd, slot(ctx, 5, 0));
            }
            if ((frc = factor_superpanel(ctx, sp, N, lda, nt, c1, c2))) return frc;
            HIPQ(ctx, hipEventRecord(ctx->ev_P[(p + 1) & 1], sp));
        }
        HIPQ(ctx, hipStreamWaitEvent(sm, ctx->ev_P[p & 1], 0));
        // tile columns after SP p+1; the last super-panel also updates a serial tail
        const int jb = p + 2 <= nsp ? spc[(size_t)p + 2] : spc[(size_t)nsp];
        // Paired bulk updates (GAPLAC_PAIR_M): at a deferring step only the next-needed band
        // (SP p+2's columns; with GAPLAC_PAIR_EXT also SP p+3's) gets SP p, and the tile
        // columns after it get SPs p and p+1 in one K = 2 x 128W update at step p+1 (band
        // first, then R(p), then the rest). Columns >= dcol lack SP pend.
        const int je = p + 3 <= nsp ? spc[(size_t)p + 3] : spc[(size_t)nsp];
        const bool defer = pair_defer(ctx, spc, nt, p, pend);
        // a band [b0, b1) with the panel columns pc .. c1-1
        auto band = [&](int b0, int b1, int pc) {
            if (b1 <= b0) return;
            wait_rest(sm, b1);
            const Panel pn{ctx->A + (int64_t)pc * NB * lda, lda, 0};
            const int kb = (c1 - pc) * NB, mbd = nt - b0;
            if (b1 - b0 == W && ctx->band_off.size() > (size_t)mbd) {
                // through the tile kernel (a list of the band's tiles; quadrants if small)
                BulkArgs ba{ctx->A, lda, pn, ctx->tiles + ctx->band_off[(size_t)mbd], W * mbd - W * (W - 1) / 2, kb,
                            b0, b0, ColMap{1, 0, W}};
                ba.max_r = mbd - 1;
                ba.max_c = W - 1;
                ba.whole = mbd >= ctx->band_tiles_m ? 1 : 0;
                band_launch(sm, ba, mbd);
            } else {
                launch_col_update(sm, ctx->A, lda, pn, nt, b0, b0, b1 - b0, kb, slot(ctx, 5, 0));
            }
        };
        // first panel column a band starting at tile column b0 still lacks: columns >= dcol
        // lack every super-panel from pend on, the others only this step's
        auto first_panel = [&](int b0) { return pend >= 0 && b0 >= dcol ? spc[(size_t)pend] : c0; };
        if (defer && pend >= 0) {
            // a deeper deferral (GAPLAC_PAIR_DEPTH > 2): the next-needed band gets this
            // step's panel, the band after it every panel from pend on
            band(jb, je, first_panel(jb));
            HIPQ(ctx, hipEventRecord(ctx->ev_R[p & 1], sm));
            const int e1 = ctx->pair_ext > 0 ? spc[(size_t)p + 4] : je;
            if (je < e1) band(je, e1, first_panel(je));
            dcol = std::max(dcol, e1);
        } else if (defer) {
            band(jb, je, c0);
            HIPQ(ctx, hipEventRecord(ctx->ev_R[p & 1], sm));
            dcol = je;
            if (ctx->pair_ext > 0) {
                dcol = spc[(size_t)p + 4];
                band(je, dcol, c0);
            }
            pend = p;
        } else if (pend >= 0) {
            band(jb, je, je <= dcol ? c0 : spc[(size_t)pend]);
            HIPQ(ctx, hipEventRecord(ctx->ev_R[p & 1], sm));
            if (je < dcol) band(je, dcol, c0);  // (not produced by the schedule above)
            const Panel pnl{ctx->A + (int64_t)spc[(size_t)pend] * NB * lda, lda, 0};
            if ((frc = bulk_tri(std::max(je, dcol), pnl, (c1 - spc[(size_t)pend]) * NB))) return frc;
            pend = -1;
        } else {
            if ((frc = bulk_tri(jb, Panel{ctx->A + (int64_t)c0 * NB * lda, lda, 0}, kd))) return frc;
            HIPQ(ctx, hipEventRecord(ctx->ev_R[p & 1], sm));
        }
        if (ctx->xr_mode) {
            // extra rows: they only need SP p final (P(p)) and touch rows no other stream
            // writes. s_extra takes SP p's column chain and then its update of SP p+1's
            // columns; the update of the columns after those (the bulk of the K = 128 W work)
            // goes on s_xrest, so the chain of SP p+1 runs beside it instead of after it
            // (DESIGN.md §9). Every tile still gets the SPs in order: the update of SP p+1's
            // columns waits for SP p-1's update of the columns after SP p, SP p's chain for
            // SP p-2's.
            hipStream_t sx = ctx->serial ? sm : ctx->s_extra;
            if (sx == sm) {
                extra_rows_chain(ctx, sx, lda, nt, c0, c1);
                extra_rows_update(ctx, sx, lda, nt, c0, c1, c1, nt);
            } else {
                hipStream_t sr = ctx->s_xrest;
                if (p >= 1) {  // SP p-1 on the columns after SP p
                    HIPQ(ctx, hipStreamWaitEvent(sr, ctx->ev_xc[(p - 1) & 1], 0));
                    extra_rows_update(ctx, sr, lda, nt, spc[(size_t)p - 1], c0, c1, nt);
                    HIPQ(ctx, hipEventRecord(ctx->ev_xr[(p - 1) & 1], sr));
                }
                HIPQ(ctx, hipStreamWaitEvent(sx, ctx->ev_P[p & 1], 0));
                if (p >= 2) HIPQ(ctx, hipStreamWaitEvent(sx, ctx->ev_xr[(p - 2) & 1], 0));
                extra_rows_chain(ctx, sx, lda, nt, c0, c1);
                HIPQ(ctx, hipEventRecord(ctx->ev_xc[p & 1], sx));
                if (p >= 1) HIPQ(ctx, hipStreamWaitEvent(sx, ctx->ev_xr[(p - 1) & 1], 0));
                extra_rows_update(ctx, sx, lda, nt, c0, c1, c1, p + 2 <= nsp ? spc[(size_t)p + 2] : nt);
            }
        }
    }
    wait_rest(sm, nt);  // every split update's rest before the tail
    if (spc[(size_t)nsp] < nt) {
        const int ts = spc[(size_t)nsp], T = nt - ts;
        // the posterior's cross-covariance rows: factored along inside the tail
        const int X = ctx->xr_mode == 2 ? ctx->xr_tiles : 0;
        if (ctx->tailk && T + X <= TAIL_TMAX && (ctx->xr_mode == 0 || X > 0)) {
            // the tail as one persistent dataflow launch
            if (ctx->xr_mode && !ctx->serial) {
                // the extra rows' super-panel updates of the tail's columns land first
                HIPQ(ctx, hipEventRecord(ctx->ev_xdone, ctx->s_extra));
                HIPQ(ctx, hipStreamWaitEvent(sm, ctx->ev_xdone, 0));
                HIPQ(ctx, hipEventRecord(ctx->ev_xdone, ctx->s_xrest));
                HIPQ(ctx, hipStreamWaitEvent(sm, ctx->ev_xdone, 0));
            }
            const bool gram = ts == 0 && gram_in_tail(ctx, nt, lda);
            if (ctx->dry) {  // gaplac_plan_check: the task list's dependency order
                std::vector<uint32_t> host;
                build_single_tail_list(T, X, ctx->tail_sim, 0, host, gram);
                std::string why;
                if (!check_tail_tasks(T, host, &why, X, gram)) return set_err(ctx, GAPLAC_E_ARG, "%s", why.c_str());
            }
            if ((ctx->ttasks_T != T || ctx->ttasks_X != X || ctx->ttasks_G != gram) && !ctx->dry) {
                std::vector<uint32_t> host;
                build_single_tail_list(T, X, ctx->tail_sim, std::max(1, ctx->ncu / std::max(1, ctx->tail_share)), host,
                                       gram);
                int rc;
                if ((rc = ensure(ctx, &ctx->ttasks, &ctx->ttasks_elems, host.size()))) return rc;
                HIPCK(ctx, hipMemcpy(ctx->ttasks, host.data(), host.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
                ctx->ttasks_T = T;
                ctx->ttasks_X = X;
                ctx->ttasks_G = gram;
                ctx->ttasks_n = (int)host.size();
            }
            if (!ctx->tctl && !ctx->dry)
                HIPCK(ctx, hipMalloc(reinterpret_cast<void**>(&ctx->tctl), sizeof(TailCtl)));
            if (!gram) HIPQ(ctx, hipMemsetAsync(ctx->tctl, 0, sizeof(TailCtl), sm));  // (gram: zeroed at the start)
            const int nts = ctx->dry ? (int)(T * (T + 1) * (T + 2) / 6 + 3 * T * T + X * T * (T + 3) / 2 +
                                             (gram ? T * (T + 1) / 2 : 0))
                                     : ctx->ttasks_n;
            if (!ctx->ttrace_path.empty() && !ctx->dry) {
                int rc;
                if ((rc = ensure(ctx, &ctx->ttrace, &ctx->ttrace_elems, 3 * (size_t)nts + (size_t)TAIL_DSTAMPS * T)))
                    return rc;
            }
            TailArgs ta{ctx->A, lda, N, ts, T, ctx->Dinv, ctx->dres, ctx->tctl, ctx->ttasks, nts,
                        ctx->ttrace_path.empty() ? nullptr : ctx->ttrace};
            ta.fault = ctx->tail_fault;
            ta.xrows = X;
            if (gram) {  // the inputs the Gram launches would have read (enqueue_eval_body)
                ta.gX = ctx->dX;
                ta.gldx = N;
                ta.gv = ctx->dv;
                ta.gtp = ctx->dtp;
            }
            // batch lanes run their tails side by side: each persistent grid takes its share
            // of the CUs (one tail workgroup fills a CU's LDS), so no tail waits for another
            launch_tail(sm, ta, std::min(std::max(1, ctx->ncu / std::max(1, ctx->tail_share)), nts), slot(ctx, 10, 0));
        } else {
            serial_tail(ctx, sm, N, lda, nt, ts);
        }
    }
    if (ctx->xr_mode && !ctx->serial) {
        HIPQ(ctx, hipEventRecord(ctx->ev_xdone, ctx->s_extra));
        HIPQ(ctx, hipStreamWaitEvent(sm, ctx->ev_xdone, 0));
        HIPQ(ctx, hipEventRecord(ctx->ev_xdone, ctx->s_xrest));
        HIPQ(ctx, hipStreamWaitEvent(sm, ctx->ev_xdone, 0));
    }
    launch_reduce(sm, ctx->A, lda, N, (int64_t)nt * NB, ColMap{1, 0, 1}, ctx->dres);
    HIPQ(ctx, hipGetLastError());
    return 0;
}

// Upload the super-tile ordered lists for every triangle size m = 1..nt (once per nt).
int ensure_tile_lists(gaplac_ctx* ctx, int nt) {
    if (ctx->tiles_nt >= nt) return 0;
    std::vector<size_t> off((size_t)nt + 1, 0);
    for (int m = 1; m <= nt; ++m) off[(size_t)m] = off[(size_t)m - 1] + (size_t)(m - 1) * m / 2;
    const size_t tri_total = off[(size_t)nt] + (size_t)nt * (nt + 1) / 2;
    const int w = ctx->spw;
    size_t total = tri_total;
    for (int m = 1; m <= nt; ++m) total += (size_t)std::min(w, m) * m - (size_t)std::min(w, m) * (std::min(w, m) - 1) / 2;
    std::vector<uint32_t> host(total);
    for (int m = 1; m <= nt; ++m) build_tile_list(m, host.data() + off[(size_t)m]);
    {
        size_t k = tri_total;
        ctx->band_off.assign((size_t)nt + 1, tri_total);
        for (int m = 1; m <= nt; ++m) {
            ctx->band_off[(size_t)m] = k;
            for (int r = 0; r < m; ++r)
                for (int c = 0; c < w && c <= r; ++c) host[k++] = (uint32_t)r | ((uint32_t)c << 16);
        }
        if (k != total) return set_err(ctx, GAPLAC_E_ARG, "band list size mismatch");
    }
    int rc;
    if ((rc = ensure(ctx, &ctx->tiles, &ctx->tiles_elems, total))) return rc;
    HIPCK(ctx, hipMemcpy(ctx->tiles, host.data(), total * sizeof(uint32_t), hipMemcpyHostToDevice));
    ctx->tile_off = off;
    ctx->tiles_nt = nt;
    return 0;
}

// Everything one evaluation puts on the streams (eager launch or graph capture): reset
// the result record (and the profiling slots), Gram build, factorisation schedule,
// reduction, result copy to the pinned host record. Inputs: ctx->dX (ld N), ctx->dv,
// ctx->dtp.
int enqueue_eval_body(gaplac_ctx* ctx, int64_t N, int32_t D, int64_t Np, int nt) {
    const int64_t lda = Np + (int64_t)NB * ctx->xr_tiles;
    const bool gram_tail = gram_in_tail(ctx, nt, lda);
    if (gram_tail && !ctx->tctl && !ctx->dry) HIPCK(ctx, hipMalloc(reinterpret_cast<void**>(&ctx->tctl), sizeof(TailCtl)));
    if (gram_tail)  // the tail's counters zeroed here (factor_and_reduce then skips its memset)
        launch_init_result_ctl(ctx->s_main, ctx->dres, ctx->tctl, *ctx->htp, ctx->dtp);
    else
        launch_init_result(ctx->s_main, ctx->dres);
    if (ctx->recording) launch_kt_reset(ctx->s_main, ctx->dkt, (int)ctx->kt_cap);
    // Gram in two launches: the first super-panel's tile columns, then the rest (the panel
    // chain starts on the first part while the second is still being written; the second as
    // a work queue of two workgroups per CU, so the chain's kernels fit beside it, §4).
    auto tri = [](double m) { return m * (m + 1) / 2; };
    const double bpt = 8.0 * NB * NB;  // bytes per tile
    const double b1 = bpt * (tri(nt) - tri(std::max(0, nt - ctx->spw))) + 8.0 * (double)N * (D + 1);
    const double b2 = bpt * tri(std::max(0, nt - ctx->spw));
    if (!gram_tail) {  // (else the tail's first tasks build it)
        launch_gram(ctx->s_main, ctx->A, lda, N, nt, ctx->dX, N, ctx->dv, ctx->dtp, 1, ctx->spw, slot(ctx, 1, b1));
        HIPQ(ctx, hipEventRecord(ctx->ev_gram, ctx->s_main));
        launch_gram_queue(ctx->s_main, ctx->A, lda, N, nt, ctx->dX, N, ctx->dv, ctx->dtp, ctx->spw, nt, 2, ctx->dres,
                          slot(ctx, 1, b2));
        HIPQ(ctx, hipEventRecord(ctx->ev_gram2, ctx->s_main));
    }
    if (ctx->xr_mode == 1) launch_init_identity_rows(ctx->s_main, ctx->A, lda, Np, nt, ctx->spw);
    if (ctx->xr_mode == 2)
        launch_cross_gram(ctx->s_main, ctx->A, lda, Np, nt, N, ctx->xr_M, ctx->xr_tiles, ctx->dX, N, ctx->dXs,
                          ctx->xr_M, ctx->dtp);
    if (ctx->xr_mode && !ctx->serial) {  // the extra-row stream starts after their init
        HIPQ(ctx, hipEventRecord(ctx->ev_xinit, ctx->s_main));
        HIPQ(ctx, hipStreamWaitEvent(ctx->s_extra, ctx->ev_xinit, 0));
    }
    int rc;
    if ((rc = factor_and_reduce(ctx, N, lda, nt))) return rc;
    if (ctx->xr_mode == 2)
        launch_posterior(ctx->s_main, ctx->A, lda, Np, N, ctx->xr_M, ctx->dXs, ctx->xr_M, ctx->dtp, ctx->gpart,
                         ctx->pmean, ctx->pvar);
    if (ctx->xr_mode == 1 && ctx->grad_fused && ctx->grad_singletons) {
        // alpha = Y z first (HBM-bound, ~0.2 ms alone), then M = -C^{-1} tile by tile contracted
        // in place with every dC/dtheta (cinv_contract_kernel: the tile is never stored nor
        // read back), then the fixed-order reduction, all on s_main
        hipStream_t sm = ctx->s_main;
        launch_zero_tail_cols(sm, ctx->A, lda, Np, N);
        launch_copy_z(sm, ctx->A, lda, N, ctx->gz);
        launch_alpha(sm, ctx->A, lda, Np, N, ctx->gz, ctx->gpart, ctx->galpha, ctx->gdv);
        size_t e0 = 0;
        const bool ev = ctx->prof_mode == 2;
        if (ev) {
            e0 = 2 * ctx->evpairs.size();
            while (ctx->evpool.size() < e0 + 2) {
                hipEvent_t e;
                HIPQ(ctx, hipEventCreate(&e));
                ctx->evpool.push_back(e);
            }
            HIPQ(ctx, hipEventRecord(ctx->evpool[e0], sm));
        }
        launch_cinv_contract(sm, ctx->A, lda, Np, N, ctx->dX, N, ctx->galpha, ctx->dtp, ctx->glist,
                             ctx->glist_blocks, ctx->gpart, slot(ctx, 8, 0));
        if (ev) {
            HIPQ(ctx, hipEventRecord(ctx->evpool[e0 + 1], sm));
            ctx->evpairs.push_back({e0, 0.0, 0.0, 8});
        }
        const int m = (int)((N + NB - 1) / NB);
        launch_grad_reduce(sm, ctx->gpart, m * (m + 1) / 2, ctx->htp->T, ctx->gout);
        HIPQ(ctx, hipMemcpyAsync(ctx->hgout, ctx->gout, sizeof(double) * (GAPLAC_MAX_TERMS + 1),
                                  hipMemcpyDeviceToHost, sm));
    } else if (ctx->xr_mode == 1) {
        // alpha = Y z on s_extra beside M = -C^{-1} over the factor storage on s_main (both only
        // read Y; z is copied out first, cinv may overwrite row N), then the contraction and
        // the reduction on s_main once alpha is in (GAPLAC_GRAD_FUSED=0)
        hipStream_t sm = ctx->s_main;
        hipStream_t sx = ctx->serial ? sm : ctx->s_extra;
        launch_zero_tail_cols(sm, ctx->A, lda, Np, N);
        launch_copy_z(sm, ctx->A, lda, N, ctx->gz);
        if (sx != sm) {
            HIPQ(ctx, hipEventRecord(ctx->ev_xinit, sm));
            HIPQ(ctx, hipStreamWaitEvent(sx, ctx->ev_xinit, 0));
        }
        launch_alpha(sx, ctx->A, lda, Np, N, ctx->gz, ctx->gpart, ctx->galpha, ctx->gdv);
        if (sx != sm) HIPQ(ctx, hipEventRecord(ctx->ev_xdone, sx));
        size_t e0 = 0;
        const bool ev = ctx->prof_mode == 2;
        if (ev) {
            e0 = 2 * ctx->evpairs.size();
            while (ctx->evpool.size() < e0 + 2) {
                hipEvent_t e;
                HIPQ(ctx, hipEventCreate(&e));
                ctx->evpool.push_back(e);
            }
            HIPQ(ctx, hipEventRecord(ctx->evpool[e0], sm));
        }
        launch_cinv_tiles(sm, ctx->A, lda, Np, ctx->glist, ctx->glist_blocks, (int)((N + NB - 1) / NB),
                          slot(ctx, 8, 0));
        if (ev) {
            HIPQ(ctx, hipEventRecord(ctx->evpool[e0 + 1], sm));
            ctx->evpairs.push_back({e0, 0.0, 0.0, 8});
        }
        if (sx != sm) HIPQ(ctx, hipStreamWaitEvent(sm, ctx->ev_xdone, 0));
        launch_grad_contract(sm, ctx->A, lda, N, ctx->dX, N, ctx->galpha, ctx->dtp, ctx->dgp, ctx->gpart,
                             slot(ctx, 9, 0));
        const int m = (int)((N + NB - 1) / NB);
        launch_grad_reduce(sm, ctx->gpart, m * (m + 1) / 2, ctx->htp->T, ctx->gout);
        HIPQ(ctx, hipMemcpyAsync(ctx->hgout, ctx->gout, sizeof(double) * (GAPLAC_MAX_TERMS + 1),
                                  hipMemcpyDeviceToHost, sm));
    }
    HIPQ(ctx, hipMemcpyAsync(ctx->hres, ctx->dres, offsetof(EvalResult, part), hipMemcpyDeviceToHost,
                              ctx->s_main));
    return 0;
}

// The schedule under a footprint guard over ctx->A (unless the caller installed one, as
// gaplac_plan_check's dry run does): a launch whose grid would touch elements outside
// the workspace is not enqueued and the evaluation fails with GAPLAC_E_ARG.
int enqueue_eval(gaplac_ctx* ctx, int64_t N, int32_t D, int64_t Np, int nt) {
    LaunchGuard local;
    LaunchGuard* g = current_guard();
    const bool own = g == nullptr;
    if (own) {
        local.base = ctx->A;
        local.elems = (int64_t)ctx->A_elems;
        g = &local;
    }
    GuardScope scope(g);
    const int64_t v0 = g->violations;
    const int rc = enqueue_eval_body(ctx, N, D, Np, nt);
    if (rc) return rc;
    if (g->violations > v0)
        return set_err(ctx, GAPLAC_E_ARG, "launch footprint outside the workspace (N=%lld): %s", (long long)N,
                       g->first.c_str());
    return 0;
}

// Workspace for order N (grown on demand).
int ensure_workspace(gaplac_ctx* ctx, int64_t N) {
    const int64_t Np = round_up(N + 1, NB);
    const int nt = (int)(Np / NB);
    int rc;
    HIPCK(ctx, hipSetDevice(ctx->device));
    if ((rc = ensure(ctx, &ctx->A, &ctx->A_elems, (size_t)(Np + (int64_t)NB * ctx->xr_tiles) * Np))) return rc;
    if (split_wanted(ctx, nt) && !ctx->s_xrest) {
        // the split bulk updates' second stream (factor_and_reduce): the extra rows' stream
        // of a gradient / posterior context, idle in a plain evaluation
        int least = 0, greatest = 0;
        HIPCK(ctx, hipDeviceGetStreamPriorityRange(&least, &greatest));
        HIPCK(ctx, hipStreamCreateWithPriority(&ctx->s_xrest, hipStreamNonBlocking, least));
    }
    if (ctx->xr_mode && !ctx->s_extra) {
        // created on first use only: a plain logpdf context keeps two streams, so the
        // batch lanes (2 contexts) fit the 4 hardware queues a process gets by default. A
        // gradient / posterior context then holds four streams (s_main, s_panel, s_extra,
        // s_xrest), all four hardware queues: another context or torch stream in the same
        // process shares a queue with one of them and may serialise behind it (the
        // measured 79.4 -> 78.0 ms of DESIGN.md §9 assumes no other streams are busy)
        int least = 0, greatest = 0;
        HIPCK(ctx, hipDeviceGetStreamPriorityRange(&least, &greatest));
        HIPCK(ctx, hipStreamCreateWithPriority(&ctx->s_extra, hipStreamNonBlocking, least));
        HIPCK(ctx, hipStreamCreateWithPriority(&ctx->s_xrest, hipStreamNonBlocking, least));
    }
    if (ctx->xr_mode == 2) {
        const size_t M = (size_t)ctx->xr_M;
        if ((rc = ensure(ctx, &ctx->gpart, &ctx->gpart_elems, 2 * M * (size_t)((N + 511) / 512)))) return rc;
        if (ctx->pmv_elems < M) {
            if (ctx->pmean) (void)hipFree(ctx->pmean);
            if (ctx->pvar) (void)hipFree(ctx->pvar);
            ctx->pmean = ctx->pvar = nullptr;
            ctx->pmv_elems = 0;
            if (hipMalloc(reinterpret_cast<void**>(&ctx->pmean), M * 8) != hipSuccess ||
                hipMalloc(reinterpret_cast<void**>(&ctx->pvar), M * 8) != hipSuccess)
                return set_err(ctx, GAPLAC_E_OOM, "hipMalloc of posterior outputs failed");
            ctx->pmv_elems = M;
        }
    }
    if (ctx->xr_mode == 1) {
        const int m = (int)((N + NB - 1) / NB);
        const size_t nk = (size_t)((N + 511) / 512);
        const size_t part = std::max(nk * (size_t)N, (size_t)m * (m + 1) / 2 * (GAPLAC_MAX_TERMS + 1));
        if ((rc = ensure(ctx, &ctx->galpha, &ctx->galpha_elems, (size_t)N))) return rc;
        if ((rc = ensure(ctx, &ctx->gdv, &ctx->gdv_elems, (size_t)N))) return rc;
        if ((rc = ensure(ctx, &ctx->gz, &ctx->gz_elems, (size_t)N))) return rc;
        if ((rc = ensure(ctx, &ctx->gpart, &ctx->gpart_elems, part))) return rc;
        if (ctx->glist_m != m) {
            std::vector<uint32_t> host;
            build_grad_list(m, host);
            if ((rc = ensure(ctx, &ctx->glist, &ctx->glist_elems, host.size()))) return rc;
            HIPCK(ctx, hipMemcpy(ctx->glist, host.data(), host.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
            ctx->glist_m = m;
            ctx->glist_blocks = (int)host.size();
        }
    }
    if ((rc = ensure(ctx, &ctx->Dinv, &ctx->Dinv_elems, (size_t)nt * DINV_PER_BLOCK))) return rc;
    return ensure_tile_lists(ctx, nt);
}

// Eager enqueue of one evaluation (no profiling, no wait): the batch lanes.
int eval_enqueue(gaplac_ctx* ctx, int64_t N, int32_t D, const TermPack& tp) {
    int rc;
    if ((rc = ensure_workspace(ctx, N))) return rc;
    const int64_t Np = round_up(N + 1, NB);
    *ctx->htp = tp;
    if (!tp_by_init(ctx, N))
        HIPCK(ctx, hipMemcpyAsync(ctx->dtp, ctx->htp, sizeof(TermPack), hipMemcpyHostToDevice, ctx->s_main));
    ctx->slots.clear();
    ctx->recording = false;
    return enqueue_eval(ctx, N, D, Np, (int)(Np / NB));
}

int eval_wait(gaplac_ctx* ctx, EvalResult* out) {
    HIPCK(ctx, hipStreamSynchronize(ctx->s_main));
    *out = *ctx->hres;
    if (out->err) return set_err(ctx, GAPLAC_E_HIP, "in-kernel wait expired (code %u)", out->err);
    return 0;
}

// Full evaluation; inputs already in ctx->dX (ld N) / ctx->dv, term pack in tp (host).
// Leaves the factor in ctx->A.
int eval_device(gaplac_ctx* ctx, int64_t N, int32_t D, const TermPack& tp, EvalResult* out) {
    const int64_t Np = round_up(N + 1, NB);
    const int nt = (int)(Np / NB);
    int rc;
    if ((rc = ensure_workspace(ctx, N))) return rc;
    const bool prof = ctx->profiling;
    if (prof) {
        const size_t need = (size_t)nt * 9 + 32;  // launches per evaluation, with margin
        if (ctx->kt_cap < need) {
            if ((rc = ensure(ctx, &ctx->dkt, &ctx->kt_cap, need))) return rc;
            if (ctx->hkt) (void)hipHostFree(ctx->hkt);
            ctx->hkt = nullptr;
            HIPCK(ctx, hipHostMalloc(reinterpret_cast<void**>(&ctx->hkt), ctx->kt_cap * sizeof(KTime), 0));
        }
    }
    *ctx->htp = tp;
    if (!tp_by_init(ctx, N))
        HIPCK(ctx, hipMemcpyAsync(ctx->dtp, ctx->htp, sizeof(TermPack), hipMemcpyHostToDevice, ctx->s_main));
    ctx->slots.clear();
    ctx->recording = prof;
    rc = enqueue_eval(ctx, N, D, Np, nt);
    ctx->recording = false;
    if (rc) return rc;
    HIPCK(ctx, hipStreamSynchronize(ctx->s_main));
    *out = *ctx->hres;
    if (out->err) return set_err(ctx, GAPLAC_E_HIP, "in-kernel wait expired (code %u)", out->err);
    if (!ctx->ttrace_path.empty() && ctx->ttrace && ctx->ttasks_n > 0) {  // diagnostics: task timeline
        std::vector<unsigned long long> tr(3 * (size_t)ctx->ttasks_n);
        std::vector<uint32_t> tk((size_t)ctx->ttasks_n);
        HIPCK(ctx, hipMemcpy(tr.data(), ctx->ttrace, tr.size() * 8, hipMemcpyDeviceToHost));
        HIPCK(ctx, hipMemcpy(tk.data(), ctx->ttasks, tk.size() * 4, hipMemcpyDeviceToHost));
        if (FILE* f = std::fopen(ctx->ttrace_path.c_str(), "a")) {
            std::fprintf(f, "# N=%lld T=%d tasks=%d\n", (long long)N, ctx->ttasks_T, ctx->ttasks_n);
            for (size_t i = 0; i < tk.size(); ++i)
                std::fprintf(f, "%zu %u %llu %llu %llu\n", i, tk[i], tr[3 * i], tr[3 * i + 1], tr[3 * i + 2]);
            std::fclose(f);
        }
        // the diagonal blocks' phase times (potrf_diag2_body), one line per tile column
        std::vector<unsigned long long> ds((size_t)TAIL_DSTAMPS * ctx->ttasks_T);
        HIPCK(ctx, hipMemcpy(ds.data(), ctx->ttrace + 3 * (size_t)ctx->ttasks_n, ds.size() * 8, hipMemcpyDeviceToHost));
        if (FILE* f = std::fopen((ctx->ttrace_path + ".d").c_str(), "a")) {
            std::fprintf(f, "# N=%lld T=%d\n", (long long)N, ctx->ttasks_T);
            for (int k = 0; k < ctx->ttasks_T; ++k) {
                std::fprintf(f, "%d", k);
                for (int i = 0; i < TAIL_DSTAMPS; ++i) std::fprintf(f, " %llu", ds[(size_t)TAIL_DSTAMPS * k + i]);
                std::fprintf(f, "\n");
            }
            std::fclose(f);
        }
    }
    if (prof) {
        rc = accumulate_slots(ctx, ctx->slots);
        ctx->slots.clear();
    }
    return rc;
}

int finish(const EvalResult& r, double* out_logpdf, double* out_logdet, double* out_quad) {
    if (out_logdet) *out_logdet = r.logdet;
    if (out_quad) *out_quad = r.quad;
    if (r.info != ~0ull) {
        if (out_logpdf) *out_logpdf = NAN;
        return (int)(r.info > 0x7fffffffull ? 0x7fffffff : r.info);
    }
    if (out_logpdf) *out_logpdf = r.logpdf;
    return 0;
}

int upload(gaplac_ctx* ctx, int64_t N, int32_t D, const double* X, int64_t ldx, const double* v) {
    int rc;
    const size_t nx = (size_t)N * (size_t)(D > 0 ? D : 1);
    if ((rc = ensure(ctx, &ctx->dX, &ctx->dX_elems, nx))) return rc;
    if ((rc = ensure(ctx, &ctx->dv, &ctx->dv_elems, (size_t)N))) return rc;
    if (D > 0)
        HIPCK(ctx, hipMemcpy2DAsync(ctx->dX, (size_t)N * 8, X, (size_t)ldx * 8, (size_t)N * 8,
                                    (size_t)D, hipMemcpyHostToDevice, ctx->s_main));
    HIPCK(ctx, hipMemcpyAsync(ctx->dv, v, (size_t)N * 8, hipMemcpyHostToDevice, ctx->s_main));
    return 0;
}

// Copy device-resident inputs into the context's buffers (ld N): a ~N*(D+1)*8-byte D2D
// copy that keeps the captured graph's pointers fixed.
int upload_device(gaplac_ctx* ctx, int64_t N, int32_t D, const double* dX, int64_t ldx, const double* dv) {
    int rc;
    const size_t nx = (size_t)N * (size_t)(D > 0 ? D : 1);
    if ((rc = ensure(ctx, &ctx->dX, &ctx->dX_elems, nx))) return rc;
    if ((rc = ensure(ctx, &ctx->dv, &ctx->dv_elems, (size_t)N))) return rc;
    if (D > 0)
        HIPCK(ctx, hipMemcpy2DAsync(ctx->dX, (size_t)N * 8, dX, (size_t)ldx * 8, (size_t)N * 8,
                                    (size_t)D, hipMemcpyDeviceToDevice, ctx->s_main));
    HIPCK(ctx, hipMemcpyAsync(ctx->dv, dv, (size_t)N * 8, hipMemcpyDeviceToDevice, ctx->s_main));
    return 0;
}

void nan_out(double* a, double* b, double* c) {
    if (a) *a = NAN;
    if (b) *b = NAN;
    if (c) *c = NAN;
}

// Shared body of gaplac_logpdf_grad / _device.
int logpdf_grad_impl(gaplac_ctx* ctx, bool on_device, int64_t N, int32_t D, const double* X, int64_t ldx,
                     int32_t T, const gaplac_term* terms, double noise, const double* v, double* out_logpdf,
                     double* out_dv, double* out_dparam, double* out_dnoise) {
    if (out_logpdf) *out_logpdf = NAN;
    if (out_dnoise) *out_dnoise = NAN;
    if (out_dparam && T > 0)
        for (int t = 0; t < T && t < GAPLAC_MAX_TERMS; ++t) out_dparam[t] = NAN;
    if (out_dv)
        for (int64_t i = 0; i < N; ++i) out_dv[i] = NAN;
    int rc = check_common(ctx, N, D, X, ldx, noise, v);
    if (rc) return rc;
    TermPack tp;
    if ((rc = pack_terms(ctx, D, T, terms, &tp))) return rc;
    if (N == 0) {
        if (out_logpdf) *out_logpdf = -0.0;
        if (out_dnoise) *out_dnoise = 0.0;
        if (out_dparam)
            for (int t = 0; t < T; ++t) out_dparam[t] = 0.0;
        return 0;
    }
    GradTermPack gp{};
    for (int t = 0; t < T; ++t) {
        int a = t, b = t + 1;
        while (a > 0 && terms[a - 1].group == terms[t].group) --a;
        while (b < T && terms[b].group == terms[t].group) ++b;
        gp.gstart[t] = a;
        gp.gend[t] = b;
    }
    ctx->grad_singletons = true;
    for (int t = 0; t < T; ++t) ctx->grad_singletons = ctx->grad_singletons && gp.gend[t] - gp.gstart[t] == 1;
    HIPCK(ctx, hipSetDevice(ctx->device));
    if ((rc = on_device ? upload_device(ctx, N, D, X, ldx, v) : upload(ctx, N, D, X, ldx, v))) return rc;
    tp.noise = noise;
    *ctx->hgp = gp;
    HIPCK(ctx, hipMemcpyAsync(ctx->dgp, ctx->hgp, sizeof(GradTermPack), hipMemcpyHostToDevice, ctx->s_main));
    ctx->xr_mode = 1;
    ctx->xr_tiles = (int)(round_up(N + 1, NB) / NB);
    EvalResult r;
    rc = eval_device(ctx, N, D, tp, &r);
    ctx->xr_mode = 0;
    ctx->xr_tiles = 0;
    if (rc) return rc;
    rc = finish(r, out_logpdf, nullptr, nullptr);
    if (rc) return rc;  // PosDefException: gradients stay NaN
    if (out_dv) HIPCK(ctx, hipMemcpy(out_dv, ctx->gdv, (size_t)N * sizeof(double), hipMemcpyDeviceToHost));
    if (out_dparam)
        for (int t = 0; t < T; ++t) out_dparam[t] = ctx->hgout[t];
    if (out_dnoise) *out_dnoise = ctx->hgout[T];
    return 0;
}

// Shared body of gaplac_posterior_mean_var.
int posterior_impl(gaplac_ctx* ctx, int64_t N, int32_t D, const double* X, int64_t ldx, int32_t T,
                   const gaplac_term* terms, double noise, const double* y, int64_t M, const double* Xs,
                   int64_t ldxs, double* out_mean, double* out_var) {
    for (int64_t j = 0; j < M; ++j) {
        if (out_mean) out_mean[j] = NAN;
        if (out_var) out_var[j] = NAN;
    }
    int rc = check_common(ctx, N, D, X, ldx, noise, y);
    if (rc) return rc;
    if (M < 0 || (M > 0 && D > 0 && (!Xs || ldxs < M)))
        return set_err(ctx, GAPLAC_E_ARG, "M < 0, or Xs NULL / ldxs < M");
    TermPack tp;
    if ((rc = pack_terms(ctx, D, T, terms, &tp))) return rc;
    if (M == 0) return 0;
    HIPCK(ctx, hipSetDevice(ctx->device));
    if (N == 0) {  // posterior of an empty FiniteGP = the prior: mean 0, var kdiag
        for (int64_t j = 0; j < M; ++j) {
            double kd = 0.0, pr = 1.0;
            for (int t = 0; t < T; ++t) {
                const double x = tp.kind[t] == GAPLAC_NOISE ? 0.0 : Xs[(int64_t)tp.col[t] * ldxs + j];
                double k = 1.0;
                if (tp.kind[t] == GAPLAC_LINEAR) k = x * x + tp.p[t];
                if (tp.kind[t] == GAPLAC_NOISE) k = tp.p[t];
                pr *= k;
                if (tp.last_in_group[t]) {
                    kd += pr;
                    pr = 1.0;
                }
            }
            if (out_mean) out_mean[j] = 0.0;
            if (out_var) out_var[j] = kd;
        }
        return 0;
    }
    if ((rc = upload(ctx, N, D, X, ldx, y))) return rc;
    const size_t nxs = (size_t)M * (size_t)(D > 0 ? D : 1);
    if ((rc = ensure(ctx, &ctx->dXs, &ctx->dXs_elems, nxs))) return rc;
    if (D > 0)
        HIPCK(ctx, hipMemcpy2DAsync(ctx->dXs, (size_t)M * 8, Xs, (size_t)ldxs * 8, (size_t)M * 8, (size_t)D,
                                    hipMemcpyHostToDevice, ctx->s_main));
    tp.noise = noise;
    ctx->xr_mode = 2;
    ctx->xr_tiles = (int)((M + NB - 1) / NB);
    ctx->xr_M = M;
    EvalResult r;
    rc = eval_device(ctx, N, D, tp, &r);
    ctx->xr_mode = 0;
    ctx->xr_tiles = 0;
    if (rc) return rc;
    rc = finish(r, nullptr, nullptr, nullptr);
    if (rc) return rc;
    if (out_mean) HIPCK(ctx, hipMemcpy(out_mean, ctx->pmean, (size_t)M * 8, hipMemcpyDeviceToHost));
    if (out_var) HIPCK(ctx, hipMemcpy(out_var, ctx->pvar, (size_t)M * 8, hipMemcpyDeviceToHost));
    return 0;
}

}  // namespace


// Batched tail: models m0 .. m0+B-1 of a select batch whose matrix lies
// whole in the persistent tail, evaluated together on workspace set p: the Grams and
// result records on s_panel (so they run beside the previous launch's tail on s_main),
// then on s_main ONE tail launch whose task list interleaves the B models' lists as a
// software pipeline (interleave_tail_tasks), and one reduction per model. Each model's
// tasks, and so its arithmetic, are those of its single evaluation: the results are
// bitwise the same. Nothing here waits for the launch; batch_tail_finish collects it.
static int batch_tail_finish(gaplac_ctx* ctx, int p, double* out_logpdf, int64_t* out_info);

static int batch_tail_enqueue(gaplac_ctx* ctx, int64_t N, const std::vector<TermPack>& packs, int m0, int B, int p,
                              double* out_logpdf, int64_t* out_info) {
    const int64_t Np = round_up(N + 1, NB);
    const int nt = (int)(Np / NB);
    const int64_t lda = Np;
    const size_t astride = (size_t)Np * (size_t)Np, dstride = (size_t)nt * DINV_PER_BLOCK;
    gaplac_ctx::BatchWs& w = ctx->bw[p];
    int rc;
    if (w.busy && (rc = batch_tail_finish(ctx, p, out_logpdf, out_info))) return rc;  // the set's last launch
    if ((rc = ensure(ctx, &w.A, &w.A_elems, astride * (size_t)B))) return rc;
    if ((rc = ensure(ctx, &w.Dinv, &w.Dinv_elems, dstride * (size_t)B))) return rc;
    if ((rc = ensure(ctx, &w.dres, &w.dres_elems, (size_t)B))) return rc;
    if ((rc = ensure(ctx, &w.dtp, &w.dtp_elems, (size_t)B))) return rc;
    if ((rc = ensure(ctx, &w.ctl, &w.ctl_elems, (size_t)B))) return rc;
    if (!w.ev_gram) HIPCK(ctx, hipEventCreateWithFlags(&w.ev_gram, hipEventDisableTiming));
    if (!w.ev_done) HIPCK(ctx, hipEventCreateWithFlags(&w.ev_done, hipEventDisableTiming));
    if (w.host_cap < B) {
        if (w.hres) (void)hipHostFree(w.hres);
        if (w.htp) (void)hipHostFree(w.htp);
        w.hres = nullptr;
        w.htp = nullptr;
        w.host_cap = 0;
        HIPCK(ctx, hipHostMalloc(reinterpret_cast<void**>(&w.hres), sizeof(EvalResult) * (size_t)B, 0));
        HIPCK(ctx, hipHostMalloc(reinterpret_cast<void**>(&w.htp), sizeof(TermPack) * (size_t)B, 0));
        w.host_cap = B;
    }
    const int lag = ctx->batch_lag >= 0 ? ctx->batch_lag : (3 * nt + 4) / 8;
    const int lkey = lag * 100 + ctx->batch_gw * 10 + ctx->batch_near;
    if (w.tasks_T != nt || w.tasks_B != B || w.tasks_lag != lkey) {
        std::vector<uint32_t> one, all;
        std::vector<size_t> cs;
        build_tail_tasks(nt, one, &cs, ctx->batch_gw, ctx->batch_near, 0, true, GAPLAC_BATCH_GROUP);
        interleave_tail_tasks(one, cs, B, lag, all);
        if ((rc = ensure(ctx, &w.tasks, &w.tasks_elems, all.size()))) return rc;
        HIPCK(ctx, hipMemcpy(w.tasks, all.data(), all.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        w.tasks_T = nt;
        w.tasks_B = B;
        w.tasks_lag = lkey;
        w.tasks_n = (int)all.size();
    }
    const bool trace = !ctx->ttrace_path.empty();  // diagnostics: launches one at a time
    // (+ the diagonal blocks' phase times, which a one-model launch records)
    if (trace && (rc = ensure(ctx, &ctx->ttrace, &ctx->ttrace_elems, 3 * (size_t)w.tasks_n + (size_t)TAIL_DSTAMPS * nt)))
        return rc;
    hipStream_t g = ctx->s_panel, s = ctx->s_main;
    for (int b = 0; b < B; ++b) w.htp[b] = packs[(size_t)(m0 + b)];
    // From the first enqueue on, a failure must not leave this call's work in flight (the
    // Grams read dX / dv, which the next call's upload overwrites): drain both streams first.
    auto bail = [&](int code) {
        (void)hipStreamSynchronize(g);
        (void)hipStreamSynchronize(s);
        return code;
    };
#define BATCHCK(call)                                                                                    \
    do {                                                                                                 \
        hipError_t e_ = (call);                                                                          \
        if (e_ != hipSuccess)                                                                            \
            return bail(set_err(ctx, GAPLAC_E_HIP, "%s failed: %s", #call, hipGetErrorString(e_)));      \
    } while (0)
    LaunchGuard guard;
    guard.base = w.A;
    guard.elems = (int64_t)(astride * (size_t)B);
    {
        GuardScope scope(&guard);
        BATCHCK(hipMemcpyAsync(w.dtp, w.htp, sizeof(TermPack) * (size_t)B, hipMemcpyHostToDevice, g));
        for (int b = 0; b < B; ++b) {
            launch_init_result(g, w.dres + b);
            launch_gram(g, w.A + astride * (size_t)b, lda, N, nt, ctx->dX, N, ctx->dv, w.dtp + b, 0, 0, nullptr);
        }
        BATCHCK(hipEventRecord(w.ev_gram, g));
        BATCHCK(hipStreamWaitEvent(s, w.ev_gram, 0));
        BATCHCK(hipMemsetAsync(w.ctl, 0, sizeof(TailCtl) * (size_t)B, s));
        TailArgs ta{w.A, lda, N, 0, nt, w.Dinv, w.dres, w.ctl, w.tasks, w.tasks_n, trace ? ctx->ttrace : nullptr};
        ta.a_stride = (int64_t)astride;
        ta.dinv_stride = (int64_t)dstride;
        ta.nmodels = B;
        ta.fault = ctx->tail_fault;
        if (!guard.violations) launch_tail(s, ta, std::min(ctx->ncu, w.tasks_n), nullptr);
        for (int b = 0; b < B; ++b)
            launch_reduce(s, w.A + astride * (size_t)b, lda, N, (int64_t)nt * NB, ColMap{1, 0, 1}, w.dres + b);
    }
    if (guard.violations)
        return bail(set_err(ctx, GAPLAC_E_ARG, "batched tail: launch footprint outside the workspace: %s",
                            guard.first.c_str()));
    BATCHCK(hipGetLastError());
    BATCHCK(hipMemcpyAsync(w.hres, w.dres, sizeof(EvalResult) * (size_t)B, hipMemcpyDeviceToHost, s));
    BATCHCK(hipEventRecord(w.ev_done, s));
#undef BATCHCK
    w.busy = true;
    w.m0 = m0;
    w.B = B;
    if (!ctx->ttrace_path.empty()) {  // diagnostics: the launch's task timeline
        if ((rc = batch_tail_finish(ctx, p, out_logpdf, out_info))) return rc;
        std::vector<unsigned long long> tr(3 * (size_t)w.tasks_n);
        std::vector<uint32_t> tk((size_t)w.tasks_n);
        HIPCK(ctx, hipMemcpy(tr.data(), ctx->ttrace, tr.size() * 8, hipMemcpyDeviceToHost));
        HIPCK(ctx, hipMemcpy(tk.data(), w.tasks, tk.size() * 4, hipMemcpyDeviceToHost));
        if (FILE* f = std::fopen(ctx->ttrace_path.c_str(), "a")) {
            std::fprintf(f, "# N=%lld T=%d tasks=%d models=%d (batched)\n", (long long)N, nt, w.tasks_n, B);
            for (size_t i = 0; i < tk.size(); ++i)
                std::fprintf(f, "%zu %u %llu %llu %llu\n", i, tk[i], tr[3 * i], tr[3 * i + 1], tr[3 * i + 2]);
            std::fclose(f);
        }
    }
    return 0;
}

static int batch_tail_finish(gaplac_ctx* ctx, int p, double* out_logpdf, int64_t* out_info) {
    gaplac_ctx::BatchWs& w = ctx->bw[p];
    if (!w.busy) return 0;
    w.busy = false;
    HIPCK(ctx, hipEventSynchronize(w.ev_done));
    for (int b = 0; b < w.B; ++b) {
        if (w.hres[b].err) return set_err(ctx, GAPLAC_E_HIP, "batched tail: in-kernel wait expired (code %u)", w.hres[b].err);
        out_info[w.m0 + b] = finish(w.hres[b], &out_logpdf[w.m0 + b], nullptr, nullptr);
    }
    return 0;
}

extern "C" {

int gaplac_abi_version(void) { return GAPLAC_ABI_VERSION; }

const char* gaplac_last_error(const gaplac_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int gaplac_ctx_create(int device, gaplac_ctx** out) {
    if (!out) return GAPLAC_E_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return GAPLAC_E_NODEVICE;
    if (device < 0 || device >= n) return GAPLAC_E_NODEVICE;
    gaplac_ctx* ctx = new gaplac_ctx();
    ctx->device = device;
    // the schedule switches
    if (const char* s = std::getenv("GAPLAC_SERIAL")) ctx->serial = s[0] == '1';
    if (const char* s = std::getenv("GAPLAC_SPW")) ctx->spw = std::max(1, std::min(8, std::atoi(s)));
    if (const char* s = std::getenv("GAPLAC_PAIR_M")) ctx->pair_m = std::max(0, std::atoi(s));
    if (const char* s = std::getenv("GAPLAC_BAND_TILES_M")) ctx->band_tiles_m = std::max(1, std::atoi(s));
    if (const char* s = std::getenv("GAPLAC_TAIL_SIM")) ctx->tail_sim = s[0] == '0' ? 0 : 1;
    if (const char* s = std::getenv("GAPLAC_GRAD_FUSED")) ctx->grad_fused = s[0] != '0';
    if (const char* s = std::getenv("GAPLAC_BATCH_LANES")) ctx->batch_lanes = std::max(1, std::min(16, std::atoi(s)));
    if (const char* s = std::getenv("GAPLAC_TAILK")) ctx->tailk = s[0] != '0';
    if (ctx->tailk) ctx->tail_s = 80;  // the persistent tail (A/B at N = 16384)
    if (const char* s = std::getenv("GAPLAC_TAIL_S")) ctx->tail_s = std::max(0, std::atoi(s));
    if (const char* s = std::getenv("GAPLAC_TAIL_TRACE")) ctx->ttrace_path = s;  // diagnostics
    if (const char* s = std::getenv("GAPLAC_TAIL_FAULT")) {  // tests only: forced expiry
        ctx->tail_fault = std::atoi(s);
        if (ctx->tail_fault >= 0)
            std::fprintf(stderr,
                         "gaplac: GAPLAC_TAIL_FAULT=%d is set (test hook): the persistent tail skips the diagonal "
                         "block of that tail column and evaluations return GAPLAC_E_HIP\n",
                         ctx->tail_fault);
    }
    if (const char* s = std::getenv("GAPLAC_BATCH_W")) ctx->batch_w = std::max(1, std::min(TAIL_MAX_MODELS, std::atoi(s)));
    if (const char* s = std::getenv("GAPLAC_BATCH_LAG")) ctx->batch_lag = std::max(0, std::atoi(s));
    auto fail = [&](const char* what, hipError_t e) {
        std::fprintf(stderr, "gaplac_ctx_create: %s: %s\n", what, hipGetErrorString(e));
        gaplac_ctx_destroy(ctx);
        return GAPLAC_E_HIP;
    };
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) return fail("hipSetDevice", e);
    // s_panel: highest priority; s_main: lowest priority. A CU mask that
    // keeps CUs free of s_main's workgroups for the chain (the 512-thread diagonal-block
    // kernel cannot share a CU with a bulk workgroup) and hipGraph replay were both measured
    // slower (round 3, N=16384: no mask 28.8 ms, 4/8/16 CUs 29.8-30.1 ms: the masked bulk
    // kernel lost ~15%) and are not kept.
    int ncu = 0;
    if ((e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device)) != hipSuccess)
        return fail("attribute", e);
    if (ncu > 0) ctx->ncu = ncu;
    int least = 0, greatest = 0;
    if ((e = hipDeviceGetStreamPriorityRange(&least, &greatest)) != hipSuccess)
        return fail("priority range", e);
    if ((e = hipStreamCreateWithPriority(&ctx->s_panel, hipStreamNonBlocking, greatest)) != hipSuccess)
        return fail("stream", e);
    if ((e = hipStreamCreateWithPriority(&ctx->s_main, hipStreamNonBlocking, least)) != hipSuccess)
        return fail("stream", e);
    for (int q = 0; q < 2; ++q) {
        if ((e = hipEventCreateWithFlags(&ctx->ev_P[q], hipEventDisableTiming)) != hipSuccess)
            return fail("event", e);
        if ((e = hipEventCreateWithFlags(&ctx->ev_R[q], hipEventDisableTiming)) != hipSuccess)
            return fail("event", e);
        if ((e = hipEventCreateWithFlags(&ctx->ev_xc[q], hipEventDisableTiming)) != hipSuccess)
            return fail("event", e);
        if ((e = hipEventCreateWithFlags(&ctx->ev_xr[q], hipEventDisableTiming)) != hipSuccess)
            return fail("event", e);
    }
    if ((e = hipEventCreateWithFlags(&ctx->ev_gram, hipEventDisableTiming)) != hipSuccess)
        return fail("event", e);
    for (int q = 0; q < 2; ++q) {
        if ((e = hipEventCreateWithFlags(&ctx->ev_split[q], hipEventDisableTiming)) != hipSuccess)
            return fail("event", e);
        if ((e = hipEventCreateWithFlags(&ctx->ev_rest[q], hipEventDisableTiming)) != hipSuccess)
            return fail("event", e);
    }
    if ((e = hipEventCreateWithFlags(&ctx->ev_gram2, hipEventDisableTiming)) != hipSuccess)
        return fail("event", e);
    if ((e = hipEventCreateWithFlags(&ctx->ev_xinit, hipEventDisableTiming)) != hipSuccess)
        return fail("event", e);
    if ((e = hipEventCreateWithFlags(&ctx->ev_xdone, hipEventDisableTiming)) != hipSuccess)
        return fail("event", e);
    if ((e = hipMalloc(reinterpret_cast<void**>(&ctx->dres), sizeof(EvalResult))) != hipSuccess)
        return fail("hipMalloc", e);
    if ((e = hipHostMalloc(reinterpret_cast<void**>(&ctx->hres), sizeof(EvalResult), 0)) != hipSuccess)
        return fail("hipHostMalloc", e);
    if ((e = hipMalloc(reinterpret_cast<void**>(&ctx->dtp), sizeof(TermPack))) != hipSuccess)
        return fail("hipMalloc", e);
    if ((e = hipHostMalloc(reinterpret_cast<void**>(&ctx->htp), sizeof(TermPack), 0)) != hipSuccess)
        return fail("hipHostMalloc", e);
    if ((e = hipMalloc(reinterpret_cast<void**>(&ctx->gout), sizeof(double) * (GAPLAC_MAX_TERMS + 1))) != hipSuccess)
        return fail("hipMalloc", e);
    if ((e = hipHostMalloc(reinterpret_cast<void**>(&ctx->hgout), sizeof(double) * (GAPLAC_MAX_TERMS + 1), 0)) !=
        hipSuccess)
        return fail("hipHostMalloc", e);
    if ((e = hipMalloc(reinterpret_cast<void**>(&ctx->dgp), sizeof(GradTermPack))) != hipSuccess)
        return fail("hipMalloc", e);
    if ((e = hipHostMalloc(reinterpret_cast<void**>(&ctx->hgp), sizeof(GradTermPack), 0)) != hipSuccess)
        return fail("hipHostMalloc", e);
    *out = ctx;
    return 0;
}

int gaplac_ctx_destroy(gaplac_ctx* ctx) {
    if (!ctx) return 0;
    (void)hipSetDevice(ctx->device);
    if (ctx->s_main) (void)hipStreamSynchronize(ctx->s_main);
    if (ctx->s_panel) (void)hipStreamSynchronize(ctx->s_panel);
    if (ctx->s_extra) (void)hipStreamSynchronize(ctx->s_extra);
    if (ctx->s_xrest) (void)hipStreamSynchronize(ctx->s_xrest);
    for (gaplac_ctx* c : ctx->lanes) gaplac_ctx_destroy(c);
    ctx->lanes.clear();
    if (ctx->borrowed_inputs) {
        ctx->dX = nullptr;
        ctx->dv = nullptr;
    }
    for (int q = 0; q < 2; ++q) {
        if (ctx->ev_P[q]) (void)hipEventDestroy(ctx->ev_P[q]);
        if (ctx->ev_R[q]) (void)hipEventDestroy(ctx->ev_R[q]);
        if (ctx->ev_xc[q]) (void)hipEventDestroy(ctx->ev_xc[q]);
        if (ctx->ev_xr[q]) (void)hipEventDestroy(ctx->ev_xr[q]);
    }
    if (ctx->ev_gram) (void)hipEventDestroy(ctx->ev_gram);
    if (ctx->ev_gram2) (void)hipEventDestroy(ctx->ev_gram2);
    for (int q = 0; q < 2; ++q) {
        if (ctx->ev_split[q]) (void)hipEventDestroy(ctx->ev_split[q]);
        if (ctx->ev_rest[q]) (void)hipEventDestroy(ctx->ev_rest[q]);
    }
    if (ctx->ev_xinit) (void)hipEventDestroy(ctx->ev_xinit);
    if (ctx->ev_xdone) (void)hipEventDestroy(ctx->ev_xdone);
    if (ctx->A) (void)hipFree(ctx->A);
    if (ctx->Dinv) (void)hipFree(ctx->Dinv);
    if (ctx->tiles) (void)hipFree(ctx->tiles);
    if (ctx->dX) (void)hipFree(ctx->dX);
    if (ctx->dv) (void)hipFree(ctx->dv);
    for (hipEvent_t e : ctx->evpool) (void)hipEventDestroy(e);
    if (ctx->dkt) (void)hipFree(ctx->dkt);
    if (ctx->hkt) (void)hipHostFree(ctx->hkt);
    if (ctx->galpha) (void)hipFree(ctx->galpha);
    if (ctx->dXs) (void)hipFree(ctx->dXs);
    if (ctx->pmean) (void)hipFree(ctx->pmean);
    if (ctx->pvar) (void)hipFree(ctx->pvar);
    if (ctx->gdv) (void)hipFree(ctx->gdv);
    if (ctx->gz) (void)hipFree(ctx->gz);
    if (ctx->gpart) (void)hipFree(ctx->gpart);
    if (ctx->gout) (void)hipFree(ctx->gout);
    if (ctx->hgout) (void)hipHostFree(ctx->hgout);
    if (ctx->dgp) (void)hipFree(ctx->dgp);
    if (ctx->hgp) (void)hipHostFree(ctx->hgp);
    if (ctx->glist) (void)hipFree(ctx->glist);
    if (ctx->tctl) (void)hipFree(ctx->tctl);
    for (auto& w : ctx->bw) {
        if (w.A) (void)hipFree(w.A);
        if (w.Dinv) (void)hipFree(w.Dinv);
        if (w.dres) (void)hipFree(w.dres);
        if (w.dtp) (void)hipFree(w.dtp);
        if (w.hres) (void)hipHostFree(w.hres);
        if (w.htp) (void)hipHostFree(w.htp);
        if (w.ctl) (void)hipFree(w.ctl);
        if (w.tasks) (void)hipFree(w.tasks);
        if (w.ev_gram) (void)hipEventDestroy(w.ev_gram);
        if (w.ev_done) (void)hipEventDestroy(w.ev_done);
    }
    if (ctx->ttasks) (void)hipFree(ctx->ttasks);
    if (ctx->ttrace) (void)hipFree(ctx->ttrace);
    if (ctx->dres) (void)hipFree(ctx->dres);
    if (ctx->dtp) (void)hipFree(ctx->dtp);
    if (ctx->htp) (void)hipHostFree(ctx->htp);
    if (ctx->hres) (void)hipHostFree(ctx->hres);
    if (ctx->s_main) (void)hipStreamDestroy(ctx->s_main);
    if (ctx->s_panel) (void)hipStreamDestroy(ctx->s_panel);
    if (ctx->s_extra) (void)hipStreamDestroy(ctx->s_extra);
    if (ctx->s_xrest) (void)hipStreamDestroy(ctx->s_xrest);
    delete ctx;
    return 0;
}

int gaplac_ctx_release(gaplac_ctx* ctx) {
    if (!ctx) return GAPLAC_E_ARG;
    HIPCK(ctx, hipSetDevice(ctx->device));
    HIPCK(ctx, hipStreamSynchronize(ctx->s_main));
    HIPCK(ctx, hipStreamSynchronize(ctx->s_panel));
    if (ctx->s_extra) HIPCK(ctx, hipStreamSynchronize(ctx->s_extra));
    if (ctx->s_xrest) HIPCK(ctx, hipStreamSynchronize(ctx->s_xrest));
    for (gaplac_ctx* c : ctx->lanes) gaplac_ctx_destroy(c);
    ctx->lanes.clear();
    auto drop = [](double*& p, size_t& n) {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    };
    drop(ctx->A, ctx->A_elems);
    drop(ctx->Dinv, ctx->Dinv_elems);
    for (auto& w : ctx->bw) {
        if (w.busy) HIPCK(ctx, hipEventSynchronize(w.ev_done));
        w.busy = false;
        drop(w.A, w.A_elems);
        drop(w.Dinv, w.Dinv_elems);
    }
    return 0;
}

int gaplac_logpdf_device(gaplac_ctx* ctx, int64_t N, int32_t D, const double* dX, int64_t ldx,
                         int32_t T, const gaplac_term* terms, double noise, const double* dv,
                         double* out_logpdf, double* out_logdet, double* out_quad) {
    nan_out(out_logpdf, out_logdet, out_quad);
    int rc = check_common(ctx, N, D, dX, ldx, noise, dv);
    if (rc) return rc;
    TermPack tp;
    if ((rc = pack_terms(ctx, D, T, terms, &tp))) return rc;
    if (N == 0) {  // logpdf of an empty FiniteGP: -(0 + 0 + 0)/2
        if (out_logpdf) *out_logpdf = -0.0;
        if (out_logdet) *out_logdet = 0.0;
        if (out_quad) *out_quad = 0.0;
        return 0;
    }
    tp.noise = noise;
    HIPCK(ctx, hipSetDevice(ctx->device));
    if ((rc = upload_device(ctx, N, D, dX, ldx, dv))) return rc;
    EvalResult r;
    if ((rc = eval_device(ctx, N, D, tp, &r))) return rc;
    return finish(r, out_logpdf, out_logdet, out_quad);
}

int gaplac_logpdf(gaplac_ctx* ctx, int64_t N, int32_t D, const double* X, int64_t ldx, int32_t T,
                  const gaplac_term* terms, double noise, const double* v, double* out_logpdf,
                  double* out_logdet, double* out_quad) {
    nan_out(out_logpdf, out_logdet, out_quad);
    int rc = check_common(ctx, N, D, X, ldx, noise, v);
    if (rc) return rc;
    TermPack tp;
    if ((rc = pack_terms(ctx, D, T, terms, &tp))) return rc;
    if (N == 0) {
        if (out_logpdf) *out_logpdf = -0.0;
        if (out_logdet) *out_logdet = 0.0;
        if (out_quad) *out_quad = 0.0;
        return 0;
    }
    HIPCK(ctx, hipSetDevice(ctx->device));
    if ((rc = upload(ctx, N, D, X, ldx, v))) return rc;
    tp.noise = noise;
    EvalResult r;
    if ((rc = eval_device(ctx, N, D, tp, &r))) return rc;
    return finish(r, out_logpdf, out_logdet, out_quad);
}

int gaplac_logpdf_batch(gaplac_ctx* ctx, int32_t nmodels, int64_t N, int32_t D, const double* X,
                        int64_t ldx, const int32_t* term_offset, const gaplac_term* terms,
                        double noise, const double* v, double* out_logpdf, int64_t* out_info) {
    if (!ctx) return GAPLAC_E_ARG;
    if (nmodels < 0 || (nmodels > 0 && (!term_offset || !out_logpdf || !out_info)))
        return set_err(ctx, GAPLAC_E_ARG, "bad batch arguments");
    for (int m = 0; m < nmodels; ++m) {
        out_logpdf[m] = NAN;
        out_info[m] = 0;
    }
    int rc = check_common(ctx, N, D, X, ldx, noise, v);
    if (rc) return rc;
    std::vector<TermPack> packs((size_t)nmodels);
    for (int m = 0; m < nmodels; ++m) {
        const int32_t a = term_offset[m], b = term_offset[m + 1];
        if (a < 0 || b < a) return set_err(ctx, GAPLAC_E_ARG, "model %d: bad term offsets", m);
        if ((rc = pack_terms(ctx, D, b - a, terms + a, &packs[(size_t)m]))) return rc;
    }
    if (N == 0) {
        for (int m = 0; m < nmodels; ++m) out_logpdf[m] = -0.0;
        return 0;
    }
    HIPCK(ctx, hipSetDevice(ctx->device));
    {
        const int nt = (int)(round_up(N + 1, NB) / NB);
        // Models per batched launch, capped by the free device memory: two workspace sets of
        // bw matrices must fit beside everything else on the device (what the sets already
        // hold is reusable). Below two models per set the lane path runs instead.
        int bwid = std::min(ctx->batch_w, std::max(nmodels, 1));
        if (nmodels >= 2 && whole_in_tail(ctx, nt)) {
            const int64_t Np = (int64_t)nt * NB;
            const size_t per = ((size_t)Np * (size_t)Np + (size_t)nt * DINV_PER_BLOCK) * sizeof(double) +
                               sizeof(TailCtl) + sizeof(EvalResult) + sizeof(TermPack);
            size_t freeb = 0, totalb = 0;
            if (hipMemGetInfo(&freeb, &totalb) == hipSuccess) {
                size_t held = 0;
                for (const auto& w : ctx->bw) held += (w.A_elems + w.Dinv_elems) * sizeof(double);
                const size_t margin = (size_t)2 << 30;  // 2 GiB for everything else
                const size_t budget = freeb + held > margin ? freeb + held - margin : 0;
                bwid = (int)std::min<size_t>((size_t)bwid, budget / (2 * per));
            }
        }
        if (nmodels >= 2 && bwid >= 2 && whole_in_tail(ctx, nt)) {  // batched tail
            for (gaplac_ctx* c : ctx->lanes) HIPCK(ctx, hipStreamSynchronize(c->s_main));
            if ((rc = upload(ctx, N, D, X, ldx, v))) return rc;
            HIPCK(ctx, hipStreamSynchronize(ctx->s_main));  // the Grams read X / v on s_panel
            for (int m = 0; m < nmodels; ++m) packs[(size_t)m].noise = noise;
            int p = 0;
            for (int m0 = 0; m0 < nmodels; m0 += bwid, p ^= 1) {
                const int B = std::min(bwid, nmodels - m0);
                if ((rc = batch_tail_enqueue(ctx, N, packs, m0, B, p, out_logpdf, out_info))) break;
            }
            // collect both sets (also after a failure: nothing of this call stays in flight)
            for (int q = 0; q < 2; ++q) {
                const int r2 = batch_tail_finish(ctx, q, out_logpdf, out_info);
                if (!rc) rc = r2;
            }
            return rc;
        }
    }
    // the lanes borrow dX / dv: nothing of an earlier call may still read them
    for (gaplac_ctx* c : ctx->lanes) HIPCK(ctx, hipStreamSynchronize(c->s_main));
    if ((rc = upload(ctx, N, D, X, ldx, v))) return rc;
    HIPCK(ctx, hipStreamSynchronize(ctx->s_main));  // lanes read X / v on their own streams
    // Models in flight on up to batch_lanes lanes (lane 0 = this context): an order-8192
    // evaluation alone fills the chip only ~half the time (its panel chain is a
    // latency-bound critical path), so concurrent models fill the gaps.
    int nl = std::max(1, std::min(ctx->batch_lanes, nmodels));
    {
        // every extra lane holds a whole evaluation workspace: keep the extra lanes that fit
        // in the free device memory beside this context's own workspace (the workspaces
        // already held are reusable; 2 GiB kept free for everything else). Lane 0 is this
        // context: it is never refused here (as a single gaplac_logpdf call would not be);
        // if even its workspace does not fit, ensure_workspace reports the real OOM.
        const int64_t Np = round_up(N + 1, NB);
        const size_t per = (size_t)Np * (size_t)Np * sizeof(double) + (size_t)(Np / NB) * DINV_PER_BLOCK * sizeof(double);
        size_t freeb = 0, totalb = 0;
        if (nl > 1 && hipMemGetInfo(&freeb, &totalb) == hipSuccess) {
            const size_t own = ctx->A_elems * sizeof(double);
            size_t held = 0;
            for (size_t l = 0; l + 1 < (size_t)nl && l < ctx->lanes.size(); ++l) held += ctx->lanes[l]->A_elems * sizeof(double);
            const size_t margin = (size_t)2 << 30;
            const size_t own_need = own >= per ? 0 : per - own;  // lane 0's workspace still to allocate
            const size_t avail = freeb + held;
            const size_t budget = avail > margin + own_need ? avail - margin - own_need : 0;
            nl = 1 + (int)std::min<size_t>((size_t)(nl - 1), budget / per);
        }
    }
    while ((int)ctx->lanes.size() < nl - 1) {
        gaplac_ctx* c = nullptr;
        if ((rc = gaplac_ctx_create(ctx->device, &c))) return set_err(ctx, rc, "batch lane creation failed");
        c->borrowed_inputs = true;
        ctx->lanes.push_back(c);
    }
    std::vector<gaplac_ctx*> lane((size_t)nl, ctx);
    for (int l = 1; l < nl; ++l) {
        gaplac_ctx* c = ctx->lanes[(size_t)l - 1];
        c->dX = ctx->dX;
        c->dX_elems = ctx->dX_elems;
        c->dv = ctx->dv;
        c->dv_elems = ctx->dv_elems;
        lane[(size_t)l] = c;
    }
    for (int l = 0; l < nl; ++l) lane[(size_t)l]->tail_share = nl;
    struct ShareReset {
        std::vector<gaplac_ctx*>& ls;
        ~ShareReset() {
            for (gaplac_ctx* c : ls) c->tail_share = 1;
        }
    } share_reset{lane};
    std::vector<int> pending((size_t)nl, -1);
    auto drain = [&](int l) -> int {
        const int m = pending[(size_t)l];
        if (m < 0) return 0;
        EvalResult r;
        int e = eval_wait(lane[(size_t)l], &r);
        if (e) return set_err(ctx, e, "batch lane %d: %s", l, lane[(size_t)l]->err.c_str());
        out_info[m] = finish(r, &out_logpdf[m], nullptr, nullptr);
        pending[(size_t)l] = -1;
        return 0;
    };
    // on an error, wait for every lane still in flight before returning: they read the
    // borrowed dX / dv, which the next call's upload overwrites
    auto quiesce = [&](int code) -> int {
        for (int l = 0; l < nl; ++l) {
            gaplac_ctx* c = lane[(size_t)l];
            (void)hipStreamSynchronize(c->s_main);
            (void)hipStreamSynchronize(c->s_panel);
            if (c->s_extra) (void)hipStreamSynchronize(c->s_extra);
            if (c->s_xrest) (void)hipStreamSynchronize(c->s_xrest);
        }
        return code;
    };
    for (int m = 0; m < nmodels; ++m) {
        const int l = m % nl;
        if ((rc = drain(l))) return quiesce(rc);
        packs[(size_t)m].noise = noise;
        if ((rc = eval_enqueue(lane[(size_t)l], N, D, packs[(size_t)m])))
            return quiesce(set_err(ctx, rc, "batch lane %d: %s", l, lane[(size_t)l]->err.c_str()));
        pending[(size_t)l] = m;
    }
    for (int l = 0; l < nl; ++l)
        if ((rc = drain(l))) return quiesce(rc);
    return 0;
}

int gaplac_gram(gaplac_ctx* ctx, int64_t N, int32_t D, const double* X, int64_t ldx, int32_t T,
                const gaplac_term* terms, double noise, double* out_C, int64_t ldc) {
    int rc = check_common(ctx, N, D, X, ldx, noise, X /* v unused */);
    if (rc && N > 0) return rc;
    if (N == 0) return 0;
    if (!out_C || ldc < N) return set_err(ctx, GAPLAC_E_ARG, "out_C NULL or ldc < N");
    TermPack tp;
    if ((rc = pack_terms(ctx, D, T, terms, &tp))) return rc;
    HIPCK(ctx, hipSetDevice(ctx->device));
    std::vector<double> zeros((size_t)N, 0.0);
    if ((rc = upload(ctx, N, D, X, ldx, zeros.data()))) return rc;
    const int64_t Np = round_up(N + 1, NB);
    const int nt = (int)(Np / NB);
    if ((rc = ensure(ctx, &ctx->A, &ctx->A_elems, (size_t)Np * Np))) return rc;
    tp.noise = noise;
    *ctx->htp = tp;
    HIPCK(ctx, hipMemcpyAsync(ctx->dtp, ctx->htp, sizeof(TermPack), hipMemcpyHostToDevice, ctx->s_main));
    {
        LaunchGuard g;
        g.base = ctx->A;
        g.elems = (int64_t)ctx->A_elems;
        GuardScope scope(&g);
        launch_gram(ctx->s_main, ctx->A, Np, N, nt, ctx->dX, N, ctx->dv, ctx->dtp, 0, 0, nullptr);
        if (g.violations) return set_err(ctx, GAPLAC_E_ARG, "launch footprint outside the workspace: %s", g.first.c_str());
    }
    HIPCK(ctx, hipGetLastError());
    HIPCK(ctx, hipMemcpy2DAsync(out_C, (size_t)ldc * 8, ctx->A, (size_t)Np * 8, (size_t)N * 8,
                                (size_t)N, hipMemcpyDeviceToHost, ctx->s_main));
    HIPCK(ctx, hipStreamSynchronize(ctx->s_main));
    // only the lower triangle is built on the device; mirror it
    for (int64_t j = 0; j < N; ++j)
        for (int64_t i = 0; i < j; ++i) out_C[j * ldc + i] = out_C[i * ldc + j];
    return 0;
}

int gaplac_gram_time(gaplac_ctx* ctx, int64_t N, int32_t D, const double* X, int64_t ldx, int32_t T,
                     const gaplac_term* terms, double noise, const double* v, int32_t reps, double* best_ms,
                     double* bytes) {
    int rc = check_common(ctx, N, D, X, ldx, noise, v);
    if (rc) return rc;
    if (N == 0 || reps < 1 || !best_ms || !bytes) return set_err(ctx, GAPLAC_E_ARG, "N = 0, reps < 1 or NULL outputs");
    TermPack tp;
    if ((rc = pack_terms(ctx, D, T, terms, &tp))) return rc;
    HIPCK(ctx, hipSetDevice(ctx->device));
    if ((rc = upload(ctx, N, D, X, ldx, v))) return rc;
    const int64_t Np = round_up(N + 1, NB);
    const int nt = (int)(Np / NB);
    if ((rc = ensure(ctx, &ctx->A, &ctx->A_elems, (size_t)Np * Np))) return rc;
    tp.noise = noise;
    *ctx->htp = tp;
    HIPCK(ctx, hipMemcpyAsync(ctx->dtp, ctx->htp, sizeof(TermPack), hipMemcpyHostToDevice, ctx->s_main));
    hipEvent_t e0, e1;
    HIPCK(ctx, hipEventCreate(&e0));
    if (hipEventCreate(&e1) != hipSuccess) {
        (void)hipEventDestroy(e0);
        return set_err(ctx, GAPLAC_E_HIP, "hipEventCreate failed");
    }
    double best = 1e300;
    {
        LaunchGuard g;
        g.base = ctx->A;
        g.elems = (int64_t)ctx->A_elems;
        GuardScope scope(&g);
        for (int r = 0; r < reps && rc == 0; ++r) {
            float ms = 0.f;
            if (hipEventRecord(e0, ctx->s_main) != hipSuccess) rc = GAPLAC_E_HIP;
            launch_gram(ctx->s_main, ctx->A, Np, N, nt, ctx->dX, N, ctx->dv, ctx->dtp, 0, 0, nullptr);
            if (rc == 0 && (hipEventRecord(e1, ctx->s_main) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
                            hipEventElapsedTime(&ms, e0, e1) != hipSuccess))
                rc = GAPLAC_E_HIP;
            if (rc == 0) best = std::min(best, (double)ms);
        }
        if (g.violations) rc = GAPLAC_E_ARG;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (rc) return set_err(ctx, rc, "gram timing failed");
    *best_ms = best;
    *bytes = 8.0 * (double)Np * (double)(Np + 1) / 2.0 + 8.0 * (double)N * (D + 1);
    return 0;
}

int gaplac_factor(gaplac_ctx* ctx, int64_t N, int32_t D, const double* X, int64_t ldx, int32_t T,
                  const gaplac_term* terms, double noise, const double* v, double* out_L,
                  int64_t ldl, double* out_z) {
    int rc = check_common(ctx, N, D, X, ldx, noise, v);
    if (rc) return rc;
    if (N == 0) return 0;
    if (!out_L || ldl < N || !out_z) return set_err(ctx, GAPLAC_E_ARG, "bad output buffers");
    TermPack tp;
    if ((rc = pack_terms(ctx, D, T, terms, &tp))) return rc;
    HIPCK(ctx, hipSetDevice(ctx->device));
    if ((rc = upload(ctx, N, D, X, ldx, v))) return rc;
    tp.noise = noise;
    EvalResult r;
    if ((rc = eval_device(ctx, N, D, tp, &r))) return rc;
    const int64_t Np = round_up(N + 1, NB);
    HIPCK(ctx, hipMemcpy2D(out_L, (size_t)ldl * 8, ctx->A, (size_t)Np * 8, (size_t)N * 8, (size_t)N,
                           hipMemcpyDeviceToHost));
    HIPCK(ctx, hipMemcpy2D(out_z, 8, ctx->A + N, (size_t)Np * 8, 8, (size_t)N, hipMemcpyDeviceToHost));
    for (int64_t j = 0; j < N; ++j)
        for (int64_t i = 0; i < j; ++i) out_L[j * ldl + i] = 0.0;
    return finish(r, nullptr, nullptr, nullptr);
}

int gaplac_logpdf_grad(gaplac_ctx* ctx, int64_t N, int32_t D, const double* X, int64_t ldx, int32_t T,
                       const gaplac_term* terms, double noise, const double* v, double* out_logpdf,
                       double* out_dv, double* out_dparam, double* out_dnoise) {
    return logpdf_grad_impl(ctx, false, N, D, X, ldx, T, terms, noise, v, out_logpdf, out_dv, out_dparam,
                            out_dnoise);
}

int gaplac_logpdf_grad_device(gaplac_ctx* ctx, int64_t N, int32_t D, const double* dX, int64_t ldx, int32_t T,
                              const gaplac_term* terms, double noise, const double* dv, double* out_logpdf,
                              double* out_dv, double* out_dparam, double* out_dnoise) {
    return logpdf_grad_impl(ctx, true, N, D, dX, ldx, T, terms, noise, dv, out_logpdf, out_dv, out_dparam,
                            out_dnoise);
}

int gaplac_posterior_mean_var(gaplac_ctx* ctx, int64_t N, int32_t D, const double* X, int64_t ldx, int32_t T,
                              const gaplac_term* terms, double noise, const double* y, int64_t M,
                              const double* Xs, int64_t ldxs, double* out_mean, double* out_var) {
    return posterior_impl(ctx, N, D, X, ldx, T, terms, noise, y, M, Xs, ldxs, out_mean, out_var);
}

int gaplac_rand(gaplac_ctx* ctx, int64_t N, int32_t D, const double* X, int64_t ldx, int32_t T,
                const gaplac_term* terms, double noise, const double* z, double* out) {
    if (out)
        for (int64_t i = 0; i < N; ++i) out[i] = NAN;
    int rc = check_common(ctx, N, D, X, ldx, noise, z);
    if (rc) return rc;
    if (N > 0 && !out) return set_err(ctx, GAPLAC_E_ARG, "out is NULL");
    TermPack tp;
    if ((rc = pack_terms(ctx, D, T, terms, &tp))) return rc;
    if (N == 0) return 0;
    HIPCK(ctx, hipSetDevice(ctx->device));
    if ((rc = upload(ctx, N, D, X, ldx, z))) return rc;  // z also rides in the v row (unused)
    tp.noise = noise;
    EvalResult r;
    if ((rc = eval_device(ctx, N, D, tp, &r))) return rc;
    if ((rc = finish(r, nullptr, nullptr, nullptr))) return rc;
    const size_t nk = (size_t)((N + 511) / 512);
    if ((rc = ensure(ctx, &ctx->gpart, &ctx->gpart_elems, nk * (size_t)N))) return rc;
    if ((rc = ensure(ctx, &ctx->gdv, &ctx->gdv_elems, (size_t)N))) return rc;
    const int64_t Np = round_up(N + 1, NB);
    {
        LaunchGuard g;
        g.base = ctx->A;
        g.elems = (int64_t)ctx->A_elems;
        GuardScope scope(&g);
        launch_lower_mv(ctx->s_main, ctx->A, Np, N, ctx->dv, ctx->gpart, ctx->gdv);
        if (g.violations) return set_err(ctx, GAPLAC_E_ARG, "launch footprint outside the workspace: %s", g.first.c_str());
    }
    HIPCK(ctx, hipGetLastError());
    HIPCK(ctx, hipMemcpyAsync(out, ctx->gdv, (size_t)N * 8, hipMemcpyDeviceToHost, ctx->s_main));
    HIPCK(ctx, hipStreamSynchronize(ctx->s_main));
    return 0;
}

// Host-only walk of one evaluation's schedule (no device needed): every launch's element
// range is checked against the workspace ensure_workspace would allocate for N.
// mode 0: logpdf; 1: logpdf + gradient (identity rows); 2: posterior at M test points.
int gaplac_plan_check(int64_t N, int32_t mode, int64_t M, int32_t spw, int64_t* out_launches,
                      int64_t* out_violations, char* msg, int64_t msglen) {
    const bool short_ws = mode >= 8;  // negative control: a workspace one element short
    if (short_ws) mode -= 8;
    if (N < 1 || mode < 0 || mode > 2 || (mode == 2 && M < 1) || spw < 1 || spw > 8) return GAPLAC_E_ARG;
    gaplac_ctx c;
    c.dry = true;
    c.spw = spw;
    const int64_t Np = round_up(N + 1, NB);
    const int nt = (int)(Np / NB);
    c.xr_mode = mode;
    c.xr_tiles = mode == 1 ? nt : mode == 2 ? (int)((M + NB - 1) / NB) : 0;
    c.xr_M = mode == 2 ? M : 0;
    // never dereferenced: the walk only does pointer arithmetic against the guard's base
    double* const fake = reinterpret_cast<double*>((uintptr_t)1 << 44);
    c.A = fake;
    c.A_elems = (size_t)(Np + (int64_t)NB * c.xr_tiles) * (size_t)Np;  // as ensure_workspace
    c.Dinv = fake;
    c.tiles = reinterpret_cast<uint32_t*>(fake);
    c.tile_off.assign((size_t)nt + 1, 0);
    for (int m = 1; m <= nt; ++m) c.tile_off[(size_t)m] = c.tile_off[(size_t)m - 1] + (size_t)(m - 1) * m / 2;
    c.tiles_nt = nt;
    // band list offsets as ensure_tile_lists lays them out (the walk launches the same bands)
    c.band_off.assign((size_t)nt + 1, 0);
    {
        size_t k = c.tile_off[(size_t)nt] + (size_t)nt * (nt + 1) / 2;
        for (int m = 1; m <= nt; ++m) {
            c.band_off[(size_t)m] = k;
            const size_t w = (size_t)std::min(c.spw, m);
            k += w * m - w * (w - 1) / 2;
        }
    }
    if (mode == 1) {
        std::vector<uint32_t> gl;
        build_grad_list((int)((N + NB - 1) / NB), gl);
        c.glist_blocks = (int)gl.size();
    }
    c.tail_s = 80;  // as gaplac_ctx_create sets it with the persistent tail
    {
        // every tail length the library can launch: the task list is a topological order
        static std::string tail_bad = [] {
            for (int T = 1; T <= TAIL_TMAX; ++T)
                for (int gw : {4, 8})
                    for (int near : {2, 3, 4, 8})
                    for (int ql : {0, 7, 24, 40, TAIL_TMAX})
                    for (int wp : {0, 1, 2, 3, 4, 5}) {
                        std::vector<uint32_t> l;
                        build_tail_tasks(T, l, nullptr, gw, near, ql, (wp & 1) != 0, 1 << (wp >> 1));
                        std::string why;
                        if (!check_tail_tasks(T, l, &why)) return why + " (gw " + std::to_string(gw) + ", near " +
                                                                  std::to_string(near) + ")";
                    }
            // single evaluations with the critical sub-diagonal quadrants, with and without the
            // posterior's extra rows
            for (int T = 1; T <= TAIL_TMAX; ++T)
                for (int ql : {GAPLAC_QUAD_LAST, TAIL_TMAX})
                    for (int cq : {0, 1, 2})
                        for (int X : {0, 2}) {
                            if (T + X > TAIL_TMAX) continue;  // (the launch condition)
                            std::vector<uint32_t> l;
                            build_tail_tasks(T, l, nullptr, 4, 4, ql, false, GAPLAC_SINGLE_GROUP, X, cq);
                            std::string why;
                            if (!check_tail_tasks(T, l, &why, X))
                                return why + " (quad_last " + std::to_string(ql) + ", crit_quads " + std::to_string(cq) +
                                       ", extra rows " + std::to_string(X) + ")";
                        }
            // the simulated order (GAPLAC_TAIL_SIM) must come out reordered and checked
            for (int T : {2, 9, 33, 65, 80, 128})
                for (int ql : {GAPLAC_QUAD_LAST, TAIL_TMAX}) {
                    std::vector<uint32_t> l;
                    build_tail_tasks(T, l, nullptr, 4, 4, ql, false, GAPLAC_SINGLE_GROUP, 0, 1);
                    const int st = sim_order_tail_tasks(T, l, 256);
                    if (st != 0)
                        return "simulated tail order (T = " + std::to_string(T) + ", quad_last " + std::to_string(ql) +
                               ") " + (st == 1 ? "stalled" : "failed the dependency check");
                }
            // batched launches: each model's tasks, read out of the interleaved list, are
            // its single list in order (so each is a topological order of its own dataflow)
            for (int T : {1, 2, 9, 33, 65, 80})
                for (int B : {1, 3, 32})
                    for (int lag : {0, 1, 6, 16}) {
                        std::vector<uint32_t> one, all;
                        std::vector<size_t> cs;
                        build_tail_tasks(T, one, &cs);
                        interleave_tail_tasks(one, cs, B, lag, all);
                        std::vector<size_t> at((size_t)B, 0);
                        char b[128];
                        std::snprintf(b, sizeof b, "interleaved tail list (T = %d, B = %d, lag = %d) breaks a model's order",
                                      T, B, lag);
                        if (all.size() != one.size() * (size_t)B) return std::string(b);
                        for (uint32_t e : all) {
                            const size_t m = e >> TAIL_MODEL_SHIFT;
                            if (m >= (size_t)B || at[m] >= one.size() ||
                                (e & ((1u << TAIL_MODEL_SHIFT) - 1)) != one[at[m]++])
                                return std::string(b);
                        }
                    }
            return std::string();
        }();
        if (!tail_bad.empty()) {
            if (msg && msglen > 0) std::snprintf(msg, (size_t)msglen, "%s", tail_bad.c_str());
            return GAPLAC_E_ARG;
        }
    }
    TermPack tp{};
    tp.T = 1;
    c.htp = &tp;
    LaunchGuard g;
    g.base = fake;
    g.elems = (int64_t)c.A_elems - (short_ws ? 1 : 0);
    g.dry = true;
    int rc;
    {
        GuardScope scope(&g);
        rc = enqueue_eval(&c, N, 1, Np, nt);
    }
    c.htp = nullptr;
    c.A = nullptr;
    c.Dinv = nullptr;
    c.tiles = nullptr;
    if (out_launches) *out_launches = g.launches;
    if (out_violations) *out_violations = g.violations;
    if (msg && msglen > 0) std::snprintf(msg, (size_t)msglen, "%s", g.first.c_str());
    return rc == GAPLAC_E_ARG && g.violations ? 0 : rc;
}

// Host-only accounting of the single-GPU schedule: a dry walk of one
// evaluation of order N with the given deferral depth / band extension / cut-off, whose
// launchers record every update (tile columns x panel columns) and every column's
// factorisation in enqueue order (LaunchGuard::acct). Checks that every tile column gets
// every earlier panel column exactly once, in increasing order, before its diagonal block
// (or before the persistent tail that factors it), and that every update reads panel
// columns already factored. 0, or GAPLAC_E_ARG with the first violation in msg.
int gaplac_plan_check_schedule(int64_t N, int32_t spw, int32_t depth, int32_t pair_ext, int32_t pair_m,
                               int64_t* out_records, char* msg, int64_t msglen) {
    if (N < 1 || spw < 1 || spw > 8 || depth < 0 || depth > 8 || pair_ext < 0 || pair_ext > 1 || pair_m < 0)
        return GAPLAC_E_ARG;
    gaplac_ctx c;
    c.dry = true;
    c.spw = spw;
    c.pair_depth = depth;
    c.pair_ext = pair_ext;
    c.pair_m = pair_m;
    const int64_t Np = round_up(N + 1, NB);
    const int nt = (int)(Np / NB);
    double* const fake = reinterpret_cast<double*>((uintptr_t)1 << 44);
    c.A = fake;
    c.A_elems = (size_t)Np * (size_t)Np;
    c.Dinv = fake;
    c.tiles = reinterpret_cast<uint32_t*>(fake);
    c.tile_off.assign((size_t)nt + 1, 0);
    for (int m = 1; m <= nt; ++m) c.tile_off[(size_t)m] = c.tile_off[(size_t)m - 1] + (size_t)(m - 1) * m / 2;
    c.tiles_nt = nt;
    c.band_off.assign((size_t)nt + 1, 0);
    {
        size_t k = c.tile_off[(size_t)nt] + (size_t)nt * (nt + 1) / 2;
        for (int m = 1; m <= nt; ++m) {
            c.band_off[(size_t)m] = k;
            const size_t w = (size_t)std::min(c.spw, m);
            k += w * m - w * (w - 1) / 2;
        }
    }
    c.tail_s = 80;
    TermPack tp{};
    tp.T = 1;
    c.htp = &tp;
    LaunchGuard g;
    g.base = fake;
    g.elems = (int64_t)c.A_elems;
    g.dry = true;
    std::vector<int> acct;
    g.acct = &acct;
    int rc;
    {
        GuardScope scope(&g);
        rc = enqueue_eval(&c, N, 1, Np, nt);
    }
    c.htp = nullptr;
    c.A = nullptr;
    c.Dinv = nullptr;
    c.tiles = nullptr;
    std::string why;
    char b[200];
    if (rc) why = "the dry walk failed";
    if (g.violations && why.empty()) why = g.first;
    std::vector<int> next((size_t)nt, 0);       // next panel column tile column j must receive
    std::vector<char> done((size_t)nt, 0);      // factored (or handed to the tail)
    for (size_t i = 0; i + 5 <= acct.size() && why.empty(); i += 5) {
        const int kind = acct[i], j0 = acct[i + 1], j1 = acct[i + 2], k0 = acct[i + 3], k1 = acct[i + 4];
        if (kind == 0) {
            for (int k = k0; k < k1 && why.empty(); ++k)
                if (k < 0 || k >= nt || !done[(size_t)k]) {
                    std::snprintf(b, sizeof b, "an update reads panel column %d before it is factored", k);
                    why = b;
                }
            for (int j = j0; j < j1 && why.empty(); ++j) {
                if (j < 0 || j >= nt || done[(size_t)j] || next[(size_t)j] != k0 || k1 > j) {
                    std::snprintf(b, sizeof b, "tile column %d gets panel columns %d..%d (expected from %d%s)", j, k0,
                                  k1 - 1, j >= 0 && j < nt ? next[(size_t)j] : -1,
                                  j >= 0 && j < nt && done[(size_t)j] ? ", after its factorisation" : "");
                    why = b;
                } else {
                    next[(size_t)j] = k1;
                }
            }
        } else if (kind == 1) {
            if (j0 < 0 || j0 >= nt) continue;
            if (!done[(size_t)j0] && next[(size_t)j0] != j0) {
                std::snprintf(b, sizeof b, "tile column %d factored with panel columns < %d only", j0,
                              next[(size_t)j0]);
                why = b;
            }
            done[(size_t)j0] = 1;
        } else {
            for (int j = j0; j < nt && why.empty(); ++j) {
                if (done[(size_t)j] || next[(size_t)j] != j0) {
                    std::snprintf(b, sizeof b, "the tail from %d starts with tile column %d at panel %d", j0, j,
                                  next[(size_t)j]);
                    why = b;
                }
                done[(size_t)j] = 1;
            }
        }
    }
    for (int j = 0; j < nt && why.empty(); ++j)
        if (!done[(size_t)j]) {
            std::snprintf(b, sizeof b, "tile column %d never factored", j);
            why = b;
        }
    if (out_records) *out_records = (int64_t)(acct.size() / 5);
    if (msg && msglen > 0) std::snprintf(msg, (size_t)msglen, "%s", why.c_str());
    return why.empty() ? 0 : GAPLAC_E_ARG;
}

int gaplac_set_profiling(gaplac_ctx* ctx, int mode) {
    if (!ctx || mode < 0 || mode > 2) return GAPLAC_E_ARG;
    ctx->prof_mode = mode;
    ctx->profiling = mode == 1;
    return 0;
}

int gaplac_get_stats(gaplac_ctx* ctx, gaplac_stats* out) {
    if (!ctx || !out) return GAPLAC_E_ARG;
    if (!ctx->evpairs.empty()) {  // fold the event-timed bulk launches in
        HIPCK(ctx, hipSetDevice(ctx->device));
        HIPCK(ctx, hipDeviceSynchronize());  // (events on s_main, s_panel and the split's s_xrest)
        std::vector<std::pair<double, double>> iv;  // bulk-type launch intervals, ms after the first event
        const hipEvent_t ref = ctx->evpool[ctx->evpairs.front().i0];
        for (const auto& p : ctx->evpairs) {
            float ms = 0.f;
            HIPCK(ctx, hipEventElapsedTime(&ms, ctx->evpool[p.i0], ctx->evpool[p.i0 + 1]));
            if (p.kind == 8) {
                ctx->stats.cinv_ms += ms;
                ctx->stats.cinv_launches += 1;
                continue;
            }
            float t0 = 0.f;
            HIPCK(ctx, hipEventElapsedTime(&t0, ref, ctx->evpool[p.i0]));
            iv.push_back({(double)t0, (double)t0 + ms});
            ctx->stats.bulk_flops += p.flops;
            ctx->stats.bulk_launches += 1;
            if (p.kind == 5) continue;  // bands, heads, lookaheads: the union only
            ctx->stats.syrk_ms += ms;
            ctx->stats.syrk_flops += p.flops;
            ctx->stats.syrk_bytes += p.bytes;
            ctx->stats.syrk_launches += 1;
        }
        // union of the intervals: the time some bulk-type launch was in flight
        std::sort(iv.begin(), iv.end());
        double cs = -1.0, ce = -1.0;
        for (const auto& x : iv) {
            if (x.first > ce) {
                if (ce > cs) ctx->stats.bulk_union_ms += ce - cs;
                cs = x.first;
                ce = x.second;
            } else {
                ce = std::max(ce, x.second);
            }
        }
        if (ce > cs) ctx->stats.bulk_union_ms += ce - cs;
        ctx->evpairs.clear();
    }
    *out = ctx->stats;
    return 0;
}

int gaplac_reset_stats(gaplac_ctx* ctx) {
    if (!ctx) return GAPLAC_E_ARG;
    ctx->stats = gaplac_stats{};
    ctx->evpairs.clear();
    return 0;
}

}  // extern "C"
