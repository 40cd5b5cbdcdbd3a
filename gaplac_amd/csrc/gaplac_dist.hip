// Distributed evaluation (BASELINE configs[3]): one rank of a 1-D
// block-column cyclic Cholesky of the (N+1)-augmented covariance.
//
// Distribution. Super-panels (SP) of W 128-wide tile columns are dealt in rounds of nranks:
// SP s belongs to rank s % nranks, or with the snake layout (gaplac_dist_set_layout) to
// nranks - 1 - s % nranks in odd rounds. A rank stores only its own tile columns (all Np
// rows, column-major, ldc = Np), in order (ColMap in gaplac_internal.h). Because the Gram is
// symmetric, a rank's block columns of the lower triangle are the block rows of the upper:
// each rank builds exactly the Gram tiles it owns, with no redistribution.
//
// Steps (the host drives them; the only exchange is the panel broadcast):
//   begin          all ranks: local Gram tiles (s_main)
//   factor(s)      owner of SP s (s_panel, critical path): apply panel s-1 to SP s
//                  (lookahead, one launch per broadcast chunk as each chunk arrives),
//                  factor SP s column by column (column updates inside the SP, diagonal
//                  potrf, panel TRSM) and pack each chunk of columns into the panel buffer
//                  as soon as its last column is final
//   bcast(s, c)    the host broadcasts chunk c of panel s from the owner (RCCL on the comm
//                  stream; gaplac_dist_comm_begin_chunk / _end_chunk bracket it)
//   update(s)      all ranks: panel s (and, with deferred updates, the panels before it in
//                  its group) applied to their SPs > s+1 following the step plan below
//                  (s_main); SP s+1 gets panel s in factor(s+1) instead
//   finish         all ranks: partial logdet / quad / info over their columns; the host
//                  sums them across ranks (one allreduce of 3 numbers)
// The host calls, per rank: begin; factor(0) [owner]; bcast(0, *); for s = 0..nsp-1:
// { factor(s+1) [owner of s+1]; update(s); bcast(s+1, *) }; finish. Every call only
// enqueues work: the streams overlap the bulk update with the next panel's chain.
//
// Step plan (build_plan, checked by check_plan / gaplac_dist_plan_check). Panels are grouped
// in aligned groups of D (GAPLAC_DIST_DEPTH; the single-GPU path's deferred updates,
// DESIGN.md §3.2 and §3.6): inside a group only the bands the next chains need (SPs s+2
// and s+3) get the panels they lack, and the SPs after them get every panel of the group
// at once at the group's last step (K = D x 128 W). Every step updates SP s+2 first and
// then records ev_step, so the owner of SP s+2 starts its chain without waiting for the
// rest of the update.
//
// Panel buffers: two GROUP buffers; the D panels of group g share buffer g & 1 with the
// rows of the group's first panel as the common origin (ld = Np - that row; panel i of the
// group starts 128 W i columns in and its rows above its own first row are never read), so
// a deferred update reads the group's panels as one K = D x 128 W panel. A chunk (cw tile
// columns, GAPLAC_DIST_CHUNK) is contiguous in the buffer. Events keep a group buffer from
// being re-filled (packed by its owner or received) before the updates, lookaheads and
// broadcasts that read its previous group have run.
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

namespace {
constexpr int MAXC = 8;  // chunks per panel (W <= 8)

// One operation of a step's bulk update: SP g alone (BAND) or every owned SP >= g (SUF),
// with the panels pf .. pl (one group); MARK: ev_step (SP s+2 is up to date).
enum { OP_BAND = 0, OP_SUF = 1, OP_MARK = 2 };
struct DOp {
    int kind, g, pf, pl;
};

// Device timestamps of the replay, 100 MHz s_memrealtime ticks, per step
// s: UPD(s) update(s) started, BAND(s) SP s+2 up to date in update(s), END(s) update(s)
// done, PACK(s, c) chunk c packed, RECV(s, c) chunk c received (sent, on its owner).
constexpr int ST_PER_STEP = 3 + 2 * MAXC;
// after the nsp steps' stamps: the end of the rank's Gram, the tail gather's modelled
// arrival (gaplac_dist_replay_tail), the end of the root's tail, the end of the replay's
// copies of the gathered segments
constexpr int ST_EXTRA = 4;
inline int st_upd(int s) { return s * ST_PER_STEP; }
inline int st_band(int s) { return s * ST_PER_STEP + 1; }
inline int st_end(int s) { return s * ST_PER_STEP + 2; }
inline int st_pack(int s, int c) { return s * ST_PER_STEP + 3 + c; }
inline int st_recv(int s, int c) { return s * ST_PER_STEP + 3 + MAXC + c; }

// Release of one modelled transfer: spin until max_i(stamps[dep_i] + add_i) (dep_i = -1:
// unused, -2: the kernel's own start), then stamp `out`. Bounded: never spins past start + 2 s.
struct Release {
    int dep[3];
    long long add[3];
    int out;
};
}  // namespace

struct gaplac_dist {
    int device = 0, nranks = 1, rank = 0, W = 4;
    int D = 2;         // GAPLAC_DIST_DEPTH: panels per deferral group
    int cw = 4;        // GAPLAC_DIST_CHUNK: tile columns per broadcast chunk
    int big_mode = 1;  // GAPLAC_DIST_BIG: 0 never, 1 per rank (no chain beside the launch), 2 by launch size
    int big_min = 2048;  // (gaplac_dist_configure) tiles of a launch for the per-rank choice
    int alone = 0;     // GAPLAC_DIST_ALONE: the owner of SP s+1 starts update(s) after its chain
    int snake = 0;     // gaplac_dist_set_layout: boustrophedon dealing of the SPs
    hipStream_t s_main = nullptr, s_panel = nullptr, s_comm = nullptr;
    hipEvent_t ev_gram = nullptr, ev_panel_done = nullptr;
    // ev_recv / ev_packed per panel parity and chunk; ev_step[s & 1]: update(s) brought SP
    // s+2 up to date; ev_free_main / ev_free_panel per group buffer: its last bulk update /
    // lookahead of the buffer's current group done (the broadcasts that refill a buffer are
    // ordered behind the earlier ones by the comm stream itself, so they need no event)
    hipEvent_t ev_recv[2][MAXC] = {}, ev_packed[2][MAXC] = {};
    hipEvent_t ev_step[2] = {}, ev_free_main[2] = {}, ev_free_panel[2] = {};
    hipEvent_t ev_upd[2] = {};  // replay: update(s) started (its UPD stamp written)
    hipEvent_t ev_col[MAXC] = {};  // factor(s): column k of the SP final (its pack may start)
    int pair_m = 40;  // GAPLAC_PAIR_M: deferred updates while >= pair_m tile rows follow SP s+3
    // geometry of the current evaluation
    int64_t N = -1, Np = 0;
    int nt = 0, nsp = 0, nloc = 0;
    int nsteps = 0;  // distributed steps (nsp, or tstop with the tail gather)
    bool factored_any = false;
    std::vector<std::vector<DOp>> plan;
    int plan_nt = -1, plan_stop = -1;
    // tail gather (gaplac_dist_set_tail): SPs tstop .. nsp-1 (the last
    // <= tail_cols tile columns) are factored by rank tail_root's persistent tail after every
    // rank sent it its columns of the trailing matrix (rows and columns >= tN0 = 128 W tstop)
    int tail_cols = 0, tail_root = 0;
    int tstop = -1;  // -1: no gather this evaluation
    int64_t tN0 = 0, tNt = 0;
    std::vector<int64_t> tseg_off, tseg_cnt;  // per segment (SP tstop + i) in this rank's segment buffer; 0: none
    double* tseg = nullptr;   // segment buffer: a sender's own segments, or every segment on the root
    size_t tseg_cap = 0;
    bool tseg_external = false;
    double* tmat = nullptr;   // root: the trailing matrix, tNt x tNt column-major
    size_t tmat_elems = 0;
    double* tDinv = nullptr;
    size_t tDinv_elems = 0;
    EvalResult* tres = nullptr;  // root: the tail's result (pivot indices relative to tN0)
    EvalResult* htres = nullptr; // pinned
    TailCtl* tctl = nullptr;
    uint32_t* ttasks = nullptr;
    size_t ttasks_elems = 0;
    int ttasks_n = 0, ttasks_T = -1;
    int ncu = 256;
    int tail_sim = -1;  // GAPLAC_TAIL_SIM, as the single-GPU path reads it
    bool tail_ended = false;
    hipEvent_t ev_tail = nullptr;  // s_main: the last update done; s_comm: the gather's transfers enqueued
    int held_step = -1;   // alone: the step whose ops after its mark wait for the next update
    size_t held_from = 0;
    // device buffers
    double* C = nullptr;
    size_t C_elems = 0;
    double* Dinv = nullptr;
    size_t Dinv_elems = 0;
    double* pbuf[2] = {};
    size_t pbuf_cap = 0;   // elements per group buffer
    bool pbuf_external = false;
    uint32_t* tiles = nullptr;
    size_t tiles_elems = 0;
    int gram_count = 0;                  // gram list at tiles[0 .. gram_count)
    std::vector<size_t> bulk_off;        // per owned-SP ordinal u: suffix list offset
    std::vector<int> bulk_cnt;           //                            and tile count
    std::vector<size_t> band_off;        // per owned-SP ordinal u: its own tiles only
    std::vector<int> band_cnt;
    int64_t lists_N = -1;
    double* dX = nullptr;
    size_t dX_elems = 0;
    double* dv = nullptr;
    size_t dv_elems = 0;
    EvalResult* dres = nullptr;
    EvalResult* hres = nullptr;  // pinned
    TermPack* dtp = nullptr;
    TermPack* htp = nullptr;     // pinned
    // replay (gaplac_dist_replay_*): device stamps, nullptr = off
    unsigned long long* stamps = nullptr;
    size_t stamps_elems = 0;
    std::string err;
};

namespace {

int derr(gaplac_dist* d, int code, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
int derr(gaplac_dist* d, int code, const char* fmt, ...) {
    if (d) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        d->err = buf;
    }
    return code;
}

#define DCK(d, call)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (call);                                                             \
        if (e_ != hipSuccess)                                                               \
            return derr(d, GAPLAC_E_HIP, "%s failed: %s", #call, hipGetErrorString(e_));    \
    } while (0)

template <typename T>
int dgrow(gaplac_dist* d, T** p, size_t* cap, size_t n) {
    if (*cap >= n) return 0;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (n == 0) return 0;
    if (hipMalloc(reinterpret_cast<void**>(p), n * sizeof(T)) != hipSuccess)
        return derr(d, GAPLAC_E_OOM, "hipMalloc of %zu bytes failed", n * sizeof(T));
    *cap = n;
    return 0;
}

// ---- the step plan (pure host logic) ----

// Does step p defer (only the bands of SPs p+2, p+3 get the group's panels)? Groups are
// aligned (a deferral starts at a group's first step and ends at its last one at the
// latest); pend: the group's first panel while a deferral runs, -1 otherwise.
// stop < nsp (tail gather, gaplac_dist_set_tail): steps stop .. nsp-1 never run, so step
// stop-1 closes any open group.
bool defers(int p, int pend, int nsp, int nt, int W, int D, int pair_m, int stop) {
    if (D < 2 || pair_m <= 0 || p + 4 > nsp || nt - (p + 4) * W < pair_m || p + 1 >= stop) return false;
    return pend < 0 ? p % D == 0 : p % D != D - 1;
}

// Steps 0 .. stop-1 (stop = nsp: all of them). With stop < nsp (the tail gather) the last
// step also applies its panel to SP stop, in place of factor(stop)'s lookahead, so that
// every SP >= stop ends with panels 0 .. stop-1: the trailing matrix the gather moves.
std::vector<std::vector<DOp>> build_plan(int nsp, int nt, int W, int D, int pair_m, int stop) {
    std::vector<std::vector<DOp>> plan((size_t)std::max(stop, 0));
    int pend = -1, dcol = nsp;  // SPs >= dcol lack every panel from pend on
    for (int p = 0; p < stop; ++p) {
        std::vector<DOp>& ops = plan[(size_t)p];
        const bool defer = defers(p, pend, nsp, nt, W, D, pair_m, stop);
        auto first = [&](int g) { return pend >= 0 && g >= dcol ? pend : p; };
        if (p + 2 < nsp) ops.push_back({OP_BAND, p + 2, first(p + 2), p});
        ops.push_back({OP_MARK, p + 2, p, p});
        if (defer) {
            if (p + 3 < nsp) ops.push_back({OP_BAND, p + 3, first(p + 3), p});
            if (pend < 0) pend = p;
            dcol = std::max(pend == p ? 0 : dcol, p + 4);
        } else if (pend >= 0) {
            // the group's last step: SP p+3 and everything after it lack panels pend .. p
            if (p + 3 < nsp) ops.push_back({OP_SUF, std::max(p + 3, dcol), pend, p});
            pend = -1;
            dcol = nsp;
        } else if (p + 3 < nsp) {
            ops.push_back({OP_SUF, p + 3, p, p});
        }
        if (p + 1 == stop && stop < nsp) ops.push_back({OP_BAND, p + 1, p, p});
    }
    return plan;
}

// Every SP g gets panels 0 .. g-1 exactly once and in order (the update ops of steps
// <= g-2, before step g-2's mark, then the lookahead with panel g-1 in factor(g)); every op
// of step p reads panels of p's group only, ending at p. With stop < nsp: every SP >= stop
// ends with panels 0 .. stop-1 (SP stop gets panel stop-1 from the last step's own band).
bool check_plan(const std::vector<std::vector<DOp>>& plan, int nsp, int D, int stop, std::string* why) {
    std::vector<int> next((size_t)nsp, 0);  // next panel SP g must receive
    char buf[256];
    auto fail = [&](const char* fmt, int a, int b, int c) {
        if (why) {
            std::snprintf(buf, sizeof buf, fmt, a, b, c);
            *why = buf;
        }
        return false;
    };
    if ((int)plan.size() != stop || stop < 1 || stop > nsp) return fail("plan of %d steps for stop %d of %d", (int)plan.size(), stop, nsp);
    for (int p = 0; p < stop; ++p) {
        bool marked = false;
        for (const DOp& op : plan[(size_t)p]) {
            if (op.kind == OP_MARK) {
                if (op.g != p + 2) return fail("step %d: mark for SP %d%s", p, op.g, 0);
                marked = true;
                continue;
            }
            if (op.pl != p || op.pf > op.pl || op.pf / D != p / D)
                return fail("step %d reads panels %d..%d", p, op.pf, op.pl);
            const int g1 = op.kind == OP_BAND ? op.g + 1 : nsp;
            for (int g = op.g; g < g1; ++g) {
                const bool last_band = p + 1 == stop && stop < nsp && g == p + 1 && op.kind == OP_BAND && op.pf == p;
                if (g <= p + 1 && !last_band) return fail("step %d updates SP %d (not after its lookahead) %d", p, g, 0);
                if (g == p + 2 && marked) return fail("step %d updates SP %d after the mark%d", p, g, 0);
                if (next[(size_t)g] != op.pf) return fail("SP %d gets panel %d, expected %d", g, op.pf, next[(size_t)g]);
                next[(size_t)g] = op.pl + 1;
            }
        }
        if (!marked) return fail("step %d has no mark%d%d", p, 0, 0);
        // factor(p+1): the lookahead applies panel p to SP p+1
        if (p + 1 < stop) {
            if (next[(size_t)p + 1] != p) return fail("SP %d reaches its chain with panels < %d, needs %d", p + 1,
                                                      next[(size_t)p + 1], p);
            next[(size_t)p + 1] = p + 1;
        }
    }
    for (int g = 0; g < nsp; ++g)
        if (next[(size_t)g] != std::min(g, stop)) return fail("SP %d ends with panels < %d%d", g, next[(size_t)g], 0);
    return true;
}

ColMap cmap(const gaplac_dist* d) { return ColMap{d->nranks, d->rank, d->W, d->snake}; }
int owner(const gaplac_dist* d, int s) {
    const int r = s % d->nranks;
    return d->snake && ((s / d->nranks) & 1) ? d->nranks - 1 - r : r;
}
int sp_first(const gaplac_dist* d, int s) { return s * d->W; }
int sp_width(const gaplac_dist* d, int s) { return std::min(d->W, d->nt - s * d->W); }
int sp_local(const gaplac_dist* d, int s) { return (s / d->nranks) * d->W; }  // first local column
bool owns(const gaplac_dist* d, int s) { return owner(d, s) == d->rank; }
int64_t panel_row0(const gaplac_dist* d, int s) { return (int64_t)sp_first(d, s) * NB; }
// group buffer of panel s: (s / D) & 1; its origin row is that of the group's first panel
int group_buf(const gaplac_dist* d, int s) { return (s / d->D) & 1; }
int group_first(const gaplac_dist* d, int s) { return s / d->D * d->D; }
int64_t group_row0(const gaplac_dist* d, int s) { return panel_row0(d, group_first(d, s)); }
int64_t group_ld(const gaplac_dist* d, int s) { return d->Np - group_row0(d, s); }
// column block of panel s in its group buffer (row origin = group_row0)
double* panel_base(const gaplac_dist* d, int s) {
    return d->pbuf[group_buf(d, s)] + (int64_t)(s - group_first(d, s)) * d->W * NB * group_ld(d, s);
}
Panel panel_of(const gaplac_dist* d, int s) { return Panel{panel_base(d, s), group_ld(d, s), group_row0(d, s)}; }
int nchunks(const gaplac_dist* d, int s) { return (sp_width(d, s) + d->cw - 1) / d->cw; }
int chunk_col0(const gaplac_dist* d, int c) { return c * d->cw; }  // first tile column of chunk c in its SP
int chunk_cols(const gaplac_dist* d, int s, int c) { return std::min(d->cw, sp_width(d, s) - c * d->cw); }
Panel chunk_panel(const gaplac_dist* d, int s, int c) {
    Panel p = panel_of(d, s);
    p.P += (int64_t)chunk_col0(d, c) * NB * p.ld;
    return p;
}
// the chunk's doubles in the buffer: from the panel's first row in its first column to the
// end of its last column (the gap rows above the panel's first row inside the chunk go along)
double* chunk_ptr(const gaplac_dist* d, int s, int c) {
    return const_cast<double*>(chunk_panel(d, s, c).P) + (panel_row0(d, s) - group_row0(d, s));
}
int64_t chunk_count(const gaplac_dist* d, int s, int c) {
    return (int64_t)chunk_cols(d, s, c) * NB * group_ld(d, s) - (panel_row0(d, s) - group_row0(d, s));
}
int64_t chunk_bytes_useful(const gaplac_dist* d, int s, int c) {  // rows >= the panel's first row only
    return (int64_t)chunk_cols(d, s, c) * NB * (d->Np - panel_row0(d, s)) * 8;
}

// ---- tail gather geometry ----
// The first gathered SP for nt tile columns: the first SP whose columns all lie in the last
// tail_cols; -1: no gather (off, or not even one distributed step would remain).
int tail_stop_of(int nt, int W, int tail_cols) {
    const int nsp = (nt + W - 1) / W;
    if (tail_cols <= 0 || nt <= tail_cols) return -1;
    const int s = (nt - tail_cols + W - 1) / W;
    return s >= 1 && s < nsp ? s : -1;
}
int tail_stop(const gaplac_dist* d, int nt, int /*nsp*/) { return tail_stop_of(nt, d->W, d->tail_cols); }
// Segment i of the gather is SP stop + i: its columns from the SP's first row down (the rows
// above it are the trailing matrix's upper triangle), column-major with ld = rows. A rank's
// segment buffer holds the segments it sends (the SPs it owns), the root's every segment.
struct TailGeom {
    int stop = -1;
    int64_t N0 = 0, Nt = 0, elems = 0;
    std::vector<int64_t> off, cnt;  // per segment in this rank's buffer (cnt 0: not on this rank)
};
int64_t tseg_rows(int64_t Nt, int W, int i) { return Nt - (int64_t)i * W * NB; }
TailGeom tail_geom(const gaplac_dist* d, int nt, int nsp, int64_t Np) {
    TailGeom g;
    g.stop = tail_stop(d, nt, nsp);
    if (g.stop < 0) return g;
    g.N0 = (int64_t)g.stop * d->W * NB;
    g.Nt = Np - g.N0;
    for (int s = g.stop; s < nsp; ++s) {
        const int i = s - g.stop;
        const bool here = d->rank == d->tail_root || owns(d, s);
        const int64_t c = (int64_t)std::min(d->W, nt - s * d->W) * NB * tseg_rows(g.Nt, d->W, i);
        g.off.push_back(here ? g.elems : 0);
        g.cnt.push_back(here ? c : 0);
        if (here) g.elems += c;
    }
    return g;
}

// Tile lists: the Gram list (all owned lower tiles), then for every owned SP ordinal u
// the suffix of local columns from u*W (the bulk update set once SPs before it are done),
// in 8x8 super-tile order over (row block, local column).
int build_lists(gaplac_dist* d) {
    if (d->lists_N == d->N) return 0;
    const ColMap cm = cmap(d);
    std::vector<uint32_t> host;
    for (int lj = 0; lj < d->nloc; ++lj)
        for (int bi = cm.global(lj); bi < d->nt; ++bi) host.push_back((uint32_t)bi | ((uint32_t)lj << 16));
    d->gram_count = (int)host.size();
    const int nown = (d->nloc + d->W - 1) / d->W;
    d->bulk_off.assign((size_t)nown, 0);
    d->bulk_cnt.assign((size_t)nown, 0);
    struct E {
        int key0, key1, bi, lj;
    };
    std::vector<E> v;
    for (int u = 0; u < nown; ++u) {
        v.clear();
        const int l0 = u * d->W;
        for (int lj = l0; lj < d->nloc; ++lj)
            for (int bi = cm.global(lj); bi < d->nt; ++bi) v.push_back({bi / 8, (lj - l0) / 8, bi, lj});
        std::sort(v.begin(), v.end(), [](const E& a, const E& b) {
            if (a.key0 != b.key0) return a.key0 < b.key0;
            if (a.key1 != b.key1) return a.key1 < b.key1;
            if (a.bi != b.bi) return a.bi < b.bi;
            return a.lj < b.lj;
        });
        d->bulk_off[(size_t)u] = host.size();
        d->bulk_cnt[(size_t)u] = (int)v.size();
        for (const E& e : v) host.push_back((uint32_t)e.bi | ((uint32_t)e.lj << 16));
    }
    d->band_off.assign((size_t)nown, 0);
    d->band_cnt.assign((size_t)nown, 0);
    for (int u = 0; u < nown; ++u) {  // SP u's tiles, rows outer (one band, as the single path's)
        d->band_off[(size_t)u] = host.size();
        const int l0 = u * d->W, l1 = std::min(d->nloc, l0 + d->W);
        for (int bi = cm.global(l0); bi < d->nt; ++bi)
            for (int lj = l0; lj < l1; ++lj)
                if (bi >= cm.global(lj)) host.push_back((uint32_t)bi | ((uint32_t)lj << 16));
        d->band_cnt[(size_t)u] = (int)(host.size() - d->band_off[(size_t)u]);
    }
    int rc;
    if ((rc = dgrow(d, &d->tiles, &d->tiles_elems, host.size()))) return rc;
    if (!host.empty())
        DCK(d, hipMemcpy(d->tiles, host.data(), host.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    d->lists_N = d->N;
    return 0;
}

// Footprint guard over this rank's column storage (Np x nloc*NB) for the launches of one
// step (gaplac_internal.h).
struct DistGuard {
    gaplac_dist* d;
    LaunchGuard g;
    GuardScope scope;
    explicit DistGuard(gaplac_dist* dd) : d(dd), g(make(dd)), scope(&g) {}
    static LaunchGuard make(const gaplac_dist* dd) {
        LaunchGuard x;
        x.base = dd->C;
        x.elems = dd->Np * (int64_t)dd->nloc * NB;
        return x;
    }
    int check() {
        if (!g.violations) return 0;
        return derr(d, GAPLAC_E_ARG, "launch footprint outside the rank's storage: %s", g.first.c_str());
    }
};

// ---- replay kernels: timestamps and modelled transfers ----
__global__ void stamp_kernel(unsigned long long* slot) {
    if (threadIdx.x == 0) *slot = (unsigned long long)__builtin_amdgcn_s_memrealtime();
}

__global__ void release_kernel(unsigned long long* stamps, Release r) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = (unsigned long long)__builtin_amdgcn_s_memrealtime();
    long long target = 0;
    for (int i = 0; i < 3; ++i)
        if (r.dep[i] >= 0) target = std::max(target, (long long)stamps[r.dep[i]] + r.add[i]);
        else if (r.dep[i] == -2) target = std::max(target, (long long)t0 + r.add[i]);
    const long long limit = (long long)t0 + 200000000ll;  // 2 s at 100 MHz
    if (target > limit) target = limit;
    unsigned long long now = t0;
    while ((long long)now < target) {
        __builtin_amdgcn_s_sleep(4);
        now = (unsigned long long)__builtin_amdgcn_s_memrealtime();
    }
    stamps[r.out] = now;
}

// One 128-column block of a panel, rows .. rows-1 (a multiple of 128) from the column
// storage into the panel buffer: 16-byte loads and stores, 512 rows per workgroup.
__global__ __launch_bounds__(256) void pack_kernel(const double* __restrict__ src, int64_t lds,
                                                   double* __restrict__ dst, int64_t ldd, int64_t rows) {
    const int64_t r = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 2;
    const int col = blockIdx.y;
    if (r >= rows) return;
    const double2 v = *reinterpret_cast<const double2*>(src + col * lds + r);
    *reinterpret_cast<double2*>(dst + col * ldd + r) = v;
}

void launch_pack(hipStream_t s, const double* src, int64_t lds, double* dst, int64_t ldd, int64_t rows) {
    if (rows <= 0 || !guard_launch("pack_kernel")) return;
    pack_kernel<<<dim3((unsigned)((rows + 511) / 512), NB), dim3(256), 0, s>>>(src, lds, dst, ldd, rows);
}

int stamp(gaplac_dist* d, hipStream_t s, int slot) {
    if (!d->stamps) return 0;
    if (!guard_launch("stamp_kernel")) return 0;
    stamp_kernel<<<dim3(1), dim3(64), 0, s>>>(d->stamps + slot);
    return 0;
}

}  // namespace

extern "C" {

const char* gaplac_dist_last_error(const gaplac_dist* d) { return d ? d->err.c_str() : "null context"; }

int gaplac_dist_create(int device, int nranks, int rank, int spw, gaplac_dist** out) {
    if (!out) return GAPLAC_E_ARG;
    *out = nullptr;
    if (nranks < 1 || rank < 0 || rank >= nranks || spw < 1 || spw > MAXC) return GAPLAC_E_ARG;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || device < 0 || device >= n) return GAPLAC_E_NODEVICE;
    gaplac_dist* d = new gaplac_dist();
    d->device = device;
    d->nranks = nranks;
    d->rank = rank;
    d->W = spw;
    // defaults from the one-GPU replay of configs[3]: with several ranks,
    // chunks of two tile columns, the chain alone, the large-launch kernel per rank; one
    // rank keeps the single-GPU rules
    d->cw = nranks > 1 ? std::min(2, spw) : spw;
    d->alone = nranks > 1 ? 1 : 0;
    d->big_mode = nranks == 1 ? 2 : 1;
    // the snake layout evens out the ranks (whole-job replay at N = 65536 over 8:
    // 246.7 -> 240.9 ms); the tail gather stays off by default
    d->snake = nranks > 1 ? 1 : 0;
    auto fail = [&](const char* what, hipError_t e) {
        std::fprintf(stderr, "gaplac_dist_create: %s: %s\n", what, hipGetErrorString(e));
        gaplac_dist_destroy(d);
        return GAPLAC_E_HIP;
    };
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) return fail("hipSetDevice", e);
    int least = 0, greatest = 0;
    if ((e = hipDeviceGetStreamPriorityRange(&least, &greatest)) != hipSuccess) return fail("priorities", e);
    if ((e = hipStreamCreateWithPriority(&d->s_panel, hipStreamNonBlocking, greatest)) != hipSuccess)
        return fail("stream", e);
    if ((e = hipStreamCreateWithPriority(&d->s_comm, hipStreamNonBlocking, greatest)) != hipSuccess)
        return fail("stream", e);
    if ((e = hipStreamCreateWithPriority(&d->s_main, hipStreamNonBlocking, least)) != hipSuccess)
        return fail("stream", e);
    if (const char* e = std::getenv("GAPLAC_PAIR_M")) d->pair_m = std::max(0, std::atoi(e));
    if (const char* e = std::getenv("GAPLAC_DIST_DEPTH")) d->D = std::max(1, std::min(8, std::atoi(e)));
    if (const char* e = std::getenv("GAPLAC_DIST_CHUNK")) d->cw = std::max(1, std::min(spw, std::atoi(e)));
    if (const char* e = std::getenv("GAPLAC_DIST_BIG")) d->big_mode = std::max(0, std::min(2, std::atoi(e)));
    if (const char* e = std::getenv("GAPLAC_DIST_ALONE")) d->alone = std::atoi(e) > 0;
    if (const char* e = std::getenv("GAPLAC_TAIL_SIM")) d->tail_sim = e[0] == '0' ? 0 : 1;
    {
        int ncu = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0)
            d->ncu = ncu;
    }
    std::vector<hipEvent_t*> evs = {&d->ev_gram, &d->ev_panel_done, &d->ev_tail};
    for (int c = 0; c < MAXC; ++c) evs.push_back(&d->ev_col[c]);
    for (int b = 0; b < 2; ++b) {
        for (int c = 0; c < MAXC; ++c) {
            evs.push_back(&d->ev_recv[b][c]);
            evs.push_back(&d->ev_packed[b][c]);
        }
        for (hipEvent_t* ev : {&d->ev_step[b], &d->ev_free_main[b], &d->ev_free_panel[b],
                               &d->ev_upd[b]})
            evs.push_back(ev);
    }
    for (hipEvent_t* ev : evs)
        if ((e = hipEventCreateWithFlags(ev, hipEventDisableTiming)) != hipSuccess) return fail("event", e);
    if ((e = hipMalloc(reinterpret_cast<void**>(&d->dres), sizeof(EvalResult))) != hipSuccess)
        return fail("hipMalloc", e);
    if ((e = hipHostMalloc(reinterpret_cast<void**>(&d->hres), sizeof(EvalResult), 0)) != hipSuccess)
        return fail("hipHostMalloc", e);
    if ((e = hipMalloc(reinterpret_cast<void**>(&d->dtp), sizeof(TermPack))) != hipSuccess)
        return fail("hipMalloc", e);
    if ((e = hipHostMalloc(reinterpret_cast<void**>(&d->htp), sizeof(TermPack), 0)) != hipSuccess)
        return fail("hipHostMalloc", e);
    if ((e = hipHostMalloc(reinterpret_cast<void**>(&d->htres), sizeof(EvalResult), 0)) != hipSuccess)
        return fail("hipHostMalloc", e);
    *out = d;
    return 0;
}

int gaplac_dist_destroy(gaplac_dist* d) {
    if (!d) return 0;
    (void)hipSetDevice(d->device);
    for (hipStream_t s : {d->s_main, d->s_panel, d->s_comm})
        if (s) (void)hipStreamSynchronize(s);
    std::vector<hipEvent_t> evs = {d->ev_gram, d->ev_panel_done, d->ev_tail};
    for (int c = 0; c < MAXC; ++c) evs.push_back(d->ev_col[c]);
    for (int b = 0; b < 2; ++b) {
        for (int c = 0; c < MAXC; ++c) {
            evs.push_back(d->ev_recv[b][c]);
            evs.push_back(d->ev_packed[b][c]);
        }
        for (hipEvent_t ev : {d->ev_step[b], d->ev_free_main[b], d->ev_free_panel[b], d->ev_upd[b]})
            evs.push_back(ev);
    }
    for (hipEvent_t ev : evs)
        if (ev) (void)hipEventDestroy(ev);
    for (void* p : {(void*)d->C, (void*)d->Dinv, (void*)d->tiles, (void*)d->dX, (void*)d->dv, (void*)d->dres,
                    (void*)d->dtp, (void*)d->stamps, (void*)d->tmat, (void*)d->tDinv, (void*)d->tres, (void*)d->tctl,
                    (void*)d->ttasks})
        if (p) (void)hipFree(p);
    if (!d->pbuf_external)
        for (double* p : d->pbuf)
            if (p) (void)hipFree(p);
    if (!d->tseg_external && d->tseg) (void)hipFree(d->tseg);
    if (d->hres) (void)hipHostFree(d->hres);
    if (d->htres) (void)hipHostFree(d->htres);
    if (d->htp) (void)hipHostFree(d->htp);
    for (hipStream_t s : {d->s_main, d->s_panel, d->s_comm})
        if (s) (void)hipStreamDestroy(s);
    delete d;
    return 0;
}

// Super-panel layout, before begin: snake = 1 deals the SPs boustrophedon (rank r owns SP
// u P + r in even rounds u and u P + P - 1 - r in odd ones), 0 round-robin.
int gaplac_dist_set_layout(gaplac_dist* d, int32_t snake) {
    if (!d || snake < 0 || snake > 1) return derr(d, GAPLAC_E_ARG, "set_layout: %d", snake);
    if (d->snake != snake) {
        d->snake = snake;
        d->lists_N = -1;
    }
    return 0;
}

// Owner rank of super-panel s under the current layout.
int gaplac_dist_owner(gaplac_dist* d, int32_t s, int32_t* out_rank) {
    if (!d || s < 0 || !out_rank) return GAPLAC_E_ARG;
    *out_rank = owner(d, s);
    return 0;
}

// Schedule options (the environment's GAPLAC_DIST_* are the defaults): depth = panels per
// deferral group (1 = none), chunk = tile columns per broadcast chunk, big = bulk kernel
// choice (0 never the large-launch kernel, 1 per rank: launches of >= big_min tiles with no
// chain of this rank beside them, 2 by launch size as on one GPU: every rank of an
// in-process loopback job shares one device), alone = 1: the owner of SP s+1 starts its
// update(s) only after its chain of SP s+1 (the chain then has the GPU to itself; the
// bulk share catches up while the rank waits for later panels). A value < 0 leaves the
// option as it is.
int gaplac_dist_configure(gaplac_dist* d, int32_t depth, int32_t chunk, int32_t big, int32_t big_min,
                          int32_t alone) {
    if (!d) return GAPLAC_E_ARG;
    if (depth > 8 || chunk > d->W || big > 2) return derr(d, GAPLAC_E_ARG, "configure: bad option");
    if (depth >= 1 && depth != d->D) {
        if (d->pbuf_external) return derr(d, GAPLAC_E_ARG, "configure: depth changes the panel buffer size");
        d->D = depth;
        d->plan_nt = -1;
    }
    if (depth == 0) return derr(d, GAPLAC_E_ARG, "configure: depth 0");
    if (chunk >= 1) d->cw = chunk;
    if (chunk == 0) return derr(d, GAPLAC_E_ARG, "configure: chunk 0");
    if (big >= 0) d->big_mode = big;
    if (big_min >= 1) d->big_min = big_min;
    if (alone >= 0) d->alone = alone > 0;
    return 0;
}

// Panel buffers provided by the caller (e.g. tensors owned by the host's collective
// library); each must hold at least gaplac_dist_geometry's panel_elems doubles. Passing
// NULLs returns to library-owned buffers.
int gaplac_dist_set_panel_buffers(gaplac_dist* d, void* b0, void* b1, int64_t capacity) {
    if (!d) return GAPLAC_E_ARG;
    DCK(d, hipSetDevice(d->device));
    if (!d->pbuf_external)
        for (double*& p : d->pbuf) {
            if (p) (void)hipFree(p);
            p = nullptr;
        }
    if (b0 && b1 && capacity > 0) {
        d->pbuf[0] = static_cast<double*>(b0);
        d->pbuf[1] = static_cast<double*>(b1);
        d->pbuf_cap = (size_t)capacity;
        d->pbuf_external = true;
    } else {
        d->pbuf[0] = d->pbuf[1] = nullptr;
        d->pbuf_cap = 0;
        d->pbuf_external = false;
    }
    return 0;
}

// Geometry for N: padded order, tile / super-panel counts, this rank's local tile
// columns, and the doubles one group buffer needs (the group of SPs 0 .. D-1).
int gaplac_dist_geometry(gaplac_dist* d, int64_t N, int64_t* Np, int32_t* nt, int32_t* nsp, int32_t* nloc,
                         int64_t* panel_elems) {
    if (!d || N < 1) return derr(d, GAPLAC_E_ARG, "bad geometry query");
    const int64_t np = (N + 1 + NB - 1) / NB * NB;
    const int t = (int)(np / NB);
    const int ns = (t + d->W - 1) / d->W;
    int nl = 0;
    for (int s = 0; s < ns; ++s)
        if (owns(d, s)) nl += std::min(d->W, t - s * d->W);
    if (Np) *Np = np;
    if (nt) *nt = t;
    if (nsp) *nsp = ns;
    if (nloc) *nloc = nl;
    if (panel_elems) *panel_elems = np * (int64_t)std::min(d->D * d->W, t) * NB;
    return 0;
}

int gaplac_dist_begin(gaplac_dist* d, int64_t N, int32_t D, const double* X, int64_t ldx, int32_t T,
                      const gaplac_term* terms, double noise, const double* v, int inputs_on_device,
                      int32_t* out_nsp) {
    if (!d) return GAPLAC_E_ARG;
    if (N < 1 || D < 0 || (D > 0 && (!X || ldx < N)) || !v)
        return derr(d, GAPLAC_E_ARG, "bad inputs (N=%lld D=%d)", (long long)N, D);
    if (!(noise >= 0.0) || !std::isfinite(noise)) return derr(d, GAPLAC_E_PARAM, "noise %g", noise);
    TermPack tp;
    int rc = pack_terms(D, T, terms, &tp, &d->err);
    if (rc) return rc;
    tp.noise = noise;
    DCK(d, hipSetDevice(d->device));
    int32_t nt, nsp, nloc;
    int64_t Np, pel;
    gaplac_dist_geometry(d, N, &Np, &nt, &nsp, &nloc, &pel);
    if (d->N != N) {
        d->N = N;
        d->lists_N = -1;
    }
    d->Np = Np;
    d->nt = nt;
    d->nsp = nsp;
    d->nloc = nloc;
    d->factored_any = false;
    d->held_step = -1;
    d->tail_ended = false;
    const TailGeom tg = tail_geom(d, nt, nsp, Np);
    d->tstop = tg.stop;
    d->nsteps = tg.stop < 0 ? nsp : tg.stop;
    d->tN0 = tg.N0;
    d->tNt = tg.Nt;
    d->tseg_off = tg.off;
    d->tseg_cnt = tg.cnt;
    if (d->plan_nt != nt || d->plan_stop != d->nsteps) {
        d->plan = build_plan(nsp, nt, d->W, d->D, d->pair_m, d->nsteps);
        std::string why;
        if (!check_plan(d->plan, nsp, d->D, d->nsteps, &why)) return derr(d, GAPLAC_E_ARG, "step plan: %s", why.c_str());
        d->plan_nt = nt;
        d->plan_stop = d->nsteps;
    }
    if (tg.stop >= 0) {
        if (d->tseg_external) {
            if (d->tseg_cap < (size_t)tg.elems)
                return derr(d, GAPLAC_E_ARG, "tail buffer holds %zu doubles, %lld needed", d->tseg_cap,
                            (long long)tg.elems);
        } else if ((rc = dgrow(d, &d->tseg, &d->tseg_cap, (size_t)tg.elems))) {
            return rc;
        }
        if (d->rank == d->tail_root) {
            const int T = nt - tg.stop * d->W;
            if ((rc = dgrow(d, &d->tmat, &d->tmat_elems, (size_t)(tg.Nt * tg.Nt)))) return rc;
            if ((rc = dgrow(d, &d->tDinv, &d->tDinv_elems, (size_t)T * DINV_PER_BLOCK))) return rc;
            if (!d->tres) DCK(d, hipMalloc(reinterpret_cast<void**>(&d->tres), sizeof(EvalResult)));
            if (!d->tctl) DCK(d, hipMalloc(reinterpret_cast<void**>(&d->tctl), sizeof(TailCtl)));
            if (d->ttasks_T != T) {
                std::vector<uint32_t> host;
                build_single_tail_list(T, 0, d->tail_sim, d->ncu, host);
                if ((rc = dgrow(d, &d->ttasks, &d->ttasks_elems, host.size()))) return rc;
                DCK(d, hipMemcpy(d->ttasks, host.data(), host.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
                d->ttasks_n = (int)host.size();
                d->ttasks_T = T;
            }
        }
    }
    if ((rc = dgrow(d, &d->C, &d->C_elems, (size_t)Np * nloc * NB))) return rc;
    if ((rc = dgrow(d, &d->Dinv, &d->Dinv_elems, (size_t)nloc * DINV_PER_BLOCK))) return rc;
    if (d->pbuf_external) {
        if (d->pbuf_cap < (size_t)pel)
            return derr(d, GAPLAC_E_ARG, "panel buffers hold %zu doubles, %lld needed", d->pbuf_cap,
                        (long long)pel);
    } else if (d->pbuf_cap < (size_t)pel) {
        size_t c0 = d->pbuf_cap, c1 = d->pbuf_cap;
        if ((rc = dgrow(d, &d->pbuf[0], &c0, (size_t)pel))) return rc;
        if ((rc = dgrow(d, &d->pbuf[1], &c1, (size_t)pel))) return rc;
        d->pbuf_cap = (size_t)pel;
    }
    if ((rc = build_lists(d))) return rc;
    const size_t nx = (size_t)N * (size_t)(D > 0 ? D : 1);
    if ((rc = dgrow(d, &d->dX, &d->dX_elems, nx))) return rc;
    if ((rc = dgrow(d, &d->dv, &d->dv_elems, (size_t)N))) return rc;
    const hipMemcpyKind kind = inputs_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    if (D > 0)
        DCK(d, hipMemcpy2DAsync(d->dX, (size_t)N * 8, X, (size_t)ldx * 8, (size_t)N * 8, (size_t)D, kind, d->s_main));
    DCK(d, hipMemcpyAsync(d->dv, v, (size_t)N * 8, kind, d->s_main));
    *d->htp = tp;
    DCK(d, hipMemcpyAsync(d->dtp, d->htp, sizeof(TermPack), hipMemcpyHostToDevice, d->s_main));
    launch_init_result(d->s_main, d->dres);
    {
        DistGuard guard(d);
        launch_gram_list(d->s_main, d->C, Np, N, d->dX, N, d->dv, d->dtp, d->tiles, d->gram_count, cmap(d), nt - 1,
                         nloc - 1, nullptr);
        if ((rc = guard.check())) return rc;
    }
    if (d->stamps && d->stamps_elems >= (size_t)nsp * ST_PER_STEP + ST_EXTRA) stamp(d, d->s_main, nsp * ST_PER_STEP);
    DCK(d, hipEventRecord(d->ev_gram, d->s_main));
    DCK(d, hipStreamWaitEvent(d->s_panel, d->ev_gram, 0));
    DCK(d, hipGetLastError());
    if (out_nsp) *out_nsp = d->nsteps;
    return 0;
}

// Owner of SP s only. Lookahead update with panel s-1 (chunk by chunk, as each arrives),
// then the SP's column chain, packing each chunk into the group buffer once its last
// column is final (all on s_panel).
int gaplac_dist_factor(gaplac_dist* d, int32_t s) {
    if (!d || s < 0 || s >= d->nsteps) return derr(d, GAPLAC_E_ARG, "factor: step %d out of range", s);
    if (!owns(d, s)) return derr(d, GAPLAC_E_ARG, "factor: rank %d does not own super-panel %d", d->rank, s);
    DCK(d, hipSetDevice(d->device));
    DistGuard guard(d);
    hipStream_t sp = d->s_panel;
    const int c0 = sp_first(d, s), w = sp_width(d, s), lc0 = sp_local(d, s);
    const int64_t ldc = d->Np;
    // update(s-2) brought SP s up to date (ev_step, recorded right after its band)
    DCK(d, hipStreamWaitEvent(sp, d->ev_step[s & 1], 0));
    if (s > 0) {
        const int q = s - 1, nc = nchunks(d, q);
        // alone: nothing of this rank runs beside the chain, so the lookahead takes the
        // whole-tile band kernel (128x128 tiles, the SP's band list); otherwise the 64x64
        // quadrant kernel, which fits beside resident bulk workgroups
        const bool whole = d->alone && d->nranks > 1;
        const size_t u = (size_t)(s / d->nranks);
        for (int c = 0; c < nc; ++c) {
            // this rank's own panel (one rank): packed on the comm stream
            DCK(d, hipStreamWaitEvent(sp, owns(d, q) ? d->ev_packed[q & 1][c] : d->ev_recv[q & 1][c], 0));
            if (whole && d->band_cnt[u] > 0) {
                BulkArgs ba{d->C, d->Np, chunk_panel(d, q, c), d->tiles + d->band_off[u], d->band_cnt[u],
                            chunk_cols(d, q, c) * NB, 0, 0, cmap(d)};
                ba.max_r = d->nt - 1;
                ba.max_c = d->nloc - 1;
                ba.whole = 1;
                launch_bulk(sp, ba, nullptr);
            } else {
                launch_col_update(sp, d->C, ldc, chunk_panel(d, q, c), d->nt, c0, lc0, w, chunk_cols(d, q, c) * NB,
                                  nullptr);
            }
        }
        // this rank's latest lookahead reading the group buffer (the receive of the
        // buffer's next group waits for it on the comm stream)
        DCK(d, hipEventRecord(d->ev_free_panel[group_buf(d, q)], sp));
    }
    const int64_t r0 = panel_row0(d, s), ldp = group_ld(d, s);
    for (int c = c0; c < c0 + w; ++c) {
        const int lc = lc0 + (c - c0);
        double* Acol = d->C + (int64_t)lc * NB * ldc;
        if (c > c0)
            launch_col_update(sp, d->C, ldc, Panel{Acol - NB * ldc, ldc, 0}, d->nt, c, lc, c0 + w - c, NB, nullptr);
        double* Dk = d->Dinv + (size_t)lc * DINV_PER_BLOCK;
        if ((int64_t)c * NB < d->N)
            launch_potrf_diag(sp, Acol + (int64_t)c * NB, ldc, d->N, (int64_t)c * NB, Dk, d->dres, nullptr);
        launch_trsm(sp, Acol, ldc, d->nt, c, Dk, nullptr);
        // column k of the SP is final: pack it on the comm stream, beside the chain's next
        // columns (the comm stream then broadcasts the chunk in order behind its packs)
        const int k = c - c0;
        const int ch = k / d->cw;
        DCK(d, hipEventRecord(d->ev_col[k], sp));
        if (k == 0 && s % d->D == 0) {
            // the packs overwrite group buffer group_buf(s): its previous group's bulk
            // updates must be done (at a group's later panels implied by ev_step, which
            // follows every update of steps <= s - 3); its broadcasts are earlier on the
            // comm stream, its lookaheads earlier on s_panel
            DCK(d, hipStreamWaitEvent(d->s_comm, d->ev_free_main[group_buf(d, s)], 0));
        }
        DCK(d, hipStreamWaitEvent(d->s_comm, d->ev_col[k], 0));
        launch_pack(d->s_comm, d->C + (int64_t)lc * NB * ldc + r0, ldc,
                    const_cast<double*>(chunk_panel(d, s, ch).P) + (int64_t)(k - chunk_col0(d, ch)) * NB * ldp +
                        (r0 - group_row0(d, s)),
                    ldp, d->Np - r0);
        if (k == w - 1 || (k + 1) % d->cw == 0) {  // the chunk's last column
            stamp(d, d->s_comm, st_pack(s, ch));
            DCK(d, hipEventRecord(d->ev_packed[s & 1][ch], d->s_comm));
        }
    }
    DCK(d, hipEventRecord(d->ev_panel_done, sp));
    d->factored_any = true;
    DCK(d, hipGetLastError());
    return guard.check();
}

int gaplac_dist_chunks(gaplac_dist* d, int32_t s, int32_t* out_chunks) {
    if (!d || s < 0 || s >= d->nsteps || !out_chunks) return derr(d, GAPLAC_E_ARG, "chunks: step %d out of range", s);
    *out_chunks = nchunks(d, s);
    return 0;
}

// Device buffer, element count and root rank of the broadcast of chunk c of panel s.
int gaplac_dist_panel_chunk(gaplac_dist* d, int32_t s, int32_t c, void** ptr, int64_t* count, int32_t* root) {
    if (!d || s < 0 || s >= d->nsteps || c < 0 || c >= nchunks(d, s))
        return derr(d, GAPLAC_E_ARG, "panel: step %d chunk %d out of range", s, c);
    if (ptr) *ptr = chunk_ptr(d, s, c);
    if (count) *count = chunk_count(d, s, c);
    if (root) *root = owner(d, s);
    return 0;
}

// The whole panel s as one broadcast (every chunk; gaplac_dist_comm_end then releases all).
int gaplac_dist_panel(gaplac_dist* d, int32_t s, void** ptr, int64_t* count, int32_t* root) {
    if (!d || s < 0 || s >= d->nsteps) return derr(d, GAPLAC_E_ARG, "panel: step %d out of range", s);
    if (ptr) *ptr = chunk_ptr(d, s, 0);
    if (count) *count = (int64_t)sp_width(d, s) * NB * group_ld(d, s) - (panel_row0(d, s) - group_row0(d, s));
    if (root) *root = owner(d, s);
    return 0;
}

// Make the comm stream ready for the broadcast of chunk c of panel s (root: the chunk is
// packed; others, at the panel's first chunk: the group buffer's previous group is no
// longer read) and return it as an opaque hipStream_t, on which the host enqueues the
// broadcast (ncclBroadcast / RCCL).
int gaplac_dist_comm_begin_chunk(gaplac_dist* d, int32_t s, int32_t c, void** stream) {
    if (!d || s < 0 || s >= d->nsteps || c < 0 || c >= nchunks(d, s))
        return derr(d, GAPLAC_E_ARG, "comm_begin: step %d chunk %d out of range", s, c);
    DCK(d, hipSetDevice(d->device));
    if (owns(d, s)) {
        DCK(d, hipStreamWaitEvent(d->s_comm, d->ev_packed[s & 1][c], 0));
    } else if (c == 0 && s % d->D == 0) {  // the buffer's previous group: its last bulk update and lookahead
        DCK(d, hipStreamWaitEvent(d->s_comm, d->ev_free_main[group_buf(d, s)], 0));
        DCK(d, hipStreamWaitEvent(d->s_comm, d->ev_free_panel[group_buf(d, s)], 0));
    }
    if (stream) *stream = d->s_comm;
    return 0;
}

int gaplac_dist_comm_begin(gaplac_dist* d, int32_t s, void** stream) {
    if (!d || s < 0 || s >= d->nsteps) return derr(d, GAPLAC_E_ARG, "comm_begin: step %d out of range", s);
    int rc = gaplac_dist_comm_begin_chunk(d, s, 0, stream);
    if (rc || !owns(d, s)) return rc;
    for (int c = 1; c < nchunks(d, s); ++c) DCK(d, hipStreamWaitEvent(d->s_comm, d->ev_packed[s & 1][c], 0));
    return 0;
}

// The broadcast of chunk c of panel s is enqueued on the comm stream: later readers wait for it.
int gaplac_dist_comm_end_chunk(gaplac_dist* d, int32_t s, int32_t c) {
    if (!d || s < 0 || s >= d->nsteps || c < 0 || c >= nchunks(d, s))
        return derr(d, GAPLAC_E_ARG, "comm_end: step %d chunk %d out of range", s, c);
    DCK(d, hipSetDevice(d->device));
    DCK(d, hipEventRecord(d->ev_recv[s & 1][c], d->s_comm));
    return 0;
}

int gaplac_dist_comm_end(gaplac_dist* d, int32_t s) {
    if (!d || s < 0 || s >= d->nsteps) return derr(d, GAPLAC_E_ARG, "comm_end: step %d out of range", s);
    for (int c = 0; c < nchunks(d, s); ++c) {
        int rc = gaplac_dist_comm_end_chunk(d, s, c);
        if (rc) return rc;
    }
    return 0;
}

// The ops [b, e) of step p's plan on s_main (chain_beside: this rank's chain runs beside
// them, so the large-launch kernel is not taken).
static int run_ops(gaplac_dist* d, int p, size_t b, size_t e, bool chain_beside) {
    // owned-SP ordinal of the first owned SP >= g (this rank owns one SP per round)
    auto ord_from = [&](int g) {
        const int u = g / d->nranks;  // SP of ordinal u: cmap.global(u W) / W, in round u
        return cmap(d).global(u * d->W) / d->W >= g ? u : u + 1;
    };
    auto launch = [&](const uint32_t* tiles, int cnt, const Panel& pn, int kd) -> int {
        if (cnt <= 0) return 0;
        BulkArgs ba{d->C, d->Np, pn, tiles, cnt, kd, 0, 0, cmap(d)};
        ba.max_r = d->nt - 1;    // list entries: global row block
        ba.max_c = d->nloc - 1;  //              and local tile column
        if (d->big_mode == 0) ba.big = 0;
        else if (d->big_mode == 1) ba.big = (!chain_beside && cnt >= d->big_min) ? 1 : 0;
        DistGuard guard(d);
        launch_bulk(d->s_main, ba, nullptr);
        return guard.check();
    };
    auto kdepth = [&](int pf, int pl) {
        int k = 0;
        for (int q = pf; q <= pl; ++q) k += sp_width(d, q) * NB;
        return k;
    };
    int rc;
    const std::vector<DOp>& ops = d->plan[(size_t)p];
    for (size_t i = b; i < e; ++i) {
        const DOp& op = ops[i];
        if (op.kind == OP_MARK) {
            stamp(d, d->s_main, st_band(p));
            DCK(d, hipEventRecord(d->ev_step[p & 1], d->s_main));
            continue;
        }
        const Panel pn = panel_of(d, op.pf);
        const int kd = kdepth(op.pf, op.pl);
        if (op.kind == OP_BAND) {
            if (op.g >= d->nsp || !owns(d, op.g)) continue;
            const size_t u = (size_t)(op.g / d->nranks);
            if ((rc = launch(d->tiles + d->band_off[u], d->band_cnt[u], pn, kd))) return rc;
        } else {
            const int u = ord_from(op.g);
            if (u >= (int)d->bulk_cnt.size()) continue;
            if ((rc = launch(d->tiles + d->bulk_off[(size_t)u], d->bulk_cnt[(size_t)u], pn, kd))) return rc;
        }
    }
    return 0;
}

// Step p's ops are all enqueued: its END stamp, and the group's last bulk reader (its last
// step, or the last step of all) releases the group buffer.
static int end_step(gaplac_dist* d, int p) {
    stamp(d, d->s_main, st_end(p));
    if (p % d->D == d->D - 1 || p + 1 >= d->nsteps)
        DCK(d, hipEventRecord(d->ev_free_main[group_buf(d, p)], d->s_main));
    return 0;
}

// Bulk trailing update of step s (s_main) following the step plan: SP s+2 first, then
// ev_step, then the rest (a deferring step: SP s+3's band; otherwise the suffix).
// alone (a rank's chain gets the GPU to itself): the owner of SP s+1 starts update(s)
// after factor(s+1), and the owner of SP s+2 holds the ops after update(s)'s mark back
// until update(s+1) (after factor(s+2)): the chain of SP s+2, which starts at that mark,
// then never shares the GPU with this rank's bulk updates.
int gaplac_dist_update(gaplac_dist* d, int32_t s) {
    if (!d || s < 0 || s >= d->nsteps) return derr(d, GAPLAC_E_ARG, "update: step %d out of range", s);
    DCK(d, hipSetDevice(d->device));
    const int last = nchunks(d, s) - 1;
    // the owner reads its own packed panel (its broadcast may still be running); the
    // others wait for the whole panel to arrive. Panels before s were waited for by the
    // updates before this one on the same stream.
    DCK(d, hipStreamWaitEvent(d->s_main, owns(d, s) ? d->ev_packed[s & 1][last] : d->ev_recv[s & 1][last], 0));
    const bool alone = d->alone && d->nranks > 1;
    const bool waits = alone && s + 1 < d->nsteps && owns(d, s + 1);
    if (waits) DCK(d, hipStreamWaitEvent(d->s_main, d->ev_panel_done, 0));  // factor(s+1), enqueued just before
    int rc;
    if (d->held_step >= 0) {  // update(s-1)'s ops after its mark (this rank's chain of SP s+1 is done)
        const int p = d->held_step;
        d->held_step = -1;
        if (p != s - 1) return derr(d, GAPLAC_E_ARG, "update: held ops of step %d at step %d", p, s);
        if ((rc = run_ops(d, p, d->held_from, d->plan[(size_t)p].size(), false)) || (rc = end_step(d, p))) return rc;
    }
    stamp(d, d->s_main, st_upd(s));
    if (d->stamps) DCK(d, hipEventRecord(d->ev_upd[s & 1], d->s_main));
    // this rank's chain runs beside the update when it owns SP s+1 and does not wait for it
    const bool chain_beside = s + 1 < d->nsteps && owns(d, s + 1) && !waits;
    const std::vector<DOp>& ops = d->plan[(size_t)s];
    size_t mark = 0;
    while (mark < ops.size() && ops[mark].kind != OP_MARK) ++mark;
    if ((rc = run_ops(d, s, 0, std::min(mark + 1, ops.size()), chain_beside))) return rc;
    // (not with D = 1: factor(s+2) packs panel s+2 into panel s's buffer slot, which the held
    // ops still read; with D >= 2 panel s+2 lands in the other group buffer or another slot)
    if (alone && d->D >= 2 && s + 2 < d->nsteps && owns(d, s + 2)) {
        d->held_step = s;
        d->held_from = mark + 1;
    } else {
        if ((rc = run_ops(d, s, mark + 1, ops.size(), chain_beside)) || (rc = end_step(d, s))) return rc;
    }
    DCK(d, hipGetLastError());
    return 0;
}

// Partial sums over this rank's columns: logdet part, quad part, and info (0 = every
// pivot of this rank's diagonal blocks was positive, else the 1-based first failing
// global column). Synchronises the rank's streams.
int gaplac_dist_finish(gaplac_dist* d, double* out_logdet, double* out_quad, int64_t* out_info) {
    if (!d) return GAPLAC_E_ARG;
    DCK(d, hipSetDevice(d->device));
    if (d->held_step >= 0) return derr(d, GAPLAC_E_ARG, "finish: step %d's update is incomplete", d->held_step);
    if (d->factored_any) DCK(d, hipStreamWaitEvent(d->s_main, d->ev_panel_done, 0));
    // the distributed SPs' columns come first in the storage (a gathered SP's columns were
    // factored by the root's tail, whose sums are in tres)
    int64_t ncols = 0;
    for (int s = 0; s < d->nsteps; ++s)
        if (owns(d, s)) ncols += sp_width(d, s);
    {
        DistGuard guard(d);
        launch_reduce(d->s_main, d->C, d->Np, d->N, ncols * NB, cmap(d), d->dres);
        int rc;
        if ((rc = guard.check())) return rc;
    }
    const bool troot = d->tstop >= 0 && d->rank == d->tail_root;
    if (troot && !d->tail_ended) return derr(d, GAPLAC_E_ARG, "finish: the tail gather was not completed (tail_end)");
    DCK(d, hipMemcpyAsync(d->hres, d->dres, offsetof(EvalResult, part), hipMemcpyDeviceToHost, d->s_main));
    if (troot) DCK(d, hipMemcpyAsync(d->htres, d->tres, offsetof(EvalResult, part), hipMemcpyDeviceToHost, d->s_main));
    DCK(d, hipStreamSynchronize(d->s_main));
    DCK(d, hipStreamSynchronize(d->s_panel));
    DCK(d, hipStreamSynchronize(d->s_comm));
    EvalResult r = *d->hres;
    if (troot) {
        const EvalResult& t = *d->htres;
        r.err |= t.err;
        r.logdet += t.logdet;
        r.quad += t.quad;
        if (t.info != ~0ull) r.info = std::min(r.info, t.info + (unsigned long long)d->tN0);  // global (j + 1)
    }
    if (r.err) return derr(d, GAPLAC_E_HIP, "in-kernel wait expired (code %u)", r.err);
    if (out_logdet) *out_logdet = r.logdet;
    if (out_quad) *out_quad = r.quad;
    if (out_info) *out_info = r.info == ~0ull ? 0 : (int64_t)r.info;
    return 0;
}

// ---- tail gather ----

// tail_cols > 0: the SPs in the last tail_cols tile columns are gathered onto rank root and
// factored there by the persistent tail; 0 = off. Before begin.
int gaplac_dist_set_tail(gaplac_dist* d, int32_t tail_cols, int32_t root) {
    if (!d) return GAPLAC_E_ARG;
    if (tail_cols < 0 || tail_cols > TAIL_TMAX || root < 0 || root >= d->nranks)
        return derr(d, GAPLAC_E_ARG, "set_tail: %d tile columns onto rank %d", tail_cols, root);
    d->tail_cols = tail_cols;
    d->tail_root = root;
    d->plan_stop = -1;
    return 0;
}

// For order N (before begin): gather segments (0: no gather), the doubles this rank's
// segment buffer needs, and the distributed steps begin will return.
int gaplac_dist_tail_geometry(gaplac_dist* d, int64_t N, int32_t* nseg, int64_t* buf_elems, int32_t* nsteps) {
    if (!d || N < 1) return derr(d, GAPLAC_E_ARG, "bad tail geometry query");
    int64_t Np;
    int32_t nt, nsp;
    gaplac_dist_geometry(d, N, &Np, &nt, &nsp, nullptr, nullptr);
    const TailGeom g = tail_geom(d, nt, nsp, Np);
    if (nseg) *nseg = g.stop < 0 ? 0 : nsp - g.stop;
    if (buf_elems) *buf_elems = g.elems;
    if (nsteps) *nsteps = g.stop < 0 ? nsp : g.stop;
    return 0;
}

// Optional caller-owned segment buffer (e.g. a tensor of the collective library's binding),
// >= buf_elems doubles; NULL returns to a library-owned one.
int gaplac_dist_set_tail_buffer(gaplac_dist* d, void* buf, int64_t capacity) {
    if (!d) return GAPLAC_E_ARG;
    DCK(d, hipSetDevice(d->device));
    if (!d->tseg_external && d->tseg) (void)hipFree(d->tseg);
    d->tseg = buf && capacity > 0 ? static_cast<double*>(buf) : nullptr;
    d->tseg_cap = d->tseg ? (size_t)capacity : 0;
    d->tseg_external = d->tseg != nullptr;
    return 0;
}

// Segment i of the current evaluation's gather (SP tstop + i): this rank's buffer for it
// (NULL when the rank neither sends nor receives it), doubles, and the sending rank.
int gaplac_dist_tail_segment(gaplac_dist* d, int32_t i, void** buf, int64_t* count, int32_t* src) {
    if (!d || d->tstop < 0 || i < 0 || i >= d->nsp - d->tstop)
        return derr(d, GAPLAC_E_ARG, "tail_segment %d: no such segment", i);
    const size_t k = (size_t)i;
    if (buf) *buf = d->tseg_cnt[k] ? d->tseg + d->tseg_off[k] : nullptr;
    if (count) *count = d->tseg_cnt[k] ? d->tseg_cnt[k] : 0;
    if (src) *src = owner(d, d->tstop + i);
    return 0;
}

// After the last step's update: this rank's segments are packed on the comm stream, which
// is returned; the host enqueues the gather there (sends of this rank's segments to the
// root, the root's receives: ncclSend / ncclRecv in one group). The root's own segments are
// packed in place and not sent.
int gaplac_dist_tail_begin(gaplac_dist* d, void** stream) {
    if (!d || d->tstop < 0) return derr(d, GAPLAC_E_ARG, "tail_begin: no tail gather in this evaluation");
    if (d->held_step >= 0) return derr(d, GAPLAC_E_ARG, "tail_begin: step %d's update is incomplete", d->held_step);
    DCK(d, hipSetDevice(d->device));
    d->tail_ended = false;
    DCK(d, hipEventRecord(d->ev_tail, d->s_main));
    DCK(d, hipStreamWaitEvent(d->s_comm, d->ev_tail, 0));
    for (int s = d->tstop; s < d->nsp; ++s) {
        if (!owns(d, s)) continue;
        const int i = s - d->tstop;
        const int64_t rows = tseg_rows(d->tNt, d->W, i);
        const int lc0 = sp_local(d, s);
        for (int k = 0; k < sp_width(d, s); ++k)
            launch_pack(d->s_comm, d->C + (int64_t)(lc0 + k) * NB * d->Np + panel_row0(d, s), d->Np,
                        d->tseg + d->tseg_off[(size_t)i] + (int64_t)k * NB * rows, rows, rows);
    }
    DCK(d, hipGetLastError());
    if (stream) *stream = d->s_comm;
    return 0;
}

// The gather is enqueued on the comm stream. The root unpacks the segments into the
// trailing matrix and factors it with the single-GPU persistent tail (tail_kernel) on
// s_main; its logdet / quad / first failing pivot join the root's partial sums in finish.
int gaplac_dist_tail_end(gaplac_dist* d) {
    if (!d || d->tstop < 0) return derr(d, GAPLAC_E_ARG, "tail_end: no tail gather in this evaluation");
    DCK(d, hipSetDevice(d->device));
    d->tail_ended = true;
    if (d->rank != d->tail_root) return 0;
    DCK(d, hipEventRecord(d->ev_tail, d->s_comm));
    DCK(d, hipStreamWaitEvent(d->s_main, d->ev_tail, 0));
    LaunchGuard g;
    g.base = d->tmat;
    g.elems = d->tNt * d->tNt;
    GuardScope scope(&g);
    hipStream_t sm = d->s_main;
    for (int s = d->tstop; s < d->nsp; ++s) {
        const int i = s - d->tstop;
        const int64_t rows = tseg_rows(d->tNt, d->W, i), r0 = (int64_t)i * d->W * NB;
        for (int k = 0; k < sp_width(d, s); ++k)
            launch_pack(sm, d->tseg + d->tseg_off[(size_t)i] + (int64_t)k * NB * rows, rows,
                        d->tmat + (r0 + (int64_t)k * NB) * d->tNt + r0, d->tNt, rows);
    }
    const int T = d->nt - d->tstop * d->W;
    const int64_t tN = d->N - d->tN0;
    launch_init_result(sm, d->tres);
    DCK(d, hipMemsetAsync(d->tctl, 0, sizeof(TailCtl), sm));
    TailArgs ta{d->tmat, d->tNt, tN, 0, T, d->tDinv, d->tres, d->tctl, d->ttasks, d->ttasks_n, nullptr};
    launch_tail(sm, ta, std::min(d->ncu, d->ttasks_n), nullptr);
    launch_reduce(sm, d->tmat, d->tNt, tN, (int64_t)T * NB, ColMap{1, 0, 1}, d->tres);
    if (d->stamps) stamp(d, sm, d->nsp * ST_PER_STEP + 2);
    DCK(d, hipGetLastError());
    if (g.violations) return derr(d, GAPLAC_E_ARG, "tail launch outside the trailing matrix: %s", g.first.c_str());
    return 0;
}

// Debug / parity: copy this rank's local storage (Np x nloc*NB, column-major) to host.
int gaplac_dist_local(gaplac_dist* d, double* out, int64_t ld) {
    if (!d || !out || ld < d->Np) return derr(d, GAPLAC_E_ARG, "local: bad output");
    DCK(d, hipSetDevice(d->device));
    DCK(d, hipStreamSynchronize(d->s_main));
    DCK(d, hipStreamSynchronize(d->s_panel));
    if (d->nloc > 0)
        DCK(d, hipMemcpy2D(out, (size_t)ld * 8, d->C, (size_t)d->Np * 8, (size_t)d->Np * 8, (size_t)d->nloc * NB,
                           hipMemcpyDeviceToHost));
    return 0;
}

// Host-only check of the step plan for nt tile columns (no HIP calls): every super-panel
// gets every earlier panel exactly once, in order, before its chain; returns 0 or
// GAPLAC_E_ARG with the first violation in msg. *out_ops: the plan's bulk launches per rank
// count (bands + suffixes), for tests.
int gaplac_dist_plan_check_tail(int32_t nt, int32_t spw, int32_t depth, int32_t pair_m, int32_t tail_cols,
                                int64_t* out_ops, char* msg, int64_t msglen) {
    if (nt < 1 || spw < 1 || spw > MAXC || depth < 1 || depth > 8 || tail_cols < 0 || tail_cols > TAIL_TMAX)
        return GAPLAC_E_ARG;
    const int nsp = (nt + spw - 1) / spw;
    const int ts = tail_stop_of(nt, spw, tail_cols);
    const int stop = ts < 0 ? nsp : ts;
    const auto plan = build_plan(nsp, nt, spw, depth, pair_m, stop);
    std::string why;
    const bool ok = check_plan(plan, nsp, depth, stop, &why);
    if (out_ops) {
        int64_t n = 0;
        for (const auto& ops : plan)
            for (const DOp& op : ops) n += op.kind != OP_MARK;
        *out_ops = n;
    }
    if (msg && msglen > 0) {
        std::snprintf(msg, (size_t)msglen, "%s", why.c_str());
    }
    return ok ? 0 : GAPLAC_E_ARG;
}

int gaplac_dist_plan_check(int32_t nt, int32_t spw, int32_t depth, int32_t pair_m, int64_t* out_ops, char* msg,
                           int64_t msglen) {
    return gaplac_dist_plan_check_tail(nt, spw, depth, pair_m, 0, out_ops, msg, msglen);
}

// The step plan itself (host-only): per op (step, kind, g, pf, pl) as 5 int32 into out
// (cap ints); *out_n = number of ops. kind: 0 band of SP g, 1 every SP >= g, 2 mark.
// tail_cols as gaplac_dist_set_tail's (the plan then has fewer steps than SPs).
int gaplac_dist_plan_tail(int32_t nt, int32_t spw, int32_t depth, int32_t pair_m, int32_t tail_cols, int32_t* out,
                          int64_t cap, int64_t* out_n) {
    if (nt < 1 || spw < 1 || spw > MAXC || depth < 1 || depth > 8 || !out_n || tail_cols < 0 || tail_cols > TAIL_TMAX)
        return GAPLAC_E_ARG;
    const int nsp = (nt + spw - 1) / spw;
    const int ts = tail_stop_of(nt, spw, tail_cols);
    const int stop = ts < 0 ? nsp : ts;
    const auto plan = build_plan(nsp, nt, spw, depth, pair_m, stop);
    int64_t n = 0;
    for (int p = 0; p < stop; ++p)
        for (const DOp& op : plan[(size_t)p]) {
            if (out && 5 * (n + 1) <= cap) {
                int32_t* o = out + 5 * n;
                o[0] = p;
                o[1] = op.kind;
                o[2] = op.g;
                o[3] = op.pf;
                o[4] = op.pl;
            }
            ++n;
        }
    *out_n = n;
    return 0;
}

int gaplac_dist_plan(int32_t nt, int32_t spw, int32_t depth, int32_t pair_m, int32_t* out, int64_t cap,
                     int64_t* out_n) {
    return gaplac_dist_plan_tail(nt, spw, depth, pair_m, 0, out, cap, out_n);
}

// ---- replay of one rank's schedule on one GPU (diagnostics) ----

// Turn the device timestamps on for the next evaluation of order N (allocate and zero
// them; N = 0: off), before gaplac_dist_begin; gaplac_dist_replay_stamps copies them out
// (ticks of 10 ns): nsp x ST_PER_STEP per-step stamps, then the end of the rank's Gram.
int gaplac_dist_replay_enable(gaplac_dist* d, int64_t N) {
    if (!d || N < 0) return GAPLAC_E_ARG;
    DCK(d, hipSetDevice(d->device));
    if (N == 0) {
        if (d->stamps) (void)hipFree(d->stamps);
        d->stamps = nullptr;
        d->stamps_elems = 0;
        return 0;
    }
    int32_t nsp = 0;
    gaplac_dist_geometry(d, N, nullptr, nullptr, &nsp, nullptr, nullptr);
    int rc;
    if ((rc = dgrow(d, &d->stamps, &d->stamps_elems, (size_t)nsp * ST_PER_STEP + ST_EXTRA))) return rc;
    DCK(d, hipMemsetAsync(d->stamps, 0, d->stamps_elems * 8, d->s_main));
    DCK(d, hipStreamSynchronize(d->s_main));
    return 0;
}

int gaplac_dist_replay_stamps(gaplac_dist* d, uint64_t* out, int64_t n) {
    if (!d || !d->stamps || !out || n < (int64_t)d->nsp * ST_PER_STEP + ST_EXTRA ||
        d->stamps_elems < (size_t)d->nsp * ST_PER_STEP + ST_EXTRA)
        return derr(d, GAPLAC_E_ARG, "stamps: bad output");
    DCK(d, hipSetDevice(d->device));
    DCK(d, hipMemcpy(out, d->stamps, ((size_t)d->nsp * ST_PER_STEP + ST_EXTRA) * 8, hipMemcpyDeviceToHost));
    return 0;
}

// Modelled transfer of chunk c of panel s on this rank's comm stream, in place of the
// broadcast. Arrival = max(owner ready + F, previous chunk's arrival) + transfer, where
//   owner ready = max(RECV(s-1, last), UPD(s-2) + band_ticks)    (the owner's chain inputs)
//   F = the owner's chain until the chunk is packed (f_ticks), transfer = lat + bytes / BW
// for a panel of another rank (src: the owner's context, factored: its columns are copied
// after the wait, and copy_ticks of that copy are taken off the wait), and
//   arrival = max(PACK(s, c) + lat, RECV(s, c-1)) + bytes / BW
// for this rank's own panel (its send). Then comm_end_chunk(s, c).
int gaplac_dist_replay_chunk(gaplac_dist* d, const gaplac_dist* src, int32_t s, int32_t c, int64_t f_ticks,
                             int64_t band_ticks, int64_t lat_ticks, int64_t xfer_ticks, int64_t copy_ticks) {
    if (!d || !d->stamps || s < 0 || s >= d->nsteps || c < 0 || c >= nchunks(d, s))
        return derr(d, GAPLAC_E_ARG, "replay: step %d chunk %d (stamps %s)", s, c, d && d->stamps ? "on" : "off");
    void* st = nullptr;
    int rc;
    if ((rc = gaplac_dist_comm_begin_chunk(d, s, c, &st))) return rc;
    Release r{{-1, -1, -1}, {0, 0, 0}, st_recv(s, c)};
    if (owns(d, s)) {
        r.dep[0] = st_pack(s, c);
        r.add[0] = lat_ticks + xfer_ticks;
        if (c > 0) {
            r.dep[1] = st_recv(s, c - 1);
            r.add[1] = xfer_ticks;
        }
    } else {
        if (!src || src->Np != d->Np || src->W != d->W || src->nranks != d->nranks || src->rank != owner(d, s) ||
            src->snake != d->snake)
            return derr(d, GAPLAC_E_ARG, "replay: source context is not the owner of panel %d", s);
        const long long wait = f_ticks + lat_ticks + xfer_ticks - copy_ticks;
        if (s == 0) {  // the owner's chain starts after its Gram (taken as long as this rank's)
            DCK(d, hipStreamWaitEvent(d->s_comm, d->ev_gram, 0));
            r.dep[0] = -2;
            r.add[0] = wait;
        } else {
            r.dep[0] = st_recv(s - 1, nchunks(d, s - 1) - 1);
            r.add[0] = wait;
        }
        if (s >= 2) {
            DCK(d, hipStreamWaitEvent(d->s_comm, d->ev_upd[s & 1], 0));  // update(s-2) started
            r.dep[1] = st_upd(s - 2);
            r.add[1] = band_ticks + wait;
        }
        if (c > 0) {
            r.dep[2] = st_recv(s, c - 1);
            r.add[2] = xfer_ticks - copy_ticks;
        }
    }
    if (guard_launch("release_kernel")) release_kernel<<<dim3(1), dim3(64), 0, d->s_comm>>>(d->stamps, r);
    if (!owns(d, s)) {
        const int lc0 = sp_local(src, s) + chunk_col0(d, c), ncol = chunk_cols(d, s, c);
        const int64_t r0 = panel_row0(d, s);
        double* dst = const_cast<double*>(chunk_panel(d, s, c).P) + (r0 - group_row0(d, s));
        DCK(d, hipMemcpy2DAsync(dst, (size_t)group_ld(d, s) * 8, src->C + (int64_t)lc0 * NB * src->Np + r0,
                                (size_t)src->Np * 8, (size_t)(d->Np - r0) * 8, (size_t)ncol * NB,
                                hipMemcpyDeviceToDevice, d->s_comm));
        stamp(d, d->s_comm, st_pack(s, c));  // a non-owner's PACK slot: the copy's end
    }
    return gaplac_dist_comm_end_chunk(d, s, c);
}

// Modelled tail gather on the replayed rank, in place of the host's sends / receives
// (between tail_begin and tail_end, which this calls). Every sender's segments leave when
// its last update is done, over its own link: the root's receives arrive at
//   max(END(last step), Gram end + senders_end) + lat + max over senders of (bytes) x ticks_per_byte
// where senders_end is the latest sender's last update end, from that rank's own replay,
// relative to its Gram end (0: taken as this rank's own END), as copies from the owners'
// segment buffers (owners[q]: rank q's context of a loopback run with the same gather;
// copy_ticks of the copies are taken off the wait). A sender's own sends end at
// END(last step) + lat + its bytes x ticks_per_byte (stamped only).
int gaplac_dist_replay_tail(gaplac_dist* d, const gaplac_dist* const* owners, int32_t nowners, int64_t lat_ticks,
                            double ticks_per_byte, int64_t copy_ticks, int64_t senders_end) {
    if (!d || !d->stamps || d->tstop < 0 || !owners || nowners != d->nranks)
        return derr(d, GAPLAC_E_ARG, "replay_tail: needs stamps, a gather and every rank's context");
    void* st = nullptr;
    int rc;
    if ((rc = gaplac_dist_tail_begin(d, &st))) return rc;
    const bool root = d->rank == d->tail_root;
    std::vector<int64_t> bytes((size_t)d->nranks, 0);
    for (int i = 0; i < d->nsp - d->tstop; ++i) {
        const int src = owner(d, d->tstop + i);
        const int64_t c = (int64_t)sp_width(d, d->tstop + i) * NB * tseg_rows(d->tNt, d->W, i) * 8;
        if (src != d->tail_root) bytes[(size_t)src] += c;
    }
    const int64_t sent = root ? *std::max_element(bytes.begin(), bytes.end()) : bytes[(size_t)d->rank];
    const long long xfer = lat_ticks + (long long)(sent * ticks_per_byte) - (root ? copy_ticks : 0);
    Release r{{st_end(d->nsteps - 1), root && senders_end > 0 ? d->nsp * ST_PER_STEP : -1, -1},
              {xfer, senders_end + xfer, 0}, d->nsp * ST_PER_STEP + 1};
    if (guard_launch("release_kernel")) release_kernel<<<dim3(1), dim3(64), 0, d->s_comm>>>(d->stamps, r);
    if (root) {
        for (int i = 0; i < d->nsp - d->tstop; ++i) {
            const int src = owner(d, d->tstop + i);
            if (src == d->tail_root) continue;
            const gaplac_dist* o = owners[src];
            if (!o || o->rank != src || o->tstop != d->tstop || o->tNt != d->tNt || !o->tseg ||
                o->tseg_cnt[(size_t)i] != d->tseg_cnt[(size_t)i])
                return derr(d, GAPLAC_E_ARG, "replay_tail: rank %d's context has no segment %d", src, i);
            DCK(d, hipMemcpyAsync(d->tseg + d->tseg_off[(size_t)i], o->tseg + o->tseg_off[(size_t)i],
                                  (size_t)d->tseg_cnt[(size_t)i] * 8, hipMemcpyDeviceToDevice, d->s_comm));
        }
        stamp(d, d->s_comm, d->nsp * ST_PER_STEP + 3);
    }
    return gaplac_dist_tail_end(d);
}

// Bytes of chunk c of panel s that a broadcast must move (rows from the panel's first
// row; the replay's transfer model) and the per-step stamp layout.
int gaplac_dist_replay_info(gaplac_dist* d, int32_t s, int32_t c, int64_t* bytes, int32_t* per_step,
                            int32_t* maxc) {
    if (!d || s < 0 || s >= d->nsp || c < 0 || c >= nchunks(d, s)) return derr(d, GAPLAC_E_ARG, "replay_info");
    if (bytes) *bytes = chunk_bytes_useful(d, s, c);
    if (per_step) *per_step = ST_PER_STEP;
    if (maxc) *maxc = MAXC;
    return 0;
}

}  // extern "C"
