// Distributed evaluation (BASELINE configs[3]): one rank of a 1-D
// block-column cyclic Cholesky of the (N+1)-augmented covariance.
//
// Distribution. Super-panels (SP) of W 128-wide tile columns are dealt round-robin: SP s
// belongs to rank s % nranks. A rank stores only its own tile columns (all Np rows,
// column-major, ldc = Np), in order (ColMap in gaplac_internal.h). Because the Gram is
// symmetric, a rank's block columns of the lower triangle are the block rows of the upper:
// each rank builds exactly the Gram tiles it owns, with no redistribution.
//
// Steps (the host drives them; the only exchange is the panel broadcast):
//   begin          all ranks: local Gram tiles (s_main)
//   factor(s)      owner of SP s (s_panel, critical path): apply panel s-1 to SP s
//                  (lookahead), factor SP s column by column (column updates inside
//                  the SP, diagonal potrf, panel TRSM), pack rows >= first row of SP s
//                  into panel buffer s&1
//   bcast(s)       the host broadcasts panel buffer s&1 from the owner (RCCL on the
//                  comm stream, gaplac_dist_comm_begin/_end bracket it)
//   update(s)      all ranks: bulk trailing update of their SPs > s+1 with panel s
//                  (s_main); SP s+1 gets panel s in factor(s+1) instead. Paired updates
//                  (the single-GPU schedule's): an even step s whose
//                  trailing matrix still has >= pair_m tile rows after SP s+3 updates only
//                  SPs s+2 and s+3 (the next chain needs them); step s+1 then updates SP
//                  s+3 with panel s+1 and every SP >= s+4 with panels s and s+1 at once
//                  (K = 2 x 128 W: half the launches, twice the depth)
//   finish         all ranks: partial logdet / quad / info over their columns; the host
//                  sums them across ranks (one allreduce of 3 numbers)
// The host calls, per rank: begin; factor(0) [owner]; bcast(0); for s = 0..nsp-1:
// { factor(s+1) [owner of s+1]; update(s); bcast(s+1) }; finish. Every call only
// enqueues work: the streams overlap the bulk update with the next panel's chain.
// Panel buffers: two PAIR buffers; panels s and s+1 (s even) share pair buffer (s/2) & 1
// with the rows of panel s as the common origin (ld = Np - first row of SP s; the odd
// panel's columns start 128 W rows down), so a paired update reads both as one K = 256 W
// panel. Events keep a pair buffer from being re-filled (packed by its owner or received)
// before the updates and lookaheads that read its previous pair have run.
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

struct gaplac_dist {
    int device = 0, nranks = 1, rank = 0, W = 4;
    hipStream_t s_main = nullptr, s_panel = nullptr, s_comm = nullptr;
    hipEvent_t ev_gram = nullptr, ev_panel_done = nullptr;
    // ev_recv / ev_packed per panel parity; ev_step[s & 1]: update(s) done (the last bulk
    // update of SP s+2's columns); ev_free_main / ev_free_panel per pair buffer: its last
    // bulk update / lookahead reader done
    hipEvent_t ev_recv[2] = {}, ev_packed[2] = {}, ev_step[2] = {}, ev_free_main[2] = {}, ev_free_panel[2] = {};
    int pair_m = 40;  // GAPLAC_PAIR_M: paired updates while >= pair_m tile rows follow SP s+3
    // geometry of the current evaluation
    int64_t N = -1, Np = 0;
    int nt = 0, nsp = 0, nloc = 0;
    bool factored_any = false;
    // device buffers
    double* C = nullptr;
    size_t C_elems = 0;
    double* Dinv = nullptr;
    size_t Dinv_elems = 0;
    double* pbuf[2] = {};
    size_t pbuf_cap = 0;   // elements per (pair) buffer
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

ColMap cmap(const gaplac_dist* d) { return ColMap{d->nranks, d->rank, d->W}; }
int sp_first(const gaplac_dist* d, int s) { return s * d->W; }
int sp_width(const gaplac_dist* d, int s) { return std::min(d->W, d->nt - s * d->W); }
int sp_local(const gaplac_dist* d, int s) { return (s / d->nranks) * d->W; }  // first local column
bool owns(const gaplac_dist* d, int s) { return s % d->nranks == d->rank; }
int64_t panel_row0(const gaplac_dist* d, int s) { return (int64_t)sp_first(d, s) * NB; }
// pair buffer of panel s: (s / 2) & 1; its origin row is that of the pair's even panel
int pair_buf(int s) { return (s >> 1) & 1; }
int64_t pair_row0(const gaplac_dist* d, int s) { return panel_row0(d, s & ~1); }
int64_t pair_ld(const gaplac_dist* d, int s) { return d->Np - pair_row0(d, s); }
// first element of panel s (its row panel_row0(s), column 0) in its pair buffer
double* panel_ptr(const gaplac_dist* d, int s) {
    return d->pbuf[pair_buf(s)] + (int64_t)(s & 1) * d->W * NB * pair_ld(d, s) + (panel_row0(d, s) - pair_row0(d, s));
}
Panel panel_of(const gaplac_dist* d, int s) {
    return Panel{d->pbuf[pair_buf(s)] + (int64_t)(s & 1) * d->W * NB * pair_ld(d, s), pair_ld(d, s), pair_row0(d, s)};
}
// does step s defer (paired updates)? Even steps only: panels s and s+1 share a buffer.
bool pair_step(const gaplac_dist* d, int s) {
    return d->pair_m > 0 && (s & 1) == 0 && s + 4 <= d->nsp && d->nt - (s + 4) * d->W >= d->pair_m;
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

}  // namespace

extern "C" {

const char* gaplac_dist_last_error(const gaplac_dist* d) { return d ? d->err.c_str() : "null context"; }

int gaplac_dist_create(int device, int nranks, int rank, int spw, gaplac_dist** out) {
    if (!out) return GAPLAC_E_ARG;
    *out = nullptr;
    if (nranks < 1 || rank < 0 || rank >= nranks || spw < 1 || spw > 8) return GAPLAC_E_ARG;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || device < 0 || device >= n) return GAPLAC_E_NODEVICE;
    gaplac_dist* d = new gaplac_dist();
    d->device = device;
    d->nranks = nranks;
    d->rank = rank;
    d->W = spw;
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
    hipEvent_t* evs[] = {&d->ev_gram, &d->ev_panel_done, &d->ev_recv[0], &d->ev_recv[1], &d->ev_packed[0],
                         &d->ev_packed[1], &d->ev_step[0], &d->ev_step[1], &d->ev_free_main[0],
                         &d->ev_free_main[1], &d->ev_free_panel[0], &d->ev_free_panel[1]};
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
    *out = d;
    return 0;
}

int gaplac_dist_destroy(gaplac_dist* d) {
    if (!d) return 0;
    (void)hipSetDevice(d->device);
    for (hipStream_t s : {d->s_main, d->s_panel, d->s_comm})
        if (s) (void)hipStreamSynchronize(s);
    hipEvent_t evs[] = {d->ev_gram, d->ev_panel_done, d->ev_recv[0], d->ev_recv[1], d->ev_packed[0],
                        d->ev_packed[1], d->ev_step[0], d->ev_step[1], d->ev_free_main[0],
                        d->ev_free_main[1], d->ev_free_panel[0], d->ev_free_panel[1]};
    for (hipEvent_t ev : evs)
        if (ev) (void)hipEventDestroy(ev);
    for (void* p : {(void*)d->C, (void*)d->Dinv, (void*)d->tiles, (void*)d->dX, (void*)d->dv, (void*)d->dres,
                    (void*)d->dtp})
        if (p) (void)hipFree(p);
    if (!d->pbuf_external)
        for (double* p : d->pbuf)
            if (p) (void)hipFree(p);
    if (d->hres) (void)hipHostFree(d->hres);
    if (d->htp) (void)hipHostFree(d->htp);
    for (hipStream_t s : {d->s_main, d->s_panel, d->s_comm})
        if (s) (void)hipStreamDestroy(s);
    delete d;
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
// columns, and the doubles one (pair) panel buffer needs (the pair of SPs 0 and 1).
int gaplac_dist_geometry(gaplac_dist* d, int64_t N, int64_t* Np, int32_t* nt, int32_t* nsp, int32_t* nloc,
                         int64_t* panel_elems) {
    if (!d || N < 1) return derr(d, GAPLAC_E_ARG, "bad geometry query");
    const int64_t np = (N + 1 + NB - 1) / NB * NB;
    const int t = (int)(np / NB);
    const int ns = (t + d->W - 1) / d->W;
    int nl = 0;
    for (int s = d->rank; s < ns; s += d->nranks) nl += std::min(d->W, t - s * d->W);
    if (Np) *Np = np;
    if (nt) *nt = t;
    if (nsp) *nsp = ns;
    if (nloc) *nloc = nl;
    if (panel_elems) *panel_elems = np * (int64_t)std::min(2 * d->W, t) * NB;
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
    DCK(d, hipEventRecord(d->ev_gram, d->s_main));
    DCK(d, hipStreamWaitEvent(d->s_panel, d->ev_gram, 0));
    DCK(d, hipGetLastError());
    if (out_nsp) *out_nsp = nsp;
    return 0;
}

// Owner of SP s only. Lookahead update with panel s-1, then the SP's panel chain, then
// the pack into panel buffer s&1 (all on s_panel).
int gaplac_dist_factor(gaplac_dist* d, int32_t s) {
    if (!d || s < 0 || s >= d->nsp) return derr(d, GAPLAC_E_ARG, "factor: step %d out of range", s);
    if (!owns(d, s)) return derr(d, GAPLAC_E_ARG, "factor: rank %d does not own super-panel %d", d->rank, s);
    DCK(d, hipSetDevice(d->device));
    DistGuard guard(d);
    hipStream_t sp = d->s_panel;
    const int c0 = sp_first(d, s), w = sp_width(d, s), lc0 = sp_local(d, s);
    const int64_t ldc = d->Np;
    // update(s-2) (s_main) was the last bulk update of SP s's columns (a paired update at
    // an odd step covers SPs >= step + 3, a deferring step's bands SPs step + 2, step + 3),
    // and the pack below overwrites pair buffer pair_buf(s): its previous pair's last bulk
    // update ran before (ev_free_main; its lookahead readers are earlier on this stream)
    DCK(d, hipStreamWaitEvent(sp, d->ev_step[s & 1], 0));
    DCK(d, hipStreamWaitEvent(sp, d->ev_free_main[pair_buf(s)], 0));
    if (s > 0) {
        DCK(d, hipStreamWaitEvent(sp, d->ev_recv[(s - 1) & 1], 0));
        launch_col_update(sp, d->C, ldc, panel_of(d, s - 1), d->nt, c0, lc0, w, sp_width(d, s - 1) * NB, nullptr);
        // this rank's latest lookahead reading the pair buffer (the receive of the buffer's
        // next pair waits for it on the comm stream)
        DCK(d, hipEventRecord(d->ev_free_panel[pair_buf(s - 1)], sp));
    }
    for (int c = c0; c < c0 + w; ++c) {
        const int lc = lc0 + (c - c0);
        double* Acol = d->C + (int64_t)lc * NB * ldc;
        if (c > c0)
            launch_col_update(sp, d->C, ldc, Panel{Acol - NB * ldc, ldc, 0}, d->nt, c, lc, c0 + w - c, NB, nullptr);
        double* Dk = d->Dinv + (size_t)lc * DINV_PER_BLOCK;
        if ((int64_t)c * NB < d->N)
            launch_potrf_diag(sp, Acol + (int64_t)c * NB, ldc, d->N, (int64_t)c * NB, Dk, d->dres, nullptr);
        launch_trsm(sp, Acol, ldc, d->nt, c, Dk, nullptr);
    }
    const int64_t r0 = panel_row0(d, s), ldp = pair_ld(d, s);
    DCK(d, hipMemcpy2DAsync(panel_ptr(d, s), (size_t)ldp * 8, d->C + (int64_t)lc0 * NB * ldc + r0, (size_t)ldc * 8,
                            (size_t)(d->Np - r0) * 8, (size_t)w * NB, hipMemcpyDeviceToDevice, sp));
    DCK(d, hipEventRecord(d->ev_packed[s & 1], sp));
    DCK(d, hipEventRecord(d->ev_panel_done, sp));
    d->factored_any = true;
    DCK(d, hipGetLastError());
    return guard.check();
}

// Device buffer, element count and root rank of the broadcast of panel s.
int gaplac_dist_panel(gaplac_dist* d, int32_t s, void** ptr, int64_t* count, int32_t* root) {
    if (!d || s < 0 || s >= d->nsp) return derr(d, GAPLAC_E_ARG, "panel: step %d out of range", s);
    // the panel's columns in its pair buffer, from its first row to the end of its last
    // column (an odd panel's column gaps above its first row go along: 128 W rows each)
    if (ptr) *ptr = panel_ptr(d, s);
    if (count) *count = (int64_t)sp_width(d, s) * NB * pair_ld(d, s) - (panel_row0(d, s) - pair_row0(d, s));
    if (root) *root = s % d->nranks;
    return 0;
}

// Make the comm stream ready for the broadcast of panel s (root: the panel is packed;
// others: the buffer's previous contents are no longer read) and return it as an opaque
// hipStream_t, on which the host enqueues the broadcast (ncclBroadcast / RCCL).
int gaplac_dist_comm_begin(gaplac_dist* d, int32_t s, void** stream) {
    if (!d || s < 0 || s >= d->nsp) return derr(d, GAPLAC_E_ARG, "comm_begin: step %d out of range", s);
    DCK(d, hipSetDevice(d->device));
    if (owns(d, s)) {
        DCK(d, hipStreamWaitEvent(d->s_comm, d->ev_packed[s & 1], 0));
    } else {  // the pair buffer's previous pair: its last bulk update and last lookahead
        DCK(d, hipStreamWaitEvent(d->s_comm, d->ev_free_main[pair_buf(s)], 0));
        DCK(d, hipStreamWaitEvent(d->s_comm, d->ev_free_panel[pair_buf(s)], 0));
    }
    if (stream) *stream = d->s_comm;
    return 0;
}

// The broadcast of panel s is enqueued on the comm stream: later readers wait for it.
int gaplac_dist_comm_end(gaplac_dist* d, int32_t s) {
    if (!d || s < 0 || s >= d->nsp) return derr(d, GAPLAC_E_ARG, "comm_end: step %d out of range", s);
    DCK(d, hipSetDevice(d->device));
    DCK(d, hipEventRecord(d->ev_recv[s & 1], d->s_comm));
    return 0;
}

// Bulk trailing update with panel s of this rank's SPs > s+1 (s_main), or with paired
// updates (pair_step): a deferring step s updates SPs s+2, s+3 only; step s+1 updates SP
// s+3 with panel s+1 and the SPs >= s+4 with panels s, s+1 (one K = 256 W launch).
int gaplac_dist_update(gaplac_dist* d, int32_t s) {
    if (!d || s < 0 || s >= d->nsp) return derr(d, GAPLAC_E_ARG, "update: step %d out of range", s);
    DCK(d, hipSetDevice(d->device));
    DCK(d, hipStreamWaitEvent(d->s_main, d->ev_recv[s & 1], 0));
    const bool defer = pair_step(d, s), paired = s >= 1 && pair_step(d, s - 1);
    // owned-SP ordinal of the first owned SP >= g
    auto ord_from = [&](int g) {
        const int rel = g - d->rank;
        return rel <= 0 ? 0 : (rel + d->nranks - 1) / d->nranks;
    };
    auto launch = [&](const uint32_t* tiles, int cnt, const Panel& pn, int kd) -> int {
        if (cnt <= 0) return 0;
        BulkArgs ba{d->C, d->Np, pn, tiles, cnt, kd, 0, 0, cmap(d)};
        ba.max_r = d->nt - 1;    // list entries: global row block
        ba.max_c = d->nloc - 1;  //              and local tile column
        DistGuard guard(d);
        launch_bulk(d->s_main, ba, nullptr);
        return guard.check();
    };
    auto band = [&](int g, const Panel& pn, int kd) -> int {  // SP g alone, if owned
        if (g >= d->nsp || !owns(d, g)) return 0;
        const size_t u = (size_t)(g / d->nranks);
        return launch(d->tiles + d->band_off[u], d->band_cnt[u], pn, kd);
    };
    auto suffix = [&](int g, const Panel& pn, int kd) -> int {  // owned SPs >= g
        const int u = ord_from(g);
        if (u >= (int)d->bulk_cnt.size()) return 0;
        return launch(d->tiles + d->bulk_off[(size_t)u], d->bulk_cnt[(size_t)u], pn, kd);
    };
    const int kd = sp_width(d, s) * NB;
    int rc;
    if (defer) {
        if ((rc = band(s + 2, panel_of(d, s), kd)) || (rc = band(s + 3, panel_of(d, s), kd))) return rc;
    } else if (paired) {
        DCK(d, hipStreamWaitEvent(d->s_main, d->ev_recv[(s - 1) & 1], 0));
        if ((rc = band(s + 2, panel_of(d, s), kd))) return rc;
        if ((rc = suffix(s + 3, panel_of(d, s - 1), sp_width(d, s - 1) * NB + kd))) return rc;
    } else {
        if ((rc = suffix(s + 2, panel_of(d, s), kd))) return rc;
    }
    DCK(d, hipEventRecord(d->ev_step[s & 1], d->s_main));
    // the pair's last bulk reader: its odd step (or an even step with no odd partner)
    if ((s & 1) || s + 1 >= d->nsp) DCK(d, hipEventRecord(d->ev_free_main[pair_buf(s)], d->s_main));
    DCK(d, hipGetLastError());
    return 0;
}

// Partial sums over this rank's columns: logdet part, quad part, and info (0 = every
// pivot of this rank's diagonal blocks was positive, else the 1-based first failing
// global column). Synchronises the rank's streams.
int gaplac_dist_finish(gaplac_dist* d, double* out_logdet, double* out_quad, int64_t* out_info) {
    if (!d) return GAPLAC_E_ARG;
    DCK(d, hipSetDevice(d->device));
    if (d->factored_any) DCK(d, hipStreamWaitEvent(d->s_main, d->ev_panel_done, 0));
    {
        DistGuard guard(d);
        launch_reduce(d->s_main, d->C, d->Np, d->N, (int64_t)d->nloc * NB, cmap(d), d->dres);
        int rc;
        if ((rc = guard.check())) return rc;
    }
    DCK(d, hipMemcpyAsync(d->hres, d->dres, offsetof(EvalResult, part), hipMemcpyDeviceToHost, d->s_main));
    DCK(d, hipStreamSynchronize(d->s_main));
    DCK(d, hipStreamSynchronize(d->s_panel));
    DCK(d, hipStreamSynchronize(d->s_comm));
    const EvalResult r = *d->hres;
    if (r.err) return derr(d, GAPLAC_E_HIP, "in-kernel wait expired (code %u)", r.err);
    if (out_logdet) *out_logdet = r.logdet;
    if (out_quad) *out_quad = r.quad;
    if (out_info) *out_info = r.info == ~0ull ? 0 : (int64_t)r.info;
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

}  // extern "C"
