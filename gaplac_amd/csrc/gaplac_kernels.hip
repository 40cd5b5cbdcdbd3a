// HIP kernels for GaPLAC's log-marginal-likelihood path on MI355X (gfx950, CDNA4).
//
// Data layout: one Np x Np fp64 column-major matrix A in HBM, Np =
// roundup(N+1, NB). Rows/cols 0..N-1 hold C = sum_t K_t + noise*I (lower triangle only),
// row N holds v^T, everything else is zero padding. A lower Cholesky factorisation of
// that augmented matrix leaves L = U^T (U = LAPACK dpotrf('U') of C) in rows/cols < N
// and z = L^{-1} v = U^{-T} v in row N, so the triangular solve of AbstractGPs.logpdf
// (sum(abs2, U' \ v)) falls out of the factorisation with no separate trsv pass.
//
// Kernels:
//   gram_kernel        Gram build, one 128x128 lower tile per workgroup (HBM-write bound)
//   potrf_diag_kernel  128x128 diagonal block Cholesky + its triangular inverse (registers)
//   trsm_subst_kernel  panel TRSM by blocked substitution on fp64 MFMA
//   tile_syrk_kernel   bulk trailing update C -= P Q^T, fp64 MFMA (v_mfma_f64_16x16x4f64)
//                      on 128x128 tiles; quad_bulk_kernel / col_update_kernel: the same
//                      on 64x64 quadrants (small updates, critical-path column updates)
//   reduce_*_kernel    logdet = 2 sum log L_jj, quad = ||z||^2, logpdf
#include "gaplac_internal.h"
#include <math.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

namespace gaplac {

typedef double d4 __attribute__((ext_vector_type(4)));

// Per-launch device timestamps (profiling only; kt == nullptr in production): first
// workgroup start / last wave end on the 100 MHz s_memrealtime clock. HIP timing events
// recorded inside a captured graph do not report elapsed times on ROCm 7.2, so the
// per-kernel breakdown of a graph replay is measured in the kernels themselves.
// Diagnostic build only (-DGAPLAC_STAMPS, tools/diag_probe.hip): phase stamps of the
// diagonal kernel into a debug array; never compiled into the library.
#ifdef GAPLAC_STAMPS
__device__ unsigned long long g_stamps[128];
#define STAMPT(th, i)                                                                   \
    do {                                                                                \
        __builtin_amdgcn_sched_barrier(0);                                              \
        if (threadIdx.x == (th)) g_stamps[i] = __builtin_amdgcn_s_memtime();            \
        __builtin_amdgcn_sched_barrier(0);                                              \
    } while (0)
#else
#define STAMPT(th, i) \
    do {              \
    } while (0)
#endif
#define STAMP(i) STAMPT(0, i)

__device__ __forceinline__ void kt_begin(KTime* kt) {
    if (kt && threadIdx.x == 0) atomicMin(&kt->start, (unsigned long long)__builtin_amdgcn_s_memrealtime());
}
__device__ __forceinline__ void kt_end(KTime* kt) {
    if (kt && (threadIdx.x & 63) == 0) atomicMax(&kt->end, (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

// Row-major triangular tile index: t = bi*(bi+1)/2 + bj, 0 <= bj <= bi.
__device__ __forceinline__ void tri_index(int64_t t, int& bi, int& bj) {
    int b = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while ((int64_t)(b + 1) * (b + 2) / 2 <= t) ++b;
    while ((int64_t)b * (b + 1) / 2 > t) --b;
    bi = b;
    bj = (int)(t - (int64_t)b * (b + 1) / 2);
}

// ---------------------------------------------------------------------------------
// Gram build. Semantics of each term follow KernelFunctions 0.10.38 as GaPLAC builds it
// (src/abstractgp_translations.jl:8-15): SqExponentialKernel / ExponentialKernel under
// ScaleTransform(1/l) (the coordinate is scaled first, then differenced), LinearKernel(c),
// CategoricalKernel (src/gp_parts.jl:11-13: distance > 0 -> 0 else 1). Groups multiply
// their terms, groups add in order (KernelSum = left fold of the term matrices), then
// noise is added on the diagonal (FiniteGP's Diagonal(Fill(noise, N))).
//
// Workgroup = one 128x128 lower tile, 256 threads. Each lane owns two consecutive rows
// (16-byte stores, a wave writes one 1 KiB column segment per instruction); the tile's
// column coordinates are staged once in LDS and read as wave-wide broadcasts.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ void gram_tile(double* __restrict__ Ccol, int64_t lda, int64_t N,
                                          const double* __restrict__ X, int64_t ldx,
                                          const double* __restrict__ v,
                                          const TermPack* __restrict__ tpp, int bi, int bj) {
    // Ccol: storage of global column bj*NB (row 0); rows are global
    // No FMA contraction: KernelFunctions scales each coordinate (rounded) and then
    // differences, so equal coordinates give exactly 0 (p*xa - p*xj fused would not).
#pragma clang fp contract(off)
    const TermPack& tp = *tpp;  // uniform: scalar loads (device copy refreshed per eval)
    const double noise = tp.noise;
    const int64_t r0 = (int64_t)bi * NB, c0 = (int64_t)bj * NB;
    __shared__ double xcol[GAPLAC_MAX_TERMS][NB];
    __shared__ double vcol[NB];
    const int tid = threadIdx.x;
    const int T = tp.T;
    for (int idx = tid; idx < T * NB; idx += 256) {
        const int t = idx / NB, c = idx % NB;
        const int64_t j = c0 + c;
        double val = 0.0;
        if (j < N && tp.kind[t] != GAPLAC_NOISE) val = X[(int64_t)tp.col[t] * ldx + j];
        xcol[t][c] = val;
    }
    if (tid < NB) {
        const int64_t j = c0 + tid;
        vcol[tid] = (j < N) ? v[j] : 0.0;
    }
    const int lane = tid & 63, w = tid >> 6;
    const int64_t i0 = r0 + 2 * lane, i1 = i0 + 1;
    double xa[GAPLAC_MAX_TERMS], xb[GAPLAC_MAX_TERMS];
#pragma unroll
    for (int t = 0; t < GAPLAC_MAX_TERMS; ++t) {
        xa[t] = 0.0;
        xb[t] = 0.0;
        if (t < T && tp.kind[t] != GAPLAC_NOISE) {
            const double* xc = X + (int64_t)tp.col[t] * ldx;
            if (i0 < N) xa[t] = xc[i0];
            if (i1 < N) xb[t] = xc[i1];
        }
    }
    __syncthreads();

    for (int cc = w; cc < NB; cc += 4) {
        const int64_t j = c0 + cc;
        double tot0 = 0.0, tot1 = 0.0, pr0 = 1.0, pr1 = 1.0;
#pragma unroll
        for (int t = 0; t < GAPLAC_MAX_TERMS; ++t) {
            if (t < T) {
                const double xj = xcol[t][cc];
                const double p = tp.p[t];
                double k0, k1;
                switch (tp.kind[t]) {
                    case GAPLAC_SQEXP: {
                        const double sj = p * xj;
                        const double d0 = p * xa[t] - sj, d1 = p * xb[t] - sj;
                        k0 = exp(-(d0 * d0) * 0.5);
                        k1 = exp(-(d1 * d1) * 0.5);
                        break;
                    }
                    case GAPLAC_OU: {
                        const double sj = p * xj;
                        k0 = exp(-fabs(p * xa[t] - sj));
                        k1 = exp(-fabs(p * xb[t] - sj));
                        break;
                    }
                    case GAPLAC_LINEAR:
                        k0 = xa[t] * xj + p;
                        k1 = xb[t] * xj + p;
                        break;
                    case GAPLAC_CAT:
                        k0 = (xa[t] == xj) ? 1.0 : 0.0;
                        k1 = (xb[t] == xj) ? 1.0 : 0.0;
                        break;
                    default:  // GAPLAC_NOISE
                        k0 = (i0 == j) ? p : 0.0;
                        k1 = (i1 == j) ? p : 0.0;
                        break;
                }
                pr0 *= k0;
                pr1 *= k1;
                if (tp.last_in_group[t]) {
                    tot0 += pr0;
                    tot1 += pr1;
                    pr0 = 1.0;
                    pr1 = 1.0;
                }
            }
        }
        double o0, o1;
        if (j < N) {
            o0 = (i0 < N) ? tot0 + ((i0 == j) ? noise : 0.0) : ((i0 == N) ? vcol[cc] : 0.0);
            o1 = (i1 < N) ? tot1 + ((i1 == j) ? noise : 0.0) : ((i1 == N) ? vcol[cc] : 0.0);
        } else {
            o0 = 0.0;
            o1 = 0.0;
        }
        *reinterpret_cast<double2*>(Ccol + (int64_t)cc * lda + i0) = make_double2(o0, o1);
    }
}

// Single-GPU layout. part 1: the first w tile columns; part 2: the lower triangle of tile
// blocks w..nt-1; part 0: everything.
__global__ __launch_bounds__(256) void gram_kernel(double* __restrict__ A, int64_t lda,
                                                   int64_t N, const double* __restrict__ X,
                                                   int64_t ldx, const double* __restrict__ v,
                                                   const TermPack* __restrict__ tpp, int nt, int part, int w0,
                                                   KTime* __restrict__ kt) {
    kt_begin(kt);
    int bi, bj;
    if (part == 1) {
        int t = (int)blockIdx.x;
        bj = 0;
        while (t >= nt - bj) {
            t -= nt - bj;
            ++bj;
        }
        bi = bj + t;
    } else {
        tri_index(blockIdx.x, bi, bj);
        bi += w0;
        bj += w0;
    }
    gram_tile(A + (int64_t)bj * NB * lda, lda, N, X, ldx, v, tpp, bi, bj);
    kt_end(kt);
}

// Distributed layout: tiles[b] = bi | lj << 16 (global row block, local tile column).
__global__ __launch_bounds__(256) void gram_list_kernel(double* __restrict__ C, int64_t ldc, int64_t N,
                                                        const double* __restrict__ X, int64_t ldx,
                                                        const double* __restrict__ v,
                                                        const TermPack* __restrict__ tpp,
                                                        const uint32_t* __restrict__ tiles, ColMap cm,
                                                        KTime* __restrict__ kt) {
    kt_begin(kt);
    const uint32_t tv = tiles[blockIdx.x];
    const int bi = (int)(tv & 0xffffu), lj = (int)(tv >> 16);
    gram_tile(C + (int64_t)lj * NB * ldc, ldc, N, X, ldx, v, tpp, bi, cm.global(lj));
    kt_end(kt);
}

// ---------------------------------------------------------------------------------
// Diagonal block: Cholesky of the 128x128 block k, plus the inverses of its eight 16x16
// diagonal sub-blocks (Dinv, consumed by the panel TRSM's blocked substitution).
// One 256-thread workgroup using 73 KiB of LDS: the same footprint as a trailing-update
// workgroup, so it can take any free slot next to them. The block lives in LDS as the
// lower triangle of an 8x8 grid of 16x16 column-major blocks (36 packed blocks).
//
// Blocked right-looking with 16-column panels, 2 barriers per panel s = 0..7:
//   phase 1: the four waves apply panel s-1 to the 8-s tiles of block column s
//            (one v_mfma_f64_16x16x4f64 chain of K = 16 each); wave 3 also inverts
//            diagonal sub-block s-1 into Dinv.
//   phase 2: wave 0 factors panel s (rows 16s..127 x 16 columns) in registers: two rows
//            per lane, pivots and L values broadcast by v_readlane, LAPACK dpotf2's
//            sqrt + reciprocal scaling, no barriers; waves 1..3 apply panel s-1 to the
//            remaining trailing tiles on MFMA.
// Pivots of padding columns (>= N) are forced to 1; a pivot <= 0 records info = j+1
// (OpenBLAS potf2's test; NaN pivots propagate, as in the reference).
// The eight 16x16 inverses are computed after the loop (off the per-panel barriers).
// ---------------------------------------------------------------------------------
constexpr int DB = 16;                    // sub-block edge
constexpr int NDB = NB / DB;              // 8
constexpr int NPK = NDB * (NDB + 1) / 2;  // 36 packed blocks
static_assert(NDB * DB * DB == DINV_PER_BLOCK, "Dinv: 8 column-major 16x16 inverses per diagonal block");

__device__ __forceinline__ int bidx(int I, int J) { return I * (I + 1) / 2 + J; }

__device__ __forceinline__ double readlane_d(double x, int l) {
    const long long v = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_readlane((int)(v & 0xffffffffll), l);
    const int hi = __builtin_amdgcn_readlane((int)(v >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// C_IJ -= L_Ik * L_Jk^T (all three column-major 16x16 blocks in Ab).
__device__ __forceinline__ void dblk_update(double* Ab, int I, int J, int k, int lane) {
    double* C = Ab + bidx(I, J) * 256;
    const double* LI = Ab + bidx(I, k) * 256;
    const double* LJ = Ab + bidx(J, k) * 256;
    const int fr = lane >> 4, fc = lane & 15;
    d4 acc;
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = C[(fr + 4 * q) * 16 + fc];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-LJ[(4 * kk + fr) * 16 + fc], LI[(4 * kk + fr) * 16 + fc],
                                                   acc, 0, 0, 0);
#pragma unroll
    for (int q = 0; q < 4; ++q) C[(fr + 4 * q) * 16 + fc] = acc[q];
}

// Dinv_s = L_ss^{-1} (column-major 16x16 into global), 16 lanes each one column.
__device__ __forceinline__ void dinv_diag(const double* Ab, double* __restrict__ Dinv,
                                          const double* rdiag, int s, int lane) {
    const double* Ls = Ab + bidx(s, s) * 256;
    asm volatile("" : "+v"(lane));  // see dpanel
    const int c = lane & 15;
    double x[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        double acc = (r == c) ? 1.0 : 0.0;
#pragma unroll
        for (int m = 0; m < r; ++m) acc -= Ls[m * 16 + r] * x[m];
        x[r] = (r >= c) ? acc * rdiag[16 * s + r] : 0.0;
    }
    if (lane < 16) {
        double* out = Dinv + s * 256;
#pragma unroll
        for (int r = 0; r < 16; ++r) out[c * 16 + r] = x[r];
    }
}

// Wave-level factorisation of panel s: rows 16s..127 x 16 columns, two rows per lane.
// Per column the critical chain is kept short: pivot (v_readlane) -> 1/sqrt (v_rsq_f64
// + two Goldschmidt steps) -> scale -> update of the NEXT column only (one v_readlane
// broadcast) -> next pivot. Column c's updates of the later columns (c+2..15) are
// deferred into iteration c+1, where they fill the latency of that pivot's 1/sqrt chain;
// their L(c2, c) factors come from an LDS broadcast (lanes 0..7 publish the scaled
// column, every lane reads it back at the end of iteration c; LDS is in order within a
// wave). The sweep is branch-free (padding pivots and the info test are selects).
__device__ __forceinline__ void dpanel(double* Ab, double* rdiag, double* colbuf, int s, int lane,
                                       int64_t gcol0, int64_t N, EvalResult* res) {
    // opaque copy of the lane id: keeps the lane-dependent masks of the sweep from being
    // hoisted out of the panel loop (and spilled) by loop-invariant code motion
    asm volatile("" : "+v"(lane));
    const int R0 = 16 * s;
    const int rel0 = 2 * lane, rel1 = rel0 + 1;
    const int row0 = R0 + rel0;
    const bool live = row0 < NB;
    double v0[16], v1[16];
    // lanes past the last row read (and never store) the panel's diagonal block
    double* blk = Ab + bidx(live ? (row0 >> 4) : s, s) * 256;
    const int rr = row0 & 15;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        v0[c] = blk[c * 16 + rr];
        v1[c] = blk[c * 16 + rr + 1];
    }
    const int64_t npiv = N - (gcol0 + R0);  // columns >= npiv are padding (unit pivots)
    double myrd = 1.0;
    int bad = 16;
    double piv = readlane_d(v0[0], 0);
    double lc[16];  // L(c2, c-1) for c2 >= c+1 (broadcast of the previous column)
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        const bool pad = c >= npiv;
        // OpenBLAS potf2 (the reference's dpotrf, 0.3.20) tests ajj <= 0 only: a NaN
        // pivot is not reported and propagates to a NaN logpdf, as in the reference.
        bad = (!pad && piv <= 0.0 && bad == 16) ? c : bad;
        const double p = pad ? 1.0 : piv;
        // Goldschmidt from v_rsq_f64: g -> sqrt(p), h -> 1/(2 sqrt(p))
        const double y = __builtin_amdgcn_rsq(p);
        double g = p * y, h = 0.5 * y;
        // deferred updates of columns c+1..15 by column c-1
        if (c >= 1) {
#pragma unroll
            for (int c2 = c + 1; c2 < 16; ++c2) {
                v0[c2] = fma(-v0[c - 1], lc[c2], v0[c2]);
                v1[c2] = fma(-v1[c - 1], lc[c2], v1[c2]);
            }
        }
        double r = fma(-g, h, 0.5);
        g = fma(g, r, g);
        h = fma(h, r, h);
        r = fma(-g, h, 0.5);
        g = fma(g, r, g);
        h = fma(h, r, h);
        const double d = g, rd = h + h;
        myrd = lane == c ? rd : myrd;
        v0[c] = rel0 > c ? v0[c] * rd : (rel0 == c ? d : v0[c]);
        v1[c] = rel1 > c ? v1[c] * rd : (rel1 == c ? d : v1[c]);
        if (c < 15) {
            double* cb = colbuf + 16 * (c & 1);
            if (c < 14 && lane < 8) *reinterpret_cast<double2*>(&cb[2 * lane]) = make_double2(v0[c], v1[c]);
            const double ln = readlane_d(((c + 1) & 1) ? v1[c] : v0[c], (c + 1) >> 1);
            v0[c + 1] = fma(-v0[c], ln, v0[c + 1]);
            v1[c + 1] = fma(-v1[c], ln, v1[c + 1]);
            piv = readlane_d(((c + 1) & 1) ? v1[c + 1] : v0[c + 1], (c + 1) >> 1);
            if (c < 14) {
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int q = (c + 2) >> 1; q < 8; ++q) {
                    const double2 w = *reinterpret_cast<const double2*>(&cb[2 * q]);
                    lc[2 * q] = w.x;
                    lc[2 * q + 1] = w.y;
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    if (bad < 16 && lane == 0) atomicMin(&res->info, (unsigned long long)(gcol0 + R0 + bad + 1));
    if (lane < 16) rdiag[R0 + lane] = myrd;
    if (live) {
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            blk[c * 16 + rr] = (rel0 >= c) ? v0[c] : 0.0;  // zero the diagonal block's upper part
            blk[c * 16 + rr + 1] = (rel1 >= c) ? v1[c] : 0.0;
        }
    }
}

__device__ __forceinline__ void potrf_diag_kernel_body(double* __restrict__ Ag, int64_t lda,
                                                         int64_t N, int64_t g0,
                                                         double* __restrict__ Dinv,
                                                         EvalResult* __restrict__ res) {
    // one LDS array, small buffers first: their addresses fit ds_read's 16-bit offset
    __shared__ double smem[32 + NB + NPK * 256];
    double* colbuf = smem;
    double* rdiag = smem + 32;
    double* Ab = smem + 32 + NB;
    __builtin_amdgcn_s_setprio(3);  // critical path: win issue arbitration on shared SIMDs
    STAMP(20);
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    // load the lower block triangle: element (r, c) of block (I, J) <- A(16I+r, 16J+c)
    {
        const double* colp = Ag + (int64_t)(t >> 4) * lda + (t & 15);
#pragma unroll
        for (int J = 0; J < NDB; ++J)
#pragma unroll
            for (int I = J; I < NDB; ++I)
                Ab[bidx(I, J) * 256 + t] = colp[(int64_t)(16 * J) * lda + 16 * I];
    }
    __syncthreads();
    STAMP(0);
    for (int s = 0; s < NDB; ++s) {
        if (s >= 1) {
            for (int I = s + wave; I < NDB; I += 4) dblk_update(Ab, I, s, s - 1, lane);
        }
        __syncthreads();
        STAMP(1 + 2 * s);
        if (wave == 0) {
            dpanel(Ab, rdiag, colbuf, s, lane, g0, N, res);
        } else if (s >= 1) {
            if (wave == 3) dinv_diag(Ab, Dinv, rdiag, s - 1, lane);  // off the barrier path
            const int ntr = (NDB - 1 - s) * (NDB - s) / 2;  // tiles (I,J), s+1 <= J <= I <= 7
            for (int task = wave - 1; task < ntr; task += 3) {
                int J = s + 1, rem = task;
                while (rem >= NDB - J) {
                    rem -= NDB - J;
                    ++J;
                }
                dblk_update(Ab, J + rem, J, s - 1, lane);
            }
        }
        if (wave == 0) STAMP(2 + 2 * s);
        __syncthreads();
    }
    STAMP(17);
    if (wave == 3) dinv_diag(Ab, Dinv, rdiag, NDB - 1, lane);
    STAMP(18);
    // write L (lower incl. diagonal) in place
    {
        const int c = t >> 4, r = t & 15;
        double* colq = Ag + (int64_t)c * lda + r;
        asm volatile("" : "+v"(colq));  // recomputed here: no load addresses live across the sweep
#pragma unroll
        for (int J = 0; J < NDB; ++J)
#pragma unroll
            for (int I = J; I < NDB; ++I)
                if (I != J || r >= c) colq[(int64_t)(16 * J) * lda + 16 * I] = Ab[bidx(I, J) * 256 + t];
    }
    STAMP(19);
}

// ---------------------------------------------------------------------------------
// Diagonal block, blocked version (default): 16x16 leaves.
//
// Per 16-column panel s only the 16x16 diagonal sub-block is factored serially (wave 0,
// one row per lane, f16_factor); the 16(7-s) rows below it are solved against it on the
// other waves (one row per lane, VALU forward substitution, f16_trsm_row), and the
// trailing sub-blocks get the panel on MFMA (dblk_update). Wave 0 updates the next
// diagonal sub-block itself and factors it right away, while waves 1-3 update the rest.
// Two barriers per panel. The serial part per column is only the 16-row pivot chain
// (readlane pivot -> v_rcp_f64 + 2 Newton steps -> the next column's own update ->
// readlane), against the whole 128-row panel sweep of the unblocked kernel above.
// ---------------------------------------------------------------------------------

// Factor the 16x16 diagonal sub-block blk (LDS, column-major) in place: L (upper part
// zeroed), rdg[c] = 1/L(c,c). Wave-level: lane r (r = lane & 15) holds row r; lanes 16..63
// mirror lanes 0..15 and never store. Schur updates use A(r,c) A(c2,c) / p (p the pivot),
// so the chain to the next pivot needs 1/p only; 1/sqrt(p) (the scaled column) is off the
// chain. Padding columns (>= npiv) get unit pivots; the first pivot <= 0 sets bad.
__device__ __forceinline__ void f16_factor(double* blk, double* rdg, int lane, int64_t npiv, int& bad) {
    asm volatile("" : "+v"(lane));  // keep the lane masks inside the loop (see dpanel)
    const int r = lane & 15;
    double a[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) a[c] = blk[c * 16 + r];
    double myrd = 1.0;
    double q = a[0];  // lane c: the updated A(c,c) when column c starts
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        const double piv = readlane_d(q, c);
        const bool pad = c >= npiv;
        // OpenBLAS potf2 tests ajj <= 0 only: a NaN pivot propagates (as in the reference)
        bad = (!pad && piv <= 0.0 && bad == 16) ? c : bad;
        const double p = pad ? 1.0 : piv;
        double y = __builtin_amdgcn_rcp(p);  // 1/p: two Newton steps
        double e = fma(-p, y, 1.0);
        y = fma(y, e, y);
        e = fma(-p, y, 1.0);
        y = fma(y, e, y);
        const double w = a[c] * y;  // A(r, c) / p
        if (c < 15) {
            q = fma(-a[c], w, a[c + 1]);  // lane c+1: next pivot from its own w
#pragma unroll
            for (int c2 = c + 1; c2 < 16; ++c2) a[c2] = fma(-a[c], readlane_d(w, c2), a[c2]);
        }
        const double z = __builtin_amdgcn_rsq(p);  // 1/sqrt(p), Goldschmidt-refined
        double g = p * z, h = 0.5 * z;
        double t = fma(-g, h, 0.5);
        g = fma(g, t, g);
        h = fma(h, t, h);
        t = fma(-g, h, 0.5);
        g = fma(g, t, g);
        h = fma(h, t, h);
        const double rs = h + h;
        myrd = r == c ? rs : myrd;
        a[c] = r > c ? a[c] * rs : (r == c ? g : 0.0);
    }
    if (lane < 16) {
#pragma unroll
        for (int c = 0; c < 16; ++c) blk[c * 16 + r] = a[c];
        rdg[r] = myrd;
    }
}

// One row of a sub-block below the diagonal: x <- x L^{-T} (forward substitution against
// the factored diagonal sub-block Ls; rd = 1/diag). L values are wave-uniform LDS reads.
__device__ __forceinline__ void f16_trsm_row(double* row, const double* Ls, const double* rd) {
    double x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = row[c * 16];
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        x[c] *= rd[c];
#pragma unroll
        for (int c2 = c + 1; c2 < 16; ++c2) x[c2] = fma(-x[c], Ls[c * 16 + c2], x[c2]);
    }
#pragma unroll
    for (int c = 0; c < 16; ++c) row[c * 16] = x[c];
}

__device__ __forceinline__ void potrf_diag_blocked_body(double* __restrict__ Ag, int64_t lda, int64_t N, int64_t g0,
                                                        double* __restrict__ Dinv, EvalResult* __restrict__ res) {
    __shared__ double smem[NB + NPK * 256];
    double* rdiag = smem;
    double* Ab = smem + NB;
    __builtin_amdgcn_s_setprio(3);
    STAMP(99);
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    {
        const double* colp = Ag + (int64_t)(t >> 4) * lda + (t & 15);
#pragma unroll
        for (int J = 0; J < NDB; ++J)
#pragma unroll
            for (int I = J; I < NDB; ++I) Ab[bidx(I, J) * 256 + t] = colp[(int64_t)(16 * J) * lda + 16 * I];
    }
    STAMP(100);
    __syncthreads();
    STAMP(101);
    int bad = 16, badpanel = -1;
    if (wave == 0) {
        f16_factor(Ab, rdiag, lane, N - g0, bad);
        if (bad < 16) badpanel = 0;
    }
    STAMP(102);
    __syncthreads();
    for (int s = 0; s < NDB; ++s) {
        // panel rows below the diagonal sub-block: waves 1..3, one row per lane;
        // wave 0 inverts the diagonal sub-block for the TRSM kernel (output only)
        STAMP(4 * s);
        if (wave == 0) {
            dinv_diag(Ab, Dinv, rdiag, s, lane);
            STAMP(4 * s + 1);
        } else {
            const double* Ls = Ab + bidx(s, s) * 256;
            for (int rr = t - 64; rr < 16 * (NDB - 1 - s); rr += 192) {
                const int I = s + 1 + (rr >> 4);
                f16_trsm_row(Ab + bidx(I, s) * 256 + (rr & 15), Ls, rdiag + 16 * s);
            }
            STAMPT(64, 40 + s);
        }
        __syncthreads();
        STAMP(4 * s + 2);
        // column s of L is final: store it (waves 1..3; a diagonal sub-block's lower part)
        if (wave > 0) {
            const int nel = (NDB - s) * 256;
            for (int e = t - 64; e < nel; e += 192) {
                const int I = s + (e >> 8), el = e & 255, c = el >> 4, r = el & 15;
                if (I != s || r >= c) Ag[(int64_t)(16 * s + c) * lda + 16 * I + r] = Ab[bidx(I, s) * 256 + el];
            }
        }
        if (s == NDB - 1) break;
        if (wave == 0) {
            dblk_update(Ab, s + 1, s + 1, s, lane);
            STAMP(4 * s + 3);
            int b2 = 16;
            f16_factor(Ab + bidx(s + 1, s + 1) * 256, rdiag + 16 * (s + 1), lane, N - g0 - 16 * (s + 1), b2);
            if (b2 < 16 && bad == 16) {
                bad = b2;
                badpanel = s + 1;
            }
        } else {
            // trailing sub-blocks (I, J), s+1 <= J <= I <= 7, except (s+1, s+1)
            const int ntr = (NDB - 1 - s) * (NDB - s) / 2;
            for (int task = wave; task < ntr; task += 3) {
                int J = s + 1, rem = task;
                while (rem >= NDB - J) {
                    rem -= NDB - J;
                    ++J;
                }
                dblk_update(Ab, J + rem, J, s, lane);
            }
            STAMPT(64, 50 + s);
        }
        STAMP(60 + s);
        __syncthreads();
    }
    STAMP(103);
    if (wave == 0 && lane == 0 && badpanel >= 0)
        atomicMin(&res->info, (unsigned long long)(g0 + 16 * badpanel + bad + 1));
}

// Diagonal kernel choice (compile time): 1 = the unblocked 128-row panel sweep (default,
// 39 us alone); 0 = the blocked 16x16-leaf kernel (44 us alone, measured slower: its
// serial leaf factor costs ~360 cycles per column, as much as the whole-panel sweep).
#ifndef GAPLAC_DIAG_V1
#define GAPLAC_DIAG_V1 1
#endif

// Ag: the diagonal block (global rows/cols g0 .. g0+127) in its storage, leading dim lda.
__global__ __launch_bounds__(256) void potrf_diag_kernel(double* __restrict__ Ag, int64_t lda,
                                                         int64_t N, int64_t g0,
                                                         double* __restrict__ Dinv,
                                                         EvalResult* __restrict__ res,
                                                         KTime* __restrict__ kt) {
    kt_begin(kt);
    if constexpr (GAPLAC_DIAG_V1)
        potrf_diag_kernel_body(Ag, lda, N, g0, Dinv, res);
    else
        potrf_diag_blocked_body(Ag, lda, N, g0, Dinv, res);
    kt_end(kt);
}

// ---------------------------------------------------------------------------------
// Panel TRSM by blocked substitution: for each 128-row tile i > k of panel column k,
//   X = B L_kk^{-T}:  X_b = (B_b - sum_{c<b} X_c L_bc^T) Dinv_b^T,  b = 0..7 (16 columns)
// computed transposed (Y_b = X_b^T = Dinv_b (B_b^T - sum_c L_bc Y_c)) so that every
// result stays in the f64 MFMA accumulator layout (row = lane/16 + 4q, col = lane%16),
// which is exactly the B-operand layout of the next MFMA: no LDS, no transposes.
// Two workgroups per tile, 4 waves x 16 rows each: the substitution is a dependent MFMA
// chain per wave (sum_b 4b+4 = 144 MFMAs), so its latency scales with rows per wave.
// The 28 strictly-lower 16x16 blocks of L_kk and the eight Dinv blocks are staged once
// per workgroup in LDS (72 KiB), column-major per block, so A-operand reads are 16
// consecutive doubles per lane group.
// ---------------------------------------------------------------------------------
constexpr int TRSM_LBLK = NDB * (NDB - 1) / 2;  // 28

// Acol: storage of the panel's first column (global column k*NB), rows global.
__device__ __forceinline__ void trsm_subst_kernel_body(double* __restrict__ Acol, int64_t lda, int k, int bi0,
                                                         const double* __restrict__ Dinv) {
    __shared__ double Ls[(TRSM_LBLK + NDB) * 256 + NB];  // + NB: padded to CHAIN_LDS (see LR8)
    __builtin_amdgcn_s_setprio(2);  // critical path
    const int tid = threadIdx.x;
    const int bi = bi0 + (int)(blockIdx.x >> 1);
    const int wave = tid >> 6, lane = tid & 63;
    const int fr = lane >> 4, fc = lane & 15;
    const int64_t k0 = (int64_t)k * NB;
    const double* L = Acol + k0;  // L_kk, column-major, lda
    double* B = Acol + (int64_t)bi * NB + 64 * (blockIdx.x & 1) + 16 * wave;
    {
        // block (b, c), c < b, at p = b(b-1)/2 + c: Ls[p*256 + m*16 + j] = L(16b + j, 16c + m)
        const double* Lt = L + (int64_t)(tid >> 4) * lda + (tid & 15);
        double lv[TRSM_LBLK], dv[NDB];
#pragma unroll
        for (int b = 1; b < NDB; ++b)
#pragma unroll
            for (int c = 0; c < b; ++c) lv[b * (b - 1) / 2 + c] = Lt[(int64_t)(16 * c) * lda + 16 * b];
#pragma unroll
        for (int q = 0; q < NDB; ++q) dv[q] = Dinv[q * 256 + tid];
#pragma unroll
        for (int p = 0; p < TRSM_LBLK; ++p) Ls[p * 256 + tid] = lv[p];
#pragma unroll
        for (int q = 0; q < NDB; ++q) Ls[(TRSM_LBLK + q) * 256 + tid] = dv[q];
    }
    // this wave's 16 rows of tile (bi, k), loaded after the L / Dinv staging so that the two
    // sets of registers are never live together (216 -> 169 VGPRs), all up front
    d4 Bt[NDB];
#pragma unroll
    for (int b = 0; b < NDB; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q)  // B_b^T in accumulator layout: [j][r] = B[r][16b + j]
            Bt[b][q] = B[(int64_t)(16 * b + fr + 4 * q) * lda + fc];
    __syncthreads();
    d4 Y[NDB];
#pragma unroll
    for (int b = 0; b < NDB; ++b) {
        d4 s0 = Bt[b], s1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int c = 0; c < b; ++c) {
            const double* Lbc = Ls + (b * (b - 1) / 2 + c) * 256;
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                const double lbc = -Lbc[(4 * kk + fr) * 16 + fc];  // L_bc[j][m], m = 4kk + fr
                // two partial sums (even / odd c): halves the dependent-accumulator chain
                if (c & 1)
                    s1 = __builtin_amdgcn_mfma_f64_16x16x4f64(lbc, Y[c][kk], s1, 0, 0, 0);
                else
                    s0 = __builtin_amdgcn_mfma_f64_16x16x4f64(lbc, Y[c][kk], s0, 0, 0, 0);
            }
        }
        s0 += s1;
        const double* Di = Ls + (TRSM_LBLK + b) * 256;  // column-major: A operand [j = fc][m = 4kk + fr]
        d4 y = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
            y = __builtin_amdgcn_mfma_f64_16x16x4f64(Di[(4 * kk + fr) * 16 + fc], s0[kk], y, 0, 0, 0);
        Y[b] = y;
#pragma unroll
        for (int q = 0; q < 4; ++q) B[(int64_t)(16 * b + fr + 4 * q) * lda + fc] = y[q];
    }
}

__global__ __launch_bounds__(256) void trsm_subst_kernel(
    double* __restrict__ Acol, int64_t lda, int k,
                                                         int bi0, const double* __restrict__ Dinv,
                                                         KTime* __restrict__ kt) {
    kt_begin(kt);
    trsm_subst_kernel_body(Acol, lda, k, bi0, Dinv);
    kt_end(kt);
}

// ---------------------------------------------------------------------------------
// Bulk trailing update, one 128x128 tile per 256-thread workgroup:
//   C(bi, bj) -= P_bi P_bj^T,   P = the kdepth panel columns (Panel operand),
// with C tile (bi, bj) stored in local tile column lj (ColMap: bj = cm.global(lj)).
// 4 waves as 2x2, each wave a 64x64 sub-tile = 4x4 v_mfma_f64_16x16x4f64 accumulators.
// Operands are staged through LDS in 16-deep k-chunks, double-buffered with a register
// prefetch of the next chunk. The MFMA computes D = Q*P^T (the j-side fragment is the A
// operand) so that a lane's accumulator column is C's row: stores are 128-byte column
// segments of the column-major matrix. The C tile is loaded straight into the
// accumulators before the k-loop and P is staged negated, so the MFMA chain produces
// C - P Q^T and the epilogue is stores only.
// Tile placement: a precomputed list maps blockIdx -> (bi, lj) = (bi0 + lo16, lj0 + hi16).
// The list is ordered so that the blocks one XCD runs (blockIdx % 8, dealt round-robin by
// the dispatcher) walk one contiguous run of 8x8 super-tiles: the panel row blocks of its
// ~64 resident tiles stay in that XCD's 4 MiB L2. Placement only affects speed; any
// blockIdx -> tile bijection is correct.
// ---------------------------------------------------------------------------------
#ifndef GAPLAC_KB
#define GAPLAC_KB 16
#endif
constexpr int KB = GAPLAC_KB;  // k-chunk staged in LDS (8 or 16)
static_assert(KB == 8 || KB == 16, "k-chunk of the tile kernels: 8 or 16");
constexpr int LR = NB + 16;  // LDS k-row stride: lanes 16..31 land on banks 32..63

__device__ __forceinline__ void tile_decode(const BulkArgs& a, int idx, int& bi, int& bj, int& lj) {
    int r, c;
    if (a.rect_rows > 0) {
        // rectangular block (rect_rows x ntiles/rect_rows), generated on the fly: strips of
        // 8 tile rows, columns outer within a strip (an XCD's contiguous run of the list
        // shares its 8 panel row blocks and walks the columns)
        const int mr = a.rect_rows, mc = a.ntiles / mr;
        const int full = (mr >> 3) * 8 * mc;
        if (idx < full) {
            const int strip = idx / (8 * mc), w = idx - strip * 8 * mc;
            c = w >> 3;
            r = strip * 8 + (w & 7);
        } else {
            const int rem = mr & 7, w = idx - full;
            c = w / rem;
            r = (mr & ~7) + (w - c * rem);
        }
    } else {
        const uint32_t tv = a.tiles[idx];
        r = (int)(tv & 0xffffu);
        c = (int)(tv >> 16);
    }
    bi = a.bi0 + r;
    lj = a.lj0 + c;
    bj = a.cm.global(lj);
}

// Shared k-loop of the 128x128 tile kernels: acc[mi][mj] (wave (wi, wj) of the 2x2 wave
// grid) += -P_i Q_j^T over kdepth panel columns, where P (rows of tile i) and Q (rows of
// tile j) are column-major with leading dimension ldp. Lane element (mi, mj, rg) is tile
// entry (row 64 wi + 16 mi + (lane & 15), column 64 wj + 16 mj + (lane >> 4) + 4 rg).
// Inactive waves (upper quadrant of a diagonal tile) only help with the staging.
__device__ __forceinline__ void tile_mma_neg(const double* __restrict__ P, const double* __restrict__ Q,
                                             int64_t ldp, int kdepth, bool active, d4 (&acc)[4][4]) {
    __shared__ double sm[2][2][KB][LR];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wi = w & 1, wj = w >> 1;
    const int fr = lane >> 4, fc = lane & 15;
    // staging: thread -> (k row krow + 4 it, rows 2 lane, 2 lane + 1) of both operands
    const int krow = tid >> 6;  // 0..3
    const double* Pr = P + (int64_t)krow * ldp + 2 * lane;
    const double* Qr = Q + (int64_t)krow * ldp + 2 * lane;
    const int64_t s4 = 4 * ldp;
    double2 p0, p1, p2, p3, q0, q1, q2, q3;
#define GAPLAC_GLOAD(ch)                                                               \
    do {                                                                               \
        const int64_t o_ = (int64_t)(ch) * KB * ldp;                                   \
        p0 = *reinterpret_cast<const double2*>(Pr + o_);                               \
        p1 = *reinterpret_cast<const double2*>(Pr + o_ + s4);                          \
        q0 = *reinterpret_cast<const double2*>(Qr + o_);                               \
        q1 = *reinterpret_cast<const double2*>(Qr + o_ + s4);                          \
        if constexpr (KB == 16) {                                                      \
            p2 = *reinterpret_cast<const double2*>(Pr + o_ + 2 * s4);                  \
            p3 = *reinterpret_cast<const double2*>(Pr + o_ + 3 * s4);                  \
            q2 = *reinterpret_cast<const double2*>(Qr + o_ + 2 * s4);                  \
            q3 = *reinterpret_cast<const double2*>(Qr + o_ + 3 * s4);                  \
        }                                                                              \
    } while (0)
#define GAPLAC_LSTORE(buf)                                                             \
    do {                                                                               \
        double* sp_ = &sm[buf][0][krow][2 * lane];                                     \
        double* sq_ = &sm[buf][1][krow][2 * lane];                                     \
        *reinterpret_cast<double2*>(sp_) = make_double2(-p0.x, -p0.y);                 \
        *reinterpret_cast<double2*>(sp_ + 4 * LR) = make_double2(-p1.x, -p1.y);        \
        *reinterpret_cast<double2*>(sq_) = q0;                                         \
        *reinterpret_cast<double2*>(sq_ + 4 * LR) = q1;                                \
        if constexpr (KB == 16) {                                                      \
            *reinterpret_cast<double2*>(sp_ + 8 * LR) = make_double2(-p2.x, -p2.y);    \
            *reinterpret_cast<double2*>(sp_ + 12 * LR) = make_double2(-p3.x, -p3.y);   \
            *reinterpret_cast<double2*>(sq_ + 8 * LR) = q2;                            \
            *reinterpret_cast<double2*>(sq_ + 12 * LR) = q3;                           \
        }                                                                              \
    } while (0)

    GAPLAC_GLOAD(0);
    GAPLAC_LSTORE(0);
    __syncthreads();
    const int NCH = kdepth / KB;
    for (int ch = 0; ch < NCH; ++ch) {
        const int buf = ch & 1;
        const bool more = ch + 1 < NCH;
        if (more) GAPLAC_GLOAD(ch + 1);
        if (active) {
#pragma unroll
            for (int ks = 0; ks < KB; ks += 4) {
                double fa[4], fb[4];
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    fa[m] = sm[buf][1][ks + fr][64 * wj + 16 * m + fc];
                    fb[m] = sm[buf][0][ks + fr][64 * wi + 16 * m + fc];
                }
#pragma unroll
                for (int mj = 0; mj < 4; ++mj)
#pragma unroll
                    for (int mi = 0; mi < 4; ++mi)
                        acc[mi][mj] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[mj], fb[mi],
                                                                            acc[mi][mj], 0, 0, 0);
            }
        }
        if (more) GAPLAC_LSTORE(buf ^ 1);
        __syncthreads();
    }
#undef GAPLAC_GLOAD
#undef GAPLAC_LSTORE
}

__device__ __forceinline__ void tile_syrk_body(const BulkArgs& a) {
    const int b = (int)blockIdx.x;
    const int chunk = (a.ntiles + 7) >> 3;
    const int idx = (b & 7) * chunk + (b >> 3);
    if (idx >= a.ntiles) return;
    int bi, bj, lj;
    tile_decode(a, idx, bi, bj, lj);
    const int64_t r0 = (int64_t)bi * NB;
    const int64_t ldc = a.ldc;
    double* __restrict__ Ct = a.C + (int64_t)lj * NB * ldc + r0;
    const double* __restrict__ P = a.pn.P + (r0 - a.pn.row0);
    const double* __restrict__ Q = a.pn.P + ((int64_t)bj * NB - a.pn.row0);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wi = w & 1, wj = w >> 1;
    const bool active = !(bi == bj && wj > wi);
    const int fr = lane >> 4, fc = lane & 15;

    d4 acc[4][4];
    if (active) {
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
            const double* Ci = Ct + 64 * wi + 16 * mi + fc;
#pragma unroll
            for (int mj = 0; mj < 4; ++mj)
#pragma unroll
                for (int rg = 0; rg < 4; ++rg)
                    acc[mi][mj][rg] = Ci[(int64_t)(64 * wj + 16 * mj + fr + 4 * rg) * ldc];
        }
    }
    tile_mma_neg(P, Q, a.pn.ld, a.kdepth, active, acc);
    if (!active) return;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
        double* Ci = Ct + 64 * wi + 16 * mi + fc;
#pragma unroll
        for (int mj = 0; mj < 4; ++mj)
#pragma unroll
            for (int rg = 0; rg < 4; ++rg)
                Ci[(int64_t)(64 * wj + 16 * mj + fr + 4 * rg) * ldc] = acc[mi][mj][rg];
    }
}

__global__ __launch_bounds__(256, 2) void tile_syrk_kernel(BulkArgs a, KTime* __restrict__ kt) {
    kt_begin(kt);
    tile_syrk_body(a);
    kt_end(kt);
}

// ---------------------------------------------------------------------------------
// Bulk trailing update, 8-wave variant (default): one 128x128 tile per 512-thread
// workgroup, waves as 2 (rows) x 4 (columns), each a 64x32 sub-tile = 4x2 f64 MFMA
// accumulators (half the accumulator registers of the 4-wave kernel). Launched with
// dynamic LDS padding so that ONE such workgroup occupies a CU (2 waves per SIMD): the
// rest of the CU — 4 KiB short of half its LDS and more than half of every SIMD's
// registers — stays free for the critical-path kernels (diagonal block, TRSM, column
// updates), which then start at once instead of waiting for a round of bulk workgroups
// to retire. Same staging scheme as tile_mma_neg.
// ---------------------------------------------------------------------------------
// LDS budget of a CU shared by one bulk workgroup and one critical-path workgroup
// (measured with tools/coresid_probe.hip and tools/cores2_probe.hip on MI355X). LDS is
// allocated contiguously per workgroup, and a pair summing to exactly 160 KiB does not
// fit. The bulk kernel's staging rows are padded (row stride LR8) to 84 KiB, so two bulk
// workgroups never share a CU, and every LDS-heavy chain kernel (diagonal block, TRSM)
// takes exactly CHAIN_LDS = 73 KiB: in whichever order the two land on a CU, the hole one
// leaves is what the other needs (a 72 KiB TRSM at offset 0 would otherwise leave a bulk
// workgroup at 72..156 KiB and no 73 KiB hole for the next diagonal block until that bulk
// workgroup retires).
constexpr int LR8 = 168;  // 86,016 B of staging (the rows past NB are padding)
constexpr int BULK8_LDS = 2 * 2 * KB * LR8 * 8;
constexpr int CHAIN_LDS = 8 * (NB + NPK * 256);  // the blocked diagonal kernel's footprint
static_assert(2 * BULK8_LDS > 163840 && BULK8_LDS + CHAIN_LDS < 163840, "one bulk + one chain workgroup per CU");
static_assert(8 * ((TRSM_LBLK + NDB) * 256 + NB) == CHAIN_LDS, "TRSM kernel padded to CHAIN_LDS");

__device__ __forceinline__ void tile_mma8_neg(const double* __restrict__ P, const double* __restrict__ Q,
                                              int64_t ldp, int kdepth, bool active, d4 (&acc)[4][2]) {
    __shared__ double sm[2][2][KB][LR8];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wi = w & 1, wj = w >> 1;
    const int fr = lane >> 4, fc = lane & 15;
    // staging: thread -> (k rows krow, krow + 8, rows 2 lane, 2 lane + 1) of both operands
    const int krow = w;  // 0..7
    const double* Pr = P + (int64_t)krow * ldp + 2 * lane;
    const double* Qr = Q + (int64_t)krow * ldp + 2 * lane;
    const int64_t s8 = 8 * ldp;
    double2 p0, p1, q0, q1;
#define GAPLAC_GLOAD8(ch)                                                              \
    do {                                                                               \
        const int64_t o_ = (int64_t)(ch) * KB * ldp;                                   \
        p0 = *reinterpret_cast<const double2*>(Pr + o_);                               \
        q0 = *reinterpret_cast<const double2*>(Qr + o_);                               \
        if constexpr (KB == 16) {                                                      \
            p1 = *reinterpret_cast<const double2*>(Pr + o_ + s8);                      \
            q1 = *reinterpret_cast<const double2*>(Qr + o_ + s8);                      \
        }                                                                              \
    } while (0)
#define GAPLAC_LSTORE8(buf)                                                            \
    do {                                                                               \
        double* sp_ = &sm[buf][0][krow][2 * lane];                                     \
        double* sq_ = &sm[buf][1][krow][2 * lane];                                     \
        *reinterpret_cast<double2*>(sp_) = make_double2(-p0.x, -p0.y);                 \
        *reinterpret_cast<double2*>(sq_) = q0;                                         \
        if constexpr (KB == 16) {                                                      \
            *reinterpret_cast<double2*>(sp_ + 8 * LR8) = make_double2(-p1.x, -p1.y);   \
            *reinterpret_cast<double2*>(sq_ + 8 * LR8) = q1;                           \
        }                                                                              \
    } while (0)

    GAPLAC_GLOAD8(0);
    GAPLAC_LSTORE8(0);
    __syncthreads();
    const int NCH = kdepth / KB;
    for (int ch = 0; ch < NCH; ++ch) {
        const int buf = ch & 1;
        const bool more = ch + 1 < NCH;
        if (more) GAPLAC_GLOAD8(ch + 1);
        if (active) {
#pragma unroll
            for (int ks = 0; ks < KB; ks += 4) {
                double fa[2], fb[4];
#pragma unroll
                for (int m = 0; m < 2; ++m) fa[m] = sm[buf][1][ks + fr][32 * wj + 16 * m + fc];
#pragma unroll
                for (int m = 0; m < 4; ++m) fb[m] = sm[buf][0][ks + fr][64 * wi + 16 * m + fc];
#pragma unroll
                for (int mj = 0; mj < 2; ++mj)
#pragma unroll
                    for (int mi = 0; mi < 4; ++mi)
                        acc[mi][mj] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[mj], fb[mi], acc[mi][mj], 0, 0, 0);
            }
        }
        if (more) GAPLAC_LSTORE8(buf ^ 1);
        __syncthreads();
    }
#undef GAPLAC_GLOAD8
#undef GAPLAC_LSTORE8
}

__global__ __launch_bounds__(512, 1) void tile_syrk8_kernel(BulkArgs a, KTime* __restrict__ kt) {
    kt_begin(kt);
    // Tiles of XCD x (= blockIdx % 8) are the contiguous run [x chunk, (x+1) chunk) of the
    // list. Persistent launches (gridDim < tiles) walk it with stride gridDim / 8.
    const int chunk = (a.ntiles + 7) >> 3;
    const int per_xcd = (int)gridDim.x >> 3;
    const int x = (int)blockIdx.x & 7;
    for (int k = (int)blockIdx.x >> 3; k < chunk; k += per_xcd) {
    const int idx = x * chunk + k;
    if (idx >= a.ntiles) break;
    {
        int bi, bj, lj;
        tile_decode(a, idx, bi, bj, lj);
        const int64_t r0 = (int64_t)bi * NB;
        const int64_t ldc = a.ldc;
        double* __restrict__ Ct = a.C + (int64_t)lj * NB * ldc + r0;
        const double* __restrict__ P = a.pn.P + (r0 - a.pn.row0);
        const double* __restrict__ Q = a.pn.P + ((int64_t)bj * NB - a.pn.row0);
        const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
        const int wi = w & 1, wj = w >> 1;
        // on a diagonal tile, waves with rows 0..63 and columns 64..127 lie above it
        const bool active = !(bi == bj && wi == 0 && wj >= 2);
        const int fr = lane >> 4, fc = lane & 15;
        d4 acc[4][2];
        if (active) {
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) {
                const double* Ci = Ct + 64 * wi + 16 * mi + fc;
#pragma unroll
                for (int mj = 0; mj < 2; ++mj)
#pragma unroll
                    for (int rg = 0; rg < 4; ++rg)
                        acc[mi][mj][rg] = Ci[(int64_t)(32 * wj + 16 * mj + fr + 4 * rg) * ldc];
            }
        }
        tile_mma8_neg(P, Q, a.pn.ld, a.kdepth, active, acc);
        if (active) {
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) {
                double* Ci = Ct + 64 * wi + 16 * mi + fc;
#pragma unroll
                for (int mj = 0; mj < 2; ++mj)
#pragma unroll
                    for (int rg = 0; rg < 4; ++rg)
                        Ci[(int64_t)(32 * wj + 16 * mj + fr + 4 * rg) * ldc] = acc[mi][mj][rg];
            }
        }
    }
    }
    kt_end(kt);
}

// ---------------------------------------------------------------------------------
// Quadrant update: C_q -= P_q Q_q^T for one 64x64 quadrant (qi, qj) of tile (bi, bj)
// (stored in local tile column lj), K = kdepth panel columns. 4 waves as 2x2 of 32x32
// (2x2 f64 MFMA accumulators each); fragments come straight from global memory (the panel
// columns are L2-resident), register double-buffered 8 k-steps (32 columns) ahead, no
// LDS, no barriers. Used where latency matters more than throughput: the lookahead column
// update on the critical path and the small trailing updates at the end of the
// factorisation (a 128x128x256 tile alone on a CU takes ~50 us; a quadrant ~4x less).
// ---------------------------------------------------------------------------------
// k-steps per prefetch group. 2 keeps the quadrant kernels at 96 VGPRs: exactly what two
// resident bulk-update waves (2 x 208) leave on a SIMD, so the critical-path column updates
// start on CUs that are busy with bulk tiles instead of waiting for one to retire
// (measured: 8 -> 2 cuts their in-situ time from ~17 to ~11 ms per N=16384 evaluation).
#ifndef GAPLAC_QG
#define GAPLAC_QG 2
#endif
constexpr int QG = GAPLAC_QG;
// Bulk updates with at most this many 128x128 tiles run as quadrants (4 WGs per tile).
constexpr int QUAD_BULK_MAX_TILES = 512;

__device__ __forceinline__ void quad_update(double* __restrict__ C, int64_t ldc, const Panel& pn, int bi,
                                            int bj, int lj, int qi, int qj, int kdepth) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wi = wave & 1, wj = wave >> 1;
    const int fr = lane >> 4, fc = lane & 15;
    const int64_t ri = (int64_t)bi * NB + 64 * qi + 32 * wi;   // this wave's 32 rows
    const int64_t cj = (int64_t)bj * NB + 64 * qj + 32 * wj;   // this wave's 32 columns (global)
    const int64_t cl = (int64_t)lj * NB + 64 * qj + 32 * wj;   // ... in storage
    const int64_t ldp = pn.ld;
    const double* P = pn.P + (ri - pn.row0) + fc;
    const double* Q = pn.P + (cj - pn.row0) + fc;
    d4 acc[2][2];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int mj = 0; mj < 2; ++mj)
#pragma unroll
            for (int rg = 0; rg < 4; ++rg)
                acc[mi][mj][rg] = C[(cl + 16 * mj + fr + 4 * rg) * ldc + ri + 16 * mi + fc];
    double fa[2][QG][2], fb[2][QG][2];  // [buffer][k-step][16-block]
    auto load = [&](int buf, int g) {
#pragma unroll
        for (int s = 0; s < QG; ++s) {
            const int64_t col = (int64_t)(g * 4 * QG + 4 * s + fr) * ldp;
            fb[buf][s][0] = P[col];
            fb[buf][s][1] = P[col + 16];
            fa[buf][s][0] = Q[col];
            fa[buf][s][1] = Q[col + 16];
        }
    };
    auto compute = [&](int buf) {
#pragma unroll
        for (int s = 0; s < QG; ++s) {
            const double b0 = -fb[buf][s][0], b1 = -fb[buf][s][1];
            acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[buf][s][0], b0, acc[0][0], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[buf][s][0], b1, acc[1][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[buf][s][1], b0, acc[0][1], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[buf][s][1], b1, acc[1][1], 0, 0, 0);
        }
    };
    const int ng = kdepth / (4 * QG);  // 4 per 128 panel columns
    load(0, 0);
    for (int g = 0; g < ng; g += 2) {
        if (g + 1 < ng) load(1, g + 1);
        compute(0);
        if (g + 1 < ng) {
            if (g + 2 < ng) load(0, g + 2);
            compute(1);
        }
    }
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int mj = 0; mj < 2; ++mj)
#pragma unroll
            for (int rg = 0; rg < 4; ++rg)
                C[(cl + 16 * mj + fr + 4 * rg) * ldc + ri + 16 * mi + fc] = acc[mi][mj][rg];
}

// Column update (critical path): tiles i >= jb of the global tile columns jb0 ..
// jb0+ncols-1, stored in local tile columns lj0 .. lj0+ncols-1 (one super-panel: its
// columns are contiguous in storage), K = kdepth panel columns.
__global__ __launch_bounds__(256) void col_update_kernel(double* __restrict__ C, int64_t ldc, Panel pn,
                                                         int jb0, int lj0, int m0, int kdepth,
                                                         KTime* __restrict__ kt) {
    kt_begin(kt);
    __builtin_amdgcn_s_setprio(2);
    const int q = (int)blockIdx.x & 3;
    int t = (int)blockIdx.x >> 2, c = 0;
    for (int mc = m0; t >= mc && mc > 0; --mc) {  // tile column jb0 + c holds m0 - c tiles
        t -= mc;
        ++c;
    }
    const int jb = jb0 + c, bi = jb + t, qi = q >> 1, qj = q & 1;
    if (!(bi == jb && qj > qi)) quad_update(C, ldc, pn, bi, jb, lj0 + c, qi, qj, kdepth);
    kt_end(kt);
}

// Small bulk trailing updates: the same tile list as tile_syrk_kernel, four quadrant
// workgroups per tile (XCD-chunked like the tile kernel).
__global__ __launch_bounds__(256) void quad_bulk_kernel(BulkArgs a, KTime* __restrict__ kt) {
    kt_begin(kt);
    const int b = (int)blockIdx.x >> 2, q = (int)blockIdx.x & 3;
    const int chunk = (a.ntiles + 7) >> 3;
    const int idx = (b & 7) * chunk + (b >> 3);
    if (idx < a.ntiles) {
        int bi, bj, lj;
        tile_decode(a, idx, bi, bj, lj);
        const int qi = q >> 1, qj = q & 1;
        if (!(bi == bj && qj > qi)) quad_update(a.C, a.ldc, a.pn, bi, bj, lj, qi, qj, a.kdepth);
    }
    kt_end(kt);
}

// ---------------------------------------------------------------------------------
// logdet / quad / logpdf (AbstractGPs.logpdf: -((N*log2pi + logdet) + quad) / 2).
// Fixed-order tree reduction: deterministic across runs.
// ---------------------------------------------------------------------------------
// Storage columns e = 0 .. ncols-1 hold global columns cm.global(e / NB) * NB + e % NB;
// only those < N contribute. With the identity map this is the whole-matrix reduction;
// on a distributed rank it is that rank's partial logdet / quad (summed across ranks by
// the host; res->logpdf then only holds this rank's share).
// Two launches, both with a fixed summation order (deterministic): REDUCE_BLOCKS
// workgroups each sum a contiguous range of columns (the loads are scattered, one cache
// line each, so spreading them over many CUs is what makes this fast), then one wave sums
// the partials in order.
__global__ __launch_bounds__(256) void reduce_partial_kernel(const double* __restrict__ C, int64_t ldc,
                                                             int64_t N, int64_t ncols, ColMap cm,
                                                             EvalResult* __restrict__ res) {
    __shared__ double s1[256], s2[256];
    const int tid = threadIdx.x;
    const int64_t per = (ncols + REDUCE_BLOCKS - 1) / REDUCE_BLOCKS;
    const int64_t e_lo = (int64_t)blockIdx.x * per;
    const int64_t e_hi = e_lo + per < ncols ? e_lo + per : ncols;
    double ld = 0.0, q = 0.0;
    for (int64_t e = e_lo + tid; e < e_hi; e += 256) {
        const int64_t j = (int64_t)cm.global((int)(e / NB)) * NB + e % NB;
        if (j < N) {
            ld += log(C[e * ldc + j]);
            const double z = C[e * ldc + N];
            q += z * z;
        }
    }
    s1[tid] = ld;
    s2[tid] = q;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if (tid < st) {
            s1[tid] += s1[tid + st];
            s2[tid] += s2[tid + st];
        }
        __syncthreads();
    }
    if (tid == 0) {
        res->part[0][blockIdx.x] = s1[0];
        res->part[1][blockIdx.x] = s2[0];
    }
}

__global__ __launch_bounds__(64) void reduce_final_kernel(int64_t N, EvalResult* __restrict__ res) {
    if (threadIdx.x != 0) return;
    double s1 = 0.0, s2 = 0.0;
    for (int b = 0; b < REDUCE_BLOCKS; ++b) {
        s1 += res->part[0][b];
        s2 += res->part[1][b];
    }
    const double logdet = s1 + s1;
    const double quad = s2;
    const double log2pi = 1.8378770664093453;  // Julia's log2π
    double lp = -(((double)N * log2pi + logdet) + quad) / 2.0;
    if (res->info != ~0ull) lp = __builtin_nan("");
    res->logdet = logdet;
    res->quad = quad;
    res->logpdf = lp;
}

__global__ void kt_reset_kernel(KTime* kt, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        kt[i].start = ~0ull;
        kt[i].end = 0ull;
    }
}

void launch_kt_reset(hipStream_t s, KTime* kt, int n) {
    if (n > 0 && guard_launch("kt_reset_kernel")) kt_reset_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s>>>(kt, n);
}

__global__ void init_result_kernel(EvalResult* res) {
    res->logpdf = 0.0;
    res->logdet = 0.0;
    res->quad = 0.0;
    res->info = ~0ull;
}

// ---------------------------------------------------------------------------------
// Gradient of logpdf: the factorisation also runs
// over identity rows E = [I 0] stored below the matrix (rows Np .. 2Np-1, lda = 2 Np),
// which leaves Y = E L^{-T} = L^{-T} there (upper triangular). Then
//   alpha = C^{-1} v = Y z                                        (alpha_*_kernel)
//   C^{-1} = Y Y^T,   tile (I, J), I >= J: sum_{k >= I NB} Y_Ik Y_Jk^T  (grad_tile_kernel)
//   dlogp/dtheta = 1/2 sum_ij (alpha_i alpha_j - Cinv_ij) dC_ij/dtheta
// with dC/dtheta evaluated on the fly from X (never stored), for every term parameter at
// once, and tile partial sums reduced in a fixed order (deterministic).
// ---------------------------------------------------------------------------------

// Identity rows: tiles (E, J) with E <= J get I on E == J and 0 elsewhere; tiles below the
// diagonal inside a super-panel's columns (J < E, same super-panel of W tile columns) are
// zeroed too: the super-panel's bulk update reads them as panel rows. The other tiles below
// the diagonal are never read.
__global__ __launch_bounds__(256) void init_identity_rows_kernel(double* __restrict__ A, int64_t lda,
                                                                 int64_t Np, int W) {
    const int J = (int)blockIdx.x, E = (int)blockIdx.y;
    if (E > J && E / W != J / W) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    double* base = A + (int64_t)J * NB * lda + Np + (int64_t)E * NB + 2 * lane;
    for (int c = w; c < NB; c += 4) {
        double2 o = make_double2(0.0, 0.0);
        if (E == J) {
            o.x = (2 * lane == c) ? 1.0 : 0.0;
            o.y = (2 * lane + 1 == c) ? 1.0 : 0.0;
        }
        *reinterpret_cast<double2*>(base + (int64_t)c * lda) = o;
    }
}

// Y[:, N .. Np) = 0 (columns of the v row and of the padding).
__global__ __launch_bounds__(256) void zero_tail_cols_kernel(double* __restrict__ A, int64_t lda, int64_t Np,
                                                             int64_t N) {
    const int64_t col = N + blockIdx.y;
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (col < Np && r < Np) A[col * lda + Np + r] = 0.0;
}

// alpha partial sums: block (x, y) = rows 256x .. 256x+255, columns 512y .. 512y+511.
__global__ __launch_bounds__(256) void alpha_partial_kernel(const double* __restrict__ A, int64_t lda,
                                                            int64_t Np, int64_t N, double* __restrict__ partial) {
    __shared__ double zs[512];
    const int tid = threadIdx.x;
    const int64_t k0 = (int64_t)blockIdx.y * 512;
    const int64_t i = (int64_t)blockIdx.x * 256 + tid;
    for (int t = tid; t < 512; t += 256) zs[t] = (k0 + t < N) ? A[(k0 + t) * lda + N] : 0.0;
    __syncthreads();
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    // Y is upper triangular: only columns k >= i are read (the tiles below the identity
    // rows' diagonal are never written and hold stale data)
    if (i < N && k0 + 512 > i) {
        const double* y = A + k0 * lda + Np + i;
        const int kn = (int)((N - k0) < 512 ? (N - k0) : 512);
        int kk = i > k0 ? (int)(i - k0) : 0;
        for (; kk + 4 <= kn; kk += 4) {
            s0 += y[(int64_t)kk * lda] * zs[kk];
            s1 += y[(int64_t)(kk + 1) * lda] * zs[kk + 1];
            s2 += y[(int64_t)(kk + 2) * lda] * zs[kk + 2];
            s3 += y[(int64_t)(kk + 3) * lda] * zs[kk + 3];
        }
        for (; kk < kn; ++kk) s0 += y[(int64_t)kk * lda] * zs[kk];
    }
    if (i < N) partial[(int64_t)blockIdx.y * N + i] = (s0 + s1) + (s2 + s3);
}

__global__ __launch_bounds__(256) void alpha_reduce_kernel(const double* __restrict__ partial, int64_t N, int nk,
                                                           double* __restrict__ alpha, double* __restrict__ dv) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    double a = 0.0;
    for (int y = 0; y < nk; ++y) a += partial[(int64_t)y * N + i];
    alpha[i] = a;
    dv[i] = -a;
}

// K_t(i, j) and dK_t/dparam_t(i, j) with the Gram kernel's arithmetic (p = 1/l for
// SqExp / OU: the coordinate is scaled first, then differenced).
__device__ __forceinline__ double term_k(int kind, double p, double xi, double xj, bool diag) {
#pragma clang fp contract(off)
    switch (kind) {
        case GAPLAC_SQEXP: {
            const double u = p * xi - p * xj;
            return exp(-(u * u) * 0.5);
        }
        case GAPLAC_OU:
            return exp(-fabs(p * xi - p * xj));
        case GAPLAC_LINEAR:
            return xi * xj + p;
        case GAPLAC_CAT:
            return (xi == xj) ? 1.0 : 0.0;
        default:
            return diag ? p : 0.0;
    }
}
__device__ __forceinline__ double term_dk(int kind, double p, double xi, double xj, bool diag) {
#pragma clang fp contract(off)
    switch (kind) {
        case GAPLAC_SQEXP: {  // d/dl exp(-u^2/2), u = (x_i - x_j)/l:  k u^2 / l
            const double u = p * xi - p * xj;
            const double u2 = u * u;
            return exp(-u2 * 0.5) * u2 * p;
        }
        case GAPLAC_OU: {  // d/dl exp(-|u|): k |u| / l
            const double a = fabs(p * xi - p * xj);
            return exp(-a) * a * p;
        }
        case GAPLAC_LINEAR:  // d/dc (x_i x_j + c)
            return 1.0;
        case GAPLAC_CAT:
            return 0.0;
        default:  // NOISE term: d/dvariance
            return diag ? 1.0 : 0.0;
    }
}

// -C^{-1} tile (I, J), I >= J, into the (no longer needed) factor storage:
// A[I, J] = -sum_{k >= I NB} Y_Ik Y_Jk^T. list[b] = I | J << 16 (0xffffffff = idle).
__global__ __launch_bounds__(256, 2) void cinv_tile_kernel(double* __restrict__ A, int64_t lda, int64_t Np,
                                                           const uint32_t* __restrict__ list,
                                                           KTime* __restrict__ kt) {
    kt_begin(kt);
    const uint32_t e = list[blockIdx.x];
    if (e != 0xffffffffu) {
        const int I = (int)(e & 0xffffu), J = (int)(e >> 16);
        const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
        const int wi = w & 1, wj = w >> 1;
        const int fr = lane >> 4, fc = lane & 15;
        const int64_t k0 = (int64_t)I * NB;
        const double* Y = A + Np;
        const bool active = !(I == J && wj > wi);
        d4 acc[4][4];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int mj = 0; mj < 4; ++mj) acc[mi][mj] = d4{0.0, 0.0, 0.0, 0.0};
        tile_mma_neg(Y + k0 * lda + (int64_t)I * NB, Y + k0 * lda + (int64_t)J * NB, lda, (int)(Np - k0), active,
                     acc);
        if (active) {
            double* Ct = A + (int64_t)J * NB * lda + (int64_t)I * NB;
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) {
                double* Ci = Ct + 64 * wi + 16 * mi + fc;
#pragma unroll
                for (int mj = 0; mj < 4; ++mj)
#pragma unroll
                    for (int rg = 0; rg < 4; ++rg)
                        Ci[(int64_t)(64 * wj + 16 * mj + fr + 4 * rg) * lda] = acc[mi][mj][rg];
            }
        }
    }
    kt_end(kt);
}

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

// Contraction of one lower tile (I, J) of M = -C^{-1} (in A) with every dC/dtheta:
//   partial[tile][t] = sum_{(i,j) in tile, i >= j, i,j < N} wt_ij (alpha_i alpha_j + M_ij) dC_ij/dtheta_t
// (wt = 2 off the diagonal: the symmetric pair), t = T: the observation variance
// (dC/dnoise = I). Same lane layout as the Gram kernel: two rows per lane, column
// coordinates staged in LDS.
__global__ __launch_bounds__(256) void grad_contract_kernel(const double* __restrict__ A, int64_t lda, int64_t N,
                                                            const double* __restrict__ X, int64_t ldx,
                                                            const double* __restrict__ alpha,
                                                            const TermPack* __restrict__ tpp,
                                                            const GradTermPack* __restrict__ gpp,
                                                            double* __restrict__ partial, KTime* __restrict__ kt) {
    kt_begin(kt);
    __shared__ double xcol[GAPLAC_MAX_TERMS][NB];
    __shared__ double acol[NB];
    __shared__ double red[4][GAPLAC_MAX_TERMS + 1];
    const TermPack& tp = *tpp;
    const int T = tp.T;
    int I, J;
    tri_index(blockIdx.x, I, J);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t c0 = (int64_t)J * NB;
    for (int idx = tid; idx < T * NB; idx += 256) {
        const int t = idx / NB, c = idx % NB;
        const int64_t j = c0 + c;
        xcol[t][c] = (j < N && tp.kind[t] != GAPLAC_NOISE) ? X[(int64_t)tp.col[t] * ldx + j] : 0.0;
    }
    if (tid < NB) acol[tid] = (c0 + tid < N) ? alpha[c0 + tid] : 0.0;
    const int64_t i0 = (int64_t)I * NB + 2 * lane;
    double xa[GAPLAC_MAX_TERMS], xb[GAPLAC_MAX_TERMS];
#pragma unroll
    for (int t = 0; t < GAPLAC_MAX_TERMS; ++t) {
        xa[t] = 0.0;
        xb[t] = 0.0;
        if (t < T && tp.kind[t] != GAPLAC_NOISE) {
            const double* xc = X + (int64_t)tp.col[t] * ldx;
            if (i0 < N) xa[t] = xc[i0];
            if (i0 + 1 < N) xb[t] = xc[i0 + 1];
        }
    }
    const double ai0 = i0 < N ? alpha[i0] : 0.0, ai1 = i0 + 1 < N ? alpha[i0 + 1] : 0.0;
    double g[GAPLAC_MAX_TERMS + 1];
#pragma unroll
    for (int t = 0; t <= GAPLAC_MAX_TERMS; ++t) g[t] = 0.0;
    __syncthreads();
    const double* Mt = A + c0 * lda + i0;
    for (int cc = w; cc < NB; cc += 4) {
        const int64_t j = c0 + cc;
        if (j >= N) break;
        const double2 m = *reinterpret_cast<const double2*>(Mt + (int64_t)cc * lda);
        const double aj = acol[cc];
        const double wt0 = (i0 < N && i0 >= j) ? (i0 == j ? 1.0 : 2.0) : 0.0;
        const double wt1 = (i0 + 1 < N && i0 + 1 >= j) ? (i0 + 1 == j ? 1.0 : 2.0) : 0.0;
        const double w0 = wt0 * (ai0 * aj + m.x), w1 = wt1 * (ai1 * aj + m.y);
        if (i0 == j) g[GAPLAC_MAX_TERMS] += w0;
        if (i0 + 1 == j) g[GAPLAC_MAX_TERMS] += w1;
#pragma unroll
        for (int t = 0; t < GAPLAC_MAX_TERMS; ++t) {
            if (t < T) {
                const int kind = tp.kind[t];
                const double p = tp.p[t], xj = xcol[t][cc];
                double d0 = term_dk(kind, p, xa[t], xj, i0 == j);
                double d1 = term_dk(kind, p, xb[t], xj, i0 + 1 == j);
                const int gs = gpp->gstart[t], ge = gpp->gend[t];
                if (ge - gs > 1) {  // product-group extension: times the group's other terms
#pragma unroll
                    for (int s2 = 0; s2 < GAPLAC_MAX_TERMS; ++s2) {
                        if (s2 >= gs && s2 < ge && s2 != t) {
                            const double y = xcol[s2][cc];
                            d0 *= term_k(tp.kind[s2], tp.p[s2], xa[s2], y, i0 == j);
                            d1 *= term_k(tp.kind[s2], tp.p[s2], xb[s2], y, i0 + 1 == j);
                        }
                    }
                }
                g[t] += w0 * d0 + w1 * d1;
            }
        }
    }
    // fixed-order reduction: wave butterflies, then the 4 waves in order
#pragma unroll
    for (int t = 0; t <= GAPLAC_MAX_TERMS; ++t) {
        const double x = wave_sum(g[t]);
        if (lane == 0) red[w][t] = x;
    }
    __syncthreads();
    if (tid <= T) {
        const int t = tid == T ? GAPLAC_MAX_TERMS : tid;
        partial[(int64_t)blockIdx.x * (T + 1) + tid] = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
    }
    kt_end(kt);
}

// out[t] = 1/2 sum_b partial[b][t], t = 0..T, fixed order.
__global__ __launch_bounds__(256) void grad_reduce_kernel(const double* __restrict__ partial, int nb, int T,
                                                          double* __restrict__ out) {
    __shared__ double s[256];
    const int t = blockIdx.x, tid = threadIdx.x;
    double x = 0.0;
    for (int b = tid; b < nb; b += 256) x += partial[(int64_t)b * (T + 1) + t];
    s[tid] = x;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (tid < o) s[tid] += s[tid + o];
        __syncthreads();
    }
    if (tid == 0) out[t] = 0.5 * s[0];
}

// ---------------------------------------------------------------------------------
// Posterior mean / variance at test points (AbstractGPs
// mean_and_var(posterior(fx, y), xs)): the rows below the matrix hold K(xs, X) (one row per
// test point); factoring them along leaves V^T = K(xs, X) L^{-T} there, so
//   mean_j = sum_k V^T[j,k] z_k          (= K(xs, X) C^{-1} y, z = L^{-1} y in row N)
//   var_j  = k(xs_j, xs_j) - sum_k V^T[j,k]^2
// ---------------------------------------------------------------------------------

// Cross-covariance rows: tile (E, J) of the extra rows = K(xs rows E NB.., X columns J NB..),
// no noise (the posterior's cross-covariance is the latent kernel); 0 outside j < M, i < N.
__global__ __launch_bounds__(256) void cross_gram_kernel(double* __restrict__ A, int64_t lda, int64_t Np,
                                                         int64_t N, int64_t M, const double* __restrict__ X,
                                                         int64_t ldx, const double* __restrict__ Xs,
                                                         int64_t ldxs, const TermPack* __restrict__ tpp) {
    __shared__ double xcol[GAPLAC_MAX_TERMS][NB];
    const TermPack& tp = *tpp;
    const int T = tp.T;
    const int J = (int)blockIdx.x, E = (int)blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t c0 = (int64_t)J * NB;
    for (int idx = tid; idx < T * NB; idx += 256) {
        const int t = idx / NB, c = idx % NB;
        xcol[t][c] = (c0 + c < N && tp.kind[t] != GAPLAC_NOISE) ? X[(int64_t)tp.col[t] * ldx + c0 + c] : 0.0;
    }
    const int64_t j0 = (int64_t)E * NB + 2 * lane;  // test points j0, j0 + 1
    double xa[GAPLAC_MAX_TERMS], xb[GAPLAC_MAX_TERMS];
#pragma unroll
    for (int t = 0; t < GAPLAC_MAX_TERMS; ++t) {
        xa[t] = 0.0;
        xb[t] = 0.0;
        if (t < T && tp.kind[t] != GAPLAC_NOISE) {
            const double* xc = Xs + (int64_t)tp.col[t] * ldxs;
            if (j0 < M) xa[t] = xc[j0];
            if (j0 + 1 < M) xb[t] = xc[j0 + 1];
        }
    }
    __syncthreads();
    double* base = A + c0 * lda + Np + j0;
    for (int cc = w; cc < NB; cc += 4) {
        double tot0 = 0.0, tot1 = 0.0, pr0 = 1.0, pr1 = 1.0;
#pragma unroll
        for (int t = 0; t < GAPLAC_MAX_TERMS; ++t) {
            if (t < T) {
                const int kind = tp.kind[t];
                const double p = tp.p[t], xj = xcol[t][cc];
                // an index-noise term couples a point only with itself: 0 across point sets
                pr0 *= kind == GAPLAC_NOISE ? 0.0 : term_k(kind, p, xa[t], xj, false);
                pr1 *= kind == GAPLAC_NOISE ? 0.0 : term_k(kind, p, xb[t], xj, false);
                if (tp.last_in_group[t]) {
                    tot0 += pr0;
                    tot1 += pr1;
                    pr0 = 1.0;
                    pr1 = 1.0;
                }
            }
        }
        const bool colok = c0 + cc < N;
        const double o0 = (colok && j0 < M) ? tot0 : 0.0, o1 = (colok && j0 + 1 < M) ? tot1 : 0.0;
        *reinterpret_cast<double2*>(base + (int64_t)cc * lda) = make_double2(o0, o1);
    }
}

// Partial sums over 512-column chunks of the extra rows: pm = V^T z, pv = |V^T|^2.
__global__ __launch_bounds__(256) void post_partial_kernel(const double* __restrict__ A, int64_t lda, int64_t Np,
                                                           int64_t N, int64_t M, double* __restrict__ pm,
                                                           double* __restrict__ pv) {
    __shared__ double zs[512];
    const int tid = threadIdx.x;
    const int64_t k0 = (int64_t)blockIdx.y * 512;
    const int64_t j = (int64_t)blockIdx.x * 256 + tid;
    for (int t = tid; t < 512; t += 256) zs[t] = (k0 + t < N) ? A[(k0 + t) * lda + N] : 0.0;
    __syncthreads();
    double m0 = 0.0, m1 = 0.0, v0 = 0.0, v1 = 0.0;
    if (j < M) {
        const double* y = A + k0 * lda + Np + j;
        const int kn = (int)((N - k0) < 512 ? (N - k0) : 512);
        int kk = 0;
        for (; kk + 2 <= kn; kk += 2) {
            const double a = y[(int64_t)kk * lda], b = y[(int64_t)(kk + 1) * lda];
            m0 += a * zs[kk];
            m1 += b * zs[kk + 1];
            v0 += a * a;
            v1 += b * b;
        }
        for (; kk < kn; ++kk) {
            const double a = y[(int64_t)kk * lda];
            m0 += a * zs[kk];
            v0 += a * a;
        }
        pm[(int64_t)blockIdx.y * M + j] = m0 + m1;
        pv[(int64_t)blockIdx.y * M + j] = v0 + v1;
    }
}

// mean_j, var_j = kdiag(xs_j) - sum of the partials (fixed order).
__global__ __launch_bounds__(256) void post_finish_kernel(const double* __restrict__ pm,
                                                          const double* __restrict__ pv, int64_t M, int nk,
                                                          const double* __restrict__ Xs, int64_t ldxs,
                                                          const TermPack* __restrict__ tpp,
                                                          double* __restrict__ mean, double* __restrict__ var) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= M) return;
    const TermPack& tp = *tpp;
    double kd = 0.0, pr = 1.0;
    for (int t = 0; t < tp.T; ++t) {
        const int kind = tp.kind[t];
        const double x = kind == GAPLAC_NOISE ? 0.0 : Xs[(int64_t)tp.col[t] * ldxs + j];
        pr *= term_k(kind, tp.p[t], x, x, true);
        if (tp.last_in_group[t]) {
            kd += pr;
            pr = 1.0;
        }
    }
    double m = 0.0, v = 0.0;
    for (int y = 0; y < nk; ++y) {
        m += pm[(int64_t)y * M + j];
        v += pv[(int64_t)y * M + j];
    }
    mean[j] = m;
    var[j] = kd - v;
}

// ---------------------------------------------------------------------------------
// rand(FiniteGP) (AbstractGPs: m + cholesky(C).U' * randn): out = L z
// over the factor's lower triangle (k <= i: the diagonal tiles' upper parts hold junk).
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void lower_mv_partial_kernel(const double* __restrict__ A, int64_t lda,
                                                               int64_t N, const double* __restrict__ z,
                                                               double* __restrict__ partial) {
    __shared__ double zs[512];
    const int tid = threadIdx.x;
    const int64_t k0 = (int64_t)blockIdx.y * 512;
    const int64_t i = (int64_t)blockIdx.x * 256 + tid;
    for (int t = tid; t < 512; t += 256) zs[t] = (k0 + t < N) ? z[k0 + t] : 0.0;
    __syncthreads();
    if (i >= N) return;
    double s0 = 0.0, s1 = 0.0;
    if (k0 <= i) {
        const double* l = A + k0 * lda + i;
        const int64_t kmax = i + 1 - k0;  // k <= i
        const int kn = (int)(kmax < 512 ? kmax : 512);
        int kk = 0;
        for (; kk + 2 <= kn; kk += 2) {
            s0 += l[(int64_t)kk * lda] * zs[kk];
            s1 += l[(int64_t)(kk + 1) * lda] * zs[kk + 1];
        }
        for (; kk < kn; ++kk) s0 += l[(int64_t)kk * lda] * zs[kk];
    }
    partial[(int64_t)blockIdx.y * N + i] = s0 + s1;
}

__global__ __launch_bounds__(256) void lower_mv_reduce_kernel(const double* __restrict__ partial, int64_t N, int nk,
                                                              double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    double a = 0.0;
    for (int y = 0; y < nk; ++y) a += partial[(int64_t)y * N + i];
    out[i] = a;
}

// ------------------------------- launchers ---------------------------------------
// Every launcher first passes the element range its grid will touch to guard_launch
// (gaplac_internal.h): derived from the same tile counts / decodes the
// kernel uses, so a wrong grid (the round-1 part-2 Gram count for N < 255) is caught on
// the host instead of writing past the allocation.
LaunchGuard*& current_guard() {
    static thread_local LaunchGuard* g = nullptr;
    return g;
}

bool guard_launch(const char* what, const double* p, int64_t lo, int64_t hi) {
    LaunchGuard* g = current_guard();
    if (!g) return true;
    ++g->launches;
    if (g->base) {
        const int64_t off = (int64_t)(((intptr_t)p - (intptr_t)g->base) / (intptr_t)sizeof(double));
        if (lo > hi || off + lo < 0 || off + hi > g->elems) {
            if (g->violations++ == 0) {
                char buf[200];
                snprintf(buf, sizeof buf, "%s touches elements [%lld, %lld) of a %lld-element workspace", what,
                         (long long)(off + lo), (long long)(off + hi), (long long)g->elems);
                g->first = buf;
            }
            return false;
        }
    }
    return !g->dry;
}

bool guard_launch(const char* what) {
    (void)what;
    LaunchGuard* g = current_guard();
    if (!g) return true;
    ++g->launches;
    return !g->dry;
}

// End (exclusive) of the elements a set of tiles with rows <= max_bi, columns <= max_bj
// touches in column storage with leading dimension ld.
static int64_t tiles_end(int64_t ld, int64_t max_bi, int64_t max_bj) {
    return ((max_bj + 1) * NB - 1) * ld + (max_bi + 1) * NB;
}

// Largest b with b (b + 1) / 2 <= t (the row tri_index decodes for workgroup t).
static int64_t tri_row(int64_t t) {
    if (t <= 0) return 0;
    int64_t b = (int64_t)((std::sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while ((b + 1) * (b + 2) / 2 <= t) ++b;
    while (b * (b + 1) / 2 > t) --b;
    return b;
}

void launch_gram(hipStream_t s, double* A, int64_t lda, int64_t N, int nt, const double* X,
                 int64_t ldx, const double* v, const TermPack* dtp, int part, int w, KTime* kt) {
    int64_t ntiles, max_bi, max_bj;
    if (part == 1) {
        w = w < nt ? w : nt;
        ntiles = 0;
        for (int c = 0; c < w; ++c) ntiles += nt - c;
        max_bi = nt - 1;
        max_bj = w - 1;
    } else {
        if (part == 0) w = 0;
        const int64_t m = nt - w;  // part 2 with nt <= w: nothing left (m <= 0)
        ntiles = m > 0 ? m * (m + 1) / 2 : 0;
        max_bi = max_bj = ntiles > 0 ? w + tri_row(ntiles - 1) : 0;
    }
    if (ntiles <= 0) return;
    if (!guard_launch("gram_kernel", A, 0, tiles_end(lda, max_bi, max_bj))) return;
    gram_kernel<<<dim3((unsigned)ntiles), dim3(256), 0, s>>>(A, lda, N, X, ldx, v, dtp, nt, part, w, kt);
}

void launch_gram_list(hipStream_t s, double* C, int64_t ldc, int64_t N, const double* X, int64_t ldx,
                      const double* v, const TermPack* dtp, const uint32_t* tiles, int ntiles, ColMap cm,
                      int max_bi, int max_lj, KTime* kt) {
    if (ntiles <= 0) return;
    if (!guard_launch("gram_list_kernel", C, 0, tiles_end(ldc, max_bi, max_lj))) return;
    gram_list_kernel<<<dim3((unsigned)ntiles), dim3(256), 0, s>>>(C, ldc, N, X, ldx, v, dtp, tiles, cm, kt);
}

void launch_potrf_diag(hipStream_t s, double* Ablk, int64_t lda, int64_t N, int64_t g0, double* Dinv,
                       EvalResult* res, KTime* kt) {
    if (!guard_launch("potrf_diag_kernel", Ablk, 0, tiles_end(lda, 0, 0))) return;
    potrf_diag_kernel<<<dim3(1), dim3(256), 0, s>>>(Ablk, lda, N, g0, Dinv, res, kt);
}

void launch_trsm(hipStream_t s, double* Acol, int64_t lda, int nt, int k, const double* Dinv, KTime* kt) {
    const int n = nt - k - 1;
    if (n <= 0) return;
    if (!guard_launch("trsm_subst_kernel", Acol, 0, tiles_end(lda, nt - 1, 0))) return;
    trsm_subst_kernel<<<dim3(2 * n), dim3(256), 0, s>>>(Acol, lda, k, k + 1, Dinv, kt);
}

void launch_trsm_rows(hipStream_t s, double* Acol, int64_t lda, int k, int bi0, int nrows, const double* Dinv,
                      KTime* kt) {
    if (nrows <= 0) return;
    if (!guard_launch("trsm_subst_kernel (rows)", Acol, 0, tiles_end(lda, std::max(k, bi0 + nrows - 1), 0))) return;
    trsm_subst_kernel<<<dim3(2 * nrows), dim3(256), 0, s>>>(Acol, lda, k, bi0, Dinv, kt);
}

bool syrk_is_small(int ntiles) { return ntiles <= QUAD_BULK_MAX_TILES; }

// Bulk kernel choice (GAPLAC_BULK8, read once): 0 = the 4-wave tile kernel, two workgroups
// per CU (default); 1 = 8-wave tile kernel, one workgroup per CU beside one chain
// workgroup; 2 = the same, persistent (one workgroup per CU walking its tiles). Measured
// at N=16384: 31.5 / 32.5 / 35.2 ms per evaluation — the chain kernels co-reside under 1
// and 2 but still run 2-4x slower beside MFMA-saturating bulk waves.
static int bulk8_mode() {
    static const int m = [] {
        const char* s = std::getenv("GAPLAC_BULK8");
        return s ? std::atoi(s) : 0;
    }();
    return m;
}

static int device_cus() {
    static const int n = [] {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        return (cus + 7) & ~7;
    }();
    return n;
}

void launch_bulk(hipStream_t s, const BulkArgs& a, KTime* kt) {
    if (a.ntiles <= 0) return;
    int64_t max_r, max_c;
    if (a.rect_rows > 0) {
        max_r = a.rect_rows - 1;
        max_c = a.ntiles / a.rect_rows - 1;
    } else if (a.max_r >= 0) {
        max_r = a.max_r;
        max_c = a.max_c;
    } else {
        max_r = max_c = tri_row(a.ntiles - 1);  // an m x m triangle list: entries < m
    }
    if (!guard_launch("bulk update", a.C, 0, tiles_end(a.ldc, a.bi0 + max_r, a.lj0 + max_c))) return;
    int grid = ((a.ntiles + 7) >> 3) << 3;
    if (syrk_is_small(a.ntiles)) {
        quad_bulk_kernel<<<dim3((unsigned)(4 * grid)), dim3(256), 0, s>>>(a, kt);
    } else if (bulk8_mode()) {
        if (bulk8_mode() == 2) grid = std::min(grid, device_cus());
        tile_syrk8_kernel<<<dim3((unsigned)grid), dim3(512), 0, s>>>(a, kt);
    } else
        tile_syrk_kernel<<<dim3((unsigned)grid), dim3(256), 0, s>>>(a, kt);
}

void launch_col_update(hipStream_t s, double* C, int64_t ldc, const Panel& pn, int nt, int jb, int lj0,
                       int ncols, int kdepth, KTime* kt) {
    const int m0 = nt - jb;
    if (m0 <= 0 || ncols <= 0) return;
    int tiles = 0;
    for (int c = 0; c < ncols && c < m0; ++c) tiles += m0 - c;
    if (!guard_launch("col_update_kernel", C, 0, tiles_end(ldc, nt - 1, lj0 + std::min(ncols, m0) - 1))) return;
    col_update_kernel<<<dim3((unsigned)(4 * tiles)), dim3(256), 0, s>>>(C, ldc, pn, jb, lj0, m0, kdepth, kt);
}

// Super-tile ordered list of the lower-triangular m x m tile set (entry = bi | bj << 16,
// relative to the first tile block): 8x8 super-tiles, super-rows outer, tiles row-major.
void build_tile_list(int m, uint32_t* out) {
    int n = 0;
    for (int I = 0; I < (m + 7) / 8; ++I)
        for (int J = 0; J <= I; ++J)
            for (int i = 8 * I; i < 8 * I + 8 && i < m; ++i)
                for (int j = 8 * J; j < 8 * J + 8 && j <= i; ++j)
                    out[n++] = (uint32_t)i | ((uint32_t)j << 16);
}

void launch_reduce(hipStream_t s, const double* C, int64_t ldc, int64_t N, int64_t ncols, ColMap cm,
                   EvalResult* res) {
    if (ncols <= 0 || !guard_launch("reduce_partial_kernel", C, 0, (ncols - 1) * ldc + N + 1)) return;
    reduce_partial_kernel<<<dim3(REDUCE_BLOCKS), dim3(256), 0, s>>>(C, ldc, N, ncols, cm, res);
    reduce_final_kernel<<<dim3(1), dim3(64), 0, s>>>(N, res);
}

void launch_init_identity_rows(hipStream_t s, double* A, int64_t lda, int64_t Np, int nt, int W) {
    if (nt <= 0) return;
    if (!guard_launch("init_identity_rows_kernel", A, 0, ((int64_t)nt * NB - 1) * lda + Np + (int64_t)nt * NB)) return;
    init_identity_rows_kernel<<<dim3((unsigned)nt, (unsigned)nt), dim3(256), 0, s>>>(A, lda, Np, W);
}

void launch_zero_tail_cols(hipStream_t s, double* A, int64_t lda, int64_t Np, int64_t N) {
    if (Np <= N) return;
    if (!guard_launch("zero_tail_cols_kernel", A, N * lda, (Np - 1) * lda + 2 * Np)) return;
    zero_tail_cols_kernel<<<dim3((unsigned)((Np + 255) / 256), (unsigned)(Np - N)), dim3(256), 0, s>>>(A, lda, Np, N);
}

void launch_alpha(hipStream_t s, const double* A, int64_t lda, int64_t Np, int64_t N, double* partial,
                  double* alpha, double* dv) {
    if (N <= 0) return;
    if (!guard_launch("alpha_partial_kernel", A, 0, (N - 1) * lda + Np + N)) return;
    const int nk = (int)((N + 511) / 512);
    alpha_partial_kernel<<<dim3((unsigned)((N + 255) / 256), (unsigned)nk), dim3(256), 0, s>>>(A, lda, Np, N,
                                                                                             partial);
    alpha_reduce_kernel<<<dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s>>>(partial, N, nk, alpha, dv);
}

void launch_cinv_tiles(hipStream_t s, double* A, int64_t lda, int64_t Np, const uint32_t* list, int nblocks, int m,
                       KTime* kt) {
    if (nblocks <= 0) return;
    if (!guard_launch("cinv_tile_kernel", A, 0, (Np - 1) * lda + Np + (int64_t)m * NB)) return;
    cinv_tile_kernel<<<dim3((unsigned)nblocks), dim3(256), 0, s>>>(A, lda, Np, list, kt);
}

void launch_grad_contract(hipStream_t s, const double* A, int64_t lda, int64_t N, const double* X, int64_t ldx,
                          const double* alpha, const TermPack* dtp, const GradTermPack* dgp, double* partial,
                          KTime* kt) {
    const int m = (int)((N + NB - 1) / NB);
    const int64_t tiles = (int64_t)m * (m + 1) / 2;
    if (tiles <= 0) return;
    if (!guard_launch("grad_contract_kernel", A, 0, tiles_end(lda, m - 1, m - 1))) return;
    grad_contract_kernel<<<dim3((unsigned)tiles), dim3(256), 0, s>>>(A, lda, N, X, ldx, alpha, dtp, dgp, partial,
                                                                     kt);
}

void launch_grad_reduce(hipStream_t s, const double* partial, int nb, int T, double* out) {
    if (!guard_launch("grad_reduce_kernel")) return;
    grad_reduce_kernel<<<dim3((unsigned)(T + 1)), dim3(256), 0, s>>>(partial, nb, T, out);
}

// Lower m x m tile triangle in 8x8 super-tiles, super-rows first (deepest Y products
// first: tile (I, J) contracts over Np - I NB columns); super-tile s goes to XCD s % 8
// (the dispatcher deals workgroup b to XCD b % 8), so every XCD gets a share of the deep
// tiles and its resident tiles share 8 + 8 panel row blocks in its L2.
void build_grad_list(int m, std::vector<uint32_t>& out) {
    std::vector<std::vector<uint32_t>> seq(8);
    int st = 0;
    for (int I = 0; I < (m + 7) / 8; ++I)
        for (int J = 0; J <= I; ++J, ++st) {
            std::vector<uint32_t>& q = seq[(size_t)(st & 7)];
            for (int i = 8 * I; i < 8 * I + 8 && i < m; ++i)
                for (int j = 8 * J; j < 8 * J + 8 && j <= i; ++j) q.push_back((uint32_t)i | ((uint32_t)j << 16));
        }
    size_t len = 0;
    for (const auto& q : seq) len = std::max(len, q.size());
    out.assign(8 * len, 0xffffffffu);
    for (size_t x = 0; x < 8; ++x)
        for (size_t k = 0; k < seq[x].size(); ++k) out[8 * k + x] = seq[x][k];
}

void launch_cross_gram(hipStream_t s, double* A, int64_t lda, int64_t Np, int nt, int64_t N, int64_t M, int mt,
                       const double* X, int64_t ldx, const double* Xs, int64_t ldxs, const TermPack* dtp) {
    if (nt <= 0 || mt <= 0) return;
    if (!guard_launch("cross_gram_kernel", A, 0, ((int64_t)nt * NB - 1) * lda + Np + (int64_t)mt * NB)) return;
    cross_gram_kernel<<<dim3((unsigned)nt, (unsigned)mt), dim3(256), 0, s>>>(A, lda, Np, N, M, X, ldx, Xs, ldxs, dtp);
}

void launch_posterior(hipStream_t s, const double* A, int64_t lda, int64_t Np, int64_t N, int64_t M,
                      const double* Xs, int64_t ldxs, const TermPack* dtp, double* partial, double* mean,
                      double* var) {
    if (M <= 0) return;
    if (!guard_launch("post_partial_kernel", A, 0, (N - 1) * lda + Np + M)) return;
    const int nk = (int)((N + 511) / 512);
    double* pm = partial;
    double* pv = partial + (size_t)nk * M;
    post_partial_kernel<<<dim3((unsigned)((M + 255) / 256), (unsigned)nk), dim3(256), 0, s>>>(A, lda, Np, N, M, pm,
                                                                                            pv);
    post_finish_kernel<<<dim3((unsigned)((M + 255) / 256)), dim3(256), 0, s>>>(pm, pv, M, nk, Xs, ldxs, dtp, mean,
                                                                             var);
}

void launch_lower_mv(hipStream_t s, const double* A, int64_t lda, int64_t N, const double* z, double* partial,
                     double* out) {
    if (N <= 0) return;
    if (!guard_launch("lower_mv_partial_kernel", A, 0, (N - 1) * lda + N)) return;
    const int nk = (int)((N + 511) / 512);
    lower_mv_partial_kernel<<<dim3((unsigned)((N + 255) / 256), (unsigned)nk), dim3(256), 0, s>>>(A, lda, N, z,
                                                                                                partial);
    lower_mv_reduce_kernel<<<dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s>>>(partial, N, nk, out);
}

void launch_init_result(hipStream_t s, EvalResult* res) {
    if (!guard_launch("init_result_kernel")) return;
    init_result_kernel<<<dim3(1), dim3(1), 0, s>>>(res);
}

}  // namespace gaplac
