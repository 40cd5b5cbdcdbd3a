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
//   tile_gemm_kernel   fp64 MFMA (v_mfma_f64_16x16x4f64) 128x128 tiles: trailing SYRK
//                      update (C -= P Q^T) and panel TRSM (P <- P Linv^T)
//   reduce_kernel      logdet = 2 sum log L_jj, quad = ||z||^2, logpdf
#include "gaplac_internal.h"
#include <math.h>

namespace gaplac {

typedef double d4 __attribute__((ext_vector_type(4)));

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
__global__ __launch_bounds__(256) void gram_kernel(double* __restrict__ A, int64_t lda,
                                                   int64_t N, const double* __restrict__ X,
                                                   int64_t ldx, const double* __restrict__ v,
                                                   TermPack tp, double noise) {
    int bi, bj;
    tri_index(blockIdx.x, bi, bj);
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
        *reinterpret_cast<double2*>(A + j * lda + i0) = make_double2(o0, o1);
    }
}

// ---------------------------------------------------------------------------------
// Diagonal block: right-looking Cholesky of the 128x128 block fused with the forward
// elimination that yields Linv = L_kk^{-1} (used to turn the panel TRSM into an MFMA
// GEMM). Runs alone on CUs reserved for it (CU-masked stream, gaplac_api.hip).
// Register-resident: 1024 threads = a 32 x 32 grid of 4x4 micro-tiles, t = cb*32 + rb:
//   rb >= cb : A micro-tile (rb, cb)                    (a[][])
//   cb >= rb : R micro-tile (cb, rb) of the RHS, R0 = I  (w[][]); after the elimination
//              row j of R scaled by 1/L_jj is row j of L^{-1}.
// Wave w holds column blocks 2w and 2w+1, so every owner of column j (and of row j of R)
// sits in wave (j/4)/2 and a wave whose column blocks are finished stops computing.
// Column j: the owning wave takes the pivot (sqrt, 1/d, LAPACK dpotf2's scaling), scales
// column j and R's row j and publishes both, zero-padded, in a double-buffered LDS
// vector; one barrier; every active wave applies the rank-1 update unconditionally
// (the zero padding masks finished rows/columns). Pivots of padding columns (>= N) are
// forced to 1; a failing pivot (<= 0 or NaN) records info = j+1.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void potrf_diag_kernel(double* __restrict__ A, int64_t lda,
                                                          int64_t N, int k,
                                                          double* __restrict__ Linv,
                                                          EvalResult* __restrict__ res) {
    __shared__ double colj[2][NB];
    __shared__ double rowj[2][NB];
    const int t = threadIdx.x;
    const int cb = t >> 5, rb = t & 31, lane = t & 63;
    const bool ownA = rb >= cb, ownR = cb >= rb;
    const int64_t g0 = (int64_t)k * NB;
    double* Ab = A + g0 * lda + g0;
    double a[4][4], w[4][4];
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            a[i][x] = ownA ? Ab[(int64_t)(4 * cb + x) * lda + 4 * rb + i] : 0.0;
            w[i][x] = (rb == cb && i == x) ? 1.0 : 0.0;
        }
    for (int j = 0; j < NB; ++j) {
        const int jb = j >> 2, jj = j & 3, p = j & 1;
        if ((t >> 6) == (jb >> 1)) {  // the wave owning column j: pivot, scale, publish
            const int plane = (jb & 1) * 32 + jb;
            double piv = 0.0;
#pragma unroll
            for (int x = 0; x < 4; ++x)
                if (x == jj) piv = a[x][x];
            piv = __shfl(piv, plane);
            double d, rd;
            if (g0 + j >= N) {
                d = 1.0;
                rd = 1.0;
            } else {
                if (lane == plane && !(piv > 0.0))
                    atomicMin(&res->info, (unsigned long long)(g0 + j + 1));
                d = sqrt(piv);
                rd = 1.0 / d;
            }
            if (cb == jb) {
#pragma unroll
                for (int x = 0; x < 4; ++x) {
                    if (x != jj) continue;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int r = 4 * rb + i;
                        const double sc = a[i][x] * rd;
                        colj[p][r] = (r > j) ? sc : 0.0;
                        a[i][x] = (r > j) ? sc : ((r == j) ? d : a[i][x]);
                    }
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    if (i != jj) continue;
#pragma unroll
                    for (int x = 0; x < 4; ++x) {
                        const double sc = w[i][x] * rd;
                        w[i][x] = sc;
                        rowj[p][4 * rb + x] = ownR ? sc : 0.0;
                    }
                }
            }
        }
        __syncthreads();
        if (2 * (t >> 6) + 1 >= jb) {
            const double2 r01 = *reinterpret_cast<const double2*>(&colj[p][4 * rb]);
            const double2 r23 = *reinterpret_cast<const double2*>(&colj[p][4 * rb + 2]);
            const double2 c01 = *reinterpret_cast<const double2*>(&colj[p][4 * cb]);
            const double2 c23 = *reinterpret_cast<const double2*>(&colj[p][4 * cb + 2]);
            const double2 w01 = *reinterpret_cast<const double2*>(&rowj[p][4 * rb]);
            const double2 w23 = *reinterpret_cast<const double2*>(&rowj[p][4 * rb + 2]);
            const double cr[4] = {r01.x, r01.y, r23.x, r23.y};
            const double cc[4] = {c01.x, c01.y, c23.x, c23.y};
            const double rw[4] = {w01.x, w01.y, w23.x, w23.y};
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int x = 0; x < 4; ++x) {
                    a[i][x] -= cr[i] * cc[x];
                    w[i][x] -= cc[i] * rw[x];
                }
        }
    }
    // L block (lower incl. diagonal) back in place; Linv = R (column-major, ld NB).
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = 4 * rb + i, c = 4 * cb + x;
            if (ownA && r >= c) Ab[(int64_t)c * lda + r] = a[i][x];
            // R micro-tile (cb, rb): Linv rows 4cb+i, cols 4rb+x; threads with rb > cb
            // own no R tile and zero the mirrored upper block instead.
            Linv[(4 * rb + x) * NB + 4 * cb + i] = ownR ? w[i][x] : 0.0;
        }
}

// ---------------------------------------------------------------------------------
// 128x128 fp64 MFMA tile kernel, K = NB = 128 (one panel).
//   MODE 0 (SYRK): C(bi,bj) -= P_bi * P_bj^T, P = panel block column k.
//   MODE 1 (TRSM): P_bi <- P_bi * Linv^T (in place), bi > k.
// 256 threads = 4 waves as 2x2, each wave a 64x64 sub-tile = 4x4 v_mfma_f64_16x16x4f64
// accumulators. Operands are staged through LDS in 16-deep k-chunks, double-buffered
// with a register prefetch of the next chunk. The MFMA computes D = Q*P^T (the j-side
// fragment is the A operand) so that a lane's accumulator column is C's row: stores are
// 128-byte column segments of the column-major matrix. In SYRK mode the C tile is loaded
// straight into the accumulators before the k-loop and P is staged negated, so the MFMA
// chain produces C - P Q^T and the epilogue is stores only.
// Tile placement: a precomputed list (tiles) maps blockIdx -> (bi, bj). For the bulk
// trailing update the list is ordered so that the blocks one XCD runs (blockIdx % 8,
// dealt round-robin by the dispatcher) walk one contiguous run of 8x8 super-tiles: the
// P/Q row blocks of its ~64 resident tiles (2 MiB) stay in that XCD's 4 MiB L2.
// Placement only affects speed; any blockIdx -> tile bijection is correct.
// ---------------------------------------------------------------------------------
constexpr int KB = 16;
constexpr int LR = NB + 16;  // LDS k-row stride: lanes 16..31 land on banks 32..63

template <int MODE>
__global__ __launch_bounds__(256, 2) void tile_gemm_kernel(double* __restrict__ A, int64_t lda,
                                                           int k, int jb, int colmode,
                                                           const double* __restrict__ Linv,
                                                           const uint32_t* __restrict__ tiles,
                                                           int ntiles) {
    __shared__ double sm[2][2][KB][LR];
    int bi, bj;
    if (MODE == 1) {
        bi = k + 1 + (int)blockIdx.x;
        bj = k;
    } else if (colmode) {
        bi = jb + (int)blockIdx.x;
        bj = jb;
    } else {
        const int b = (int)blockIdx.x;
        const int chunk = (ntiles + 7) >> 3;
        const int idx = (b & 7) * chunk + (b >> 3);
        if (idx >= ntiles) return;
        const uint32_t tv = tiles[idx];
        bi = jb + (int)(tv & 0xffffu);
        bj = jb + (int)(tv >> 16);
    }
    const int64_t r0 = (int64_t)bi * NB, c0 = (int64_t)bj * NB, k0 = (int64_t)k * NB;
    const double* P = A + k0 * lda + r0;
    const double* Q;
    int64_t ldq;
    if (MODE == 1) {
        Q = Linv;
        ldq = NB;
    } else {
        Q = A + k0 * lda + c0;
        ldq = lda;
    }
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wi = w & 1, wj = w >> 1;
    const bool active = !(MODE == 0 && bi == bj && wj > wi);
    const int fr = lane >> 4, fc = lane & 15;

    d4 acc[4][4];
    if (MODE == 0 && active) {
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
            const double* Ci = A + c0 * lda + r0 + 64 * wi + 16 * mi + fc;
#pragma unroll
            for (int mj = 0; mj < 4; ++mj)
#pragma unroll
                for (int rg = 0; rg < 4; ++rg)
                    acc[mi][mj][rg] = Ci[(int64_t)(64 * wj + 16 * mj + fr + 4 * rg) * lda];
        }
    } else {
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
    }

    double2 pp[4], pq[4];
    const int krow = tid >> 6;  // 0..3
    auto gload = [&](int ch) {
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int64_t col = (int64_t)ch * KB + krow + 4 * it;
            pp[it] = *reinterpret_cast<const double2*>(P + col * lda + 2 * lane);
            pq[it] = *reinterpret_cast<const double2*>(Q + col * ldq + 2 * lane);
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int kk = krow + 4 * it;
            double2 v = pp[it];
            if (MODE == 0) {
                v.x = -v.x;
                v.y = -v.y;
            }
            *reinterpret_cast<double2*>(&sm[buf][0][kk][2 * lane]) = v;
            *reinterpret_cast<double2*>(&sm[buf][1][kk][2 * lane]) = pq[it];
        }
    };

    gload(0);
    lstore(0);
    __syncthreads();
    constexpr int NCH = NB / KB;
    for (int ch = 0; ch < NCH; ++ch) {
        const int buf = ch & 1;
        if (ch + 1 < NCH) gload(ch + 1);
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
        if (ch + 1 < NCH) lstore(buf ^ 1);
        __syncthreads();
    }
    if (!active) return;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
        double* Ci = A + c0 * lda + r0 + 64 * wi + 16 * mi + fc;
#pragma unroll
        for (int mj = 0; mj < 4; ++mj)
#pragma unroll
            for (int rg = 0; rg < 4; ++rg)
                Ci[(int64_t)(64 * wj + 16 * mj + fr + 4 * rg) * lda] = acc[mi][mj][rg];
    }
}

// ---------------------------------------------------------------------------------
// logdet / quad / logpdf (AbstractGPs.logpdf: -((N*log2pi + logdet) + quad) / 2).
// Fixed-order tree reduction: deterministic across runs.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void reduce_kernel(const double* __restrict__ A, int64_t lda,
                                                      int64_t N, EvalResult* __restrict__ res) {
    __shared__ double s1[1024], s2[1024];
    const int tid = threadIdx.x;
    double ld = 0.0, q = 0.0;
    for (int64_t j = tid; j < N; j += 1024) {
        ld += log(A[j * lda + j]);
        const double z = A[j * lda + N];
        q += z * z;
    }
    s1[tid] = ld;
    s2[tid] = q;
    __syncthreads();
    for (int s = 512; s > 0; s >>= 1) {
        if (tid < s) {
            s1[tid] += s1[tid + s];
            s2[tid] += s2[tid + s];
        }
        __syncthreads();
    }
    if (tid == 0) {
        const double logdet = s1[0] + s1[0];
        const double quad = s2[0];
        const double log2pi = 1.8378770664093453;  // Julia's log2π
        double lp = -(((double)N * log2pi + logdet) + quad) / 2.0;
        if (res->info != ~0ull) lp = __builtin_nan("");
        res->logdet = logdet;
        res->quad = quad;
        res->logpdf = lp;
    }
}

__global__ void init_result_kernel(EvalResult* res) {
    res->logpdf = 0.0;
    res->logdet = 0.0;
    res->quad = 0.0;
    res->info = ~0ull;
}

// ------------------------------- launchers ---------------------------------------
void launch_gram(hipStream_t s, double* A, int64_t lda, int64_t N, int nt, const double* X,
                 int64_t ldx, const double* v, const TermPack& tp, double noise) {
    const int64_t ntiles = (int64_t)nt * (nt + 1) / 2;
    gram_kernel<<<dim3((unsigned)ntiles), dim3(256), 0, s>>>(A, lda, N, X, ldx, v, tp, noise);
}

void launch_potrf_diag(hipStream_t s, double* A, int64_t lda, int64_t N, int k, double* Linv,
                       EvalResult* res) {
    potrf_diag_kernel<<<dim3(1), dim3(1024), 0, s>>>(A, lda, N, k, Linv, res);
}

void launch_trsm(hipStream_t s, double* A, int64_t lda, int nt, int k, const double* Linv) {
    const int n = nt - k - 1;
    if (n <= 0) return;
    tile_gemm_kernel<1><<<dim3(n), dim3(256), 0, s>>>(A, lda, k, 0, 0, Linv, nullptr, 0);
}

void launch_syrk(hipStream_t s, double* A, int64_t lda, int nt, int k, int jb, int colmode,
                 const uint32_t* tiles) {
    const int m = nt - jb;
    if (m <= 0) return;
    if (colmode) {
        tile_gemm_kernel<0><<<dim3((unsigned)m), dim3(256), 0, s>>>(A, lda, k, jb, 1, nullptr, nullptr, 0);
        return;
    }
    const int ntiles = m * (m + 1) / 2;
    const int grid = ((ntiles + 7) >> 3) << 3;
    tile_gemm_kernel<0><<<dim3((unsigned)grid), dim3(256), 0, s>>>(A, lda, k, jb, 0, nullptr, tiles, ntiles);
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

void launch_reduce(hipStream_t s, const double* A, int64_t lda, int64_t N, EvalResult* res) {
    reduce_kernel<<<dim3(1), dim3(1024), 0, s>>>(A, lda, N, res);
}

void launch_init_result(hipStream_t s, EvalResult* res) {
    init_result_kernel<<<dim3(1), dim3(1), 0, s>>>(res);
}

}  // namespace gaplac
