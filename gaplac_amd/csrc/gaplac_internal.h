// Internal declarations shared by the HIP kernels (gaplac_kernels.hip) and the host
// orchestration (gaplac_api.hip). Not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
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
struct EvalResult {
    double logpdf;
    double logdet;
    double quad;
    unsigned long long info;  // min over failing pivots of (j+1); ULLONG_MAX = none
};

// Per-launch device timestamps (profiling): 100 MHz s_memrealtime ticks.
struct KTime {
    unsigned long long start;  // min over workgroups (init ~0)
    unsigned long long end;    // max over waves (init 0)
};

// Launchers (gaplac_kernels.hip). Every launcher takes a KTime slot (nullptr = off).
// A is the Np x Np column-major augmented matrix
// (lda = Np, Np = roundup(N+1, NB)): rows/cols 0..N-1 hold C, row N holds v^T.
// part 0: all lower tiles; part 1: the first w tile columns; part 2: tiles with both
// block indices >= w (parts 1 + 2 = part 0).
void launch_gram(hipStream_t s, double* A, int64_t lda, int64_t N, int nt,
                 const double* X, int64_t ldx, const double* v, const TermPack* dtp, int part, int w,
                 KTime* kt);
// Diagonal block k: L_kk in place + Dinv (DINV_ELEMS doubles: 8 column-major 16x16
// inverses of L_kk's diagonal sub-blocks).
void launch_potrf_diag(hipStream_t s, double* A, int64_t lda, int64_t N, int k,
                       double* Dinv, EvalResult* res, KTime* kt);
// TRSM of the panel rows below diagonal block k: A[i,k] <- A[i,k] * L_kk^{-T}, i>k.
void launch_trsm(hipStream_t s, double* A, int64_t lda, int nt, int k, const double* Dinv, KTime* kt);
// Bulk trailing update: lower triangle of tile blocks jb..nt-1 minus the kdepth columns
// starting at tile column k (kdepth 128 or 256). tiles: super-tile ordered list for the
// m x m triangle, m = nt - jb (build_tile_list).
// valu: 1 = v_fma_f64 register-tile kernel, 0 = fp64 MFMA kernel.
void launch_syrk(hipStream_t s, double* A, int64_t lda, int nt, int k, int jb, int kdepth,
                 const uint32_t* tiles, int valu, KTime* kt);
// True when launch_syrk over an m x m tile triangle runs the small (quadrant) kernel.
bool syrk_is_small(int m);
// Lookahead update of tile columns jb (and jb+1 if ncols == 2) with the kdepth columns
// starting at tile column k.
void launch_col_update(hipStream_t s, double* A, int64_t lda, int nt, int k, int jb, int ncols,
                       int kdepth, KTime* kt);
void build_tile_list(int m, uint32_t* out);
void launch_reduce(hipStream_t s, const double* A, int64_t lda, int64_t N, EvalResult* res);
void launch_kt_reset(hipStream_t s, KTime* kt, int n);
void launch_init_result(hipStream_t s, EvalResult* res);

}  // namespace gaplac
