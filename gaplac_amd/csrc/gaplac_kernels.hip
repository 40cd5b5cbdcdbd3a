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
#include <functional>
#include <queue>
#include <type_traits>
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
// exp(x) for the Gram kernel's arguments (x = -u^2/2 or -|u|, so x <= 0), table-driven:
// x = (256 k + j) ln2/256 + r with |r| <~ ln2/512, exp(x) = 2^k 2^(j/256) (1 + p(r)),
// p the degree-4 Taylor polynomial of exp(r) - 1 (truncation r^5/120 < 4e-17).
// n = round(x 256/ln2) comes from the low word of x 256/ln2 + 1.5 2^52 (one fma; the
// nearest integer to the exact product, so |r| may exceed ln2/512 by an ulp's worth),
// ln2/256 is split Cody-Waite style into a 33-bit head (n * head exact for |n| < 2^20)
// and a tail. 2^(j/256) is correctly rounded from a 60-digit evaluation (decimal module).
// Within 1 ulp of the library exp (tools/exp_probe.hip, 2^27 points per range) at ~15
// instead of ~30 VALU instructions: the multi-term Gram build is VALU-bound on its exps.
// Results below 2^-1074 flush to 0 (x < -745.2); NaN propagates.
// ---------------------------------------------------------------------------------
__constant__ double kExp2Tbl256[256] = {
    0x1.0000000000000p+0, 0x1.00b1afa5abcbfp+0, 0x1.0163da9fb3335p+0, 0x1.02168143b0281p+0,
    0x1.02c9a3e778061p+0, 0x1.037d42e11bbccp+0, 0x1.04315e86e7f85p+0, 0x1.04e5f72f654b1p+0,
    0x1.059b0d3158574p+0, 0x1.0650a0e3c1f89p+0, 0x1.0706b29ddf6dep+0, 0x1.07bd42b72a836p+0,
    0x1.0874518759bc8p+0, 0x1.092bdf66607e0p+0, 0x1.09e3ecac6f383p+0, 0x1.0a9c79b1f3919p+0,
    0x1.0b5586cf9890fp+0, 0x1.0c0f145e46c85p+0, 0x1.0cc922b7247f7p+0, 0x1.0d83b23395decp+0,
    0x1.0e3ec32d3d1a2p+0, 0x1.0efa55fdfa9c5p+0, 0x1.0fb66affed31bp+0, 0x1.1073028d7233ep+0,
    0x1.11301d0125b51p+0, 0x1.11edbab5e2ab6p+0, 0x1.12abdc06c31ccp+0, 0x1.136a814f204abp+0,
    0x1.1429aaea92de0p+0, 0x1.14e95934f312ep+0, 0x1.15a98c8a58e51p+0, 0x1.166a45471c3c2p+0,
    0x1.172b83c7d517bp+0, 0x1.17ed48695bbc0p+0, 0x1.18af9388c8deap+0, 0x1.1972658375d2fp+0,
    0x1.1a35beb6fcb75p+0, 0x1.1af99f8138a1cp+0, 0x1.1bbe084045cd4p+0, 0x1.1c82f95281c6bp+0,
    0x1.1d4873168b9aap+0, 0x1.1e0e75eb44027p+0, 0x1.1ed5022fcd91dp+0, 0x1.1f9c18438ce4dp+0,
    0x1.2063b88628cd6p+0, 0x1.212be3578a819p+0, 0x1.21f49917ddc96p+0, 0x1.22bdda27912d1p+0,
    0x1.2387a6e756238p+0, 0x1.2451ffb82140ap+0, 0x1.251ce4fb2a63fp+0, 0x1.25e85711ece75p+0,
    0x1.26b4565e27cddp+0, 0x1.2780e341ddf29p+0, 0x1.284dfe1f56381p+0, 0x1.291ba7591bb70p+0,
    0x1.29e9df51fdee1p+0, 0x1.2ab8a66d10f13p+0, 0x1.2b87fd0dad990p+0, 0x1.2c57e39771b2fp+0,
    0x1.2d285a6e4030bp+0, 0x1.2df961f641589p+0, 0x1.2ecafa93e2f56p+0, 0x1.2f9d24abd886bp+0,
    0x1.306fe0a31b715p+0, 0x1.31432edeeb2fdp+0, 0x1.32170fc4cd831p+0, 0x1.32eb83ba8ea32p+0,
    0x1.33c08b26416ffp+0, 0x1.3496266e3fa2dp+0, 0x1.356c55f929ff1p+0, 0x1.36431a2de883bp+0,
    0x1.371a7373aa9cbp+0, 0x1.37f26231e754ap+0, 0x1.38cae6d05d866p+0, 0x1.39a401b7140efp+0,
    0x1.3a7db34e59ff7p+0, 0x1.3b57fbfec6cf4p+0, 0x1.3c32dc313a8e5p+0, 0x1.3d0e544ede173p+0,
    0x1.3dea64c123422p+0, 0x1.3ec70df1c5175p+0, 0x1.3fa4504ac801cp+0, 0x1.40822c367a024p+0,
    0x1.4160a21f72e2ap+0, 0x1.423fb2709468ap+0, 0x1.431f5d950a897p+0, 0x1.43ffa3f84b9d4p+0,
    0x1.44e086061892dp+0, 0x1.45c2042a7d232p+0, 0x1.46a41ed1d0057p+0, 0x1.4786d668b3237p+0,
    0x1.486a2b5c13cd0p+0, 0x1.494e1e192aed2p+0, 0x1.4a32af0d7d3dep+0, 0x1.4b17dea6db7d7p+0,
    0x1.4bfdad5362a27p+0, 0x1.4ce41b817c114p+0, 0x1.4dcb299fddd0dp+0, 0x1.4eb2d81d8abffp+0,
    0x1.4f9b2769d2ca7p+0, 0x1.508417f4531eep+0, 0x1.516daa2cf6642p+0, 0x1.5257de83f4eefp+0,
    0x1.5342b569d4f82p+0, 0x1.542e2f4f6ad27p+0, 0x1.551a4ca5d920fp+0, 0x1.56070dde910d2p+0,
    0x1.56f4736b527dap+0, 0x1.57e27dbe2c4cfp+0, 0x1.58d12d497c7fdp+0, 0x1.59c0827ff07ccp+0,
    0x1.5ab07dd485429p+0, 0x1.5ba11fba87a03p+0, 0x1.5c9268a5946b7p+0, 0x1.5d84590998b93p+0,
    0x1.5e76f15ad2148p+0, 0x1.5f6a320dceb71p+0, 0x1.605e1b976dc09p+0, 0x1.6152ae6cdf6f4p+0,
    0x1.6247eb03a5585p+0, 0x1.633dd1d1929fdp+0, 0x1.6434634ccc320p+0, 0x1.652b9febc8fb7p+0,
    0x1.6623882552225p+0, 0x1.671c1c70833f6p+0, 0x1.68155d44ca973p+0, 0x1.690f4b19e9538p+0,
    0x1.6a09e667f3bcdp+0, 0x1.6b052fa75173ep+0, 0x1.6c012750bdabfp+0, 0x1.6cfdcddd47645p+0,
    0x1.6dfb23c651a2fp+0, 0x1.6ef9298593ae5p+0, 0x1.6ff7df9519484p+0, 0x1.70f7466f42e87p+0,
    0x1.71f75e8ec5f74p+0, 0x1.72f8286ead08ap+0, 0x1.73f9a48a58174p+0, 0x1.74fbd35d7cbfdp+0,
    0x1.75feb564267c9p+0, 0x1.77024b1ab6e09p+0, 0x1.780694fde5d3fp+0, 0x1.790b938ac1cf6p+0,
    0x1.7a11473eb0187p+0, 0x1.7b17b0976cfdbp+0, 0x1.7c1ed0130c132p+0, 0x1.7d26a62ff86f0p+0,
    0x1.7e2f336cf4e62p+0, 0x1.7f3878491c491p+0, 0x1.80427543e1a12p+0, 0x1.814d2add106d9p+0,
    0x1.82589994cce13p+0, 0x1.8364c1eb941f7p+0, 0x1.8471a4623c7adp+0, 0x1.857f4179f5b21p+0,
    0x1.868d99b4492edp+0, 0x1.879cad931a436p+0, 0x1.88ac7d98a6699p+0, 0x1.89bd0a478580fp+0,
    0x1.8ace5422aa0dbp+0, 0x1.8be05bad61778p+0, 0x1.8cf3216b5448cp+0, 0x1.8e06a5e0866d9p+0,
    0x1.8f1ae99157736p+0, 0x1.902fed0282c8ap+0, 0x1.9145b0b91ffc6p+0, 0x1.925c353aa2fe2p+0,
    0x1.93737b0cdc5e5p+0, 0x1.948b82b5f98e5p+0, 0x1.95a44cbc8520fp+0, 0x1.96bdd9a7670b3p+0,
    0x1.97d829fde4e50p+0, 0x1.98f33e47a22a2p+0, 0x1.9a0f170ca07bap+0, 0x1.9b2bb4d53fe0dp+0,
    0x1.9c49182a3f090p+0, 0x1.9d674194bb8d5p+0, 0x1.9e86319e32323p+0, 0x1.9fa5e8d07f29ep+0,
    0x1.a0c667b5de565p+0, 0x1.a1e7aed8eb8bbp+0, 0x1.a309bec4a2d33p+0, 0x1.a42c980460ad8p+0,
    0x1.a5503b23e255dp+0, 0x1.a674a8af46052p+0, 0x1.a799e1330b358p+0, 0x1.a8bfe53c12e59p+0,
    0x1.a9e6b5579fdbfp+0, 0x1.ab0e521356ebap+0, 0x1.ac36bbfd3f37ap+0, 0x1.ad5ff3a3c2774p+0,
    0x1.ae89f995ad3adp+0, 0x1.afb4ce622f2ffp+0, 0x1.b0e07298db666p+0, 0x1.b20ce6c9a8952p+0,
    0x1.b33a2b84f15fbp+0, 0x1.b468415b749b1p+0, 0x1.b59728de5593ap+0, 0x1.b6c6e29f1c52ap+0,
    0x1.b7f76f2fb5e47p+0, 0x1.b928cf22749e4p+0, 0x1.ba5b030a1064ap+0, 0x1.bb8e0b79a6f1fp+0,
    0x1.bcc1e904bc1d2p+0, 0x1.bdf69c3f3a207p+0, 0x1.bf2c25bd71e09p+0, 0x1.c06286141b33dp+0,
    0x1.c199bdd85529cp+0, 0x1.c2d1cd9fa652cp+0, 0x1.c40ab5fffd07ap+0, 0x1.c544778fafb22p+0,
    0x1.c67f12e57d14bp+0, 0x1.c7ba88988c933p+0, 0x1.c8f6d9406e7b5p+0, 0x1.ca3405751c4dbp+0,
    0x1.cb720dcef9069p+0, 0x1.ccb0f2e6d1675p+0, 0x1.cdf0b555dc3fap+0, 0x1.cf3155b5bab74p+0,
    0x1.d072d4a07897cp+0, 0x1.d1b532b08c968p+0, 0x1.d2f87080d89f2p+0, 0x1.d43c8eacaa1d6p+0,
    0x1.d5818dcfba487p+0, 0x1.d6c76e862e6d3p+0, 0x1.d80e316c98398p+0, 0x1.d955d71ff6075p+0,
    0x1.da9e603db3285p+0, 0x1.dbe7cd63a8315p+0, 0x1.dd321f301b460p+0, 0x1.de7d5641c0658p+0,
    0x1.dfc97337b9b5fp+0, 0x1.e11676b197d17p+0, 0x1.e264614f5a129p+0, 0x1.e3b333b16ee12p+0,
    0x1.e502ee78b3ff6p+0, 0x1.e653924676d76p+0, 0x1.e7a51fbc74c83p+0, 0x1.e8f7977cdb740p+0,
    0x1.ea4afa2a490dap+0, 0x1.eb9f4867cca6ep+0, 0x1.ecf482d8e67f1p+0, 0x1.ee4aaa2188510p+0,
    0x1.efa1bee615a27p+0, 0x1.f0f9c1cb6412ap+0, 0x1.f252b376bba97p+0, 0x1.f3ac948dd7274p+0,
    0x1.f50765b6e4540p+0, 0x1.f6632798844f8p+0, 0x1.f7bfdad9cbe14p+0, 0x1.f91d802243c89p+0,
    0x1.fa7c1819e90d8p+0, 0x1.fbdba3692d514p+0, 0x1.fd3c22b8f71f1p+0, 0x1.fe9d96b2a23d9p+0};

__device__ __forceinline__ double exp_nonpos(double x, const double* __restrict__ tbl) {
    const double kd = fma(x, 0x1.71547652b82fep+8, 0x1.8p52);  // x * 256 / ln2 + 1.5 2^52
    const int n = (int)(uint32_t)__double_as_longlong(kd);
    const double nf = kd - 0x1.8p52;
    double r = fma(-nf, 0x1.62e42fee00000p-9, x);
    r = fma(-nf, 0x1.a39ef35793c76p-41, r);
    double p = fma(r, 1.0 / 24.0, 1.0 / 6.0);
    p = fma(p, r, 0.5);
    p = p * r;
    p = fma(p, r, r);  // exp(r) - 1
    const double t = tbl[n & 255];
    const double y = __builtin_ldexp(fma(t, p, t), n >> 8);
    return x < -745.2 ? 0.0 : y;
}

// threadIdx.x through an opaque copy: in the persistent kernel nothing derived from it is
// hoisted out of the task loop (LICM would keep every body's addresses live: spills)
__device__ __forceinline__ int otid() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

// ---------------------------------------------------------------------------------
// Gram term evaluation, specialised at compile time on the term kind and on how the term
// combines with its group (KernelProduct inside a group, KernelSum across groups):
//   GM_SUM_FIRST  singleton group, first group      tot  = k
//   GM_SUM        singleton group                   tot += k
//   GM_PR_FIRST   first term of a product group     pr   = k
//   GM_PR         inner term of a product group     pr  *= k
//   GM_PR_LAST0   last term, first group            tot  = pr * k
//   GM_PR_LAST    last term                         tot += pr * k
// which is the left fold tot = 0 + (1 * k1 * k2 ...) + ... without the exact no-op
// operations (1 * k = k, 0 + x = x): the same values, ~2 VALU instructions per element
// and term fewer for the common all-singleton formulas (configs[2]: SqExp + OU + Cat).
// ---------------------------------------------------------------------------------
enum GramMode { GM_SUM_FIRST, GM_SUM, GM_PR_FIRST, GM_PR, GM_PR_LAST0, GM_PR_LAST };
#ifndef GAPLAC_GRAM_CB
#define GAPLAC_GRAM_CB 4
#endif
constexpr int GRAM_CB = GAPLAC_GRAM_CB;  // tile columns per batch and wave

template <int KIND>
__device__ __forceinline__ double gram_term(double xi, double xj, double p, int64_t i, int64_t j,
                                            const double* __restrict__ etbl) {
#pragma clang fp contract(off)
    if constexpr (KIND == GAPLAC_SQEXP) {
        const double d = xi - xj;  // coordinates pre-scaled by (1/l)/sqrt(2)
        return exp_nonpos(-(d * d), etbl);
    } else if constexpr (KIND == GAPLAC_OU) {
        return exp_nonpos(-fabs(xi - xj), etbl);
    } else if constexpr (KIND == GAPLAC_LINEAR) {
        return xi * xj + p;
    } else if constexpr (KIND == GAPLAC_CAT) {
        return (xi == xj) ? 1.0 : 0.0;
    } else {  // GAPLAC_NOISE: index identity
        return (i == j) ? p : 0.0;
    }
}

// A wave's batch: tile columns j0l + NW q, q < CB (NW: the workgroup's waves).
template <int KIND, int MODE, int CB, int NW = 4>
__device__ __forceinline__ void gram_batch(double (&tot0)[CB], double (&tot1)[CB],
                                           double (&pr0)[CB], double (&pr1)[CB],
                                           const double* __restrict__ xc, double2 xr, double p,
                                           int64_t i0, int64_t j0, const double* __restrict__ etbl) {
#pragma clang fp contract(off)
#pragma unroll
    for (int q = 0; q < CB; ++q) {
        const double xj = xc[NW * q];
        const int64_t j = j0 + NW * q;
        const double k0 = gram_term<KIND>(xr.x, xj, p, i0, j, etbl);
        const double k1 = gram_term<KIND>(xr.y, xj, p, i0 + 1, j, etbl);
        if constexpr (MODE == GM_SUM_FIRST) { tot0[q] = k0; tot1[q] = k1; }
        else if constexpr (MODE == GM_SUM) { tot0[q] += k0; tot1[q] += k1; }
        else if constexpr (MODE == GM_PR_FIRST) { pr0[q] = k0; pr1[q] = k1; }
        else if constexpr (MODE == GM_PR) { pr0[q] *= k0; pr1[q] *= k1; }
        else if constexpr (MODE == GM_PR_LAST0) { tot0[q] = pr0[q] * k0; tot1[q] = pr1[q] * k1; }
        else { tot0[q] += pr0[q] * k0; tot1[q] += pr1[q] * k1; }
    }
}

template <int KIND, int CB, int NW = 4>
__device__ __forceinline__ void gram_batch_mode(int mode, double (&tot0)[CB], double (&tot1)[CB],
                                                double (&pr0)[CB], double (&pr1)[CB],
                                                const double* __restrict__ xc, double2 xr, double p,
                                                int64_t i0, int64_t j0, const double* __restrict__ etbl) {
    switch (mode) {
        case GM_SUM_FIRST: gram_batch<KIND, GM_SUM_FIRST, CB, NW>(tot0, tot1, pr0, pr1, xc, xr, p, i0, j0, etbl); break;
        case GM_SUM: gram_batch<KIND, GM_SUM, CB, NW>(tot0, tot1, pr0, pr1, xc, xr, p, i0, j0, etbl); break;
        case GM_PR_FIRST: gram_batch<KIND, GM_PR_FIRST, CB, NW>(tot0, tot1, pr0, pr1, xc, xr, p, i0, j0, etbl); break;
        case GM_PR: gram_batch<KIND, GM_PR, CB, NW>(tot0, tot1, pr0, pr1, xc, xr, p, i0, j0, etbl); break;
        case GM_PR_LAST0: gram_batch<KIND, GM_PR_LAST0, CB, NW>(tot0, tot1, pr0, pr1, xc, xr, p, i0, j0, etbl); break;
        default: gram_batch<KIND, GM_PR_LAST, CB, NW>(tot0, tot1, pr0, pr1, xc, xr, p, i0, j0, etbl); break;
    }
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
// NW = 8: the persistent tail's 512-thread workgroup builds a tile as a task (tail_kernel,
// TAIL_G): the same per-element arithmetic, eight waves taking every eighth column, the
// stores with the AUX cache policy (sc1: the tail's hand-off protocol).
// ---------------------------------------------------------------------------------
constexpr int GRAM_LDS = 2 * GAPLAC_MAX_TERMS * NB + NB + 256;  // doubles of LDS gram_tile works in

template <int CB = GRAM_CB, int NW = 4, int AUX = 0>
__device__ __forceinline__ void gram_tile(double* __restrict__ Ccol, int64_t lda, int64_t N,
                                          const double* __restrict__ X, int64_t ldx,
                                          const double* __restrict__ v,
                                          const TermPack* __restrict__ tpp, int bi, int bj, double* lds) {
    // Ccol: storage of global column bj*NB (row 0); rows are global
    // No FMA contraction: KernelFunctions scales each coordinate (rounded) and then
    // differences, so equal coordinates give exactly 0 (p*xa - p*xj fused would not).
#pragma clang fp contract(off)
    const TermPack& tp = *tpp;  // uniform: scalar loads (device copy refreshed per eval)
    const double noise = tp.noise;
    const int64_t r0 = (int64_t)bi * NB, c0 = (int64_t)bj * NB;
    // Coordinates of the tile's columns (xcol) and rows (xrow) per term, staged once.
    // SqExp / OU coordinates are stored already scaled (OU: p * x, rounded exactly as
    // KernelFunctions' ScaleTransform; SqExp: by p/sqrt(2), within an ulp of it);
    // Linear / Cat keep the raw coordinate.
    double (*xcol)[NB] = reinterpret_cast<double (*)[NB]>(lds);
    double (*xrow)[NB] = xcol + GAPLAC_MAX_TERMS;
    double* vcol = lds + 2 * GAPLAC_MAX_TERMS * NB;
    double* etbl = vcol + NB;
    static_assert(NW == 4 || NW == 8, "gram_tile: 4 or 8 waves");
    static_assert(NB % (NW * CB) == 0, "gram_tile: whole batches per wave");
    const int tid = NW == 4 ? (int)threadIdx.x : otid();
    const int T = tp.T;
    // Staging: thread tid owns coordinate slot c = tid % NB of the columns (tid < NB) or
    // the rows (tid >= NB); the term index is uniform (scalar TermPack loads) and every
    // global load is issued before the first one is consumed (one latency per tile).
    if (NW == 4 || tid < 2 * NB) {
        const int c = tid & (NB - 1);
        const bool is_row = tid >= NB;
        const int64_t j = (is_row ? r0 : c0) + c;
        const bool in = j < N;
        const double e = kExp2Tbl256[tid];
        const double vj = (!is_row && in) ? v[j] : 0.0;
        double val[GAPLAC_MAX_TERMS];
#pragma unroll
        for (int t = 0; t < GAPLAC_MAX_TERMS; ++t) {
            val[t] = 0.0;
            if (t < T && in && tp.kind[t] != GAPLAC_NOISE) val[t] = X[(int64_t)tp.col[t] * ldx + j];
        }
        etbl[tid] = e;
        if (!is_row) vcol[c] = vj;
        double (*dst)[NB] = is_row ? xrow : xcol;
#pragma unroll
        for (int t = 0; t < GAPLAC_MAX_TERMS; ++t) {
            if (t < T) {
                const int kind = tp.kind[t];
                // SqExp: scaled by (1/l)/sqrt(2), so the kernel is exp(-d^2) (one multiply
                // fewer per element; equal coordinates still give exactly d = 0).
                const double sc = kind == GAPLAC_SQEXP ? tp.p[t] * 0x1.6a09e667f3bcdp-1 : tp.p[t];
                dst[t][c] = (kind == GAPLAC_SQEXP || kind == GAPLAC_OU) ? sc * val[t] : val[t];
            }
        }
    }
    const int lane = tid & 63, w = tid >> 6;
    const int64_t i0 = r0 + 2 * lane, i1 = i0 + 1;
    __syncthreads();

    // Wave w: tile columns cc = w + NW (cb + q), in batches of CB columns. Kind and
    // group position are switched on once per term and batch (uniform branches); each
    // term gives 2 CB independent evaluations for the VALU pipeline to overlap.
    // Off the diagonal a singleton Noise group is all zeros and is skipped; interior
    // off-diagonal tiles (no padding row/column, no diagonal, no v row) store the sums
    // as they are. Formulas whose groups are all single terms (the common case) take a
    // path with one running sum and no group bookkeeping.
    const bool diag_tile = bi == bj;
    const bool plain = !diag_tile && r0 + NB <= N && c0 + NB <= N;
    bool all_single = true;
    for (int t = 0; t < T; ++t) all_single = all_single && tp.last_in_group[t];
    // Stores through a buffer resource over the tile's columns: the lane's row offset is
    // the voffset, the wave-uniform column offset the soffset (no per-store 64-bit address
    // arithmetic). The descriptor inputs are made provably uniform (readfirstlane).
    const int wu = __builtin_amdgcn_readfirstlane(w);
    const uint64_t tbase = (uint64_t)(Ccol + r0);
    const int64_t span = ((int64_t)(NB - 1) * lda + NB) * 8;
    const bool use_buf = span < ((int64_t)1 << 31);
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((uint64_t)__builtin_amdgcn_readfirstlane((unsigned)(tbase >> 32)) << 32) |
                (uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)tbase)),
        0, use_buf ? (int)span : 0, 0x00020000);
    static_assert(AUX == 0 || NW == 8, "gram_tile: a cache policy only for the tail's tiles");
    auto store2 = [&](int cc, double o0, double o1) {
#ifdef GAPLAC_GRAM_NOSTORE  // tools/gram_probe: compute-only timing (never true for real data)
        if (o0 != 1.2345e300) return;
#endif
        if (use_buf) {
            typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
            const double2 d = make_double2(o0, o1);
            u32x4 bits;
            __builtin_memcpy(&bits, &d, 16);
            __builtin_amdgcn_raw_buffer_store_b128(bits, rsrc, 16 * lane,
                                                   __builtin_amdgcn_readfirstlane((int)((int64_t)cc * lda * 8)), AUX);
        } else {
            *reinterpret_cast<double2*>(Ccol + (int64_t)cc * lda + i0) = make_double2(o0, o1);
        }
    };
    auto store_batch = [&](int j0l, const double (&tot0)[CB], const double (&tot1)[CB]) {
#pragma unroll
        for (int q = 0; q < CB; ++q) {
            const int cc = j0l + NW * q;
            const int64_t j = c0 + cc;
            double o0 = tot0[q], o1 = tot1[q];
            if (!plain) {
                if (j < N) {
                    o0 = (i0 < N) ? o0 + ((i0 == j) ? noise : 0.0) : ((i0 == N) ? vcol[cc] : 0.0);
                    o1 = (i1 < N) ? o1 + ((i1 == j) ? noise : 0.0) : ((i1 == N) ? vcol[cc] : 0.0);
                } else {
                    o0 = 0.0;
                    o1 = 0.0;
                }
            }
            store2(cc, o0, o1);
        }
    };
    if (all_single) {
        for (int cb = 0; cb < NB / NW; cb += CB) {
            double tot0[CB], tot1[CB], pr0[CB], pr1[CB];
#pragma unroll
            for (int q = 0; q < CB; ++q) tot0[q] = tot1[q] = 0.0;  // 0 + k = k
            const int j0l = wu + NW * cb;
            for (int t = 0; t < T; ++t) {
                const int kind = tp.kind[t];
                if (kind == GAPLAC_NOISE && !diag_tile) continue;
                const double p = tp.p[t];
                const double* xc = &xcol[t][j0l];
                const double2 xr = *reinterpret_cast<const double2*>(&xrow[t][2 * lane]);
                const int64_t j0 = c0 + j0l;
                switch (kind) {
                    case GAPLAC_SQEXP: gram_batch<GAPLAC_SQEXP, GM_SUM, CB, NW>(tot0, tot1, pr0, pr1, xc, xr, p, i0, j0, etbl); break;
                    case GAPLAC_OU: gram_batch<GAPLAC_OU, GM_SUM, CB, NW>(tot0, tot1, pr0, pr1, xc, xr, p, i0, j0, etbl); break;
                    case GAPLAC_LINEAR: gram_batch<GAPLAC_LINEAR, GM_SUM, CB, NW>(tot0, tot1, pr0, pr1, xc, xr, p, i0, j0, etbl); break;
                    case GAPLAC_CAT: gram_batch<GAPLAC_CAT, GM_SUM, CB, NW>(tot0, tot1, pr0, pr1, xc, xr, p, i0, j0, etbl); break;
                    default: gram_batch<GAPLAC_NOISE, GM_SUM, CB, NW>(tot0, tot1, pr0, pr1, xc, xr, p, i0, j0, etbl); break;
                }
            }
            store_batch(j0l, tot0, tot1);
        }
        return;
    }
    for (int cb = 0; cb < NB / NW; cb += CB) {
        double tot0[CB], tot1[CB], pr0[CB], pr1[CB];
        bool have_tot = false;
        const int j0l = wu + NW * cb;  // tile column of q = 0
        for (int t = 0; t < T; ++t) {
            const int kind = tp.kind[t];
            const bool first = t == 0 || tp.last_in_group[t - 1];
            const bool last = tp.last_in_group[t];
            if (kind == GAPLAC_NOISE && first && last && !diag_tile) continue;
            const int mode = first ? (last ? (have_tot ? GM_SUM : GM_SUM_FIRST) : GM_PR_FIRST)
                                   : (last ? (have_tot ? GM_PR_LAST : GM_PR_LAST0) : GM_PR);
            have_tot = have_tot || last;
            const double p = tp.p[t];
            const double* xc = &xcol[t][j0l];
            const double2 xr = *reinterpret_cast<const double2*>(&xrow[t][2 * lane]);
            const int64_t j0 = c0 + j0l;
            switch (kind) {
                case GAPLAC_SQEXP: gram_batch_mode<GAPLAC_SQEXP, CB, NW>(mode, tot0, tot1, pr0, pr1, xc, xr, p, i0, j0, etbl); break;
                case GAPLAC_OU: gram_batch_mode<GAPLAC_OU, CB, NW>(mode, tot0, tot1, pr0, pr1, xc, xr, p, i0, j0, etbl); break;
                case GAPLAC_LINEAR: gram_batch_mode<GAPLAC_LINEAR, CB, NW>(mode, tot0, tot1, pr0, pr1, xc, xr, p, i0, j0, etbl); break;
                case GAPLAC_CAT: gram_batch_mode<GAPLAC_CAT, CB, NW>(mode, tot0, tot1, pr0, pr1, xc, xr, p, i0, j0, etbl); break;
                default: gram_batch_mode<GAPLAC_NOISE, CB, NW>(mode, tot0, tot1, pr0, pr1, xc, xr, p, i0, j0, etbl); break;
            }
        }
        if (!have_tot) {
#pragma unroll
            for (int q = 0; q < CB; ++q) tot0[q] = tot1[q] = 0.0;
        }
        store_batch(j0l, tot0, tot1);
    }
}

// Single-GPU layout. part 1: the first w tile columns; part 2: the lower triangle of tile
// blocks w..nt-1; part 0: everything.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void gram_kernel(double* __restrict__ A, int64_t lda,
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
    __shared__ double glds[GRAM_LDS];
    gram_tile(A + (int64_t)bj * NB * lda, lda, N, X, ldx, v, tpp, bi, bj, glds);
    kt_end(kt);
}

// Second Gram launch as a work queue (head of the evaluation). The panel
// chain's first super-panel (diagonal block: 264 registers per wave and 75 KB of LDS;
// TRSM: 146 registers, 74 KB; column updates: up to ~1500 workgroups) runs beside this
// launch. A plain grid keeps four Gram workgroups on every CU and refills each freed slot
// with its next tile, so the chain waited for the whole launch to drain (a 35 us diagonal
// block took 389 us at N = 16384). Here a fixed number of workgroups per CU take tiles from
// a per-evaluation ticket (EvalResult::gram_ticket, zeroed by init_result_kernel on the
// same stream) until the tiles run out; at two per CU a chain workgroup fits beside them
// on every CU.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void gram_queue_kernel(
    double* __restrict__ A, int64_t lda, int64_t N, const double* __restrict__ X, int64_t ldx,
    const double* __restrict__ v, const TermPack* __restrict__ tpp, int w0, int w1, int nt, int ntiles,
    EvalResult* __restrict__ res, KTime* __restrict__ kt) {
    kt_begin(kt);
    __shared__ int s_tile;
    __shared__ double glds[GRAM_LDS];
    for (;;) {
        __syncthreads();  // the previous tile's LDS reads are complete
        if (threadIdx.x == 0) s_tile = (int)atomicAdd(&res->gram_ticket, 1u);
        __syncthreads();
        int t = s_tile;
        if (t >= ntiles) break;
        int bi, bj;
        if (w1 >= nt) {  // the triangle of tile blocks w0 .. nt-1
            tri_index(t, bi, bj);
            bi += w0;
            bj += w0;
        } else {  // the lower tiles of tile columns w0 .. w1-1, column by column
            bj = w0;
            while (t >= nt - bj) {
                t -= nt - bj;
                ++bj;
            }
            bi = bj + t;
        }
        gram_tile(A + (int64_t)bj * NB * lda, lda, N, X, ldx, v, tpp, bi, bj, glds);
    }
    kt_end(kt);
}

// Distributed layout: tiles[b] = bi | lj << 16 (global row block, local tile column).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void gram_list_kernel(double* __restrict__ C, int64_t ldc, int64_t N,
                                                        const double* __restrict__ X, int64_t ldx,
                                                        const double* __restrict__ v,
                                                        const TermPack* __restrict__ tpp,
                                                        const uint32_t* __restrict__ tiles, ColMap cm,
                                                        KTime* __restrict__ kt) {
    kt_begin(kt);
    const uint32_t tv = tiles[blockIdx.x];
    const int bi = (int)(tv & 0xffffu), lj = (int)(tv >> 16);
    __shared__ double glds[GRAM_LDS];
    gram_tile(C + (int64_t)lj * NB * ldc, ldc, N, X, ldx, v, tpp, bi, cm.global(lj), glds);
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
// Diagonal kernel phase 2: wave 3 only inverts, waves 1-2 take the trailing tiles in
// interleaved pairs (1), or all three waves share the trailing tiles (0).
// Panels 4-7 of the diagonal kernel with one row per lane (1) or two (0).
#ifndef GAPLAC_DPANEL1
#define GAPLAC_DPANEL1 1
#endif
#ifndef GAPLAC_DIAG_SPLIT
#define GAPLAC_DIAG_SPLIT 1
#endif
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
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(LJ[(4 * kk + fr) * 16 + fc], LI[(4 * kk + fr) * 16 + fc],
                                                   acc, 0, 0, 1);  // neg A
#pragma unroll
    for (int q = 0; q < 4; ++q) C[(fr + 4 * q) * 16 + fc] = acc[q];
}

// Two independent updates C_I1J1 -= L_I1k L_J1k^T and C_I2J2 -= L_I2k L_J2k^T with their
// MFMA chains interleaved (the dependent-accumulator latency of one hides the other's).
__device__ __forceinline__ void dblk_update2(double* Ab, int I1, int J1, int I2, int J2, int k, int lane) {
    double* C1 = Ab + bidx(I1, J1) * 256;
    double* C2 = Ab + bidx(I2, J2) * 256;
    const double* LI1 = Ab + bidx(I1, k) * 256;
    const double* LJ1 = Ab + bidx(J1, k) * 256;
    const double* LI2 = Ab + bidx(I2, k) * 256;
    const double* LJ2 = Ab + bidx(J2, k) * 256;
    const int fr = lane >> 4, fc = lane & 15;
    d4 a1, a2;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        a1[q] = C1[(fr + 4 * q) * 16 + fc];
        a2[q] = C2[(fr + 4 * q) * 16 + fc];
    }
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
        a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(LJ1[(4 * kk + fr) * 16 + fc], LI1[(4 * kk + fr) * 16 + fc], a1, 0, 0, 1);
        a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(LJ2[(4 * kk + fr) * 16 + fc], LI2[(4 * kk + fr) * 16 + fc], a2, 0, 0, 1);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        C1[(fr + 4 * q) * 16 + fc] = a1[q];
        C2[(fr + 4 * q) * 16 + fc] = a2[q];
    }
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

// Wave-level factorisation of panel s: rows 16s..127 x 16 columns, RPL rows per lane (2 for
// panels 0-3; 1 from panel 4 on, where at most 64 rows remain: the sweep is issue-bound in
// one wave, ~50 instructions and ~440 cycles per column with two rows per lane, against a
// ~120-cycle dependent chain -- tools/lat_chain_probe.hip).
// Per column the critical chain is kept short: pivot (v_readlane) -> 1/sqrt (v_rsq_f64
// + one third-order step) -> scale -> update of the NEXT column only (one v_readlane
// broadcast) -> next pivot. Column c's updates of the later columns (c+2..15) are
// deferred into iteration c+1, where they fill the latency of that pivot's 1/sqrt chain;
// their L(c2, c) factors come from an LDS broadcast (the lanes holding the panel's first 16
// rows publish the scaled column, every lane reads it back at the end of iteration c; LDS
// is in order within a wave). The sweep is branch-free (padding pivots and the info test
// are selects).
template <int RPL>
__device__ __forceinline__ void dpanel_t(double* Ab, double* rdiag, double* colbuf, int s, int lane,
                                         int64_t gcol0, int64_t N, EvalResult* res) {
    // opaque copy of the lane id: keeps the lane-dependent masks of the sweep from being
    // hoisted out of the panel loop (and spilled) by loop-invariant code motion
    asm volatile("" : "+v"(lane));
    const int R0 = 16 * s;
    const int rel0 = RPL * lane;
    const int row0 = R0 + rel0;
    const bool live = row0 < NB;
    double v[RPL][16];
    // lanes past the last row read (and never store) the panel's diagonal block
    double* blk = Ab + bidx(live ? (row0 >> 4) : s, s) * 256;
    const int rr = row0 & 15;
#pragma unroll
    for (int c = 0; c < 16; ++c)
#pragma unroll
        for (int r = 0; r < RPL; ++r) v[r][c] = blk[c * 16 + rr + r];
    const int64_t npiv = N - (gcol0 + R0);  // columns >= npiv are padding (unit pivots)
    double myrd = 1.0;
    int bad = 16;
    double piv = readlane_d(v[0][0], 0);
    double lc[16];  // L(c2, c-1) for c2 >= c+1 (broadcast of the previous column)
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        const bool pad = c >= npiv;
        // OpenBLAS potf2 (the reference's dpotrf, 0.3.20) tests ajj <= 0 only: a NaN
        // pivot is not reported and propagates to a NaN logpdf, as in the reference.
        bad = (!pad && piv <= 0.0 && bad == 16) ? c : bad;
        const double p = pad ? 1.0 : piv;
        // v_rsq_f64 (~24 bits) refined by one third-order step: e = 1 - p y^2,
        // 1/sqrt(p) = y + y e (1/2 + 3/8 e), sqrt(p) = t + t e (1/2 + 3/8 e) with t = p y
        // (<= 1 ulp, tools/rsq_probe.hip; 1/sqrt(p) at dependency level 4, where two
        // Goldschmidt steps took 6)
        const double y = __builtin_amdgcn_rsq(p);
        const double t = p * y;
        // deferred updates of columns c+1..15 by column c-1
        if (c >= 1) {
#pragma unroll
            for (int c2 = c + 1; c2 < 16; ++c2)
#pragma unroll
                for (int r = 0; r < RPL; ++r) v[r][c2] = fma(-v[r][c - 1], lc[c2], v[r][c2]);
        }
        const double e = fma(-t, y, 1.0);
        const double cc = fma(e, 0.375, 0.5);
        const double rd = fma(y * e, cc, y);
        const double d = fma(t * e, cc, t);
        myrd = lane == c ? rd : myrd;
#pragma unroll
        for (int r = 0; r < RPL; ++r) v[r][c] = rel0 + r > c ? v[r][c] * rd : (rel0 + r == c ? d : v[r][c]);
        if (c < 15) {
            double* cb = colbuf + 16 * (c & 1);
            if (c < 14) {
                if constexpr (RPL == 2) {
                    if (lane < 8) *reinterpret_cast<double2*>(&cb[2 * lane]) = make_double2(v[0][c], v[1][c]);
                } else {
                    if (lane < 16) cb[lane] = v[0][c];
                }
            }
            const double ln = readlane_d(v[(c + 1) % RPL][c], (c + 1) / RPL);
#pragma unroll
            for (int r = 0; r < RPL; ++r) v[r][c + 1] = fma(-v[r][c], ln, v[r][c + 1]);
            piv = readlane_d(v[(c + 1) % RPL][c + 1], (c + 1) / RPL);
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
        for (int c = 0; c < 16; ++c)
#pragma unroll
            for (int r = 0; r < RPL; ++r)
                blk[c * 16 + rr + r] = (rel0 + r >= c) ? v[r][c] : 0.0;  // zero the diagonal block's upper part
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
#if GAPLAC_DPANEL1
            if (s >= NDB / 2)
                dpanel_t<1>(Ab, rdiag, colbuf, s, lane, g0, N, res);
            else
#endif
                dpanel_t<2>(Ab, rdiag, colbuf, s, lane, g0, N, res);
        } else if (s >= 1) {
            const int ntr = (NDB - 1 - s) * (NDB - s) / 2;  // tiles (I,J), s+1 <= J <= I <= 7
            auto tile_of = [&](int task, int& I, int& J) {
                int rem = task;
                J = s + 1;
                while (rem >= NDB - J) {
                    rem -= NDB - J;
                    ++J;
                }
                I = J + rem;
            };
#if GAPLAC_DIAG_SPLIT
            // wave 3 inverts block s-1 (~4K cycles, the length of wave 0's panel sweep);
            // waves 1 and 2 take the trailing tiles, two at a time (interleaved MFMA chains)
            if (wave == 3) {
                dinv_diag(Ab, Dinv, rdiag, s - 1, lane);
            } else {
                int task = wave - 1;
                for (; task + 2 < ntr; task += 4) {
                    int I1, J1, I2, J2;
                    tile_of(task, I1, J1);
                    tile_of(task + 2, I2, J2);
                    dblk_update2(Ab, I1, J1, I2, J2, s - 1, lane);
                }
                if (task < ntr) {
                    int I, J;
                    tile_of(task, I, J);
                    dblk_update(Ab, I, J, s - 1, lane);
                }
            }
#else
            if (wave == 3) dinv_diag(Ab, Dinv, rdiag, s - 1, lane);  // off the barrier path
            for (int task = wave - 1; task < ntr; task += 3) {
                int I, J;
                tile_of(task, I, J);
                dblk_update(Ab, I, J, s - 1, lane);
            }
#endif
        }
        if (wave == 0) STAMP(2 + 2 * s);
        STAMPT(192, 21 + s);  // wave 3: inverse of block s-1 + its trailing share
        STAMPT(64, 29 + s);   // wave 1: its trailing share
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
// Global accesses through a buffer resource over a wave-uniform base with a cache policy:
// AUX = 0 plain, AUX = GM_SC1 (16) device-coherent "sc1" loads / write-through stores.
// The persistent tail kernel (tail_kernel) hands tiles between workgroups on different
// XCDs with sc1 stores + a flag and sc1 loads (MI355X_MICROARCH.md, "Valid forms",
// table row 1); the stand-alone kernels use AUX = 0. Offsets are in doubles, < 2^28.
// ---------------------------------------------------------------------------------
constexpr int GM_SC1 = 16;
typedef unsigned gm_u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned gm_u32x4 __attribute__((ext_vector_type(4)));
// address-space views for __builtin_amdgcn_global_load_lds (LDS-DMA)
typedef __attribute__((address_space(1))) const void* GlobalCPtr;
typedef __attribute__((address_space(3))) void* LdsPtr;

template <int AUX>
struct Gm {
    __amdgpu_buffer_rsrc_t r;
    __device__ __forceinline__ explicit Gm(const void* base) {
        const uint64_t b = (uint64_t)base;
        const uint64_t u = ((uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)(b >> 32)) << 32) |
                           (uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)b);
        r = __builtin_amdgcn_make_buffer_rsrc((void*)u, 0, 0x7fffffff, 0x00020000);
    }
    __device__ __forceinline__ double ld(uint32_t i) const {
        const gm_u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, i * 8u, 0, AUX);
        double d;
        __builtin_memcpy(&d, &v, 8);
        return d;
    }
    __device__ __forceinline__ double2 ld2(uint32_t i) const {
        const gm_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, i * 8u, 0, AUX);
        double2 d;
        __builtin_memcpy(&d, &v, 16);
        return d;
    }
    __device__ __forceinline__ void st(uint32_t i, double d) const {
        gm_u32x2 v;
        __builtin_memcpy(&v, &d, 8);
        __builtin_amdgcn_raw_buffer_store_b64(v, r, i * 8u, 0, AUX);
    }
    __device__ __forceinline__ void st2(uint32_t i, double2 d) const {
        gm_u32x4 v;
        __builtin_memcpy(&v, &d, 16);
        __builtin_amdgcn_raw_buffer_store_b128(v, r, i * 8u, 0, AUX);
    }
};

// ---------------------------------------------------------------------------------
// Diagonal block, round 3 (potrf_diag2_body): the same blocked right-looking structure
// with 16-column panels, but the panel sweep is split over two waves and scheduled around
// its dependency chain (measured on gfx950, one wave alone: dependent v_fma_f64 10 cycles,
// v_rsq_f64 17, v_readlane of a double ~18 latency / ~16 issue, independent fp64 VALU
// ~4.9 cycles issue; tools/lat_chain_probe.hip, tools/issue_probe.hip).
//
// Wave 0 ("A") holds rows 16s .. 16s+63 of panel s, one row per lane, and runs the pivot
// chain. Per column c the chain is
//   pivot -> rsq -> t = p y -> e = 1 - t y -> c = 1/2 + 3/8 e -> rd = y + y e c
//         -> l = v rd -> readlane(l, c+1) -> v[c+1] -= l * ln -> readlane(v[c+1], c+1)
// and everything else is taken off it: column c+1 receives columns c-2 and c-1 at the top
// of iteration c (in the shadow of the rsq), columns c+2..15 receive column c-2 ("2-deep
// deferral"; its L values come from an LDS broadcast written two iterations earlier, so
// the LDS latency is never waited for), and those independent FMAs are placed between the
// chain's dependent instructions by scheduling barriers.
// Wave 1 ("B", panels 0-3) holds rows 16s+64 .. 127 and consumes each column as wave A
// publishes it (L values of the 16 diagonal rows + rd, flagged per column in LDS).
// Waves 2-3 (and wave 1 from panel 4 on) apply panel s-1 to the trailing block columns
// and invert the finished 16x16 diagonal sub-blocks (Dinv) where the sweep leaves slack.
// Results agree with the round-2 kernel to rounding (different but fixed summation order);
// pivots of padding columns are 1, a pivot <= 0 records info (OpenBLAS potf2's test).
// ---------------------------------------------------------------------------------
// LDS: the small buffers first (their addresses fit the 16-bit DS offset), then the block.
constexpr int DIAG2_COLBUF = 16 * 64;  // colbuf[c * 64 + lane]: column c's record (diag2_sweep_a)
constexpr int DIAG2_SMEM = DIAG2_COLBUF + NB + NPK * 256;  // colbuf, rdiag, Ab (doubles)

#define SB() __builtin_amdgcn_sched_barrier(0)
#define PIN(x) asm volatile("" : "+v"(x))

// Wave A's sweep of panel s (rows 16s + lane). Per column the published 16-lane record
// colbuf[c * 64 + 0..15] holds L(16s + r, 16s + c) for r > c and rd_c = 1/L_cc in slot c;
// slot c doubles as the record's flag (reset to -1 before the panel; rd is never -1): the
// record is one ds_write_b64 whose lanes 0-15 form one LDS lane group, written in one cycle.
__device__ __forceinline__ void diag2_sweep_a(double* Ab, double* colbuf, int s, int lane, int64_t gcol0, int64_t N,
                                              EvalResult* res) {
    asm volatile("" : "+v"(lane));
    const int R0 = 16 * s;
    const int row = R0 + lane;
    const bool live = row < NB;
    double* blk = Ab + bidx(live ? (row >> 4) : s, s) * 256;
    const int rr = row & 15;
    double v[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) v[c] = blk[c * 16 + rr];
    const int64_t npiv64 = N - (gcol0 + R0);  // columns >= npiv are padding (unit pivots)
    const int npiv = (int)(npiv64 < 0 ? 0 : (npiv64 > 16 ? 16 : npiv64));
    const unsigned padmask = (0xffffu << npiv) & 0xffffu;
    double lcA[16], lcB[16];  // L(R0 + c2, c - 2) / L(R0 + c2, c - 1), uniform
#pragma unroll
    for (int c = 0; c < 16; ++c) lcA[c] = lcB[c] = 0.0;
    double k375 = 0.375;  // kept in a VGPR (not an inline constant)
    PIN(k375);
    double ln2 = 0.0;  // L(R0 + c + 1, c - 1), uniform
    double mypiv = 1.0;
    double piv = readlane_d(v[0], 0);
    SB();
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        // fillers: column c-2 into columns c+2 .. 15, pinned where they are placed
        auto fill = [&](int k) {
            const int c2 = c + 2 + k;
            if (c >= 2 && c2 < 16) {
                v[c2] = fma(-v[c - 2], lcA[c2], v[c2]);
                PIN(v[c2]);
            }
        };
        const bool pad = (padmask >> c) & 1u;
        const double p = pad ? 1.0 : piv;
        // G1: rsq; column c+1 gets columns c-2 and c-1; LDS reads of column c-1's L values
        const double y = __builtin_amdgcn_rsq(p);
        mypiv = lane == c ? v[c] : mypiv;  // the non-PD test runs after the sweep
        if (c >= 1) {
#pragma unroll
            for (int c2 = c + 2; c2 < 16; ++c2) lcB[c2] = colbuf[(c - 1) * 64 + c2];
        }
        if (c >= 2 && c + 1 < 16) v[c + 1] = fma(-v[c - 2], lcA[c + 1], v[c + 1]);
        if (c >= 1 && c + 1 < 16) {
            v[c + 1] = fma(-v[c - 1], ln2, v[c + 1]);
            PIN(v[c + 1]);
        }
        fill(0);
        SB();
        const double t = p * y;  // G2
        fill(1);
        fill(2);
        SB();
        const double e = fma(-t, y, 1.0);  // G3
        fill(3);
        fill(4);
        SB();
        const double cc = fma(e, k375, 0.5);  // G4
        const double ye = y * e;
        fill(5);
        SB();
        const double rd = fma(ye, cc, y);  // G5: 1/sqrt(p), <= 1 ulp
        fill(6);
        fill(7);
        SB();
        // G6: scale column c. The diagonal lane's own value is its pivot, so it becomes
        // p * rd = sqrt(p) (padding columns: fixed to 1 at the write-back); lanes above the
        // diagonal get junk * rd, never read, zeroed at the write-back.
        v[c] = v[c] * rd;
        fill(8);
        SB();
        // G7: the two readlanes of the chain, then the column's record
        double ln = 0.0, ln2n = 0.0;
        if (c + 1 < 16) ln = readlane_d(v[c], c + 1);
        if (c + 2 < 16) ln2n = readlane_d(v[c], c + 2);
        colbuf[c * 64 + lane] = lane == c ? rd : v[c];
        fill(9);
        fill(10);
        SB();
        if (c + 1 < 16) v[c + 1] = fma(-v[c], ln, v[c + 1]);  // G8
        fill(11);
        SB();
        if (c + 1 < 16) piv = readlane_d(v[c + 1], c + 1);  // G9
        fill(12);
        ln2 = ln2n;
#pragma unroll
        for (int c2 = 0; c2 < 16; ++c2) lcA[c2] = lcB[c2];
        SB();
    }
    // OpenBLAS potf2 (the reference's dpotrf, 0.3.20) tests ajj <= 0 only: a NaN pivot is
    // not reported and propagates to a NaN logpdf, as in the reference
    const unsigned long long badm = __ballot(lane < 16 && !((padmask >> lane) & 1u) && mypiv <= 0.0);
    if (badm && lane == 0) atomicMin(&res->info, (unsigned long long)(gcol0 + R0 + __builtin_ctzll(badm) + 1));
    if (live) {
        const bool padlane = lane < 16 && ((padmask >> lane) & 1u);
#pragma unroll
        for (int c = 0; c < 16; ++c)  // zero the diagonal block's upper part, unit padding pivots
            blk[c * 16 + rr] = lane > c ? v[c] : (lane == c ? (padlane ? 1.0 : v[c]) : 0.0);
    }
}

// Wave B's rows of panel s (rows 16s + 64 + lane, s < 4): consumes wave A's records. The
// flag of column c+1 is read while column c is computed; its L values after the flag.
__device__ __forceinline__ void diag2_sweep_b(double* Ab, double* colbuf, int s, int lane, EvalResult* res) {
    asm volatile("" : "+v"(lane));
    const int row = 16 * s + 64 + lane;
    const bool live = row < NB;
    double* blk = Ab + bidx(live ? (row >> 4) : NDB - 1, s) * 256;
    const int rr = row & 15;
    double v[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) v[c] = blk[c * 16 + rr];
    bool timeout = false;
    double fl = __hip_atomic_load(&colbuf[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        // bounded wait for wave A (same workgroup: it never waits for this wave)
        for (int it = 0; fl == -1.0 && it < (1 << 20); ++it) {
            __builtin_amdgcn_s_sleep(1);
            fl = __hip_atomic_load(&colbuf[c * 64 + c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (fl == -1.0) {
            timeout = true;
            fl = __builtin_nan("");
        }
        const double rd = fl;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // the record's values after its flag
        double lc[16];
#pragma unroll
        for (int c2 = c + 1; c2 < 16; ++c2) lc[c2] = colbuf[c * 64 + c2];
        if (c + 1 < 16) fl = __hip_atomic_load(&colbuf[(c + 1) * 64 + c + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const double l = v[c] * rd;
        v[c] = l;
#pragma unroll
        for (int c2 = c + 1; c2 < 16; ++c2) v[c2] = fma(-l, lc[c2], v[c2]);
    }
    if (timeout && lane == 0) atomicOr(&res->err, 1u);
    if (live) {
#pragma unroll
        for (int c = 0; c < 16; ++c) blk[c * 16 + rr] = v[c];
    }
}

// Dinv_s = L_ss^{-1} (column-major 16x16 into global): lane j < 16 solves L x = e_j
// right-looking (x[m] final, then every later row updated with it).
template <int AUX>
__device__ __forceinline__ void diag2_dinv(const double* Ab, double* __restrict__ Dinv, const double* rdiag, int s,
                                           int lane, double* Dl = nullptr) {
    const double* Ls = Ab + bidx(s, s) * 256;  // L(r, m) = Ls[m * 16 + r]
    asm volatile("" : "+v"(lane));
    const int j = lane & 15;
    double x[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) x[r] = r == j ? 1.0 : 0.0;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        x[m] *= rdiag[16 * s + m];
#pragma unroll
        for (int r = m + 1; r < 16; ++r) x[r] = fma(-Ls[m * 16 + r], x[m], x[r]);
    }
    const Gm<AUX> g(Dinv);
    if (lane < 16) {
#pragma unroll
        for (int r = 0; r < 16; r += 2) g.st2((uint32_t)(s * 256 + j * 16 + r), make_double2(x[r], x[r + 1]));
        if (Dl) {  // LDS copy for a TRSM in the same workgroup (tail_kernel)
#pragma unroll
            for (int r = 0; r < 16; r += 2)
                *reinterpret_cast<double2*>(&Dl[s * 256 + j * 16 + r]) = make_double2(x[r], x[r + 1]);
        }
    }
}

// Trailing blocks (I, J), s+1 <= J <= I <= 7, with panel s-1: tasks t = first, first+step, ...
__device__ __forceinline__ void diag2_trailing(double* Ab, int s, int first, int step, int lane) {
    const int ntr = (NDB - 1 - s) * (NDB - s) / 2;
    auto tile_of = [&](int task, int& I, int& J) {
        int rem = task;
        J = s + 1;
        while (rem >= NDB - J) {
            rem -= NDB - J;
            ++J;
        }
        I = J + rem;
    };
    int task = first;
    for (; task + step < ntr; task += 2 * step) {
        int I1, J1, I2, J2;
        tile_of(task, I1, J1);
        tile_of(task + step, I2, J2);
        dblk_update2(Ab, I1, J1, I2, J2, s - 1, lane);
    }
    if (task < ntr) {
        int I, J;
        tile_of(task, I, J);
        dblk_update(Ab, I, J, s - 1, lane);
    }
}

// Block m of the 28 below-and-right-of-column-0 blocks of the 8x8 block triangle (J >= 1).
__device__ __forceinline__ void diag2_block_of(int m, int& I, int& J) {
    J = 1;
    while (m >= NDB - J) {
        m -= NDB - J;
        ++J;
    }
    I = J + m;
}

// Store block column s of L (blocks (I, s), I = s..7) to global, pairs of rows: every
// 16-row column segment (one 128-byte line) by 8 consecutive lanes of one instruction; the
// diagonal 16x16 block's upper part goes out as the zeros sweep A left in LDS. Threads
// tt = 0 .. nthr-1 (a multiple of 64) of the storing waves.
template <int AUX>
__device__ __forceinline__ void diag2_store_column(const double* Ab, double* Ag, int64_t lda, int s, int tt, int nthr) {
    const int npairs = (NDB - s) * 128;
    const Gm<AUX> g(Ag);
    for (int q = tt; q < npairs; q += nthr) {
        const int I = s + (q >> 7), pr = q & 127;
        const int c = pr >> 3, r = 2 * (pr & 7);
        const double2 x = *reinterpret_cast<const double2*>(&Ab[bidx(I, s) * 256 + c * 16 + r]);
        g.st2((uint32_t)((int64_t)(16 * s + c) * lda + 16 * I + r), x);
    }
}

// 512 threads: wave 0 = A (the pivot chain), wave 1 = B (rows 64+ of panels 0-3), waves 2-7
// the trailing updates, the stores of finished block columns and (wave 7) the inverses.
// Waves w and w + 4 share a SIMD, so every SIMD's matrix pipe takes trailing work.
template <int AUX>
__device__ __forceinline__ void potrf_diag2_body(double* smem, double* __restrict__ Ag, int64_t lda, int64_t N,
                                                 int64_t g0, double* __restrict__ Dinv, EvalResult* __restrict__ res,
                                                 double* Dl = nullptr, unsigned* prog = nullptr,
                                                 unsigned long long* dst = nullptr) {
    double* colbuf = smem;
    double* rdiag = colbuf + DIAG2_COLBUF;
    double* Ab = rdiag + NB;
    const int t = otid(), wave = t >> 6, lane = t & 63;
    // diagnostics (tail trace): phase times on the 100 MHz clock, thread 0
    auto dstamp = [&](int i) {
        if (dst && t == 0) dst[i] = wall_clock64();
    };
    dstamp(0);
    // the chain first (wave-uniform branches: s_setprio takes an immediate)
    if (wave == 0) __builtin_amdgcn_s_setprio(3);
    else if (wave == 1) __builtin_amdgcn_s_setprio(2);
    else __builtin_amdgcn_s_setprio(1);
    STAMP(20);
    // Load: block column 0 by everyone first (panel 0 needs it), the other 28 blocks by
    // waves 2-7, written to LDS while panel 0 is swept.
    double2 rest[10];
    const int tt = t - 128;  // waves 2-7: 0 .. 383
    {
        const Gm<AUX> g(Ag);
        double2 col0[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int q = t + 512 * i, I = q >> 7, pr = q & 127, c = pr >> 3, r = 2 * (pr & 7);
            col0[i] = g.ld2((uint32_t)((int64_t)c * lda + 16 * I + r));
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int q = t + 512 * i, I = q >> 7, pr = q & 127;
            *reinterpret_cast<double2*>(&Ab[bidx(I, 0) * 256 + 2 * pr]) = col0[i];
        }
        // issued after column 0 is in LDS: behind the wave-dependent branch the compiler
        // can no longer count the loads in flight, and a column-0 write placed after it
        // waited for all of them (vmcnt(0)), the whole block's latency before panel 0
        if (wave >= 2) {
#pragma unroll
            for (int i = 0; i < 10; ++i) {
                const int q = tt + 384 * i;
                if (q < 28 * 128) {
                    int I, J;
                    diag2_block_of(q >> 7, I, J);
                    const int pr = q & 127, c = pr >> 3, r = 2 * (pr & 7);
                    rest[i] = g.ld2((uint32_t)((int64_t)(16 * J + c) * lda + 16 * I + r));
                }
            }
        }
    }
    if (wave == 3 && lane < 16) colbuf[lane * 64 + lane] = -1.0;  // the records' flags
    // a barrier that does not wait for the other blocks' loads (__syncthreads would)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    STAMP(0);
    dstamp(1);
    for (int s = 0; s < NDB; ++s) {
        if (s >= 1) {
            // phase 1: panel s-1 into block column s (the diagonal block first, on wave 0)
            for (int I = s + wave; I < NDB; I += 8) dblk_update(Ab, I, s, s - 1, lane);
            if (wave == 3 && lane < 16) {
                rdiag[16 * (s - 1) + lane] = colbuf[lane * 64 + lane];  // rd of panel s-1's columns
                colbuf[lane * 64 + lane] = -1.0;                        // the records' flags
            }
            // progress hand-off (tail_kernel): the stores of block column s-2 and Dinv(s-2)
            // (phase 2 of panel s-1) complete before this phase's barrier, published after it
            if (prog && wave >= 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
        STAMP(1 + 2 * s);
        dstamp(2 + 2 * s);
        // phase 2
        if (prog && s >= 2 && wave == 3 && lane == 0)  // columns and inverses 0 .. s-2 final
            __hip_atomic_store(prog, (unsigned)(s - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (wave == 0) {
            diag2_sweep_a(Ab, colbuf, s, lane, g0, N, res);
        } else if (wave == 1 && s < 4) {
            diag2_sweep_b(Ab, colbuf, s, lane, res);
        } else {
            if (s == 0 && wave >= 2) {  // the rest of the block into LDS
#pragma unroll
                for (int i = 0; i < 10; ++i) {
                    const int q = tt + 384 * i;
                    if (q < 28 * 128) {
                        int I, J;
                        diag2_block_of(q >> 7, I, J);
                        *reinterpret_cast<double2*>(&Ab[bidx(I, J) * 256 + 2 * (q & 127)]) = rest[i];
                    }
                }
            }
            if (s >= 1) {
                // wave 4 shares wave A's SIMD: it only stores and inverts (light), the
                // trailing blocks go to waves 2, 3, 5, 6, 7 (and 1 from panel 4 on)
                if (wave >= 2) diag2_store_column<AUX>(Ab, Ag, lda, s - 1, t - 128, 384);
                STAMPT(128, 40 + s);  // wave 2: after its share of the stores
                if (wave == 4) {
                    diag2_dinv<AUX>(Ab, Dinv, rdiag, s - 1, lane, Dl);
                } else {
                    const int w = wave == 1 ? 0 : (s < 4 ? 0 : 1) + (wave < 4 ? wave - 2 : wave - 3);
                    diag2_trailing(Ab, s, w, s < 4 ? 5 : 6, lane);
                }
            }
        }
        if (wave == 0) STAMP(2 + 2 * s);
        STAMPT(64, 29 + s);
        STAMPT(128, 21 + s);
        STAMPT(192, 48 + s);
        STAMPT(256, 80 + s);
        STAMPT(320, 56 + s);
        STAMPT(384, 64 + s);
        STAMPT(448, 72 + s);
        __syncthreads();
        dstamp(3 + 2 * s);
    }
    if (wave == 3 && lane < 16) rdiag[16 * (NDB - 1) + lane] = colbuf[lane * 64 + lane];
    if (prog && wave >= 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (prog && wave == 3 && lane == 0)  // columns and inverses 0 .. 6 final
        __hip_atomic_store(prog, (unsigned)(NDB - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    STAMP(17);
    if (wave == 4) diag2_dinv<AUX>(Ab, Dinv, rdiag, NDB - 1, lane, Dl);
    STAMP(18);
    if (wave != 4) diag2_store_column<AUX>(Ab, Ag, lda, NDB - 1, wave < 4 ? t : t - 64, 448);
    STAMP(19);
    dstamp(19);
}
#undef SB
#undef PIN

// The diagonal block of the super-panel chain (256 threads: 255 + 16 registers, one wave per
// SIMD, 75 KB of LDS) fits on a CU beside ONE resident bulk workgroup (208 registers, 72 KB).
// potrf_diag2_body (512 threads, 199 registers, two waves per SIMD: 27 us alone against
// ~32) does not: beside the bulk updates it waited for a CU with both bulk workgroups
// retired, i.e. for the end of the launch (3.2 ms of a 3.6 ms K = 1024 update in a kernel
// trace, profiles/r03r_timeline.txt), so the chain kernel here is this one and diag2 runs
// only inside the persistent tail, where nothing else is resident.
__global__ __launch_bounds__(256) void potrf_diag_kernel(double* __restrict__ Ag, int64_t lda, int64_t N,
                                                         int64_t g0, double* __restrict__ Dinv,
                                                         EvalResult* __restrict__ res, KTime* __restrict__ kt) {
    kt_begin(kt);
    potrf_diag_kernel_body(Ag, lda, N, g0, Dinv, res);
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
                                                         const double* __restrict__ Dinv, int vb) {
    __shared__ double Ls[(TRSM_LBLK + NDB) * 256];
    __builtin_amdgcn_s_setprio(2);  // critical path
    const int tid = threadIdx.x;
    const int bi = bi0 + (int)(vb >> 1);
    const int wave = tid >> 6, lane = tid & 63;
    const int fr = lane >> 4, fc = lane & 15;
    const int64_t k0 = (int64_t)k * NB;
    const double* L = Acol + k0;  // L_kk, column-major, lda
    double* B = Acol + (int64_t)bi * NB + 64 * (vb & 1) + 16 * wave;
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
                const double lbc = Lbc[(4 * kk + fr) * 16 + fc];  // L_bc[j][m], m = 4kk + fr (negated: neg A)
                // two partial sums (even / odd c): halves the dependent-accumulator chain
                if (c & 1)
                    s1 = __builtin_amdgcn_mfma_f64_16x16x4f64(lbc, Y[c][kk], s1, 0, 0, 1);
                else
                    s0 = __builtin_amdgcn_mfma_f64_16x16x4f64(lbc, Y[c][kk], s0, 0, 0, 1);
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
    trsm_subst_kernel_body(Acol, lda, k, bi0, Dinv, (int)blockIdx.x);
    kt_end(kt);
}

// ---------------------------------------------------------------------------------
// Bulk trailing update, one 128x128 tile per 256-thread workgroup:
//   C(bi, bj) -= P_bi P_bj^T,   P = the kdepth panel columns (Panel operand),
// with C tile (bi, bj) stored in local tile column lj (ColMap: bj = cm.global(lj)).
// 4 waves as 2x2, each wave a 64x64 sub-tile = 4x4 v_mfma_f64_16x16x4f64 accumulators.
// Operands are staged through LDS in 16-deep k-chunks by LDS-DMA, double-buffered (the
// next chunk in flight while the current one is multiplied). The MFMA computes D = Q*P^T
// (the j-side fragment is the A operand) so that a lane's accumulator column is C's row:
// stores are 128-byte column segments of the column-major matrix. The C tile is loaded
// straight into the accumulators before the k-loop and the MFMA negates P (neg modifier),
// so the chain produces C - P Q^T and the epilogue is stores only.
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
template <int KBT>
using MmaLdsT = double[2][2][KBT][LR];  // the k-chunk staging buffers of tile_mma_neg
typedef MmaLdsT<KB> MmaLds;
static_assert(sizeof(MmaLds) >= GRAM_LDS * sizeof(double), "gram_tile reuses the staging LDS");

template <int KBT = KB>
__device__ __forceinline__ void tile_mma_neg(const double* __restrict__ P, const double* __restrict__ Q,
                                             int64_t ldp, int kdepth, bool active, d4 (&acc)[4][4],
                                             MmaLdsT<KBT>& sm) {
    constexpr int KB = KBT;
    const int tid = threadIdx.x;
    const int lane = tid & 63, w = tid >> 6;
    const int wi = w & 1, wj = w >> 1;
    const int fr = lane >> 4, fc = lane & 15;
    // LDS-DMA staging: the chunk's 2 KB rows (KB panel columns of P, then of Q: 128 contiguous
    // rows each) go straight into LDS, one global_load_lds (16 B per lane) per row, wave w
    // taking rows w, w + 4, ...; no staging registers and no LDS stores in the MFMA stream.
    // P stays unnegated in LDS: the MFMA's B-operand neg modifier (blgp = 2 on f64 MFMA)
    // makes the chain C - P Q^T, bitwise what staging -P gave (register-staged version: 208
    // VGPRs, 0.794 / 0.833 of peak at the 16k / 64k shapes alone; this one 189 VGPRs, 0.819 /
    // 0.852, tools/bulk_probe.hip, profiles/r04y_bulk_probe.txt).
    auto issue = [&](int ch, int buf) {
#pragma unroll
        for (int it = 0; it < 2 * KB / 4; ++it) {
            const int t = w + 4 * it, o = t / KB, r = t % KB;
            const double* src = (o ? Q : P) + (int64_t)(ch * KB + r) * ldp + 2 * lane;
            __builtin_amdgcn_global_load_lds((GlobalCPtr)src, (LdsPtr)&sm[buf][o][r][0], 16, 0, 0);
        }
    };
    const int NCH = kdepth / KB;
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int ch = 0; ch < NCH; ++ch) {
        const int buf = ch & 1;
        if (ch + 1 < NCH) issue(ch + 1, buf ^ 1);  // the buffer every wave left at the last barrier
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
                        acc[mi][mj] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[mj], fb[mi], acc[mi][mj], 0, 0, 2);
            }
        }
        // the next chunk landed (every wave's own DMA), then visible to all waves
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
}

template <int KBT = KB>
__device__ __forceinline__ void tile_syrk_body(const BulkArgs& a, int b) {
    const int chunk = (a.ntiles + 7) >> 3;
    const int idx = (b & 7) * chunk + (b >> 3);
    if (idx >= a.ntiles) return;
    __shared__ MmaLdsT<KBT> sm;
    int bi, bj, lj;
    tile_decode(a, idx, bi, bj, lj);
    const int64_t r0 = (int64_t)bi * NB;
    const int64_t ldc = a.ldc;
    double* __restrict__ Ct = a.C + (int64_t)lj * NB * ldc + r0;
    const double* __restrict__ P = a.pn.P + (r0 - a.pn.row0);
    const double* __restrict__ Q = a.pn.P + ((int64_t)bj * NB - a.pn.row0);
    const int tid = threadIdx.x;
    const int lane = tid & 63, w = tid >> 6;
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
    tile_mma_neg<KBT>(P, Q, a.pn.ld, a.kdepth, active, acc, sm);
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

// One tile per workgroup, 189 VGPRs (208 with register staging): two resident bulk
// workgroups leave 134 registers per SIMD lane, more than the 96 a quadrant chain kernel needs.
// Diagnostic build only (-DGAPLAC_CLOCK=1): each workgroup of the bulk tile kernels adds
// its shader cycles (s_memtime) and 100 MHz ticks (s_memrealtime) to its launch's KTime
// slot; the host prints the clock held per launch (MI355X_MICROARCH.md 'DVFS give-back'
// item 6). Never compiled into the library.
#ifndef GAPLAC_CLOCK
#define GAPLAC_CLOCK 0
#endif
struct ClkStamp {
    unsigned long long mt = 0, rt = 0;
    __device__ __forceinline__ void begin(const KTime* kt) {
        if (GAPLAC_CLOCK && kt && threadIdx.x == 0) {
            __builtin_amdgcn_sched_barrier(0);
            mt = __builtin_amdgcn_s_memtime();
            rt = __builtin_amdgcn_s_memrealtime();
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    __device__ __forceinline__ void end(KTime* kt) {
        if (GAPLAC_CLOCK && kt && threadIdx.x == 0) {
            __builtin_amdgcn_sched_barrier(0);
            const unsigned long long m1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
            __builtin_amdgcn_s_waitcnt(0xC07F);
            atomicAdd(&kt->clk_mt, m1 - mt);
            atomicAdd(&kt->clk_rt, r1 - rt);
            atomicAdd(&kt->clk_n, 1ull);
        }
    }
};

__global__ __launch_bounds__(256, 2) void tile_syrk_kernel(BulkArgs a, KTime* __restrict__ kt) {
    kt_begin(kt);
    ClkStamp ck;
    ck.begin(kt);
    tile_syrk_body(a, (int)blockIdx.x);
    ck.end(kt);
    kt_end(kt);
}

// The same kernel under its own name for the band updates of the paired schedule (a short
// list of a super-panel's tiles ahead of the bulk update), so that kernel traces keep the
// bulk launches (tile_syrk_kernel, the roofline kernel) apart.
__global__ __launch_bounds__(256, 2) void tile_band_kernel(BulkArgs a, KTime* __restrict__ kt) {
    kt_begin(kt);
    ClkStamp ck;
    ck.begin(kt);
    tile_syrk_body(a, (int)blockIdx.x);
    ck.end(kt);
    kt_end(kt);
}

// Large trailing updates (at least BULK_BIG_TILES tiles, N >= ~26k): 8-deep chunks (37 KB
// of LDS) and 168 VGPRs, three resident workgroups per CU. Alone 0.874 vs 0.852 of peak at
// the 64k shape; not for the 16k schedule, where three bulk workgroups leave no registers
// for the chain's quadrant kernels.
constexpr int BULK_BIG_TILES = 20000;
__global__ __launch_bounds__(256, 3) void tile_syrk_big_kernel(BulkArgs a, KTime* __restrict__ kt) {
    kt_begin(kt);
    tile_syrk_body<8>(a, (int)blockIdx.x);
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
static_assert((NB / 4) % QG == 0, "the quadrant k-loop takes K in groups of 4 QG columns");
// Bulk updates with at most this many 128x128 tiles run as quadrants (4 WGs per tile).
constexpr int QUAD_BULK_MAX_TILES = 512;

__device__ __forceinline__ void quad_update(double* __restrict__ C, int64_t ldc, const Panel& pn, int bi,
                                            int bj, int lj, int qi, int qj, int kdepth) {
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
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
            const double b0 = fb[buf][s][0], b1 = fb[buf][s][1];  // negated by the MFMA (neg B)
            acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[buf][s][0], b0, acc[0][0], 0, 0, 2);
            acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[buf][s][0], b1, acc[1][0], 0, 0, 2);
            acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[buf][s][1], b0, acc[0][1], 0, 0, 2);
            acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[buf][s][1], b1, acc[1][1], 0, 0, 2);
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
    const int chunk = (a.ntiles + 7) >> 3;
    const int b = (int)blockIdx.x >> 2, q = (int)blockIdx.x & 3;
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
        kt[i].clk_mt = kt[i].clk_rt = kt[i].clk_n = 0ull;
    }
}

void launch_kt_reset(hipStream_t s, KTime* kt, int n) {
    if (n > 0 && guard_launch("kt_reset_kernel")) kt_reset_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s>>>(kt, n);
}

__device__ __forceinline__ void init_result_kernel_body(EvalResult* res) {
    res->logpdf = 0.0;
    res->logdet = 0.0;
    res->quad = 0.0;
    res->info = ~0ull;
    res->gram_ticket = 0u;
    res->err = 0u;
}
__global__ void init_result_kernel(EvalResult* res) { init_result_kernel_body(res); }

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

// z = row N of the factor (z_k = A[k * lda + N]) into a contiguous buffer: alpha reads it
// from there while cinv_tile_kernel, which may overwrite row N, runs beside it.
__global__ __launch_bounds__(256) void copy_z_kernel(const double* __restrict__ A, int64_t lda, int64_t N,
                                                     double* __restrict__ z) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k < N) z[k] = A[k * lda + N];
}

// alpha partial sums: block (x, y) = rows 256x .. 256x+255, columns 512y .. 512y+511.
__global__ __launch_bounds__(256) void alpha_partial_kernel(const double* __restrict__ A, int64_t lda,
                                                            int64_t Np, int64_t N, const double* __restrict__ z,
                                                            double* __restrict__ partial) {
    __shared__ double zs[512];
    const int tid = threadIdx.x;
    const int64_t k0 = (int64_t)blockIdx.y * 512;
    const int64_t i = (int64_t)blockIdx.x * 256 + tid;
    for (int t = tid; t < 512; t += 256) zs[t] = (k0 + t < N) ? z[k0 + t] : 0.0;
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
        __shared__ MmaLds sm;
        tile_mma_neg(Y + k0 * lda + (int64_t)I * NB, Y + k0 * lda + (int64_t)J * NB, lda, (int)(Np - k0), active,
                     acc, sm);
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

// dC/dl of a SqExp / OU term (term_dk's arithmetic, the Gram kernel's table exp): no FMA
// contraction, so equal coordinates give exactly u = 0
__device__ __forceinline__ double dk_sqexp(double p, double xi, double xj, const double* tbl) {
#pragma clang fp contract(off)
    const double u = p * xi - p * xj;
    const double u2 = u * u;
    return exp_nonpos(-u2 * 0.5, tbl) * u2 * p;
}
__device__ __forceinline__ double dk_ou(double p, double xi, double xj, const double* tbl) {
#pragma clang fp contract(off)
    const double a = fabs(p * xi - p * xj);
    return exp_nonpos(-a, tbl) * a * p;
}

// -C^{-1} tile (I, J) as cinv_tile_kernel computes it, contracted in place with every
// dC/dtheta (grad_contract_kernel's sum over the tile) instead of being stored: the tile
// never goes to HBM and is never read back. Formulas whose groups are all single terms (the
// reference's lowering; product groups keep the two-kernel path). alpha must be final
// before the launch. partial[b][t] for the tile's triangle index b = I (I + 1) / 2 + J,
// t <= T. After the k-loop the accumulators become the weights wt (alpha_i alpha_j + M_ij)
// in place (wt = 2 off the diagonal, 1 on it, 0 outside the lower triangle / past N); then
// one pass per term over the 64 weights of a lane, each term kind a loop of its own (the
// code stays small: a fully unrolled term x element nest overflowed the instruction cache).
// The k-loop's LDS staging buffer holds the tile's coordinates, alpha, the exp table and the
// per-wave sums (checked at compile time). With GAPLAC_KB = 8 the sums do not fit and get a
// small array of their own; with the default KB = 16 they stay in the staging buffer (an
// extra __shared__ array there cost the gradient 1.8 ms).
static_assert(sizeof(MmaLds) >= (2 * GAPLAC_MAX_TERMS * NB + 2 * NB + 256) * sizeof(double),
              "cinv_contract_kernel's coordinates, alpha and exp table must fit the staging LDS");
#if GAPLAC_KB == 16
static_assert(sizeof(MmaLds) >= (2 * GAPLAC_MAX_TERMS * NB + 2 * NB + 256 + 4 * (GAPLAC_MAX_TERMS + 1)) * sizeof(double),
              "cinv_contract_kernel's per-wave sums must fit the staging LDS");
#endif
__global__ __launch_bounds__(256, 2) void cinv_contract_kernel(const double* __restrict__ A, int64_t lda, int64_t Np,
                                                               int64_t N, const double* __restrict__ X, int64_t ldx,
                                                               const double* __restrict__ alpha,
                                                               const TermPack* __restrict__ tpp,
                                                               const uint32_t* __restrict__ list,
                                                               double* __restrict__ partial, KTime* __restrict__ kt) {
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
        __shared__ MmaLds sm;
        tile_mma_neg(Y + k0 * lda + (int64_t)I * NB, Y + k0 * lda + (int64_t)J * NB, lda, (int)(Np - k0), active,
                     acc, sm);
        // (tile_mma_neg ends on a barrier: the staging buffer is free)
        const TermPack& tp = *tpp;
        const int T = tp.T;
        double* const xr = &sm[0][0][0][0];           // xr[t * 128 + r]
        double* const xc = xr + GAPLAC_MAX_TERMS * NB;  // xc[t * 128 + c]
        double* const ar = xc + GAPLAC_MAX_TERMS * NB;  // alpha of the rows, then of the columns
        double* const ac = ar + NB;
        double* const tbl = ac + NB;                    // exp table
#if GAPLAC_KB == 16
        double* const red = tbl + 256;  // red[w * (T + 1) + t]
#else
        __shared__ double red[4 * (GAPLAC_MAX_TERMS + 1)];
#endif
        const int64_t r0 = (int64_t)I * NB, c0 = (int64_t)J * NB;
        for (int idx = tid; idx < T * NB; idx += 256) {
            const int t = idx / NB, q = idx % NB;
            const bool x = tp.kind[t] != GAPLAC_NOISE;
            const double* xcol = X + (int64_t)tp.col[t] * ldx;
            xr[t * NB + q] = (x && r0 + q < N) ? xcol[r0 + q] : 0.0;
            xc[t * NB + q] = (x && c0 + q < N) ? xcol[c0 + q] : 0.0;
        }
        if (tid < NB) {
            ar[tid] = r0 + tid < N ? alpha[r0 + tid] : 0.0;
            ac[tid] = c0 + tid < N ? alpha[c0 + tid] : 0.0;
        }
        tbl[tid] = kExp2Tbl256[tid];
        __syncthreads();
        // weights in place (inactive waves: all zero)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
            const int rr = 64 * wi + 16 * mi + fc;
            const int64_t i = r0 + rr;
            const double ai = ar[rr];
#pragma unroll
            for (int mj = 0; mj < 4; ++mj)
#pragma unroll
                for (int rg = 0; rg < 4; ++rg) {
                    const int cc = 64 * wj + 16 * mj + fr + 4 * rg;
                    const int64_t j = c0 + cc;
                    const bool in = active && i < N && j < N && i >= j;
                    const double wt = in ? (i == j ? 1.0 : 2.0) : 0.0;
                    acc[mi][mj][rg] = wt * (ai * ac[cc] + acc[mi][mj][rg]);
                }
        }
        // the diagonal elements of a diagonal tile (row rr == column cc)
        auto diag_sum = [&]() {
            double g = 0.0;
            if (I == J) {
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int mj = 0; mj < 4; ++mj)
#pragma unroll
                        for (int rg = 0; rg < 4; ++rg)
                            if (64 * wi + 16 * mi + fc == 64 * wj + 16 * mj + fr + 4 * rg) g += acc[mi][mj][rg];
            }
            return g;
        };
#pragma unroll 1
        for (int t = 0; t <= T; ++t) {
            double g = 0.0;
            const int kind = t < T ? tp.kind[t] : GAPLAC_NOISE;
            if (kind == GAPLAC_SQEXP) {
                const double p = tp.p[t];
#pragma unroll
                for (int mi = 0; mi < 4; ++mi) {
                    const double xi = xr[t * NB + 64 * wi + 16 * mi + fc];
#pragma unroll
                    for (int mj = 0; mj < 4; ++mj)
#pragma unroll
                        for (int rg = 0; rg < 4; ++rg)
                            g += acc[mi][mj][rg] * dk_sqexp(p, xi, xc[t * NB + 64 * wj + 16 * mj + fr + 4 * rg], tbl);
                }
            } else if (kind == GAPLAC_OU) {
                const double p = tp.p[t];
#pragma unroll
                for (int mi = 0; mi < 4; ++mi) {
                    const double xi = xr[t * NB + 64 * wi + 16 * mi + fc];
#pragma unroll
                    for (int mj = 0; mj < 4; ++mj)
#pragma unroll
                        for (int rg = 0; rg < 4; ++rg)
                            g += acc[mi][mj][rg] * dk_ou(p, xi, xc[t * NB + 64 * wj + 16 * mj + fr + 4 * rg], tbl);
                }
            } else if (kind == GAPLAC_LINEAR) {  // d/dc (x_i x_j + c) = 1
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int mj = 0; mj < 4; ++mj)
#pragma unroll
                        for (int rg = 0; rg < 4; ++rg) g += acc[mi][mj][rg];
            } else if (kind == GAPLAC_NOISE) {  // a Noise term's variance, and (t = T) the observation noise
                g = diag_sum();
            }  // Cat: no parameter
            const double x = wave_sum(g);
            if (lane == 0) red[w * (T + 1) + t] = x;
        }
        __syncthreads();
        if (tid <= T) {
            const int64_t b = (int64_t)I * (I + 1) / 2 + J;
            const int S = T + 1;
            partial[b * S + tid] = (red[tid] + red[S + tid]) + (red[2 * S + tid] + red[3 * S + tid]);
        }
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

// =================================================================================
// Persistent tail: the last T <= TAIL_TMAX tile columns ts .. nt-1
// of the factorisation in ONE launch, as a dataflow of tile tasks instead of per-column
// kernel launches (the serial tail paid the full K = 128 update of the remaining triangle
// and three launch boundaries per column on its critical path):
//   D(k)      diagonal block of tile column k            (potrf_diag2_body)
//   S(i,k,h)  TRSM of rows 64h.. of tile (i,k), i > k   (tail_trsm_pipe, 4 waves x 16
//             rows, block row b as soon as D(k) has published L_kk's rows up to b)
//   U(i,j;k)  tile (i,j) -= L(i,k) L(j,k)^T, k < j <= i  (tail_update, whole tile, or four
//             64x64 quadrant tasks for the tile (k+2,k+1) the next TRSM needs first)
//   Q(i,i;k)  the same for one 32x32 block (10 of them: the lower block triangle) of the
//             next diagonal tile (the critical path; tail_q32)
// Tasks are dequeued from one counter in a fixed order that is a topological order of
// their dependencies (build_tail_tasks): per column the critical set first (the next
// diagonal tile's ten blocks, D, the TRSM behind it and the tile it needs), then the rest
// of the column's TRSMs and updates. A workgroup waits only for tasks dequeued
// before its own, so the earliest unfinished task always has its inputs: no deadlock, and
// no co-residency assumption (a workgroup that never starts holds no task).
// Hand-offs between workgroups (any XCD): the producer stores its tile with sc1
// (write-through) stores, every wave waits vmcnt(0), the workgroup meets a barrier and one
// lane bumps the task's counter with an agent-scope atomic; the consumer's lane 0 polls
// the counters with sc1 loads, the workgroup meets a barrier, and every load of handed-off
// data is an sc1 load (MI355X_MICROARCH.md "Valid forms", table row 1). Every wait is
// bounded (0.2 s); an expired wait sets TailCtl::err, which the host turns into GAPLAC_E_HIP.
// =================================================================================
enum { TK_D = 0, TK_S = 1, TK_U = 2, TK_Q = 3 };
constexpr unsigned long long TAIL_WAIT_TICKS = 20000000ull;  // 0.2 s of the 100 MHz wall clock

__device__ __forceinline__ unsigned tail_ld(const unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
constexpr int TAIL_S_WHOLE = 2;  // S task q: the whole 128-row tile, after D(k) (else q = row half)
constexpr int TAIL_G = 1;        // D-type task q: build Gram tile (i, j) (TailArgs::gX; waits for nothing)
constexpr unsigned TAIL_NQ = 10;  // Q blocks per diagonal tile (= units a diagonal U adds)

// task word: type (2 bits) | q (4) | k (7) | i (7) | j (7), tile indices relative to ts
__host__ __device__ __forceinline__ uint32_t tail_enc(int type, int q, int k, int i, int j) {
    return (uint32_t)type | ((uint32_t)q << 2) | ((uint32_t)k << 6) | ((uint32_t)i << 13) | ((uint32_t)j << 20);
}
constexpr int TAIL_UD = 5;     // U task q: a whole tile with the 4 columns k .. k+3 (K = 512)
constexpr int TAIL_UD8 = 6;    // U task q: a whole tile with the 8 columns k .. k+7 (K = 1024)
constexpr int TAIL_UD2 = 7;    // U task q: a whole tile with the 2 columns k, k+1 (K = 256)
// panel columns a task applies (deep U tasks 2, 4 or 8, every other update 1)
__host__ __device__ __forceinline__ int tail_deep_cols(int type, int q) {
    return type == TK_U ? (q == TAIL_UD ? 4 : q == TAIL_UD8 ? 8 : q == TAIL_UD2 ? 2 : 1) : 1;
}
// units an update task adds to its tile's counter (a tile column's update is 4 units off
// the diagonal, TAIL_NQ = 10 on it). Quadrant tasks q = 1 .. 4 (qi = (q-1) >> 1, qj =
// (q-1) & 1): 1 unit off the diagonal; on it only the lower three run, holding 3, 4 and 3
// of the ten lower 32x32 blocks (q = 2, the upper quadrant, is never listed there).
__host__ __device__ __forceinline__ unsigned tail_unit_add(int type, int q, int i, int j) {
    const unsigned whole = i == j ? TAIL_NQ : 4u;
    if (type == TK_Q) return 1u;
    if (q == 0) return whole;
    const int nk = tail_deep_cols(type, q);
    if (nk > 1) return (unsigned)nk * whole;
    return i != j ? 1u : q == 3 ? 4u : q == 2 ? 0u : 3u;
}

// Progress of a sub-diagonal TRSM's 16-row group (its wave's stores of blocks < nb
// complete: the caller has waited vmcnt past them), for the Q blocks behind it.
__device__ __forceinline__ void tail_sprog(unsigned* sp, unsigned nb) {
    if ((threadIdx.x & 63) == 0) __hip_atomic_store(sp, nb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Stage L_kk's 28 strictly-lower 16x16 blocks and the 8 inverses in LDS for the tail's
// TRSM: block (b, c), c < b, at p = b(b-1)/2 + c, Ls[p*256 + m*16 + j] = L(16b + j, 16c + m);
// inverses at p = 28 + b. Half the block (tid >> 8) takes the even p, half the odd; every
// address is a select between two compile-time block positions, so the 18 loads of a
// thread are issued back to back (a data-dependent decode here put a divergent branch and
// a full vmcnt wait around every load: 11 us of the task, round 3).
__host__ __device__ constexpr int tri_b_of(int p) {
    int b = 1;
    while ((b + 1) * b / 2 <= p) ++b;
    return b;
}
template <int AUX>
__device__ __forceinline__ void tail_trsm_stage(double* Ls, const Gm<AUX>& gA, const Gm<AUX>& gD, int64_t lda,
                                                int64_t k0, int tid) {
    const int e = tid & 255, m = e >> 4, j = e & 15;
    const bool odd = (tid >> 8) != 0;
    double x[18];
#pragma unroll
    for (int hh = 0; hh < 14; ++hh) {
        const int p0 = 2 * hh, p1 = 2 * hh + 1;
        const int b0 = tri_b_of(p0), b1 = tri_b_of(p1);
        const int c0 = p0 - b0 * (b0 - 1) / 2, c1 = p1 - b1 * (b1 - 1) / 2;
        const int b = odd ? b1 : b0, c = odd ? c1 : c0;
        x[hh] = gA.ld((uint32_t)((16 * c + m) * lda + k0 + 16 * b + j));
    }
#pragma unroll
    for (int hh = 14; hh < 18; ++hh) x[hh] = gD.ld((uint32_t)((2 * hh + (odd ? 1 : 0) - TRSM_LBLK) * 256 + e));
#pragma unroll
    for (int hh = 0; hh < 18; ++hh) Ls[(2 * hh + (odd ? 1 : 0)) * 256 + e] = x[hh];
}

// TRSM of rows 64h .. 64h+63 of tile (bi, k): X = B L_kk^{-T} by blocked substitution
// (trsm_subst_kernel_body's arithmetic). Waves 0-3 (one per SIMD, so the four dependent
// MFMA chains do not share a matrix pipe) own 16 rows each; all 8 waves stage L_kk's 28
// strictly-lower 16x16 blocks and the 8 inverses in LDS.
template <int AUX>
__device__ __forceinline__ void tail_trsm(double* smem, double* Acol, int64_t lda, int k, int bi, int h,
                                          const double* Dk, unsigned* sprog = nullptr) {
    double* Ls = smem;  // (TRSM_LBLK + NDB) x 256
    const int tid = otid(), wave = tid >> 6, lane = tid & 63;
    const int fr = lane >> 4, fc = lane & 15;
    const int64_t k0 = (int64_t)k * NB;
    const Gm<AUX> gA(Acol), gD(Dk);
    // h = 0, 1: rows 64h .. 64h+63 on waves 0-3; h = 2 (TAIL_S_WHOLE): the whole tile, 16
    // rows per wave on all eight (two independent substitution chains per SIMD)
    const bool whole = h == 2;
    const uint32_t rowb = (uint32_t)((int64_t)bi * NB + (whole ? 16 * wave : 64 * h + 16 * (wave & 3)));
    d4 Bt[NDB];
    if (wave < 4 || whole) {
#pragma unroll
        for (int b = 0; b < NDB; ++b)
#pragma unroll
            for (int q = 0; q < 4; ++q) Bt[b][q] = gA.ld((uint32_t)((int64_t)(16 * b + fr + 4 * q) * lda + rowb + fc));
    }
    tail_trsm_stage(Ls, gA, gD, lda, k0, tid);
    __syncthreads();
    if (wave >= 4 && !whole) return;
    d4 Y[NDB];
#pragma unroll
    for (int b = 0; b < NDB; ++b) {
        d4 s0 = Bt[b], s1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int c = 0; c < b; ++c) {
            const double* Lbc = Ls + (b * (b - 1) / 2 + c) * 256;
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                const double lbc = Lbc[(4 * kk + fr) * 16 + fc];  // negated by the MFMA (neg A)
                if (c & 1)
                    s1 = __builtin_amdgcn_mfma_f64_16x16x4f64(lbc, Y[c][kk], s1, 0, 0, 1);
                else
                    s0 = __builtin_amdgcn_mfma_f64_16x16x4f64(lbc, Y[c][kk], s0, 0, 0, 1);
            }
        }
        s0 += s1;
        const double* Di = Ls + (TRSM_LBLK + b) * 256;
        d4 y = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
            y = __builtin_amdgcn_mfma_f64_16x16x4f64(Di[(4 * kk + fr) * 16 + fc], s0[kk], y, 0, 0, 0);
        Y[b] = y;
#pragma unroll
        for (int q = 0; q < 4; ++q) gA.st((uint32_t)((int64_t)(16 * b + fr + 4 * q) * lda + rowb + fc), y[q]);
        if (sprog && b >= 2) {  // blocks < b-1 stored (blocks b-1 and b's stores may be in flight)
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            tail_sprog(&sprog[(rowb / 16) & 7], (unsigned)(b - 1));
        }
    }
    if (sprog) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        tail_sprog(&sprog[(rowb / 16) & 7], (unsigned)NDB);
    }
}

// The same TRSM pipelined behind the diagonal block: it may start while D(k) is still
// running. Waves 4-7 stage block row b of L_kk (blocks (b, c), c < b) and Dinv_b as soon as
// D(k) has published them (prog >= b + 1: potrf_diag2_body's progress counter, b <= 6;
// row 7 when D(k) is done), each wave the blocks c = w - 4 (mod 4), then mark the row in
// LDS (rowf[b] counts the four waves); waves 0-3 (16 rows each) take rows as they arrive:
// Y_b = Dinv_b (B_b - sum_{c<b} L_bc Y_c), the arithmetic of tail_trsm. The chain after
// D(k) ends is the last two rows instead of the whole substitution.
template <int AUX>
__device__ __forceinline__ void tail_trsm_pipe(double* smem, unsigned* rowf, double* Acol, int64_t lda, int k, int bi,
                                               int h, const double* Dk, const unsigned* prog, const unsigned* ddone,
                                               unsigned* err, unsigned* rerr, unsigned* sprog = nullptr) {
    double* Ls = smem;  // (TRSM_LBLK + NDB) x 256, as tail_trsm_stage lays it out
    const int tid = otid(), wave = tid >> 6, lane = tid & 63;
    const int fr = lane >> 4, fc = lane & 15;
    const int64_t k0 = (int64_t)k * NB;
    const Gm<AUX> gA(Acol), gD(Dk);
    if (tid < NDB) rowf[tid] = 0u;
    __syncthreads();
    if (wave >= 4) {
        const int w = wave - 4;
        bool timeout = false;
        int next = 0;  // first row not staged yet
        while (next < NDB) {
            // lane 0 polls D(k)'s progress (sc1 loads), bounded; the wave follows its verdict:
            // rows next .. avail-1 are final (row b <= 6 needs prog >= b + 1, row 7 D done)
            int avail = 0;
            if (lane == 0) {
                const unsigned long long t0 = wall_clock64();
                for (unsigned it = 1;; ++it) {
                    if (__hip_atomic_load(ddone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
                        avail = NDB;
                    } else {
                        const int pr = (int)__hip_atomic_load(prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        avail = pr < NDB - 1 ? pr : NDB - 1;
                    }
                    if (avail > next) break;
                    // expired (or, checked every 32 polls off the fast path, another task
                    // already failed): stage what is there, flag it
                    if (wall_clock64() - t0 > TAIL_WAIT_TICKS || ((it & 31u) == 0u && tail_ld(err) != 0u)) {
                        avail = NDB;
                        timeout = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
            }
            avail = __builtin_amdgcn_readfirstlane(avail);
            // every block c = w, w + 4, ... <= b of the rows b in [next, avail) (c == b: Dinv_b)
            // by LDS-DMA (global_load_lds, 16 B per lane: half a block per instruction, the
            // LDS image lane-linear), all in flight together, then one wait
            for (int b = next; b < avail; ++b) {
                for (int c = w; c <= b; c += 4) {
                    const int p = c < b ? b * (b - 1) / 2 + c : TRSM_LBLK + b;
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const int q = 64 * u + lane, m = q >> 3, j = 2 * (q & 7);  // pair q = (m, j..j+1)
                        const double* src = c < b ? Acol + (int64_t)(16 * c + m) * lda + k0 + 16 * b + j
                                                  : Dk + b * 256 + 2 * q;
                        __builtin_amdgcn_global_load_lds((GlobalCPtr)src, (LdsPtr)(Ls + p * 256 + 128 * u), 16, 0, AUX);
                    }
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0)
                for (int b = next; b < avail; ++b)
                    __hip_atomic_fetch_add(&rowf[b], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            next = avail;
        }
        if (timeout && lane == 0) {
            atomicOr(err, 1u);
            atomicOr(rerr, 2u);  // straight into the result record (no exit-time read needed)
        }
        return;
    }
    const uint32_t rowb = (uint32_t)((int64_t)bi * NB + 64 * h + 16 * wave);
    d4 Bt[NDB];
#pragma unroll
    for (int b = 0; b < NDB; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) Bt[b][q] = gA.ld((uint32_t)((int64_t)(16 * b + fr + 4 * q) * lda + rowb + fc));
    d4 Y[NDB];
#pragma unroll
    for (int b = 0; b < NDB; ++b) {
        // row b staged by all four staging waves. Bounded: 2^23 polls of at least one
        // s_sleep(1) (64 clocks) each, > 0.25 s, longer than the staging waves' own 0.2 s
        // wall-clock bound (they always get here: a timed-out wait above stages stale data and
        // flags it); an expiry here flags the evaluation too, never a silent result. (The
        // wall clock is not read per poll: on this chain's critical path that cost ~10%.)
        {
            bool got = false;
            for (int it = 0; it < (1 << 23); ++it) {
                if (__hip_atomic_load(&rowf[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= 4u) {
                    got = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (!got && lane == 0) {
                atomicOr(err, 1u);
                atomicOr(rerr, 2u);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        d4 s0 = Bt[b], s1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int c = 0; c < b; ++c) {
            const double* Lbc = Ls + (b * (b - 1) / 2 + c) * 256;
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                const double lbc = Lbc[(4 * kk + fr) * 16 + fc];  // negated by the MFMA (neg A)
                if (c & 1)
                    s1 = __builtin_amdgcn_mfma_f64_16x16x4f64(lbc, Y[c][kk], s1, 0, 0, 1);
                else
                    s0 = __builtin_amdgcn_mfma_f64_16x16x4f64(lbc, Y[c][kk], s0, 0, 0, 1);
            }
        }
        s0 += s1;
        const double* Di = Ls + (TRSM_LBLK + b) * 256;
        d4 y = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
            y = __builtin_amdgcn_mfma_f64_16x16x4f64(Di[(4 * kk + fr) * 16 + fc], s0[kk], y, 0, 0, 0);
        Y[b] = y;
#pragma unroll
        for (int q = 0; q < 4; ++q) gA.st((uint32_t)((int64_t)(16 * b + fr + 4 * q) * lda + rowb + fc), y[q]);
        if (sprog && b >= 2) {  // blocks < b-1 stored (blocks b-1 and b's stores may be in flight)
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            tail_sprog(&sprog[4 * h + wave], (unsigned)(b - 1));
        }
    }
    if (sprog) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        tail_sprog(&sprog[4 * h + wave], (unsigned)NDB);
    }
}

// C -= P Q^T over the K = 128 KD columns of tile columns k .. k+KD-1 (contiguous in
// storage; the k-steps in order, so a deep update rounds exactly as KD successive ones),
// for a region of RB*32 rows x CB*64
// columns of tile column j (whole tile: RB = 4, CB = 2; quadrant: RB = 2, CB = 1). 8 waves
// as 2 (rows) x 4 (columns), each RB x CB blocks of 16x16; fragments straight from global
// (sc1), two groups of 4 k-steps in flight. P rows start at row0, Q rows at qrow0 (global
// rows of the panel), C columns at ccol0 within tile column j's storage.
template <int AUX, int RB, int CB, int KD = 1>
__device__ __forceinline__ void tail_update(const Gm<AUX>& gC, const Gm<AUX>& gP, int64_t lda, int row0, int ccol0,
                                            int qrow0) {
    const int tid = otid(), wave = tid >> 6, lane = tid & 63;
    const int fr = lane >> 4, fc = lane & 15;
    const int wr = wave & 1, wc = wave >> 1;
    const int r0 = row0 + wr * RB * 16, c0 = ccol0 + wc * CB * 16, q0 = qrow0 + wc * CB * 16;
    d4 acc[RB][CB];
#pragma unroll
    for (int mi = 0; mi < RB; ++mi)
#pragma unroll
        for (int mj = 0; mj < CB; ++mj)
#pragma unroll
            for (int rg = 0; rg < 4; ++rg)
                acc[mi][mj][rg] = gC.ld((uint32_t)((int64_t)(c0 + 16 * mj + fr + 4 * rg) * lda + r0 + 16 * mi + fc));
    constexpr int G = 4;  // k-steps per group
    double fa[2][G][CB], fb[2][G][RB];
    auto load = [&](int buf, int g) {
#pragma unroll
        for (int st = 0; st < G; ++st) {
            const int64_t col = (int64_t)(4 * (G * g + st) + fr) * lda;
#pragma unroll
            for (int mi = 0; mi < RB; ++mi) fb[buf][st][mi] = gP.ld((uint32_t)(col + r0 + 16 * mi + fc));
#pragma unroll
            for (int mj = 0; mj < CB; ++mj) fa[buf][st][mj] = gP.ld((uint32_t)(col + q0 + 16 * mj + fc));
        }
    };
    auto compute = [&](int buf) {
#pragma unroll
        for (int st = 0; st < G; ++st)
#pragma unroll
            for (int mi = 0; mi < RB; ++mi) {
                const double b = fb[buf][st][mi];  // negated by the MFMA (neg B)
#pragma unroll
                for (int mj = 0; mj < CB; ++mj)
                    acc[mi][mj] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[buf][st][mj], b, acc[mi][mj], 0, 0, 2);
            }
    };
    constexpr int NG = KD * NB / (4 * G);  // 8 groups per 128 panel columns
    load(0, 0);
#pragma unroll 1
    for (int g = 0; g < NG; g += 2) {
        load(1, g + 1);
        compute(0);
        if (g + 2 < NG) load(0, g + 2);
        compute(1);
    }
#pragma unroll
    for (int mi = 0; mi < RB; ++mi)
#pragma unroll
        for (int mj = 0; mj < CB; ++mj)
#pragma unroll
            for (int rg = 0; rg < 4; ++rg)
                gC.st((uint32_t)((int64_t)(c0 + 16 * mj + fr + 4 * rg) * lda + r0 + 16 * mi + fc), acc[mi][mj][rg]);
}

// (An LDS-staged whole-tile variant of tail_update, panels moved once per workgroup by
// LDS-DMA instead of per wave from L2, was measured in round 3 and not kept)
// One 32x32 block of C -= P Q^T, K = 128 (the critical diagonal-tile update, split ten
// ways): waves 0-3 take one 16x16 sub-block each and load all 32 k-steps of their two
// fragments before the first MFMA, so the handed-off panel's memory latency is paid once.
// Each accumulator starts from C and takes the k-steps in order: the same rounding as the
// per-column chain kernels, so a matrix factored in the tail and through super-panels
// (gradient / posterior workspaces) gives bitwise the same factor.
// Pipelined behind the sub-diagonal TRSM (sprog: its per-16-row-group progress, round 5;
// only the next diagonal tile's blocks, i = k + 1: a Q block of a later diagonal tile gets
// sprog = nullptr and was dispatched after its TRSM finished):
// the k-steps of column block b are loaded once both 16-row groups this wave reads have
// stored block b, so the block's last MFMAs follow the TRSM's end instead of its publish.
// Bounded like the TRSM's own row wait (2^23 polls); an expiry flags the evaluation.
template <int AUX>
__device__ __forceinline__ void tail_q32(const Gm<AUX>& gC, const Gm<AUX>& gP, int64_t lda, int row0, int ccol0,
                                         int qrow0, const unsigned* sprog, int grow, unsigned* err, unsigned* rerr) {
    const int tid = otid(), wave = tid >> 6, lane = tid & 63;
    if (wave >= 4) return;
    const int fr = lane >> 4, fc = lane & 15;
    const int r0 = row0 + 16 * (wave & 1), c0 = ccol0 + 16 * (wave >> 1), q0 = qrow0 + 16 * (wave >> 1);
    // 16-row groups (within the tile) of the P rows and the Q rows
    const int ga = ((r0 - grow) >> 4) & 7, gb = ((q0 - grow) >> 4) & 7;
    d4 acc;
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) acc[rg] = gC.ld((uint32_t)((int64_t)(c0 + fr + 4 * rg) * lda + r0 + fc));
    unsigned have = sprog ? 0u : (unsigned)NDB;  // blocks both groups have stored (no sprog: all, waited before)
#pragma unroll
    for (int b = 0; b < NDB; ++b) {
        if (have <= (unsigned)b) {  // lane 0 polls (light on the TRSM's counters), the wave follows
            if (lane == 0) {
                bool got = false;
                for (int it = 0; it < (1 << 23); ++it) {
                    const unsigned x = tail_ld(&sprog[ga]), y = tail_ld(&sprog[gb]);
                    have = x < y ? x : y;
                    if (have > (unsigned)b) {
                        got = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                if (!got) {
                    have = (unsigned)NDB;  // expired: go on with what is there, flagged
                    atomicOr(err, 1u);
                    atomicOr(rerr, 2u);
                }
            }
            have = (unsigned)__builtin_amdgcn_readfirstlane((int)have);
        }
        double fa[4], fb[4];
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            const int64_t col = (int64_t)(16 * b + 4 * st + fr) * lda;
            fb[st] = gP.ld((uint32_t)(col + r0 + fc));
            fa[st] = gP.ld((uint32_t)(col + q0 + fc));
        }
#pragma unroll
        for (int st = 0; st < 4; ++st) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[st], fb[st], acc, 0, 0, 2);  // neg B
    }
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) gC.st((uint32_t)((int64_t)(c0 + fr + 4 * rg) * lda + r0 + fc), acc[rg]);
}

// Lane 0: wait until the task's inputs are final (bounded: 0.2 s of the 100 MHz clock).
// Returns false when the bound expires or another task has already failed (TailCtl::err
// set: then every later wait returns at once and the launch drains quickly).
__device__ __forceinline__ bool tail_wait(const TailCtl* c, int type, int q, int k, int i, int j, bool gram) {
    if (type == TK_D && q == TAIL_G) return true;
    const unsigned long long t0 = wall_clock64();
    // the Gram inside the tail: a tile's first-column tasks (k = 0) find it built first
    const int gt = !gram || k != 0 ? -1 : type == TK_D ? 0 : type == TK_S ? i * TAIL_TMAX : i * TAIL_TMAX + j;
    for (unsigned it = 1;; ++it) {
        bool ok = gt < 0 || tail_ld(&c->gdone[gt]) != 0u;
        if (!ok) {
        } else if (type == TK_D) {
            ok = tail_ld(&c->units[k * TAIL_TMAX + k]) >= TAIL_NQ * (unsigned)k;
        } else if (type == TK_S) {  // the block itself; D(k)'s progress inside tail_trsm_pipe
            ok = tail_ld(&c->units[i * TAIL_TMAX + k]) >= 4u * k;
            if (q == TAIL_S_WHOLE && ok) ok = tail_ld(&c->ddone[k]) != 0u;  // not pipelined: D(k) done
        } else {
            const unsigned ups = i == j ? TAIL_NQ : 4u;
            const int nk = tail_deep_cols(type, q);  // panel columns k .. k+nk-1
            ok = tail_ld(&c->units[i * TAIL_TMAX + j]) >= ups * k;
            // (a Q block of the next diagonal tile, i = k + 1, follows its TRSM's progress
            // inside tail_q32; the other Q blocks wait for their TRSM to finish)
            for (int c2 = 0; c2 < nk && ok && !(type == TK_Q && i == k + 1); ++c2)
                ok = tail_ld(&c->sdone[i * TAIL_TMAX + k + c2]) >= 2u && tail_ld(&c->sdone[j * TAIL_TMAX + k + c2]) >= 2u;
        }
        if (ok) return true;
        // the other task's failure is checked every 32 polls, off the fast path
        if (wall_clock64() - t0 > TAIL_WAIT_TICKS || ((it & 31u) == 0u && tail_ld(&c->err) != 0u)) return false;
        __builtin_amdgcn_s_sleep(2);
    }
}

// The tail's diagonal blocks run potrf_diag2_body (round 3); its LDS also holds the TRSM's
// staged L_kk and inverses (tail_trsm_stage: 36 x 256 doubles).
static_assert(DIAG2_SMEM >= (TRSM_LBLK + NDB) * 256, "tail_kernel LDS too small for the TRSM staging");
static_assert(DIAG2_SMEM >= GRAM_LDS, "tail_kernel LDS too small for a Gram tile");
// GRAM: the variant whose list holds the Gram's tile tasks (TailArgs::gX set); the other
// tails (batched lanes, the 16k tail) do not carry its code (its registers cost them
// SGPR spills: select -0.8%, profiles/r07g2_gram_tail_ab.txt)
template <bool GRAM>
__global__ __launch_bounds__(512) void tail_kernel(TailArgs a, KTime* __restrict__ kt) {
    __shared__ double smem[DIAG2_SMEM];
    __shared__ unsigned s_task;
    __shared__ unsigned s_rowf[NDB];
    kt_begin(kt);
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) s_task = atomicAdd(&a.ctl->head, 1u);
        __syncthreads();
        const unsigned tk = s_task;
        if (tk >= (unsigned)a.ntasks) break;
        const uint32_t e = a.tasks[tk];
        const int type = (int)(e & 3u), q = (int)((e >> 2) & 15u), k = (int)((e >> 6) & 127u);
        const int i = (int)((e >> 13) & 127u), j = (int)((e >> 20) & 127u);
        const int m = (int)(e >> TAIL_MODEL_SHIFT);
        TailCtl* ctl = a.ctl + m;
        double* const A = a.A + m * a.a_stride;
        double* const Dinv = a.Dinv + m * a.dinv_stride;
        EvalResult* const res = a.res + m;
        if (a.trace && threadIdx.x == 0) a.trace[3 * tk] = wall_clock64();
        if (threadIdx.x == 0 && !tail_wait(ctl, type, q, k, i, j, GRAM)) {
            atomicOr(&ctl->err, 1u);
            atomicOr(&res->err, 2u);  // the result record itself: the host sees it whatever the exit order
        }
        __syncthreads();
        if (a.trace && threadIdx.x == 0) a.trace[3 * tk + 1] = wall_clock64();
        const int gk = a.ts + k;
        double* colk = A + (int64_t)gk * NB * a.lda;
        // debug (GAPLAC_TAIL_FAULT): D(fault) never runs nor publishes
        const bool faulted = type == TK_D && q == 0 && k == a.fault;
        if (faulted) {
        } else if (GRAM && type == TK_D && q == TAIL_G) {  // Gram tile (i, j), sc1 stores (ts = 0)
            gram_tile<GRAM_CB, 8, GM_SC1>(A + (int64_t)(a.ts + j) * NB * a.lda, a.lda, a.N, a.gX, a.gldx, a.gv, a.gtp,
                                          a.ts + i, a.ts + j, smem);
        } else if (type == TK_D) {
            if ((int64_t)gk * NB < a.N) {
                potrf_diag2_body<GM_SC1>(smem, colk + (int64_t)gk * NB, a.lda, a.N, (int64_t)gk * NB,
                                         Dinv + (size_t)gk * DINV_PER_BLOCK, res, nullptr, &ctl->dprog[k],
                                         a.trace && a.nmodels == 1
                                             ? a.trace + 3 * (size_t)a.ntasks + (size_t)TAIL_DSTAMPS * k
                                             : nullptr);
            }
        } else if (type == TK_S && q == TAIL_S_WHOLE) {
            tail_trsm<GM_SC1>(smem, colk, a.lda, gk, a.ts + i, q, Dinv + (size_t)gk * DINV_PER_BLOCK,
                              i == k + 1 ? ctl->sprog[k] : nullptr);
        } else if (type == TK_S) {
            tail_trsm_pipe<GM_SC1>(smem, s_rowf, colk, a.lda, gk, a.ts + i, q, Dinv + (size_t)gk * DINV_PER_BLOCK,
                                   &ctl->dprog[k], &ctl->ddone[k], &ctl->err, &res->err,
                                   i == k + 1 ? ctl->sprog[k] : nullptr);
        } else {
            const int gi = a.ts + i, gj = a.ts + j;
            const Gm<GM_SC1> gC(A + (int64_t)gj * NB * a.lda), gP(colk);
            if (type == TK_U && q == 0) {
                tail_update<GM_SC1, 4, 2>(gC, gP, a.lda, gi * NB, 0, gj * NB);
            } else if (type == TK_U && q == TAIL_UD) {
                tail_update<GM_SC1, 4, 2, 4>(gC, gP, a.lda, gi * NB, 0, gj * NB);
            } else if (type == TK_U && q == TAIL_UD8) {
                tail_update<GM_SC1, 4, 2, 8>(gC, gP, a.lda, gi * NB, 0, gj * NB);
            } else if (type == TK_U && q == TAIL_UD2) {
                tail_update<GM_SC1, 4, 2, 2>(gC, gP, a.lda, gi * NB, 0, gj * NB);
            } else if (type == TK_U) {  // quadrant q - 1 of an off-diagonal tile
                const int qi = (q - 1) >> 1, qj = (q - 1) & 1;
                tail_update<GM_SC1, 2, 1>(gC, gP, a.lda, gi * NB + 64 * qi, 64 * qj, gj * NB + 64 * qj);
            } else {
                // q = qa (qa + 1) / 2 + qb, qb <= qa: 32x32 block (qa, qb) of the diagonal tile
                const int qa = q >= 6 ? 3 : q >= 3 ? 2 : q >= 1 ? 1 : 0, qb = q - qa * (qa + 1) / 2;
                tail_q32<GM_SC1>(gC, gP, a.lda, gi * NB + 32 * qa, 32 * qb, gj * NB + 32 * qb,
                                 i == k + 1 ? ctl->sprog[k] : nullptr, gi * NB, &ctl->err, &res->err);
            }
        }
        // publish: every wave's stores complete, then one lane bumps the counter
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0 && !faulted) {
            if (GRAM && type == TK_D && q == TAIL_G) {
                __hip_atomic_fetch_add(&ctl->gdone[i * TAIL_TMAX + j], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else if (type == TK_D) {
                __hip_atomic_fetch_add(&ctl->ddone[k], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else if (type == TK_S) {  // two halves per tile (or one whole-tile task): done at 2
                __hip_atomic_fetch_add(&ctl->sdone[i * TAIL_TMAX + k], q == TAIL_S_WHOLE ? 2u : 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            } else {
                __hip_atomic_fetch_add(&ctl->units[i * TAIL_TMAX + j], tail_unit_add(type, q, i, j), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
            if (a.trace) a.trace[3 * tk + 2] = wall_clock64();
        }
    }
    if (threadIdx.x < a.nmodels && tail_ld(&a.ctl[threadIdx.x].err) != 0u) atomicOr(&a.res[threadIdx.x].err, 2u);
    kt_end(kt);
}

void interleave_tail_tasks(const std::vector<uint32_t>& one, const std::vector<size_t>& colstart, int B, int lag,
                           std::vector<uint32_t>& out) {
    out.clear();
    out.reserve(one.size() * (size_t)B);
    auto tag = [](uint32_t e, int m) { return e | ((uint32_t)m << TAIL_MODEL_SHIFT); };
    if (lag <= 0 || colstart.empty()) {
        for (uint32_t e : one)
            for (int m = 0; m < B; ++m) out.push_back(tag(e, m));
        return;
    }
    // column g of the list: [colstart[g], colstart[g+1]) (the last runs to the end)
    const int ncol = (int)colstart.size();
    auto col_end = [&](int g) { return g + 1 < ncol ? colstart[(size_t)g + 1] : one.size(); };
    std::vector<size_t> pos((size_t)B);
    for (int step = 0; step < ncol + lag * (B - 1); ++step) {
        // the models whose current column is step - lag * m, their tasks task by task
        for (int m = 0; m < B; ++m) {
            const int g = step - lag * m;
            pos[(size_t)m] = (g >= 0 && g < ncol) ? colstart[(size_t)g] : 0;
        }
        for (bool any = true; any;) {
            any = false;
            for (int m = 0; m < B; ++m) {
                const int g = step - lag * m;
                if (g < 0 || g >= ncol || pos[(size_t)m] >= col_end(g)) continue;
                out.push_back(tag(one[pos[(size_t)m]++], m));
                any = true;
            }
        }
    }
}

// The Gram inside the tail (single evaluations whose matrix lies whole in the tail): a
// TAIL_G task per lower tile ahead of the list, tile (0, 0) first and D(0) right behind it
// (the chain's start waits only for its own tile), then the other tiles column by column,
// the order in which the list's first-column tasks need them. The ~T^2/2 tile builds run on
// the other workgroups while D(0) factors.
void add_gram_tasks(int T, std::vector<uint32_t>& list) {
    std::vector<uint32_t> out;
    out.reserve(list.size() + (size_t)T * (T + 1) / 2);
    out.push_back(tail_enc(TK_D, TAIL_G, 0, 0, 0));
    const uint32_t d0 = tail_enc(TK_D, 0, 0, 0, 0);
    bool have_d0 = false;
    for (uint32_t e : list) have_d0 = have_d0 || e == d0;
    if (have_d0) out.push_back(d0);
    for (int j = 0; j < T; ++j)
        for (int i = j; i < T; ++i)
            if (i || j) out.push_back(tail_enc(TK_D, TAIL_G, 0, i, j));
    for (uint32_t e : list)
        if (!(have_d0 && e == d0)) out.push_back(e);
    list.swap(out);
}

// Dequeue order of the tail's tasks (see the block comment above). Every task waits only
// for tasks listed before it. Per g = 0 .. T-2 the tasks of column g, the ones the chain
// needs soonest first:
//   S(g+2,g)  Q(g+1,g+1;g) x10  U(g+2,g+1;g) x4 quadrants  D(g+1)  S(g+2,g+1) (pipelined
//   behind D(g+1))  Q(g+2,g+2;g) x10  S(g+3,g)  U(g+3,g+1;g) x4  S(i,g) i >= g+4
//   U(i,g+1;g) x4 i >= g+4  U(i,j;g) for the near tile columns g+2 <= j < 4b+4+NEAR
//   (but (g+2,g+2)), b = g / 4
// after D(0) and S(1,0): the next tile column's tiles are updated in small (quadrant)
// tasks early, so each TRSM, the one behind D(g+1) above all, and the next diagonal
// update find their inputs final instead of queued behind the bulk of column g's updates
// (a tile's S -> U -> S -> ... chain down the sub-diagonals must keep the chain's pace).
// Far tiles (j >= GW b + GW + NEAR) of a complete block b of GW (4 or 8) columns get the
// block's columns in ONE deep task (K = 128 GW: 1/GW of the dequeues, waits, tile loads and
// stores of GW K = 128 tasks): those that turn near in block b+1 right after column
// GW b + GW - 1 (before their first per-column update), the rest spread over the lists of
// the block's next GW columns, nearest tile column first, behind each column's own tasks.
// Single evaluations use GW = 4, NEAR = 4 (latency); batched launches fewer per-column
// updates (throughput).
void build_tail_tasks(int T, std::vector<uint32_t>& out, std::vector<size_t>* colstart, int gw, int near,
                      int quad_last, bool whole_trsm, int group, int xrows, int crit_quads) {
    group = group >= 4 ? 4 : group >= 2 ? 2 : 1;  // divides the deep width (4 or 8): groups stay in a block
    // deep width; near distance (>= 2: the next two diagonal tiles take per-column Q tasks)
    const int GW = gw == 8 ? 8 : 4, NEAR = std::max(2, near);
    const int qdeep = GW == 8 ? TAIL_UD8 : TAIL_UD;
    out.clear();
    if (colstart) colstart->clear();
    auto S = [&](int i, int k) {
        if (i < T)
        {
            if (whole_trsm && k < T - quad_last)
                out.push_back(tail_enc(TK_S, TAIL_S_WHOLE, k, i, 0));  // the whole tile (throughput)
            else
                for (int h = 0; h < 2; ++h) out.push_back(tail_enc(TK_S, h, k, i, 0));  // row halves
        }
    };
    auto Qs = [&](int i, int k) {  // the ten 32x32 blocks of diagonal tile i
        if (i < T)
            for (int q = 0; q < (int)TAIL_NQ; ++q) out.push_back(tail_enc(TK_Q, q, k, i, i));
    };
    auto Uq = [&](int i, int j, int k) {  // quadrants of off-diagonal tile (i, j) (or the whole tile)
        if (i < T) {
            // (the next column's first crit_quads sub-diagonal tiles always in quadrants: the
            // TRSM pipelined behind D(k+1) needs tile (k+2, k+1) within one D)
            if (k < T - quad_last && !(j == k + 1 && i - j <= crit_quads))
                out.push_back(tail_enc(TK_U, 0, k, i, j));
            else
                for (int q = 1; q <= 4; ++q) out.push_back(tail_enc(TK_U, q, k, i, j));
        }
    };
    // block b of GW columns is deep-updated when all its columns update something
    auto deep_block = [&](int b) { return GW * b + GW - 1 <= T - 2; };
    auto far_from = [&](int b) { return GW * b + GW + NEAR; };  // first far tile column
    std::vector<std::vector<uint32_t>> later((size_t)std::max(T, 1));  // spread deep tasks per column
    // Extra rows (xrows > 0), off the chain, at the end of column g's list: their whole-tile
    // TRSMs with column g, column g's update of their tiles in the rest of g's block of 4
    // columns, and at the block's last column ONE K = 512 task per extra tile right of the
    // block (those of the next block at once, the rest spread over the next 4 columns'
    // lists: always before the TRSM of the tile that needs them). The last block, if not
    // followed by a whole block, takes per-column updates throughout.
    auto xcol = [&](int g) {
        if (xrows <= 0) return;
        const int k0 = g - g % 4;
        const bool deep = k0 + 4 <= T - 1;  // a tile column right of the block exists
        const int jend = deep ? k0 + 4 : T;
        for (int e = T; e < T + xrows; ++e) out.push_back(tail_enc(TK_S, TAIL_S_WHOLE, g, e, 0));
        for (int e = T; e < T + xrows; ++e)
            for (int j = g + 1; j < jend; ++j) out.push_back(tail_enc(TK_U, 0, g, e, j));
        if (deep && g == k0 + 3) {
            std::vector<uint32_t> rest;
            for (int j = k0 + 4; j < T; ++j)
                for (int e = T; e < T + xrows; ++e) (j < k0 + 8 ? out : rest).push_back(tail_enc(TK_U, TAIL_UD, k0, e, j));
            const size_t n = rest.size();
            for (size_t x = 0; x < n; ++x) {
                const int col = g + 1 + (int)(x * 4 / std::max<size_t>(n, 1));
                later[(size_t)std::min(col, T - 2)].push_back(rest[x]);
            }
        }
    };
    out.push_back(tail_enc(TK_D, 0, 0, 0, 0));
    S(1, 0);
    for (int g = 0; g + 1 < T; ++g) {
        if (colstart) colstart->push_back(g == 0 ? 0 : out.size());
        const int b = g / GW;
        const int jfar = deep_block(b) ? far_from(b) : T;  // per-column updates below this tile column
        S(g + 2, g);
        Qs(g + 1, g);
        Uq(g + 2, g + 1, g);
        out.push_back(tail_enc(TK_D, 0, g + 1, 0, 0));
        S(g + 2, g + 1);
        Qs(g + 2, g);
        S(g + 3, g);
        Uq(g + 3, g + 1, g);
        for (int i = g + 4; i < T; ++i) S(i, g);
        for (int i = g + 4; i < T; ++i) Uq(i, g + 1, g);
        // near tiles: column g's update, or (group = 2 / 4 columns, before the latency-shaped
        // end) the group's columns g0 .. g1 in ONE task at g1 for the tiles the chain does not
        // need before then: off the diagonal j >= g1 + 2 (tile column j is next at column
        // j - 1), on it j >= g1 + 3 (it takes Q tasks from column j - 2 on)
        const int r = g % group, g0 = g - r, g1 = g0 + group - 1;
        const bool grouped = group > 1 && g1 <= T - 2 && g1 < T - quad_last;
        const int qgroup = group == 2 ? TAIL_UD2 : group == 4 ? TAIL_UD : TAIL_UD8;
        for (int j = g + 2; j < std::min(jfar, T); ++j)
            for (int i = j; i < T; ++i) {
                if (i == g + 2 && j == g + 2) continue;  // the Q tasks above
                if (grouped && (i == j ? j >= g1 + 3 : j >= g1 + 2)) {
                    if (g == g1) out.push_back(tail_enc(TK_U, qgroup, g0, i, j));
                    continue;
                }
                out.push_back(tail_enc(TK_U, 0, g, i, j));
            }
        for (uint32_t e : later[(size_t)g]) out.push_back(e);
        if (deep_block(b) && g == GW * b + GW - 1) {
            // block b's deep tasks: near in block b+1 -> now; the rest -> columns g+1 .. g+4
            const int k0 = GW * b, jnear = deep_block(b + 1) ? far_from(b + 1) : T;
            std::vector<uint32_t> rest;
            for (int j = jfar; j < T; ++j)
                for (int i = j; i < T; ++i) (j < jnear ? out : rest).push_back(tail_enc(TK_U, qdeep, k0, i, j));
            const size_t n = rest.size();
            for (size_t x = 0; x < n; ++x) {
                const int col = g + 1 + (int)(x * GW / std::max<size_t>(n, 1));
                later[(size_t)std::min(col, T - 2)].push_back(rest[x]);
            }
        }
        xcol(g);
    }
    xcol(T - 1);
}

// simulation constants (build switches for A/Bs): the pipelined consumer's part after its
// producer ends (us), and the share of the grid the simulation schedules (percent)
#ifndef GAPLAC_SIM_PIPE
#define GAPLAC_SIM_PIPE 3.5
#endif
#ifndef GAPLAC_SIM_WPCT
#define GAPLAC_SIM_WPCT 100
#endif
// Reorder a single evaluation's list (no extra rows) by a simulated schedule: the tasks'
// dependencies as tail_wait has them (the TRSMs pipelined behind their diagonal block and
// the next diagonal tile's Q blocks behind their TRSM), durations as measured in the N =
// 4096 task traces, `workers` persistent workgroups, and among ready
// tasks the one with the longest path to the end first. Sorted by simulated start (ties:
// list order) the list stays a topological order: every task starts no earlier than what
// it waits for.
int sim_order_tail_tasks(int T, std::vector<uint32_t>& list, int workers) {
    const int n = (int)list.size();
    if (n == 0 || workers < 1) return 1;
    struct Tk {
        int type, q, k, i, j, nk;
        double dur;
    };
    std::vector<Tk> tk((size_t)n);
    for (int x = 0; x < n; ++x) {
        const uint32_t e = list[(size_t)x];
        Tk& t = tk[(size_t)x];
        t.type = (int)(e & 3u), t.q = (int)((e >> 2) & 15u), t.k = (int)((e >> 6) & 127u);
        t.i = (int)((e >> 13) & 127u), t.j = (int)((e >> 20) & 127u);
        if (t.k >= T || t.i >= T || t.j >= T || (e >> TAIL_MODEL_SHIFT) != 0u) return 1;  // (extra rows, models)
        t.nk = tail_deep_cols(t.type, t.q);
        t.dur = t.type == TK_D ? 24.5 : t.type == TK_S ? 12.0 : t.type == TK_Q ? 5.0
              : t.nk > 1 ? 19.0 * t.nk : t.q == 0 ? 25.0 : 8.4;
    }
    // predecessors; pipelined ones (S behind D, the next tile's Q behind its TRSM) marked
    std::vector<std::vector<int>> pred((size_t)n), succ((size_t)n);
    std::vector<std::vector<int>> pipe((size_t)n);  // the pipelined producers, if any
    std::vector<int> dof((size_t)T, -1);
    std::vector<std::vector<int>> sof((size_t)T * T);
    struct Tile {
        int col = -1;
        std::vector<int> group, prev;
    };
    std::vector<Tile> tile((size_t)T * T);
    for (int x = 0; x < n; ++x) {
        const Tk& t = tk[(size_t)x];
        std::vector<int>& p = pred[(size_t)x];
        if (t.type == TK_D) {
            const Tile& tl = tile[(size_t)t.k * T + t.k];
            p = tl.group;
            dof[(size_t)t.k] = x;
        } else if (t.type == TK_S) {
            p = tile[(size_t)t.i * T + t.k].group;
            if (dof[(size_t)t.k] >= 0) pipe[(size_t)x].push_back(dof[(size_t)t.k]);
            sof[(size_t)t.i * T + t.k].push_back(x);
        } else {
            Tile& tl = tile[(size_t)t.i * T + t.j];
            const int col = t.k + t.nk - 1;
            if (col > tl.col) {
                tl.prev = tl.group;
                tl.group.clear();
                tl.col = col;
            }
            p = tl.prev;
            const bool piped = t.type == TK_Q && t.i == t.k + 1;
            for (int c = 0; c < t.nk; ++c) {
                for (int s : sof[(size_t)t.i * T + t.k + c]) {
                    if (piped)
                        pipe[(size_t)x].push_back(s);
                    else
                        p.push_back(s);
                }
                if (t.i != t.j)
                    for (int s : sof[(size_t)t.j * T + t.k + c]) p.push_back(s);
            }
            tl.group.push_back(x);
        }
        for (int y : pipe[(size_t)x]) p.push_back(y);
        for (int y : p) succ[(size_t)y].push_back(x);
    }
    // longest path to the end (a pipelined consumer adds only its part after the producer)
    auto piped_on = [&](int s, int x) {
        for (int y : pipe[(size_t)s])
            if (y == x) return true;
        return false;
    };
    std::vector<double> rank((size_t)n, 0.0);
    for (int x = n - 1; x >= 0; --x) {
        double m = 0.0;
        for (int s : succ[(size_t)x]) m = std::max(m, rank[(size_t)s] - (piped_on(s, x) ? tk[(size_t)s].dur - GAPLAC_SIM_PIPE : 0.0));
        rank[(size_t)x] = tk[(size_t)x].dur + m;
    }
    // event simulation: a task is ready when its plain predecessors have finished and its
    // pipelined producer has started; it then ends at max(start + dur, producer end + GAPLAC_SIM_PIPE)
    std::vector<int> wait((size_t)n, 0);
    std::vector<double> start((size_t)n, -1.0), fin((size_t)n, 0.0);
    for (int x = 0; x < n; ++x) wait[(size_t)x] = (int)pred[(size_t)x].size();
    using Ev = std::pair<double, int>;  // (time, task): finish events
    std::priority_queue<Ev, std::vector<Ev>, std::greater<Ev>> ends;
    auto cmp = [&](int a, int b) { return rank[(size_t)a] != rank[(size_t)b] ? rank[(size_t)a] < rank[(size_t)b] : a > b; };
    std::priority_queue<int, std::vector<int>, decltype(cmp)> ready(cmp);
    // a pipelined consumer's dependency on its producer is released at the producer's start
    auto release = [&](int y) {
        if (--wait[(size_t)y] == 0) ready.push(y);
    };
    for (int x = 0; x < n; ++x)
        if (wait[(size_t)x] == 0) ready.push(x);
    int free_w = std::max(1, workers * GAPLAC_SIM_WPCT / 100), done = 0;
    double now = 0.0;
    while (done < n) {
        while (free_w > 0 && !ready.empty()) {
            const int x = ready.top();
            ready.pop();
            start[(size_t)x] = now;
            double f = now + tk[(size_t)x].dur;
            for (int y : pipe[(size_t)x]) f = std::max(f, fin[(size_t)y] + GAPLAC_SIM_PIPE);
            fin[(size_t)x] = f;
            --free_w;
            ends.push({f, x});
            for (int s : succ[(size_t)x])
                if (piped_on(s, x)) release(s);
        }
        if (ends.empty()) break;  // (cannot happen for a topological list)
        const Ev ev = ends.top();
        ends.pop();
        now = ev.first;
        ++free_w;
        ++done;
        for (int s : succ[(size_t)ev.second])
            if (!piped_on(s, ev.second)) release(s);
    }
    if (done < n) return 1;  // keep the list as built
    std::vector<int> ord((size_t)n);
    for (int x = 0; x < n; ++x) ord[(size_t)x] = x;
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return start[(size_t)a] < start[(size_t)b]; });
    std::vector<uint32_t> out((size_t)n);
    for (int x = 0; x < n; ++x) out[(size_t)x] = list[(size_t)ord[(size_t)x]];
    std::string why;
    if (!check_tail_tasks(T, out, &why, 0)) return 2;  // keep the list as built
    list.swap(out);
    return 0;
}

// Host check of a task list (gaplac_plan_check's dry walk): run the tasks one at a time in
// list order, each only once its wait condition (tail_wait) holds on the tasks before it,
// i.e. the list is a topological order of the dataflow, and at the end every tile has
// received every column's update exactly once, every TRSM and diagonal block has run.
bool check_tail_tasks(int T, const std::vector<uint32_t>& list, std::string* why, int xrows, bool gram) {
    const int R = T + xrows;  // tile rows (the extra rows below the matrix: TRSMs and updates only)
    std::vector<unsigned> units((size_t)R * T, 0), sdone((size_t)R * T, 0), ddone((size_t)T, 0);
    std::vector<unsigned> built((size_t)T * T, 0);  // Gram tiles built by their tasks (gram)
    auto fail = [&](size_t n, const char* what) {
        char b[160];
        std::snprintf(b, sizeof b, "tail task %zu of %zu (T = %d): %s", n, list.size(), T, what);
        *why = b;
        return false;
    };
    for (size_t n = 0; n < list.size(); ++n) {
        const uint32_t e = list[n];
        const int type = (int)(e & 3u), q = (int)((e >> 2) & 15u), k = (int)((e >> 6) & 127u);
        const int i = (int)((e >> 13) & 127u), j = (int)((e >> 20) & 127u);
        const unsigned whole = i == j ? TAIL_NQ : 4u;
        if (k >= T || i >= R || j >= T || (i >= T && (type == TK_D || type == TK_Q)))
            return fail(n, "task outside the tile range");
        if (type == TK_D && q == TAIL_G) {
            if (!gram || xrows) return fail(n, "a Gram tile task in a list without the Gram inside");
            if (k != 0 || j > i) return fail(n, "a Gram tile task outside the lower tile triangle");
            if (built[(size_t)i * T + j]++) return fail(n, "a Gram tile built twice");
            continue;
        }
        // the Gram inside the tail: a tile's first-column tasks after its Gram tile
        if (gram && k == 0) {
            const int gi = type == TK_D ? 0 : i, gj = type == TK_D ? 0 : type == TK_S ? 0 : j;
            if (!built[(size_t)gi * T + gj]) return fail(n, "a task before its Gram tile");
        }
        if (type == TK_D) {
            if (q != 0) return fail(n, "a diagonal block task of an unknown kind");
            if (units[(size_t)k * T + k] != TAIL_NQ * (unsigned)k) return fail(n, "D before its tile is updated");
            ddone[(size_t)k] += 1;
        } else if (type == TK_S) {
            if (units[(size_t)i * T + k] != 4u * (unsigned)k || i <= k) return fail(n, "S before its tile is updated");
            if (!ddone[(size_t)k]) return fail(n, "S before D is dequeued");  // (pipelined behind D)
            sdone[(size_t)i * T + k] += q == TAIL_S_WHOLE ? 2u : 1u;
        } else {
            const int nk = tail_deep_cols(type, q);
            if (i < j || j <= k + nk - 1) return fail(n, "update of a tile not right of its panel");
            if (units[(size_t)i * T + j] < whole * (unsigned)k) return fail(n, "update before the tile's earlier columns");
            for (int c = 0; c < nk; ++c)
                if (sdone[(size_t)i * T + k + c] < 2u || sdone[(size_t)j * T + k + c] < 2u)
                    return fail(n, "update before its panel TRSMs");
            if (type == TK_U && nk == 1 && q != 0 && (q > 4 || (i == j && q == 2)))
                return fail(n, "an update quadrant that does not exist (or the diagonal tile's upper one)");
            const unsigned add = tail_unit_add(type, q, i, j);
            // a whole-column step must start exactly at column k (no column skipped or repeated)
            if ((type == TK_U && (q == 0 || nk > 1)) && units[(size_t)i * T + j] != whole * (unsigned)k)
                return fail(n, "update repeats or skips a column");
            units[(size_t)i * T + j] += add;
        }
    }
    for (int j = 0; j < T; ++j) {
        if (ddone[(size_t)j] != 1u) return fail(list.size(), "a diagonal block missing or repeated");
        for (int i = j; gram && i < T; ++i)
            if (!built[(size_t)i * T + j]) return fail(list.size(), "a Gram tile never built");
        for (int i = j; i < R; ++i) {
            const unsigned whole = i == j ? TAIL_NQ : 4u;
            if (units[(size_t)i * T + j] != whole * (unsigned)j) return fail(list.size(), "a tile missed an update");
            if (i > j && sdone[(size_t)i * T + j] != 2u) return fail(list.size(), "a TRSM missing or repeated");
        }
    }
    return true;
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

void acct_record(int kind, int j0, int j1, int k0, int k1) {
    LaunchGuard* g = current_guard();
    if (!g || !g->acct) return;
    for (int v : {kind, j0, j1, k0, k1}) g->acct->push_back(v);
}

int acct_panel_col(const double* P, int64_t ld) {
    LaunchGuard* g = current_guard();
    if (!g || !g->base || ld <= 0) return -1;
    const int64_t off = (int64_t)(((intptr_t)P - (intptr_t)g->base) / (intptr_t)sizeof(double));
    return (int)(off / (ld * NB));
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

static int device_cus();

void launch_gram_queue(hipStream_t s, double* A, int64_t lda, int64_t N, int nt, const double* X, int64_t ldx,
                       const double* v, const TermPack* dtp, int w, int w1, int per_cu, EvalResult* res, KTime* kt) {
    w1 = std::min(w1, nt);
    int64_t ntiles, max_b;
    if (w1 >= nt) {
        const int64_t m = nt - w;
        ntiles = m > 0 ? m * (m + 1) / 2 : 0;
        max_b = ntiles > 0 ? w + tri_row(ntiles - 1) : 0;
    } else {
        ntiles = 0;
        for (int c = w; c < w1; ++c) ntiles += nt - c;
        max_b = nt - 1;
    }
    if (ntiles <= 0) return;
    if (!guard_launch("gram_queue_kernel", A, 0, tiles_end(lda, max_b, w1 >= nt ? max_b : w1 - 1))) return;
    const int grid = (int)std::min<int64_t>(ntiles, (int64_t)per_cu * device_cus());
    gram_queue_kernel<<<dim3((unsigned)grid), dim3(256), 0, s>>>(A, lda, N, X, ldx, v, dtp, w, w1, nt, (int)ntiles,
                                                                 res, kt);
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
    acct_record(1, (int)(g0 / NB), (int)(g0 / NB) + 1, 0, 0);
    if (!guard_launch("potrf_diag_kernel", Ablk, 0, tiles_end(lda, 0, 0))) return;
    potrf_diag_kernel<<<dim3(1), dim3(256), 0, s>>>(Ablk, lda, N, g0, Dinv, res, kt);
}

void launch_trsm(hipStream_t s, double* Acol, int64_t lda, int nt, int k, const double* Dinv, KTime* kt) {
    acct_record(1, k, k + 1, 0, 0);
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

// GAPLAC_BULK_BIG=0 keeps every bulk update on tile_syrk_kernel (A/B)
static bool bulk_big_enabled() {
    static const bool on = [] {
        const char* v = std::getenv("GAPLAC_BULK_BIG");
        return !(v && v[0] == '0');
    }();
    return on;
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
    if (a.rect_rows == 0 && a.bi0 == a.lj0 && a.cm.nranks == 1 && a.pn.row0 == 0) {
        const int k0 = acct_panel_col(a.pn.P, a.pn.ld);
        acct_record(0, a.lj0, a.lj0 + (int)max_c + 1, k0, k0 + a.kdepth / NB);
    }
    if (!guard_launch("bulk update", a.C, 0, tiles_end(a.ldc, a.bi0 + max_r, a.lj0 + max_c))) return;
    const int grid = ((a.ntiles + 7) >> 3) << 3;
    if (syrk_is_small(a.ntiles) && !a.whole && !(a.tile_min > 0 && a.ntiles >= a.tile_min))
        quad_bulk_kernel<<<dim3((unsigned)(4 * grid)), dim3(256), 0, s>>>(a, kt);
    else if (a.whole)
        tile_band_kernel<<<dim3((unsigned)grid), dim3(256), 0, s>>>(a, kt);
    else if (bulk_big_enabled() && (a.big > 0 || (a.big < 0 && a.ntiles >= BULK_BIG_TILES)))
        tile_syrk_big_kernel<<<dim3((unsigned)grid), dim3(256), 0, s>>>(a, kt);
    else
        tile_syrk_kernel<<<dim3((unsigned)grid), dim3(256), 0, s>>>(a, kt);
}

void launch_col_update(hipStream_t s, double* C, int64_t ldc, const Panel& pn, int nt, int jb, int lj0,
                       int ncols, int kdepth, KTime* kt) {
    const int m0 = nt - jb;
    if (m0 <= 0 || ncols <= 0) return;
    int tiles = 0;
    for (int c = 0; c < ncols && c < m0; ++c) tiles += m0 - c;
    if (pn.row0 == 0 && jb == lj0) {
        const int k0 = acct_panel_col(pn.P, pn.ld);
        acct_record(0, jb, jb + std::min(ncols, m0), k0, k0 + kdepth / NB);
    }
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

void launch_copy_z(hipStream_t s, const double* A, int64_t lda, int64_t N, double* z) {
    if (N <= 0) return;
    if (!guard_launch("copy_z_kernel", A, 0, (N - 1) * lda + N + 1)) return;
    copy_z_kernel<<<dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s>>>(A, lda, N, z);
}

void launch_alpha(hipStream_t s, const double* A, int64_t lda, int64_t Np, int64_t N, const double* z,
                  double* partial, double* alpha, double* dv) {
    if (N <= 0) return;
    if (!guard_launch("alpha_partial_kernel", A, 0, (N - 1) * lda + Np + N)) return;
    const int nk = (int)((N + 511) / 512);
    alpha_partial_kernel<<<dim3((unsigned)((N + 255) / 256), (unsigned)nk), dim3(256), 0, s>>>(A, lda, Np, N, z,
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

void launch_cinv_contract(hipStream_t s, const double* A, int64_t lda, int64_t Np, int64_t N, const double* X,
                          int64_t ldx, const double* alpha, const TermPack* dtp, const uint32_t* list, int nblocks,
                          double* partial, KTime* kt) {
    if (nblocks <= 0) return;
    const int m = (int)((N + NB - 1) / NB);
    if (!guard_launch("cinv_contract_kernel", A, 0, (Np - 1) * lda + Np + (int64_t)m * NB)) return;
    cinv_contract_kernel<<<dim3((unsigned)nblocks), dim3(256), 0, s>>>(A, lda, Np, N, X, ldx, alpha, dtp, list,
                                                                       partial, kt);
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

void launch_tail(hipStream_t s, const TailArgs& a, int grid, KTime* kt) {
    if (a.ntasks <= 0 || a.T <= 0) return;
    if (a.nmodels == 1) acct_record(2, a.ts, a.ts + a.T, 0, 0);
    if (a.nmodels < 1 || a.nmodels > TAIL_MAX_MODELS ||
        !guard_launch("tail_kernel", a.A, 0,
                      (int64_t)(a.nmodels - 1) * a.a_stride + tiles_end(a.lda, a.ts + a.T + a.xrows - 1, a.ts + a.T - 1)))
        return;
    if (a.gX)
        tail_kernel<true><<<dim3((unsigned)grid), dim3(512), 0, s>>>(a, kt);
    else
        tail_kernel<false><<<dim3((unsigned)grid), dim3(512), 0, s>>>(a, kt);
}

void launch_init_result(hipStream_t s, EvalResult* res) {
    if (!guard_launch("init_result_kernel")) return;
    init_result_kernel<<<dim3(1), dim3(1), 0, s>>>(res);
}

// The result record and the tail's counters in one launch (the Gram inside the tail: the
// evaluation's first launch is then this one, the tail the second; a hipMemsetAsync of the
// counters was two fill launches of ~5 us each on the N = 4096 evaluation's critical path).
// It also stores the evaluation's term descriptor, passed by value, into dtp: that replaces the
// descriptor's host-to-device copy, one more operation on the evaluation's stream.
__global__ __launch_bounds__(256) void init_result_ctl_kernel(EvalResult* res, unsigned* __restrict__ ctl, int nwords,
                                                              const TermPack tp, TermPack* __restrict__ dtp) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        init_result_kernel_body(res);
        *dtp = tp;
    }
    for (int w = (int)(blockIdx.x * 256 + threadIdx.x); w < nwords; w += (int)gridDim.x * 256) ctl[w] = 0u;
}

void launch_init_result_ctl(hipStream_t s, EvalResult* res, TailCtl* ctl, const TermPack& tp, TermPack* dtp) {
    if (!guard_launch("init_result_ctl_kernel")) return;
    static_assert(sizeof(TailCtl) % sizeof(unsigned) == 0, "TailCtl: whole words");
    static_assert(sizeof(TermPack) <= 1024, "TermPack: passed as a kernel argument");
    init_result_ctl_kernel<<<dim3(64), dim3(256), 0, s>>>(res, reinterpret_cast<unsigned*>(ctl),
                                                          (int)(sizeof(TailCtl) / sizeof(unsigned)), tp, dtp);
}

}  // namespace gaplac
