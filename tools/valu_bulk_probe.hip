// Probe: bulk trailing update C -= P Q^T on the fp64 VALU with the column operand in
// SGPRs (v_fma_f64 v, v, s) vs the fp64 MFMA tile kernel, on the first bulk launch of an
// N=16384 evaluation (121 trailing tile rows, K=512), random data. Prints TF/s of both
// and the max difference of their results.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_bulk_probe tools/valu_bulk_probe.hip \
//          gaplac_amd/csrc/gaplac_kernels.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>
#include <cmath>
#include "../gaplac_amd/csrc/gaplac_internal.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); exit(1); } } while (0)

using namespace gaplac;

constexpr int VR = 512;   // rows per block: 4 row tiles, lane rows 128*i + 2*lane + {0,1}
constexpr int VCW = 8;    // columns per wave (SGPR operand: one s_load_dwordx16 per k)
constexpr int VW = 8;     // waves per block -> 64 columns
#ifndef VKC_
#define VKC_ 16
#endif
#ifndef UNR
#define UNR 4
#endif
#define DO_PRAGMA_(x) _Pragma(#x)
#define DO_PRAGMA(x) DO_PRAGMA_(x)
constexpr int VKC = VKC_;   // k-chunk staged in LDS

// block entry: bi (bits 0..10) | lj (11..21) | half (22) | nvalid-1 (23..24)
__global__ __launch_bounds__(512, 1) void valu_bulk_kernel(BulkArgs a) {
    __shared__ double sm[2][VKC][VR];
    const int idx = (int)blockIdx.x;
    if (idx >= a.ntiles) return;
    const uint32_t e = a.tiles[idx];
    const int bi = a.bi0 + (int)(e & 0x7ffu);
    const int lj = a.lj0 + (int)((e >> 11) & 0x7ffu);
    const int h = (int)((e >> 22) & 1u);
    const int nv = (int)((e >> 23) & 3u) + 1;
    const int bj = a.cm.global(lj);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t ldc = a.ldc, ldp = a.pn.ld;
    const int64_t r0 = (int64_t)bi * NB;
    const int64_t gc0 = (int64_t)bj * NB + 64 * h + VCW * wave;  // wave's first global column
    const int64_t sc0 = (int64_t)lj * NB + 64 * h + VCW * wave;  // ... in storage
    double* __restrict__ Cw = a.C + sc0 * ldc + r0 + 2 * lane;
    const double* __restrict__ Pg = a.pn.P + (r0 - a.pn.row0);
    const double* __restrict__ Qw = a.pn.P + (gc0 - a.pn.row0);

    double2 acc[4][VCW];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < VCW; ++j)
            acc[i][j] = i < nv ? *reinterpret_cast<const double2*>(Cw + j * ldc + 128 * i) : double2{0.0, 0.0};

    // fill: thread t -> row pair rp = t & 255, k rows (t >> 8) + 2*it
    const int rp = tid & 255, kq = tid >> 8;
    const bool rv = 2 * rp < 128 * nv;
    double2 st[VKC / 2];
    auto gload = [&](int ch) {
#pragma unroll
        for (int it = 0; it < VKC / 2; ++it) {
            const int64_t col = (int64_t)ch * VKC + kq + 2 * it;
            st[it] = rv ? *reinterpret_cast<const double2*>(Pg + col * ldp + 2 * rp) : double2{0.0, 0.0};
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int it = 0; it < VKC / 2; ++it)
            *reinterpret_cast<double2*>(&sm[buf][kq + 2 * it][2 * rp]) = st[it];
    };
    gload(0);
    lstore(0);
    __syncthreads();
    const int NCH = a.kdepth / VKC;
    for (int ch = 0; ch < NCH; ++ch) {
        const int buf = ch & 1;
        if (ch + 1 < NCH) gload(ch + 1);
        const double* __restrict__ q = Qw + (int64_t)ch * VKC * ldp;
    DO_PRAGMA(unroll UNR)
        for (int kk = 0; kk < VKC; ++kk) {
            double qv[VCW];
#pragma unroll
            for (int j = 0; j < VCW; ++j) qv[j] = q[kk * ldp + j];
            double2 pv[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) pv[i] = *reinterpret_cast<const double2*>(&sm[buf][kk][128 * i + 2 * lane]);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < VCW; ++j) {
                    acc[i][j].x = fma(-pv[i].x, qv[j], acc[i][j].x);
                    acc[i][j].y = fma(-pv[i].y, qv[j], acc[i][j].y);
                }
        }
        if (ch + 1 < NCH) lstore(buf ^ 1);
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (i < nv)
#pragma unroll
            for (int j = 0; j < VCW; ++j) *reinterpret_cast<double2*>(Cw + j * ldc + 128 * i) = acc[i][j];
}

// Blocks of the lower m x m tile triangle (relative tile indices): column tile c, row
// groups starting at c, c+4, ..., two 64-column halves each.
static std::vector<uint32_t> build_blocks(int m) {
    std::vector<uint32_t> out;
    for (int c = 0; c < m; ++c)
        for (int r = c; r < m; r += 4) {
            const int nv = std::min(4, m - r);
            for (int h = 0; h < 2; ++h)
                out.push_back((uint32_t)r | ((uint32_t)c << 11) | ((uint32_t)h << 22) | ((uint32_t)(nv - 1) << 23));
        }
    return out;
}

int main(int argc, char** argv) {
    const int nt = 129, Np = nt * NB, K = 512, jb = 8, m = nt - jb;
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    const size_t nA = (size_t)Np * Np;
    std::vector<double> h(nA);
    std::mt19937_64 g(1);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    for (auto& x : h) x = U(g);
    double *A0, *A1, *A2;
    CK(hipMalloc(&A0, nA * 8)); CK(hipMalloc(&A1, nA * 8)); CK(hipMalloc(&A2, nA * 8));
    CK(hipMemcpy(A0, h.data(), nA * 8, hipMemcpyHostToDevice));
    // MFMA tile list
    std::vector<uint32_t> tl((size_t)m * (m + 1) / 2);
    build_tile_list(m, tl.data());
    std::vector<uint32_t> bl = build_blocks(m);
    uint32_t *dtl, *dbl;
    CK(hipMalloc(&dtl, tl.size() * 4)); CK(hipMalloc(&dbl, bl.size() * 4));
    CK(hipMemcpy(dtl, tl.data(), tl.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dbl, bl.data(), bl.size() * 4, hipMemcpyHostToDevice));
    const ColMap cm{1, 0, 4};
    auto args = [&](double* A, const uint32_t* list, int n) {
        return BulkArgs{A, (int64_t)Np, Panel{A, (int64_t)Np, 0}, list, n, K, jb, jb, cm};
    };
    // correctness: one launch each from the same start
    CK(hipMemcpy(A1, A0, nA * 8, hipMemcpyDeviceToDevice));
    CK(hipMemcpy(A2, A0, nA * 8, hipMemcpyDeviceToDevice));
    launch_bulk(0, args(A1, dtl, (int)tl.size()), nullptr);
    valu_bulk_kernel<<<dim3((unsigned)bl.size()), dim3(512)>>>(args(A2, dbl, (int)bl.size()));
    CK(hipDeviceSynchronize());
    std::vector<double> h1(nA), h2(nA);
    CK(hipMemcpy(h1.data(), A1, nA * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), A2, nA * 8, hipMemcpyDeviceToHost));
    double md = 0, mref = 0;
    for (int c = jb * NB; c < Np; ++c)
        for (int r = (c / NB) * NB; r < Np; ++r) {
            // skip upper part of diagonal tiles (MFMA kernel leaves one quadrant untouched)
            if (r / NB == c / NB && r < c) continue;
            const size_t o = (size_t)c * Np + r;
            md = std::max(md, std::fabs(h1[o] - h2[o]));
            mref = std::max(mref, std::fabs(h1[o] - h[o]));
        }
    printf("max |mfma - valu| = %.3e (max update %.3e)\n", md, mref);
    const double flops_tri = 2.0 * NB * NB * (double)K * ((double)m * (m - 1) / 2) + (double)NB * (NB + 1) * K * m;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int pass = 0; pass < 2; ++pass) {
        float ms;
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch_bulk(0, args(A1, dtl, (int)tl.size()), nullptr);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
        printf("mfma tile kernel: %.3f ms/launch  %.2f TF/s (triangle flops)\n", ms / reps, flops_tri / (ms / reps) / 1e9);
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r)
            valu_bulk_kernel<<<dim3((unsigned)bl.size()), dim3(512)>>>(args(A2, dbl, (int)bl.size()));
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
        printf("valu sgpr kernel: %.3f ms/launch  %.2f TF/s (triangle flops; %zu blocks)\n", ms / reps,
               flops_tri / (ms / reps) / 1e9, bl.size());
    }
    return 0;
}
