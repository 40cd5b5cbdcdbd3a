// Probe: the bulk tile kernel (tile_syrk_kernel via launch_bulk) alone on the GPU, one
// triangle of m trailing tile rows with a K-deep panel, for a given matrix order (the
// leading dimension): is its per-tile rate a property of the kernel or of the 16k schedule?
// usage: tools/bulk_probe NT M K [reps]   (NT tile columns of storage, lda = 128 NT)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/bin/bulk_probe tools/bulk_probe.hip \
//          gaplac_amd/csrc/gaplac_kernels.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../gaplac_amd/csrc/gaplac_internal.h"

#define CK(x)                                                                                    \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));             \
            exit(1);                                                                             \
        }                                                                                        \
    } while (0)

using namespace gaplac;

// a smooth Gram-like matrix (SqExp of a 1-D coordinate, + 0.1 on the diagonal), column-major
__global__ void fill_gram_kernel(double* A, int64_t Np, double inv_l) {
    const size_t n = (size_t)Np * Np;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int64_t r = (int64_t)(i % Np), c = (int64_t)(i / Np);
        const double d = (double)(r - c) * 10.0 / (double)Np * inv_l;
        A[i] = exp(-0.5 * d * d) + (r == c ? 0.1 : 0.0);
    }
}
// streams over a large buffer (evicts L2 / MALL) between timed launches
__global__ void scrub_kernel(double* B, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        B[i] = B[i] * 0.5 + 1.0;
}

__global__ void fill_kernel(double* A, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned long long h = i * 0x9E3779B97F4A7C15ull;
        h ^= h >> 29;
        h *= 0xBF58476D1CE4E5B9ull;
        h ^= h >> 32;
        A[i] = (double)(h & 0xFFFFF) / 1048576.0 - 0.5;
    }
}

int main(int argc, char** argv) {
    if (argc < 4) {
        printf("usage: bulk_probe NT M K [reps]\n");
        return 2;
    }
    const int nt = atoi(argv[1]), m = atoi(argv[2]), K = atoi(argv[3]);
    const int reps = argc > 4 ? atoi(argv[4]) : 5;
    // mode (argv[5]): 0 random fill (default), 1 Gram-like fill, 2 random fill + a 2 GB
    // scrub before every timed launch (cold L2 / MALL), 3 Gram-like + scrub
    const int mode = argc > 5 ? atoi(argv[5]) : 0;
    const int jb = nt - m;  // the triangle of tile rows/columns jb .. nt-1; panel = columns 0 .. K/128-1
    if (m <= 0 || jb * NB < K || K % 128 != 0) {
        printf("bad sizes: need nt - m >= K / 128\n");
        return 2;
    }
    const int64_t Np = (int64_t)nt * NB;
    const size_t nA = (size_t)Np * Np;
    double* A;
    CK(hipMalloc(&A, nA * 8));
    if (mode & 1)
        fill_gram_kernel<<<4096, 256>>>(A, Np, 1.0 / 1.5);
    else
        fill_kernel<<<4096, 256>>>(A, nA);
    double* scrub = nullptr;
    const size_t nscrub = (size_t)1 << 28;  // 2 GiB
    if (mode & 2) CK(hipMalloc(&scrub, nscrub * 8));
    std::vector<uint32_t> tl((size_t)m * (m + 1) / 2);
    build_tile_list(m, tl.data());
    uint32_t* dtl;
    CK(hipMalloc(&dtl, tl.size() * 4));
    CK(hipMemcpy(dtl, tl.data(), tl.size() * 4, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    const BulkArgs a{A, Np, Panel{A, Np, 0}, dtl, (int)tl.size(), K, jb, jb, ColMap{1, 0, 4}};
    const double flops = 2.0 * NB * NB * (double)K * ((double)m * (m - 1) / 2) + (double)NB * (NB + 1) * K * m;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    launch_bulk(0, a, nullptr);  // warm, and one update from the fill state for the checksum
    CK(hipDeviceSynchronize());
    {
        // bit hash of the trailing columns jb and nt-1 after that one launch (variants of the
        // kernel must agree bitwise)
        std::vector<double> h((size_t)Np * NB);
        unsigned long long hash = 1469598103934665603ull;
        for (int c : {jb, nt - 1}) {
            CK(hipMemcpy(h.data(), A + (size_t)c * NB * Np, h.size() * 8, hipMemcpyDeviceToHost));
            for (int cc = 0; cc < NB; ++cc)
                for (int64_t r = (int64_t)c * NB; r < Np; ++r) {
                    unsigned long long u;
                    memcpy(&u, &h[(size_t)cc * Np + r], 8);
                    hash = (hash ^ u) * 1099511628211ull;
                }
        }
        printf("checksum %016llx\n", hash);
    }
#if GAPLAC_CLOCK
    {  // the clock one launch holds (diagnostic build): 3 launches, each its own slot
        KTime* dk;
        CK(hipMalloc(&dk, 3 * sizeof(KTime)));
        launch_kt_reset(0, dk, 3);
        for (int r = 0; r < 30; ++r) launch_bulk(0, a, nullptr);  // the clock the sustained load holds
        for (int r = 0; r < 3; ++r) launch_bulk(0, a, dk + r);
        KTime hk[3];
        CK(hipMemcpy(hk, dk, sizeof hk, hipMemcpyDeviceToHost));
        for (int r = 0; r < 3; ++r)
            printf("  clock launch %d: %.3f ms %.3f GHz, %llu workgroups, %.0f cycles each\n", r,
                   (hk[r].end - hk[r].start) * 1e-5, (double)hk[r].clk_mt / (double)hk[r].clk_rt * 0.1, hk[r].clk_n,
                   (double)hk[r].clk_mt / (double)(hk[r].clk_n ? hk[r].clk_n : 1));
        CK(hipFree(dk));
    }
#endif
    float best = 1e30f, sum = 0.f;
    for (int r = 0; r < reps; ++r) {
        float ms;
        if (scrub) scrub_kernel<<<8192, 256>>>(scrub, nscrub);
        CK(hipEventRecord(e0));
        launch_bulk(0, a, nullptr);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
        sum += ms;
    }
    printf("mode %d nt %d (lda %lld) m %d K %d tiles %zu: best %.3f ms avg %.3f ms  %.2f TF/s best (%.3f of 78.6)\n", mode, nt,
           (long long)Np, m, K, tl.size(), best, sum / reps, flops / best / 1e9, flops / best / 1e9 / 78.6);
    {
        // sustained: the same launches back to back (no host sync between them), as the
        // evaluation runs them; the chip's clock under a long dense f64 MFMA load
        float ms;
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch_bulk(0, a, nullptr);
        CK(hipEventRecord(e1));
        // (with a scrub this is still back to back: the scrub only runs before single launches)
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double per = ms / reps;
        printf("  sustained %d launches back to back: %.3f ms per launch  %.2f TF/s (%.3f of 78.6)\n", reps, per,
               flops / per / 1e9, flops / per / 1e9 / 78.6);
    }
    CK(hipFree(A));
    return 0;
}
