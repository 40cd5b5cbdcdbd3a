// The tail's TRSM task (both 64-row halves of tile (1, 0): X = B L_00^{-T}) and its 32x32
// diagonal-update task (all 16 blocks of tile (1, 1) -= X X^T) alone on an idle GPU: event
// time and the slowest block's s_memtime cycles. Checked against CPU results computed from
// the GPU's own L_00 and X. Feeds DESIGN.md §3.3 (round 3: a right-looking substitution
// measured the same as the left-looking one; 64x64 quadrant tasks took 6.6 us per block).
#include "../gaplac_amd/csrc/gaplac_kernels.hip"
#include <cmath>
#include <cstdio>
#include <vector>
using namespace gaplac;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ __launch_bounds__(512) void k_left(double* Acol, int64_t lda, const double* Dk, unsigned long long* cyc) {
  __shared__ double smem[DIAG2_SMEM];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  tail_trsm<0>(smem, Acol, lda, 0, 1, blockIdx.x, Dk);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
__global__ __launch_bounds__(512) void k_q32(double* A, int64_t lda, unsigned long long* cyc) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const int qa = blockIdx.x >> 2, qb = blockIdx.x & 3;
  const Gm<0> gC(A + NB * lda), gP(A);
  tail_q32<0>(gC, gP, lda, NB + 32 * qa, 32 * qb, NB + 32 * qb);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  const int Np = 2 * NB;
  std::vector<double> h((size_t)Np * Np, 0.0);
  for (int j = 0; j < Np; ++j)
    for (int i = 0; i < Np; ++i) {
      const double d = (i - j) * 0.013;
      h[(size_t)j * Np + i] = std::exp(-0.5 * d * d) + (i == j ? 0.1 : 0.0);
    }
  double *A, *Dinv; EvalResult* res; unsigned long long* cyc;
  CK(hipMalloc(&A, h.size() * 8)); CK(hipMalloc(&Dinv, 2 * DINV_PER_BLOCK * 8));
  CK(hipMalloc(&res, sizeof(EvalResult))); CK(hipMalloc(&cyc, 16 * 8));
  CK(hipMemcpy(A, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  launch_init_result(0, res);
  launch_potrf_diag(0, A, Np, Np, 0, Dinv, res, nullptr);
  CK(hipDeviceSynchronize());
  std::vector<double> f(h.size());
  CK(hipMemcpy(f.data(), A, f.size() * 8, hipMemcpyDeviceToHost));
  // CPU: X (128 x 128 rows 128.., cols 0..127) = B L^{-T}, row by row forward substitution
  std::vector<double> X(NB * NB);
  for (int r = 0; r < NB; ++r)
    for (int j = 0; j < NB; ++j) {
      double x = f[(size_t)j * Np + NB + r];
      for (int m = 0; m < j; ++m) x -= X[r * NB + m] * f[(size_t)m * Np + j];
      X[r * NB + j] = x / f[(size_t)j * Np + j];
    }
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<double> o(h.size());
  for (int v = 0; v < 1; ++v) {
    float best = 1e9f; unsigned long long bc[2] = {~0ull, ~0ull};
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipMemcpy(A, f.data(), f.size() * 8, hipMemcpyHostToDevice));
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      k_left<<<2, 512>>>(A, Np, Dinv, cyc);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
      unsigned long long c[2]; CK(hipMemcpy(c, cyc, 16, hipMemcpyDeviceToHost));
      for (int q = 0; q < 2; ++q) if (c[q] < bc[q]) bc[q] = c[q];
    }
    CK(hipMemcpy(o.data(), A, o.size() * 8, hipMemcpyDeviceToHost));
    double err = 0.0;
    for (int r = 0; r < NB; ++r)
      for (int j = 0; j < NB; ++j) err = std::fmax(err, std::fabs(o[(size_t)j * Np + NB + r] - X[r * NB + j]));
    printf("%-6s %.1f us (event)  block cycles %llu / %llu (= %.2f / %.2f us at 2.4 GHz)  max err %.2e\n",
           "trsm", best * 1e3, bc[0], bc[1], bc[0] / 2400.0, bc[1] / 2400.0, err);
  }
  // Q: tile (1, 1) -= P P^T with P = the TRSM result (left variant's output)
  std::vector<double> g = o;
  std::vector<double> Cr(NB * NB);
  for (int c = 0; c < NB; ++c)
    for (int r = 0; r < NB; ++r) {
      double x = g[(size_t)(NB + c) * Np + NB + r];
      for (int m = 0; m < NB; ++m) x -= g[(size_t)m * Np + NB + r] * g[(size_t)m * Np + NB + c];
      Cr[c * NB + r] = x;
    }
  for (int v = 1; v < 2; ++v) {
    float best = 1e9f; unsigned long long bc = ~0ull;
    const int nb = 16;
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipMemcpy(A, g.data(), g.size() * 8, hipMemcpyHostToDevice));
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      k_q32<<<nb, 512>>>(A, Np, cyc);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
      unsigned long long c[16]; CK(hipMemcpy(c, cyc, nb * 8, hipMemcpyDeviceToHost));
      unsigned long long mx = 0; for (int q = 0; q < nb; ++q) mx = c[q] > mx ? c[q] : mx;
      if (mx < bc) bc = mx;
    }
    CK(hipMemcpy(o.data(), A, o.size() * 8, hipMemcpyDeviceToHost));
    double err = 0.0;
    for (int c = 0; c < NB; ++c)
      for (int r = c; r < NB; ++r) err = std::fmax(err, std::fabs(o[(size_t)(NB + c) * Np + NB + r] - Cr[c * NB + r]));
    printf("%-6s %.1f us (event)  slowest block %llu cycles (= %.2f us at 2.4 GHz)  max err %.2e\n",
           "q32", best * 1e3, bc, bc / 2400.0, err);
  }
  return 0;
}
