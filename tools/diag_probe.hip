// Diagnostic: the diagonal-block kernel on an idle GPU. Checks it against a CPU Cholesky of
// the same 128x128 block (L and the 16x16 inverses), prints its per-wave stamps per panel
// (the "v1" lines; the blocked 16x16-leaf variant that was "v2" was measured slower and
// removed), and times the other chain kernels alone.
#define GAPLAC_STAMPS 1
#include "../gaplac_amd/csrc/gaplac_kernels.hip"
#include <cmath>
#include <cstdio>
#include <vector>
using namespace gaplac;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ __launch_bounds__(256) void diag_v1(double* Ag, int64_t lda, int64_t N, int64_t g0, double* Dinv, EvalResult* res) {
  potrf_diag_kernel_body(Ag, lda, N, g0, Dinv, res);
}

int main() {
  const int nt = 4, Np = nt * NB;
  std::vector<double> h((size_t)Np * Np, 0.0);
  for (int j = 0; j < Np; ++j)
    for (int i = 0; i < Np; ++i) {
      double d = (i - j) * 0.013 + 0.001 * ((i * 7 + j * 3) % 11 == 0 && i != j ? 0 : 0);
      h[(size_t)j * Np + i] = std::exp(-0.5 * d * d) + (i == j ? 0.1 : 0.0);
    }
  // CPU reference: lower Cholesky of the leading 128x128 block
  std::vector<double> L(NB * NB, 0.0);
  for (int j = 0; j < NB; ++j) {
    double s = h[(size_t)j * Np + j];
    for (int k = 0; k < j; ++k) s -= L[k * NB + j] * L[k * NB + j];
    const double d = std::sqrt(s);
    L[j * NB + j] = d;
    for (int i = j + 1; i < NB; ++i) {
      double x = h[(size_t)j * Np + i];
      for (int k = 0; k < j; ++k) x -= L[k * NB + i] * L[k * NB + j];
      L[j * NB + i] = x / d;
    }
  }
  double *A, *Dinv; EvalResult* res;
  CK(hipMalloc(&A, h.size() * 8)); CK(hipMalloc(&Dinv, nt * DINV_PER_BLOCK * 8));
  CK(hipMalloc(&res, sizeof(EvalResult)));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<double> out(h.size()), dinv(DINV_PER_BLOCK);
  for (int v = 1; v <= 1; ++v) {
    for (int rep = 0; rep < 4; ++rep) {
      CK(hipMemcpy(A, h.data(), h.size() * 8, hipMemcpyHostToDevice));
      launch_init_result(0, res);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      if (v == 1) diag_v1<<<1, 256>>>(A, Np, 1 << 30, 0, Dinv, res);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      CK(hipMemcpy(out.data(), A, out.size() * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(dinv.data(), Dinv, dinv.size() * 8, hipMemcpyDeviceToHost));
      EvalResult hr; CK(hipMemcpy(&hr, res, sizeof hr, hipMemcpyDeviceToHost));
      double errL = 0, errD = 0;
      for (int j = 0; j < NB; ++j)
        for (int i = j; i < NB; ++i) errL = std::fmax(errL, std::fabs(out[(size_t)j * Np + i] - L[j * NB + i]));
      // Dinv_b * L_bb = I
      for (int b = 0; b < 8; ++b)
        for (int c = 0; c < 16; ++c)
          for (int r = 0; r < 16; ++r) {
            double s = 0;
            for (int m = 0; m < 16; ++m) s += dinv[b * 256 + m * 16 + r] * (m >= c ? L[(16 * b + c) * NB + 16 * b + m] : 0.0);
            errD = std::fmax(errD, std::fabs(s - (r == c ? 1.0 : 0.0)));
          }
      printf("diag v%d: %.1f us (event)  max|L-Lcpu| %.2e  max|Dinv L - I| %.2e  info %llx\n", v, ms * 1e3, errL, errD,
             (unsigned long long)hr.info);
      if (v == 1 && rep == 3) {  // v1: per panel s, phase 2 of each wave (cycles, s_memtime)
        unsigned long long st[128]; CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamps), sizeof st));
        printf("  v1 load %llu\n", st[0] - st[20]);
        for (int s = 0; s < 8; ++s) {
          const unsigned long long p2 = st[1 + 2 * s];
          printf("  v1 s=%d: phase1+barrier %5llu | phase2 w0 dpanel %5llu w1 trailing %5llu w3 dinv+trailing %5llu\n", s,
                 p2 - (s ? st[2 * s] : st[0]), st[2 + 2 * s] - p2, st[29 + s] - p2, st[21 + s] - p2);
        }
        printf("  v1 last dinv+store %llu total %llu cycles\n", st[19] - st[17], st[19] - st[20]);
      }
    }
  }
  // non-PD: zero the block's (37,37) pivot region -> info must be 38 in both
  for (int v = 1; v <= 1; ++v) {
    std::vector<double> hb = h;
    for (int i = 0; i < Np; ++i) { hb[(size_t)37 * Np + i] = 0; hb[(size_t)i * Np + 37] = 0; }
    CK(hipMemcpy(A, hb.data(), hb.size() * 8, hipMemcpyHostToDevice));
    launch_init_result(0, res);
    if (v == 1) diag_v1<<<1, 256>>>(A, Np, 1 << 30, 0, Dinv, res);
    EvalResult hr; CK(hipMemcpy(&hr, res, sizeof hr, hipMemcpyDeviceToHost));
    printf("non-PD v%d: info %llu (expect 38)\n", v, (unsigned long long)hr.info);
  }
  // standalone latencies of the chain kernels (one tile each)
  CK(hipMemcpy(A, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  launch_potrf_diag(0, A, Np, 1 << 30, 0, Dinv, res, nullptr);
  for (int rep = 0; rep < 3; ++rep) {
    float ms;
    CK(hipEventRecord(e0)); launch_trsm(0, A, Np, 2, 0, Dinv, nullptr); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1)); printf("trsm 1 tile: %.1f us  ", ms * 1e3);
    CK(hipEventRecord(e0)); launch_col_update(0, A, Np, Panel{A, Np, 0}, nt, 1, 1, 1, NB, nullptr); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1)); printf("col_update 3 tiles K=128: %.1f us  ", ms * 1e3);
    CK(hipEventRecord(e0)); launch_col_update(0, A, Np, Panel{A, Np, 0}, nt, 2, 2, 2, 256, nullptr); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1)); printf("col_update 2 cols K=256: %.1f us\n", ms * 1e3);
  }
  return 0;
}
