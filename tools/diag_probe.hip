// Diagnostic: phase timing of the diagonal-block kernel (s_memtime stamps, -DGAPLAC_STAMPS)
// and standalone per-kernel latencies of the critical-path kernels on an idle GPU.
#define GAPLAC_STAMPS 1
#include "../gaplac_amd/csrc/gaplac_kernels.hip"
#include <cmath>
#include <cstdio>
#include <vector>
using namespace gaplac;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
int main() {
  const int nt = 4, Np = nt * NB;
  std::vector<double> h((size_t)Np * Np, 0.0);
  for (int j = 0; j < Np; ++j)
    for (int i = 0; i < Np; ++i) {
      double d = (i - j) * 0.01;
      h[(size_t)j * Np + i] = std::exp(-0.5 * d * d) + (i == j ? 0.1 : 0.0);
    }
  double *A, *Dinv; EvalResult* res; KTime* kt;
  CK(hipMalloc(&A, h.size() * 8)); CK(hipMalloc(&Dinv, nt * DINV_PER_BLOCK * 8));
  CK(hipMalloc(&res, sizeof(EvalResult))); CK(hipMalloc(&kt, 64 * sizeof(KTime)));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipMemcpy(A, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    launch_init_result(0, res);
    CK(hipEventRecord(e0));
    launch_potrf_diag(0, A, Np, 1 << 30, 0, Dinv, res, nullptr);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long st[64]; CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamps), sizeof st));
    printf("diag kernel %.1f us (event); phases in shader cycles from start:\n", ms * 1e3);
    printf("  load %llu\n", st[0] - st[20]);
    for (int s = 0; s < 8; ++s)
      printf("  panel %d: phase1 %6llu  panel(wave0) %6llu  barrier-wait %6llu\n", s, st[1 + 2 * s] - (s ? st[2 * s] : st[0]),
             st[2 + 2 * s] - st[1 + 2 * s], (s < 7 ? st[3 + 2 * s] : st[17]) - st[2 + 2 * s]);
    printf("  dinv %llu  store %llu  total %llu\n", st[18] - st[17], st[19] - st[18], st[19] - st[20]);
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
