// Gram kernel alone at N = 16384 (all lower tiles, one launch): algorithmic GB/s for term
// mixes from pure stores (T = 0) to the configs[2] kernel, to find what bounds it.
// Built twice: gram_probe, and gram_probe_ns with -DGAPLAC_GRAM_NOSTORE (compute only).
#include "../gaplac_amd/csrc/gaplac_kernels.hip"
#include <cstdio>
#include <vector>
#include <cstring>
using namespace gaplac;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
  const int64_t N = 16384, Np = (N + 1 + NB - 1) / NB * NB;
  const int nt = (int)(Np / NB);
  double *A, *X, *v; TermPack* dtp;
  CK(hipMalloc(&A, (size_t)Np * Np * 8)); CK(hipMalloc(&X, N * 2 * 8)); CK(hipMalloc(&v, N * 8));
  CK(hipMalloc(&dtp, sizeof(TermPack)));
  std::vector<double> hx(2 * N), hv(N);
  unsigned s = 1;
  for (auto& x : hx) { s = s * 1664525u + 1013904223u; x = (s >> 8) * (10.0 / 16777216.0); }
  for (int64_t i = 0; i < N; ++i) hx[N + i] = (double)((int)hx[N + i] * 500);  // subject ids
  CK(hipMemcpy(X, hx.data(), hx.size() * 8, hipMemcpyHostToDevice)); CK(hipMemcpy(v, hx.data(), N * 8, hipMemcpyHostToDevice));
  struct Mix { const char* name; int T; int kind[4]; int col[4]; double p[4]; int one_group = 0; };
  const Mix mixes[] = {{"T=0 (noise only: stores)", 0, {}, {}, {}},
                       {"Cat", 1, {GAPLAC_CAT}, {1}, {0}},
                       {"SqExp", 1, {GAPLAC_SQEXP}, {0}, {1 / 1.5}},
                       {"OU", 1, {GAPLAC_OU}, {0}, {1 / 3.0}},
                       {"SqExp+OU", 2, {GAPLAC_SQEXP, GAPLAC_OU}, {0, 0}, {1 / 1.5, 1 / 3.0}},
                       {"SqExp*Cat (one group)", 2, {GAPLAC_SQEXP, GAPLAC_CAT}, {0, 1}, {1 / 1.5, 0}},
                       {"SqExp+OU+Cat+Noise", 4, {GAPLAC_SQEXP, GAPLAC_OU, GAPLAC_CAT, GAPLAC_NOISE}, {0, 0, 1, 0}, {1 / 1.5, 1 / 3.0, 0, 1.0}}};
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const double bytes = 8.0 * (double)Np * (Np + 1) / 2 + 8.0 * N * 3;
  for (const Mix& m : mixes) {
    TermPack tp; std::memset(&tp, 0, sizeof tp);
    tp.T = m.T; tp.noise = 0.1;
    for (int t = 0; t < m.T; ++t) { tp.kind[t] = m.kind[t]; tp.col[t] = m.col[t]; tp.p[t] = m.p[t]; tp.last_in_group[t] = (t == m.T - 1) || !strstr(m.name, "one group"); }
    CK(hipMemcpy(dtp, &tp, sizeof tp, hipMemcpyHostToDevice));
    float best = 1e9f;
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipEventRecord(e0));
      launch_gram(0, A, Np, N, nt, X, N, v, dtp, 0, 0, nullptr);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
    }
    printf("%-26s %7.3f ms  %7.1f GB/s (%.1f%% of 8 TB/s)\n", m.name, best, bytes / best / 1e6, bytes / best / 1e6 / 80.0);
  }
  return 0;
}
