// Diagnostic: the diagonal-block kernel on an idle GPU. Checks it against a CPU Cholesky of
// the same 128x128 block (L and the 16x16 inverses), prints its per-wave stamps per panel
// (v1 = potrf_diag_kernel_body, the super-panel chain's; v2 = potrf_diag2_body, the tail's;
// round 5's diag3 variant is in git history, commit 0770b8a), checks v2 against v1 with padding
// inside the block and on a non-PD block, and times the other chain kernels alone.
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
__global__ __launch_bounds__(512) void diag_v2(double* Ag, int64_t lda, int64_t N, int64_t g0, double* Dinv, EvalResult* res) {
  __shared__ double smem[DIAG2_SMEM];
  potrf_diag2_body<0>(smem, Ag, lda, N, g0, Dinv, res);
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
  auto run = [&](int v, const std::vector<double>& in, int64_t N, float* ms) -> int {
    CK(hipMemcpy(A, in.data(), in.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemset(Dinv, 0, DINV_PER_BLOCK * 8));
    launch_init_result(0, res);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    if (v == 1) diag_v1<<<1, 256>>>(A, Np, N, 0, Dinv, res);
    else diag_v2<<<1, 512>>>(A, Np, N, 0, Dinv, res);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(ms, e0, e1));
    CK(hipMemcpy(out.data(), A, out.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(dinv.data(), Dinv, dinv.size() * 8, hipMemcpyDeviceToHost));
    return 0;
  };
  for (int v = 1; v <= 2; ++v) {
    for (int rep = 0; rep < 4; ++rep) {
      float ms;
      if (run(v, h, 1 << 30, &ms)) return 1;
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
      double upper = 0;  // the block's upper triangle must be written as zeros
      for (int j = 0; j < NB; ++j)
        for (int i = 0; i < j; ++i) upper = std::fmax(upper, std::fabs(out[(size_t)j * Np + i]));
      printf("diag v%d: %.1f us (event)  max|L-Lcpu| %.2e  max|Dinv L - I| %.2e  upper %.1e  info %llx err %u\n", v, ms * 1e3,
             errL, errD, upper, (unsigned long long)hr.info, hr.err);
      if (rep == 3 && v <= 2) {  // per panel s, phase 2 of each wave (cycles, s_memtime)
        unsigned long long st[128]; CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamps), sizeof st));
        printf("  v%d load %llu\n", v, st[0] - st[20]);
        for (int s = 0; s < 8; ++s) {
          const unsigned long long p2 = st[1 + 2 * s];
          printf("  v%d s=%d: phase1+barrier %5llu | phase2 w0 %5llu w1 %5llu w%d %5llu\n", v, s,
                 p2 - (s ? st[2 * s] : st[0]), st[2 + 2 * s] - p2, st[29 + s] - p2, v == 1 ? 3 : 2, st[21 + s] - p2);  // v2: stamps of waves 1 and 2
        }
        if (v == 2)
          for (int s = 0; s < 8; ++s) {
            const unsigned long long p2 = st[1 + 2 * s];
            printf("  v%d s=%d phase2 ends: w0 %5llu w1 %5llu w2 %5llu (stores %5llu) w3 %5llu w4 %5llu w5 %5llu w6 %5llu w7 %5llu\n", v, s,
                   st[2 + 2 * s] - p2, st[29 + s] - p2, st[21 + s] - p2, s ? st[40 + s] - p2 : 0ull, st[48 + s] - p2,
                   st[80 + s] - p2, st[56 + s] - p2, st[64 + s] - p2, st[72 + s] - p2);
          }
        printf("  v%d last dinv %llu store %llu total %llu cycles\n", v, st[18] - st[17], st[19] - st[18], st[19] - st[20]);
      }
    }
  }
  // v2 against v1 with padding inside the block (N = 100, 127, 37, 1: unit pivots from
  // there) and without (N = 2^30)
  for (int64_t Npad : {(int64_t)1 << 30, (int64_t)100, (int64_t)127, (int64_t)37, (int64_t)1}) {
    float ms;
    std::vector<double> hp = h;
    for (int j = 0; j < Np; ++j)
      for (int i = 0; i < Np; ++i)
        if ((i >= Npad || j >= Npad) && i != j) hp[(size_t)j * Np + i] = (i == Npad && j < Npad) ? 0.3 * std::sin(j) : 0.0;
    std::vector<double> o[3], d[3];
    EvalResult hv[3];
    for (int v = 1; v <= 2; ++v) {
      if (run(v, hp, Npad, &ms)) return 1;
      o[v] = out;
      d[v] = dinv;
      CK(hipMemcpy(&hv[v], res, sizeof hv[v], hipMemcpyDeviceToHost));
    }
    for (int v = 2; v <= 2; ++v) {
      double dl = 0, dd = 0;
      for (int j = 0; j < NB; ++j)
        for (int i = j; i < NB; ++i) dl = std::fmax(dl, std::fabs(o[v][(size_t)j * Np + i] - o[1][(size_t)j * Np + i]));
      for (int k = 0; k < DINV_PER_BLOCK; ++k) dd = std::fmax(dd, std::fabs(d[v][k] - d[1][k]));
      printf("padded N=%lld: max|L%d-L1| %.2e max|Dinv%d-Dinv1| %.2e | info %llx/%llx err %u\n", (long long)Npad, v, dl, v,
             dd, (unsigned long long)hv[1].info, (unsigned long long)hv[v].info, hv[v].err);
    }
  }
  // non-PD: zero the block's (37,37) pivot region -> info must be 38 in both
  for (int v = 1; v <= 2; ++v) {
    std::vector<double> hb = h;
    for (int i = 0; i < Np; ++i) { hb[(size_t)37 * Np + i] = 0; hb[(size_t)i * Np + 37] = 0; }
    float ms;
    if (run(v, hb, 1 << 30, &ms)) return 1;
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
