// Accuracy of v_rsq_f64 (__builtin_amdgcn_rsq) and of one / two Goldschmidt steps from it,
// against 1/sqrt(x) computed in long double on the host for sampled x, and against
// sqrt(x) for the refined g = x * y (the diagonal kernel's pivot chain).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k(const double* x, double* y0, double* g1, double* h1, double* g2, double* h2, double* gh,
                  double* hh3, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double p = x[i];
  const double y = __builtin_amdgcn_rsq(p);
  double g = p * y, h = 0.5 * y;
  y0[i] = y;
  double r = fma(-g, h, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  g1[i] = g;
  h1[i] = h + h;
  r = fma(-g, h, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  g2[i] = g;
  h2[i] = h + h;
  // third-order (Halley) correction of the seed: e = 1 - p y^2, y' = y + y e (1/2 + 3/8 e)
  const double t = p * y;
  const double e = fma(-t, y, 1.0);
  const double c = fma(e, 0.375, 0.5);
  hh3[i] = fma(y * e, c, y);
  gh[i] = fma(t * e, c, t);
}

static double ulps(double a, long double ref) {
  const double r = (double)ref;
  const double u = std::nextafter(std::fabs(r), INFINITY) - std::fabs(r);
  return (double)std::fabs((long double)a - ref) / u;
}

int main() {
  const int n = 1 << 22;
  std::vector<double> hx(n);
  unsigned long long s = 88172645463325252ull;
  for (int i = 0; i < n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    const double e = -20.0 + 40.0 * (double)(s >> 11) / 9007199254740992.0;  // 2^-20 .. 2^20
    hx[i] = std::exp2(e);
  }
  double *x, *y0, *g1, *h1, *g2, *h2, *gh, *hh3;
  CK(hipMalloc(&x, n * 8)); CK(hipMalloc(&y0, n * 8)); CK(hipMalloc(&g1, n * 8)); CK(hipMalloc(&h1, n * 8));
  CK(hipMalloc(&g2, n * 8)); CK(hipMalloc(&h2, n * 8)); CK(hipMalloc(&gh, n * 8)); CK(hipMalloc(&hh3, n * 8));
  CK(hipMemcpy(x, hx.data(), n * 8, hipMemcpyHostToDevice));
  k<<<n / 256, 256>>>(x, y0, g1, h1, g2, h2, gh, hh3, n);
  CK(hipDeviceSynchronize());
  std::vector<double> a(n), b(n), c(n), d(n), hh(n);
  CK(hipMemcpy(a.data(), y0, n * 8, hipMemcpyDeviceToHost)); CK(hipMemcpy(b.data(), g1, n * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(c.data(), h1, n * 8, hipMemcpyDeviceToHost)); CK(hipMemcpy(d.data(), g2, n * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hh.data(), h2, n * 8, hipMemcpyDeviceToHost));
  std::vector<double> G(n), H(n);
  CK(hipMemcpy(G.data(), gh, n * 8, hipMemcpyDeviceToHost)); CK(hipMemcpy(H.data(), hh3, n * 8, hipMemcpyDeviceToHost));
  double mgh = 0, mhh = 0;
  double m0 = 0, mg1 = 0, mh1 = 0, mg2 = 0, mh2 = 0;
  for (int i = 0; i < n; ++i) {
    const long double sq = std::sqrt((long double)hx[i]), rs = 1.0L / sq;
    m0 = std::fmax(m0, ulps(a[i], rs));
    mg1 = std::fmax(mg1, ulps(b[i], sq)); mh1 = std::fmax(mh1, ulps(c[i], rs));
    mg2 = std::fmax(mg2, ulps(d[i], sq)); mh2 = std::fmax(mh2, ulps(hh[i], rs));
    mgh = std::fmax(mgh, ulps(G[i], sq)); mhh = std::fmax(mhh, ulps(H[i], rs));
  }
  printf("v_rsq_f64: max %.3g ulp of 1/sqrt\n", m0);
  printf("1 Goldschmidt step: sqrt %.3g ulp, 1/sqrt %.3g ulp\n", mg1, mh1);
  printf("2 Goldschmidt steps: sqrt %.3g ulp, 1/sqrt %.3g ulp\n", mg2, mh2);
  printf("1 Halley step: sqrt %.3g ulp, 1/sqrt %.3g ulp\n", mgh, mhh);
  return 0;
}
