// Accuracy of the Gram kernel's exp_nonpos against the library exp (ocml), in ulps of the
// library result, over x in [-750, 0] (uniform) and [-1, 0] (where Gram entries live).
#include "../gaplac_amd/csrc/gaplac_kernels.hip"
#include <cstdio>
using namespace gaplac;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k(double lo, double hi, unsigned long long n, unsigned long long* maxulp, unsigned long long* nbad) {
  __shared__ double tbl[256];
  tbl[threadIdx.x] = kExp2Tbl256[threadIdx.x];
  __syncthreads();
  unsigned long long worst = 0, bad = 0;
  for (unsigned long long i = blockIdx.x * 256ull + threadIdx.x; i < n; i += 256ull * gridDim.x) {
    const double x = lo + (hi - lo) * ((double)i / (double)n);
    const double a = exp_nonpos(x, tbl), b = exp(x);
    const long long ua = __double_as_longlong(a), ub = __double_as_longlong(b);
    const unsigned long long d = (unsigned long long)(ua > ub ? ua - ub : ub - ua);
    if (d > worst) worst = d;
    if (d > 1) ++bad;
  }
  atomicMax(maxulp, worst);
  atomicAdd(nbad, bad);
}

int main() {
  unsigned long long *m, *b;
  CK(hipMalloc(&m, 8)); CK(hipMalloc(&b, 8));
  const double rng[][2] = {{-750.0, 0.0}, {-1.0, 0.0}, {-1e-6, 0.0}, {-745.2, -700.0}};
  for (auto& r : rng) {
    CK(hipMemset(m, 0, 8)); CK(hipMemset(b, 0, 8));
    k<<<1024, 256>>>(r[0], r[1], 1ull << 27, m, b);
    unsigned long long hm, hb; CK(hipMemcpy(&hm, m, 8, hipMemcpyDeviceToHost)); CK(hipMemcpy(&hb, b, 8, hipMemcpyDeviceToHost));
    printf("x in [%g, %g]: max |exp_nonpos - exp| = %llu ulp, %llu of 2^27 points beyond 1 ulp\n", r[0], r[1], hm, hb);
  }
  return 0;
}
