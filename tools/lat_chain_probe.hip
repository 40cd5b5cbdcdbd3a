// Dependent-chain latencies on gfx950, one wave alone on its SIMD (s_memtime cycles per step):
//   fma64   x = fma(x, a, b)                         (f64 FMA result -> next FMA)
//   rsq64   x = rsq(x) * c + d                         (v_rsq_f64 + an FMA)
//   rl64    x = fma(readlane(x, 5), a, b)             (f64 result -> 2x v_readlane -> FMA)
//   fma32   x = fma(x, a, b) in f32                    (reference)
// Explains the diagonal kernel's ~440 cycles per column.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__device__ __forceinline__ double rl(double x, int l) {
  const long long v = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane((int)(v & 0xffffffffll), l);
  const int hi = __builtin_amdgcn_readlane((int)(v >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

template <int MODE>
__global__ void k(double* out, unsigned long long* cyc, double a, double b) {
  double x = out[threadIdx.x];
  float xf = (float)x;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < 256; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (MODE == 0) x = fma(x, a, b);
      if constexpr (MODE == 1) x = fma(__builtin_amdgcn_rsq(x), a, b);
      if constexpr (MODE == 2) x = fma(rl(x, 5), a, b);
      if constexpr (MODE == 3) xf = fmaf(xf, (float)a, (float)b);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x + xf;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  double* out; unsigned long long* cyc;
  CK(hipMalloc(&out, 64 * 8)); CK(hipMalloc(&cyc, 8)); CK(hipMemset(out, 0, 64 * 8));
  const char* names[] = {"fma64 chain", "rsq64 + fma chain", "readlane64 + fma chain", "fma32 chain"};
  for (int m = 0; m < 4; ++m) {
    unsigned long long best = ~0ull;
    for (int rep = 0; rep < 5; ++rep) {
      if (m == 0) k<0><<<1, 64>>>(out, cyc, 0.999, 0.001);
      if (m == 1) k<1><<<1, 64>>>(out, cyc, 0.5, 1.0);
      if (m == 2) k<2><<<1, 64>>>(out, cyc, 0.999, 0.001);
      if (m == 3) k<3><<<1, 64>>>(out, cyc, 0.999, 0.001);
      CK(hipDeviceSynchronize());
      unsigned long long c; CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost)); if (c < best) best = c;
    }
    printf("%-24s %.1f cycles per dependent step\n", names[m], (double)best / 2048.0);
  }
  return 0;
}
