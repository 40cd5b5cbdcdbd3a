// Latency probe (one wave, s_memtime cycles): dependent chains of fp64 MFMA / FMA /
// v_rsq_f64 / readlane broadcast, and independent-issue rates, on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int IT = 256;

__global__ void k_mfma_dep(double* out, unsigned long long* clk, double a) {
  d4 c = {0, 0, 0, 0};
  double x = a + threadIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
  for (int i = 0; i < IT; ++i) c = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, c, 0, 0, 0);
  __builtin_amdgcn_sched_barrier(0);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = c[0] + c[1] + c[2] + c[3];
  if (threadIdx.x == 0) clk[0] = t1 - t0;
}
__global__ void k_mfma_ind(double* out, unsigned long long* clk, double a) {
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  double x = a + threadIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 4
  for (int i = 0; i < IT / 4; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, c3, 0, 0, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
  if (threadIdx.x == 0) clk[0] = t1 - t0;
}
__global__ void k_fma_dep(double* out, unsigned long long* clk, double a) {
  double x = a + threadIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
  for (int i = 0; i < IT; ++i) x = fma(x, a, 0.5);
  __builtin_amdgcn_sched_barrier(0);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) clk[0] = t1 - t0;
}
__global__ void k_fma_ind(double* out, unsigned long long* clk, double a) {
  double x0 = a + threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 4
  for (int i = 0; i < IT / 8; ++i) {
    x0 = fma(x0, a, 0.5); x1 = fma(x1, a, 0.5); x2 = fma(x2, a, 0.5); x3 = fma(x3, a, 0.5);
    x4 = fma(x4, a, 0.5); x5 = fma(x5, a, 0.5); x6 = fma(x6, a, 0.5); x7 = fma(x7, a, 0.5);
  }
  __builtin_amdgcn_sched_barrier(0);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
  if (threadIdx.x == 0) clk[0] = t1 - t0;
}
__global__ void k_rsq_dep(double* out, unsigned long long* clk, double a) {
  double x = a + threadIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
  for (int i = 0; i < IT; ++i) x = __builtin_amdgcn_rsq(x);
  __builtin_amdgcn_sched_barrier(0);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) clk[0] = t1 - t0;
}
__device__ __forceinline__ double readlane_d(double x, int l) {
  const long long v = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane((int)(v & 0xffffffffll), l);
  const int hi = __builtin_amdgcn_readlane((int)(v >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
// x = fma(readlane(x, 5), a, x): readlane -> VALU consumer, dependent
__global__ void k_rl_dep(double* out, unsigned long long* clk, double a) {
  double x = a + threadIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
  for (int i = 0; i < IT; ++i) x = fma(readlane_d(x, 5), a, x);
  __builtin_amdgcn_sched_barrier(0);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) clk[0] = t1 - t0;
}
// LDS round trip: lane 0 writes, all read, dependent
__global__ void k_lds_dep(double* out, unsigned long long* clk, double a) {
  __shared__ double buf[64];
  double x = a + threadIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
  for (int i = 0; i < IT; ++i) {
    if (threadIdx.x == 0) buf[i & 63] = x;
    __builtin_amdgcn_wave_barrier();
    x = fma(buf[i & 63], a, x);
  }
  __builtin_amdgcn_sched_barrier(0);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) clk[0] = t1 - t0;
}
int main() {
  double* out; unsigned long long* clk; CK(hipMalloc(&out, 64 * 8)); CK(hipMalloc(&clk, 8));
  unsigned long long h;
  struct { const char* n; void (*f)(double*, unsigned long long*, double); } ks[] = {
    {"mfma_f64_16x16x4 dependent", k_mfma_dep}, {"mfma_f64_16x16x4 4 indep", k_mfma_ind},
    {"v_fma_f64 dependent", k_fma_dep}, {"v_fma_f64 8 indep", k_fma_ind}, {"v_rsq_f64 dependent", k_rsq_dep},
    {"readlane+fma dependent", k_rl_dep}, {"lds write/read+fma dependent", k_lds_dep}};
  for (int rep = 0; rep < 2; ++rep)
    for (auto& k : ks) {
      hipLaunchKernelGGL(k.f, dim3(1), dim3(64), 0, 0, out, clk, 0.999);
      CK(hipDeviceSynchronize()); CK(hipMemcpy(&h, clk, 8, hipMemcpyDeviceToHost));
      if (rep) printf("%-34s %7.1f cycles/op\n", k.n, (double)h / IT);
    }
  return 0;
}
