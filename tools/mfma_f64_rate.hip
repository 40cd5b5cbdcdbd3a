// Microbenchmark: fp64 matrix (v_mfma_f64_16x16x4f64) and vector (v_fma_f64) peak rates on
// gfx950, in-kernel clock (s_memtime / s_memrealtime at 100 MHz), and whether MFMA waves
// and VALU waves on the same CU add up. Used to pick the roofline peak for DESIGN.md.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__device__ void mfma_body(double* out, int iters, double a, double b) {
  d4 c[NACC];
#pragma unroll
  for (int q = 0; q < NACC; ++q) c[q] = d4{0, 0, 0, 0};
  double x = a + threadIdx.x * 1e-9, y = b - threadIdx.x * 1e-9;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int q = 0; q < NACC; ++q) c[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(q & 1 ? x : y, q & 2 ? y : x, c[q], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int q = 0; q < NACC; ++q) s += c[q][0] + c[q][1] + c[q][2] + c[q][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__device__ void fma_body(double* out, int iters, double a, double b) {
  double c[8];
  for (int k = 0; k < 8; ++k) c[k] = threadIdx.x * k;
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = fma(c[k], a, b);
  double s = 0;
  for (int k = 0; k < 8; ++k) s += c[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
__global__ __launch_bounds__(256) void mfma_loop(double* out, int iters, double a, double b, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  mfma_body<NACC>(out, iters, a, b);
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}
__global__ __launch_bounds__(256) void fma_loop(double* out, int iters, double a, double b) { fma_body(out, iters, a, b); }
// waves 0,1 run MFMA (iters_m), waves 2,3 run VALU FMA (iters_v)
__global__ __launch_bounds__(256) void mixed_loop(double* out, int iters_m, int iters_v, double a, double b) {
  if ((threadIdx.x >> 6) < 2) mfma_body<4>(out, iters_m, a, b);
  else fma_body(out, iters_v, a, b);
}

int main() {
  double* out; CK(hipMalloc(&out, 256 * 8192 * 8));
  unsigned long long* clk; CK(hipMalloc(&clk, 16 * 8192));
  unsigned long long hclk[2 * 2048];
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int iters = 4000;
  for (int rep = 0; rep < 2; ++rep) {
    for (int bpc : {1, 2, 4}) {
      int blocks = 256 * bpc;
      float ms;
      CK(hipEventRecord(e0)); mfma_loop<4><<<blocks, 256>>>(out, iters, 0.999, 1e-3, clk); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      double fl = (double)blocks * 4 * iters * 4 * 2048.0;
      CK(hipMemcpy(hclk, clk, 16 * blocks, hipMemcpyDeviceToHost));
      double ghz = (double)hclk[0] / (double)hclk[1] * 0.1;
      printf("mfma16x16x4 acc4  blocks/CU=%d: %.3f ms %.2f TF/s  clk %.2f GHz  cyc/mfma/SIMD %.1f\n", bpc, ms, fl / ms / 1e9, ghz,
             (double)hclk[0] / ((double)iters * 4 * bpc));
      CK(hipEventRecord(e0)); mfma_loop<8><<<blocks, 256>>>(out, iters / 2, 0.999, 1e-3, clk); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      fl = (double)blocks * 4 * (iters / 2) * 8 * 2048.0;
      CK(hipMemcpy(hclk, clk, 16 * blocks, hipMemcpyDeviceToHost));
      ghz = (double)hclk[0] / (double)hclk[1] * 0.1;
      printf("mfma16x16x4 acc8  blocks/CU=%d: %.3f ms %.2f TF/s  clk %.2f GHz\n", bpc, ms, fl / ms / 1e9, ghz);
      CK(hipEventRecord(e0)); fma_loop<<<blocks, 256>>>(out, iters, 0.999, 1e-3); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      fl = (double)blocks * 256 * iters * 8 * 2.0;
      printf("v_fma_f64         blocks/CU=%d: %.3f ms %.2f TF/s\n", bpc, ms, fl / ms / 1e9);
    }
    // mixed: balance so both halves take similar time
    for (int iv : {2000, 4000, 8000}) {
      int blocks = 512; float ms;
      CK(hipEventRecord(e0)); mixed_loop<<<blocks, 256>>>(out, iters, iv, 0.999, 1e-3); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      double flm = (double)blocks * 2 * iters * 4 * 2048.0, flv = (double)blocks * 128 * iv * 8 * 2.0;
      printf("mixed (2 mfma waves + 2 valu waves, valu iters %d): %.3f ms  total %.2f TF/s (mfma part %.2f, valu part %.2f)\n", iv, ms,
             (flm + flv) / ms / 1e9, flm / ms / 1e9, flv / ms / 1e9);
    }
  }
  return 0;
}
