// Microbenchmark: fp64 MFMA (v_mfma_f64_16x16x4f64) and fp64 VALU FMA peak rates on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void mfma_loop(double* out, int iters, double a, double b) {
  d4 c0 = {0,0,0,0}, c1 = c0, c2 = c0, c3 = c0;
  double x = a + threadIdx.x * 1e-9, y = b - threadIdx.x * 1e-9;
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c0, 0,0,0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, x, c1, 0,0,0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, c2, 0,0,0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, y, c3, 0,0,0);
  }
  d4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * 256 + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}
__global__ __launch_bounds__(256) void fma_loop(double* out, int iters, double a, double b) {
  double c[8]; for (int k = 0; k < 8; ++k) c[k] = threadIdx.x * k;
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = fma(c[k], a, b);
  double s = 0; for (int k = 0; k < 8; ++k) s += c[k];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
  double* out; hipMalloc(&out, 256 * 4096 * 8);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  int blocks = 256 * 4, iters = 4000;
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0); mfma_loop<<<blocks, 256>>>(out, iters, 0.999, 1e-3); hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double flops = (double)blocks * 4 /*waves*/ * iters * 4 * 2.0 * 16 * 16 * 4;
    printf("mfma_f64_16x16x4: %.3f ms  %.2f TFLOP/s\n", ms, flops / ms / 1e9);
    hipEventRecord(e0); fma_loop<<<blocks, 256>>>(out, iters, 0.999, 1e-3); hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    flops = (double)blocks * 256 * iters * 8 * 2.0;
    printf("v_fma_f64:       %.3f ms  %.2f TFLOP/s\n", ms, flops / ms / 1e9);
  }
  return 0;
}
