// fp64 MFMA ceiling on gfx950: v_mfma_f64_16x16x4f64 back to back with NACC independent
// accumulators per wave and 8 distinct A/B operand pairs (tools/mfma_f64_rate.hip reuses one
// pair), W waves per SIMD, every CU busy for ~100 ms; reports TFLOP/s and the shader clock
// the chip held (s_memtime / s_memrealtime) so the bulk kernel's fraction can be read
// against what the matrix pipes deliver under a sustained fp64 load.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void peak(double* out, int iters, unsigned long long* clk) {
  d4 c[NACC];
#pragma unroll
  for (int q = 0; q < NACC; ++q) c[q] = d4{0, 0, 0, 0};
  double a[8], b[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a[k] = 1.0 + 1e-9 * (threadIdx.x + k);
    b[k] = 1e-3 - 1e-12 * (threadIdx.x * 3 + k);
  }
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int q = 0; q < NACC; ++q) c[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[q & 7], b[(q >> 1) & 7], c[q], 0, 0, 0);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  double s = 0;
#pragma unroll
  for (int q = 0; q < NACC; ++q) s += c[q][0] + c[q][1] + c[q][2] + c[q][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

template <int NACC>
int run(double* out, unsigned long long* clk, int bpc, int iters) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int blocks = 256 * bpc;
  peak<NACC><<<blocks, 256>>>(out, 10, clk);  // warm
  CK(hipDeviceSynchronize());
  float ms;
  CK(hipEventRecord(e0));
  peak<NACC><<<blocks, 256>>>(out, iters, clk);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long h[2];
  CK(hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost));
  const double fl = (double)blocks * 4 * iters * NACC * 2048.0;  // 4 waves per block
  const double ghz = (double)h[0] / (double)h[1] * 0.1;
  printf("NACC=%2d waves/SIMD=%d: %8.3f ms  %6.2f TFLOP/s  clock %.2f GHz  -> %.1f FLOP/clk/CU\n", NACC, bpc, ms,
         fl / ms / 1e9, ghz, fl / (ms * 1e-3) / (256.0 * ghz * 1e9));
  return 0;
}

int main() {
  double* out; CK(hipMalloc(&out, 256 * 4096 * 8));
  unsigned long long* clk; CK(hipMalloc(&clk, 16 * 4096));
  for (int rep = 0; rep < 2; ++rep) {
    if (run<16>(out, clk, 1, 12000)) return 1;
    if (run<16>(out, clk, 2, 6000)) return 1;
    if (run<8>(out, clk, 2, 12000)) return 1;
    if (run<16>(out, clk, 4, 3000)) return 1;
  }
  return 0;
}
