// Issue rates of one wave alone on its SIMD (s_memtime cycles per instruction), gfx950:
//   fma64 x8   8 independent v_fma_f64 chains interleaved (issue-bound)
//   fma64 x8, 2 rows  the same with 16 chains
//   mul+fma mix
//   rsq64 x8   8 independent v_rsq_f64
//   readlane   v_readlane_b32 pairs feeding an fma (independent)
//   ldsbcast   ds_read_b128 of one address by all lanes + fma use, 8 in flight
// and the same fma64 x8 loop with 1..4 waves on ONE SIMD (launch 64*w threads, one block;
// waves w and w+4 share a SIMD, so blockDim 320 puts 2 waves on SIMD 0).
// Feeds the diagonal-block design.
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
  __shared__ double sh[64];
  double x[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) x[j] = out[threadIdx.x] + j;
  sh[threadIdx.x & 63] = x[0];
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < 128; ++i) {
    if constexpr (MODE == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = fma(x[j], a, b);
    } else if constexpr (MODE == 1) {
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int j = 0; j < 16; ++j) x[j] = fma(x[j], a, b);
    } else if constexpr (MODE == 2) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = (j & 1) ? x[j] * a : fma(x[j], a, b);
    } else if constexpr (MODE == 3) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = __builtin_amdgcn_rsq(x[j]);
    } else if constexpr (MODE == 4) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = fma(rl(x[(j + 1) & 7], j), a, x[j]);
    } else if constexpr (MODE == 5) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double y[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = sh[(8 * r + j) & 63];
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = fma(x[j], y[j], b);
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < 16; ++j) s += x[j];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  double* out; unsigned long long* cyc;
  CK(hipMalloc(&out, 1024 * 8)); CK(hipMalloc(&cyc, 8)); CK(hipMemset(out, 0, 1024 * 8));
  const char* names[] = {"fma64 x8 (1 wave)", "fma64 x16 (1 wave)", "mul/fma64 mix x8", "rsq64 x8", "readlane64+fma x8",
                         "ds_read bcast + fma x8"};
  const double per[] = {32, 32, 32, 32, 32, 40};  // instructions per outer iteration (fma / rsq / pair / read+fma)
  for (int m = 0; m < 6; ++m) {
    unsigned long long best = ~0ull;
    for (int rep = 0; rep < 5; ++rep) {
      switch (m) {
        case 0: k<0><<<1, 64>>>(out, cyc, 0.999, 0.001); break;
        case 1: k<1><<<1, 64>>>(out, cyc, 0.999, 0.001); break;
        case 2: k<2><<<1, 64>>>(out, cyc, 0.999, 0.001); break;
        case 3: k<3><<<1, 64>>>(out, cyc, 0.999, 0.001); break;
        case 4: k<4><<<1, 64>>>(out, cyc, 0.999, 0.001); break;
        case 5: k<5><<<1, 64>>>(out, cyc, 0.999, 0.001); break;
      }
      CK(hipDeviceSynchronize());
      unsigned long long c; CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost)); if (c < best) best = c;
    }
    printf("%-26s %.2f cycles per instruction\n", names[m], (double)best / (128.0 * per[m]));
  }
  // fma64 x8 with 2 waves on one SIMD (blockDim 320: waves 0 and 4 share SIMD 0; wave 0 timed)
  for (int w : {1, 5}) {
    unsigned long long best = ~0ull;
    for (int rep = 0; rep < 5; ++rep) {
      k<0><<<1, 64 * w>>>(out, cyc, 0.999, 0.001);
      CK(hipDeviceSynchronize());
      unsigned long long c; CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost)); if (c < best) best = c;
    }
    printf("fma64 x8, blockDim %3d      %.2f cycles per instruction (wave 0)\n", 64 * w, (double)best / (128.0 * 32));
  }
  return 0;
}
