// Issue cost of the cross-lane moves the round-5 diagonal kernel uses, one wave alone
// (s_memtime cycles per instruction, gfx950): 64-bit DPP row_newbcast (v_mov_b64_dpp),
// the same as two 32-bit DPP moves, v_permlane32_swap, and fp64 FMA for reference.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <int R> __device__ __forceinline__ double bc64(double x) {
  return __longlong_as_double(__builtin_amdgcn_mov_dpp(__double_as_longlong(x), 0x150 + R, 0xf, 0xf, false));
}
template <int R> __device__ __forceinline__ double bc32x2(double x) {
  const long long v = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_mov_dpp((int)v, 0x150 + R, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(v >> 32), 0x150 + R, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

template <int MODE>
__global__ void k(double* out, unsigned long long* cyc, double a, double b) {
  double x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = out[threadIdx.x] + j;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < 128; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if constexpr (MODE == 0) {  // fma64 x8
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = fma(x[j], a, b);
      } else if constexpr (MODE == 1) {  // v_mov_b64_dpp x8 (independent)
        x[0] = bc64<1>(x[0]); x[1] = bc64<2>(x[1]); x[2] = bc64<3>(x[2]); x[3] = bc64<4>(x[3]);
        x[4] = bc64<5>(x[4]); x[5] = bc64<6>(x[5]); x[6] = bc64<7>(x[6]); x[7] = bc64<8>(x[7]);
      } else if constexpr (MODE == 2) {  // 2 x v_mov_b32_dpp x8
        x[0] = bc32x2<1>(x[0]); x[1] = bc32x2<2>(x[1]); x[2] = bc32x2<3>(x[2]); x[3] = bc32x2<4>(x[3]);
        x[4] = bc32x2<5>(x[4]); x[5] = bc32x2<6>(x[5]); x[6] = bc32x2<7>(x[6]); x[7] = bc32x2<8>(x[7]);
      } else if constexpr (MODE == 3) {  // dpp64 + fma pairs
        x[0] = fma(bc64<1>(x[1]), a, x[0]); x[1] = fma(bc64<2>(x[2]), a, x[1]); x[2] = fma(bc64<3>(x[3]), a, x[2]);
        x[3] = fma(bc64<4>(x[4]), a, x[3]); x[4] = fma(bc64<5>(x[5]), a, x[4]); x[5] = fma(bc64<6>(x[6]), a, x[5]);
        x[6] = fma(bc64<7>(x[7]), a, x[6]); x[7] = fma(bc64<8>(x[0]), a, x[7]);
      } else if constexpr (MODE == 4) {  // v_permlane32_swap x8 (32-bit)
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const auto p = __builtin_amdgcn_permlane32_swap((unsigned)__double_as_longlong(x[j]),
                                                          (unsigned)__double_as_longlong(x[j + 1]), false, false);
          x[j] = __longlong_as_double((long long)p[0]);
          x[j + 1] = __longlong_as_double((long long)p[1]);
        }
      } else if constexpr (MODE == 5) {  // dependent fma64 chain (latency)
        x[0] = fma(x[0], a, b); x[0] = fma(x[0], a, b); x[0] = fma(x[0], a, b); x[0] = fma(x[0], a, b);
        x[0] = fma(x[0], a, b); x[0] = fma(x[0], a, b); x[0] = fma(x[0], a, b); x[0] = fma(x[0], a, b);
      } else if constexpr (MODE == 6) {  // dependent dpp64 -> fma chain
        x[0] = fma(bc64<3>(x[0]), a, b); x[0] = fma(bc64<3>(x[0]), a, b); x[0] = fma(bc64<3>(x[0]), a, b);
        x[0] = fma(bc64<3>(x[0]), a, b); x[0] = fma(bc64<3>(x[0]), a, b); x[0] = fma(bc64<3>(x[0]), a, b);
        x[0] = fma(bc64<3>(x[0]), a, b); x[0] = fma(bc64<3>(x[0]), a, b);
      } else if constexpr (MODE == 7) {  // dependent rsq64 chain
        x[0] = __builtin_amdgcn_rsq(x[0]); x[0] = __builtin_amdgcn_rsq(x[0]); x[0] = __builtin_amdgcn_rsq(x[0]);
        x[0] = __builtin_amdgcn_rsq(x[0]); x[0] = __builtin_amdgcn_rsq(x[0]); x[0] = __builtin_amdgcn_rsq(x[0]);
        x[0] = __builtin_amdgcn_rsq(x[0]); x[0] = __builtin_amdgcn_rsq(x[0]);
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += x[j];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  double* out; unsigned long long* cyc;
  CK(hipMalloc(&out, 1024 * 8)); CK(hipMalloc(&cyc, 8)); CK(hipMemset(out, 0, 1024 * 8));
  const char* names[] = {"fma64 x8 independent", "mov_b64_dpp x8", "2x mov_b32_dpp x8 (per pair)", "dpp64+fma x8 (per pair)",
                         "permlane32_swap x4 (per swap)", "fma64 dependent (latency)", "dpp64->fma dependent (per pair)",
                         "rsq64 dependent (latency)"};
  const double per[] = {32, 32, 32, 32, 16, 32, 32, 32};
  for (int m = 0; m < 8; ++m) {
    unsigned long long best = ~0ull;
    for (int rep = 0; rep < 5; ++rep) {
      switch (m) {
        case 0: k<0><<<1, 64>>>(out, cyc, 0.999, 0.001); break;
        case 1: k<1><<<1, 64>>>(out, cyc, 0.999, 0.001); break;
        case 2: k<2><<<1, 64>>>(out, cyc, 0.999, 0.001); break;
        case 3: k<3><<<1, 64>>>(out, cyc, 0.999, 0.001); break;
        case 4: k<4><<<1, 64>>>(out, cyc, 0.999, 0.001); break;
        case 5: k<5><<<1, 64>>>(out, cyc, 0.999, 0.001); break;
        case 6: k<6><<<1, 64>>>(out, cyc, 0.999, 0.001); break;
        case 7: k<7><<<1, 64>>>(out, cyc, 0.999, 0.001); break;
      }
      CK(hipDeviceSynchronize());
      unsigned long long c; CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost)); if (c < best) best = c;
    }
    printf("%-34s %.2f cycles\n", names[m], (double)best / (128.0 * per[m]));
  }
  return 0;
}
