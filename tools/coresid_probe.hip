// Co-residency probe: can a workgroup of kernel B (one WG, 256 threads, LDS_B bytes,
// VGPR_B registers) start on a CU while kernel A (one WG of 512 threads per CU, LDS_A,
// VGPR_A) occupies every CU? A's workgroups sleep for a fixed wall time (bounded loop on
// s_memrealtime), B records its start. B starting ~0 us after A means it fit beside A.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int V>
__device__ __forceinline__ void touch_vgpr() {
  if constexpr (V == 112) asm volatile("v_mov_b32 v111, 0" ::: "v111");
  if constexpr (V == 152) asm volatile("v_mov_b32 v151, 0" ::: "v151");
  if constexpr (V == 208) asm volatile("v_mov_b32 v207, 0" ::: "v207");
  if constexpr (V == 96) asm volatile("v_mov_b32 v95, 0" ::: "v95");
}

template <int V>
__global__ __launch_bounds__(512, 1) void kA(unsigned long long* t, unsigned long long dur) {
  extern __shared__ double lds[];
  touch_vgpr<V>();
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (blockIdx.x == 0 && threadIdx.x == 0) t[0] = t0;
  if (threadIdx.x == 0) lds[0] = 1.0;
  for (int i = 0; i < 100000; ++i) {  // bounded: at most ~100000 sleeps
    if (__builtin_amdgcn_s_memrealtime() - t0 > dur) break;
    __builtin_amdgcn_s_sleep(20);
  }
  if (threadIdx.x == 1) t[2 + blockIdx.x % 4] = (unsigned long long)lds[0];
}

template <int V>
__global__ __launch_bounds__(256, 1) void kB(unsigned long long* t) {
  extern __shared__ double lds[];
  touch_vgpr<V>();
  if (threadIdx.x == 0) { lds[0] = 2.0; t[1] = __builtin_amdgcn_s_memrealtime(); }
}

template <int VA, int VB>
int run(hipStream_t sa, hipStream_t sb, unsigned long long* d, int ldsA, int ldsB, int gridA) {
  CK(hipFuncSetAttribute((const void*)kA<VA>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
  CK(hipFuncSetAttribute((const void*)kB<VB>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
  CK(hipMemset(d, 0, 64));
  kA<VA><<<gridA, 512, ldsA, sa>>>(d, 200000);  // 2 ms
  CK(hipGetLastError());
  // give A time to fill the chip, then launch B on the high-priority stream
  unsigned long long h[2];
  kB<VB><<<1, 256, ldsB, sb>>>(d);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(h, d, 16, hipMemcpyDeviceToHost));
  printf("A: grid %4d lds %6d vgpr %3d | B: lds %6d vgpr %3d -> B starts %8.1f us after A\n", gridA, ldsA, VA, ldsB, VB,
         ((long long)h[1] - (long long)h[0]) / 100.0);
  return 0;
}

int main() {
  unsigned long long* d;
  CK(hipMalloc(&d, 64));
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  hipStream_t sa, sb;
  CK(hipStreamCreateWithPriority(&sa, hipStreamNonBlocking, lo));
  CK(hipStreamCreateWithPriority(&sb, hipStreamNonBlocking, hi));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  printf("CUs %d\n", cus);
  const int ldsAs[] = {83968, 81920, 65536, 40960};
  const int ldsBs[] = {74752, 73728, 65536, 49152, 32768, 16384, 0};
  for (int la : ldsAs)
    for (int lb : ldsBs) run<112, 96>(sa, sb, d, la, lb, cus);
  // registers: A at 112 / 208 per wave (2 waves per SIMD), B at 96 / 152
  for (int lb : {0, 65536}) {
    run<112, 152>(sa, sb, d, 40960, lb, cus);
    run<208, 96>(sa, sb, d, 40960, lb, cus);
    run<208, 152>(sa, sb, d, 40960, lb, cus);
  }
  // the bulk kernel's real occupancy: two A workgroups per CU
  run<112, 96>(sa, sb, d, 40960, 0, 2 * cus);
  run<112, 96>(sa, sb, d, 40960, 65536, 2 * cus);
  return 0;
}
