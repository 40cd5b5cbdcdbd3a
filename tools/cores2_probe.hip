// Co-residency of the real kernels: a bulk trailing update (tile_syrk8_kernel, persistent
// grid) on a low-priority stream, then one diagonal-block kernel and one TRSM launch on a
// high-priority stream. Prints when each started (first workgroup, s_memrealtime) and
// ended relative to the bulk launch's start. Values in the matrix are irrelevant here.
#include "../gaplac_amd/csrc/gaplac_kernels.hip"
#include <cstdio>
#include <vector>
using namespace gaplac;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

// resident stand-in with the bulk kernel's footprint (512 threads, BULK8_LDS) that only
// sleeps: no MFMA, no memory traffic
__global__ __launch_bounds__(512, 1) void sleeper(KTime* kt, unsigned long long dur) {
  extern __shared__ double lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { atomicMin(&kt->start, t0); lds[0] = 1.0; }
  for (int i = 0; i < 100000; ++i) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > dur) break;
    __builtin_amdgcn_s_sleep(20);
  }
  if (threadIdx.x == 0) atomicMax(&kt->end, (unsigned long long)__builtin_amdgcn_s_memrealtime() + (unsigned long long)lds[0]);
}

int main(int argc, char** argv) {
  const int nt = 64, Np = nt * NB;
  double *A, *Dinv; EvalResult* res; KTime* kt; uint32_t* tiles;
  CK(hipMalloc(&A, (size_t)Np * Np * 8)); CK(hipMemset(A, 0, (size_t)Np * Np * 8));
  CK(hipMalloc(&Dinv, nt * DINV_PER_BLOCK * 8)); CK(hipMalloc(&res, sizeof(EvalResult)));
  CK(hipMalloc(&kt, 8 * sizeof(KTime)));
  const int m = nt - 8;  // trailing tiles 8..63 updated with tile columns 0..3 (K = 512)
  std::vector<uint32_t> h((size_t)m * (m + 1) / 2);
  build_tile_list(m, h.data());
  CK(hipMalloc(&tiles, h.size() * 4)); CK(hipMemcpy(tiles, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  int lo = 0, hi = 0; CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  hipStream_t sm, sp;
  CK(hipStreamCreateWithPriority(&sm, hipStreamNonBlocking, lo)); CK(hipStreamCreateWithPriority(&sp, hipStreamNonBlocking, hi));
  CK(hipFuncSetAttribute((const void*)sleeper, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
  for (int mode = 0; mode <= 3; ++mode) {
    setenv("GAPLAC_BULK8", mode == 1 ? "1" : "2", 1);
    for (int rep = 0; rep < 2; ++rep) {
      launch_kt_reset(sm, kt, 8); launch_init_result(sm, res);
      CK(hipStreamSynchronize(sm));
      BulkArgs ba{A, Np, Panel{A, Np, 0}, tiles, (int)h.size(), 512, 8, 8, ColMap{1, 0, 4}};
      if (mode == 1 || mode == 2) launch_bulk(sm, ba, kt + 0);
      if (mode == 3) sleeper<<<256, 512, BULK8_LDS, sm>>>(kt, 60000);
      if (mode == 0) launch_kt_reset(sm, kt, 1);  // t0 = the chain's own start
      if (mode == 0) CK(hipStreamSynchronize(sm));
      launch_potrf_diag(sp, A + (size_t)4 * NB * Np + 4 * NB, Np, 1 << 30, 4 * NB, Dinv, res, kt + 1);
      launch_trsm(sp, A + (size_t)4 * NB * Np, Np, nt, 4, Dinv, kt + 2);
      launch_col_update(sp, A, Np, Panel{A + (size_t)4 * NB * Np, Np, 0}, nt, 5, 5, 1, NB, kt + 3);
      launch_potrf_diag(sp, A + (size_t)5 * NB * Np + 5 * NB, Np, 1 << 30, 5 * NB, Dinv, res, kt + 4);
      CK(hipDeviceSynchronize());
      KTime t[8]; CK(hipMemcpy(t, kt, sizeof t, hipMemcpyDeviceToHost));
      if (mode == 0) t[0].start = t[1].start;
      auto us = [&](unsigned long long x) { return ((long long)x - (long long)t[0].start) / 100.0; };
      static const char* what[] = {"nothing resident", "bulk, all tiles", "bulk, 1 WG per CU", "sleeper, bulk footprint"};
      printf("%-24s: bulk %.0f..%.0f us | diag %.1f..%.1f | trsm %.1f..%.1f | colupd %.1f..%.1f | diag %.1f..%.1f\n",
             what[mode], us(t[0].start), us(t[0].end), us(t[1].start), us(t[1].end),
             us(t[2].start), us(t[2].end), us(t[3].start), us(t[3].end), us(t[4].start), us(t[4].end));
    }
  }
  return 0;
}
