// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access patterns of
// the bulk trailing-update kernel (MI355X_MICROARCH.md §HBM: only 16 B/lane streaming
// reads / writes are calibrated there). Each kernel touches a known byte count of a 2 GiB
// column-major matrix (far beyond the 256 MiB Infinity Cache, so no re-use):
//   k_rd16    16 B/lane coalesced reads (the panel staging loads, double2 per lane)
//   k_rd8col  8 B/lane reads in the C-tile pattern of tile_syrk_kernel: lane (fr, fc) reads
//             row fc of column fr + 4 rg -> 16 lanes cover one 128 B column segment,
//             one instruction covers 4 columns
//   k_wr8col  8 B/lane stores in the same pattern (the epilogue)
//   k_wr16    16 B/lane coalesced stores (Gram kernel)
// usage: rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib ; rocprofv3 --pmc WRITE_SIZE -- ./fetch_calib
// then: python tools/pmc_calib.py DIR  (bytes reported / bytes touched per kernel)
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int64_t LD = 16384;  // rows (column length), doubles
constexpr int64_t NCOL = 16384;  // 2 GiB

__global__ __launch_bounds__(256) void k_rd16(const double* __restrict__ A, double* __restrict__ out) {
  // each workgroup: 16 columns, 256 threads x double2 = 512 rows per pass
  const int64_t c0 = (int64_t)blockIdx.x * 16;
  double s = 0.0;
  for (int c = 0; c < 16; ++c)
    for (int64_t r = 2 * threadIdx.x; r < LD; r += 512) {
      const double2 v = *reinterpret_cast<const double2*>(A + (c0 + c) * LD + r);
      s += v.x + v.y;
    }
  if (s == 12345.0) out[threadIdx.x] = s;  // never true for the zero-filled input
}

__global__ __launch_bounds__(256) void k_rd8col(const double* __restrict__ A, double* __restrict__ out) {
  // each workgroup: one 128 x 128 tile (column-major), 4 waves x 64 x 64 like the bulk kernel
  const int tr = blockIdx.x % (LD / 128), tc = blockIdx.x / (LD / 128);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wi = w & 1, wj = w >> 1;
  const int fr = lane >> 4, fc = lane & 15;
  const double* T = A + (int64_t)tc * 128 * LD + (int64_t)tr * 128;
  double s = 0.0;
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int mj = 0; mj < 4; ++mj)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) s += T[(int64_t)(64 * wj + 16 * mj + fr + 4 * rg) * LD + 64 * wi + 16 * mi + fc];
  if (s == 12345.0) out[threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_wr8col(double* __restrict__ A) {
  const int tr = blockIdx.x % (LD / 128), tc = blockIdx.x / (LD / 128);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wi = w & 1, wj = w >> 1;
  const int fr = lane >> 4, fc = lane & 15;
  double* T = A + (int64_t)tc * 128 * LD + (int64_t)tr * 128;
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int mj = 0; mj < 4; ++mj)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) T[(int64_t)(64 * wj + 16 * mj + fr + 4 * rg) * LD + 64 * wi + 16 * mi + fc] = 1.0;
}

__global__ __launch_bounds__(256) void k_wr16(double* __restrict__ A) {
  const int64_t c0 = (int64_t)blockIdx.x * 16;
  for (int c = 0; c < 16; ++c)
    for (int64_t r = 2 * threadIdx.x; r < LD; r += 512)
      *reinterpret_cast<double2*>(A + (c0 + c) * LD + r) = make_double2(2.0, 2.0);
}

int main() {
  double *A, *out;
  const size_t bytes = (size_t)LD * NCOL * 8;
  CK(hipMalloc(&A, bytes));
  CK(hipMalloc(&out, 256 * 8));
  CK(hipMemset(A, 0, bytes));
  const int tiles = (int)((LD / 128) * (NCOL / 128));
  for (int rep = 0; rep < 2; ++rep) {
    k_rd16<<<(unsigned)(NCOL / 16), 256>>>(A, out);
    k_rd8col<<<(unsigned)tiles, 256>>>(A, out);
    k_wr8col<<<(unsigned)tiles, 256>>>(A);
    k_wr16<<<(unsigned)(NCOL / 16), 256>>>(A);
  }
  CK(hipDeviceSynchronize());
  printf("bytes per kernel: %zu (each kernel touches the whole matrix once)\n", bytes);
  return 0;
}
