// Cycles per column of the diagonal kernel's panel sweep (wave A of potrf_diag2_body), one
// wave alone, by what the sweep carries:
//   bit 1: the deferred (filler) FMAs of columns c+2..15
//   bit 2: the LDS broadcast (publish column c, read back column c-1)
//   bit 4: the padding pivot select
//   bit 8: the non-PD test in the loop (else: each lane keeps its pivot, tested after the loop)
//   bit 16: rd of the diagonal lane kept by a select (else: from the LDS flag array afterwards)
//   bit 32: sqrt(p) refined (t + t e c; else p * rd)
//   bit 64: L(c+2, c) for the next iteration from the LDS broadcast instead of readlane
//   bit 128: the rd flag written by lane 0 only (else every lane writes the same address)
//   bit 256: the column broadcast written by lanes 0-15 only
// Each variant runs the 16-column sweep 8 times on a 64-row panel held in registers.
#include "../gaplac_amd/csrc/gaplac_kernels.hip"
#include <cmath>
#include <cstdio>
#include <vector>
using namespace gaplac;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

#define SB() __builtin_amdgcn_sched_barrier(0)
#define PIN(x) asm volatile("" : "+v"(x))

// the library's own sweep (diag2_sweep_a) on one wave, panel s = 4 of a block in LDS;
// nwaves > 1: the other waves of the block sit at the barrier (as in the real kernel)
__global__ __launch_bounds__(512) void real_sweep(const double* blk, unsigned long long* cyc, EvalResult* res) {
  __shared__ double sm[DIAG2_SMEM];
  double* colbuf = sm;
  double* Ab = sm + DIAG2_COLBUF + NB;
  for (int i = threadIdx.x; i < NPK * 256; i += blockDim.x) Ab[i] = blk[i];
  __syncthreads();
  unsigned long long best = ~0ull;
  for (int rep = 0; rep < 4; ++rep) {
    if (threadIdx.x < 64) {
      const unsigned long long t0 = __builtin_amdgcn_s_memtime();
      diag2_sweep_a(Ab, colbuf, 4, threadIdx.x, 0, 1 << 30, res);
      const unsigned long long t1 = __builtin_amdgcn_s_memtime();
      if (t1 - t0 < best) best = t1 - t0;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *cyc = best;
}

template <int MODE>
__global__ __launch_bounds__(64) void sweep(double* io, unsigned long long* cyc, long long npiv_in, unsigned* info) {
  __shared__ double colbuf[16 * 64];
  __shared__ double rdbuf[16];
  int lane = threadIdx.x;
  asm volatile("" : "+v"(lane));
  double v[16];
  double v0[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) v0[c] = io[c * 64 + lane];
  const long long npiv = npiv_in;
  const int npiv32 = (int)(npiv < 0 ? 0 : (npiv > 16 ? 16 : npiv));
  const unsigned padmask = npiv32 >= 16 ? 0u : (0xffffu << npiv32) & 0xffffu;
  int bad = 16;
  double myrd = 1.0, mypiv = 1.0;
  unsigned long long best = ~0ull;
  for (int rep = 0; rep < 8; ++rep) {
#pragma unroll
    for (int c = 0; c < 16; ++c) v[c] = v0[c];
    double lcA[16], lcB[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) lcA[c] = lcB[c] = 0.001 * c;
    double k375 = 0.375;
    PIN(k375);
    double ln2 = 0.0;
    double piv = readlane_d(v[0], 0);
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    SB();
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      auto fill = [&](int k) {
        const int c2 = c + 2 + k;
        if ((MODE & 1) && c >= 2 && c2 < 16) {
          v[c2] = fma(-v[c - 2], lcA[c2], v[c2]);
          PIN(v[c2]);
        }
      };
      const bool pad = (padmask >> c) & 1u;
      const double p = (MODE & 4) ? (pad ? 1.0 : piv) : piv;
      const double y = __builtin_amdgcn_rsq(p);
      if constexpr (MODE & 8) bad = (!pad && piv <= 0.0 && bad == 16) ? c : bad;
      if constexpr (!(MODE & 8)) mypiv = lane == c ? v[c] : mypiv;
      if ((MODE & 2) && c >= 1) {
#pragma unroll
        for (int c2 = c + 2; c2 < 16; ++c2) lcB[c2] = colbuf[(c - 1) * 64 + c2];
      }
      if ((MODE & 1) && c >= 2 && c + 1 < 16) v[c + 1] = fma(-v[c - 2], lcA[c + 1], v[c + 1]);
      if (c >= 1 && c + 1 < 16) {
        v[c + 1] = fma(-v[c - 1], ln2, v[c + 1]);
        PIN(v[c + 1]);
      }
      fill(0);
      SB();
      const double t = p * y;
      fill(1);
      fill(2);
      SB();
      const double e = fma(-t, y, 1.0);
      fill(3);
      fill(4);
      SB();
      const double cc = fma(e, k375, 0.5);
      const double ye = y * e;
      const double te = t * e;
      fill(5);
      SB();
      const double rd = fma(ye, cc, y);
      const double d = (MODE & 32) ? fma(te, cc, t) : p * rd;
      fill(6);
      fill(7);
      SB();
      const double l = v[c] * rd;
      v[c] = lane == c ? d : l;
      if constexpr (MODE & 16) myrd = lane == c ? rd : myrd;
      fill(8);
      SB();
      double ln = 0.0, ln2n = 0.0;
      if (c + 1 < 16) ln = readlane_d(l, c + 1);
      if (!(MODE & 64) && c + 2 < 16) ln2n = readlane_d(l, c + 2);
      if constexpr (MODE & 2) {
        if (!(MODE & 256) || lane < 16) colbuf[c * 64 + lane] = v[c];
        asm volatile("" ::: "memory");
        if (!(MODE & 128) || lane == 0) rdbuf[c] = rd;
      }
      fill(9);
      fill(10);
      SB();
      if (c + 1 < 16) v[c + 1] = fma(-v[c], ln, v[c + 1]);
      fill(11);
      SB();
      if (c + 1 < 16) piv = readlane_d(v[c + 1], c + 1);
      fill(12);
      if constexpr (MODE & 64) {
        if (c + 2 < 16) ln2n = colbuf[c * 64 + c + 2];
      }
      ln2 = ln2n;
#pragma unroll
      for (int c2 = 0; c2 < 16; ++c2) lcA[c2] = lcB[c2];
      SB();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (t1 - t0 < best) best = t1 - t0;
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) io[c * 64 + lane] = v[c] + myrd;
  if constexpr (!(MODE & 8)) {
    const unsigned long long m = __ballot(lane < 16 && !((padmask >> lane) & 1u) && mypiv <= 0.0);
    bad = m ? __builtin_ctzll(m) : 16;
  }
  if (lane == 0) { *cyc = best; info[0] = bad; }
}

int main() {
  double* io; unsigned long long* cyc; unsigned* info;
  CK(hipMalloc(&io, 16 * 64 * 8)); CK(hipMalloc(&cyc, 8)); CK(hipMalloc(&info, 4));
  double h[16 * 64];
  for (int c = 0; c < 16; ++c)
    for (int r = 0; r < 64; ++r) {
      const double d = (r - c) * 0.013;
      h[c * 64 + r] = std::exp(-0.5 * d * d) + (r == c ? 0.1 : 0.0);
    }
  struct V { int mode; const char* name; };
  const V vs[] = {{0, "chain only"}, {1, "+fillers"}, {3, "+fillers+LDS"},
                  {1 | 2 | 4 | 8 | 16 | 32, "round-3 v2 as built"},
                  {1 | 2 | 4 | 16 | 32, "- non-PD test in loop"},
                  {1 | 2 | 4 | 32, "- rd select"},
                  {1 | 2 | 4, "- refined sqrt"},
                  {1 | 2 | 4 | 64, "+ L(c+2,c) via LDS"},
                  {1 | 2 | 4 | 128, "rd flag by lane 0"},
                  {1 | 2 | 4 | 128 | 256, "rd flag lane 0, column lanes 0-15"},
                  {2, "LDS only"}, {2 | 128, "LDS only, rd flag lane 0"}};
  for (const V& vv : vs) {
    unsigned long long c = 0;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipMemcpy(io, h, sizeof h, hipMemcpyHostToDevice));
      switch (vv.mode) {
#define CASE(M) case M: sweep<M><<<1, 64>>>(io, cyc, 1 << 20, info); break;
        CASE(0) CASE(1) CASE(3) CASE(63) CASE(55) CASE(39) CASE(7) CASE(71) CASE(135) CASE(391) CASE(2) CASE(130)
#undef CASE
      }
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
    }
    unsigned b; CK(hipMemcpy(&b, info, 4, hipMemcpyDeviceToHost));
    printf("%-34s %6llu cycles per 16 columns = %.0f per column (bad %u)\n", vv.name, c, c / 16.0, b);
  }
  {
    std::vector<double> hb(NPK * 256);
    for (int I = 0; I < 8; ++I)
      for (int J = 0; J <= I; ++J)
        for (int c = 0; c < 16; ++c)
          for (int r = 0; r < 16; ++r) {
            const int gi = 16 * I + r, gj = 16 * J + c;
            const double d = (gi - gj) * 0.013;
            hb[(I * (I + 1) / 2 + J) * 256 + c * 16 + r] = std::exp(-0.5 * d * d) + (gi == gj ? 0.1 : 0.0);
          }
    double* db; EvalResult* res;
    CK(hipMalloc(&db, hb.size() * 8)); CK(hipMalloc(&res, sizeof(EvalResult)));
    CK(hipMemcpy(db, hb.data(), hb.size() * 8, hipMemcpyHostToDevice));
    for (int nt : {64, 256, 512}) {
      unsigned long long c = 0;
      for (int rep = 0; rep < 2; ++rep) {
        real_sweep<<<1, nt>>>(db, cyc, res);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
      }
      printf("library diag2_sweep_a (panel 4), block of %3d threads: %6llu cycles = %.0f per column\n", nt, c, c / 16.0);
    }
  }
  return 0;
}
