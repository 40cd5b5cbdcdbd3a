// Microbenchmark: dependent-kernel boundary cost on one stream, with event records in
// between, across two streams via events, and on CU-masked / priority streams.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
__global__ void tiny(int* p) { if (threadIdx.x == 0) atomicAdd(p, 1); }
__global__ void busy(int* p, int n) { // ~n iterations of dependent work per lane
  double x = threadIdx.x;
  for (int i = 0; i < n; ++i) x = x * 0.999999 + 1e-7;
  if (x < -1) p[0] = 1;
}
int main() {
  int* d; CK(hipMalloc(&d, 64));
  hipStream_t s1, s2, sm, sp;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  int least, greatest; CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  CK(hipStreamCreateWithPriority(&sp, hipStreamNonBlocking, greatest));
  uint32_t mask[8]; for (int i = 0; i < 8; ++i) mask[i] = 0xffffffffu; mask[0] &= ~1u;
  CK(hipExtStreamCreateWithCUMask(&sm, 8, mask));
  hipEvent_t e0, e1, ev[2]; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int q = 0; q < 2; ++q) CK(hipEventCreateWithFlags(&ev[q], hipEventDisableTiming));
  const int n = 400;
  auto run = [&](const char* name, auto body, hipStream_t s) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, s)); body(); CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep) printf("%-48s %8.2f us per step\n", name, ms * 1000.f / n);
    }
    return 0;
  };
  run("tiny kernels, one stream", [&] { for (int i = 0; i < n; ++i) tiny<<<1, 64, 0, s1>>>(d); }, s1);
  run("tiny kernels + event record each, one stream", [&] { for (int i = 0; i < n; ++i) { tiny<<<1, 64, 0, s1>>>(d); (void)hipEventRecord(ev[i & 1], s1); } }, s1);
  run("ping-pong s1<->s2 via events (2 kernels/step)", [&] {
    for (int i = 0; i < n; ++i) {
      tiny<<<1, 64, 0, s1>>>(d); (void)hipEventRecord(ev[0], s1); (void)hipStreamWaitEvent(s2, ev[0], 0);
      tiny<<<1, 64, 0, s2>>>(d); (void)hipEventRecord(ev[1], s2); (void)hipStreamWaitEvent(s1, ev[1], 0);
    } }, s1);
  run("ping-pong masked<->priority via events", [&] {
    for (int i = 0; i < n; ++i) {
      tiny<<<1, 64, 0, sm>>>(d); (void)hipEventRecord(ev[0], sm); (void)hipStreamWaitEvent(sp, ev[0], 0);
      tiny<<<1, 64, 0, sp>>>(d); (void)hipEventRecord(ev[1], sp); (void)hipStreamWaitEvent(sm, ev[1], 0);
    } }, sm);
  run("tiny kernels, priority stream", [&] { for (int i = 0; i < n; ++i) tiny<<<1, 64, 0, sp>>>(d); }, sp);
  run("tiny kernels, CU-masked stream", [&] { for (int i = 0; i < n; ++i) tiny<<<1, 64, 0, sm>>>(d); }, sm);
  run("busy(20k) kernels, one stream", [&] { for (int i = 0; i < n; ++i) busy<<<1, 64, 0, s1>>>(d, 20000); }, s1);
  // graph of the ping-pong pattern
  hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s1, hipStreamCaptureModeGlobal));
  for (int i = 0; i < n; ++i) {
    tiny<<<1, 64, 0, s1>>>(d); (void)hipEventRecord(ev[0], s1); (void)hipStreamWaitEvent(s2, ev[0], 0);
    tiny<<<1, 64, 0, s2>>>(d); (void)hipEventRecord(ev[1], s2); (void)hipStreamWaitEvent(s1, ev[1], 0);
  }
  CK(hipStreamEndCapture(s1, &g)); CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  run("graph: ping-pong s1<->s2 (2 kernels/step)", [&] { (void)hipGraphLaunch(ge, s1); }, s1);
  return 0;
}
