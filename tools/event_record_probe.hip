// event_record_probe.hip -- what one exchange event costs on the compute queue (the data-parallel
// step's Submit records an event after each gradient kernel; the kernel trace shows a ~5 us compute-queue gap at
// each).  A chain of K short kernels (every workgroup spins ~10 us on s_memrealtime) on one stream:
//   plain     kernel, kernel, ...                                   (the reference gap)
//   record    kernel, hipEventRecord(ev), kernel, ...               (DisableTiming | DisableSystemFence)
//   record+w  the same, and a second stream waits on each event      (Submit's pattern, nothing queued there)
//   ext       hipExtLaunchKernelGGL(kernel, ..., stopEvent = ev), kernel, ...   (the event bound to the kernel's
//             own completion signal instead of a marker packet of its own)
// Output: us per kernel over the chain (wall clock of the whole chain / K), one JSON line per case.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/event_record_probe tools/event_record_probe.hip
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ __launch_bounds__(256) void spin(long ticks, int* sink) {
  const long t0 = (long)__builtin_amdgcn_s_memrealtime();
  while ((long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
  if (threadIdx.x == 0 && blockIdx.x == 0 && ticks < 0) *sink = 1;
}

#define CK(x)                                                      \
  do {                                                             \
    hipError_t e_ = (x);                                           \
    if (e_ != hipSuccess) {                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      std::exit(1);                                                \
    }                                                              \
  } while (0)

int main() {
  constexpr int K = 200;
  const long ticks = 1000;  // 10 us of the 100 MHz clock
  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  int* sink;
  CK(hipMalloc(&sink, 4));
  std::vector<hipEvent_t> ev(K), evt(K);
  for (int i = 0; i < K; ++i) {
    CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming | hipEventDisableSystemFence));
    CK(hipEventCreate(&evt[i]));  // hipExtLaunchKernel records with the kernel's timestamps
  }
  const char* names[] = {"plain", "record", "record+wait", "ext_stop_event", "ext_stop_event+wait"};
  for (int rep = 0; rep < 3; ++rep)
    for (int c = 0; c < 5; ++c) {
      CK(hipDeviceSynchronize());
      const auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < K; ++i) {
        if (c >= 3) {
          hipExtLaunchKernelGGL(spin, dim3(256), dim3(256), 0, s, nullptr, evt[i], 0, ticks, sink);
          if (c == 4) CK(hipStreamWaitEvent(s2, evt[i], 0));
        } else {
          spin<<<256, 256, 0, s>>>(ticks, sink);
          if (c >= 1) CK(hipEventRecord(ev[i], s));
          if (c == 2) CK(hipStreamWaitEvent(s2, ev[i], 0));
        }
      }
      CK(hipStreamSynchronize(s));
      CK(hipStreamSynchronize(s2));
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      std::printf("{\"case\": \"%s\", \"rep\": %d, \"us_per_kernel\": %.2f}\n", names[c], rep, us / K);
      std::fflush(stdout);
    }
  return 0;
}
