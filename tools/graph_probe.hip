// graph_probe.hip -- is a chain of small dependent kernels cheaper as one hipGraph replay than as
// eager stream launches on this stack?  (Decides whether TRecurrentCu's per-frame launch chain --
// 9 launches a frame, ~4 us each -- is bounded by host submission or by the GPU's kernel boundary.)
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/graph_probe tools/graph_probe.hip
//   ./tools/graph_probe [launches] [workgroups] [work]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

// a dependent step: every workgroup reads the previous step's value and writes its own slot
// (`work` dependent FMAs per thread stretch the kernel to a few microseconds: GPU-bound chains)
__global__ void step_kernel(float* __restrict__ p, int i, int work) {
  const int slot = blockIdx.x * blockDim.x + threadIdx.x;
  float v = p[slot];
  for (int k = 0; k < work; ++k) v = v * 0.999f + 1e-3f;
  p[slot] = v * 0.5f + (float)(i & 7);
}

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 9000;
  const int wg = argc > 2 ? atoi(argv[2]) : 16;
  const int work = argc > 3 ? atoi(argv[3]) : 0;
  float* d;
  CK(hipMalloc(&d, (size_t)wg * 256 * 4));
  CK(hipMemset(d, 0, (size_t)wg * 256 * 4));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int i = 0; i < 200; ++i) step_kernel<<<wg, 256, 0, s>>>(d, i, work);
  CK(hipStreamSynchronize(s));

  for (int rep = 0; rep < 3; ++rep) {
    double t0 = now();
    for (int i = 0; i < n; ++i) step_kernel<<<wg, 256, 0, s>>>(d, i, work);
    const double t_enq = now() - t0;
    CK(hipStreamSynchronize(s));
    const double t_eager = now() - t0;

    hipGraph_t g;
    hipGraphExec_t ge;
    t0 = now();
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < n; ++i) step_kernel<<<wg, 256, 0, s>>>(d, i, work);
    CK(hipStreamEndCapture(s, &g));
    const double t_cap = now() - t0;
    t0 = now();
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    const double t_inst = now() - t0;
    CK(hipGraphLaunch(ge, s));  // first launch (uploads)
    CK(hipStreamSynchronize(s));
    t0 = now();
    CK(hipGraphLaunch(ge, s));
    const double t_glaunch = now() - t0;
    CK(hipStreamSynchronize(s));
    const double t_graph = now() - t0;
    printf("launches %d wg %d work %d: eager %.2f us/launch (host enqueue %.2f), graph replay %.2f us/launch "
           "(hipGraphLaunch call %.1f us), capture %.1f ms, instantiate %.1f ms\n",
           n, wg, work, 1e6 * t_eager / n, 1e6 * t_enq / n, 1e6 * t_graph / n, 1e6 * t_glaunch, 1e3 * t_cap,
           1e3 * t_inst);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  CK(hipFree(d));
  return 0;
}
