// Does HIP stream capture take what the GP fit enqueues: H2D copies from
// pinned memory, memsets, ~200 kernel launches, and an event record in the
// middle (ev_fit_x) that another stream waits on?  And what does replaying the
// instantiated graph cost the host against launching the kernels one by one?
//   hipcc -O3 --offload-arch=gfx950 scripts/exp/graph_capture_probe.hip -o scripts/exp/graph_capture_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      printf("HIP error %s (%d) at %s:%d\n", hipGetErrorString(e_), (int)e_, __FILE__, __LINE__); \
      exit(1);                                                                                 \
    }                                                                                          \
  } while (0)

__global__ void k_step(double* x, int n, double a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = x[i] * a + 1.0;
}

static void enqueue(hipStream_t s, double* d, const double* h, int n, int nk, hipEvent_t mid) {
  CK(hipMemcpyAsync(d, h, sizeof(double) * n, hipMemcpyHostToDevice, s));
  CK(hipMemsetAsync(d + n, 0, sizeof(double) * 16, s));
  for (int k = 0; k < nk; ++k) {
    hipLaunchKernelGGL(k_step, dim3((n + 255) / 256), dim3(256), 0, s, d, n, 0.5);
    if (k == nk / 4) CK(hipEventRecord(mid, s));
  }
}

int main() {
  const int n = 1 << 16, nk = 200;
  double *d, *h, *o;
  CK(hipMalloc(&d, sizeof(double) * (n + 16)));
  CK(hipMalloc(&o, sizeof(double) * n));
  CK(hipHostMalloc((void**)&h, sizeof(double) * n, hipHostMallocDefault));
  for (int i = 0; i < n; ++i) h[i] = i;
  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t mid, done;
  CK(hipEventCreateWithFlags(&mid, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
  // direct
  enqueue(s, d, h, n, nk, mid);
  CK(hipStreamSynchronize(s));
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < 10; ++r) enqueue(s, d, h, n, nk, mid);
  auto t1 = std::chrono::steady_clock::now();
  CK(hipStreamSynchronize(s));
  double ref;
  CK(hipMemcpy(&ref, d + 1234, sizeof(double), hipMemcpyDeviceToHost));
  // captured
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  enqueue(s, d, h, n, nk, mid);
  CK(hipStreamEndCapture(s, &g));
  size_t nn = 0;
  CK(hipGraphGetNodes(g, nullptr, &nn));
  auto t2 = std::chrono::steady_clock::now();
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  auto t3 = std::chrono::steady_clock::now();
  CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  auto t4 = std::chrono::steady_clock::now();
  for (int r = 0; r < 10; ++r) {
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamWaitEvent(s2, mid, 0));   // the mid-graph event, waited on by another stream
    hipLaunchKernelGGL(k_step, dim3((n + 255) / 256), dim3(256), 0, s2, o, n, 0.0);
  }
  auto t5 = std::chrono::steady_clock::now();
  CK(hipStreamSynchronize(s));
  CK(hipStreamSynchronize(s2));
  double got;
  CK(hipMemcpy(&got, d + 1234, sizeof(double), hipMemcpyDeviceToHost));
  auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
  printf("graph nodes %zu; direct enqueue %.1f us per fit (%d launches); instantiate %.1f us; "
         "graph launch %.1f us per fit; result %s (%.17g vs %.17g)\n",
         nn, us(t0, t1) / 10, nk, us(t2, t3), us(t4, t5) / 10, got == ref ? "equal" : "DIFFERENT", got, ref);
  return got == ref ? 0 : 1;
}
