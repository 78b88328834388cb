// Round-4 follow-up of tools/graph_edge_repro.hip: hipStreamEndCapture segfaulted for the ping-pong of
// tests/test_gpu_primitives.py::test_hip_graph_side_stream_ping_pong (captured through the library's own
// nmgp_graph_* calls, torch only supplying streams, events and elementwise kernels), while the round-3 raw
// repro passed.  This replays that test's exact API sequence and variants of it, one pattern per process:
//   base      m: record e0 (nothing launched on m yet); s1: wait e0, k, record e1; s2: wait e0, wait e1, k,
//             record e2; s1: wait e2, k, record e3; m: wait e3, wait e2
//   mfirst    base with a kernel on m before e0
//   s2k       base with a kernel on s2 between its two waits
//   nojoin2   base without m's (redundant) wait on e2
//   s1only    base without s2's wait on e0 (s2 joins the capture through e1 only)
//   hipGraphInstantiate + launch + check of the result follow the end of capture.
//   hipcc --offload-arch=gfx950 -O2 tools/graph_edge_repro2.hip -o tools/bin/graph_edge_repro2
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#define CK(x)                                                                \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      std::printf("FAIL %s -> %s\n", #x, hipGetErrorString(e_));             \
      std::fflush(stdout);                                                   \
      return 1;                                                              \
    }                                                                        \
  } while (0)

__global__ void axpb(double* x, const double* y, double a, double b) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  x[i] = a * x[i] + b + (y ? y[i] : 0.0);
}

static void stage(const char* s) {
  std::printf("stage %s\n", s);
  std::fflush(stdout);
}

int main(int argc, char** argv) {
  const char* pat = argc > 1 ? argv[1] : "base";
  const bool mfirst = !std::strcmp(pat, "mfirst"), s2k = !std::strcmp(pat, "s2k");
  const bool nojoin2 = !std::strcmp(pat, "nojoin2"), s1only = !std::strcmp(pat, "s1only");
  hipStream_t m, s1, s2;
  CK(hipStreamCreateWithPriority(&m, hipStreamNonBlocking, 0));
  CK(hipStreamCreateWithPriority(&s1, hipStreamNonBlocking, 0));
  CK(hipStreamCreateWithPriority(&s2, hipStreamNonBlocking, 0));
  double *x, *y, *z;
  CK(hipMalloc(&x, 4096 * 8));
  CK(hipMalloc(&y, 4096 * 8));
  CK(hipMalloc(&z, 4096 * 8));
  CK(hipMemset(x, 0, 4096 * 8));
  CK(hipMemset(y, 0, 4096 * 8));
  CK(hipMemset(z, 0, 4096 * 8));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1, e2, e3;
  for (hipEvent_t* e : {&e0, &e1, &e2, &e3}) CK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  stage("begin_capture");
  CK(hipStreamBeginCapture(m, hipStreamCaptureModeThreadLocal));
  if (mfirst) hipLaunchKernelGGL(axpb, dim3(16), dim3(256), 0, m, z, nullptr, 1.0, 1.0);
  CK(hipEventRecord(e0, m));
  CK(hipStreamWaitEvent(s1, e0, 0));
  hipLaunchKernelGGL(axpb, dim3(16), dim3(256), 0, s1, x, nullptr, 1.0, 1.0);      // x += 1
  CK(hipEventRecord(e1, s1));
  if (!s1only) CK(hipStreamWaitEvent(s2, e0, 0));
  if (s2k) hipLaunchKernelGGL(axpb, dim3(16), dim3(256), 0, s2, z, nullptr, 1.0, 1.0);
  CK(hipStreamWaitEvent(s2, e1, 0));                                                 // s1 -> s2
  hipLaunchKernelGGL(axpb, dim3(16), dim3(256), 0, s2, y, x, 1.0, 0.0);            // y += x
  CK(hipEventRecord(e2, s2));
  CK(hipStreamWaitEvent(s1, e2, 0));                                                 // s2 -> s1
  hipLaunchKernelGGL(axpb, dim3(16), dim3(256), 0, s1, x, nullptr, 2.0, 0.0);      // x *= 2
  CK(hipEventRecord(e3, s1));
  CK(hipStreamWaitEvent(m, e3, 0));
  if (!nojoin2) CK(hipStreamWaitEvent(m, e2, 0));
  CK(hipGetLastError());
  stage("end_capture");
  hipGraph_t g;
  CK(hipStreamEndCapture(m, &g));
  stage("instantiate");
  hipGraphExec_t ge;
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  stage("launch");
  for (int r = 0; r < 3; ++r) CK(hipGraphLaunch(ge, m));
  CK(hipStreamSynchronize(m));
  double hx, hy;
  CK(hipMemcpy(&hx, x, 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&hy, y, 8, hipMemcpyDeviceToHost));
  std::printf("ok pattern=%s x=%g y=%g (expect 14 11)\n", pat, hx, hy);
  return 0;
}
