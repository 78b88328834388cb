// Minimal HIP-only reproducer of the hipGraph crash seen with the DSVI step schedule:
// stream capture on `m`, fork to two side streams s / s2, then an event edge s -> s2 followed by an
// edge s2 -> s (each edge: record on the source, wait on the destination, one kernel after the
// wait), join both to `m`, end capture, instantiate, launch.  Each stage prints before it starts, so
// the last line names the call that crashed.  tools/graph_edge_probe.py found the same pattern
// ("ping_pong") segfaulting through torch; this takes torch out of the picture.
//
//   hipcc --offload-arch=gfx950 -O2 tools/graph_edge_repro.hip -o tools/bin/graph_edge_repro
//   tools/bin/graph_edge_repro <pattern> [global] [autofree]   pattern: ping_pong | one_way | relay
//   global: hipStreamCaptureModeGlobal (torch's default) instead of ThreadLocal; autofree: instantiate with
//   hipGraphInstantiateFlagAutoFreeOnLaunch through hipGraphInstantiateWithFlags (what torch's CUDAGraph uses);
//   destroy: hipEventDestroy on each edge's event right after the wait, while the capture is still open
//   (what Python's garbage collection of a torch.cuda.Event does mid-capture); query: hipStreamGetCaptureInfo(_v2)
//   on the launching stream before every launch (what torch's caching allocator does for its ops)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::printf("FAIL %s -> %s\n", #x, hipGetErrorString(e_));                       \
      std::fflush(stdout);                                                             \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

__global__ void bump(float* x, float v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  x[i] += v;
}

static void stage(const char* s) {
  std::printf("stage %s\n", s);
  std::fflush(stdout);
}

static bool g_destroy = false;   // destroy each edge's event right after the wait (still capturing)
static bool g_query = false;     // query the capture info of the launching stream before every launch

static void query(hipStream_t s) {
  if (!g_query) return;
  hipStreamCaptureStatus st;
  unsigned long long id = 0;
  hipGraph_t gr = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t nd = 0;
  (void)hipStreamGetCaptureInfo(s, &st, &id);
  (void)hipStreamGetCaptureInfo_v2(s, &st, &id, &gr, &deps, &nd);
}

static int edge(hipStream_t from, hipStream_t to, float* buf, float v) {
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  CK(hipEventRecord(ev, from));
  CK(hipStreamWaitEvent(to, ev, 0));
  if (g_destroy) CK(hipEventDestroy(ev));
  query(to);
  hipLaunchKernelGGL(bump, dim3(4), dim3(256), 0, to, buf, v);
  CK(hipGetLastError());
  return 0;
}

int main(int argc, char** argv) {
  const char* pat = argc > 1 ? argv[1] : "ping_pong";
  bool global = false, autofree = false;
  for (int i = 2; i < argc; ++i) {
    if (!std::strcmp(argv[i], "global")) global = true;
    if (!std::strcmp(argv[i], "autofree")) autofree = true;
    if (!std::strcmp(argv[i], "destroy")) g_destroy = true;
    if (!std::strcmp(argv[i], "query")) g_query = true;
  }
  std::printf("mode=%s instantiate=%s\n", global ? "global" : "thread_local", autofree ? "with_flags(autofree)" : "plain");
  std::fflush(stdout);
  hipStream_t m, s, s2;
  int prio = 0;
  bool use_prio = false;
  for (int i = 2; i < argc; ++i)
    if (!std::strncmp(argv[i], "prio=", 5)) {
      use_prio = true;
      prio = atoi(argv[i] + 5);
    }
  if (use_prio) {   // what torch's stream pool does (cudaStreamCreateWithPriority, non-blocking)
    CK(hipStreamCreateWithPriority(&m, hipStreamNonBlocking, prio));
    CK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, prio));
    CK(hipStreamCreateWithPriority(&s2, hipStreamNonBlocking, prio));
  } else {
    CK(hipStreamCreateWithFlags(&m, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  }
  float *a, *b, *c;
  CK(hipMalloc(&a, 4096));
  CK(hipMalloc(&b, 4096));
  CK(hipMalloc(&c, 4096));
  CK(hipMemset(a, 0, 4096));
  CK(hipMemset(b, 0, 4096));
  CK(hipMemset(c, 0, 4096));
  CK(hipDeviceSynchronize());

  stage("begin_capture");
  CK(hipStreamBeginCapture(m, global ? hipStreamCaptureModeGlobal : hipStreamCaptureModeThreadLocal));
  hipEvent_t fork;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventRecord(fork, m));
  CK(hipStreamWaitEvent(s, fork, 0));
  CK(hipStreamWaitEvent(s2, fork, 0));
  query(m);
  hipLaunchKernelGGL(bump, dim3(4), dim3(256), 0, m, a, 1.f);
  query(s);
  hipLaunchKernelGGL(bump, dim3(4), dim3(256), 0, s, b, 1.f);
  query(s2);
  hipLaunchKernelGGL(bump, dim3(4), dim3(256), 0, s2, c, 1.f);
  if (!std::strcmp(pat, "ping_pong")) {            // s -> s2, then s2 -> s
    if (edge(s, s2, c, 1.f) || edge(s2, s, b, 1.f)) return 1;
  } else if (!std::strcmp(pat, "one_way")) {       // s -> s2 only
    if (edge(s, s2, c, 1.f)) return 1;
  } else if (!std::strcmp(pat, "relay")) {         // the shipped workaround: s -> m -> s2, s2 -> m -> s
    if (edge(s, m, a, 1.f) || edge(m, s2, c, 1.f) || edge(s2, m, a, 1.f) || edge(m, s, b, 1.f)) return 1;
  }
  hipEvent_t j1, j2;
  CK(hipEventCreateWithFlags(&j1, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&j2, hipEventDisableTiming));
  CK(hipEventRecord(j1, s));
  CK(hipEventRecord(j2, s2));
  CK(hipStreamWaitEvent(m, j1, 0));
  CK(hipStreamWaitEvent(m, j2, 0));
  stage("end_capture");
  hipGraph_t g;
  CK(hipStreamEndCapture(m, &g));
  size_t nn = 0;
  CK(hipGraphGetNodes(g, nullptr, &nn));
  std::printf("graph nodes %zu\n", nn);
  stage("instantiate");
  hipGraphExec_t ge;
  if (autofree)
    CK(hipGraphInstantiateWithFlags(&ge, g, hipGraphInstantiateFlagAutoFreeOnLaunch));
  else
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  stage("launch");
  CK(hipGraphLaunch(ge, m));
  CK(hipStreamSynchronize(m));
  float hb[4];
  CK(hipMemcpy(hb, b, sizeof(hb), hipMemcpyDeviceToHost));
  std::printf("ok pattern=%s b[0]=%g\n", pat, hb[0]);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return 0;
}
