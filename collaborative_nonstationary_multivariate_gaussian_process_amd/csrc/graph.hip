// Whole-step HIP graphs through the HIP runtime itself (include/nmgp_hip.h nmgp_graph_*).  Host code only.
// Round 4: the step graph used to be captured by torch.cuda.CUDAGraph; on this stack its capture_end crashed
// (SIGSEGV) on a side <-> side2 event ping-pong that the same HIP sequence captures and replays cleanly
// (tools/graph_edge_repro.hip), so the engine's schedule had to relay those edges through the main stream.
#include <hip/hip_runtime.h>

#include "common.hpp"

extern "C" {
int nmgp_graph_begin(hipStream_t stream) {
  if (stream == nullptr) return -1;   // the legacy null stream cannot be captured
  return hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal) == hipSuccess ? NMGP_OK : NMGP_ERR_LAUNCH;
}

int nmgp_graph_end(hipStream_t stream, void** exec_out) {
  if (stream == nullptr) return -1;
  if (exec_out == nullptr) return -2;
  *exec_out = nullptr;
  hipGraph_t g = nullptr;
  if (hipStreamEndCapture(stream, &g) != hipSuccess || g == nullptr) {
    (void)hipGetLastError();
    if (g) (void)hipGraphDestroy(g);
    return NMGP_ERR_LAUNCH;
  }
  hipGraphExec_t ex = nullptr;
  const hipError_t e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);   // the executable graph keeps what it needs
  if (e != hipSuccess || ex == nullptr) {
    (void)hipGetLastError();
    return NMGP_ERR_LAUNCH;
  }
  *exec_out = (void*)ex;
  return NMGP_OK;
}

int nmgp_graph_launch(void* exec, hipStream_t stream) {
  if (exec == nullptr) return -1;
  return hipGraphLaunch((hipGraphExec_t)exec, stream) == hipSuccess ? NMGP_OK : NMGP_ERR_LAUNCH;
}

int nmgp_graph_destroy(void* exec) {
  if (exec == nullptr) return NMGP_OK;
  return hipGraphExecDestroy((hipGraphExec_t)exec) == hipSuccess ? NMGP_OK : NMGP_ERR_LAUNCH;
}
}
