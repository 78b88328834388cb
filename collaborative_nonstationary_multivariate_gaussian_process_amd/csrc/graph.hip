// Whole-step HIP graphs through the HIP runtime itself (include/nmgp_hip.h nmgp_graph_*).  Host code only.
// Round 4: the step graph used to be captured by torch.cuda.CUDAGraph; on this stack its capture_end crashed
// (SIGSEGV) on a side <-> side2 event ping-pong that the same HIP sequence captures and replays cleanly
// (tools/graph_edge_repro.hip), so the engine's schedule had to relay those edges through the main stream.
#include <hip/hip_runtime.h>

#include <cstdio>

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

int nmgp_event_create(void** event_out) {
  if (event_out == nullptr) return -1;
  *event_out = nullptr;
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return NMGP_ERR_LAUNCH;
  *event_out = (void*)e;
  return NMGP_OK;
}

int nmgp_event_destroy(void* event) {
  if (event == nullptr) return NMGP_OK;
  return hipEventDestroy((hipEvent_t)event) == hipSuccess ? NMGP_OK : NMGP_ERR_LAUNCH;
}

// During a capture the event record node is added to the capture graph explicitly (the torch-bundled ROCm 7.0
// runtime refuses hipEventRecordWithFlags(..., hipEventRecordExternal) on a capturing stream): it depends on
// the stream's current capture dependencies, and becomes the stream's only dependency, so everything captured
// on the stream afterwards follows it.  Outside a capture: a plain event record.
int nmgp_event_record_external(void* event, hipStream_t stream) {
  if (event == nullptr) return -1;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  hipGraph_t g = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t ndeps = 0;
  hipError_t e = hipStreamGetCaptureInfo_v2(stream, &st, &id, &g, &deps, &ndeps);
  if (e != hipSuccess) {
    std::fprintf(stderr, "nmgp_event_record_external: hipStreamGetCaptureInfo_v2: %s\n", hipGetErrorString(e));
    return NMGP_ERR_LAUNCH;
  }
  if (st != hipStreamCaptureStatusActive)
    return hipEventRecord((hipEvent_t)event, stream) == hipSuccess ? NMGP_OK : NMGP_ERR_LAUNCH;
  hipGraphNode_t node = nullptr;
  e = hipGraphAddEventRecordNode(&node, g, deps, ndeps, (hipEvent_t)event);
  if (e != hipSuccess) {
    std::fprintf(stderr, "nmgp_event_record_external: hipGraphAddEventRecordNode: %s\n", hipGetErrorString(e));
    return NMGP_ERR_LAUNCH;
  }
  e = hipStreamUpdateCaptureDependencies(stream, &node, 1, hipStreamSetCaptureDependencies);
  if (e != hipSuccess) {
    std::fprintf(stderr, "nmgp_event_record_external: hipStreamUpdateCaptureDependencies: %s\n", hipGetErrorString(e));
    return NMGP_ERR_LAUNCH;
  }
  return NMGP_OK;
}

int nmgp_stream_wait_event(hipStream_t stream, void* event) {
  if (event == nullptr) return -2;
  return hipStreamWaitEvent(stream, (hipEvent_t)event, 0) == hipSuccess ? NMGP_OK : NMGP_ERR_LAUNCH;
}
}
