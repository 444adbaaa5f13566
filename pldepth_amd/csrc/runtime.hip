// Runtime glue of libpldepth_hip.so: error text, version, hipGraph capture of a training step.
#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "common.h"

namespace pld {

static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return PLD_ERR_HIP;
  }
  return PLD_OK;
}

}  // namespace pld

extern "C" {

const char* pld_last_error(void) { return pld::g_err; }

int pld_version(void) { return 1; }

int pld_graph_begin(void* stream) {
  PLD_HIP(hipStreamBeginCapture(pld::as_stream(stream), hipStreamCaptureModeThreadLocal));
  return PLD_OK;
}

int pld_graph_end(void* stream, void** graph_exec) {
  hipGraph_t g = nullptr;
  PLD_HIP(hipStreamEndCapture(pld::as_stream(stream), &g));
  hipGraphExec_t ex = nullptr;
  hipError_t e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  hipGraphDestroy(g);
  if (e != hipSuccess) {
    pld::set_error("hipGraphInstantiate failed: %s", hipGetErrorString(e));
    return PLD_ERR_HIP;
  }
  *graph_exec = reinterpret_cast<void*>(ex);
  return PLD_OK;
}

int pld_graph_launch(void* graph_exec, void* stream) {
  PLD_HIP(hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(graph_exec), pld::as_stream(stream)));
  return PLD_OK;
}

int pld_graph_destroy(void* graph_exec) {
  PLD_HIP(hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(graph_exec)));
  return PLD_OK;
}

}  // extern "C"
