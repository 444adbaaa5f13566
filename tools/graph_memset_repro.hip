// Minimal HIP-only reproduction of the hipGraph replay drift: a captured
// hipMemsetAsync followed, on the same stream, by a kernel that atomically accumulates into the
// cleared buffer — the pattern of pld_listmle_fwd_bwd (zero dpred, scatter-add the ListMLE
// gradient), the one call tools/graph_bisect.py found drifting when replayed from a graph.
//
// Every replay must leave sum(buf) == number of adds. Variants: the clear as a memset node or as
// a kernel node, on a small (the bisect's 2x64x64) and the benchmark's (32x448x448) buffer, the
// graph launched onto an idle stream or behind a long-running kernel.
// Run with DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 (the runtime default) and =0.
//   hipcc --offload-arch=gfx950 -O2 tools/graph_memset_repro.hip -o tools/bin/graph_memset_repro
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      std::printf("%s: %s\n", #x, hipGetErrorString(e));                            \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

__global__ void zero_kernel(float* p, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    p[i] = 0.f;
}

// m adds of 1.0 spread over the buffer (duplicates included), like the ListMLE scatter
__global__ void scatter_kernel(float* p, long n, long m) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) atomicAdd(p + (i * 7919) % n, 1.0f);
}

// keeps the stream busy when the graph is launched (the training step's forward runs ahead of
// the ListMLE call): a dependent FMA chain per thread, result stored so it is not elided
__global__ void busy_kernel(float* sink, int iters) {
  float a = threadIdx.x * 1e-3f, b = 0.999f;
  for (int i = 0; i < iters; ++i) a = fmaf(a, b, 1e-4f);
  if (a == 12345.f) sink[threadIdx.x] = a;
}

__global__ void sum_kernel(const float* p, long n, double* out) {
  __shared__ double red[256];
  double a = 0.0;
  for (long i = threadIdx.x; i < n; i += 256) a += p[i];
  red[threadIdx.x] = a;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = red[0];
}

static int run(long n, long m, bool memset_node, bool busy, int reps) {
  float* buf;
  double* dsum;
  CK(hipMalloc(&buf, n * sizeof(float)));
  CK(hipMalloc(&dsum, sizeof(double)));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  // pre-fill with garbage so a skipped or late clear shows up
  zero_kernel<<<1024, 256, 0, st>>>(buf, n);
  scatter_kernel<<<(unsigned)((m + 255) / 256), 256, 0, st>>>(buf, n, m);
  CK(hipStreamSynchronize(st));
  hipGraph_t g;
  hipGraphExec_t ex;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  if (memset_node)
    CK(hipMemsetAsync(buf, 0, n * sizeof(float), st));
  else
    zero_kernel<<<1024, 256, 0, st>>>(buf, n);
  scatter_kernel<<<(unsigned)((m + 255) / 256), 256, 0, st>>>(buf, n, m);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  int bad = 0, first = -1;
  double worst = (double)m;
  for (int r = 0; r < reps; ++r) {
    if (busy) busy_kernel<<<1024, 256, 0, st>>>(buf, 20000);
    CK(hipGraphLaunch(ex, st));
    sum_kernel<<<1, 256, 0, st>>>(buf, n, dsum);
    double s = 0;
    CK(hipMemcpyAsync(&s, dsum, sizeof(double), hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    if (s != (double)m) {
      if (first < 0) first = r;
      ++bad;
      if (s != worst && (first == r || s > worst)) worst = s;
    }
  }
  std::printf("%-11s %-4s n=%-9ld adds=%-7ld replays=%d  wrong=%d  first_wrong=%d  "
              "example_sum=%.0f (expected %ld)\n",
              memset_node ? "memset-node" : "kernel-node", busy ? "busy" : "idle", n, m, reps,
              bad, first,
              bad ? worst : (double)m, m);
  CK(hipGraphExecDestroy(ex));
  CK(hipGraphDestroy(g));
  CK(hipStreamDestroy(st));
  CK(hipFree(buf));
  CK(hipFree(dsum));
  return bad;
}

int main() {
  const char* pc = std::getenv("DEBUG_CLR_GRAPH_PACKET_CAPTURE");
  std::printf("DEBUG_CLR_GRAPH_PACKET_CAPTURE=%s\n", pc ? pc : "<unset>");
  int bad = 0;
  for (long n : {2L * 64 * 64, 32L * 448 * 448})
    for (long m : {200L, 16000L})
      for (bool ms : {true, false})
        for (bool busy : {false, true}) bad += run(n, m, ms, busy, 100);
  return bad ? 2 : 0;
}
