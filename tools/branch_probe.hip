// Probe: do two independent kernels overlap on the device (a) launched on
// two streams, (b) as the two branches of a captured hipGraph (fork / join
// through events during stream capture)?  Each kernel is 64 blocks that
// sleep ~T us: serialised they take 2T, overlapped T.  Prints one JSON line
// of microseconds per pair (median of 20).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__global__ void k_sleep(unsigned long long ticks, unsigned* out) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
  if (threadIdx.x == 0 && out) out[blockIdx.x] = 1;
}

using clk = std::chrono::steady_clock;

int main() {
  unsigned* buf;
  CK(hipMalloc(&buf, 1 << 16));
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  hipEvent_t fork, join;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  const unsigned long long T = 100ull * 100;  // 100 us of the 100 MHz wall clock
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  auto pair_on = [&](hipStream_t s1, hipStream_t s2) -> int {
    CK(hipEventRecord(fork, s1));
    CK(hipStreamWaitEvent(s2, fork, 0));
    hipLaunchKernelGGL(k_sleep, dim3(64), dim3(64), 0, s1, T, buf);
    hipLaunchKernelGGL(k_sleep, dim3(64), dim3(64), 0, s2, T, buf + 4096);
    CK(hipEventRecord(join, s2));
    CK(hipStreamWaitEvent(s1, join, 0));
    return 0;
  };
  std::vector<double> one, two, graph;
  for (int r = 0; r < 25; ++r) {
    CK(hipStreamSynchronize(a));
    auto t0 = clk::now();
    hipLaunchKernelGGL(k_sleep, dim3(64), dim3(64), 0, a, T, buf);
    hipLaunchKernelGGL(k_sleep, dim3(64), dim3(64), 0, a, T, buf + 4096);
    CK(hipStreamSynchronize(a));
    auto t1 = clk::now();
    if (pair_on(a, b)) return 1;
    CK(hipStreamSynchronize(a));
    auto t2 = clk::now();
    if (r >= 5) {
      one.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
      two.push_back(std::chrono::duration<double, std::micro>(t2 - t1).count());
    }
  }
  hipGraph_t g;
  CK(hipStreamBeginCapture(a, hipStreamCaptureModeThreadLocal));
  if (pair_on(a, b)) return 1;
  CK(hipStreamEndCapture(a, &g));
  hipGraphExec_t ge;
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  size_t nn = 0;
  CK(hipGraphGetNodes(g, nullptr, &nn));
  for (int r = 0; r < 25; ++r) {
    CK(hipStreamSynchronize(a));
    auto t0 = clk::now();
    CK(hipGraphLaunch(ge, a));
    CK(hipStreamSynchronize(a));
    auto t1 = clk::now();
    if (r >= 5) graph.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
  }
  std::printf("{\"kernel_us\": 100, \"one_stream_us\": %.1f, \"two_streams_us\": %.1f, "
              "\"graph_branches_us\": %.1f, \"graph_nodes\": %zu}\n",
              med(one), med(two), med(graph), nn);
  return 0;
}
