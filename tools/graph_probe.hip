// Probe: host-side cost of graph replay with a parameter update, D2H readback
// into pageable vs pinned memory, and stream sync (MI355X host overheads).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

struct P { unsigned k; unsigned pad; double now; void* out; unsigned long long tick; };
__global__ void k_param(P p, unsigned* ctl) { if (threadIdx.x == 0 && blockIdx.x == 0) ctl[0] = p.k; }
__global__ void k_work(unsigned* ctl, int i) { if (threadIdx.x == 0 && blockIdx.x == 0) ctl[1 + (i & 7)] += ctl[0]; }

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  unsigned* ctl;
  (void)hipMalloc(&ctl, 4096);
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  const int K = 14, R = 300;
  hipGraph_t g;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  P p0{1, 0, 1.0, nullptr, 0};
  hipLaunchKernelGGL(k_param, dim3(2048), dim3(256), 0, s, p0, ctl);
  for (int i = 0; i < K; ++i) hipLaunchKernelGGL(k_work, dim3(512), dim3(256), 0, s, ctl, i);
  (void)hipStreamEndCapture(s, &g);
  hipGraphExec_t ge;
  (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphNode_t root;
  size_t nr = 1;
  (void)hipGraphGetRootNodes(g, &root, &nr);
  hipKernelNodeParams kp;
  (void)hipGraphKernelNodeGetParams(root, &kp);
  unsigned* pinned;
  (void)hipHostMalloc(&pinned, 4096, 0);
  unsigned pageable[64];
  for (int w = 0; w < 10; ++w) (void)hipGraphLaunch(ge, s);
  (void)hipStreamSynchronize(s);
  double t_set = 0, t_launch = 0, t_sync = 0, t_total = 0;
  for (int r = 0; r < R; ++r) {
    auto a = clk::now();
    P p{(unsigned)r, 0, 1.0 + r, nullptr, 0};
    void* args[] = {&p, &ctl};
    kp.kernelParams = args;
    (void)hipGraphExecKernelNodeSetParams(ge, root, &kp);
    auto b = clk::now();
    (void)hipGraphLaunch(ge, s);
    auto c = clk::now();
    (void)hipStreamSynchronize(s);
    auto d = clk::now();
    t_set += us(a, b); t_launch += us(b, c); t_sync += us(c, d); t_total += us(a, d);
  }
  printf("graph(%d kernels): setparams %.2f us, launch %.2f us, sync-wait %.2f us, total %.2f us\n",
         K + 1, t_set / R, t_launch / R, t_sync / R, t_total / R);
  t_total = 0;
  for (int r = 0; r < R; ++r) {
    auto a = clk::now();
    (void)hipGraphLaunch(ge, s);
    (void)hipStreamSynchronize(s);
    t_total += us(a, clk::now());
  }
  printf("graph launch+sync without setparams: %.2f us\n", t_total / R);
  // readback variants after a tiny kernel
  for (int mode = 0; mode < 3; ++mode) {
    double t = 0;
    for (int r = 0; r < R; ++r) {
      auto a = clk::now();
      hipLaunchKernelGGL(k_work, dim3(1), dim3(64), 0, s, ctl, r);
      if (mode == 0) (void)hipMemcpyAsync(pageable, ctl, 64, hipMemcpyDeviceToHost, s);
      if (mode == 1) (void)hipMemcpyAsync(pinned, ctl, 64, hipMemcpyDeviceToHost, s);
      (void)hipStreamSynchronize(s);
      t += us(a, clk::now());
    }
    printf("kernel + %s + sync: %.2f us\n", mode == 0 ? "D2H pageable" : mode == 1 ? "D2H pinned" : "no copy", t / R);
  }
  // H2D small copies
  for (int mode = 0; mode < 2; ++mode) {
    double t = 0;
    for (int r = 0; r < R; ++r) {
      auto a = clk::now();
      (void)hipMemcpyAsync(ctl + 64, mode ? (void*)pinned : (void*)pageable, 32, hipMemcpyHostToDevice, s);
      t += us(a, clk::now());
    }
    (void)hipStreamSynchronize(s);
    printf("H2D 32B %s enqueue: %.2f us\n", mode ? "pinned" : "pageable", t / R);
  }
  return 0;
}
