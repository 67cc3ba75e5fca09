// Probe: cost of a chain of dependent small kernels on one stream, launched
// one by one vs. captured into a hipGraph (MI355X launch-overhead model).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void k_tiny(unsigned* p, int i) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[i & 1023] += 1;
}
__global__ void k_touch(double* a, size_t n) {  // streams n doubles
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = a[i] * 1.0000001;
}


// grid barrier via a monotone arrival counter (all blocks co-resident)
__device__ void grid_barrier(unsigned* ctr, unsigned nblocks, unsigned& epoch) {
  __syncthreads();
  epoch += nblocks;
  if (threadIdx.x == 0) {
    __threadfence();
    atomicAdd(ctr, 1u);
    unsigned spins = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < epoch &&
           ++spins < (1u << 18))
      __builtin_amdgcn_s_sleep(1);
  }
  __syncthreads();
}
__global__ void k_persist(unsigned* ctr, int iters, double* a, size_t n) {
  unsigned epoch = 0;
  for (int i = 0; i < iters; ++i) {
    if (a) {
      size_t j = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
      for (; j < n; j += (size_t)gridDim.x * blockDim.x) a[j] = a[j] * 1.0000001;
    }
    grid_barrier(ctr, gridDim.x, epoch);
  }
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  unsigned* p;
  double* a;
  size_t n = 1 << 20;
  hipMalloc(&p, 4096 * 4);
  hipMalloc(&a, n * 8);
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  const int K = 32, R = 200;
  for (int mode = 0; mode < 2; ++mode) {
    for (int big = 0; big < 2; ++big) {
      auto chain = [&]() {
        for (int i = 0; i < K; ++i) {
          if (big)
            hipLaunchKernelGGL(k_touch, dim3(1024), dim3(256), 0, s, a, n);
          else
            hipLaunchKernelGGL(k_tiny, dim3(big ? 4096 : 64), dim3(256), 0, s, p, i);
        }
      };
      hipGraphExec_t ge = nullptr;
      if (mode == 1) {
        hipGraph_t g;
        hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
        chain();
        hipStreamEndCapture(s, &g);
        hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
      }
      for (int w = 0; w < 5; ++w) {
        if (mode) hipGraphLaunch(ge, s); else chain();
      }
      hipStreamSynchronize(s);
      auto t0 = std::chrono::steady_clock::now();
      double host_us = 0;
      for (int r = 0; r < R; ++r) {
        auto h0 = std::chrono::steady_clock::now();
        if (mode) hipGraphLaunch(ge, s); else chain();
        host_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count();
      }
      hipStreamSynchronize(s);
      double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      std::printf("%s %s: %.2f us per kernel (host enqueue %.2f us per kernel)\n",
                  mode ? "graph " : "stream", big ? "touch8MB" : "tiny    ", us / R / K,
                  host_us / R / K);
      // single sync round trip
    }
  }
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < R; ++r) {
    hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, p, r);
    hipStreamSynchronize(s);
  }
  double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  std::printf("launch+sync round trip: %.2f us\n", us / R);

  for (int nb : {256, 512, 1024}) for (int big = 0; big < 2; ++big) {
    unsigned* ctr; hipMalloc(&ctr, 4);
    hipMemset(ctr, 0, 4);
    hipLaunchKernelGGL(k_persist, dim3(nb), dim3(256), 0, s, ctr, 10, big ? a : nullptr, n);
    hipStreamSynchronize(s);
    hipMemset(ctr, 0, 4);
    auto t1 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(k_persist, dim3(nb), dim3(256), 0, s, ctr, 200, big ? a : nullptr, n);
    hipStreamSynchronize(s);
    double us2 = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t1).count();
    std::printf("persistent %d blocks %s: %.2f us per barrier\n", nb, big ? "touch8MB" : "empty", us2 / 200);
    hipFree(ctr);
  }
  return 0;
}
