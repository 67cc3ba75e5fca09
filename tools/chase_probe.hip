// Probe: the latency of one dependent memory round trip as the tie-exact
// heap mode (DMC_OPT_HEAP_ORDER, csrc/dmc_heap.h) pays it -- one wave, each
// access's address taken from the previous access's data (a pointer chase
// over a random cyclic permutation), lanes reading neighbouring 16-byte
// entries of one 1-KB node as a wave-parallel sift does.  Working sets: 48 MB
// (the three heaps of 1M clients: 3 x 16 B x 1M), 256 MB and 4 GB.  Prints
// one JSON line: nanoseconds per dependent round trip per working set, and
// the same for LDS.
#include <hip/hip_runtime.h>

#include <cstdint>
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

constexpr uint32_t kNode = 1024;  // bytes per node: 64 lanes x 16 B

// nxt[node] (first dword of the node's first entry) = the next node
__global__ void k_chase(const uint4* __restrict__ buf, uint32_t start, uint32_t steps,
                        unsigned long long* out) {
  const uint32_t lane = threadIdx.x;
  uint32_t node = start;
  const unsigned long long t0 = wall_clock64();
  for (uint32_t i = 0; i < steps; ++i) {
    const uint4 v = buf[(size_t)node * (kNode / 16) + lane];
    node = __builtin_amdgcn_readfirstlane(v.x);
  }
  const unsigned long long t1 = wall_clock64();
  if (lane == 0) {
    out[0] = t1 - t0;
    out[1] = node;
  }
}

__global__ void k_link(uint4* buf, const uint32_t* nxt, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) reinterpret_cast<uint32_t*>(buf)[(size_t)i * (kNode / 4)] = nxt[i];
}

__global__ void k_chase_lds(uint32_t steps, unsigned long long* out) {
  __shared__ uint4 s[64 * 64];
  const uint32_t lane = threadIdx.x;
  for (uint32_t i = lane; i < 64 * 64; i += 64)
    s[i] = make_uint4(((i / 64) * 37 + 11) % 64, 0, 0, 0);
  __syncthreads();
  uint32_t node = 0;
  const unsigned long long t0 = wall_clock64();
  for (uint32_t i = 0; i < steps; ++i) {
    const uint4 v = s[node * 64 + lane];
    node = __builtin_amdgcn_readfirstlane(v.x);
  }
  const unsigned long long t1 = wall_clock64();
  if (lane == 0) {
    out[0] = t1 - t0;
    out[1] = node;
  }
}

int main() {
  const size_t sizes[] = {48ull << 20, 256ull << 20, 4ull << 30};
  const uint32_t steps = 4000;
  unsigned long long* d_out;
  CK(hipMalloc(&d_out, 16));
  std::printf("{");
  for (size_t sz : sizes) {
    const uint32_t n = (uint32_t)(sz / kNode);
    // a random cyclic permutation of the nodes (Sattolo)
    std::vector<uint32_t> perm(n);
    for (uint32_t i = 0; i < n; ++i) perm[i] = i;
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (uint32_t i = n - 1; i > 0; --i) {
      x ^= x << 13;
      x ^= x >> 7;
      x ^= x << 17;
      const uint32_t j = (uint32_t)(x % i);
      std::swap(perm[i], perm[j]);
    }
    uint4* d_buf;
    uint32_t* d_nxt;
    CK(hipMalloc(&d_buf, sz));
    CK(hipMalloc(&d_nxt, 4ull * n));
    CK(hipMemset(d_buf, 0, sz));
    // node perm[i] -> perm[i + 1]: each node's first dword
    std::vector<uint32_t> nxt(n);
    for (uint32_t i = 0; i < n; ++i) nxt[perm[i]] = perm[(i + 1) % n];
    CK(hipMemcpy(d_nxt, nxt.data(), 4ull * n, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_link, dim3((n + 255) / 256), dim3(256), 0, 0, d_buf, d_nxt, n);
    CK(hipDeviceSynchronize());
    CK(hipFree(d_nxt));
    hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, 0, d_buf, perm[0], 200, d_out);  // warm
    hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, 0, d_buf, perm[n / 2], steps, d_out);
    unsigned long long h[2];
    CK(hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost));
    std::printf("\"ns_per_trip_%zuMB\": %.1f, ", sz >> 20, h[0] * 10.0 / steps);  // 100 MHz clock
    CK(hipFree(d_buf));
  }
  hipLaunchKernelGGL(k_chase_lds, dim3(1), dim3(64), 0, 0, steps, d_out);
  unsigned long long h[2];
  CK(hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost));
  std::printf("\"ns_per_trip_lds\": %.1f}\n", h[0] * 10.0 / steps);
  return 0;
}
