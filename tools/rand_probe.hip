// SPDX-License-Identifier: LGPL-2.1
//
// Random-record read rates on the engine's access shapes (HIP events, no
// profiler): what one walker level costs when each lane reads
//   r64     one random 64-byte record (a ring entry or a ClientRec)
//   r128    one random 128-byte-aligned record (two adjacent 64-byte lines)
//   r64x2   two independent random 64-byte records
//   r64x4   four independent random 64-byte records (k_remit's first level:
//           the client record and three ring entries)
//   r64adj2 two adjacent 64-byte records from a random 64-byte boundary
//           (queue positions 0 and 1 of a ring: one 128-byte line or two)
// over a 4 GiB buffer (the 1M-client rings), at n lanes (71,680: a config-3
// round's candidates; and 1M), each pattern after an Infinity Cache
// eviction pass.  Prints one JSON line: per pattern and n, microseconds per
// launch, records/s and 64-byte lines/s.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

constexpr uint64_t kBuf = 4ull << 30;
constexpr uint32_t kThreads = 256;

__device__ inline uint64_t perm(uint64_t i, uint64_t salt, int bits) {
  return ((i + salt) * 0x9E3779B97F4A7C15ull >> 7) & ((1ull << bits) - 1);
}

__global__ void evict(const uint4* __restrict__ p, uint64_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

// L lines of 64 bytes per lane: `adj` consecutive ones from each of R random
// starts (64-byte aligned, or 128-byte aligned when a128)
template <int R, int ADJ, bool A128>
__global__ void probe(const uint4* __restrict__ p, uint64_t n, uint64_t salt, uint32_t* out) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint4 v[R * ADJ * 4];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    uint64_t line = perm(i * R + r, salt, 25);  // of 2^26 64-byte lines
    if (A128) line &= ~1ull;
#pragma unroll
    for (int a = 0; a < ADJ; ++a)
#pragma unroll
      for (int k = 0; k < 4; ++k) v[(r * ADJ + a) * 4 + k] = p[(line + a) * 4 + k];
  }
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < R * ADJ * 4; ++j) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
  if (acc == 0x9e3779b9u) out[0] = acc;
}

template <int R, int ADJ, bool A128>
int run(const char* name, const uint4* p, uint32_t* out, uint64_t n, bool first) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const dim3 g((unsigned)((n + kThreads - 1) / kThreads));
  float tot = 0.f;
  const int reps = 8;
  for (int rep = 0; rep < reps; ++rep) {
    hipLaunchKernelGGL(evict, dim3(8192), dim3(kThreads), 0, 0, p, kBuf / 16, out);
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((probe<R, ADJ, A128>), g, dim3(kThreads), 0, 0, p, n,
                       (uint64_t)rep * 977 + 13, out);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    if (rep) tot += ms;  // (the first launch warms the code)
  }
  const double us = tot / (reps - 1) * 1e3;
  const double lines = (double)n * R * ADJ;
  std::printf("%s\"%s_n%llu\": {\"us\": %.2f, \"records_per_s\": %.4g, \"lines64_per_s\": %.4g}",
              first ? "" : ", ", name, (unsigned long long)n, us, n * R / (us * 1e-6),
              lines / (us * 1e-6));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return 0;
}

int main() {
  void* buf = nullptr;
  uint32_t* out = nullptr;
  CK(hipMalloc(&buf, kBuf));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(buf, 1, kBuf));
  CK(hipDeviceSynchronize());
  const uint4* p = static_cast<const uint4*>(buf);
  std::printf("{");
  bool first = true;
  for (uint64_t n : {71680ull, 1ull << 20}) {
    if (run<1, 1, false>("r64", p, out, n, first)) return 1;
    first = false;
    if (run<1, 2, true>("r128", p, out, n, first)) return 1;
    if (run<2, 1, false>("r64x2", p, out, n, first)) return 1;
    if (run<4, 1, false>("r64x4", p, out, n, first)) return 1;
    if (run<1, 2, false>("r64adj2", p, out, n, first)) return 1;
    if (run<1, 3, false>("r64adj3", p, out, n, first)) return 1;
  }
  std::printf("}\n");
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
