// SPDX-License-Identifier: LGPL-2.1
//
// FETCH_SIZE calibration on known byte counts, per access pattern
// (MI355X_MICROARCH.md, HBM: "other access widths are uncalibrated:
// calibrate on a known byte count in your own access pattern").  Each kernel
// reads a known set of distinct bytes of a 2 GiB buffer (far past the 256 MiB
// Infinity Cache, each line touched once) with one of the engine's access
// shapes:
//   stream16  16 B per lane, coalesced (the guide's calibrated case)
//   rand64    one 64-byte record per lane at a pseudo-random distinct slot
//             (4 x 16 B loads; the ring entries / ClientRec of the walkers)
//   rand32    one 32-byte record per lane (ScanRec)
//   rand16    one 16-byte load per lane, one per distinct 64-byte record
//   rand8     one 8-byte load per lane, one per distinct 128-byte line
// Run under `rocprofv3 --pmc FETCH_SIZE` (and a separate --kernel-trace
// pass); tools/pmc_traffic.py --calib turns the counter into bytes-per-count
// factors.  Prints the known bytes of each kernel as JSON.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

constexpr uint64_t kBuf = 2ull << 30;  // 2 GiB
constexpr uint32_t kThreads = 256;

// i -> a distinct pseudo-random index in [0, 2^bits): an odd multiplier is a
// bijection modulo a power of two
__device__ inline uint64_t perm(uint64_t i, int bits) {
  return (i * 0x9E3779B97F4A7C15ull) & ((1ull << bits) - 1);
}

__global__ void stream16(const uint4* __restrict__ p, uint64_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

template <int WORDS16>
__global__ void rand_rec(const uint4* __restrict__ p, uint64_t n, int bits, uint32_t* out) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t r = perm(i, bits);
  const uint4* q = p + r * WORDS16;
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < WORDS16; ++k) {
    uint4 v = q[k];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

// one 16-byte load from each of n distinct 64-byte records
__global__ void rand16(const uint4* __restrict__ p, uint64_t n, int bits, uint32_t* out) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint4 v = p[perm(i, bits) * 4];
  if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9e3779b9u) out[0] = v.x;
}

// one 8-byte load from each of n distinct 128-byte lines
__global__ void rand8(const uint64_t* __restrict__ p, uint64_t n, int bits, uint32_t* out) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t v = p[perm(i, bits) * 16];
  if ((uint32_t)v == 0x9e3779b9u) out[0] = (uint32_t)v;
}

int main() {
  void* buf = nullptr;
  uint32_t* out = nullptr;
  CK(hipMalloc(&buf, kBuf));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(buf, 1, kBuf));
  CK(hipDeviceSynchronize());
  const uint4* p = static_cast<const uint4*>(buf);
  // 512 MiB of each pattern's useful bytes (rand8 / rand16: 2^22 lanes)
  const uint64_t n_stream = (512ull << 20) / 16;
  const uint64_t n64 = (512ull << 20) / 64;   // 2^23 records of 2^25 in 2 GiB
  const uint64_t n32 = (512ull << 20) / 32;   // 2^24 of 2^26
  const uint64_t n16 = 1ull << 22;            // of 2^25 records
  const uint64_t n8 = 1ull << 22;             // of 2^24 lines
  auto g = [](uint64_t n) { return dim3((unsigned)((n + kThreads - 1) / kThreads)); };
  for (int rep = 0; rep < 3; ++rep) {
    // a 2 GiB streaming pass between kernels evicts the Infinity Cache
    hipLaunchKernelGGL(stream16, dim3(8192), dim3(kThreads), 0, 0, p, kBuf / 16, out);
    hipLaunchKernelGGL(stream16, dim3(8192), dim3(kThreads), 0, 0, p, n_stream, out);
    hipLaunchKernelGGL(stream16, dim3(8192), dim3(kThreads), 0, 0, p, kBuf / 16, out);
    hipLaunchKernelGGL(rand_rec<4>, g(n64), dim3(kThreads), 0, 0, p, n64, 25, out);
    hipLaunchKernelGGL(stream16, dim3(8192), dim3(kThreads), 0, 0, p, kBuf / 16, out);
    hipLaunchKernelGGL(rand_rec<2>, g(n32), dim3(kThreads), 0, 0, p, n32, 26, out);
    hipLaunchKernelGGL(stream16, dim3(8192), dim3(kThreads), 0, 0, p, kBuf / 16, out);
    hipLaunchKernelGGL(rand16, g(n16), dim3(kThreads), 0, 0, p, n16, 25, out);
    hipLaunchKernelGGL(stream16, dim3(8192), dim3(kThreads), 0, 0, p, kBuf / 16, out);
    hipLaunchKernelGGL(rand8, g(n8), dim3(kThreads), 0, 0,
                       static_cast<const uint64_t*>(buf), n8, 24, out);
  }
  CK(hipDeviceSynchronize());
  std::printf("{\"evict_pass_bytes\": %llu, \"stream16\": %llu, \"rand64\": %llu, "
              "\"rand32\": %llu, \"rand16\": %llu, \"rand8\": %llu, \"repeats\": 3, "
              "\"dispatch_order\": [\"evict\", \"stream16\", \"evict\", \"rand64\", "
              "\"evict\", \"rand32\", \"evict\", \"rand16\", \"evict\", \"rand8\"]}\n",
              (unsigned long long)kBuf, (unsigned long long)(n_stream * 16),
              (unsigned long long)(n64 * 64), (unsigned long long)(n32 * 32),
              (unsigned long long)(n16 * 16), (unsigned long long)(n8 * 8));
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
