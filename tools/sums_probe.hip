// Tracker-sum scatter rates (config 5's epoch delivery, k_track_sums): 8
// servers x 2M slots, 40 % of slots with a response count, each slot's
// client a random one of 4M global clients (unique within a server).
// Variants: one launch per server with device atomics (the engine's form),
// one launch over all servers, and per-server launches with plain
// read-modify-write (safe there: a server's slots map to distinct clients).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("hip %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void sums_atomic(uint32_t n, const uint32_t* cmap, const uint32_t* cd, const uint32_t* cr,
                            uint32_t* sd, uint32_t* sr) {
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < n; s += gridDim.x * blockDim.x) {
    const uint32_t d = cd[s];
    if (!d) continue;
    const uint32_t r = cr[s], c = cmap[s];
    atomicAdd(&sd[c], d);
    if (r) atomicAdd(&sr[c], r);
  }
}
__global__ void sums_atomic_m(uint32_t n, const uint32_t* cmap, const uint32_t* cd, const uint32_t* cr,
                              uint32_t* sd, uint32_t* sr) {
  const size_t o = (size_t)blockIdx.y * n;
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < n; s += gridDim.x * blockDim.x) {
    const uint32_t d = cd[o + s];
    if (!d) continue;
    const uint32_t r = cr[o + s], c = cmap[o + s];
    atomicAdd(&sd[c], d);
    if (r) atomicAdd(&sr[c], r);
  }
}
__global__ void sums_rmw(uint32_t n, const uint32_t* cmap, const uint32_t* cd, const uint32_t* cr,
                         uint32_t* sd, uint32_t* sr) {
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < n; s += gridDim.x * blockDim.x) {
    const uint32_t d = cd[s];
    if (!d) continue;
    const uint32_t r = cr[s], c = cmap[s];
    sd[c] += d;
    if (r) sr[c] += r;
  }
}

int main() {
  const uint32_t S = 8, N = 1u << 21, G = 1u << 22;
  std::mt19937 rng(7);
  std::vector<uint32_t> perm(G), cmap((size_t)S * N), cd((size_t)S * N), cr((size_t)S * N);
  for (uint32_t i = 0; i < G; ++i) perm[i] = i;
  for (uint32_t s = 0; s < S; ++s) {
    std::shuffle(perm.begin(), perm.end(), rng);
    for (uint32_t i = 0; i < N; ++i) {
      cmap[(size_t)s * N + i] = perm[i];
      const bool on = (rng() % 10) < 4;
      cd[(size_t)s * N + i] = on ? 1 + rng() % 3 : 0;
      cr[(size_t)s * N + i] = on ? rng() % 2 : 0;
    }
  }
  uint32_t *dm, *dd, *dr, *sd, *sr;
  CK(hipMalloc(&dm, 4ull * S * N)); CK(hipMalloc(&dd, 4ull * S * N)); CK(hipMalloc(&dr, 4ull * S * N));
  CK(hipMalloc(&sd, 4ull * G)); CK(hipMalloc(&sr, 4ull * G));
  CK(hipMemcpy(dm, cmap.data(), 4ull * S * N, hipMemcpyHostToDevice));
  CK(hipMemcpy(dd, cd.data(), 4ull * S * N, hipMemcpyHostToDevice));
  CK(hipMemcpy(dr, cr.data(), 4ull * S * N, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  std::vector<uint32_t> ref, got(G);
  for (int v = 0; v < 3; ++v) {
    for (int rep = 0; rep < 4; ++rep) {
      CK(hipMemset(sd, 0, 4ull * G)); CK(hipMemset(sr, 0, 4ull * G));
      CK(hipEventRecord(a));
      if (v == 0) {
        for (uint32_t s = 0; s < S; ++s)
          hipLaunchKernelGGL(sums_atomic, dim3(2048), dim3(256), 0, 0, N, dm + (size_t)s * N, dd + (size_t)s * N, dr + (size_t)s * N, sd, sr);
      } else if (v == 1) {
        hipLaunchKernelGGL(sums_atomic_m, dim3(2048, S), dim3(256), 0, 0, N, dm, dd, dr, sd, sr);
      } else {
        for (uint32_t s = 0; s < S; ++s)
          hipLaunchKernelGGL(sums_rmw, dim3(2048), dim3(256), 0, 0, N, dm + (size_t)s * N, dd + (size_t)s * N, dr + (size_t)s * N, sd, sr);
      }
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      CK(hipMemcpy(got.data(), sd, 4ull * G, hipMemcpyDeviceToHost));
      if (v == 0 && rep == 0) ref = got;
      const bool same = got == ref;
      if (rep == 3) printf("variant %d (%s): %.1f us for %u servers, sums %s\n", v,
                           v == 0 ? "atomics, launch per server" : v == 1 ? "atomics, one launch" : "plain RMW, launch per server",
                           ms * 1000.0f, S, same ? "equal" : "DIFFER");
    }
  }
  return 0;
}
