// SPDX-License-Identifier: LGPL-2.1
//
// dmc_sort.h -- hand-written device-wide scans and the radix path's exact
// LSD sort (no library kernels: every launch here is ours, uses no scratch
// memory, and reports nothing a caller could ignore).
//
//   scans     exclusive scans (sum of u32, min of u64) over n items in three
//             launches: per-tile reductions, one block scanning the tile
//             partials, per-tile down-sweeps with the carry-in
//   LSD sort  the radix path's ranking (a round whose rank bins overflowed:
//             massively tied keys): the dense entries' indices sorted by the
//             exact order key (phase, okey, slot, queue position) with stable
//             8-bit digit passes, least significant first -- queue position,
//             slot, the ordered key's eight bytes, phase.  Exact for every
//             key, so no fix-up of equal runs (the 32-bit keys of round 2
//             needed an O(run^2) insertion sort per run of equal keys).
#pragma once

#include "dmc_round.h"

namespace dmc {

constexpr int kScT = 256;                       // threads per scan / sort block
constexpr int kScItems = 8;                     // items per thread
constexpr uint32_t kScTile = kScT * kScItems;  // 2048 items per block

struct SumU32 {
  using T = uint32_t;
  __device__ static T id() { return 0u; }
  __device__ static T op(T a, T b) { return a + b; }
};
struct MinU64 {
  using T = uint64_t;
  __device__ static T id() { return ~0ull; }
  __device__ static T op(T a, T b) { return a < b ? a : b; }
};

template <typename T>
__device__ inline T shfl_up_any(T v, int d) {
  if constexpr (sizeof(T) == 8) {
    const uint64_t u = (uint64_t)v;
    const uint32_t lo = __shfl_up((uint32_t)u, d), hi = __shfl_up((uint32_t)(u >> 32), d);
    return (T)(((uint64_t)hi << 32) | lo);
  } else {
    return (T)__shfl_up((uint32_t)v, d);
  }
}

// Exclusive scan of one value per thread over a block of kScT threads; *tot
// (optional) gets the block total.  wsum: kScT / 64 entries of LDS.
template <typename Op>
__device__ inline typename Op::T block_excl(typename Op::T v, typename Op::T* wsum,
                                            typename Op::T* tot = nullptr) {
  using T = typename Op::T;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  T incl = v;
  for (int d = 1; d < 64; d <<= 1) {
    const T o = shfl_up_any(incl, d);
    if (lane >= d) incl = Op::op(o, incl);
  }
  T ex = shfl_up_any(incl, 1);
  if (lane == 0) ex = Op::id();
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  T pre = Op::id(), all = Op::id();
  for (int i = 0; i < kScT / 64; ++i) {
    if (i < w) pre = Op::op(pre, wsum[i]);
    all = Op::op(all, wsum[i]);
  }
  __syncthreads();  // (wsum is reused by the caller's next scan)
  if (tot) *tot = all;
  return Op::op(pre, ex);
}

// 1. per-tile reductions (tile b: items [b * kScTile, (b + 1) * kScTile))
template <typename Op>
__global__ void __launch_bounds__(kScT)
k_scan_reduce(const typename Op::T* in, uint32_t n, typename Op::T* parts) {
  using T = typename Op::T;
  __shared__ T wsum[kScT / 64];
  const uint32_t base = blockIdx.x * kScTile;
  T a = Op::id();
#pragma unroll
  for (int j = 0; j < kScItems; ++j) {
    const uint32_t i = base + j * kScT + threadIdx.x;
    if (i < n) a = Op::op(a, in[i]);
  }
  T tot;
  (void)block_excl<Op>(a, wsum, &tot);
  if (threadIdx.x == 0) parts[blockIdx.x] = tot;
}

// 2. one block: the tile partials, scanned exclusively in place
template <typename Op>
__global__ void __launch_bounds__(kScT) k_scan_top(typename Op::T* parts, uint32_t np) {
  using T = typename Op::T;
  __shared__ T wsum[kScT / 64];
  T carry = Op::id();
  for (uint32_t c0 = 0; c0 < np; c0 += kScT) {
    const uint32_t i = c0 + threadIdx.x;
    const T v = i < np ? parts[i] : Op::id();
    T tot;
    const T ex = block_excl<Op>(v, wsum, &tot);
    if (i < np) parts[i] = Op::op(carry, ex);
    carry = Op::op(carry, tot);
  }
}

// 3. per tile: the exclusive scan of its items with the tile's carry-in
// (coalesced loads into LDS, each thread scans kScItems consecutive items;
// in == out is allowed)
template <typename Op>
__global__ void __launch_bounds__(kScT)
k_scan_down(const typename Op::T* in, typename Op::T* out, uint32_t n,
            const typename Op::T* parts) {
  using T = typename Op::T;
  __shared__ T tile[kScTile];
  __shared__ T wsum[kScT / 64];
  const uint32_t base = blockIdx.x * kScTile;
#pragma unroll
  for (int j = 0; j < kScItems; ++j) {
    const uint32_t i = base + j * kScT + threadIdx.x;
    tile[j * kScT + threadIdx.x] = i < n ? in[i] : Op::id();
  }
  __syncthreads();
  T v[kScItems];
  T a = Op::id();
#pragma unroll
  for (int j = 0; j < kScItems; ++j) {
    v[j] = a;
    a = Op::op(a, tile[threadIdx.x * kScItems + j]);
  }
  const T ex = Op::op(parts[blockIdx.x], block_excl<Op>(a, wsum));
#pragma unroll
  for (int j = 0; j < kScItems; ++j) tile[threadIdx.x * kScItems + j] = Op::op(ex, v[j]);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kScItems; ++j) {
    const uint32_t i = base + j * kScT + threadIdx.x;
    if (i < n) out[i] = tile[j * kScT + threadIdx.x];
  }
}

inline uint32_t scan_tiles(uint32_t n) { return (n + kScTile - 1) / kScTile; }

// Exclusive scan of n items (host side: three launches on `st`); parts needs
// scan_tiles(n) entries.
template <typename Op>
void scan_excl(const typename Op::T* in, typename Op::T* out, uint32_t n,
               typename Op::T* parts, hipStream_t st) {
  if (!n) return;
  const uint32_t nb = scan_tiles(n);
  hipLaunchKernelGGL(k_scan_reduce<Op>, dim3(nb), dim3(kScT), 0, st, in, n, parts);
  hipLaunchKernelGGL(k_scan_top<Op>, dim3(1), dim3(kScT), 0, st, parts, nb);
  hipLaunchKernelGGL(k_scan_down<Op>, dim3(nb), dim3(kScT), 0, st, in, out, n,
                     (const typename Op::T*)parts);
}

// ------------------------------------------------------------ radix path sort
// The dense entries a radix round emitted (k_remit, rd->dense_n of them, at
// most dcap): an overflowing round (dense_n > dcap) is flagged for the host's
// retry with a larger buffer and every later kernel of the round sees n = 0.
__global__ void k_dcheck(Round* rd, uint32_t dcap) {
  if (threadIdx.x == 0 && rd->dense_n > dcap && !rd->overflow) rd->overflow = 1;
}

__device__ inline uint32_t dense_valid(const Round* rd, uint32_t dcap) {
  return (!rd->overflow && rd->dense_n <= dcap) ? rd->dense_n : 0u;
}

// One digit pass of the order key (phase, okey, slot, queue position):
// field 0 queue position, 1 slot, 2 ordered key, 3 phase; `shift` the digit's
// bit offset inside the field.
enum : uint32_t { kDigPos = 0, kDigSlot = 1, kDigKey = 2, kDigPhase = 3 };
__device__ inline uint32_t dent_digit(const DEnt& e, uint32_t field, uint32_t shift) {
  switch (field) {
    case kDigPos: return (e.seq & 0x7fffffffu) >> shift & 0xffu;
    case kDigSlot: return e.slot >> shift & 0xffu;
    case kDigKey: return (uint32_t)(e.okey >> shift) & 0xffu;
    default: return e.seq >> 31;
  }
}

// Pass step 1: per tile, the count of each digit (digit-major: cnt[d * nblk + b],
// so that one exclusive scan gives every (digit, tile) its output offset).
// src: the previous pass's order (null: identity).
__global__ void __launch_bounds__(kScT)
k_lsd_count(const Round* rd, uint32_t dcap, const DEnt* dense, const uint32_t* src,
            uint32_t nblk, uint32_t field, uint32_t shift, uint32_t* cnt) {
  __shared__ uint32_t h[256];
  const uint32_t n = dense_valid(rd, dcap);
  h[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * kScTile;
#pragma unroll
  for (int j = 0; j < kScItems; ++j) {
    const uint32_t i = base + j * kScT + threadIdx.x;
    if (i < n) atomicAdd(&h[dent_digit(dense[src ? src[i] : i], field, shift)], 1u);
  }
  __syncthreads();
  cnt[threadIdx.x * nblk + blockIdx.x] = h[threadIdx.x];
}

// Pass step 3 (after the scan of cnt into off): stable scatter.  The tile is
// taken in kScItems rounds of kScT consecutive items; within a wave the
// items sharing a digit are found by eight ballots, ranked by lane, counted
// per (round, wave, digit) and those counts scanned in item order.
__global__ void __launch_bounds__(kScT)
k_lsd_scatter(const Round* rd, uint32_t dcap, const DEnt* dense, const uint32_t* src,
              uint32_t* dst, uint32_t nblk, uint32_t field, uint32_t shift,
              const uint32_t* off) {
  constexpr int NW = kScT / 64;
  __shared__ uint32_t wc[kScItems][NW][256];
  const uint32_t n = dense_valid(rd, dcap);
  const uint32_t base = blockIdx.x * kScTile;
  if (base >= n) return;  // (block-uniform)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < kScItems * NW * 256; i += kScT)
    (&wc[0][0][0])[i] = 0;
  __syncthreads();
  const uint64_t lt = (1ull << lane) - 1ull;
  uint32_t val[kScItems], dig[kScItems], rk[kScItems];
#pragma unroll
  for (int j = 0; j < kScItems; ++j) {
    const uint32_t i = base + j * kScT + threadIdx.x;
    const bool in = i < n;
    val[j] = in ? (src ? src[i] : i) : 0u;
    dig[j] = in ? dent_digit(dense[val[j]], field, shift) : 0u;
    uint64_t m = __ballot(in);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const bool bit = (dig[j] >> b) & 1u;
      const uint64_t bb = __ballot(in && bit);
      m &= bit ? bb : ~bb;
    }
    rk[j] = (uint32_t)__popcll(m & lt);
    if (in && rk[j] == 0) wc[j][w][dig[j]] = (uint32_t)__popcll(m);
  }
  __syncthreads();
  {
    // thread d: the digit's exclusive prefix over (round, wave), item order
    const uint32_t d = threadIdx.x;
    uint32_t run = 0;
    for (int j = 0; j < kScItems; ++j)
      for (int v = 0; v < NW; ++v) {
        const uint32_t c = wc[j][v][d];
        wc[j][v][d] = run;
        run += c;
      }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kScItems; ++j) {
    const uint32_t i = base + j * kScT + threadIdx.x;
    if (i < n) dst[off[dig[j] * nblk + blockIdx.x] + wc[j][w][dig[j]] + rk[j]] = val[j];
  }
}

// The digit passes of a table of 2^slot_bits slots: queue position (6 bits),
// the slot's bytes, the ordered key's 8 bytes, phase.
struct LsdPass {
  uint32_t field, shift;
};
inline int lsd_passes(int slot_bits, LsdPass* out) {
  int np = 0;
  out[np++] = LsdPass{kDigPos, 0};
  for (int s = 0; s < slot_bits; s += 8) out[np++] = LsdPass{kDigSlot, (uint32_t)s};
  for (int s = 0; s < 64; s += 8) out[np++] = LsdPass{kDigKey, (uint32_t)s};
  out[np++] = LsdPass{kDigPhase, 0};
  return np;
}

}  // namespace dmc
