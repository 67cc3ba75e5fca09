// SPDX-License-Identifier: LGPL-2.1
//
// dmc_engine.hip -- MI355X (gfx950) dmClock server-queue engine behind the
// C-ABI of include/dmclock_gpu.h.
//
// Reference path replaced: crimson::dmclock::PriorityQueueBase /
// PullPriorityQueue (/root/reference/src/dmclock_server.h:283-1501):
//   add path     do_add_request          :913-1018   -> add pipeline below
//   select path  do_next_request         :1115-1186  -> pull pipeline below
//   pop/reduce   pop_process_request     :1046-1073,
//                reduce_reservation_tags :1077-1111  -> apply kernels
// The three IndIntruHeaps are replaced by data-parallel scans over a
// struct-of-arrays client table plus a per-batch radix sort of the candidate
// pops; see DESIGN.md for why the result is the reference's dispatch order.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <mutex>
#include <vector>

#include "../../include/dmclock_gpu.h"
#include "dmc_device.h"
#include "dmc_add.h"
#include "dmc_round.h"
#include "dmc_sort.h"
#include "dmc_tracker.h"

using namespace dmc;

namespace {

constexpr int kBlock = 256;
constexpr uint32_t kNone = 0xffffffffu;

#define HIP_OK(expr)                                              \
  do {                                                            \
    hipError_t e_ = (expr);                                       \
    if (e_ != hipSuccess) {                                       \
      std::fprintf(stderr, "dmclock_gpu: %s failed: %s (%s:%d)\n", \
                   #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
      return DMC_EDEVICE;                                         \
    }                                                             \
  } while (0)

// Single-step (one do_next_request) reduction record.
struct ArgMin {
  uint64_t key;
  uint32_t slot;
  uint32_t cnt;  // how many slots share the minimum key
};

struct StepRed {
  ArgMin r;       // min front reservation over clients with requests
  ArgMin p;       // min p+pd over ready (after marking) fronts with p < inf
  ArgMin pnr;     // min p+pd over not-ready fronts (Allow: ready-heap top)
  uint64_t lmin_nr, lmin_rd;  // min limit (ordered) over not-ready / ready
  uint32_t n_any, n_ready, n_notready, pad;
};

struct StepCtl {
  int32_t type;    // DMC_NEXT_*
  int32_t prio;    // 1: ready-heap pop (reduce), 0: reservation-heap pop
  uint32_t slot;
  uint32_t mark;   // the limit scan ran: commit ready marks
  uint32_t tie;
  uint32_t pad;
  double when;
};

__device__ inline ArgMin argmin_combine(ArgMin a, ArgMin b) {
  if (a.key < b.key) return a;
  if (b.key < a.key) return b;
  ArgMin o;
  o.key = a.key;
  o.slot = a.slot < b.slot ? a.slot : b.slot;
  o.cnt = a.cnt + b.cnt;
  return o;
}

__device__ inline uint64_t shfl_u64(uint64_t v, int src) {
  uint32_t lo = __shfl((uint32_t)v, src), hi = __shfl((uint32_t)(v >> 32), src);
  return ((uint64_t)hi << 32) | lo;
}
__device__ inline uint64_t shfl_up_u64(uint64_t v, int d) {
  uint32_t lo = __shfl_up((uint32_t)v, d), hi = __shfl_up((uint32_t)(v >> 32), d);
  return ((uint64_t)hi << 32) | lo;
}
__device__ inline uint64_t shfl_down_u64(uint64_t v, int d) {
  uint32_t lo = __shfl_down((uint32_t)v, d), hi = __shfl_down((uint32_t)(v >> 32), d);
  return ((uint64_t)hi << 32) | lo;
}

__device__ inline ArgMin wave_argmin(ArgMin a) {
  for (int d = 32; d > 0; d >>= 1) {
    ArgMin b;
    b.key = shfl_down_u64(a.key, d);
    b.slot = __shfl_down(a.slot, d);
    b.cnt = __shfl_down(a.cnt, d);
    a = argmin_combine(a, b);
  }
  return a;
}
__device__ inline uint64_t wave_min_u64(uint64_t v) {
  for (int d = 32; d > 0; d >>= 1) {
    uint64_t o = shfl_down_u64(v, d);
    v = o < v ? o : v;
  }
  return v;
}
__device__ inline uint64_t wave_max_u64(uint64_t v) {
  for (int d = 32; d > 0; d >>= 1) {
    uint64_t o = shfl_down_u64(v, d);
    v = o > v ? o : v;
  }
  return v;
}
__device__ inline uint32_t wave_sum_u32(uint32_t v) {
  for (int d = 32; d > 0; d >>= 1) v += __shfl_down(v, d);
  return v;
}

// ------------------------------------------------------------------ register
__global__ void k_register(Table tb, BoundInfo* binfo, uint32_t n, const uint32_t* slots,
                           const double* rinv, const double* winv,
                           const double* linv, int active, uint64_t tick) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t s = slots[i];
  if (s >= tb.n) return;
  // ClientRec(client, info, tick), dmclock_server.h:381-393
  tb.rec[s] = ClientRec{0.0, 0.0, 0.0, 0.0, rinv[i], winv[i], linv[i], 0.0};
  binfo[s] = BoundInfo{rinv[i], winv[i], linv[i], 0.0};
  tb.sc[s] = ScanRec{0.0, 0.0, 0.0, 0, 0, (uint8_t)(F_REG | (active ? 0 : F_IDLE)), 0, 0};
  tb.aux[s] = ClientAux{1, 1, tick};
}

// ------------------------------------------------------------------ add path
// (per-client replay: dmc_add.h)
// The first node of an add segment: its arguments are the segment's per-call
// parameters (updated in place on graph replays); block 0 publishes them for
// k_add_chain.
// (bid: the block's index among the filing blocks; prev: k_apply_link, where
// the previous call's round is applied beside this filing -- its gate is
// being written by that launch, so the round's outcome is read instead:
// the gate shut before it (the round skipped), or the round failing or
// needing the host, shuts this call too, exactly as the gate would)
__device__ __attribute__((always_inline)) inline void add_link_body(AddParams p, Table tb, uint32_t* abuf, uint32_t* apos, uint32_t* aslot, AddParams* pblk, ActBuf act, uint32_t bid = 0xffffffffu, const Round* prev = nullptr) {
  uint32_t i = (bid == 0xffffffffu ? blockIdx.x : bid) * blockDim.x + threadIdx.x;
  // (the request's slot requested with the gate word: one level of loads)
  uint32_t s = 0;
  if (DMC_EARLY_LOADS && i < p.n) s = p.reqs[i].slot;
  if (prev) {
    if (!round_ends_call(*prev)) return;
  } else if (tb.gate && *tb.gate) {
    return;  // (DMC_OPT_PIPELINE: a shut gate, see Table::gate)
  }
  if (i == 0) *pblk = p;
  if (i >= p.n) return;
  if (act.cold) {
    act.cold[i] = kMaxKey;
    act.cnew[i] = kMaxKey;
    if (act.flag) act.flag[i] = 0;
    act.hev_q[i] = kNone;
    act.hard[i] = 0u;
    if (i == 0) *act.anyhard = 0u;
  }
  if (tb.hev) tb.hev[i] = 0;  // (positions the chain never visits: no heap call)
  if (!DMC_EARLY_LOADS) s = p.reqs[i].slot;
  aslot[i] = s;
  if (s >= tb.n) {
    apos[i] = kNone;
    p.rc[i] = DMC_ENOTREG;  // (no replay will see this request)
    return;
  }
  uint32_t pos = atomicAdd(&tb.sc[s].nadd, 1u);
  apos[i] = pos;
  // (k_chain_scan's scan leaves the slot: the stamp on the line the atomic
  // just took, or the separate touch array)
  if (p.epoch) {
    if (DMC_STAMP_SC) tb.sc[s].stamp = (uint8_t)p.epoch;
    else tb.touch[s] = p.epoch;
  }
  // (filing order 0 replays the client's requests and knows its own position)
  if (pos - 1u < kAddSlots - 1u) abuf[(size_t)s * kAddSlots + pos] = i;
}
// A pipelined call's filing beside the previous call's apply, one launch
// (DMC_DEFER_APPLY): blocks [0, napply) apply the previous round (its
// k_rapply, deferred to this launch), the rest file this call's requests
// (its k_add_link).  The two touch disjoint state: the apply writes a slot's
// front keys and cursor bytes (sc_store_front), the filing its batch count
// and stamp (bytes 27-31 of the same ScanRec) and the batch buffers.
__global__ void __launch_bounds__(kBlockR, DMC_APPLY_MINB)
k_apply_link(Table tb, Round* rd, const CandRec* cand, const uint32_t* bcand,
             const uint32_t* decof, const PostRec* post, unsigned long long* sched,
             HostRound* h, uint32_t napply, AddParams ap, uint32_t* abuf, uint32_t* apos,
             uint32_t* aslot, AddParams* pblk) {
  if (blockIdx.x < napply) {
    rapply_body(tb, rd, cand, bcand, decof, post, sched, h, nullptr, blockIdx.x, napply);
    return;
  }
  add_link_body(ap, tb, abuf, apos, aslot, pblk, ActBuf{}, blockIdx.x - napply, rd);
}
// the epoch wrapped: no slot may keep a stamp equal to a later batch's
__global__ void k_clear_stamps(Table tb) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < tb.n) tb.sc[s].stamp = 0;
}
__global__ void 
k_add_link(AddParams p, Table tb,
                           uint32_t* abuf, uint32_t* apos, uint32_t* aslot,
                           AddParams* pblk, ActBuf act = ActBuf{}) {
  add_link_body(p, tb, abuf, apos, aslot, pblk, act);
}

__device__ __attribute__((always_inline)) inline void add_chain_body(Table tb, const AddParams* pblk, const uint32_t* abuf, const uint32_t* apos, const uint32_t* aslot, ActBuf act, const TrackFill* tf = nullptr, int bid = -1) {
  if (tb.gate && *tb.gate) return;
  uint32_t i = (bid < 0 ? blockIdx.x : (uint32_t)bid) * blockDim.x + threadIdx.x;
  // one level of loads: the call's parameters and this position's filing
  // (apos / aslot are padded to whole blocks: in bounds for the grid)
  const AddParams p = *pblk;
  const uint32_t pos0 = apos[i];
  const uint32_t s = aslot[i];
  if (i >= p.n) return;
  if (pos0 == kNone) {
    p.rc[i] = DMC_ENOTREG;
    return;
  }
  if (pos0 != 0) return;  // the client's first filer replays its requests
  // the next: the client's batch count with its state
  AddState st;
  add_chain_slot(tb, p, s, 0, i, abuf, aslot, act, &st, true, tf);
}
__global__ void 
k_add_chain(Table tb, const AddParams* pblk,
                            const uint32_t* abuf, const uint32_t* apos,
                            const uint32_t* aslot, ActBuf act = ActBuf{}) {
  add_chain_body(tb, pblk, abuf, apos, aslot, act);
}

// A fused call's add chain and its round's scan in one launch, side by side
// (blocks [0, nchain): the chain; the rest: the scan, kScanChainSlots slots
// per thread, which leaves the batch's slots to the chain -- each client's
// first filer scans its slot once its adds are in): the chain's random
// client accesses and the scan's stream overlap instead of running one
// after the other.  Partials: the scan's nscan blocks', then the chain's.
#ifndef DMC_CHAIN_SCAN_SLOTS
#define DMC_CHAIN_SCAN_SLOTS 3
#endif
constexpr int kScanChainSlots = DMC_CHAIN_SCAN_SLOTS;

// the chain side: block bid of the batch (tf: a queue group's trackers)
__device__ __attribute__((always_inline)) inline void chain_scan_chain(
    const Table& tb, const AddParams& p, const uint32_t* abuf, const uint32_t* apos,
    const uint32_t* aslot, const TrackFill* tf, double now, uint64_t* keyr, uint64_t* keyp,
    uint32_t* meta, uint64_t* skr, uint64_t* skp, uint2* k32, RoundPart* part, uint32_t bid) {
  if (!DMC_EARLY_LOADS && tb.gate && *tb.gate) return;
  const uint32_t i = bid * kBlock + threadIdx.x;
  // (one level of loads: this position's filing, with the request itself --
  // the call's parameters are kernel arguments; apos / aslot are padded to
  // whole blocks)
  const uint32_t pos0 = apos[i];
  const uint32_t s = aslot[i];
  // (this position's request with them: add_chain_slot's first load of it
  // is then no level of its own)
  dmc_request rq0{};
  if (i < p.n) rq0 = p.reqs[i];
  // (DMC_OPT_PIPELINE: a shut gate, see Table::gate; its word requested with
  // the loads above)
  if (DMC_EARLY_LOADS && tb.gate && *tb.gate) return;
  keep((double)rq0.time);
  RoundPart acc = rpart_ident();
  if (i < p.n) {
    if (pos0 == kNone) {
      p.rc[i] = DMC_ENOTREG;  // (as k_add_chain: no replay sees this request)
    } else if (pos0 == 0) {
      // the slot's heap keys before the adds (the cursor's line: no extra
      // request) and its prop_delta, with the chain's own loads
      const ScanRec r0 = tb.sc[s];
      const double pd = tb.rec[s].pd;
      AddState st;
      add_chain_slot(tb, p, s, 0, i, abuf, aslot, ActBuf{}, &st, true, tf);
      // the scan of the slot after its adds, from the chain's registers (what
      // k_rscan would load): the front is the batch's first request if the
      // queue was empty, else unchanged; queue position 1 is a request of
      // the batch unless two were queued before
      ScanCols x;
      x.c = st.count;
      x.h = st.head;
      x.f = st.flags;
      if (st.front_set) {
        x.fr = st.front.r;
        x.pk = __dadd_rn(st.front.p, pd);
        x.fl = st.front.l;
      } else {
        x.fr = r0.r;
        x.pk = r0.pk;
        x.fl = r0.l;
      }
      ScanPre pre{0.0, 0.0, 0.0, 0.0};
      if (x.c > 1 && x.fr <= now && !tb.delayed) {
        pre.pd = pd;
        const uint32_t c0 = r0.count;
        if (c0 >= 2) {
          const ReqEntry& e = tb.ring[(size_t)s * tb.q + ((x.h + 1) & tb.qmask)];
          pre.r1 = e.r;
          pre.p1 = e.p;
          pre.l1 = e.l;
        } else if (c0 == 1) {  // position 1: the batch's first request
          pre.r1 = st.n0r;
          pre.p1 = st.n0p;
          pre.l1 = st.n0l;
        } else {  // the batch's second
          pre.r1 = st.n1r;
          pre.p1 = st.n1p;
          pre.l1 = st.n1l;
        }
      }
      const ScanOut o = scan_compute(tb, s, x, pre, now);
      scan_store(tb, s, x, o, keyr, keyp, meta, skr, skp, k32, acc);
    }
  }
  block_rpart_store<kBlock>(acc, part);
}

// (DMC_CHAIN_SCAN_MINW waves per SIMD: its register bound; at 117 VGPRs,
// 4 waves, the scan's 1,024 blocks and the chain's 256 did not fit at once)
#ifndef DMC_CHAIN_SCAN_MINW
#define DMC_CHAIN_SCAN_MINW 4
#endif
__global__ void __launch_bounds__(kBlock, DMC_CHAIN_SCAN_MINW)
k_chain_scan(Table tb, AddParams ap, const uint32_t* abuf, const uint32_t* apos,
             const uint32_t* aslot, uint32_t nchain, uint32_t nscan, uint64_t* keyr,
             uint64_t* keyp, uint32_t* meta, RoundPart* parts, Round* rd, CallParams cp,
             uint64_t* skr, uint64_t* skp, uint2* k32, uint32_t* hist) {
#ifdef DMC_DBG_CS_SIDE  // (timing probe, wrong results: 1 = scan side only, 2 = chain side only)
  if ((DMC_DBG_CS_SIDE == 1) == (blockIdx.x < nchain)) return;
#endif
  if (blockIdx.x >= nchain) {
    rscan_body_g<false, kBlock, true, kScanChainSlots>(tb, keyr, keyp, meta, parts, rd, cp, skr,
                                                       skp, k32, hist, blockIdx.x - nchain,
                                                       nscan);
    return;
  }
  chain_scan_chain(tb, ap, abuf, apos, aslot, nullptr, cp.now, keyr, keyp, meta, skr, skp,
                   k32, parts + nscan + blockIdx.x, blockIdx.x);
}

// (multi-table: per-table arguments of a queue group's add kernels, indexed
// by blockIdx.y; dmc_round.h's multi-table rounds)
struct AddArgs {
  AddParams p;
  Table tb;
  uint32_t *abuf, *apos, *aslot;
  AddParams* pblk;
  TrackFill tf;  // the server's trackers, fused into the add (tf.reqs null: none)
};
__global__ void __launch_bounds__(kBlock) k_add_link_m(const AddArgs* a) {
  const AddArgs& x = a[blockIdx.y];
  add_link_body(x.p, x.tb, x.abuf, x.apos, x.aslot, x.pblk, ActBuf{});
}
__global__ void __launch_bounds__(kBlock) k_add_chain_m(const AddArgs* a) {
  const AddArgs& x = a[blockIdx.y];
  add_chain_body(x.tb, x.pblk, x.abuf, x.apos, x.aslot, ActBuf{}, x.tf.reqs ? &x.tf : nullptr);
}

// Queue groups, DMC_GROUP_OVERLAP: the add chain and the round's scan as
// two launches that run at the same time (the two branches of the step's
// graph: one kernel each, so that each keeps its own occupancy -- one
// merged launch held the scan side to the chain's 162 VGPRs, r05).  As in
// k_chain_scan, the filing stamps the batch's slots with the call's epoch,
// the scan (k_rscan_mt) leaves them, and each client's first filer scans
// its slot once its adds are in (k_chain_scan_m); partials: the scan's
// nscan blocks', then the chain's.
__global__ void __launch_bounds__(kBlock) k_chain_scan_m(const AddArgs* a, const RScanArgs* sa,
                                                         uint32_t nscan) {
  const AddArgs& x = a[blockIdx.y];
  const RScanArgs& r = sa[blockIdx.y];
  chain_scan_chain(x.tb, x.p, x.abuf, x.apos, x.aslot, x.tf.reqs ? &x.tf : nullptr, r.cp.now,
                   r.keyr, r.keyp, r.meta, r.skr, r.skp, r.k32, r.parts + nscan + blockIdx.x,
                   blockIdx.x);
}
// (nblk: the scan's blocks of slots; a grid of fewer blocks strides over
// them, leaving CUs to the chain launched beside it, DMC_GROUP_SCAN_BLOCKS)
__global__ void __launch_bounds__(kScanBlock) k_rscan_mt(const RScanArgs* a,
                                                                        uint32_t nblk) {
  const RScanArgs& x = a[blockIdx.y];
  for (uint32_t b = blockIdx.x; b < nblk; b += gridDim.x) {
    rscan_body_g<false, kScanBlock, true, kScanSlots>(x.tb, x.keyr, x.keyp, x.meta, x.parts,
                                                      x.rd, x.cp, x.skr, x.skp, x.k32, x.hist,
                                                      b, nblk);
    __syncthreads();  // (the body's LDS partials, reused by the next block)
  }
}

// The end of an idle reset (:981-984): the client's new prop_delta, its
// front's cached proportion key recomputed with it, idle cleared.
__device__ inline void activate_slot(const Table& tb, uint32_t s, double pd) {
  tb.rec[s].pd = pd;
  const ScanRec r = tb.sc[s];
  if (r.count)
    tb.sc[s].pk = __dadd_rn(tb.ring[(size_t)s * tb.q + (r.head & tb.qmask)].p, pd);
  tb.sc[s].flags = (uint8_t)(r.flags & ~F_IDLE);
}

// idle reset, :937-985: L = min over non-idle clients of
// (has_request ? front.p : prev.p) + prop_delta
__global__ void k_contrib_min(Table tb, uint64_t* parts) {
  uint64_t m = kMaxKey;
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < tb.n;
       s += gridDim.x * blockDim.x) {
    const ScanRec r = tb.sc[s];
    if ((r.flags & F_REG) && !(r.flags & F_IDLE)) {
      // (has_request ? front.p : prev.p) + prop_delta; pk is the former
      uint64_t k = okey(r.count ? r.pk : __dadd_rn(tb.rec[s].prev_p, tb.rec[s].pd));
      m = k < m ? k : m;
    }
  }
  m = wave_min_u64(m);
  __shared__ uint64_t sh[kBlock / 64];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < (int)(blockDim.x / 64); ++i) m = sh[i] < m ? sh[i] : m;
    parts[blockIdx.x] = m;
  }
}

__global__ void k_activate(Table tb, uint32_t s, double t, const uint64_t* parts,
                           uint32_t nparts) {
  __shared__ uint64_t sh[kBlock];
  uint64_t m = kMaxKey;
  for (uint32_t i = threadIdx.x; i < nparts; i += blockDim.x)
    m = parts[i] < m ? parts[i] : m;
  sh[threadIdx.x] = m;
  __syncthreads();
  for (int d = blockDim.x / 2; d > 0; d >>= 1) {
    if ((int)threadIdx.x < d && sh[threadIdx.x + d] < sh[threadIdx.x])
      sh[threadIdx.x] = sh[threadIdx.x + d];
    __syncthreads();
  }
  if (threadIdx.x) return;
  const uint64_t* lmin = &sh[0];
  constexpr double trigger = 1.7976931348623157e308 / 3.0;  // DBL_MAX / 3, :957
  double lowest = 1.7976931348623157e308;                    // DBL_MAX, :960
  if (*lmin != kMaxKey) {
    double L = from_okey(*lmin);
    if (L < lowest) lowest = L;
  }
  activate_slot(tb, s, lowest < trigger ? __dsub_rn(lowest, t) : tb.rec[s].pd);
}

// Batched activations, step 1 (after k_add_link, before k_add_chain): the
// idle reset's minimum over the clients whose contribution the batch does
// not change: registered, non-idle, and not (empty and touched by the batch).
__global__ void k_act_base(Table tb, uint64_t* parts) {
  uint64_t m = kMaxKey;
  // kBaseUnroll records per thread in flight before the first is used
  constexpr int kBaseUnroll = 4;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t s0 = blockIdx.x * blockDim.x + threadIdx.x; s0 < tb.n;
       s0 += kBaseUnroll * stride) {
    ScanRec rs[kBaseUnroll];
#pragma unroll
    for (int u = 0; u < kBaseUnroll; ++u) {
      const uint32_t s = s0 + u * stride;
      if (s < tb.n) rs[u] = tb.sc[s];
      else rs[u].flags = 0;
    }
#pragma unroll
    for (int u = 0; u < kBaseUnroll; ++u) {
      const ScanRec& r = rs[u];
      const uint32_t s = s0 + u * stride;
      if ((r.flags & F_REG) && !(r.flags & F_IDLE)) {
        if (r.count == 0 && r.nadd) continue;  // changes inside the batch: positions
        uint64_t k = okey(r.count ? r.pk : __dadd_rn(tb.rec[s].prev_p, tb.rec[s].pd));
        m = k < m ? k : m;
      }
    }
  }
  m = wave_min_u64(m);
  __shared__ uint64_t sh[kBlock / 64];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < (int)(blockDim.x / 64); ++i) m = sh[i] < m ? sh[i] : m;
    parts[blockIdx.x] = m;
  }
}

constexpr int kActThreads = 1024;

// block-wide inclusive min-scan of one value per thread (u64 ordered keys)
__device__ inline uint64_t block_incl_min(uint64_t v, uint64_t* wpart) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int d = 1; d < 64; d <<= 1) {
    uint64_t o = shfl_up_u64(v, d);
    if (lane >= d && o < v) v = o;
  }
  if (lane == 63) wpart[w] = v;
  __syncthreads();
  uint64_t b = kMaxKey;
  for (int i = 0; i < w; ++i) b = wpart[i] < b ? wpart[i] : b;
  __syncthreads();
  return b < v ? b : v;
}

// the idle reset's value for minimum key x (:957-969): lowest_prop_tag starts
// at DBL_MAX and takes x if smaller; prop_delta = lowest - t iff below the
// trigger, else unchanged
__device__ inline double act_pd(uint64_t x, double t, double pd_old) {
  constexpr double trigger = 1.7976931348623157e308 / 3.0;
  double lowest = 1.7976931348623157e308;
  if (x != kMaxKey) {
    double L = from_okey(x);
    if (L < lowest) lowest = L;
  }
  return lowest < trigger ? __dsub_rn(lowest, t) : pd_old;
}

// Batched activations, step 2 (after k_add_chain and two min-scans over the
// batch positions: pre = exclusive prefix minima of cnew, sufr = exclusive
// prefix minima of cold in reversed position order, i.e. suffix minima).
// The idle reset of the k-th activating request (batch position q_k, time
// t_k) is L_k = min over the clients non-idle at that moment of their
// contribution: unchanged clients (k_act_base), touched empty clients before
// their first accepted request (cold at positions > q_k) or after it (cnew
// at positions < q_k), and the clients activated earlier in the batch
// (M_{k-1} = min_{j<k} p_j + pd_j, pd_j = L_j - t_j).  This kernel gathers
// each activation's inputs (one thread per activation).
__global__ void k_act_inputs(const AddParams* pblk, Table tb, ActBuf act,
                             uint64_t* ax, double* ap, double* at, double* apd,
                             uint32_t* aslot) {
  const AddParams p = *pblk;
  const uint32_t m = act.dm ? *act.dm : act.m;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < m;
       k += gridDim.x * blockDim.x) {
    uint32_t q = act.idx[k];
    uint64_t a = act.pre[q], b = act.suf[p.n - 1 - q];
    ax[k] = a < b ? a : b;
    const dmc_request& rq = p.reqs[q];
    ap[k] = act.actp[q];
    at[k] = rq.time;
    aslot[k] = rq.slot;
    apd[k] = tb.rec[rq.slot].pd;
  }
}

// The batch positions' scans of the activation bookkeeping, in two launches
// (tile totals, then each tile's scan with its carry-in from the totals
// before it, fused over the three arrays): pre =
// exclusive prefix minima of cnew, suf = exclusive prefix minima of cold
// (stored in reversed position order: suffix minima), and, for activations
// the device detected (act.flag), the flagged positions compacted into idx,
// ascending, with their count in *dm.
struct ActScanPart {
  uint64_t mn, mo;
  uint32_t c, pad;
};

__global__ void __launch_bounds__(kScT)
k_act_scan_reduce(ActBuf act, uint32_t n, ActScanPart* parts) {
  __shared__ uint64_t w64[kScT / 64];
  __shared__ uint32_t w32[kScT / 64];
  const uint32_t base = blockIdx.x * kScTile;
  uint64_t a = kMaxKey, b = kMaxKey;
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < kScItems; ++j) {
    const uint32_t i = base + j * kScT + threadIdx.x;
    if (i < n) {
      a = MinU64::op(a, act.cnew[i]);
      b = MinU64::op(b, act.cold[i]);
      if (act.flag) c += act.flag[i];
    }
  }
  uint64_t ta, tb;
  uint32_t tc;
  (void)block_excl<MinU64>(a, w64, &ta);
  (void)block_excl<MinU64>(b, w64, &tb);
  (void)block_excl<SumU32>(c, w32, &tc);
  if (threadIdx.x == 0) parts[blockIdx.x] = ActScanPart{ta, tb, tc, 0};
}


__global__ void __launch_bounds__(kScT)
k_act_scan_down(ActBuf act, uint32_t n, const ActScanPart* parts, uint32_t* idx,
                uint32_t* dm) {
  __shared__ uint64_t ta[kScTile], tb[kScTile];
  __shared__ uint32_t tc[kScTile];
  __shared__ uint64_t w64[kScT / 64];
  __shared__ uint32_t w32[kScT / 64];
  const uint32_t base = blockIdx.x * kScTile;
#pragma unroll
  for (int j = 0; j < kScItems; ++j) {
    const uint32_t i = base + j * kScT + threadIdx.x, l = j * kScT + threadIdx.x;
    const bool in = i < n;
    ta[l] = in ? act.cnew[i] : kMaxKey;
    tb[l] = in ? act.cold[i] : kMaxKey;
    tc[l] = in && idx ? act.flag[i] : 0u;
  }
  __syncthreads();
  uint64_t va[kScItems], vb[kScItems];
  uint32_t vc[kScItems];
  uint64_t a = kMaxKey, b = kMaxKey;
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < kScItems; ++j) {
    const uint32_t l = threadIdx.x * kScItems + j;
    va[j] = a;
    vb[j] = b;
    vc[j] = c;
    a = MinU64::op(a, ta[l]);
    b = MinU64::op(b, tb[l]);
    c += tc[l];
  }
  // the carry-in: the tile totals of the blocks before this one (k_act_scan_
  // reduce's), combined here by every block (no separate top-level launch)
  ActScanPart cin;
  {
    uint64_t ma = kMaxKey, mb = kMaxKey;
    uint32_t mc = 0;
    for (uint32_t i = threadIdx.x; i < blockIdx.x; i += kScT) {
      const ActScanPart v = parts[i];
      ma = MinU64::op(ma, v.mn);
      mb = MinU64::op(mb, v.mo);
      mc += v.c;
    }
    ma = wave_min_u64(ma);
    mb = wave_min_u64(mb);
    mc = wave_sum_u32(mc);
    if ((threadIdx.x & 63) == 0) {
      w64[threadIdx.x >> 6] = ma;
      w32[threadIdx.x >> 6] = mc;
    }
    __syncthreads();
    cin.mn = w64[0];
    cin.c = w32[0];
    for (int i = 1; i < kScT / 64; ++i) {
      cin.mn = MinU64::op(cin.mn, w64[i]);
      cin.c += w32[i];
    }
    __syncthreads();
    if ((threadIdx.x & 63) == 0) w64[threadIdx.x >> 6] = mb;
    __syncthreads();
    cin.mo = w64[0];
    for (int i = 1; i < kScT / 64; ++i) cin.mo = MinU64::op(cin.mo, w64[i]);
    __syncthreads();  // (w64 is reused by the scans below)
  }
  uint32_t tot;
  const uint64_t ea = MinU64::op(cin.mn, block_excl<MinU64>(a, w64));
  const uint64_t eb = MinU64::op(cin.mo, block_excl<MinU64>(b, w64));
  const uint32_t ec = cin.c + block_excl<SumU32>(c, w32, &tot);
#pragma unroll
  for (int j = 0; j < kScItems; ++j) {
    const uint32_t l = threadIdx.x * kScItems + j;
    if (idx && tc[l]) idx[ec + vc[j]] = base + l;  // (flags are 0 / 1)
    ta[l] = MinU64::op(ea, va[j]);
    tb[l] = MinU64::op(eb, vb[j]);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kScItems; ++j) {
    const uint32_t i = base + j * kScT + threadIdx.x, l = j * kScT + threadIdx.x;
    if (i < n) {
      act.pre[i] = ta[l];
      act.suf[i] = tb[l];
    }
  }
  if (dm && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *dm = cin.c + tot;
}

// The sequential part of the idle resets, from activation j0 on with the
// exact running minimum *M of the earlier activations' contributions:
//   L_j = min(X_j, M_j), pd_j = L_j - t_j, c_j = p_j + pd_j,
//   M_{j+1} = min(M_j, c_j)                                   (:957-984)
// evaluated in windows of kActThreads activations, one per thread:
//  1. speculate: on the integer grid g of M's binade every rounded
//     operation above is an integer add (x - t rounds to x/g - rint(t/g)
//     when the result stays in the binade), so the recurrence becomes the
//     min-plus affine map m_{j+1} = min(m_j + min(0, d_j), rint(X_j/g) + d_j),
//     d_j = rint(p_j/g) - rint(t_j/g), whose composition is associative: one
//     block scan gives every M_j of the window;
//  2. verify: every thread evaluates its activation exactly (the reference's
//     double arithmetic) from the speculated M_j and checks that it yields the
//     speculated M_{j+1}.  Up to and including the first failing activation
//     the values are exact (its M_j was verified by its predecessor); the
//     window commits them and the next one starts after it.
// Binade crossings, rounding ties and X-restarts off the grid fail a
// check, which costs one window; a window that advances less than 64
// activations hands the next kActThreads to the wave-stepped recurrence
// (act_wave_steps), whose cost is the number of new minima.
__device__ inline double act_grid(double ref) {
  int e = 0;
  (void)frexp(ref, &e);  // ref = f * 2^e, 0.5 <= |f| < 1
  return ldexp(1.0, e - 53);
}

struct AffMin {  // y -> min(y + a, b) on the grid (integer-valued doubles)
  double a, b;
};
__device__ inline AffMin aff_then(AffMin f, AffMin g) {  // g after f
  return AffMin{f.a + g.a, fmin(f.b + g.a, g.b)};
}

// a barrier over the threads running the chain: the block, or one wave
// (whose LDS operations complete in order: a fence for the compiler)
template <uint32_t NT>
__device__ __attribute__((always_inline)) inline void act_sync() {
  if constexpr (NT == 64) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
}

// (NT: the threads that run it -- the block, or wave 0 alone, whose
// synchronisations are then the wave's)
template <uint32_t NT = kActThreads>
__device__ inline void act_wave_steps(uint32_t c0, uint32_t e, uint64_t base,
                                      const uint64_t* ax, const double* ap,
                                      const double* at, double* apd, double* s_M,
                                      uint64_t* mout = nullptr) {
  // one wave steps the recurrence: with M fixed, every lane evaluates its
  // activation; the first lane whose contribution undercuts M (a new
  // minimum) ends the step, lanes up to it commit (their M was exact), and
  // M takes that lane's value.  Steps: the new minima plus e / 64.
  const uint32_t t = threadIdx.x;
  if (t < 64) {
    constexpr double dmax = 1.7976931348623157e308;  // :960
    constexpr double trigger = dmax / 3.0;            // :957
    double M = *s_M;
    for (uint32_t j0 = 0; j0 < e; j0 += 64) {
      const uint32_t j = c0 + j0 + t;
      const bool in = j0 + t < e;
      double rx = kInf, rp = 0.0, rt = 0.0, rpd0 = 0.0;
      if (in) {
        const uint64_t x = ax[j] < base ? ax[j] : base;
        rx = x == kMaxKey ? kInf : from_okey(x);
        rp = ap[j];
        rt = at[j];
        rpd0 = apd[j];
      }
      const uint32_t w = e - j0 < 64u ? e - j0 : 64u;
      double out = rpd0, mo = 0.0;
      for (uint32_t done = 0; done < w;) {
        const bool act = in && t >= done;
        double L = M < rx ? M : rx;
        double lowest = L < dmax ? L : dmax;
        const double pd = lowest < trigger ? __dsub_rn(lowest, rt) : rpd0;
        const double c = __dadd_rn(rp, pd);
        const uint64_t rec = __ballot(act && c < M);
        const uint32_t r = rec ? (uint32_t)(__ffsll((unsigned long long)rec) - 1) : 64u;
        if (act && t <= r) {
          out = pd;
          mo = t == r ? c : M;
        }
        if (rec) M = __shfl(c, (int)r);
        done = r == 64u ? 64u : r + 1;
      }
      if (in) apd[j] = out;  // committed by k_act_commit
      if (in && mout) mout[j] = mo == kInf ? kMaxKey : okey(mo);
    }
    if (t == 0) *s_M = M;
  }
  act_sync<NT>();
}

constexpr int kChainK = 4;  // activations per thread and window (4096 per window)

// (mout: M after each activation, as an ordered key; wave_below: a window
// that advances less than this many activations hands the next kActThreads
// to the wave-stepped recurrence)
// (always inlined: three kernels call it, and a call frame is scratch)
template <uint32_t NT = kActThreads>
__device__ __attribute__((always_inline)) inline void act_chain(
    uint32_t j0, uint32_t m, uint64_t base, const uint64_t* ax,
                          const double* ap, const double* at, double* apd, double* s_M,
                          uint64_t* dbg, uint64_t* mout = nullptr, uint32_t wave_below = 64,
                          uint32_t wave_len = kActThreads) {
  constexpr double dmax = 1.7976931348623157e308;
  constexpr double trigger = dmax / 3.0;
  __shared__ double s_ref, s_last[NT];
  __shared__ AffMin s_w[NT / 64];
  __shared__ uint32_t s_f;
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  constexpr uint32_t WW = NT * kChainK;
  uint32_t nwin = 0, nwave = 0;  // (debug counts)
  while (j0 < m) {
    const uint32_t W = m - j0 < WW ? m - j0 : WW;
    // this thread's activations: j0 + kChainK * t + u
    double rx[kChainK], rp[kChainK], rt[kChainK], rpd0[kChainK];
#pragma unroll
    for (int u = 0; u < kChainK; ++u) {
      const uint32_t i = kChainK * t + u;
      rx[u] = kInf;
      rp[u] = rt[u] = rpd0[u] = 0.0;
      if (i < W) {
        const uint64_t x = ax[j0 + i] < base ? ax[j0 + i] : base;
        rx[u] = x == kMaxKey ? kInf : from_okey(x);
        rp[u] = ap[j0 + i];
        rt[u] = at[j0 + i];
        rpd0[u] = apd[j0 + i];
      }
    }
    const double M0 = *s_M;
    if (t == 0) {
      s_ref = M0 < kInf ? M0 : rx[0];  // the chain's binade (else the first X's)
      s_f = W;
      if (dbg && nwin < 12) dbg[16 + 2 * nwin] = wall_clock64();
    }
    act_sync<NT>();
    const double g = act_grid(s_ref);
    const double gi = 1.0 / g;  // a power of two: x * gi == x / g exactly
    // 1. speculate: the thread's composed map, then a block scan of the maps
    AffMin fu[kChainK];
    AffMin f{0.0, kInf};
#pragma unroll
    for (int u = 0; u < kChainK; ++u) {
      const bool in = kChainK * t + u < W;
      const double d = rint(rp[u] * gi) - rint(rt[u] * gi);
      fu[u] = AffMin{in ? fmin(0.0, d) : 0.0, in && rx[u] < kInf ? rint(rx[u] * gi) + d : kInf};
      f = aff_then(f, fu[u]);
    }
    AffMin incl = f;
    for (int o = 1; o < 64; o <<= 1) {
      AffMin v{__shfl_up(incl.a, o), __shfl_up(incl.b, o)};
      if ((int)lane >= o) incl = aff_then(v, incl);
    }
    if (lane == 63) s_w[wv] = incl;
    AffMin exw{__shfl_up(incl.a, 1), __shfl_up(incl.b, 1)};
    if (lane == 0) exw = AffMin{0.0, kInf};
    act_sync<NT>();
    AffMin pre{0.0, kInf};
    for (uint32_t i = 0; i < wv; ++i) pre = aff_then(pre, s_w[i]);
    const AffMin ex = aff_then(pre, exw);  // everything before this thread
    // this thread's speculated M after each of its activations, stepwise
    // from the exclusive prefix; the last one is the next thread's start
    double cur = fmin(M0 * gi + ex.a, ex.b);
    double spec[kChainK];
#pragma unroll
    for (int u = 0; u < kChainK; ++u) {
      cur = fmin(cur + fu[u].a, fu[u].b);
      spec[u] = cur * g;
    }
    s_last[t] = spec[kChainK - 1];
    act_sync<NT>();
    // 2. verify, in order (the reference's arithmetic from the speculated
    // M_j; a thread starts from its predecessor's last verified value)
    double Mj = t ? s_last[t - 1] : M0;
    double pd[kChainK], Mn[kChainK];
    uint32_t bad = 0xffffffffu;
#pragma unroll
    for (int u = 0; u < kChainK; ++u) {
      const uint32_t i = kChainK * t + u;
      const double L = Mj < rx[u] ? Mj : rx[u];
      const double lowest = L < dmax ? L : dmax;
      pd[u] = lowest < trigger ? __dsub_rn(lowest, rt[u]) : rpd0[u];
      const double c = __dadd_rn(rp[u], pd[u]);
      Mn[u] = c < Mj ? c : Mj;
      if (i < W && bad == 0xffffffffu && dbits(Mn[u]) != dbits(spec[u])) bad = i;
      Mj = spec[u];
    }
    if (bad != 0xffffffffu) atomicMin(&s_f, bad);
    act_sync<NT>();
    const uint32_t fl = s_f;  // first failing activation (W: none)
#pragma unroll
    for (int u = 0; u < kChainK; ++u) {
      const uint32_t i = kChainK * t + u;
      if (i < W && i <= fl) {
        apd[j0 + i] = pd[u];  // committed by k_act_commit
        if (mout) mout[j0 + i] = Mn[u] == kInf ? kMaxKey : okey(Mn[u]);
      }
      if (i == (fl < W ? fl : W - 1)) *s_M = Mn[u];
    }
    act_sync<NT>();
    const uint32_t adv = fl < W ? fl + 1 : W;
    if (dbg && t == 0 && nwin < 12)
      dbg[17 + 2 * nwin] = (uint64_t)j0 | ((uint64_t)adv << 32) | ((uint64_t)W << 48);
    ++nwin;
    j0 += adv;
    if (adv < wave_below && j0 < m) {
      // the grid does not describe this stretch: step it exactly
      const uint32_t e = m - j0 < wave_len ? m - j0 : wave_len;
      act_wave_steps<NT>(j0, e, base, ax, ap, at, apd, s_M, mout);
      ++nwave;
      j0 += e;
    }
  }
  if (dbg && t == 0) {
    dbg[5] = nwin;
    dbg[6] = nwave;
  }
}

// Step 3 (one block): only the M term is sequential.  Every L_k is first
// taken as X_k = min(unchanged, pre, suf), which is exact as long as
// M_{k-1} >= X_k for all k (checked chunk by chunk); from the first k where
// an earlier activation undercuts (an idle client whose old front tag lies
// behind the clock contributes below the reset it got) the recurrence runs
// on one thread over LDS-staged inputs.
__global__ void __launch_bounds__(kActThreads)
k_act_resolve(Table tb, ActBuf act, const uint64_t* ax, const double* ap,
              const double* at, double* apd, const uint32_t* aslot,
              uint64_t* dbg = nullptr) {
  // dbg (debug): [0] start [1] base [2] first pass [3] end clocks, [4] first
  // undercut, [5] windows, [6] wave fallbacks, [7] activations
  if (*act.anyhard) return;  // (k_act_hard's batch: it resolved and committed)
  if (dbg && threadIdx.x == 0) dbg[0] = wall_clock64();
  __shared__ uint64_t wpart[kActThreads / 64];
  __shared__ uint64_t s_base, s_carry, s_minpre;
  __shared__ uint32_t s_fail;
  __shared__ uint64_t sv[kActThreads];
  const uint32_t t = threadIdx.x, m = act.dm ? *act.dm : act.m;
  uint64_t b = kMaxKey;
  for (uint32_t i = t; i < act.nparts; i += kActThreads) b = act.parts[i] < b ? act.parts[i] : b;
  b = block_incl_min(b, wpart);
  if (t == kActThreads - 1) {
    uint64_t e = *act.extra;
    s_base = e < b ? e : b;
    s_carry = kMaxKey;  // M over the activations handled so far
    s_fail = 0xffffffffu;
  }
  __syncthreads();
  const uint64_t base = s_base;
  if (dbg && t == 0) dbg[1] = wall_clock64();
  uint32_t k0 = 0;
  // speculative: L_k = X_k
  for (; k0 < m; k0 += kActThreads) {
    const uint32_t k = k0 + t;
    const bool in = k < m;
    uint64_t x = kMaxKey, c = kMaxKey;
    double pd = 0.0;
    if (in) {
      x = ax[k] < base ? ax[k] : base;
      pd = act_pd(x, at[k], apd[k]);
      c = okey(__dadd_rn(ap[k], pd));
    }
    const uint64_t incl = block_incl_min(c, wpart);
    sv[t] = incl;
    __syncthreads();
    const uint64_t carry = s_carry;
    uint64_t mprev = t ? sv[t - 1] : kMaxKey;
    mprev = carry < mprev ? carry : mprev;
    if (in && mprev < x) atomicMin(&s_fail, k);
    __syncthreads();
    const uint32_t fail = s_fail;
    if (in && k < fail) apd[k] = pd;  // committed by k_act_commit
    if (fail != 0xffffffffu) {
      if (fail > k0 && t == fail - k0 - 1) s_minpre = incl;
      break;
    }
    if (t == kActThreads - 1) s_carry = carry < incl ? carry : incl;
    __syncthreads();
  }
  __syncthreads();
  const uint32_t fail = s_fail;
  if (fail != 0xffffffffu) {
    __shared__ double s_M;
    if (t == 0) {
      uint64_t M = s_carry;
      if (fail > k0) M = s_minpre < M ? s_minpre : M;
      s_M = M == kMaxKey ? kInf : from_okey(M);
    }
    __syncthreads();
    if (dbg && t == 0) dbg[2] = wall_clock64();
    act_chain(fail, m, base, ax, ap, at, apd, &s_M, dbg);
  }
  if (dbg && t == 0) {
    dbg[3] = wall_clock64();
    dbg[4] = fail;
    dbg[7] = m;
  }
  if (t == 0) *act.extra = kMaxKey;  // ready for the next batch
}

// ------------------------------------------------ segmented resolution
// The recurrence above, M_{j+1} = min(M_j, c_j(M_j)) with c_j(M) the
// contribution p_j + pd_j for L_j = min(X_j, M), resolved in tiles of
// kActTile activations:
//  * a "simple" activation -- X_j finite and p_j - t_j well above the
//    rounding of the operands -- has c_j(M) >= M for every M < X_j and
//    c_j(M) = K_j := c_j(X_j) for M >= X_j: its step is M -> min(M, K_j),
//    independent of M (config 4: about 98 % of them);
//  * so between two "complex" ones (an idle client whose proportion tag lies
//    behind the clock, p_j <= t_j, or X_j infinite) M only takes the minimum
//    of the run's K values, a segmented min-scan (k_act_keys, per tile);
//  * the complex ones are stepped in order by one wave (k_act_seq), with
//    the runs' minima between them: a lane per complex activation evaluates
//    its step with M fixed, and the first lane that changes M ends the
//    step, so the cost is the number of changes plus one step per 64;
//  * k_act_apply gives every activation its exact M_j (its segment's entry
//    and the run's minimum before it), evaluates it with the reference's
//    arithmetic, checks the simple ones' step (exact M_j and a holding step
//    prove M_{j+1}; the first failing activation, if any, is re-resolved
//    from its exact M by k_act_fixup's speculated min-plus chain) and
//    commits the idle reset.
constexpr uint32_t kActTile = kActThreads;
constexpr uint32_t kActItems = kActTile + 1;  // per tile: its complex steps and the tail

// The sequential steps, per tile (at t * kActItems): the tile's complex
// activations in order, each with the minimum of the simple run before it
// (S), then the tail pseudo-step (S = the run after the last one, X = none,
// no contribution: M -> min(M, S)).
struct ActTiles {
  uint64_t* K;      // n: c_j(X_j) (ordered key)
  uint32_t* nst;    // tiles: steps per tile (complex ones + 1)
  uint64_t* sS;     // tiles * kActItems: each step's run minimum
  uint64_t* sX;     // ... its X (kMaxKey: the tail)
  double *sP, *sT, *sPd0;  // ... its p, t, old prop_delta
  uint64_t* Mtile;  // tiles + 1: M entering each tile (k_act_seq)
  uint64_t* Mout;   // tiles * kActItems: M after each step (k_act_seq)
  uint64_t* Mj;     // n: M entering each activation (k_act_apply)
  uint64_t* cX;     // n: the complex steps, concatenated (k_act_seq's scratch)
  double *cP, *cT, *cPd;
  uint64_t* cMo;    // n: M after each of them
  uint64_t* xbase;  // 1: the unchanged clients' minimum (k_act_keys, block 0)
  uint32_t* fail;   // 1: the first activation whose simple step failed (~0: none)
};

// p + pd for L (ordered keys in, ordered key out): the reference's arithmetic
__device__ inline uint64_t act_contrib(uint64_t L, double p, double t, double pd0,
                                       double* pd_out) {
  const double pd = act_pd(L, t, pd0);
  if (pd_out) *pd_out = pd;
  return okey(__dadd_rn(p, pd));
}

__device__ inline bool act_simple(uint64_t X, double p, double t) {
  constexpr double trigger = 1.7976931348623157e308 / 3.0;
  if (X == kMaxKey) return false;
  const double x = from_okey(X);
  if (!(x < trigger)) return false;
  const double d = __dsub_rn(p, t);
  return d > 0x1p-40 * (fabs(x) + fabs(t) + fabs(p) + 1.0);
}

// segmented inclusive min-scan over a block (1024 threads): a reset element
// (a complex activation) starts a new run with its own value
struct SegMin {
  uint32_t r;
  uint64_t m;
};
__device__ inline SegMin seg_op(SegMin a, SegMin b) {  // a then b
  return b.r ? b : SegMin{a.r, a.m < b.m ? a.m : b.m};
}
__device__ inline SegMin block_seg_min(SegMin v, SegMin* wpart) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int d = 1; d < 64; d <<= 1) {
    SegMin o{(uint32_t)__shfl_up((int)v.r, d), shfl_up_u64(v.m, d)};
    if (lane >= d) v = seg_op(o, v);
  }
  if (lane == 63) wpart[w] = v;
  __syncthreads();
  SegMin b{0, kMaxKey};
  for (int i = 0; i < w; ++i) b = seg_op(b, wpart[i]);
  __syncthreads();
  return seg_op(b, v);
}

// the tile's activations: X, K, classification, the complex ones compacted
// with the runs' minima before them
// (its inputs gathered here, as k_act_inputs would, and stored for the
// kernels after it: one launch and one level of loads fewer)
__global__ void __launch_bounds__(kActThreads)
k_act_keys(const AddParams* pblk, Table tb, ActBuf act, uint64_t* ax, double* ap, double* at,
           double* apd, uint32_t* aslot, ActTiles tl) {
  __shared__ uint64_t wmin[kActThreads / 64];
  __shared__ SegMin wseg[kActThreads / 64];
  __shared__ uint32_t wcnt[kActThreads / 64];
  __shared__ uint64_t s_incl[kActThreads];
  const uint32_t m = act.dm ? *act.dm : act.m;
  const uint32_t t = blockIdx.x, j0 = t * kActTile;
  if (j0 >= m) return;
  // this activation's inputs (k_act_inputs' gather)
  const uint32_t j = j0 + threadIdx.x;
  const bool in = j < m;
  uint64_t xj = kMaxKey;
  double pj = 0.0, tj = 0.0, pdj = 0.0;
  if (in) {
    const AddParams p = *pblk;
    const uint32_t q = act.idx[j];
    const uint64_t a = act.pre[q], b = act.suf[p.n - 1 - q];
    xj = a < b ? a : b;
    const dmc_request& rq = p.reqs[q];
    pj = act.actp[q];
    tj = rq.time;
    pdj = tb.rec[rq.slot].pd;
    ax[j] = xj;
    ap[j] = pj;
    at[j] = tj;
    aslot[j] = rq.slot;
    apd[j] = pdj;
  }
  if (*act.anyhard) return;  // (anyhard: k_act_hard's batch, resolved by k_act_fixup)
  // the unchanged clients' minimum (every block; block 0 publishes it)
  uint64_t b = kMaxKey;
  for (uint32_t i = threadIdx.x; i < act.nparts; i += kActThreads)
    b = act.parts[i] < b ? act.parts[i] : b;
  b = block_incl_min(b, wmin);
  __shared__ uint64_t s_base;
  if (threadIdx.x == kActThreads - 1) {
    const uint64_t e = *act.extra;
    s_base = e < b ? e : b;
    if (t == 0) *tl.xbase = s_base;
  }
  __syncthreads();
  const uint64_t base = s_base;
  uint64_t K = kMaxKey;
  bool cx = false;
  if (in) {
    const uint64_t X = xj < base ? xj : base;
    K = act_contrib(X, pj, tj, pdj, nullptr);
    cx = !act_simple(X, pj, tj);
    tl.K[j] = K;
  }
  const SegMin incl = block_seg_min(SegMin{cx ? 1u : 0u, cx ? kMaxKey : K}, wseg);
  s_incl[threadIdx.x] = incl.m;
  // the complex ones' ranks in the tile
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t bal = __ballot(in && cx);
  if (lane == 0) wcnt[w] = (uint32_t)__popcll(bal);
  __syncthreads();
  uint32_t rank = (uint32_t)__popcll(bal & ((1ull << lane) - 1ull)), tot = 0;
  for (int i = 0; i < kActThreads / 64; ++i) {
    rank += i < w ? wcnt[i] : 0u;
    tot += wcnt[i];
  }
  const uint32_t o = t * kActItems;
  if (in && cx) {
    tl.sS[o + rank] = threadIdx.x ? s_incl[threadIdx.x - 1] : kMaxKey;
    tl.sX[o + rank] = xj < base ? xj : base;
    tl.sP[o + rank] = pj;
    tl.sT[o + rank] = tj;
    tl.sPd0[o + rank] = pdj;
  }
  const uint32_t last = (m - j0 < kActTile ? m - j0 : kActTile) - 1;
  if (threadIdx.x == last) {
    // the tail pseudo-step (a complex last one: its own run, empty)
    tl.nst[t] = tot + 1;
    tl.sS[o + tot] = incl.m;
    tl.sX[o + tot] = kMaxKey;
    tl.sP[o + tot] = 0.0;
    tl.sT[o + tot] = 0.0;
    tl.sPd0[o + tot] = 0.0;
  }
}

// The complex steps in order (one block): concatenated over the tiles, then
// resolved by act_chain's speculated min-plus scan (windows of up to 4096
// steps checked with the reference's arithmetic; a window advancing fewer
// than 8 steps hands the next 64 to the wave-stepped recurrence), starting
// from the minimum of every simple run before the first one.  The runs'
// minima between later complex steps are not applied here (they lie above M
// in practice): k_act_apply checks each step from its exact entry, and a
// run minimum below M fails that check (the batch is re-resolved from
// there).  Each tile's entry M is then stepped over the tiles exactly.
constexpr uint32_t kActMaxTiles = 1024;  // (batches of up to 2^20 activations)
#ifndef DMC_SEQ_LDS
#define DMC_SEQ_LDS 2048
#endif
constexpr uint32_t kSeqLds = DMC_SEQ_LDS;  // complex steps chained in LDS (k_act_seq)
#ifndef DMC_SEQ_WAVE
#define DMC_SEQ_WAVE 1  // ... by wave 0 alone
#endif
// (dbg, debug queues: [0..4] clocks -- start, offsets, complex steps
// gathered, chain done, end; [5] windows, [6] wave fallbacks, [7] complex
// steps, [8] tiles)
__global__ void __launch_bounds__(kActThreads)
k_act_seq(ActBuf act, ActTiles tl, uint64_t* dbg = nullptr) {
  if (*act.anyhard) return;
  if (dbg && threadIdx.x == 0) dbg[0] = wall_clock64();
  __shared__ uint32_t s_off[kActMaxTiles + 1];  // complex steps before each tile
  __shared__ uint32_t wsum[kActThreads / 64];
  __shared__ uint64_t s_tail[kActMaxTiles];     // each tile's tail run minimum
  __shared__ uint64_t wmin[kActThreads / 64];
  __shared__ double s_M;
  const uint32_t m = act.dm ? *act.dm : act.m;
  const uint32_t T = (m + kActTile - 1) / kActTile;
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  {
    const uint32_t v = tid < T ? tl.nst[tid] - 1u : 0u;
    uint32_t incl = v;
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t o = __shfl_up(incl, d);
      if ((int)lane >= d) incl += o;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t b = 0, tot = 0;
    for (int i = 0; i < kActThreads / 64; ++i) {
      b += i < (int)w ? wsum[i] : 0u;
      tot += wsum[i];
    }
    if (tid < T) {
      s_off[tid] = b + incl - v;
      s_tail[tid] = tl.sS[tid * kActItems + v];
    }
    if (tid == 0) s_off[T] = tot;
  }
  __syncthreads();
  const uint32_t nc = s_off[T];
  if (dbg && tid == 0) {
    dbg[1] = wall_clock64();
    dbg[7] = nc;
    dbg[8] = T;
  }
  {
    // M entering the first complex step: every simple run before it (the
    // tails of the tiles before its tile, and its own run)
    uint64_t mn = kMaxKey;
    if (tid < T && s_off[tid + 1] == 0) mn = s_tail[tid];  // (no complex step up to it)
    if (nc && tid < T && s_off[tid] == 0 && s_off[tid + 1] > 0) {
      const uint64_t s0 = tl.sS[tid * kActItems];
      mn = s0 < mn ? s0 : mn;
    }
    mn = block_incl_min(mn, wmin);
    if (tid == kActThreads - 1) s_M = mn == kMaxKey ? kInf : from_okey(mn);
  }
  __syncthreads();
  auto tile_of = [&](uint32_t g) -> uint32_t {  // s_off[t] <= g < s_off[t + 1]
    uint32_t lo = 0, hi = T;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (s_off[mid] <= g) lo = mid;
      else hi = mid;
    }
    return lo;
  };
#ifndef DMC_ACT_WAVE_BELOW
#define DMC_ACT_WAVE_BELOW 8
#endif
#ifndef DMC_ACT_WAVE_LEN
#define DMC_ACT_WAVE_LEN 64
#endif
  // the complex steps gathered in order, chained, their M scattered back
  // (cx..cmo: LDS for up to kSeqLds of them -- every chain window then reads
  // and writes LDS instead of waiting on global stores and loads -- else the
  // global scratch)
  __shared__ uint64_t s_last[kActMaxTiles];
  auto run = [&](uint64_t* cx, double* cp, double* ct, double* cpd, uint64_t* cmo, bool wave) {
    for (uint32_t g = tid; g < nc; g += kActThreads) {
      const uint32_t t = tile_of(g), at = t * kActItems + (g - s_off[t]);
      cx[g] = tl.sX[at];
      cp[g] = tl.sP[at];
      ct[g] = tl.sT[at];
      cpd[g] = tl.sPd0[at];
    }
    __threadfence();
    __syncthreads();
    if (dbg && tid == 0) dbg[2] = wall_clock64();
    if (nc && wave) {
      // (wave 0 alone: the windows' barriers and scans are the wave's)
      if (tid < 64)
        act_chain<64>(0, nc, kMaxKey, cx, cp, ct, cpd, &s_M, dbg, cmo, DMC_ACT_WAVE_BELOW,
                      DMC_ACT_WAVE_LEN);
    } else if (nc) {
      act_chain(0, nc, kMaxKey, cx, cp, ct, cpd, &s_M, dbg, cmo, DMC_ACT_WAVE_BELOW,
                DMC_ACT_WAVE_LEN);
    }
    __threadfence();
    __syncthreads();
    if (dbg && tid == 0) dbg[3] = wall_clock64();
    for (uint32_t g = tid; g < nc; g += kActThreads) {
      const uint32_t t = tile_of(g);
      tl.Mout[t * kActItems + (g - s_off[t])] = cmo[g];
    }
    for (uint32_t t = tid; t < T; t += kActThreads)
      s_last[t] = s_off[t + 1] > s_off[t] ? cmo[s_off[t + 1] - 1] : kMaxKey;
  };
  if (nc <= kSeqLds) {
    __shared__ uint64_t l_x[kSeqLds], l_mo[kSeqLds];
    __shared__ double l_p[kSeqLds], l_t[kSeqLds], l_pd[kSeqLds];
    run(l_x, l_p, l_t, l_pd, l_mo, DMC_SEQ_WAVE != 0);
  } else {
    run(tl.cX, tl.cP, tl.cT, tl.cPd, tl.cMo, false);
  }
  // M entering each tile, stepped over the tiles: after a tile's last
  // complex step (if any), then its tail run
  __syncthreads();
  if (tid == 0) {
    uint64_t M = kMaxKey;
    for (uint32_t t = 0; t < T; ++t) {
      tl.Mtile[t] = M;
      if (s_off[t + 1] > s_off[t]) M = s_last[t];
      M = s_tail[t] < M ? s_tail[t] : M;
    }
    tl.Mtile[T] = M;
    if (dbg) dbg[4] = wall_clock64();
  }
}

// Every activation's exact M_j, its idle reset evaluated and committed; the
// simple ones' steps checked (the first failure: k_act_fixup)
__global__ void __launch_bounds__(kActThreads)
k_act_apply(Table tb, ActBuf act, const uint64_t* ax, const double* ap, const double* at,
            const double* apd, const uint32_t* aslot, ActTiles tl) {
  __shared__ SegMin wseg[kActThreads / 64];
  __shared__ uint32_t wcnt[kActThreads / 64];
  const uint32_t m = act.dm ? *act.dm : act.m;
  const uint32_t t = blockIdx.x, j0 = t * kActTile;
  if (j0 >= m || *act.anyhard) return;
  const uint64_t base = *tl.xbase;
  const uint32_t j = j0 + threadIdx.x;
  const bool in = j < m;
  uint64_t X = kMaxKey, K = kMaxKey;
  double p = 0.0, tt = 0.0, pd0 = 0.0;
  uint32_t slot = 0;
  bool cx = false;
  ScanRec sr{};
  double fp = 0.0;
  if (in) {
    X = ax[j] < base ? ax[j] : base;
    p = ap[j];
    tt = at[j];
    pd0 = apd[j];
    K = tl.K[j];
    slot = aslot[j];
    cx = !act_simple(X, p, tt);
    // the idle reset's own loads (activate_slot's), issued ahead of the scan
    sr = tb.sc[slot];
    if (sr.count) fp = tb.ring[(size_t)slot * tb.q + (sr.head & tb.qmask)].p;
  }
  // exclusive run minimum before j (a complex j: its run's, cxS)
  const SegMin incl = block_seg_min(SegMin{cx ? 1u : 0u, cx ? kMaxKey : K}, wseg);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  SegMin ex{(uint32_t)__shfl_up((int)incl.r, 1), shfl_up_u64(incl.m, 1)};
  __shared__ SegMin s_wlast[kActThreads / 64];
  if (lane == 63) s_wlast[w] = incl;
  // complex ones strictly before j in the tile: the segment's entry is the
  // last one's M after it, else the tile's entry
  const uint64_t bal = __ballot(in && cx);
  if (lane == 0) wcnt[w] = (uint32_t)__popcll(bal);
  __syncthreads();
  if (lane == 0) ex = w ? s_wlast[w - 1] : SegMin{0, kMaxKey};
  uint32_t before = (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
  for (int i = 0; i < w; ++i) before += wcnt[i];
  if (!in) return;
  // (a run's minimum restarts after each complex one: ex.m is the current
  // run's minimum before j, at a complex j the run before it)
  const uint64_t run = threadIdx.x ? ex.m : kMaxKey;
  const uint64_t entry = before ? tl.Mout[t * kActItems + before - 1] : tl.Mtile[t];
  uint64_t Mj = run < entry ? run : entry;
  double pd;
  const uint64_t L = X < Mj ? X : Mj;
  const uint64_t c = act_contrib(L, p, tt, pd0, &pd);
  if (!cx) {
    // a simple step: min(M, c(M)) must be min(M, K)
    const uint64_t a = c < Mj ? c : Mj, b2 = K < Mj ? K : Mj;
    if (a != b2) atomicMin(tl.fail, j);
  } else {
    // a complex step: k_act_seq's M after it, from this exact entry
    const uint64_t a = c < Mj ? c : Mj;
    if (a != tl.Mout[t * kActItems + before]) atomicMin(tl.fail, j);
  }
  tl.Mj[j] = Mj;
  // activate_slot with its loads made above
  tb.rec[slot].pd = pd;
  if (sr.count) tb.sc[slot].pk = __dadd_rn(fp, pd);
  tb.sc[slot].flags = (uint8_t)(sr.flags & ~F_IDLE);
}

// AtLimit::Reject: the batches where an activated client's activating
// request was rejected (it stays non-idle and empty, :969-993) and later
// requests of the batch move its proportion basis (ActBuf::hev_q).  Such a
// "hard" client contributes basis + its new prop_delta, a value that rises
// at each change, which the tile resolution's running minimum cannot
// express.  One wave resolves these batches in activation order instead:
//   L_k = min(X_k, M, Mh),  pd_k = L_k - t_k (or unchanged above the trigger),
//   c_k = p_k + pd_k, then M = min(M, c_k), or for a hard client Mh (the
//   minimum over the hard clients' current values) takes c_k,
// and before activation k every basis change at a position below q_k
// raises its client's value to P + pd (Mh recomputed when the raised value
// was the minimum).  X_k is the tile path's (base, cold / cnew scans).  The
// per-activation inputs come from k_act_inputs; the wave loads 64 of them
// at a time and steps through them with uniform (readlane) values.
// Commits the idle resets; the tile kernels see *anyhard and do nothing.
// Run by wave 0 of k_act_fixup (no launch of its own), or by k_act_hard
// before the one-block k_act_resolve.  (Any mode: an activating request
// whose tag calculation failed leaves its client empty too.)
__device__ __attribute__((always_inline)) inline double rl_d(double v, uint32_t l) {
  const uint64_t b = dbits(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, (int)l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), (int)l);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __attribute__((always_inline)) inline uint64_t rl_u64(uint64_t v, uint32_t l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)l);
  return ((uint64_t)hi << 32) | lo;
}
__device__ inline double wave_min_d(double v) {
  for (int d = 32; d > 0; d >>= 1) {
    const double o = __shfl_xor(v, d);
    v = o < v ? o : v;
  }
  return v;
}

struct ActHard {
  uint32_t* hmap;   // per batch position: the hard client's activation index
  uint32_t* hlist;  // the hard clients' activation indices, in order
  double *hval, *hpd;  // per activation index: current value, prop_delta
  uint64_t* nhard;  // batches resolved here (counter)
};

__device__ inline void act_hard_body(const Table& tb, const ActBuf& act, const uint64_t* ax,
                                     const double* ap, const double* at, double* apd,
                                     const uint32_t* aslot, const ActHard& hs) {
  constexpr double dmax = 1.7976931348623157e308;  // :960
  constexpr double trigger = dmax / 3.0;            // :957
  const uint32_t lane = threadIdx.x;
  const uint32_t m = act.dm ? *act.dm : act.m;
  uint64_t b = kMaxKey;
  for (uint32_t i = lane; i < act.nparts; i += 64) b = act.parts[i] < b ? act.parts[i] : b;
  b = rl_u64(wave_min_u64(b), 0);
  const uint64_t e = *act.extra;
  const uint64_t base = e < b ? e : b;
  double M = kInf, Mh = kInf;
  uint32_t H = 0, pos = 0;
  for (uint32_t k0 = 0; k0 < m; k0 += 64) {
    const uint32_t k = k0 + lane;
    const bool in = k < m;
    uint32_t q = 0, hd = 0;
    uint64_t x = kMaxKey;
    double p = 0.0, t = 0.0, pd0 = 0.0;
    if (in) {
      q = act.idx[k];
      x = ax[k] < base ? ax[k] : base;
      p = ap[k];
      t = at[k];
      pd0 = apd[k];
      hd = act.hard[q];
    }
    double mypd = pd0;
    const uint32_t cnt = m - k0 < 64u ? m - k0 : 64u;
    for (uint32_t u = 0; u < cnt; ++u) {
      const uint32_t qu = (uint32_t)__builtin_amdgcn_readlane((int)q, (int)u);
      // the hard clients' basis changes at positions below qu
      while (pos < qu && H) {
        const uint32_t r = pos + lane;
        const uint32_t hq = r < qu ? act.hev_q[r] : kNone;
        uint64_t bal = __ballot(hq != kNone);
        while (bal) {
          const uint32_t j = (uint32_t)(__ffsll((unsigned long long)bal) - 1);
          bal &= bal - 1;
          const uint32_t aq = (uint32_t)__builtin_amdgcn_readlane((int)hq, (int)j);
          const uint32_t h = hs.hmap[aq];
          const double old = hs.hval[h];
          const double nv = __dadd_rn(act.hev_p[pos + j], hs.hpd[h]);
          if (lane == 0) hs.hval[h] = nv;
          __threadfence_block();
          if (nv < Mh) {
            Mh = nv;
          } else if (old == Mh && nv != old) {
            double mn = kInf;
            for (uint32_t i = lane; i < H; i += 64) {
              const double v = hs.hval[hs.hlist[i]];
              mn = v < mn ? v : mn;
            }
            Mh = rl_d(wave_min_d(mn), 0);
          }
        }
        pos = pos + 64 < qu ? pos + 64 : qu;
      }
      if (!H) pos = qu;  // (no hard client yet: nothing to raise)
      pos = qu + 1 > pos ? qu + 1 : pos;
      const uint64_t xu = rl_u64(x, u);
      const double rx = xu == kMaxKey ? kInf : from_okey(xu);
      double L = M < rx ? M : rx;
      L = Mh < L ? Mh : L;
      const double lowest = L < dmax ? L : dmax;
      const double pd = lowest < trigger ? __dsub_rn(lowest, rl_d(t, u)) : rl_d(pd0, u);
      const double c = __dadd_rn(rl_d(p, u), pd);
      if (lane == u) mypd = pd;
      if (__builtin_amdgcn_readlane((int)hd, (int)u)) {
        const uint32_t ku = k0 + u;
        if (lane == 0) {
          hs.hmap[qu] = ku;
          hs.hlist[H] = ku;
          hs.hval[ku] = c;
          hs.hpd[ku] = pd;
        }
        __threadfence_block();
        ++H;
        Mh = c < Mh ? c : Mh;
      } else {
        M = c < M ? c : M;
      }
    }
    if (in) {
      apd[k] = mypd;
      activate_slot(tb, aslot[k], mypd);
    }
  }
  if (lane == 0) ++*hs.nhard;
}

__global__ void __launch_bounds__(64)
k_act_hard(Table tb, ActBuf act, const uint64_t* ax, const double* ap, const double* at,
           double* apd, const uint32_t* aslot, ActHard hs) {
  if (!*act.anyhard) return;
  act_hard_body(tb, act, ax, ap, at, apd, aslot, hs);
  __threadfence_block();
  if (threadIdx.x == 0) *act.extra = kMaxKey;  // ready for the next batch
}

// The first activation whose simple step failed (if any): from its exact M
// the rest of the batch is resolved by act_chain and committed again (the
// idle reset is idempotent: k_act_apply's commits of these are overwritten)
__global__ void __launch_bounds__(kActThreads)
k_act_fixup(Table tb, ActBuf act, const uint64_t* ax, const double* ap, const double* at,
            double* apd, const uint32_t* aslot, ActTiles tl, ActHard hs) {
  if (threadIdx.x < 64 && *act.anyhard) act_hard_body(tb, act, ax, ap, at, apd, aslot, hs);
  const uint32_t f = *tl.fail;
  const uint32_t m = act.dm ? *act.dm : act.m;
  if (f != 0xffffffffu && f < m && !*act.anyhard) {
    __shared__ double s_M;
    if (threadIdx.x == 0) {
      const uint64_t M = tl.Mj[f];
      s_M = M == kMaxKey ? kInf : from_okey(M);
    }
    __syncthreads();
    act_chain(f, m, *tl.xbase, ax, ap, at, apd, &s_M, nullptr);
    for (uint32_t j = f + threadIdx.x; j < m; j += kActThreads) activate_slot(tb, aslot[j], apd[j]);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    *tl.fail = 0xffffffffu;
    *act.extra = kMaxKey;  // ready for the next batch
  }
}

// Step 4 (grid): every activation's idle reset takes effect -- prop_delta,
// its front's cached key, idle cleared (k_act_resolve left the resolved
// prop_deltas in apd; the resolution reads none of the state written here)
__global__ void k_act_commit(Table tb, const uint32_t* dm, uint32_t m0, const double* apd,
                             const uint32_t* aslot) {
  const uint32_t m = dm ? *dm : m0;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < m;
       k += gridDim.x * blockDim.x)
    activate_slot(tb, aslot[k], apd[k]);
}

// ------------------------------------------------------------------ future
__device__ inline double min_not_0(double cur, double possible) {  // :1192-1195
  return possible == 0.0 ? cur : (possible < cur ? possible : cur);
}

// ------------------------------------------------------------------ single step
// General do_next_request(now) one pull at a time (used for small k and for
// AtLimit::Allow limit breaks, :1157-1165).  Reductions are per block, then
// one block combines them.
// ATOMIC: the block's partial is stored with device-scope atomics (performed
// at the memory side, visible to a last block after its acquire with no
// release fence: an agent-scope release writes back the whole L2)
template <int THREADS = kBlock, bool ATOMIC = false>
__device__ __forceinline__ void step_scan_body(const Table& tb, double now, StepRed* part) {
  ArgMin r{kMaxKey, kNone, 0}, p{kMaxKey, kNone, 0}, pnr{kMaxKey, kNone, 0};
  uint64_t lnr = kMaxKey, lrd = kMaxKey;
  uint32_t nany = 0, nrd = 0, nnr = 0;
  // four records per thread in flight (their loads issued before the first
  // is used: the pass is bound by memory latency, not bandwidth)
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t s0 = blockIdx.x * blockDim.x + threadIdx.x; s0 < tb.n; s0 += 4 * stride) {
    ScanRec rs[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t su = s0 + u * stride;
      if (su < tb.n) rs[u] = tb.sc[su];
      else rs[u].count = 0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
    const uint32_t s = s0 + u * stride;
    const ScanRec sr = rs[u];
    if (!sr.count) continue;
    ++nany;
    ArgMin a{okey(sr.r), s, 1};
    r = argmin_combine(r, a);
    double l = sr.l;
    bool rdy = (sr.flags & F_READY) || l <= now;
    double pv = sr.pk;  // p + prop_delta: p < inf iff pv < inf
    uint64_t kp = okey(pv);
    uint64_t kl = okey(l);
    if (rdy) {
      ++nrd;
      lrd = kl < lrd ? kl : lrd;
      if (pv < kInf) p = argmin_combine(p, ArgMin{kp, s, 1});
    } else {
      ++nnr;
      lnr = kl < lnr ? kl : lnr;
      pnr = argmin_combine(pnr, ArgMin{kp, s, 1});
    }
    }
  }
  r = wave_argmin(r);
  p = wave_argmin(p);
  pnr = wave_argmin(pnr);
  lnr = wave_min_u64(lnr);
  lrd = wave_min_u64(lrd);
  nany = wave_sum_u32(nany);
  nrd = wave_sum_u32(nrd);
  nnr = wave_sum_u32(nnr);
  __shared__ StepRed sh[THREADS / 64];
  int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[w].r = r;
    sh[w].p = p;
    sh[w].pnr = pnr;
    sh[w].lmin_nr = lnr;
    sh[w].lmin_rd = lrd;
    sh[w].n_any = nany;
    sh[w].n_ready = nrd;
    sh[w].n_notready = nnr;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    StepRed o = sh[0];
    for (int i = 1; i < THREADS / 64; ++i) {
      o.r = argmin_combine(o.r, sh[i].r);
      o.p = argmin_combine(o.p, sh[i].p);
      o.pnr = argmin_combine(o.pnr, sh[i].pnr);
      o.lmin_nr = sh[i].lmin_nr < o.lmin_nr ? sh[i].lmin_nr : o.lmin_nr;
      o.lmin_rd = sh[i].lmin_rd < o.lmin_rd ? sh[i].lmin_rd : o.lmin_rd;
      o.n_any += sh[i].n_any;
      o.n_ready += sh[i].n_ready;
      o.n_notready += sh[i].n_notready;
    }
    if (ATOMIC) {
      static_assert(sizeof(StepRed) % 8 == 0, "StepRed is stored in 8-byte words");
      unsigned long long* dst = reinterpret_cast<unsigned long long*>(part + blockIdx.x);
#pragma unroll
      for (int i = 0; i < (int)(sizeof(StepRed) / 8); ++i)
        atomicExch(dst + i, ld_as<unsigned long long>(reinterpret_cast<const char*>(&o) + 8 * i));
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      part[blockIdx.x] = o;
    }
  }
}

__global__ void k_step_scan(Table tb, double now, StepRed* part) {
  step_scan_body(tb, now, part);
}

__device__ __attribute__((always_inline)) inline void stepred_combine(StepRed& o, const StepRed& b) {
  o.r = argmin_combine(o.r, b.r);
  o.p = argmin_combine(o.p, b.p);
  o.pnr = argmin_combine(o.pnr, b.pnr);
  o.lmin_nr = b.lmin_nr < o.lmin_nr ? b.lmin_nr : o.lmin_nr;
  o.lmin_rd = b.lmin_rd < o.lmin_rd ? b.lmin_rd : o.lmin_rd;
  o.n_any += b.n_any;
  o.n_ready += b.n_ready;
  o.n_notready += b.n_notready;
}

// launched with one block of kBlock threads; combines the per-block partials
// (tree reduction in LDS), then thread 0 decides
// do_next_request's decision from the combined reduction (:1115-1200)
__device__ inline StepCtl step_decision(const StepRed& o, double now, int at_limit,
                                        uint32_t nregistered) {
  StepCtl c{};
  c.type = DMC_NEXT_NONE;
  c.slot = kNone;
  if (nregistered == 0) return c;  // resv_heap.empty(), :1118-1120
  double rtop = o.n_any ? from_okey(o.r.key) : kInf;
  if (o.n_any && rtop <= now) {  // :1124-1128
    c.type = DMC_NEXT_RETURNING;
    c.prio = 0;
    c.slot = o.r.slot;
    c.tie = o.r.cnt > 1;
    return c;
  }
  c.mark = 1;  // the limit scan ran
  if (o.p.slot != kNone) {  // :1146-1151
    c.type = DMC_NEXT_RETURNING;
    c.prio = 1;
    c.slot = o.p.slot;
    c.tie = o.p.cnt > 1;
    return c;
  }
  if (at_limit == DMC_AT_LIMIT_ALLOW && o.n_any) {  // :1157-1165
    // ready-heap top: ready fronts first (all have p == inf here), else the
    // min p+pd over not-ready fronts
    bool top_ready = o.n_ready > 0;
    if (!top_ready && o.pnr.slot != kNone && from_okey(o.pnr.key) < kInf) {
      c.type = DMC_NEXT_RETURNING;
      c.prio = 1;
      c.slot = o.pnr.slot;
      c.tie = o.pnr.cnt > 1;
      return c;
    }
    if (rtop < kInf) {
      c.type = DMC_NEXT_RETURNING;
      c.prio = 0;
      c.slot = o.r.slot;
      c.tie = o.r.cnt > 1;
      return c;
    }
  }
  const double tmax = 1.7976931348623157e308;
  double next = tmax;
  if (o.n_any) {
    next = min_not_0(next, rtop);
    double lt = o.n_notready ? from_okey(o.lmin_nr) : from_okey(o.lmin_rd);
    next = min_not_0(next, lt);
  }
  if (next < tmax) {
    c.type = DMC_NEXT_FUTURE;
    c.when = next;
  }
  return c;
}

// launched with one block of THREADS threads; combines the per-block
// partials (tree reduction in LDS), then thread 0 decides (hsc: an optional
// host-mapped mirror of the decision)
template <int THREADS = kBlock>
__device__ __forceinline__ void step_decide(uint32_t nparts, const StepRed* part, double now,
                            int at_limit, uint32_t nregistered,
                            StepCtl* sc, Round* ctl, StepCtl* hsc = nullptr) {
  if (ctl && (ctl->overflow || !ctl->terminal)) return;
  if (ctl) now = ctl->now;
  __shared__ StepRed sh[THREADS];
  StepRed acc;
  acc.r = ArgMin{kMaxKey, kNone, 0};
  acc.p = acc.r;
  acc.pnr = acc.r;
  acc.lmin_nr = kMaxKey;
  acc.lmin_rd = kMaxKey;
  acc.n_any = acc.n_ready = acc.n_notready = 0;
  acc.pad = 0;
  for (uint32_t i = threadIdx.x; i < nparts; i += blockDim.x)
    stepred_combine(acc, part[i]);
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int d = THREADS / 2; d > 0; d >>= 1) {
    if ((int)threadIdx.x < d) stepred_combine(sh[threadIdx.x], sh[threadIdx.x + d]);
    __syncthreads();
  }
  if (threadIdx.x) return;
  const StepCtl c = step_decision(sh[0], now, at_limit, nregistered);
  *sc = c;
  if (hsc) *hsc = c;
  if (ctl) {
    ctl->next_type = c.type;
    ctl->when = c.when;
  }
}

// The general decision; a round's terminal pull also ends the round (h: the
// host-mapped summary, k_rfinish's work folded in).
__global__ void k_step_decide(uint32_t nparts, const StepRed* part, double now,
                              int at_limit, uint32_t nregistered,
                              StepCtl* sc, Round* ctl, HostRound* h) {
  step_decide(nparts, part, now, at_limit, nregistered, sc, ctl);
  if (h) {
    __syncthreads();
    rfinish_body(ctl, h);
  }
}

// A round's terminal pull in one kernel: the blocks scan the table and store
// their partials with memory-side atomics, and the last block to finish (one
// ticket counter; agent-scope acquire after it: MI355X_MICROARCH.md,
// inter-workgroup visibility) combines the partials, decides and ends the
// round again under `seq`.  The host launches it only after a round that
// ran out of work (k_rapply's last block published that round's summary).
constexpr int kFutThreads = 256;  // (1024-thread blocks spill the reductions to scratch)
constexpr uint32_t kFutBlocks = 1024;
__global__ void __launch_bounds__(kFutThreads)
k_round_future(Table tb, StepRed* part, int at_limit, uint32_t nregistered,
               StepCtl* sc, Round* ctl, HostRound* h, uint32_t* done, uint64_t seq) {
  // thread 0 stores the partial with memory-side atomics
  step_scan_body<kFutThreads, true>(tb, ctl->now, part);
  __shared__ uint32_t s_last;
  if (threadIdx.x == 0) {
    const bool last = atomicAdd(done, 1u) == gridDim.x - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  step_decide<kFutThreads>(gridDim.x, part, 0.0, at_limit, nregistered, sc, ctl);
  if (threadIdx.x == 0) ctl->seq = seq;  // the summary's second publication
  __syncthreads();
  if (threadIdx.x == 0) *done = 0;  // ready for the next round
  rfinish_body(ctl, h);
}

__global__ void k_step_mark(Table tb, double now, const StepCtl* sc) {
  if (!sc->mark) return;
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < tb.n;
       s += gridDim.x * blockDim.x) {
    const ScanRec sr = tb.sc[s];
    if (sr.count && !(sr.flags & F_READY) && sr.l <= now)
      tb.sc[s].flags = sr.flags | F_READY;
  }
}

// pop_process_request (+ reduce_reservation_tags for ready-heap pops) of the
// chosen client, :1046-1111.
__device__ void step_apply_body(const Table& tb, uint64_t tick, const StepCtl* sc,
                                dmc_decision* out, uint32_t out_idx,
                                unsigned long long* sched) {
  if (sc->type != DMC_NEXT_RETURNING) return;
  uint32_t s = sc->slot;
  bool prio = sc->prio != 0;
  ReqEntry* ring = tb.ring + (size_t)s * tb.q;
  const ScanRec sr = tb.sc[s];
  uint32_t h = sr.head, c = sr.count;
  ReqEntry popped = ring[h];
  dmc_decision d;
  d.handle = popped.handle;
  d.tag_r = popped.r;
  d.tag_p = popped.p;
  d.tag_l = popped.l;
  d.slot = s;
  d.cost = popped.cost;
  d.phase = prio ? DMC_PHASE_PRIORITY : DMC_PHASE_RESERVATION;
  d.flags = sc->tie ? 1u : 0u;
  out[out_idx] = d;
  uint32_t nh = (h + 1) & tb.qmask, nc = c - 1;
  double rinv = tb.rec[s].r_inv;
  if (tb.delayed && nc) {  // update_next_tag, :1021-1036
    ReqEntry& f = ring[nh];
    Tag3 pt{popped.r, popped.p, popped.l, popped.arrival};
    Tag3 nt;
    uint32_t cd = tb.aux[s].cur_delta, cr = tb.aux[s].cur_rho;
    double winv = tb.rec[s].w_inv, linv = tb.rec[s].l_inv;
    if (tb.binfo) {  // U1: get_cli_info (:870-875) becomes client.info
      const BoundInfo b = tb.binfo[s];
      rinv = b.r_inv;
      winv = b.w_inv;
      linv = b.l_inv;
      tb.rec[s].r_inv = rinv;
      tb.rec[s].w_inv = winv;
      tb.rec[s].l_inv = linv;
    }
    if (make_tag(pt, rinv, winv, linv, cd, cr, f.arrival, f.cost,
                 tb.antic, &nt)) {
      f.r = nt.r;
      f.p = nt.p;
      f.l = nt.l;
      f.delta = cd;
      f.rho = cr;
      double pr = tb.rec[s].prev_r, pp = tb.rec[s].prev_p, pl = tb.rec[s].prev_l;
      assign_unpinned(pr, nt.r);
      assign_unpinned(pl, nt.l);
      assign_unpinned(pp, nt.p);
      tb.rec[s].prev_r = pr;
      tb.rec[s].prev_p = pp;
      tb.rec[s].prev_l = pl;
      tb.rec[s].prev_arr = nt.arrival;
      tb.aux[s].last_tick = tick;
    }
  }
  if (prio) {  // reduce_reservation_tags, :1077-1111
    double o = resv_offset(rinv, popped.cost, popped.rho);
    if (tb.delayed) {
      if (nc) ring[nh].r = __dsub_rn(ring[nh].r, o);
    } else {
      for (uint32_t i = 1; i < c; ++i) {
        ReqEntry& e = ring[(h + i) & tb.qmask];
        e.r = __dsub_rn(e.r, o);
      }
    }
    tb.rec[s].prev_r = __dsub_rn(tb.rec[s].prev_r, o);
  }
  ScanRec o{0.0, 0.0, 0.0, (uint8_t)nh, (uint8_t)nc, (uint8_t)(sr.flags & ~F_READY), 0, 0};
  if (nc) {
    const ReqEntry& f = ring[nh];
    o.r = f.r;
    o.pk = __dadd_rn(f.p, tb.rec[s].pd);
    o.l = f.l;
  }
  tb.sc[s] = o;
  atomicAdd(&sched[prio ? 1 : 0], 1ull);
}

__global__ void k_step_apply(Table tb, uint64_t tick, const StepCtl* sc,
                             dmc_decision* out, uint32_t out_idx,
                             unsigned long long* sched) {
  if (threadIdx.x || blockIdx.x) return;
  step_apply_body(tb, tick, sc, out, out_idx, sched);
}

// ------------------------------------------------------------------ single-op path
// One pull_request(now) in two kernels and one host round trip (the facade's
// per-call path): k_fast_decide scans and, in its last block, decides
// (mirrored to host-mapped memory); k_fast_apply commits the limit scan's
// ready marks (grid) and, in its last block, pops the chosen client, writing
// the decision to host-mapped memory.  Cross-block hand-off as k_round_future:
// agent-scope release before the ticket, acquire in the last block.
// (the blocks' partials were stored with memory-side atomics, completed
// before the ticket: no release fence)
__device__ inline bool last_block(uint32_t* done) {
  __shared__ uint32_t s_last;
  if (threadIdx.x == 0) {
    const bool last = atomicAdd(done, 1u) == gridDim.x - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      *done = 0;  // ready for the next call (no other block touches it now)
    }
    s_last = last;
  }
  __syncthreads();
  return s_last != 0;
}

__global__ void __launch_bounds__(kFutThreads)
k_fast_decide(Table tb, double now, StepRed* part, int at_limit, uint32_t nregistered,
              StepCtl* sc, StepCtl* hsc, uint32_t* done) {
  step_scan_body<kFutThreads, true>(tb, now, part);
  if (!last_block(done)) return;
  step_decide<kFutThreads>(gridDim.x, part, now, at_limit, nregistered, sc, nullptr, hsc);
}

// The marks and the pop touch disjoint state (the popped client's own mark
// is moot: its new front is not ready), so block 0 pops while the grid marks.
__global__ void k_fast_apply(Table tb, double now, uint64_t tick, const StepCtl* sc,
                             dmc_decision* out, uint32_t out_idx,
                             unsigned long long* sched) {
  const StepCtl c = *sc;
  if (blockIdx.x == 0 && threadIdx.x == 0) step_apply_body(tb, tick, sc, out, out_idx, sched);
  if (!c.mark) return;
  const uint32_t skip = c.type == DMC_NEXT_RETURNING ? c.slot : kNone;
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < tb.n;
       s += gridDim.x * blockDim.x) {  // k_step_mark
    if (s == skip) continue;
    const ScanRec sr = tb.sc[s];
    if (sr.count && !(sr.flags & F_READY) && sr.l <= now)
      tb.sc[s].flags = sr.flags | F_READY;
  }
}

// One add_request of a client that needs no idle reset (the facade's
// per-call path): the request and its status in host-mapped memory.
__global__ void k_add_one(Table tb, const dmc_request* req, int32_t* rc, uint64_t tick) {
  if (threadIdx.x || blockIdx.x) return;
  const uint32_t s = req->slot;
  if (s >= tb.n || !(tb.sc[s].flags & F_REG)) {
    *rc = DMC_ENOTREG;
    return;
  }
  AddParams p{req, rc, tick, 1, 0};
  AddState st;
  add_chain_slot(tb, p, s, 1, 0, nullptr, nullptr, ActBuf{}, &st);
}

// ------------------------------------------------------------------ stats
__global__ void k_count_requests(Table tb, unsigned long long* out) {
  unsigned long long t = 0;
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < tb.n;
       s += gridDim.x * blockDim.x)
    t += tb.sc[s].count;
  for (int d = 32; d > 0; d >>= 1) t += shfl_down_u64(t, d);
  __shared__ unsigned long long sh[kBlock / 64];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < (int)(blockDim.x / 64); ++i) t += sh[i];
    if (t) atomicAdd(out, t);
  }
}

uint32_t grid_for(uint32_t n, uint32_t cap = 4096) {
  uint32_t g = (n + kBlock - 1) / kBlock;
  if (g < 1) g = 1;
  return g > cap ? cap : g;
}

}  // namespace

// ====================================================================== host
// A stage timer: HIP events around a stage on the queue's stream.
struct ProfRec {
  hipEvent_t a, b;
  int stage;
};

struct GraphRec {
  uint64_t key = 0;
  uint64_t last_use = 0;
  hipGraph_t graph = nullptr;
  // two instances, launched alternately: a call returns while its launch's
  // last kernel may still run, so the next call updates and launches the
  // other one and never touches an instance in flight
  hipGraphExec_t exec = nullptr, exec2 = nullptr;
  bool flip = false;
  hipGraphNode_t param_node = nullptr;
  hipKernelNodeParams kp{};
  hipGraphNode_t param_node2 = nullptr;  // fused add + pull: the round's k_rscan
  hipKernelNodeParams kp2{};
};

// host-mapped I/O of the single-op path
constexpr uint32_t kFastK = 8;
struct FastIO {
  StepCtl sc;
  dmc_decision dec[kFastK];
  dmc_request req;
  int32_t rc;
  int32_t pad;
};

namespace {
#include "dmc_serve.h"
#include "dmc_heap.h"
}  // namespace

struct dmc_queue {
  dmc_queue_params p{};
  hipStream_t stream = nullptr;
  // a member of a queue group (dmc_group_create) runs on the group's stream;
  // its own is kept here and restored when the group is destroyed
  hipStream_t own_stream = nullptr;
  dmc_group* group = nullptr;
  // graphs are captured on a stream of their own (created on first use):
  // a group's members share their execution stream with other host threads,
  // whose launches must never land in (or break) a capture
  hipStream_t cap_stream = nullptr;
  Table tb{};
  std::mutex mtx;  // C-ABI calls on one handle are serialised (data_mtx, :762)
  // host mirrors
  std::vector<uint8_t> reg_h, idle_h;
  // the bound ClientInfo (U1, dmc_client_bind_info_batch): device column and
  // its host shadow (3 inverses per slot, to skip unchanged pushes)
  BoundInfo* binfo = nullptr;
  std::vector<double> binfo_h;
  dmc_info_fn info_fn = nullptr;  // dmc_queue_set_info_fn
  void* info_ctx = nullptr;
  // single-op path (DMC_OPT_SINGLE_OP): host-mapped request / status /
  // decisions and the two kernels' ticket counters
  bool single_op = true;
  FastIO* h_fast = nullptr;
  FastIO* d_fast = nullptr;
  uint32_t* fast_done = nullptr;
  // the serve path (DMC_OPT_SERVE, dmc_serve.h): k_serve running on the
  // queue's stream; the group summaries are valid while no other call has
  // run since k_serve last wrote them
  bool serve_on = false;
  bool serving = false;
  bool gsum_valid = false;
  ServeIO* h_serve = nullptr;
  ServeIO* d_serve = nullptr;
  StepRed* gsum = nullptr;
  uint32_t gshift = 10, ngroups = 0;
  uint64_t serve_seq = 0;
  uint64_t serve_idle_ticks = 20000;  // 0.2 ms of the 100 MHz wall clock (lifetime: 5x)
  bool serve_reg = false;  // listed in the process's serve registry (serve_registry)
  // k_serve did not exit within kServeStopWait of a stop command: the
  // queue's stream is presumed wedged and every later call returns
  // DMC_EDEVICE instead of blocking on it
  bool wedged = false;
  // DMC_OPT_PIPELINE: the error of the last pipelined call that failed when
  // a later call finished it (that later call returned DMC_ENOTRUN or the
  // error itself); dmc_queue_pipelined_error reads it
  int pipe_err = 0;
  // DMC_OPT_HEAP_ORDER (dmc_heap.h): the reference's heaps on the device,
  // every add and pull in call order
  bool heap = false;
  HeapDev hd{};
  HeapPullRes* h_hres = nullptr;  // pinned
  HeapPullRes* d_hres = nullptr;
  // DMC_SERVE_TRACE: per-call phases (k_serve's wall-clock stamps), printed
  // at destroy: read, work, publish (ticks) and the host's call time (ns)
  bool serve_trace = getenv("DMC_SERVE_TRACE") != nullptr;
  double serve_tr[4] = {0, 0, 0, 0};
  double serve_ph[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};  // [add, pull]: phases, calls
  double serve_mhz = 0;
  // dmc_client_mark_idle_batch_device: the host idle mirror (idle_h /
  // n_idle) is stale until sync_idle reads the flags back
  bool idle_unknown = false;
  // queue-content generation (bumped by every call that can change a queue)
  // and the one dmc_queue_requests read, for dmc_queue_filter's check
  uint64_t gen = 0, maint_gen = ~0ull, maint_total = 0;
  uint32_t n_registered = 0;
  uint32_t n_idle = 0;
  uint64_t tick = 0;
  // device scratch
  CandRec* cand = nullptr;    // N (rounded up to emit blocks): candidates of the
                              // round, kEmitChunk per k_remit block
  uint32_t* bcand = nullptr;  // per k_remit block: its candidates
  PostRec* post = nullptr;    // per candidate: a fast candidate's state after its pop
  uint32_t* decof = nullptr;  // per candidate: kSlowCand, kNoDec or its decision offset
  uint64_t *keyr = nullptr, *keyp = nullptr;  // N: first keys per phase (unsampled rounds)
  uint2* k32 = nullptr;       // N: 32-bit quantized first keys (R, P), k_remit's stream
  uint32_t* meta = nullptr;   // N: k_rscan's per-slot R-prefix length, flags, head, count
  RoundPart* rparts = nullptr; // k_rscan's per-block partials
  Round* rd = nullptr;
  Round h_rd_copy{};          // host copy of the last round's summary
  Round* h_rd = &h_rd_copy;
  HostRound* h_round = nullptr;  // fine-grained pinned, written by k_rfinish (two: seq parity)
  HostRound* d_hround = nullptr; // its device address
  uint64_t round_seq = 0;
  uint32_t* hist = nullptr;   // 2 x kHistBinsR
  uint64_t *skr = nullptr, *skp = nullptr;  // N / kSample: the threshold histogram's sample
  bool exact_next = false;    // re-run a round whose sampled threshold failed exactly
  int sample_mode = 1;        // DMC_OPT_SAMPLE: 0 exact, 1 sampled, 2 sampled (test: no margin)
  uint32_t* bcount = nullptr;  // kNBR rank-bin counters, 8 bytes each (k_remit's atomics:
                               // records | group sizes << 32)
  unsigned long long* bsup = nullptr;  // kNSup super-bin sums of them (k_remit's blocks)
  BRecR* brec = nullptr;      // kNBR * kBinCapR rank-bin records
  StepRed* red = nullptr;     // step partials (grid) + future record
  StepCtl* sctl = nullptr;
  uint32_t* fut_done = nullptr;   // k_round_future's block ticket counter
  StepCtl* h_sctl = nullptr;  // pinned
  uint64_t* act_min = nullptr;
  // batched activations (k_act_base / k_act_resolve), grown on demand
  uint32_t acap = 0;
  uint64_t *act_cold = nullptr, *act_cnew = nullptr, *act_pre = nullptr,
           *act_suf = nullptr, *act_extra = nullptr, *act_parts = nullptr;
  double* act_p = nullptr;
  uint32_t* act_idx = nullptr;
  ActTiles atl{};              // the segmented resolution's buffers (ensure_act)
  uint64_t* act_xbase = nullptr;
  uint32_t* act_fail = nullptr;
  uint64_t* act_x = nullptr;   // per activation: X_k without the unchanged term
  double *act_ip = nullptr, *act_it = nullptr, *act_ipd = nullptr;
  uint32_t* act_islot = nullptr;
  uint32_t* act_flag = nullptr;  // device-detected activations: position flags
  ActScanPart* act_sparts = nullptr;  // the bookkeeping scans' tile partials
  uint32_t* act_dm = nullptr;    // and their count
  uint32_t* h_actm = nullptr;    // pinned copy of the count
  // AtLimit::Reject's rejected activations that move their client's basis
  // again later in the batch (k_act_hard): per batch position the change
  // events and the activation flags, per activation the sequential
  // resolution's scratch, the any-flag and the count of such batches
  uint32_t *act_hev_q = nullptr, *act_hard = nullptr, *act_hmap = nullptr,
           *act_hlist = nullptr, *act_anyhard = nullptr;
  double *act_hev_p = nullptr, *act_hval = nullptr, *act_hpd = nullptr;
  uint64_t* h_nhard = nullptr;   // (host-mapped: read by dmc_queue_counters)
  uint64_t nhard_base = 0;       // its value at the last counters reset
  uint64_t* act_nhard = nullptr;  // its device pointer
  bool act_pending = false;
  int act_dumps = 0;             // debug: resolve inputs dumped (DMC_DUMP_ACT)
  void* stage = nullptr;         // small host-to-device lists (ensure_stage)
  size_t stage_cap = 0;      // h_act / h_actm hold a batch the idle mirror has not seen
  // dmc_client_mark_idle_batch staging (pinned) and device list
  uint32_t* h_mark = nullptr;
  uint32_t* d_mark = nullptr;
  uint32_t mark_cap = 0;
  hipEvent_t mark_ev = nullptr;
  bool mark_ev_live = false;
  uint32_t* h_act = nullptr;  // pinned staging of the activation positions
  bool act_split = false;     // DMC_OPT_ACT_SPLIT: one host split per activation
  // DMC_OPT_PIPELINE: the gate word (Table::gate) and the call left pending
  bool pipeline = false;
  uint32_t* gate = nullptr;
  uint32_t epoch = 0;  // k_chain_scan's batches (AddParams::epoch)
  uint32_t fused_ndec = 0;  // the pre-launched round's decisions (a group's tallied ones)
  struct PendCall {
    bool on = false;
    uint64_t seq = 0;  // its round's sequence number
    uint32_t k = 0;
    double now = 0.0;
    dmc_decision* out = nullptr;
    dmc_pull_result* res = nullptr;
    bool apply = false;  // its round's k_rapply not launched yet (DMC_DEFER_APPLY)
  } pend;
  unsigned long long* sched = nullptr;  // [0] reservation, [1] priority
  unsigned long long* reqcount = nullptr;
  // radix path (grown on demand)
  uint32_t ecap = 0, dense_hint = 1u << 16;
  DEnt* dense = nullptr;
  uint32_t *sa = nullptr, *sb = nullptr;  // the LSD sort's index buffers
  uint32_t *lcnt = nullptr, *sparts = nullptr;  // its digit counts; scan partials
  uint32_t *gsz = nullptr, *goff = nullptr, *gisp = nullptr, *gpoff = nullptr;
  // add batch buffers
  uint32_t bcap = 0;
  dmc_request* d_reqs = nullptr;
  int32_t* d_rc = nullptr;
  uint32_t *apos = nullptr, *aslot = nullptr;   // per batch request
  uint8_t* d_hev = nullptr;                      // per batch request: heap events (Table::hev)
  uint32_t* abuf = nullptr;  // per client: later filers' batch positions (N * kAddSlots)
  AddParams* apblk = nullptr;
  // decisions (host API)
  uint32_t dcap = 0;
  dmc_decision* d_dec = nullptr;
  uint32_t step_grid = 0;
  uint32_t small_k = 8;  // pulls with k <= small_k run the single-step path
  int fail_allocs = 0;   // DMC_OPT_FAIL_ALLOC (test hook): device allocations to fail
  bool brk_rounds = true;  // DMC_OPT_BREAK_ROUNDS: Allow's limit breaks as rounds
  uint32_t fault = 0;          // DMC_OPT_FAULT (test hook): CallParams::fault of the next round
  bool force_radix = false;    // DMC_OPT_FORCE_RADIX
  bool debug = getenv("DMC_DEBUG") != nullptr;  // per-round diagnostics
  uint32_t* dbg_bins = nullptr;  // debug: bin counts of the last round
  uint64_t* dbg_wtime = nullptr; // debug: per-wave rank start/end clocks
  uint64_t* dbg_atime = nullptr; // debug: per-candidate apply start/end clocks
  uint64_t* dbg_etime = nullptr; // debug: per-block k_remit phase clocks (5 per block)
  uint64_t* dbg_actseq = nullptr; // debug: k_act_seq's clocks and counts (16)
  uint32_t radix_batches = 0;  // rounds left on the fallback path
  uint32_t ovf_streak = 0;     // bin-rank rounds in a row that overflowed (saturates at 5)
  dmc_counters ctr{};          // dmc_queue_counters
  // captured pull rounds / add segments (see launch_round)
  bool use_graphs = true;
  std::vector<GraphRec> graphs = std::vector<GraphRec>(8);
  std::vector<uint64_t> graph_seen = std::vector<uint64_t>(8, 0);
  uint32_t graph_seen_pos = 0;
  uint64_t graph_clock = 0;
  // stage timers (HIP events on the queue's stream), see dmc_profile_*
  bool prof_on = false;
  std::vector<ProfRec> prof_pool;
  size_t prof_n = 0;
  double prof_ms[DMC_PROF_NSTAGES] = {};
  uint64_t prof_cnt[DMC_PROF_NSTAGES] = {};
};

// A queue group (dmc_group_create, dmc_group_step_device below).
struct dmc_group {
  std::vector<dmc_queue*> qs;
  int device = 0;
  hipStream_t stream = nullptr, cap_stream = nullptr;
  // DMC_GROUP_OVERLAP: the scan's branch (eager steps, captures) and the
  // events that fork it from and join it to the step
  hipStream_t stream2 = nullptr, cap_stream2 = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // dmc_group_tracker_collect_sums: the epoch's per-client sums on a stream
  // of their own beside the group's next steps, joined by
  // dmc_group_tracker_join
  hipStream_t side = nullptr;
  hipEvent_t ev_side_in = nullptr, ev_side_out = nullptr;
  bool side_pending = false;
  // per-step kernel arguments: pinned staging and its device copy (one
  // memcpy per step, the graph's first node), S entries per kernel
  uint8_t* h_blob = nullptr;
  uint8_t* d_blob = nullptr;
  size_t bytes = 0, o_trk = 0, o_add = 0, o_scan = 0, o_hist = 0, o_emit = 0, o_rank = 0,
         o_apply = 0, o_tally = 0, tally_bytes = 0;
  struct G {
    uint64_t key = 0;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
  } graphs[4];
  uint64_t seen[4] = {0, 0, 0, 0};
  uint32_t seen_pos = 0, graph_next = 0;
  uint64_t steps = 0, fused_steps = 0, graph_launches = 0;
  // dmc_group_profile_enable: fused steps launched eagerly, each multi-table
  // kernel's execution timed by its own dispatch (hipExtLaunchKernel) -- the
  // kernels the group's timed steps run, per launch over all S tables
  bool prof_on = false;
  struct PRec {
    hipEvent_t a = nullptr, b = nullptr;
    int stage = 0;
  };
  std::vector<PRec> prof_pool;
  size_t prof_n = 0;
  double prof_ms[DMC_PROF_NSTAGES] = {};
  uint64_t prof_cnt[DMC_PROF_NSTAGES] = {};
};

void group_prof_flush(dmc_group* g) {
  if (!g->prof_n) return;
  (void)hipEventSynchronize(g->prof_pool[g->prof_n - 1].b);
  for (size_t i = 0; i < g->prof_n; ++i) {
    float ms = 0.f;
    const dmc_group::PRec& r = g->prof_pool[i];
    if (hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
      g->prof_ms[r.stage] += ms;
      g->prof_cnt[r.stage] += 1;
    }
  }
  g->prof_n = 0;
}

void group_graphs_destroy(dmc_group* g) {
  for (auto& x : g->graphs) {
    if (x.exec) (void)hipGraphExecDestroy(x.exec);
    if (x.graph) (void)hipGraphDestroy(x.graph);
    x = dmc_group::G{};
  }
}

// Every entry point of a queue holds its mutex (the reference's data_mtx) and
// makes the queue's device current for the calling thread, so that servers
// of one rank can be driven from one host thread each.
//
// Stopping k_serve: a stop command, then a bounded wait for the kernel to
// report its exit (it reads the command at its next poll, writes the
// summaries back and exits); only then the stream synchronisation.  A
// kernel that does not exit in time marks the queue wedged (DMC_EDEVICE
// from then on) rather than blocking the caller forever.
constexpr auto kServeStopWait = std::chrono::seconds(1);
int serve_stop(dmc_queue* q) {
  if (!q->serving) return DMC_OK;
  ServeIO* io = q->h_serve;
  {  // the stop command
    const uint64_t seq = ++q->serve_seq;
    io->now = 0.0;
    std::memset((void*)&io->req, 0, sizeof(io->req));
    io->cmd = (uint64_t)kServeStop | (serve_check(seq, kServeStop, 0, 0, 0, 0, 0) << 16);
    __atomic_store_n(&io->req_seq, seq, __ATOMIC_RELEASE);
  }
  const auto t0 = std::chrono::steady_clock::now();
  while (__atomic_load_n(&io->state, __ATOMIC_ACQUIRE) != kServeExited) {
    if (std::chrono::steady_clock::now() - t0 > kServeStopWait) {
      q->wedged = true;
      std::fprintf(stderr, "dmclock_gpu: k_serve did not stop; queue marked failed\n");
      return DMC_EDEVICE;
    }
    __builtin_ia32_pause();
  }
  q->serving = false;
  return hipStreamSynchronize(q->stream) == hipSuccess ? DMC_OK : DMC_EDEVICE;
}

// Stops k_serve before a call that launches other work on the queue's
// stream or changes the table; the summaries are then stale until rebuilt.
int serve_quiesce(dmc_queue* q) {
  q->gsum_valid = false;
  return serve_stop(q);
}

// The process's serving queues (DMC_OPT_SERVE).  A persistent k_serve holds
// its stream's hardware queue; a process has few of them (HIP's
// GPU_MAX_HW_QUEUES, 4 by default) and streams share them round-robin, so
// work queued behind another queue's k_serve waits until that kernel exits
// (idle timeout or lifetime).  Before any call launches work, every other
// serving queue of the device that is not in a call of its own (its mutex is
// free) is stopped -- its summaries stay valid, its next serve call
// relaunches it (a few microseconds) -- so that at most the queues busy in
// other threads hold a hardware queue.  DMCLOCK_SERVE_SHARED=1 turns this
// off (callers that know their streams map to distinct hardware queues).
struct ServeRegistry {
  std::mutex m;
  std::vector<dmc_queue*> qs;
  bool shared = getenv("DMCLOCK_SERVE_SHARED") && std::atoi(getenv("DMCLOCK_SERVE_SHARED"));
};
ServeRegistry& serve_registry() {
  static ServeRegistry r;
  return r;
}
void serve_register(dmc_queue* q, bool on) {
  ServeRegistry& r = serve_registry();
  std::lock_guard<std::mutex> g(r.m);
  auto it = std::find(r.qs.begin(), r.qs.end(), q);
  if (on && it == r.qs.end()) r.qs.push_back(q);
  if (!on && it != r.qs.end()) r.qs.erase(it);
  q->serve_reg = on;
}
void serve_yield_others(dmc_queue* q) {
  ServeRegistry& r = serve_registry();
  if (r.shared) return;
  std::lock_guard<std::mutex> g(r.m);
  for (dmc_queue* o : r.qs) {
    if (o == q || o->p.device != q->p.device) continue;
    if (!__atomic_load_n(&o->serving, __ATOMIC_RELAXED)) continue;
    std::unique_lock<std::mutex> l(o->mtx, std::try_to_lock);
    if (!l.owns_lock()) continue;  // in a call of its own (another thread)
    if (o->serving) {
      ++o->ctr.serve_yields;
      (void)serve_stop(o);  // (its summaries stay valid)
    }
  }
}

// Every C-ABI call holds the queue's lock; all but the serve path's calls
// quiesce k_serve first.  rc: DMC_EDEVICE once the queue is wedged.
namespace {
int settle_pending(dmc_queue* q, bool* clean_out = nullptr);
}  // namespace

// (settle: finish a pipelined call left pending, DMC_OPT_PIPELINE -- every
// entry point but dmc_add_pull_batch_device, which does it after its launch)
struct QueueLock {
  std::lock_guard<std::mutex> l;
  int rc = DMC_OK;
  explicit QueueLock(dmc_queue* q, bool serve = false, bool settle = true) : l(q->mtx) {
    (void)hipSetDevice(q->p.device);
    if (q->wedged) {
      rc = DMC_EDEVICE;
      return;
    }
    if (!serve) rc = serve_quiesce(q);
    if (serve_registry().qs.size() > (q->serve_reg ? 1u : 0u)) serve_yield_others(q);
    if (!rc && settle && q->pend.on && (rc = settle_pending(q))) q->pipe_err = rc;
  }
};

namespace {

const char* kStageNames[DMC_PROF_NSTAGES] = {
    "add_link", "add_chain", "activate", "scan", "select", "emit", "sort",
    "rank", "apply", "step", "future", "cand", "chain_scan", "apply_link"};

// Profiling launches eagerly; a short GPU-side delay queued ahead of a
// profiled call lets the host enqueue all of the call's kernels before the
// first one starts, so that each stage timer brackets GPU time only (kernel
// plus its launch boundary), not the host's per-launch cost.
__global__ void k_prof_gate(uint32_t iters) {
  for (uint32_t i = 0; i < iters; ++i) __builtin_amdgcn_s_sleep(127);
}

void prof_gate(dmc_queue* q) {
  if (q->prof_on)
    hipLaunchKernelGGL(k_prof_gate, dim3(1), dim3(64), 0, q->stream, 50u);  // ~170 us
}

bool prof_slot(dmc_queue* q, int stage) {
  if (!q->prof_on) return false;
  if (q->prof_n == q->prof_pool.size()) {
    ProfRec r;
    // timing-only events: no system-scope fence (no L2 writeback/invalidate
    // between the stages they bracket)
    if (hipEventCreateWithFlags(&r.a, hipEventDisableSystemFence) != hipSuccess ||
        hipEventCreateWithFlags(&r.b, hipEventDisableSystemFence) != hipSuccess) {
      q->prof_on = false;
      return false;
    }
    q->prof_pool.push_back(r);
  }
  q->prof_pool[q->prof_n].stage = stage;
  return true;
}

void pb(dmc_queue* q, int stage) {
  if (prof_slot(q, stage)) (void)hipEventRecord(q->prof_pool[q->prof_n].a, q->stream);
}

// A stage that is one kernel.  Profiling: the kernel's own dispatch records
// the stage's events at its start and end (hipExtLaunchKernel), so the stage
// time is the kernel's execution, as rocprofv3 reports it, without the
// launch gap a pair of stream events around it would add.
template <typename F, typename... Args>
void klaunch(dmc_queue* q, int stage, F kernel, dim3 g, dim3 b, uint32_t sh, Args... args) {
  if (!prof_slot(q, stage)) {
    hipLaunchKernelGGL(kernel, g, b, sh, q->stream, args...);
    return;
  }
  const ProfRec& r = q->prof_pool[q->prof_n];
  hipExtLaunchKernelGGL(kernel, g, b, sh, q->stream, r.a, r.b, 0, args...);
  ++q->prof_n;
}

void pe(dmc_queue* q) {
  if (!q->prof_on) return;
  (void)hipEventRecord(q->prof_pool[q->prof_n].b, q->stream);
  ++q->prof_n;
}

void prof_accumulate(dmc_queue* q, const ProfRec* recs, size_t n) {
  if (!n) return;
  (void)hipEventSynchronize(recs[n - 1].b);
  for (size_t i = 0; i < n; ++i) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, recs[i].a, recs[i].b) == hipSuccess) {
      q->prof_ms[recs[i].stage] += ms;
      q->prof_cnt[recs[i].stage] += 1;
    }
  }
}

// Collect the stage timers of everything enqueued since the last flush.
void pflush(dmc_queue* q) {
  if (!q->prof_on || !q->prof_n) return;
  prof_accumulate(q, q->prof_pool.data(), q->prof_n);
  q->prof_n = 0;
}

int dfree(void* p) {
  if (!p) return DMC_OK;
  const hipError_t e = hipFree(p);
  if (e != hipSuccess) {
    std::fprintf(stderr, "dmclock_gpu: hipFree failed: %s\n", hipGetErrorString(e));
    return DMC_EDEVICE;
  }
  return DMC_OK;
}

int graph_replay(dmc_queue* q, GraphRec& g, void** args, void** args2 = nullptr) {
  ++q->ctr.graph_replays;
  hipGraphExec_t ex = g.flip ? g.exec2 : g.exec;
  g.flip = !g.flip;
  hipKernelNodeParams kp = g.kp;
  kp.kernelParams = args;
  kp.extra = nullptr;
  HIP_OK(hipGraphExecKernelNodeSetParams(ex, g.param_node, &kp));
  if (args2) {
    hipKernelNodeParams kp2 = g.kp2;
    kp2.kernelParams = args2;
    kp2.extra = nullptr;
    HIP_OK(hipGraphExecKernelNodeSetParams(ex, g.param_node2, &kp2));
  }
  HIP_OK(hipGraphLaunch(ex, q->stream));
  return DMC_OK;
}

// Capture `enqueue` (which must start with the parameter kernel) as a graph.
template <typename F>
int graph_capture(dmc_queue* q, GraphRec& g, F enqueue, const void* func2 = nullptr) {
  if (!q->cap_stream)
    HIP_OK(hipStreamCreateWithFlags(&q->cap_stream, hipStreamNonBlocking));
  // (enqueue launches on q->stream: pointed at the capture stream meanwhile)
  hipStream_t exec = q->stream;
  q->stream = q->cap_stream;
  if (hipStreamBeginCapture(q->stream, hipStreamCaptureModeThreadLocal) != hipSuccess) {
    q->stream = exec;
    return DMC_EDEVICE;
  }
  enqueue();
  hipGraph_t graph = nullptr;
  const hipError_t ce = hipStreamEndCapture(q->stream, &graph);
  q->stream = exec;
  if (ce != hipSuccess) {
    std::fprintf(stderr, "dmclock_gpu: hipStreamEndCapture failed: %s\n", hipGetErrorString(ce));
    return DMC_EDEVICE;
  }
  size_t nroot = 0;
  HIP_OK(hipGraphGetRootNodes(graph, nullptr, &nroot));
  if (nroot != 1) {
    (void)hipGraphDestroy(graph);
    return DMC_EDEVICE;
  }
  hipGraphNode_t root;
  HIP_OK(hipGraphGetRootNodes(graph, &root, &nroot));
  hipGraphNodeType ty;
  HIP_OK(hipGraphNodeGetType(root, &ty));
  if (ty != hipGraphNodeTypeKernel) {
    (void)hipGraphDestroy(graph);
    return DMC_EDEVICE;
  }
  HIP_OK(hipGraphKernelNodeGetParams(root, &g.kp));
  if (func2) {  // the second parameter node: the kernel node running func2
    size_t nn = 0;
    HIP_OK(hipGraphGetNodes(graph, nullptr, &nn));
    std::vector<hipGraphNode_t> nodes(nn);
    HIP_OK(hipGraphGetNodes(graph, nodes.data(), &nn));
    for (auto nd : nodes) {
      hipGraphNodeType t2;
      HIP_OK(hipGraphNodeGetType(nd, &t2));
      if (t2 != hipGraphNodeTypeKernel) continue;
      hipKernelNodeParams kp{};
      HIP_OK(hipGraphKernelNodeGetParams(nd, &kp));
      if (kp.func == func2) {
        g.param_node2 = nd;
        g.kp2 = kp;
        break;
      }
    }
    if (!g.param_node2) {
      (void)hipGraphDestroy(graph);
      return DMC_EDEVICE;
    }
  }
  g.graph = graph;
  HIP_OK(hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0));
  HIP_OK(hipGraphInstantiate(&g.exec2, graph, nullptr, nullptr, 0));
  g.param_node = root;
  return DMC_OK;
}

void graph_destroy(GraphRec& g) {
  if (g.exec) (void)hipGraphExecDestroy(g.exec);
  if (g.exec2) (void)hipGraphExecDestroy(g.exec2);
  if (g.graph) (void)hipGraphDestroy(g.graph);
  g = GraphRec{};
}

// Find (or, on the second sighting, build) the graph for `key`; nullptr if the
// caller should launch eagerly this time.
template <typename F>
GraphRec* graph_for(dmc_queue* q, uint64_t key, F enqueue, int* err,
                    const void* func2 = nullptr) {
  // stage timers run eagerly: event-record nodes inside a replayed graph do
  // not bracket the kernels they were captured between
  if (!q->use_graphs || q->prof_on) return nullptr;
  for (auto& g : q->graphs)
    if (g.exec && g.key == key) {
      g.last_use = ++q->graph_clock;
      return &g;
    }
  bool seen = false;
  for (uint64_t k : q->graph_seen) seen |= (k == key);
  if (!seen) {
    q->graph_seen[q->graph_seen_pos++ % q->graph_seen.size()] = key;
    return nullptr;
  }
  GraphRec* slot = &q->graphs[0];
  for (auto& g : q->graphs)
    if (!g.exec || g.last_use < slot->last_use) slot = &g;
  if (slot->exec && hipStreamSynchronize(q->stream) != hipSuccess) {  // (see invalidate_graphs)
    *err = DMC_EDEVICE;
    return nullptr;
  }
  graph_destroy(*slot);
  if (graph_capture(q, *slot, enqueue, func2) != DMC_OK) {
    graph_destroy(*slot);
    q->use_graphs = false;  // capture unsupported: stay eager
    return nullptr;
  }
  slot->key = key;
  slot->last_use = ++q->graph_clock;
  return slot;
}

// Buffers captured into graphs are about to move: drop every graph.  The
// stream drains first: a call returns once its round's summary is published,
// while that round's last kernel may still run (and a graph, its kernel
// arguments or a buffer must not go away under it).
int invalidate_graphs(dmc_queue* q) {
  const hipError_t e = hipStreamSynchronize(q->stream);
  pflush(q);
  for (auto& g : q->graphs) graph_destroy(g);
  if (e != hipSuccess) {
    std::fprintf(stderr, "dmclock_gpu: stream drain failed: %s\n", hipGetErrorString(e));
    return DMC_EDEVICE;
  }
  return DMC_OK;
}

// Device allocation of a queue buffer: DMC_OPT_FAIL_ALLOC (a test hook)
// makes the next n of them fail as an exhausted device would; a failed
// growth leaves the buffer absent (its capacity 0) and the call returns
// DMC_ENOMEM before launching anything that would use it.
int dalloc(dmc_queue* q, void** p, size_t bytes) {
  *p = nullptr;
  if (q->fail_allocs > 0) {
    --q->fail_allocs;
    return DMC_ENOMEM;
  }
  if (hipMalloc(p, bytes) != hipSuccess) {
    *p = nullptr;
    (void)hipGetLastError();  // (not sticky: the queue stays usable)
    return DMC_ENOMEM;
  }
  return DMC_OK;
}
#define DALLOC(q, ptr, bytes)                                         \
  do {                                                                \
    if (int e_ = dalloc((q), reinterpret_cast<void**>(ptr), (bytes))) \
      return e_;                                                      \
  } while (0)

// The radix path's buffers for `n` dense entries (grown on demand): the
// entries, the sort's two index buffers, its per-(digit, tile) counts, the
// scans' tile partials and the group sizes / offsets.
int ensure_entries(dmc_queue* q, uint32_t n) {
  if (n <= q->ecap) return DMC_OK;
  uint32_t cap = std::max<uint32_t>(n, 1u << 16);
  int rc = invalidate_graphs(q);
  for (void** p : {(void**)&q->dense, (void**)&q->sa, (void**)&q->sb, (void**)&q->lcnt,
                   (void**)&q->sparts, (void**)&q->gsz, (void**)&q->goff,
                   (void**)&q->gisp, (void**)&q->gpoff}) {
    if (int e = dfree(*p)) rc = e;
    *p = nullptr;
  }
  q->ecap = 0;
  if (rc) return rc;
  const uint32_t nblk = scan_tiles(cap);
  const uint32_t ncnt = 256u * nblk;
  DALLOC(q, &q->dense, sizeof(DEnt) * cap);
  DALLOC(q, &q->sa, sizeof(uint32_t) * cap);
  DALLOC(q, &q->sb, sizeof(uint32_t) * cap);
  DALLOC(q, &q->lcnt, sizeof(uint32_t) * ncnt);
  DALLOC(q, &q->sparts, sizeof(uint32_t) * scan_tiles(std::max(ncnt, cap)));
  DALLOC(q, &q->gsz, sizeof(uint32_t) * cap);
  DALLOC(q, &q->goff, sizeof(uint32_t) * cap);
  DALLOC(q, &q->gisp, sizeof(uint32_t) * cap);
  DALLOC(q, &q->gpoff, sizeof(uint32_t) * cap);
  q->ecap = cap;
  return DMC_OK;
}

// The rank-bin records (kNBR x kBinCapR x 24 B = 48 MiB per queue), allocated
// by the first bin-ranked round: queues that only ever take single steps or
// the radix path do not pay for them.
int ensure_brec(dmc_queue* q) {
  if (q->brec) return DMC_OK;
  DALLOC(q, &q->brec, sizeof(BRecR) * (size_t)kNBR * kBinCapR);
  return DMC_OK;
}

int ensure_batch(dmc_queue* q, uint32_t n) {
  if (n <= q->bcap) return DMC_OK;
  uint32_t cap = std::max<uint32_t>(n, 1024);
  if (int rc = invalidate_graphs(q)) return rc;
  for (void** p : {(void**)&q->d_reqs, (void**)&q->d_rc, (void**)&q->apos, (void**)&q->aslot,
                   (void**)&q->d_hev}) {
    if (int rc = dfree(*p)) return rc;
    *p = nullptr;
  }
  q->bcap = 0;
  DALLOC(q, &q->d_reqs, sizeof(dmc_request) * cap);
  DALLOC(q, &q->d_rc, sizeof(int32_t) * cap);
  // (padded to whole blocks: k_add_chain loads them before its bounds check)
  DALLOC(q, &q->apos, sizeof(uint32_t) * (cap + kBlock));
  DALLOC(q, &q->aslot, sizeof(uint32_t) * (cap + kBlock));
  DALLOC(q, &q->d_hev, cap);
  q->tb.hev = q->heap ? q->d_hev : nullptr;
  q->bcap = cap;
  return DMC_OK;
}

int ensure_dec(dmc_queue* q, uint32_t n) {
  if (n <= q->dcap) return DMC_OK;
  HIP_OK(hipStreamSynchronize(q->stream));  // (see invalidate_graphs)
  if (int rc = dfree(q->d_dec)) return rc;
  q->d_dec = nullptr;
  q->dcap = 0;
  uint32_t cap = std::max<uint32_t>(n, 1024);
  DALLOC(q, &q->d_dec, sizeof(dmc_decision) * cap);
  q->dcap = cap;
  return DMC_OK;
}

int slot_bits(uint32_t n) {
  int b = 1;
  while (b < 32 && (1u << b) < n) ++b;
  return b;
}

// Add a contiguous run of requests that contains no activation except,
// possibly, its first request (which has already been activated).
// Add a contiguous run of requests that contains no activation except,
// possibly, its first request (which has already been activated).  The two
// kernels are captured once per batch size and replayed with k_add_link's
// arguments updated (see launch_round).
void enqueue_add(dmc_queue* q, const AddParams& ap) {
  prof_gate(q);
  uint32_t g = (ap.n + kBlock - 1) / kBlock;
  klaunch(q, DMC_PROF_ADD_LINK, k_add_link, dim3(g), dim3(kBlock), 0, ap, q->tb,
          q->abuf, q->apos, q->aslot, q->apblk, ActBuf{});
  klaunch(q, DMC_PROF_ADD_CHAIN, k_add_chain, dim3(g), dim3(kBlock), 0, q->tb,
          (const AddParams*)q->apblk, (const uint32_t*)q->abuf,
          (const uint32_t*)q->apos, (const uint32_t*)q->aslot, ActBuf{});
}

int add_segment(dmc_queue* q, const dmc_request* d_reqs, uint32_t n,
                int32_t* d_rc, uint64_t tick_base) {
  if (!n) return DMC_OK;
  AddParams ap{d_reqs, d_rc, tick_base, n, 0};
  uint64_t key = (2ull << 56) | n;
  int err = DMC_OK;
  GraphRec* g = graph_for(q, key, [&] { enqueue_add(q, ap); }, &err);
  if (err) return err;
  if (!g) {
    enqueue_add(q, ap);
    HIP_OK(hipGetLastError());
    return DMC_OK;
  }
  Table tb = q->tb;
  ActBuf noact{};
  void* args[] = {&ap, &tb, &q->abuf, &q->apos, &q->aslot, &q->apblk, &noact};
  return graph_replay(q, *g, args);
}

int activate(dmc_queue* q, uint32_t slot, double t) {
  pb(q, DMC_PROF_ACTIVATE);
  uint32_t g = grid_for(q->tb.n, 2048);
  hipLaunchKernelGGL(k_contrib_min, dim3(g), dim3(kBlock), 0, q->stream, q->tb,
                     q->act_min);
  hipLaunchKernelGGL(k_activate, dim3(1), dim3(kBlock), 0, q->stream, q->tb, slot,
                     t, (const uint64_t*)q->act_min, g);
  pe(q);
  HIP_OK(hipGetLastError());
  return DMC_OK;
}

// Host-ordered add: split the batch at activations (first request of an idle
// client); each activation's idle reset sees the state left by everything
// before it, exactly as the sequential reference does.
int add_host_split(dmc_queue* q, const dmc_request* h_reqs, uint32_t n,
                   const dmc_request* d_reqs, int32_t* d_rc) {
  uint32_t start = 0;
  uint64_t tick0 = q->tick;
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t s = h_reqs[i].slot;
    bool act = s < q->p.max_clients && q->reg_h[s] && q->idle_h[s] &&
               h_reqs[i].rho <= h_reqs[i].delta;
    if (!act) continue;
    int rc = add_segment(q, d_reqs + start, i - start, d_rc + start, tick0 + start);
    if (rc) return rc;
    rc = activate(q, s, h_reqs[i].time);
    if (rc) return rc;
    q->idle_h[s] = 0;
    --q->n_idle;
    start = i;
  }
  return add_segment(q, d_reqs + start, n - start, d_rc + start, tick0 + start);
}

int ensure_act(dmc_queue* q, uint32_t n) {
  if (n <= q->acap) return DMC_OK;
  HIP_OK(hipStreamSynchronize(q->stream));  // (see invalidate_graphs)
  q->acap = 0;
  uint32_t cap = std::max<uint32_t>(n, 4096);
  dfree(q->act_cold); dfree(q->act_cnew); dfree(q->act_pre); dfree(q->act_suf);
  dfree(q->act_p); dfree(q->act_idx); dfree(q->act_x); dfree(q->act_ip);
  dfree(q->act_it); dfree(q->act_ipd); dfree(q->act_islot); dfree(q->act_flag);
  dfree(q->act_sparts);
  dfree(q->act_hev_q); dfree(q->act_hard); dfree(q->act_hmap); dfree(q->act_hlist);
  dfree(q->act_hev_p); dfree(q->act_hval); dfree(q->act_hpd);
  {
    ActTiles& a = q->atl;
    dfree(a.K); dfree(a.nst); dfree(a.sS); dfree(a.sX); dfree(a.sP); dfree(a.sT);
    dfree(a.sPd0); dfree(a.Mtile); dfree(a.Mout); dfree(a.Mj);
    dfree(a.cX); dfree(a.cP); dfree(a.cT); dfree(a.cPd); dfree(a.cMo);
    a = ActTiles{};
  }
  if (q->h_act) (void)hipHostFree(q->h_act);
  q->h_act = nullptr;
  DALLOC(q, &q->act_cold, 8ull * cap);
  DALLOC(q, &q->act_cnew, 8ull * cap);
  DALLOC(q, &q->act_pre, 8ull * cap);
  DALLOC(q, &q->act_suf, 8ull * cap);
  DALLOC(q, &q->act_p, 8ull * cap);
  DALLOC(q, &q->act_idx, 4ull * cap);
  DALLOC(q, &q->act_x, 8ull * cap);
  DALLOC(q, &q->act_ip, 8ull * cap);
  DALLOC(q, &q->act_it, 8ull * cap);
  DALLOC(q, &q->act_ipd, 8ull * cap);
  DALLOC(q, &q->act_islot, 4ull * cap);
  DALLOC(q, &q->act_flag, 4ull * cap);
  DALLOC(q, &q->act_hev_q, 4ull * cap);
  DALLOC(q, &q->act_hard, 4ull * cap);
  DALLOC(q, &q->act_hmap, 4ull * cap);
  DALLOC(q, &q->act_hlist, 4ull * cap);
  DALLOC(q, &q->act_hev_p, 8ull * cap);
  DALLOC(q, &q->act_hval, 8ull * cap);
  DALLOC(q, &q->act_hpd, 8ull * cap);
  HIP_OK(hipHostMalloc((void**)&q->h_act, 4ull * cap, 0));
  // (each one-time buffer guarded by its own pointer: a failed allocation
  // is retried by the next call, never skipped because its pair exists)
  if (!q->act_dm) DALLOC(q, &q->act_dm, 4);
  if (!q->h_actm) HIP_OK(hipHostMalloc((void**)&q->h_actm, 4, 0));
  if (!q->act_anyhard) DALLOC(q, &q->act_anyhard, 4);
  if (!q->h_nhard) {
    HIP_OK(hipHostMalloc((void**)&q->h_nhard, 8, hipHostMallocMapped | hipHostMallocCoherent));
    *q->h_nhard = 0;
    HIP_OK(hipHostGetDevicePointer((void**)&q->act_nhard, q->h_nhard, 0));
  }
  DALLOC(q, &q->act_sparts, sizeof(ActScanPart) * scan_tiles(cap));
  {
    ActTiles& a = q->atl;
    const uint32_t T = (cap + kActTile - 1) / kActTile;
    DALLOC(q, &a.K, 8ull * cap);
    DALLOC(q, &a.nst, 4ull * T);
    DALLOC(q, &a.sS, 8ull * T * kActItems);
    DALLOC(q, &a.sX, 8ull * T * kActItems);
    DALLOC(q, &a.sP, 8ull * T * kActItems);
    DALLOC(q, &a.sT, 8ull * T * kActItems);
    DALLOC(q, &a.sPd0, 8ull * T * kActItems);
    DALLOC(q, &a.Mtile, 8ull * (T + 1));
    DALLOC(q, &a.Mout, 8ull * T * kActItems);
    DALLOC(q, &a.Mj, 8ull * cap);
    DALLOC(q, &a.cX, 8ull * cap);
    DALLOC(q, &a.cP, 8ull * cap);
    DALLOC(q, &a.cT, 8ull * cap);
    DALLOC(q, &a.cPd, 8ull * cap);
    DALLOC(q, &a.cMo, 8ull * cap);
    if (!q->act_xbase) DALLOC(q, &q->act_xbase, 8);
    if (!q->act_fail) {
      DALLOC(q, &q->act_fail, 4);
      HIP_OK(hipMemsetAsync(q->act_fail, 0xff, 4, q->stream));
      HIP_OK(hipStreamSynchronize(q->stream));
    }
    a.xbase = q->act_xbase;
    a.fail = q->act_fail;
  }
  if (!q->act_extra) {
    DALLOC(q, &q->act_extra, 8);
    const uint64_t mx = kMaxKey;
    HIP_OK(hipMemcpyAsync(q->act_extra, &mx, 8, hipMemcpyHostToDevice, q->stream));
    HIP_OK(hipStreamSynchronize(q->stream));
  }
  if (!q->act_parts) DALLOC(q, &q->act_parts, 8ull * 2048);
  q->acap = cap;
  return DMC_OK;
}

// the Reject bookkeeping's buffers (ActBuf::hev_q ...)
void act_hard_bufs(dmc_queue* q, ActBuf& act) {
  act.hev_q = q->act_hev_q;
  act.hev_p = q->act_hev_p;
  act.hard = q->act_hard;
  act.anyhard = q->act_anyhard;
}

// The idle resets of a batch's activations (m of them, at most n: the
// device count act.dm, or act.m), resolved and committed (see k_act_keys)
void act_resolve(dmc_queue* q, const ActBuf& act, uint32_t n) {
  if (!n) return;
  const AddParams* pblk = (const AddParams*)q->apblk;
  const ActHard hs{q->act_hmap, q->act_hlist, q->act_hval, q->act_hpd, q->act_nhard};
  const uint32_t T = (n + kActTile - 1) / kActTile;
  const uint64_t* ax = q->act_x;
  const double *ap = q->act_ip, *at = q->act_it;
  if (T > kActMaxTiles) {
    // (more than 2^20 activations in one batch: the one-block resolution)
    hipLaunchKernelGGL(k_act_inputs, dim3(grid_for(n, 1024)), dim3(kBlock), 0, q->stream, pblk,
                       q->tb, act, q->act_x, q->act_ip, q->act_it, q->act_ipd, q->act_islot);
    hipLaunchKernelGGL(k_act_hard, dim3(1), dim3(64), 0, q->stream, q->tb, act, ax, ap, at,
                       q->act_ipd, (const uint32_t*)q->act_islot, hs);
    hipLaunchKernelGGL(k_act_resolve, dim3(1), dim3(kActThreads), 0, q->stream, q->tb,
                       act, ax, ap, at, q->act_ipd, (const uint32_t*)q->act_islot);
    hipLaunchKernelGGL(k_act_commit, dim3(grid_for(n, 1024)), dim3(kBlock), 0, q->stream,
                       q->tb, (const uint32_t*)act.dm, n, (const double*)q->act_ipd,
                       (const uint32_t*)q->act_islot);
    return;
  }
  hipLaunchKernelGGL(k_act_keys, dim3(T), dim3(kActThreads), 0, q->stream, pblk, q->tb, act,
                     q->act_x, q->act_ip, q->act_it, q->act_ipd, q->act_islot, q->atl);
  if (q->debug && q->dbg_actseq)
    (void)hipMemsetAsync(q->dbg_actseq, 0, 48 * 8, q->stream);
  hipLaunchKernelGGL(k_act_seq, dim3(1), dim3(kActThreads), 0, q->stream, act, q->atl,
                     q->debug ? q->dbg_actseq : nullptr);
  if (q->debug && q->dbg_actseq) {
    uint64_t d[48];
    if (hipMemcpy(d, q->dbg_actseq, sizeof d, hipMemcpyDeviceToHost) == hipSuccess && d[0]) {
      for (int k = 0; k < 12 && d[16 + 2 * k]; ++k)
        std::fprintf(stderr, "act_seq window %d: at %.2f us, from %llu, W %llu, advanced %llu\n",
                     k, (d[16 + 2 * k] - d[2]) / 100.0,
                     (unsigned long long)(d[17 + 2 * k] & 0xffffffffu),
                     (unsigned long long)(d[17 + 2 * k] >> 48),
                     (unsigned long long)((d[17 + 2 * k] >> 32) & 0xffffu));
      std::fprintf(stderr,
                   "act_seq: complex %llu tiles %llu windows %llu wave %llu | offsets %.2f "
                   "gather %.2f chain %.2f end %.2f us\n",
                   (unsigned long long)d[7], (unsigned long long)d[8],
                   (unsigned long long)d[5], (unsigned long long)d[6], (d[1] - d[0]) / 100.0,
                   (d[2] - d[1]) / 100.0, (d[3] - d[2]) / 100.0, (d[4] - d[3]) / 100.0);
    }
  }
  hipLaunchKernelGGL(k_act_apply, dim3(T), dim3(kActThreads), 0, q->stream, q->tb, act, ax,
                     ap, at, (const double*)q->act_ipd, (const uint32_t*)q->act_islot, q->atl);
  hipLaunchKernelGGL(k_act_fixup, dim3(1), dim3(kActThreads), 0, q->stream, q->tb, act, ax,
                     ap, at, q->act_ipd, (const uint32_t*)q->act_islot, q->atl, hs);
}

// the activation bookkeeping's scans (and, flagged, the compaction) of an
// n-position batch: two launches
void act_scans(dmc_queue* q, const ActBuf& act, uint32_t n, bool flagged) {
  const uint32_t nb = scan_tiles(n);
  hipLaunchKernelGGL(k_act_scan_reduce, dim3(nb), dim3(kScT), 0, q->stream, act, n,
                     q->act_sparts);
  hipLaunchKernelGGL(k_act_scan_down, dim3(nb), dim3(kScT), 0, q->stream, act, n,
                     (const ActScanPart*)q->act_sparts, flagged ? q->act_idx : nullptr,
                     flagged ? q->act_dm : nullptr);
}

// A batch with activations in one pass: the host only
// finds the activating requests (to keep its idle mirror); the idle resets
// are resolved on the device by k_act_base + k_add_chain's bookkeeping +
// k_act_resolve, exactly as a sequential replay would compute them.
int add_act_batch(dmc_queue* q, const dmc_request* h_reqs, uint32_t n,
                  const dmc_request* d_reqs, int32_t* d_rc) {
  int rc = ensure_act(q, n);
  if (rc) return rc;
  uint32_t m = 0;
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t s = h_reqs[i].slot;
    if (s < q->p.max_clients && q->reg_h[s] && q->idle_h[s] &&
        h_reqs[i].rho <= h_reqs[i].delta) {
      q->h_act[m++] = i;
      q->idle_h[s] = 0;
      --q->n_idle;
    }
  }
  if (m == 0) return add_segment(q, d_reqs, n, d_rc, q->tick);
  HIP_OK(hipMemcpyAsync(q->act_idx, q->h_act, 4ull * m, hipMemcpyHostToDevice,
                        q->stream));
  prof_gate(q);
  const uint32_t gb = grid_for(q->tb.n, 1024);  // (k_act_base: four records per thread at 1M)
  ActBuf act{q->act_cold, q->act_cnew, q->act_p, q->act_pre, q->act_suf,
             q->act_idx, m, q->act_parts, gb, q->act_extra};
  act_hard_bufs(q, act);
  AddParams ap{d_reqs, d_rc, q->tick, n, 0};
  uint32_t g = (n + kBlock - 1) / kBlock;
  pb(q, DMC_PROF_ADD_LINK);
  hipLaunchKernelGGL(k_add_link, dim3(g), dim3(kBlock), 0, q->stream, ap, q->tb,
                     q->abuf, q->apos, q->aslot, q->apblk, act);
  pe(q);
  ++q->ctr.act_batches;
  pb(q, DMC_PROF_ACTIVATE);
  hipLaunchKernelGGL(k_act_base, dim3(gb), dim3(kBlock), 0, q->stream, q->tb,
                     q->act_parts);
  pe(q);
  pb(q, DMC_PROF_ADD_CHAIN);
  hipLaunchKernelGGL(k_add_chain, dim3(g), dim3(kBlock), 0, q->stream, q->tb,
                     (const AddParams*)q->apblk, (const uint32_t*)q->abuf,
                     (const uint32_t*)q->apos, (const uint32_t*)q->aslot, act);
  pe(q);
  pb(q, DMC_PROF_ACTIVATE);
  act_scans(q, act, n, false);
  act_resolve(q, act, act.m);  // (its first kernel gathers the inputs)
  pe(q);
  HIP_OK(hipGetLastError());
  // the pinned staging is reused by the next batch: wait for the copy
  HIP_OK(hipStreamSynchronize(q->stream));
  return DMC_OK;
}

// The device API's batch with activations: k_add_chain flags the activating
// requests itself, so the requests never travel to the host; the host's idle
// mirror learns the activated slots lazily (settle_act) before anything reads
// it, with no synchronisation between the add and the pulls that follow.
int add_act_batch_dev(dmc_queue* q, uint32_t n, const dmc_request* d_reqs,
                      int32_t* d_rc) {
  int rc = ensure_act(q, n);
  if (rc) return rc;
  prof_gate(q);
  const uint32_t gb = grid_for(q->tb.n, 1024);  // (k_act_base: four records per thread at 1M)
  ActBuf act{q->act_cold, q->act_cnew, q->act_p, q->act_pre, q->act_suf,
             q->act_idx, 0, q->act_parts, gb, q->act_extra, q->act_flag, q->act_dm};
  act_hard_bufs(q, act);
  AddParams ap{d_reqs, d_rc, q->tick, n, 0};
  uint32_t g = (n + kBlock - 1) / kBlock;
  pb(q, DMC_PROF_ADD_LINK);
  hipLaunchKernelGGL(k_add_link, dim3(g), dim3(kBlock), 0, q->stream, ap, q->tb,
                     q->abuf, q->apos, q->aslot, q->apblk, act);
  pe(q);
  ++q->ctr.act_batches;
  pb(q, DMC_PROF_ACTIVATE);
  hipLaunchKernelGGL(k_act_base, dim3(gb), dim3(kBlock), 0, q->stream, q->tb,
                     q->act_parts);
  pe(q);
  pb(q, DMC_PROF_ADD_CHAIN);
  hipLaunchKernelGGL(k_add_chain, dim3(g), dim3(kBlock), 0, q->stream, q->tb,
                     (const AddParams*)q->apblk, (const uint32_t*)q->abuf,
                     (const uint32_t*)q->apos, (const uint32_t*)q->aslot, act);
  pe(q);
  pb(q, DMC_PROF_ACTIVATE);
  act_scans(q, act, n, true);
  const char* dump = q->debug ? getenv("DMC_DUMP_ACT") : nullptr;
  if (dump && q->act_dumps < 4) {
    // debug: the resolve's inputs (tools/act_chain_study.py; k_act_keys
    // gathers them again, the same values)
    hipLaunchKernelGGL(k_act_inputs, dim3(grid_for(n, 1024)), dim3(kBlock), 0, q->stream,
                       (const AddParams*)q->apblk, q->tb, act, q->act_x, q->act_ip,
                       q->act_it, q->act_ipd, q->act_islot);
    HIP_OK(hipStreamSynchronize(q->stream));
    uint32_t m = 0;
    HIP_OK(hipMemcpy(&m, q->act_dm, 4, hipMemcpyDeviceToHost));
    std::vector<uint64_t> parts(gb + 1), ax(m);
    std::vector<double> apv(m), atv(m), apdv(m);
    HIP_OK(hipMemcpy(parts.data(), q->act_parts, 8ull * gb, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(&parts[gb], q->act_extra, 8, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(ax.data(), q->act_x, 8ull * m, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(apv.data(), q->act_ip, 8ull * m, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(atv.data(), q->act_it, 8ull * m, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(apdv.data(), q->act_ipd, 8ull * m, hipMemcpyDeviceToHost));
    uint64_t base = kMaxKey;
    for (uint64_t v : parts) base = v < base ? v : base;
    if (FILE* f = std::fopen(dump, "ab")) {
      std::fwrite(&m, 4, 1, f);
      std::fwrite(&base, 8, 1, f);
      std::fwrite(ax.data(), 8, m, f);
      std::fwrite(apv.data(), 8, m, f);
      std::fwrite(atv.data(), 8, m, f);
      std::fwrite(apdv.data(), 8, m, f);
      std::fclose(f);
    }
    ++q->act_dumps;
  }
  act_resolve(q, act, n);
  pe(q);
  HIP_OK(hipGetLastError());
  // the host idle mirror learns the activated slots (not needed while it is
  // stale anyway: device-side idle marking, sync_idle rebuilds it)
  if (!q->idle_unknown) {
    HIP_OK(hipMemcpyAsync(q->h_actm, q->act_dm, 4, hipMemcpyDeviceToHost, q->stream));
    HIP_OK(hipMemcpyAsync(q->h_act, q->act_islot, 4ull * n, hipMemcpyDeviceToHost,
                          q->stream));
    q->act_pending = true;
  }
  return DMC_OK;
}

// the idle mirror catches up with the last device-detected activations
int settle_act(dmc_queue* q) {
  if (!q->act_pending) return DMC_OK;
  HIP_OK(hipStreamSynchronize(q->stream));
  q->act_pending = false;
  if (q->idle_unknown) return DMC_OK;  // sync_idle rebuilds the mirror
  const uint32_t m = *q->h_actm;
  for (uint32_t k = 0; k < m; ++k) {
    const uint32_t s = q->h_act[k];
    if (q->idle_h[s]) {
      q->idle_h[s] = 0;
      --q->n_idle;
    }
  }
  return DMC_OK;
}

__global__ void k_idle_flags(Table tb, uint8_t* out) {
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < tb.n;
       s += gridDim.x * blockDim.x) {
    const uint8_t f = tb.sc[s].flags;
    out[s] = (f & F_REG) && (f & F_IDLE) ? 1 : 0;
  }
}

// The host idle mirror, rebuilt from the device flags after device-side
// idle marking (one pass over the flags, N bytes back).
int sync_idle(dmc_queue* q) {
  if (!q->idle_unknown) return DMC_OK;
  if (int rc = settle_act(q)) return rc;
  const uint32_t N = q->tb.n;
  uint8_t* d = nullptr;
  HIP_OK(hipMalloc(&d, N));
  hipLaunchKernelGGL(k_idle_flags, dim3(grid_for(N, 2048)), dim3(kBlock), 0, q->stream,
                     q->tb, d);
  HIP_OK(hipMemcpyAsync(q->idle_h.data(), d, N, hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  dfree(d);
  uint32_t n = 0;
  for (uint32_t s = 0; s < N; ++s) n += q->idle_h[s];
  q->n_idle = n;
  q->idle_unknown = false;
  return DMC_OK;
}

// whether an add batch may contain an activation
bool maybe_idle(const dmc_queue* q) { return q->n_idle || q->idle_unknown; }

int add_with_idle(dmc_queue* q, const dmc_request* h_reqs, uint32_t n,
                  const dmc_request* d_reqs, int32_t* d_rc) {
  // (AtLimit::Reject: on the device too.  A rejected request still updates
  // the client's prev tag (update_req_tag precedes the reject check,
  // :899-906, :988-992), so an empty client's contribution can change at
  // every request of the batch -- k_add_chain's bookkeeping records each
  // change; a rejected activation followed by more requests of its client
  // sends the batch to the host split (k_act_reject_check).  A rejected
  // activating request also returns before the heap adjustments (:992 vs
  // :995-1015), which only the heap-order mode models -- DESIGN section 8)
  if (q->act_split) return add_host_split(q, h_reqs, n, d_reqs, d_rc);
  return add_act_batch(q, h_reqs, n, d_reqs, d_rc);
}

// --------------------------------------------------------------- pull rounds
// A pull round takes at most kBinRankMaxK pulls (larger k: several rounds
// at the same `now`): the kNBR x kBinCapR rank bins hold about a million
// entries when balanced, and 2^18 decisions keep them at a quarter of that.
constexpr uint32_t kBinRankMaxK = 1u << 18;
// rounds of at least this many pulls whose rank bins overflow are re-run as
// smaller rounds (pull_impl); smaller ones on the radix path
constexpr uint32_t kSplitMinK = 4096;

uint32_t pow2_at_least(uint32_t x) {
  uint32_t p = 4096;
  while (p < x && p < (1u << 31)) p <<= 1;
  return p;
}

// Terminal pull of a Wait/Reject batch: one general do_next_request, which
// (nothing being eligible) computes min_not_0 over the reservation- and
// limit-heap tops, :1170-1185.  No-op unless the round is terminal.
int launch_future(dmc_queue* q, uint64_t seq) {
  klaunch(q, DMC_PROF_FUTURE, k_round_future, dim3(std::min(q->step_grid, kFutBlocks)),
          dim3(kFutThreads), 0, q->tb, q->red, q->p.at_limit, q->n_registered, q->sctl,
          q->rd, q->d_hround, q->fut_done, seq);
  HIP_OK(hipGetLastError());
  return DMC_OK;
}

// bound infos of distinct slots (dmc_client_bind_info_batch)
__global__ void k_bind_info(BoundInfo* binfo, uint32_t n, const uint32_t* slots,
                            const BoundInfo* v) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) binfo[slots[i]] = v[i];
}

// queue counts of n slots (U1 + delayed: which clients' next add calculates a tag)
__global__ void k_slot_counts(Table tb, uint32_t n, const uint32_t* slots, uint8_t* out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = tb.sc[slots[i]].count;
}

double inv_of(double x) { return x == 0.0 ? 0.0 : 1.0 / x; }  // :115-117

// The queue's persistent device staging for small host-to-device lists
// (bound infos, slot lists), grown on demand.
int ensure_stage(dmc_queue* q, size_t bytes) {
  if (bytes <= q->stage_cap) return DMC_OK;
  HIP_OK(hipStreamSynchronize(q->stream));  // (its last user may still run)
  if (int rc = dfree(q->stage)) return rc;
  q->stage = nullptr;
  q->stage_cap = 0;
  const size_t cap = std::max<size_t>(bytes + (bytes >> 1), 4096);
  DALLOC(q, &q->stage, cap);
  q->stage_cap = cap;
  return DMC_OK;
}

// Publish bound infos (U1): slots whose inverses differ from the host shadow
// are written by one staged kernel (a slot repeated in the batch takes its
// last values); the shadow takes the new values only once the device has
// them, so a failed push is retried by the next bind of the same values.
int bind_infos(dmc_queue* q, uint32_t n, const uint32_t* slots, const double* r,
               const double* w, const double* l) {
  std::vector<uint32_t> ch;
  // the last occurrence of each slot wins
  std::vector<std::pair<uint32_t, uint32_t>> sl(n);
  for (uint32_t i = 0; i < n; ++i) sl[i] = {slots[i], i};
  std::stable_sort(sl.begin(), sl.end(),
                   [](const auto& a, const auto& b) { return a.first < b.first; });
  std::vector<BoundInfo> v;
  for (uint32_t j = 0; j < n; ++j) {
    if (j + 1 < n && sl[j + 1].first == sl[j].first) continue;
    const uint32_t s = sl[j].first, i = sl[j].second;
    const double x[3] = {inv_of(r[i]), inv_of(w[i]), inv_of(l[i])};
    if (std::memcmp(&q->binfo_h[3ull * s], x, sizeof(x)) == 0) continue;
    ch.push_back(s);
    v.push_back(BoundInfo{x[0], x[1], x[2], 0.0});
  }
  if (ch.empty()) return DMC_OK;
  const uint32_t m = (uint32_t)ch.size();
  const size_t sb = (4ull * m + 63) & ~size_t(63);
  if (int rc = ensure_stage(q, sb + sizeof(BoundInfo) * m)) return rc;
  uint32_t* d_s = static_cast<uint32_t*>(q->stage);
  BoundInfo* d_v = reinterpret_cast<BoundInfo*>(static_cast<char*>(q->stage) + sb);
  HIP_OK(hipMemcpyAsync(d_s, ch.data(), 4ull * m, hipMemcpyHostToDevice, q->stream));
  HIP_OK(hipMemcpyAsync(d_v, v.data(), sizeof(BoundInfo) * m, hipMemcpyHostToDevice,
                        q->stream));
  hipLaunchKernelGGL(k_bind_info, dim3((m + kBlock - 1) / kBlock), dim3(kBlock), 0,
                     q->stream, q->binfo, m, (const uint32_t*)d_s, (const BoundInfo*)d_v);
  HIP_OK(hipGetLastError());
  HIP_OK(hipStreamSynchronize(q->stream));
  for (uint32_t j = 0; j < m; ++j) {
    double* h = &q->binfo_h[3ull * ch[j]];
    h[0] = v[j].r_inv;
    h[1] = v[j].w_inv;
    h[2] = v[j].l_inv;
  }
  return DMC_OK;
}

// U1 with a host client_info_f (dmc_queue_set_info_fn): fetch and bind the
// infos of the distinct registered slots among n.  For an add batch
// (adding) in delayed mode, get_cli_info runs only for a client whose queue
// is empty (initial_tag, :878-893): slots with queued requests are skipped
// (their counts read back from the device).  A delayed pop's
// update_next_tag (:1021-1036) always fetches.
int fetch_infos(dmc_queue* q, uint32_t n, const uint32_t* slots, size_t stride,
                bool adding) {
  if (!q->info_fn || !q->tb.binfo || !n) return DMC_OK;
  std::vector<uint32_t> sl;
  sl.reserve(n);
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t s = *reinterpret_cast<const uint32_t*>(
        reinterpret_cast<const char*>(slots) + stride * i);
    if (s < q->p.max_clients && q->reg_h[s]) sl.push_back(s);
  }
  std::sort(sl.begin(), sl.end());
  sl.erase(std::unique(sl.begin(), sl.end()), sl.end());
  if (sl.empty()) return DMC_OK;
  if (adding && q->tb.delayed) {
    const uint32_t m = (uint32_t)sl.size();
    const size_t sb = (4ull * m + 63) & ~size_t(63);
    if (int rc = ensure_stage(q, sb + m)) return rc;
    uint32_t* d_s = static_cast<uint32_t*>(q->stage);
    uint8_t* d_c = static_cast<uint8_t*>(q->stage) + sb;
    std::vector<uint8_t> cnt(m);
    HIP_OK(hipMemcpyAsync(d_s, sl.data(), 4ull * m, hipMemcpyHostToDevice, q->stream));
    hipLaunchKernelGGL(k_slot_counts, dim3((m + kBlock - 1) / kBlock), dim3(kBlock), 0,
                       q->stream, q->tb, m, (const uint32_t*)d_s, d_c);
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpyAsync(cnt.data(), d_c, m, hipMemcpyDeviceToHost, q->stream));
    HIP_OK(hipStreamSynchronize(q->stream));
    size_t o = 0;
    for (uint32_t j = 0; j < m; ++j)
      if (!cnt[j]) sl[o++] = sl[j];
    sl.resize(o);
  }
  std::vector<double> r(sl.size()), w(sl.size()), l(sl.size());
  for (size_t j = 0; j < sl.size(); ++j)
    if (q->info_fn(q->info_ctx, sl[j], &r[j], &w[j], &l[j]) != 0) return DMC_EINVAL;
  return bind_infos(q, (uint32_t)sl.size(), sl.data(), r.data(), w.data(), l.data());
}

// U1 + delayed with a host client_info_f: pulls run one at a time, each
// fetching the dispatched client's info between selection and pop
bool info_steps(const dmc_queue* q) {
  return q->info_fn && q->tb.binfo && q->tb.delayed;
}

// one general pull_request(now); returns the NextReqType in *type
int step_once(dmc_queue* q, double now, dmc_decision* d_out, uint32_t idx,
              int* type, double* when) {
  const Table& tb = q->tb;
  ++q->ctr.single_steps;
  pb(q, DMC_PROF_STEP);
  hipLaunchKernelGGL(k_step_scan, dim3(q->step_grid), dim3(kBlock), 0, q->stream,
                     tb, now, q->red);
  hipLaunchKernelGGL(k_step_decide, dim3(1), dim3(kBlock), 0, q->stream,
                     q->step_grid, (const StepRed*)q->red, now, q->p.at_limit,
                     q->n_registered, q->sctl, (Round*)nullptr, (HostRound*)nullptr);
  if (info_steps(q)) {
    // get_cli_info of the client this pull pops (update_next_tag, :1021-1036)
    HIP_OK(hipMemcpyAsync(q->h_sctl, q->sctl, sizeof(StepCtl), hipMemcpyDeviceToHost,
                          q->stream));
    HIP_OK(hipStreamSynchronize(q->stream));
    if (q->h_sctl->type == DMC_NEXT_RETURNING) {
      const uint32_t s = q->h_sctl->slot;
      if (int rc = fetch_infos(q, 1, &s, sizeof(uint32_t), false)) return rc;
    }
  }
  hipLaunchKernelGGL(k_step_mark, dim3(grid_for(tb.n, 2048)), dim3(kBlock), 0,
                     q->stream, tb, now, (const StepCtl*)q->sctl);
  hipLaunchKernelGGL(k_step_apply, dim3(1), dim3(64), 0, q->stream, tb, q->tick,
                     (const StepCtl*)q->sctl, d_out, idx, q->sched);
  pe(q);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(q->h_sctl, q->sctl, sizeof(StepCtl), hipMemcpyDeviceToHost,
                        q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  pflush(q);
  *type = q->h_sctl->type;
  *when = q->h_sctl->when;
  return DMC_OK;
}

// One pull round (dmc_round.h): scan, histograms, thresholds, emission,
// ranking, apply (+ the terminal pull).  The sequence depends on the
// per-call parameters only through k_rscan's arguments, so it is captured
// once per shape (ranking path, dense capacity, terminal pull) into a hipGraph
// and replayed with k_rscan's arguments updated: one graph launch instead of
// 8-13 kernel launches, which takes the host's per-launch cost off the
// critical path.  A shape is captured the second time it is seen; profiling
// runs eagerly (the stage timers are events between kernels).
// Sampled thresholds (kSample) for tables of at least kSampleMinN slots on
// the bin-rank path, unless the previous round's sample failed validation.
// limit-break rounds: AtLimit::Allow, immediate mode (walk_p's brk groups),
// no host client_info_f between selection and pop (DMC_OPT_BREAK_ROUNDS)
bool brk_ok(const dmc_queue* q) {
  return q->brk_rounds && q->p.at_limit == DMC_AT_LIMIT_ALLOW && !q->tb.delayed &&
         !info_steps(q);
}

bool use_sample(const dmc_queue* q, bool radix) {
  return !radix && q->sample_mode && q->tb.n >= kSampleMinN && !q->exact_next;
}

// (scanned: the scan already ran with that many partials -- k_chain_scan,
// enqueue_add_round_overlap)
void launch_apply(dmc_queue* q);
void enqueue_round(dmc_queue* q, const CallParams& cp, bool radix, uint32_t scanned = 0,
                   bool defer_apply = false) {
  if (!scanned) prof_gate(q);
  const bool sampled = use_sample(q, radix);
  const Table& tb = q->tb;
  uint32_t N = tb.n;
  uint32_t gN = (N + kScanBlock * kScanSlots - 1) / (kScanBlock * kScanSlots);
  // k_remit blocks (kEmitChunk slots each); k_rapply takes kApplyPerEmit per emit block
  const uint32_t gEm = (N + kEmitChunk - 1) / kEmitChunk;
  if (scanned)
    gN = scanned;
  else
    klaunch(q, DMC_PROF_SCAN, cp.brk ? k_rscan_brk : k_rscan, dim3(gN),
            dim3(kScanBlock), 0, tb, sampled ? nullptr : q->keyr, sampled ? nullptr : q->keyp,
            q->meta, q->rparts, q->rd, cp, sampled ? q->skr : nullptr,
            sampled ? q->skp : nullptr, q->k32, q->hist);
  if (sampled)
    klaunch(q, DMC_PROF_SELECT, k_rhist, dim3(kHistBlocksSampled), dim3(1024), 0,
            (N + kSample - 1) / kSample, (const uint64_t*)q->skr, (const uint64_t*)q->skp,
            (const RoundPart*)q->rparts, gN, q->rd, q->hist,
            q->sample_mode == 2 ? 2 : 1, (unsigned long long*)q->bcount, q->bsup);
  else
    klaunch(q, DMC_PROF_SELECT, k_rhist, dim3(kHistBlocksR), dim3(1024), 0, N,
            (const uint64_t*)q->keyr, (const uint64_t*)q->keyp, (const RoundPart*)q->rparts,
            gN, q->rd, q->hist, 0, (unsigned long long*)q->bcount, q->bsup);
  klaunch(q, DMC_PROF_EMIT, cp.brk ? k_remit_brk : k_remit, dim3(gEm),
          dim3(kEmitThreads), 0, tb, q->rd, (const uint2*)q->k32, (const uint32_t*)q->meta, q->cand, q->bcand, q->post,
          q->decof, radix ? nullptr : q->brec, q->bcount, q->bsup, (const uint32_t*)q->hist,
          q->dense, q->ecap, q->debug ? q->dbg_etime : nullptr);
  if (!radix) {
    if (q->debug)  // (the record counts: the rank-bin counters' low words)
      (void)hipMemcpy2DAsync(q->dbg_bins, sizeof(uint32_t), q->bcount, 2 * sizeof(uint32_t),
                             sizeof(uint32_t), kNBR, hipMemcpyDeviceToDevice, q->stream);
    klaunch(q, DMC_PROF_RANK, k_rrank, dim3(kRankBlocksR), dim3(kRankThreads), 0, q->rd,
            (const unsigned long long*)q->bcount, (const unsigned long long*)q->bsup,
            (const BRecR*)q->brec, tb.ring, q->decof, q->debug ? q->dbg_wtime : nullptr);
  } else {
    // the exact LSD sort of the dense entries (dmc_sort.h), then each
    // entry's group size, two exclusive sums and the decisions
    const uint32_t E = q->ecap;
    const uint32_t gE = grid_for(E, 1024);
    const uint32_t nblk = scan_tiles(E);
    pb(q, DMC_PROF_SORT);
    hipLaunchKernelGGL(k_dcheck, dim3(1), dim3(64), 0, q->stream, q->rd, E);
    LsdPass ps[16];
    const int np = lsd_passes(slot_bits(tb.n), ps);
    const uint32_t* src = nullptr;
    for (int i = 0; i < np; ++i) {
      uint32_t* dst = (i & 1) ? q->sb : q->sa;
      hipLaunchKernelGGL(k_lsd_count, dim3(nblk), dim3(kScT), 0, q->stream,
                         (const Round*)q->rd, E, (const DEnt*)q->dense, src, nblk,
                         ps[i].field, ps[i].shift, q->lcnt);
      scan_excl<SumU32>(q->lcnt, q->lcnt, 256u * nblk, q->sparts, q->stream);
      hipLaunchKernelGGL(k_lsd_scatter, dim3(nblk), dim3(kScT), 0, q->stream,
                         (const Round*)q->rd, E, (const DEnt*)q->dense, src, dst, nblk,
                         ps[i].field, ps[i].shift, (const uint32_t*)q->lcnt);
      src = dst;
    }
    pe(q);
    pb(q, DMC_PROF_RANK);
    hipLaunchKernelGGL(k_dsizes, dim3(gE), dim3(kBlock), 0, q->stream,
                       (const Round*)q->rd, E, E, src, (const DEnt*)q->dense, q->gsz,
                       q->gisp);
    scan_excl<SumU32>(q->gsz, q->goff, E, q->sparts, q->stream);
    scan_excl<SumU32>(q->gisp, q->gpoff, E, q->sparts, q->stream);
    hipLaunchKernelGGL(k_ddecide, dim3(gE), dim3(kBlock), 0, q->stream, q->rd, E, src,
                       (const DEnt*)q->dense, (const uint32_t*)q->gsz,
                       (const uint32_t*)q->goff, (const uint32_t*)q->gpoff, tb.ring);
    pe(q);
  }
  // (its last block ends the round: a round that ran out of work under
  // Wait / Reject is followed by the terminal pull, launched by the host)
  if (!defer_apply) launch_apply(q);
}
uint32_t apply_blocks(const dmc_queue* q) {
  return kApplyPerEmit * ((q->tb.n + kEmitChunk - 1) / kEmitChunk) + 1;
}
void launch_apply(dmc_queue* q) {
  klaunch(q, DMC_PROF_APPLY, k_rapply, dim3(apply_blocks(q)), dim3(kBlockR), 0, q->tb, q->rd,
          (const CandRec*)q->cand, (const uint32_t*)q->bcand, (const uint32_t*)q->decof,
          (const PostRec*)q->post, q->sched, q->d_hround,
          q->debug ? q->dbg_atime : nullptr);
}

// A fused call's add + round launched eagerly: the add chain and the scan
// side by side (k_chain_scan: the scan leaves the batch's slots, which the
// chain scans after their adds), then the rest of the round.
constexpr uint32_t kFixPartsMax = 4096;  // (batches of up to 2^20 requests)
#ifndef DMC_DEFER_APPLY
#define DMC_DEFER_APPLY 1
#endif
#ifndef DMC_GROUP_OVERLAP
#define DMC_GROUP_OVERLAP 0  // (1: a queue group's add chain beside its scan, two graph branches)
#endif
#ifndef DMC_GROUP_SCAN_BLOCKS
#define DMC_GROUP_SCAN_BLOCKS 0  // (overlap: the scan's grid per table; 0: one block per 1,024 slots)
#endif
#ifndef DMC_OVERLAP
#define DMC_OVERLAP 1  // (0: the add kernels then k_rscan, for A/B)
#endif
bool overlap_ok(const dmc_queue* q, uint32_t n) {
  return DMC_OVERLAP && !q->use_graphs && (n + kBlock - 1) / kBlock <= kFixPartsMax;
}
// (merge_prev: the previous pipelined call's apply, deferred, runs in this
// call's filing launch, k_apply_link; defer: this call's apply is left to
// the next call's filing launch or to settle_pending)
static_assert(kBlock == kBlockR, "k_apply_link: one block size for both parts");
void enqueue_add_round_overlap(dmc_queue* q, AddParams ap, const CallParams& cp,
                               bool merge_prev = false, bool defer = false) {
  const bool sampled = use_sample(q, false);
  const Table& tb = q->tb;
  ap.epoch = cp.epoch;
  const uint32_t g = (ap.n + kBlock - 1) / kBlock;
  prof_gate(q);
  if (merge_prev) {
    const uint32_t na = apply_blocks(q);
    klaunch(q, DMC_PROF_APPLY_LINK, k_apply_link, dim3(na + g), dim3(kBlockR), 0, tb, q->rd,
            (const CandRec*)q->cand, (const uint32_t*)q->bcand, (const uint32_t*)q->decof,
            (const PostRec*)q->post, q->sched, q->d_hround, na, ap, q->abuf, q->apos,
            q->aslot, q->apblk);
  } else {
    klaunch(q, DMC_PROF_ADD_LINK, k_add_link, dim3(g), dim3(kBlock), 0, ap, tb, q->abuf,
            q->apos, q->aslot, q->apblk, ActBuf{});
  }
  const uint32_t nS = (tb.n + kBlock * kScanChainSlots - 1) / (kBlock * kScanChainSlots);
  klaunch(q, DMC_PROF_CHAIN_SCAN, k_chain_scan, dim3(g + nS), dim3(kBlock), 0, tb,
          ap, (const uint32_t*)q->abuf, (const uint32_t*)q->apos,
          (const uint32_t*)q->aslot, g, nS, sampled ? nullptr : q->keyr,
          sampled ? nullptr : q->keyp, q->meta, q->rparts, q->rd, cp,
          sampled ? q->skr : nullptr, sampled ? q->skp : nullptr, q->k32, q->hist);
  enqueue_round(q, cp, false, nS + g, defer);
}

int launch_round(dmc_queue* q, double now, uint32_t kk, dmc_decision* out,
                 dmc_pull_result* d_result, bool radix, bool brk = false) {
  const bool sampled = use_sample(q, radix);
  CallParams cp{kk, brk ? 1u : 0u, now, out, q->tick, d_result, ++q->round_seq, q->fault, 0};
  uint64_t key = (3ull << 56) | ((uint64_t)q->ecap << 5) | (brk ? 8 : 0) |
                 (sampled ? 4 : 0) | (radix ? 2 : 0);
  int err = DMC_OK;
  GraphRec* g = graph_for(q, key, [&] { enqueue_round(q, cp, radix); }, &err);
  if (err) return err;
  if (!g) {
    enqueue_round(q, cp, radix);
    HIP_OK(hipGetLastError());
    return DMC_OK;
  }
  Table tb = q->tb;
  uint64_t* skr = sampled ? q->skr : nullptr;
  uint64_t* skp = sampled ? q->skp : nullptr;
  uint64_t* kr = sampled ? nullptr : q->keyr;
  uint64_t* kp = sampled ? nullptr : q->keyp;
  void* args[] = {&tb, &kr, &kp, &q->meta, &q->rparts, &q->rd, &cp,
                  &skr, &skp, &q->k32, &q->hist};
  return graph_replay(q, *g, args);
}

// Wait for round `seq`'s summary in host memory (k_rfinish).  Polls; after
// 2 ms (a long round, or a device fault) blocks on the stream instead, which
// reports errors.
int wait_round(dmc_queue* q, uint64_t seq) {
  const HostRound* hr = q->h_round + (seq & 1);
  const volatile uint64_t* flag = &hr->seq;
  auto t0 = std::chrono::steady_clock::now();
  for (uint32_t spin = 1;; ++spin) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) break;
    if ((spin & 255) == 0 &&
        std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
      HIP_OK(hipStreamSynchronize(q->stream));
      if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) return DMC_EDEVICE;
      break;
    }
    __builtin_ia32_pause();
  }
  std::memcpy(q->h_rd, (const void*)&hr->r, sizeof(Round));
  return DMC_OK;
}

// The single-op path: k <= kFastK pulls, each two kernels and one round
// trip, decisions straight to the caller's buffer from host-mapped memory.
bool fast_pull_ok(const dmc_queue* q, uint32_t k) {
  return q->single_op && k <= q->small_k && k <= kFastK && !info_steps(q) && !q->prof_on;
}

int fast_pull(dmc_queue* q, double now, uint32_t k, dmc_decision* out,
              dmc_pull_result* res) {
  dmc_pull_result r{};
  r.next_type = DMC_NEXT_RETURNING;
  uint32_t n = 0;
  const uint32_t gd = std::min(q->step_grid, kFutBlocks);
  const uint32_t ga = grid_for(q->tb.n, 1024);
  while (n < k) {
    if (q->n_registered == 0) {
      r.next_type = DMC_NEXT_NONE;
      break;
    }
    hipLaunchKernelGGL(k_fast_decide, dim3(gd), dim3(kFutThreads), 0, q->stream, q->tb,
                       now, q->red, q->p.at_limit, q->n_registered, q->sctl,
                       &q->d_fast->sc, q->fast_done);
    hipLaunchKernelGGL(k_fast_apply, dim3(ga), dim3(kBlock), 0, q->stream, q->tb, now,
                       q->tick, (const StepCtl*)q->sctl, q->d_fast->dec, n, q->sched);
    HIP_OK(hipGetLastError());
    HIP_OK(hipStreamSynchronize(q->stream));
    ++q->ctr.single_steps;
    const StepCtl c = q->h_fast->sc;  // written before the stream sync
    if (c.type != DMC_NEXT_RETURNING) {
      r.next_type = c.type;
      r.when = c.when;
      break;
    }
    (c.prio ? r.n_priority : r.n_reservation)++;
    ++n;
  }
  if (n) std::memcpy(out, (const void*)q->h_fast->dec, sizeof(dmc_decision) * n);
  r.n_decisions = n;
  if (res) *res = r;
  return DMC_OK;
}

// ------------------------------------------------------------------ serve path
int serve_start(dmc_queue* q, uint64_t seq0) {
  if (!q->gsum_valid) {
    hipLaunchKernelGGL(k_gsum_build, dim3(q->ngroups), dim3(kServeThreads), 0, q->stream,
                       q->tb, q->gsum, q->gshift);
    q->gsum_valid = true;
  }
  __atomic_store_n(&q->h_serve->state, (uint32_t)kServeRunning, __ATOMIC_RELEASE);
  hipLaunchKernelGGL(k_serve, dim3(1), dim3(kServeThreads), 0, q->stream, q->tb, q->gsum,
                     q->ngroups, q->gshift, q->d_serve, q->p.at_limit, q->n_registered,
                     q->sched, seq0, q->serve_idle_ticks, q->tick, q->serve_trace);
  if (hipGetLastError() != hipSuccess) {
    q->gsum_valid = false;
    return DMC_EDEVICE;
  }
  q->serving = true;
  ++q->ctr.serve_launches;
  return DMC_OK;
}

// One command to k_serve (the command fields already written): launch it if
// it is not running, post, and wait for the answer.  A kernel that idled out
// just before the post is relaunched to take the posted command.
int serve_call(dmc_queue* q, uint32_t op, uint32_t k) {
  ServeIO* io = q->h_serve;
  if (q->serving && __atomic_load_n(&io->state, __ATOMIC_ACQUIRE) == kServeExited) {
    HIP_OK(hipStreamSynchronize(q->stream));  // (it idled out or its lifetime ended)
    q->serving = false;
  }
  if (!q->serving) {
    int rc = serve_start(q, q->serve_seq);
    if (rc) return rc;
  }
  const uint64_t seq = ++q->serve_seq;
  uint64_t rw[4];
  std::memcpy(rw, (const void*)&io->req, sizeof(rw));
  const uint64_t opk = (uint64_t)op | ((uint64_t)k << 8);
  io->cmd = opk | (serve_check(seq, opk, __builtin_bit_cast(uint64_t, io->now), rw[0], rw[1],
                               rw[2], rw[3]) << 16);
  __atomic_store_n(&io->req_seq, seq, __ATOMIC_RELEASE);
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t spin = 1;; ++spin) {
    if (__atomic_load_n(&io->done_seq, __ATOMIC_ACQUIRE) == seq) break;
    if ((spin & 255) == 0) {
      if (__atomic_load_n(&io->state, __ATOMIC_ACQUIRE) == kServeExited &&
          __atomic_load_n(&io->done_seq, __ATOMIC_ACQUIRE) != seq) {
        HIP_OK(hipStreamSynchronize(q->stream));
        q->serving = false;
        int rc = serve_start(q, seq - 1);
        if (rc) return rc;
      }
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
        // no answer: a bounded stop (a kernel that does not take it marks
        // the queue wedged); never an unbounded wait on the stream
        q->gsum_valid = false;
        (void)serve_stop(q);
        return DMC_EDEVICE;
      }
    }
    __builtin_ia32_pause();
  }
  ++q->ctr.serve_calls;
  if (q->serve_trace) {
    q->serve_tr[0] += (double)(io->clk[1] - io->clk[0]);
    q->serve_tr[1] += (double)(io->clk[2] - io->clk[1]);
    q->serve_tr[2] += (double)(io->clk[3] - io->clk[2]);
    q->serve_tr[3] += std::chrono::duration<double, std::nano>(
                          std::chrono::steady_clock::now() - t0).count();
    double* ph = q->serve_ph[op == kServePull ? 1 : 0];
    ph[0] += (double)(io->phase[0] - io->clk[1]);
    ph[1] += (double)(io->phase[1] - io->phase[0]);
    ph[2] += (double)(io->phase[2] - (op == kServePull ? io->phase[1] : io->phase[0]));
    ph[3] += 1;
    q->serve_tr[2] += 0;  // (publish stamp unused: the fence is not observable)
    q->serve_mhz += 100.0 * (double)(io->cyc[1] - io->cyc[0]) /
                    (double)std::max<uint64_t>(1, io->clk[2] - io->clk[1]);
  }
  return DMC_OK;
}

bool serve_add_ok(const dmc_queue* q, const dmc_request& r) {
  return q->serve_on && q->single_op && !q->prof_on && !q->act_pending && !q->idle_unknown &&
         !(q->info_fn && q->tb.binfo) && (r.slot >= q->p.max_clients || !q->idle_h[r.slot]);
}

int serve_add(dmc_queue* q, const dmc_request& r, int32_t* rc_out) {
  ServeIO* io = q->h_serve;
  io->now = 0.0;
  io->req = r;
  int rc = serve_call(q, kServeAdd, 0);
  if (rc) return rc;
  q->tick += 1;
  if (rc_out) rc_out[0] = io->rc;
  return DMC_OK;
}

int serve_pull(dmc_queue* q, double now, uint32_t k, dmc_decision* out,
               dmc_pull_result* res) {
  ServeIO* io = q->h_serve;
  io->now = now;
  std::memset((void*)&io->req, 0, sizeof(io->req));
  int rc = serve_call(q, kServePull, k);
  if (rc) return rc;
  dmc_pull_result r{};
  r.n_decisions = io->n;
  r.n_reservation = io->n_res;
  r.n_priority = io->n_prio;
  r.next_type = io->type;
  if (io->type == DMC_NEXT_FUTURE) r.when = io->when;
  q->ctr.single_steps += io->n + (io->type != DMC_NEXT_RETURNING ? 1 : 0);
  if (io->n) std::memcpy(out, (const void*)io->dec, sizeof(dmc_decision) * io->n);
  if (res) *res = r;
  return DMC_OK;
}

// k successive pull_request(now).  Each round is one graph launch and one
// host round trip; a round ends the batch unless the radix path's dense
// buffer overflowed (retry with more capacity), a rank bin overflowed (retry
// on the radix path) or, with AtLimit::Allow, the eligible work ran out (one
// general limit-break step, then another round).  d_result (device API) is
// written by the first round's k_rfinish when that round ends the call;
// *dev_wrote says so.
// (pre_seq: the pre-launched round's sequence number when later rounds were
// launched since -- a pipelined call's, DMC_OPT_PIPELINE)
int pull_impl(dmc_queue* q, double now, uint32_t k, dmc_decision* d_out,
              dmc_pull_result* res, dmc_pull_result* d_result = nullptr,
              bool* dev_wrote = nullptr, bool pre_launched = false, uint64_t pre_seq = 0) {
  if (dev_wrote) *dev_wrote = false;
  bool first_round = true;
  bool retry_radix = false;  // re-run an overflowed round on the radix path
  dmc_pull_result r{};
  r.next_type = DMC_NEXT_RETURNING;
  uint32_t n_dec = 0;
  bool allow = q->p.at_limit == DMC_AT_LIMIT_ALLOW;
  // this call's round size: kBinRankMaxK, lowered after a rank-bin overflow
  uint32_t kcap = kBinRankMaxK;
  // the next round is a limit-break round (AtLimit::Allow, after a round ran
  // out of eligible work: walk_p's brk groups instead of single steps);
  // after one found the state not break-ready, none until a general round
  // has made progress
  bool brk = false, brk_fallback = false;
  while (n_dec < k) {
    if (q->n_registered == 0) {
      r.next_type = DMC_NEXT_NONE;
      break;
    }
    uint32_t kk = k - n_dec;
    if ((kk <= q->small_k || info_steps(q)) && !pre_launched) {
      int type;
      double when;
      int rc = step_once(q, now, d_out, n_dec, &type, &when);
      if (rc) return rc;
      if (type != DMC_NEXT_RETURNING) {
        r.next_type = type;
        r.when = when;
        break;
      }
      ++n_dec;
      (q->h_sctl->prio ? r.n_priority : r.n_reservation)++;
      continue;
    }
    const bool retry = retry_radix;
    retry_radix = false;
    bool radix = q->force_radix || q->radix_batches > 0 || retry;
    // a round takes at most kBinRankMaxK pulls (the rank bins' design
    // size); k beyond that is the next rounds' at the same `now`, exactly
    // the reference's sequence of pulls
    const uint32_t kr = std::min(kk, kcap);
    // the first round of a call may end it: its k_rfinish writes d_result
    dmc_pull_result* dres = (first_round && n_dec == 0 && kr == k) ? d_result : nullptr;
    int rc = DMC_OK;
    uint64_t wseq = 0;
    const bool was_pre = pre_launched;
    if (pre_launched) {  // the fused add + pull graph launched this round
      pre_launched = false;
      radix = false;
      wseq = pre_seq;
    } else {
      if (q->radix_batches && !retry) --q->radix_batches;
      rc = radix ? ensure_entries(q, q->dense_hint) : ensure_brec(q);
      if (rc) return rc;
      rc = launch_round(q, now, kr, d_out + n_dec, dres, radix, brk);
      if (rc) return rc;
    }
    // one host round trip per round, through host-mapped memory
    rc = wait_round(q, wseq ? wseq : q->round_seq);
    if (rc) return rc;
    // (a queue group's fused round tallied its own decisions, k_tally_m
    // skips them; a round that failed wrote none)
    if (was_pre) q->fused_ndec = q->h_rd->overflow ? 0u : q->h_rd->n_dec;
    if (!allow && q->h_rd->terminal && !q->h_rd->overflow) {
      // the round ran out of work: the terminal pull (do_next_request's
      // future / none, :1170-1185) ends it
      rc = launch_future(q, ++q->round_seq);
      if (rc) return rc;
      rc = wait_round(q, q->round_seq);
      if (rc) return rc;
    }
    // (debug readbacks below: k_rapply's other blocks may still run)
    if (q->debug) HIP_OK(hipStreamSynchronize(q->stream));
    pflush(q);
    const Round c = *q->h_rd;
    bool wrote = dres && !c.overflow;
    first_round = false;
    if (q->debug && getenv("DMC_DEBUG_BINS")) {
      std::vector<uint32_t> hb(kNBR);
      (void)hipMemcpy(hb.data(), q->dbg_bins, hb.size() * 4, hipMemcpyDeviceToHost);
      std::vector<uint64_t> wt(2 * kNBR);
      (void)hipMemcpy(wt.data(), q->dbg_wtime, wt.size() * 8, hipMemcpyDeviceToHost);
      std::vector<uint64_t> at(2 * 262144);
      (void)hipMemcpy(at.data(), q->dbg_atime, at.size() * 8, hipMemcpyDeviceToHost);
      FILE* f = std::fopen(getenv("DMC_DEBUG_BINS"), "ab");
      if (f) {
        std::fwrite(hb.data(), 4, hb.size(), f);
        std::fwrite(wt.data(), 8, wt.size(), f);
        std::fwrite(at.data(), 8, at.size(), f);
        std::fwrite(&c.n_cand, 4, 1, f);
        std::fclose(f);
      }
    }
    if (q->debug && getenv("DMC_EMIT_CLOCKS")) {
      const uint32_t nb = (q->tb.n + kEmitChunk - 1) / kEmitChunk;
      std::vector<uint64_t> e((size_t)kEClk * nb + 1);
      (void)hipMemcpy(e.data(), q->dbg_etime, 8ull * e.size(), hipMemcpyDeviceToHost);
      uint64_t t0 = ~0ull;
      for (uint32_t b = 0; b < nb; ++b) t0 = std::min(t0, e[(size_t)kEClk * b]);
      // per phase: median and max over blocks, in us from the first block's start
      for (int ph = 0; ph < kEClk; ++ph) {
        std::vector<double> v(nb);
        for (uint32_t b = 0; b < nb; ++b) v[b] = (e[(size_t)kEClk * b + ph] - t0) / 100.0;
        std::sort(v.begin(), v.end());
        std::fprintf(stderr, "emit clock %d: min %.2f med %.2f max %.2f us\n", ph, v[0],
                     v[nb / 2], v[nb - 1]);
      }
      // per candidate: staging and walk durations
      std::vector<uint64_t> ck(4ull * nb * 512);
      (void)hipMemcpy(ck.data(), q->dbg_etime + 5 * 4096 + 8, 8ull * ck.size(),
                      hipMemcpyDeviceToHost);
      (void)hipMemset(q->dbg_etime + 5 * 4096 + 8, 0, 8ull * ck.size());
      std::vector<double> a, b, st;
      for (size_t i = 0; i < ck.size() / 4; ++i) {
        if (!ck[4 * i]) continue;
        a.push_back((ck[4 * i + 1] - ck[4 * i]) / 100.0);
        b.push_back((ck[4 * i + 2] - ck[4 * i + 1]) / 100.0);
        st.push_back((ck[4 * i] - t0) / 100.0);
      }
      std::sort(a.begin(), a.end());
      std::sort(b.begin(), b.end());
      std::sort(st.begin(), st.end());
      if (!a.empty())
        std::fprintf(stderr, "emit cand (%zu): start p50 %.2f | stage p50 %.2f p90 %.2f | walk+records p50 %.2f p90 %.2f us\n",
                     a.size(), st[st.size() / 2], a[a.size() / 2], a[a.size() * 9 / 10],
                     b[b.size() / 2], b[b.size() * 9 / 10]);
    }
    if (q->debug)
      std::fprintf(stderr,
                   "dmc round: k=%u n_r=%llu p_runs=%u cand=%u R(elig=%u T=%s) "
                   "P(elig=%u) dec=%u prio=%u bins max R %u P %u sumsq %llu "
                   "ovf=%u radix=%d dense=%u pgroups=%u P keys [%.9g, %.9g] T %.9g "
                   "now %.9g fast %u multi %u run %u slow %u\n",
                   kk, (unsigned long long)c.n_r, c.p_runs, c.n_cand,
                   c.ph[0].n_elig, c.ph[0].T == kMaxKey - 1 ? "all" : "thr",
                   c.ph[1].n_elig, c.n_dec, c.n_prio, c.bin_max[0], c.bin_max[1],
                   c.bin_sq, c.overflow, (int)radix, c.dense_n, c.n_pgroups,
                   from_okey(c.ph[1].kmin), from_okey(c.ph[1].kmax),
                   c.ph[1].T ? from_okey(c.ph[1].T) : 0.0, c.now, c.ecnt[0], c.ecnt[1],
                   c.ecnt[2], c.ecnt[3]);
    ++q->ctr.rounds;
    if (radix) ++q->ctr.radix_rounds;
    if (!radix && c.bin_max[0] > q->ctr.max_bin) q->ctr.max_bin = c.bin_max[0];
    if (!radix && c.bin_max[1] > q->ctr.max_bin) q->ctr.max_bin = c.bin_max[1];
#ifdef DMC_TAIL_TIMING
    if (q->debug)
      std::fprintf(stderr, "dmc tails (us): hist body %.2f pick %.2f [reads %.2f scan %.2f thr %.2f rest %.2f] | emit body %.2f prefix %.2f [reads %.2f scan %.2f rest %.2f]\n",
                   (c.tdbg[1] - c.tdbg[0]) / 100.0, (c.tdbg[2] - c.tdbg[1]) / 100.0,
                   (c.tdbg[6] - c.tdbg[1]) / 100.0, (c.tdbg[7] - c.tdbg[6]) / 100.0,
                   (c.tdbg[8] - c.tdbg[7]) / 100.0, (c.tdbg[2] - c.tdbg[8]) / 100.0,
                   (c.tdbg[4] - c.tdbg[3]) / 100.0, (c.tdbg[5] - c.tdbg[4]) / 100.0,
                   (c.tdbg[9] - c.tdbg[4]) / 100.0, (c.tdbg[10] - c.tdbg[9]) / 100.0,
                   (c.tdbg[11] - c.tdbg[10]) / 100.0);
#endif
    if (c.overflow == 1) {  // dense entries: grow and retry
      ++q->ctr.dense_overflows;
      q->dense_hint = pow2_at_least(c.dense_n + (c.dense_n >> 2) + 1);
      // a radix retry of a bin-overflowed round stays a retry: without this
      // the next round would try the bins again, overflow again, and the
      // streak would send the following call to the radix path as well
      retry_radix = retry;
      continue;
    }
    if (c.overflow == 7) {
      // the round failed its outcome check (k_rrank: a phase's selection
      // unset, R-prefix entries not emitted, or fewer decisions than the
      // eligible work allows): nothing of it was applied; an engine fault,
      // reported, never a short dispatch
      ++q->ctr.bad_rounds;
      std::fprintf(stderr, "dmclock_gpu: round %llu failed its outcome check (k=%u)\n",
                   (unsigned long long)c.seq, kr);
      return DMC_EDEVICE;
    }
    if (c.overflow == 5) {
      // a limit-break round found the state not break-ready (a front with
      // r <= now or l <= now, or a weight-0 client's infinite p): nothing of
      // it took effect; general rounds and steps take over
      ++q->ctr.brk_fallbacks;
      brk = false;
      brk_fallback = true;
      continue;
    }
    if (c.overflow == 3) {
      // the sampled threshold admitted too few first keys (k_remit's exact
      // count): this round is re-run with the exact histogram
      ++q->ctr.sample_retries;
      q->exact_next = true;
      continue;
    }
    if (c.overflow == 2) {
      // a rank bin outgrew kBinCapR (the bins are spread by the first keys'
      // histogram; deep queues put more entries near the threshold).  A
      // round of at least kSplitMinK pulls is re-run with fewer, scaled so
      // that the largest bin would hold 3/4 of its capacity (at most half,
      // at least 1/16 of the pulls; the rest are the next rounds' at the
      // same `now`).  Otherwise it is re-run on the radix path: an isolated
      // skewed round costs only that; massively tied keys (radix re-runs in
      // a row) keep the next 1, 2, 4, then 8 calls on it.  The overflowed
      // round's emitted-entry total (dense_n) sizes the radix retry's dense
      // buffer up front.
      ++q->ctr.bin_overflows;
      const uint32_t bmax = std::max(c.bin_max[0], c.bin_max[1]);
      if (kr >= kSplitMinK && bmax > kBinCapR) {
        uint64_t kn = (uint64_t)kr * (kBinCapR * 3 / 4) / bmax;
        kn = std::max<uint64_t>(kn, kr / 16);
        kn = std::min<uint64_t>(kn, kr / 2);
        if (kn >= kSplitMinK / 2) {
          kcap = (uint32_t)kn;
          ++q->ctr.bin_splits;
          continue;
        }
      }
      retry_radix = true;
      q->dense_hint = std::max(q->dense_hint, pow2_at_least(c.dense_n + (c.dense_n >> 2) + 1));
      q->ovf_streak = std::min<uint32_t>(q->ovf_streak + 1, 5);
      if (q->ovf_streak > 1)
        q->radix_batches = std::min<uint32_t>(8, 1u << (q->ovf_streak - 2));
      continue;
    }
    if (!radix) q->ovf_streak = 0;
    q->exact_next = false;
    q->ctr.candidates += c.n_cand;
    q->ctr.entries += radix ? c.dense_n : c.n_emit;
    q->ctr.decisions += c.n_dec;
    if (!brk && c.n_dec) brk_fallback = false;
    n_dec += c.n_dec;
    r.n_priority += c.n_prio;
    r.n_reservation += c.n_dec - c.n_prio;
    if (n_dec >= k) {
      if (dev_wrote) *dev_wrote = wrote;
      break;
    }
    if (!c.terminal) continue;  // a capped round took all kr: the next takes the rest
    if (allow && !brk && !brk_fallback && brk_ok(q)) {
      // the eligible work ran out: the limit breaks (:1157-1165) as rounds
      brk = true;
      ++q->ctr.brk_rounds;
      continue;
    }
    if (allow) {
      int type;
      double when;
      brk = false;
      rc = step_once(q, now, d_out, n_dec, &type, &when);
      if (rc) return rc;
      if (type != DMC_NEXT_RETURNING) {
        r.next_type = type;
        r.when = when;
        break;
      }
      ++n_dec;
      (q->h_sctl->prio ? r.n_priority : r.n_reservation)++;
      continue;
    }
    r.next_type = c.next_type;
    r.when = c.when;
    if (dev_wrote) *dev_wrote = wrote;
    break;
  }
  r.n_decisions = n_dec;
  if (res) *res = r;
  return DMC_OK;
}

// DMC_OPT_PIPELINE: finish the call left pending -- its round's outcome
// read; a round that needs the host (re-runs, the terminal pull, further
// rounds) shut the gate, which is opened again before pull_impl goes on.
// *clean_out: the round ended its call (the gate stayed open, so a graph
// queued behind it ran).
int settle_pending(dmc_queue* q, bool* clean_out) {
  if (clean_out) *clean_out = true;
  if (!q->pend.on) return DMC_OK;
  const dmc_queue::PendCall p = q->pend;
  q->pend.on = false;
  if (p.apply) {  // (its round's apply, deferred and not merged: on its own)
    q->pend.apply = false;
    launch_apply(q);
    HIP_OK(hipGetLastError());
  }
  int rc = wait_round(q, p.seq);
  if (rc) return rc;
  const bool clean = round_ends_call(*q->h_rd);
  if (clean_out) *clean_out = clean;
  if (!clean) HIP_OK(hipMemsetAsync(q->gate, 0, 4, q->stream));
  dmc_pull_result r{};
  bool dev_wrote = false;
  rc = pull_impl(q, p.now, p.k, p.out, &r, p.res, &dev_wrote, true, p.seq);
  if (rc) return rc;
  if (p.res && !dev_wrote) {
    hipLaunchKernelGGL(k_put_result, dim3(1), dim3(1), 0, q->stream, p.res, r);
    HIP_OK(hipGetLastError());
  }
  return DMC_OK;
}

// ------------------------------------------------------------ heap order
// (DMC_OPT_HEAP_ORDER: dmc_heap.h)
int heap_enable(dmc_queue* q, uint32_t k) {
  if (q->n_registered || k < 2 || k > 64) return DMC_EINVAL;
  if (q->heap) return DMC_OK;
  const size_t N = q->p.max_clients;
  DALLOC(q, &q->hd.ent, 3 * sizeof(HEnt) * N);
  DALLOC(q, &q->hd.hix, 3 * 4 * N);
  DALLOC(q, &q->hd.cnt, 4 * 4);
  HIP_OK(hipMemsetAsync(q->hd.cnt, 0, 16, q->stream));
  if (!q->h_hres) HIP_OK(hipHostMalloc((void**)&q->h_hres, sizeof(HeapPullRes), 0));
  DALLOC(q, &q->d_hres, sizeof(HeapPullRes));
  HIP_OK(hipStreamSynchronize(q->stream));
  q->hd.n = (uint32_t)N;
  q->hd.k = k;
  q->heap = true;
  if (int rc = invalidate_graphs(q)) return rc;  // (the captured Table gains hev)
  q->tb.hev = q->d_hev;
  return DMC_OK;
}

// n adds in call order (d_reqs, d_rc device-resident): the batched add path
// (tags, Reject checks, idle resets: the reference's values, resolved in
// parallel) leaves each position's heap calls in tb.hev; k_heap_events then
// makes them in batch order.  (DMC_HEAP_SEQ_ADD: every add and its heap
// calls in order on one wave, k_heap_add -- round 4's form, for A/B.)
#ifndef DMC_HEAP_SEQ_ADD
#define DMC_HEAP_SEQ_ADD 0
#endif
int heap_add(dmc_queue* q, uint32_t n, const dmc_request* d_reqs, int32_t* d_rc) {
  if (!n) return DMC_OK;
  if (DMC_HEAP_SEQ_ADD) {
    AddParams p{d_reqs, d_rc, q->tick, n, 0};
    hipLaunchKernelGGL(k_heap_add, dim3(1), dim3(kHeapThreads), 0, q->stream, q->tb, q->hd, p);
    HIP_OK(hipGetLastError());
    q->tick += n;
    if (q->n_idle) q->idle_unknown = true;  // (activations happened on the device)
    return DMC_OK;
  }
  int rc = ensure_batch(q, n);
  if (!rc) rc = settle_act(q);
  if (rc) return rc;
  rc = maybe_idle(q) ? add_act_batch_dev(q, n, d_reqs, d_rc)
                     : add_segment(q, d_reqs, n, d_rc, q->tick);
  if (rc) return rc;
  hipLaunchKernelGGL(k_heap_events, dim3(1), dim3(64 * kHeapWaves), 0, q->stream, q->tb, q->hd, d_reqs,
                     (const uint8_t*)q->d_hev, n);
  HIP_OK(hipGetLastError());
  q->tick += n;
  return DMC_OK;
}

// k pulls at `now` into d_out; the result (also to d_result when given)
int heap_pull(dmc_queue* q, double now, uint32_t k, dmc_decision* d_out,
              dmc_pull_result* d_result, dmc_pull_result* r) {
  if (info_steps(q)) {
    // U1 + delayed with a host client_info_f: one pull at a time, the
    // popped client's info fetched between its selection and its pop
    dmc_pull_result acc{};
    acc.next_type = DMC_NEXT_RETURNING;
    uint32_t n = 0;
    while (n < k) {
      hipLaunchKernelGGL(k_heap_pull, dim3(1), dim3(64 * kHeapWaves), 0, q->stream, q->tb, q->hd, now, 1u,
                         q->p.at_limit, q->tick, d_out + n, q->d_hres,
                         (dmc_pull_result*)nullptr, q->sched, 1);
      HIP_OK(hipGetLastError());
      HIP_OK(hipMemcpyAsync(q->h_hres, q->d_hres, sizeof(HeapPullRes), hipMemcpyDeviceToHost,
                            q->stream));
      HIP_OK(hipStreamSynchronize(q->stream));
      const HeapPullRes h = *q->h_hres;
      if (h.type != DMC_NEXT_RETURNING) {
        acc.next_type = h.type;
        acc.when = h.type == DMC_NEXT_FUTURE ? h.when : 0.0;
        break;
      }
      const uint32_t s = h.pend_slot;
      if (int rc = fetch_infos(q, 1, &s, sizeof(uint32_t), false)) return rc;
      hipLaunchKernelGGL(k_heap_pull, dim3(1), dim3(64 * kHeapWaves), 0, q->stream, q->tb, q->hd, now, 1u,
                         q->p.at_limit, q->tick, d_out + n, q->d_hres,
                         (dmc_pull_result*)nullptr, q->sched, 2);
      HIP_OK(hipGetLastError());
      ++n;
      (h.pend_prio ? acc.n_priority : acc.n_reservation)++;
    }
    HIP_OK(hipStreamSynchronize(q->stream));
    acc.n_decisions = n;
    q->ctr.decisions += n;
    q->ctr.single_steps += n;
    if (d_result) {
      hipLaunchKernelGGL(k_put_result, dim3(1), dim3(1), 0, q->stream, d_result, acc);
      HIP_OK(hipGetLastError());
    }
    if (r) *r = acc;
    return DMC_OK;
  }
  if (DMC_HEAP_ASYNC && q->hd.k == 2)  // (the heap waves decoupled from the decisions)
    hipLaunchKernelGGL(k_heap_pull_async, dim3(1), dim3(256), 0, q->stream, q->tb, q->hd, now, k,
                       q->p.at_limit, q->tick, d_out, q->d_hres, d_result, q->sched);
  else
    hipLaunchKernelGGL(k_heap_pull, dim3(1), dim3(64 * kHeapWaves), 0, q->stream, q->tb, q->hd, now,
                       k, q->p.at_limit, q->tick, d_out, q->d_hres, d_result, q->sched, 0);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(q->h_hres, q->d_hres, sizeof(HeapPullRes), hipMemcpyDeviceToHost,
                        q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  const HeapPullRes h = *q->h_hres;
  dmc_pull_result x{};
  x.n_decisions = h.n;
  x.next_type = h.type;
  x.when = h.type == DMC_NEXT_FUTURE ? h.when : 0.0;
  x.n_priority = h.n_prio;
  x.n_reservation = h.n_res;
  q->ctr.decisions += h.n;
  q->ctr.single_steps += h.n;
  if (r) *r = x;
  return DMC_OK;
}

// a host list of slots to one of the heap kernels
int heap_list(dmc_queue* q, void (*kern)(Table, HeapDev, const uint32_t*, uint32_t),
              const std::vector<uint32_t>& slots) {
  if (slots.empty()) return DMC_OK;
  uint32_t* d = nullptr;
  HIP_OK(hipMalloc(&d, 4 * slots.size()));
  HIP_OK(hipMemcpyAsync(d, slots.data(), 4 * slots.size(), hipMemcpyHostToDevice, q->stream));
  hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, q->stream, q->tb, q->hd, (const uint32_t*)d,
                     (uint32_t)slots.size());
  const hipError_t e = hipGetLastError();
  HIP_OK(hipStreamSynchronize(q->stream));
  dfree(d);
  return e == hipSuccess ? DMC_OK : DMC_EDEVICE;
}

}  // namespace

// ====================================================================== C-ABI
extern "C" {

const char* dmc_strerror(int code) {
  switch (code) {
    case DMC_OK: return "ok";
    case DMC_EAGAIN: return "rejected at limit (EAGAIN)";
    case DMC_EINVAL: return "invalid argument";
    case DMC_ENOMEM: return "out of device memory";
    case DMC_EDEVICE: return "HIP runtime error";
    case DMC_EBADTAG: return "bad tag (cost 0, or reservation and weight both 0)";
    case DMC_EBADPARAMS: return "bad ReqParams (rho > delta)";
    case DMC_EQUEUEFULL: return "client request ring full";
    case DMC_ENOTREG: return "client slot not registered";
    default: return "unknown error";
  }
}

int dmc_queue_create(const dmc_queue_params* params, dmc_queue** out) {
  if (!params || !out) return DMC_EINVAL;
  const dmc_queue_params& p = *params;
  if (p.max_clients == 0 || p.ring_capacity == 0 || p.ring_capacity > 64 ||
      (p.ring_capacity & (p.ring_capacity - 1)))
    return DMC_EINVAL;
  if (p.at_limit < 0 || p.at_limit > 2) return DMC_EINVAL;
  // AtLimit::Reject depends on ImmediateTagCalc, :856-857
  if (p.at_limit == DMC_AT_LIMIT_REJECT && p.delayed) return DMC_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return DMC_EDEVICE;
  if (p.device < 0 || p.device >= ndev) return DMC_EINVAL;
  HIP_OK(hipSetDevice(p.device));
  dmc_queue* q = new dmc_queue;
  q->p = p;
  HIP_OK(hipStreamCreateWithFlags(&q->stream, hipStreamNonBlocking));
  uint32_t N = p.max_clients;
  Table& t = q->tb;
  t.n = N;
  t.q = p.ring_capacity;
  t.qmask = p.ring_capacity - 1;
  t.delayed = p.delayed;
  t.at_limit = p.at_limit;
  t.reject_thr = p.at_limit == DMC_AT_LIMIT_REJECT ? p.reject_threshold : 0.0;
  t.antic = p.anticipation_timeout;
  auto A = [&](auto** ptr, size_t elems) -> int {
    if (hipMalloc((void**)ptr, elems * sizeof(**ptr)) != hipSuccess) return DMC_ENOMEM;
    return hipMemsetAsync(*ptr, 0, elems * sizeof(**ptr), q->stream) == hipSuccess
               ? DMC_OK : DMC_EDEVICE;
  };
  int rc = 0;
  rc |= A(&t.rec, N); rc |= A(&t.sc, N); rc |= A(&t.aux, N);
  rc |= A(&q->binfo, N);
  t.binfo = p.dynamic_info ? q->binfo : nullptr;
  rc |= A(&t.ring, (size_t)N * p.ring_capacity);
  {
    // (blocks of kEmitChunk slots, or a queue group's kEmitChunkM: room for either)
    const size_t nb = (N + kEmitChunk - 1) / kEmitChunk;
    const size_t nbm = (N + kEmitChunkM - 1) / kEmitChunkM;
    const size_t nc = std::max(nb * kEmitChunk, nbm * kEmitChunkM);
    rc |= A(&q->cand, nc);
    rc |= A(&q->bcand, nb);
    rc |= A(&q->post, nc);
    rc |= A(&q->decof, nc);
  }
  rc |= A(&q->keyr, N);
  rc |= A(&q->keyp, N);
  rc |= A(&q->k32, N);
  rc |= A(&q->meta, N);
  rc |= A(&q->hist, (kShards + 1) * 2 * kHistBinsR);  // (+ the pre-picked rank-bin tables)
  rc |= A(&q->skr, (N + kSample - 1) / kSample);
  rc |= A(&q->skp, (N + kSample - 1) / kSample);
  q->step_grid = grid_for(N, 1024);
  rc |= A(&q->red, q->step_grid + 1);
  rc |= A(&q->sctl, 1);
  rc |= A(&q->fut_done, 1);
  rc |= A(&q->rd, 1);
  // (k_rscan's partials, or k_chain_scan's: its scan's and its chain's)
  rc |= A(&q->rparts, (N + kBlock - 1) / kBlock + kFixPartsMax);
  rc |= A(&q->bcount, 2 * kNBR);  // 8-byte counters: records | group sizes << 32
  rc |= A(&q->bsup, kNSup);
  if (q->debug) rc |= A(&q->dbg_bins, kNBR);
  if (q->debug) rc |= A(&q->dbg_wtime, 2 * kNBR);
  if (q->debug) rc |= A(&q->dbg_atime, 2 * 262144);
  if (q->debug) rc |= A(&q->dbg_etime, 5 * 4096 + 8 + 4 * 4096 * 512);
  if (q->debug) rc |= A(&q->dbg_actseq, 48);
  // q->brec (kNBR x kBinCapR rank-bin records, 48 MiB) is allocated by the
  // first bin-ranked round (ensure_brec)
  rc |= A(&q->act_min, 2048);  // per-block minima of the activation scan
  rc |= A(&q->abuf, (size_t)N * kAddSlots);
  rc |= A(&q->apblk, 1);
  rc |= A(&q->sched, 2);
  rc |= A(&q->fast_done, 2);
  while (((uint64_t)N + (1ull << q->gshift) - 1) >> q->gshift > kServeMaxG) ++q->gshift;
  q->ngroups = (uint32_t)(((uint64_t)N + (1ull << q->gshift) - 1) >> q->gshift);
  rc |= A(&q->gsum, q->ngroups);
  {
    int khz = 0;  // the wall clock k_serve's idle limit counts
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, p.device) == hipSuccess &&
        khz > 0)
      q->serve_idle_ticks = (uint64_t)khz / 5;  // 0.2 ms
  }
  rc |= A(&q->reqcount, 1);
  t.gate = nullptr;
  rc |= A(&t.touch, N);
  rc |= A(&q->gate, 1);
  if (hipHostMalloc((void**)&q->h_round, 2 * sizeof(HostRound),
                    hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void**)&q->d_hround, q->h_round, 0) != hipSuccess ||
      hipHostMalloc((void**)&q->h_sctl, sizeof(StepCtl), 0) != hipSuccess ||
      hipHostMalloc((void**)&q->h_fast, sizeof(FastIO),
                    hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void**)&q->d_fast, q->h_fast, 0) != hipSuccess ||
      hipHostMalloc((void**)&q->h_serve, sizeof(ServeIO),
                    hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void**)&q->d_serve, q->h_serve, 0) != hipSuccess)
    rc |= DMC_ENOMEM;
  else {
    std::memset((void*)q->h_round, 0, 2 * sizeof(HostRound));
    std::memset((void*)q->h_serve, 0, sizeof(ServeIO));
  }
  if (rc) {
    dmc_queue_destroy(q);
    return DMC_ENOMEM;
  }
  if (ensure_entries(q, 1u << 16) ||
      ensure_batch(q, std::max<uint32_t>(p.max_batch, 1024)) ||
      ensure_dec(q, std::max<uint32_t>(p.max_batch, 1024))) {
    dmc_queue_destroy(q);
    return DMC_ENOMEM;
  }
  q->reg_h.assign(N, 0);
  q->idle_h.assign(N, 0);
  q->binfo_h.assign(3ull * N, 0.0);
  if (hipStreamSynchronize(q->stream) != hipSuccess) {
    dmc_queue_destroy(q);
    return DMC_EDEVICE;
  }
  *out = q;
  return DMC_OK;
}

int dmc_queue_destroy(dmc_queue* q) {
  if (!q) return DMC_EINVAL;
  (void)hipSetDevice(q->p.device);
  if (q->pend.on) (void)settle_pending(q);  // (DMC_OPT_PIPELINE: its work completes)
  if (q->group) {  // (the group keeps running its other members)
    dmc_group* g = q->group;
    (void)hipStreamSynchronize(q->stream);
    g->qs.erase(std::find(g->qs.begin(), g->qs.end(), q));
    group_graphs_destroy(g);
    q->stream = q->own_stream;
    q->group = nullptr;
  }
  if (q->serve_reg) serve_register(q, false);
  if (q->h_serve && !q->wedged) (void)serve_quiesce(q);
  if (q->serve_trace && q->ctr.serve_calls) {
    const double c = (double)q->ctr.serve_calls;
    std::fprintf(stderr, "dmc serve: %llu calls, %llu launches; per call: read %.0f, work %.0f, "
                 "publish %.0f wall-clock ticks; host %.0f ns\n",
                 (unsigned long long)q->ctr.serve_calls,
                 (unsigned long long)q->ctr.serve_launches, q->serve_tr[0] / c,
                 q->serve_tr[1] / c, q->serve_tr[2] / c, q->serve_tr[3] / c);
    std::fprintf(stderr, "dmc serve: shader clock %.0f MHz while answering\n",
                 q->serve_mhz / c);
    for (int o = 0; o < 2; ++o)
      if (q->serve_ph[o][3] > 0)
        std::fprintf(stderr, "dmc serve %s: first phase %.0f, pop %.0f, summary %.0f ticks\n",
                     o ? "pull" : "add", q->serve_ph[o][0] / q->serve_ph[o][3],
                     q->serve_ph[o][1] / q->serve_ph[o][3], q->serve_ph[o][2] / q->serve_ph[o][3]);
  }
  if (q->stream) (void)hipStreamSynchronize(q->stream);
  invalidate_graphs(q);
  Table& t = q->tb;
  void* ptrs[] = {t.rec, t.sc, t.aux, q->binfo,
                  t.ring,
                  q->cand, q->bcand, q->post, q->decof, q->keyr, q->keyp, q->k32, q->meta, q->hist,
                  q->skr, q->skp, q->red, q->sctl, q->fut_done, q->rd, q->rparts, q->bcount, q->bsup, q->dbg_bins, q->dbg_wtime, q->dbg_atime,
                  q->brec, q->act_min, q->sched, q->reqcount, q->dense, q->sa,
                  q->sb, q->lcnt, q->sparts, q->gsz, q->goff, q->gisp, q->gpoff,
                  q->d_reqs, q->d_rc, q->apos, q->aslot, q->abuf, q->d_hev,
                  q->apblk, q->d_dec, q->stage};
  for (void* p : ptrs)
    dfree(p);
  if (q->h_round) (void)hipHostFree(q->h_round);
  dfree(q->gate);
  dfree(q->tb.touch);
  if (q->h_act) (void)hipHostFree(q->h_act);
  dfree(q->act_cold); dfree(q->act_cnew); dfree(q->act_pre); dfree(q->act_suf);
  dfree(q->act_p); dfree(q->act_idx); dfree(q->act_extra); dfree(q->act_parts);
  dfree(q->act_x); dfree(q->act_ip); dfree(q->act_it); dfree(q->act_ipd); dfree(q->act_islot);
  dfree(q->act_flag); dfree(q->act_dm);
  dfree(q->atl.K); dfree(q->atl.nst); dfree(q->atl.sS); dfree(q->atl.sX); dfree(q->atl.sP);
  dfree(q->atl.sT); dfree(q->atl.sPd0); dfree(q->atl.Mtile); dfree(q->atl.Mout);
  dfree(q->atl.Mj); dfree(q->atl.cX); dfree(q->atl.cP); dfree(q->atl.cT); dfree(q->atl.cPd);
  dfree(q->atl.cMo);
  dfree(q->act_xbase); dfree(q->act_fail);
  dfree(q->act_hev_q); dfree(q->act_hard); dfree(q->act_hmap); dfree(q->act_hlist);
  dfree(q->act_anyhard); dfree(q->act_hev_p); dfree(q->act_hval); dfree(q->act_hpd);
  if (q->h_nhard) (void)hipHostFree(q->h_nhard);
  dfree(q->hd.ent); dfree(q->hd.hix); dfree(q->hd.cnt); dfree(q->d_hres);
  if (q->h_hres) (void)hipHostFree(q->h_hres);
  if (q->h_actm) (void)hipHostFree(q->h_actm);
  dfree(q->d_mark);
  if (q->h_mark) (void)hipHostFree(q->h_mark);
  if (q->mark_ev) (void)hipEventDestroy(q->mark_ev);
  if (q->h_sctl) (void)hipHostFree(q->h_sctl);
  if (q->h_fast) (void)hipHostFree(q->h_fast);
  dfree(q->fast_done);
  if (q->h_serve) (void)hipHostFree(q->h_serve);
  dfree(q->gsum);
  for (auto& r : q->prof_pool) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  if (q->stream) (void)hipStreamDestroy(q->stream);
  if (q->cap_stream) (void)hipStreamDestroy(q->cap_stream);
  delete q;
  return DMC_OK;
}

void* dmc_queue_stream(dmc_queue* q) {
  if (!q) return nullptr;
  QueueLock g(q);  // (work the caller queues on it must not wait behind k_serve)
  return (void*)q->stream;
}

int dmc_queue_sync(dmc_queue* q) {
  if (!q) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  HIP_OK(hipStreamSynchronize(q->stream));
  return DMC_OK;
}

int dmc_client_register_batch(dmc_queue* q, uint32_t n, const uint32_t* slots,
                              const double* r, const double* w, const double* l,
                              int active) {
  if (!q || (n && (!slots || !r || !w || !l))) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  ++q->gen;
  if (int rc0 = settle_act(q)) return rc0;
  if (int rc0 = sync_idle(q)) return rc0;
  for (uint32_t i = 0; i < n; ++i)
    if (slots[i] >= q->p.max_clients) return DMC_EINVAL;
  if (!n) return DMC_OK;
  if (q->heap) {  // heap order: new, distinct clients only (client_map.emplace)
    std::vector<uint32_t> v(slots, slots + n);
    std::sort(v.begin(), v.end());
    if (std::adjacent_find(v.begin(), v.end()) != v.end()) return DMC_EINVAL;
    for (uint32_t i = 0; i < n; ++i)
      if (q->reg_h[slots[i]]) return DMC_EINVAL;
  }
  std::vector<double> ri(n), wi(n), li(n);
  for (uint32_t i = 0; i < n; ++i) {
    ri[i] = inv_of(r[i]);
    wi[i] = inv_of(w[i]);
    li[i] = inv_of(l[i]);
  }
  uint32_t* d_slots;
  double *d_r, *d_w, *d_l;
  HIP_OK(hipMalloc(&d_slots, 4ull * n));
  HIP_OK(hipMalloc(&d_r, 8ull * n));
  HIP_OK(hipMalloc(&d_w, 8ull * n));
  HIP_OK(hipMalloc(&d_l, 8ull * n));
  HIP_OK(hipMemcpyAsync(d_slots, slots, 4ull * n, hipMemcpyHostToDevice, q->stream));
  HIP_OK(hipMemcpyAsync(d_r, ri.data(), 8ull * n, hipMemcpyHostToDevice, q->stream));
  HIP_OK(hipMemcpyAsync(d_w, wi.data(), 8ull * n, hipMemcpyHostToDevice, q->stream));
  HIP_OK(hipMemcpyAsync(d_l, li.data(), 8ull * n, hipMemcpyHostToDevice, q->stream));
  hipLaunchKernelGGL(k_register, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0,
                     q->stream, q->tb, q->binfo, n, d_slots, d_r, d_w, d_l, active, q->tick);
  if (q->heap) {  // three pushes per client, in the given order (:925-931)
    hipLaunchKernelGGL(k_heap_push, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, q->stream,
                       q->tb, q->hd, (const uint32_t*)d_slots, n);
    hipLaunchKernelGGL(k_heap_count_add, dim3(1), dim3(64), 0, q->stream, q->hd, n);
  }
  HIP_OK(hipStreamSynchronize(q->stream));
  dfree(d_slots); dfree(d_r); dfree(d_w); dfree(d_l);
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t s = slots[i];
    q->binfo_h[3ull * s] = ri[i];
    q->binfo_h[3ull * s + 1] = wi[i];
    q->binfo_h[3ull * s + 2] = li[i];
    if (!q->reg_h[s]) ++q->n_registered;
    if (q->idle_h[s]) --q->n_idle;
    q->reg_h[s] = 1;
    q->idle_h[s] = active ? 0 : 1;
    if (!active) ++q->n_idle;
  }
  return DMC_OK;
}

int dmc_client_register(dmc_queue* q, uint32_t slot, double r, double w,
                        double l, int active) {
  return dmc_client_register_batch(q, 1, &slot, &r, &w, &l, active);
}

int dmc_client_update_info(dmc_queue* q, uint32_t slot, double r, double w,
                           double l) {
  if (!q || slot >= q->p.max_clients) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  if (!q->reg_h[slot]) return DMC_ENOTREG;
  double v[3] = {inv_of(r), inv_of(w), inv_of(l)};
  // r_inv, w_inv, l_inv are contiguous in ClientRec and in BoundInfo
  HIP_OK(hipMemcpyAsync(&q->tb.rec[slot].r_inv, v, sizeof(v), hipMemcpyHostToDevice,
                        q->stream));
  HIP_OK(hipMemcpyAsync(&q->binfo[slot].r_inv, v, sizeof(v), hipMemcpyHostToDevice,
                        q->stream));
  std::memcpy(&q->binfo_h[3ull * slot], v, sizeof(v));
  HIP_OK(hipStreamSynchronize(q->stream));
  return DMC_OK;
}

int dmc_client_bind_info_batch(dmc_queue* q, uint32_t n, const uint32_t* slots,
                               const double* r, const double* w, const double* l) {
  if (!q || (n && (!slots || !r || !w || !l))) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  for (uint32_t i = 0; i < n; ++i)
    if (slots[i] >= q->p.max_clients) return DMC_EINVAL;
  return bind_infos(q, n, slots, r, w, l);
}

int dmc_queue_set_info_fn(dmc_queue* q, dmc_info_fn fn, void* ctx) {
  if (!q) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  q->info_fn = fn;
  q->info_ctx = ctx;
  return DMC_OK;
}

int dmc_client_mark_idle(dmc_queue* q, uint32_t slot) {
  if (!q || slot >= q->p.max_clients) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  if (int rc0 = settle_act(q)) return rc0;
  if (int rc0 = sync_idle(q)) return rc0;
  if (!q->reg_h[slot]) return DMC_ENOTREG;
  uint8_t f;
  HIP_OK(hipMemcpyAsync(&f, &q->tb.sc[slot].flags, 1, hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  f |= F_IDLE;
  HIP_OK(hipMemcpyAsync(&q->tb.sc[slot].flags, &f, 1, hipMemcpyHostToDevice, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  if (!q->idle_h[slot]) {
    q->idle_h[slot] = 1;
    ++q->n_idle;
  }
  return DMC_OK;
}

__global__ void k_mark_idle(Table tb, uint32_t n, const uint32_t* slots) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) tb.sc[slots[i]].flags |= F_IDLE;
}

int dmc_client_mark_idle_batch(dmc_queue* q, uint32_t n, const uint32_t* slots) {
  if (!q || (n && !slots)) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  if (int rc0 = settle_act(q)) return rc0;
  if (int rc0 = sync_idle(q)) return rc0;
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t s = slots[i];
    if (s >= q->p.max_clients) return DMC_EINVAL;
    if (!q->reg_h[s]) return DMC_ENOTREG;
  }
  // pinned staging and a device list kept across calls; the previous
  // call's copy must have left the staging before it is rewritten
  if (q->mark_ev_live) {
    HIP_OK(hipEventSynchronize(q->mark_ev));
    q->mark_ev_live = false;
  }
  if (n > q->mark_cap) {
    HIP_OK(hipStreamSynchronize(q->stream));  // (see invalidate_graphs)
    if (q->h_mark) (void)hipHostFree(q->h_mark);
    dfree(q->d_mark);
    q->h_mark = nullptr;
    q->d_mark = nullptr;
    q->mark_cap = 0;
    const uint32_t cap = std::max<uint32_t>(n, 4096);
    HIP_OK(hipHostMalloc((void**)&q->h_mark, 4ull * cap, 0));
    DALLOC(q, &q->d_mark, 4ull * cap);
    q->mark_cap = cap;
  }
  if (!q->mark_ev) HIP_OK(hipEventCreateWithFlags(&q->mark_ev, hipEventDisableTiming));
  uint32_t m = 0;
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t s = slots[i];
    if (!q->idle_h[s]) {
      q->idle_h[s] = 1;
      ++q->n_idle;
      q->h_mark[m++] = s;
    }
  }
  if (m == 0) return DMC_OK;
  HIP_OK(hipMemcpyAsync(q->d_mark, q->h_mark, 4ull * m, hipMemcpyHostToDevice,
                        q->stream));
  hipLaunchKernelGGL(k_mark_idle, dim3((m + kBlock - 1) / kBlock), dim3(kBlock), 0,
                     q->stream, q->tb, m, (const uint32_t*)q->d_mark);
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(q->mark_ev, q->stream));
  q->mark_ev_live = true;
  return DMC_OK;
}

// ------------------------------------------------------------------ maintenance
// Whole-queue maintenance in a fixed number of device passes: one slot list
// (null: every slot), queued counts, their exclusive scan, then one pass that
// gathers the handles, filters, or clears.  One thread per listed slot; a
// slot's ring is walked in FIFO order.
__device__ inline uint32_t list_slot(const uint32_t* slots, uint32_t i) {
  return slots ? slots[i] : i;
}

__global__ void k_list_counts(Table tb, uint32_t n, const uint32_t* slots,
                              uint32_t* counts) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) counts[i] = tb.sc[list_slot(slots, i)].count;
}

__global__ void k_list_gather(Table tb, uint32_t n, const uint32_t* slots,
                              const uint32_t* offs, uint64_t* handles) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t s = list_slot(slots, i);
  const ScanRec sr = tb.sc[s];
  const ReqEntry* ring = tb.ring + (size_t)s * tb.q;
  uint64_t* out = handles + offs[i];
  for (uint32_t j = 0; j < sr.count; ++j) out[j] = ring[(sr.head + j) & tb.qmask].handle;
}

// ClientRec::remove_by_req_filter's erase (:440-480): the kept requests keep
// their order and tags (a removed delayed-mode front leaves the next
// request's stored tag as the front tag, as the reference's deque does); the
// front's ready flag survives only with the front; the heap keys follow the
// new front.  *any != 0 if anything was removed.
// one client's compaction (kp: its keep flags, FIFO order); false: nothing removed
__device__ inline bool list_filter_slot(const Table& tb, uint32_t s, const uint8_t* kp) {
  const ScanRec sr = tb.sc[s];
  uint32_t c = sr.count, m = 0;
  for (uint32_t j = 0; j < c; ++j) m += kp[j] != 0;
  if (m == c) return false;
  ReqEntry* ring = tb.ring + (size_t)s * tb.q;
  uint32_t w = 0;
  for (uint32_t j = 0; j < c; ++j) {
    if (!kp[j]) continue;
    if (w != j) ring[(sr.head + w) & tb.qmask] = ring[(sr.head + j) & tb.qmask];
    ++w;
  }
  const uint8_t fl = (!kp[0] || m == 0) ? (uint8_t)(sr.flags & ~F_READY) : sr.flags;
  ScanRec o{0.0, 0.0, 0.0, sr.head, (uint8_t)m, fl, sr.stamp, sr.nadd};
  if (m) {
    const ReqEntry& f = ring[sr.head & tb.qmask];
    o.r = f.r;
    o.pk = __dadd_rn(f.p, tb.rec[s].pd);
    o.l = f.l;
  }
  tb.sc[s] = o;
  return true;
}

__global__ void k_list_filter(Table tb, uint32_t n, const uint32_t* slots,
                              const uint32_t* offs, const uint8_t* keep,
                              uint32_t* any) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (list_filter_slot(tb, list_slot(slots, i), keep + offs[i])) atomicOr(any, 1u);
}

// heap order (dmc_heap.h): remove_by_req_filter's loop (:567-585) in client
// order -- each modified client filtered, then adjusted in the three heaps,
// before the next one is filtered (a later client's adjust must see the
// earlier clients' new fronts and the later ones' old ones)
__global__ void __launch_bounds__(64) k_heap_filter(Table tb, HeapDev hd, uint32_t n,
                                                    const uint32_t* slots, const uint32_t* offs,
                                                    const uint8_t* keep) {
  __shared__ HEnt cache[3 * kHeapLds];
  const uint32_t T = heap_cache_fill(hd, cache);
  WHeaps W(tb, hd, cache, T);
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t s = slots[i];
    uint32_t mod = 0;
    if (W.lane == 0) mod = list_filter_slot(tb, s, keep + offs[s]) ? 1u : 0u;
    wave_sync();
    if (uread(mod, 0)) W.adjust3(s);
  }
  heap_cache_flush(hd, cache, T);
}

// do_clean's erase (:1244-1255) of the listed clients: queue dropped, slot
// unregistered
__global__ void k_list_erase(Table tb, uint32_t n, const uint32_t* slots) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) tb.sc[list_slot(slots, i)] = ScanRec{0.0, 0.0, 0.0, 0, 0, 0, 0, 0};
}

// Counts and offsets of a slot list, on the device and on the host; the
// total in *total.
static int list_offsets(dmc_queue* q, uint32_t n, const uint32_t* d_slots,
                        uint32_t* d_counts, uint32_t* d_offs,
                        std::vector<uint32_t>* h_counts, uint64_t* total) {
  hipLaunchKernelGGL(k_list_counts, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0,
                     q->stream, q->tb, n, d_slots, d_counts);
  h_counts->resize(n);
  HIP_OK(hipMemcpyAsync(h_counts->data(), d_counts, 4ull * n, hipMemcpyDeviceToHost,
                        q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  // offsets on the host (n * 4 bytes each way; ring capacity <= 64 keeps the
  // total below 2^32 for any table that fits in HBM)
  std::vector<uint32_t> offs(n);
  uint64_t t = 0;
  for (uint32_t i = 0; i < n; ++i) {
    offs[i] = (uint32_t)t;
    t += (*h_counts)[i];
  }
  HIP_OK(hipMemcpyAsync(d_offs, offs.data(), 4ull * n, hipMemcpyHostToDevice, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  *total = t;
  return DMC_OK;
}

struct DevBuf {
  void* p = nullptr;
  ~DevBuf() { dfree(p); }
  int alloc(size_t bytes) {
    return hipMalloc(&p, bytes ? bytes : 1) == hipSuccess ? DMC_OK : DMC_ENOMEM;
  }
  uint32_t* u32() const { return static_cast<uint32_t*>(p); }
  uint64_t* u64() const { return static_cast<uint64_t*>(p); }
  uint8_t* u8() const { return static_cast<uint8_t*>(p); }
};

__global__ void k_mark_idle_dev(Table tb, uint32_t n, const uint32_t* slots) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t s = slots[i];
  if (s < tb.n && (tb.sc[s].flags & F_REG)) tb.sc[s].flags |= F_IDLE;
}

int dmc_client_mark_idle_batch_device(dmc_queue* q, uint32_t n, const uint32_t* d_slots) {
  if (!q || (n && !d_slots)) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  if (!n) return DMC_OK;
  hipLaunchKernelGGL(k_mark_idle_dev, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0,
                     q->stream, q->tb, n, d_slots);
  HIP_OK(hipGetLastError());
  q->idle_unknown = true;
  return DMC_OK;
}

static int read_handles(dmc_queue* q, uint32_t slot, std::vector<ReqEntry>* ents,
                        uint32_t* head) {
  ScanRec sr;
  HIP_OK(hipMemcpyAsync(&sr, q->tb.sc + slot, sizeof(sr), hipMemcpyDeviceToHost,
                        q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  uint32_t h = sr.head, c = sr.count;
  std::vector<ReqEntry> ring(q->p.ring_capacity);
  HIP_OK(hipMemcpyAsync(ring.data(), q->tb.ring + (size_t)slot * q->p.ring_capacity,
                        sizeof(ReqEntry) * q->p.ring_capacity, hipMemcpyDeviceToHost,
                        q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  ents->clear();
  for (uint32_t i = 0; i < c; ++i) ents->push_back(ring[(h + i) & q->tb.qmask]);
  *head = h;
  return DMC_OK;
}

// rewrite a client's queue (after filtering), keeping the front's ready flag
// only if the front survived; the new front's keys with the client's
// prop_delta (an IEEE double add on the host, no contraction: the same
// value as the device's __dadd_rn)
static int write_queue(dmc_queue* q, uint32_t slot, const std::vector<ReqEntry>& ents,
                       bool front_kept) {
  uint32_t Q = q->p.ring_capacity;
  std::vector<ReqEntry> ring(Q);
  for (size_t i = 0; i < ents.size(); ++i) ring[i] = ents[i];
  HIP_OK(hipMemcpyAsync(q->tb.ring + (size_t)slot * Q, ring.data(), sizeof(ReqEntry) * Q,
                        hipMemcpyHostToDevice, q->stream));
  ScanRec sr;
  double pd = 0.0;
  HIP_OK(hipMemcpyAsync(&sr, q->tb.sc + slot, sizeof(sr), hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipMemcpyAsync(&pd, &q->tb.rec[slot].pd, 8, hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  const uint32_t c = (uint32_t)ents.size();
  ScanRec o{0.0, 0.0, 0.0, 0, (uint8_t)c, sr.flags, 0, 0};
  if (c) {
    o.r = ring[0].r;
    volatile double pk = ring[0].p + pd;
    o.pk = pk;
    o.l = ring[0].l;
  }
  if (!front_kept || !c) o.flags &= (uint8_t)~F_READY;
  HIP_OK(hipMemcpyAsync(q->tb.sc + slot, &o, sizeof(o), hipMemcpyHostToDevice, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  return DMC_OK;
}

int dmc_client_erase(dmc_queue* q, uint32_t slot, uint64_t* handles_out,
                     uint32_t cap, uint32_t* n_out) {
  if (!q || slot >= q->p.max_clients) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  ++q->gen;
  if (int rc0 = settle_act(q)) return rc0;
  if (int rc0 = sync_idle(q)) return rc0;
  if (!q->reg_h[slot]) return DMC_ENOTREG;
  std::vector<ReqEntry> ents;
  uint32_t h;
  int rc = read_handles(q, slot, &ents, &h);
  if (rc) return rc;
  for (size_t i = 0; i < ents.size() && i < cap; ++i)
    if (handles_out) handles_out[i] = ents[i].handle;
  if (n_out) *n_out = (uint32_t)ents.size();
  if (q->heap && (rc = heap_list(q, k_heap_remove, {slot}))) return rc;
  const ScanRec z{0.0, 0.0, 0.0, 0, 0, 0, 0, 0};  // no requests, not registered
  HIP_OK(hipMemcpyAsync(q->tb.sc + slot, &z, sizeof(z), hipMemcpyHostToDevice, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  if (q->idle_h[slot]) --q->n_idle;
  q->reg_h[slot] = 0;
  q->idle_h[slot] = 0;
  --q->n_registered;
  return DMC_OK;
}

int dmc_client_get_state(dmc_queue* q, uint32_t slot, dmc_client_state* s) {
  if (!q || !s || slot >= q->p.max_clients) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  std::memset(s, 0, sizeof(*s));
  const Table& t = q->tb;
  uint8_t f = 0;
  ClientRec cr;
  ScanRec sr;
  ClientAux ax;
  HIP_OK(hipMemcpyAsync(&cr, t.rec + slot, sizeof(cr), hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipMemcpyAsync(&sr, t.sc + slot, sizeof(sr), hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipMemcpyAsync(&ax, t.aux + slot, sizeof(ax), hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  f = sr.flags;
  s->prop_delta = cr.pd;
  s->prev_r = cr.prev_r;
  s->prev_p = cr.prev_p;
  s->prev_l = cr.prev_l;
  s->prev_arrival = cr.prev_arr;
  s->r_inv = cr.r_inv;
  s->w_inv = cr.w_inv;
  s->l_inv = cr.l_inv;
  s->last_tick = ax.last_tick;
  s->count = sr.count;
  s->cur_delta = ax.cur_delta;
  s->cur_rho = ax.cur_rho;
  uint32_t head = sr.head;
  if (s->count) {
    // the front's tag is its ring entry's (ScanRec caches r, p + pd, l)
    ReqEntry e;
    HIP_OK(hipMemcpyAsync(&e, t.ring + (size_t)slot * t.q + head, sizeof(e),
                          hipMemcpyDeviceToHost, q->stream));
    HIP_OK(hipStreamSynchronize(q->stream));
    s->front_r = e.r;
    s->front_p = e.p;
    s->front_l = e.l;
    s->front_arrival = e.arrival;
  } else {
    s->front_r = s->front_p = s->front_l = 0.0;
  }
  s->idle = (f & F_IDLE) ? 1 : 0;
  s->front_ready = (f & F_READY) && s->count ? 1 : 0;
  s->registered = (f & F_REG) ? 1 : 0;
  return s->registered ? DMC_OK : DMC_ENOTREG;
}

int dmc_client_last_ticks(dmc_queue* q, uint32_t n, uint64_t* out) {
  if (!q || !out || n > q->p.max_clients) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  if (n)
    HIP_OK(hipMemcpy2DAsync(out, sizeof(uint64_t), &q->tb.aux[0].last_tick,
                            sizeof(ClientAux), sizeof(uint64_t), n,
                            hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  return DMC_OK;
}

int dmc_add_batch(dmc_queue* q, uint32_t n, const dmc_request* reqs,
                  int32_t* rc_out) {
  if (!q || (n && !reqs)) return DMC_EINVAL;
  QueueLock g(q, true);
  ++q->gen;
  if (g.rc) return g.rc;
  if (q->heap) {  // heap order: every add in call order on the device
    if (int rc0 = serve_quiesce(q)) return rc0;
    if (!n) return DMC_OK;
    int rc = ensure_batch(q, n);
    if (rc) return rc;
    // U1 with a host client_info_f: the infos the batch's tags read
    rc = fetch_infos(q, n, &reqs[0].slot, sizeof(dmc_request), true);
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(q->d_reqs, reqs, sizeof(dmc_request) * n, hipMemcpyHostToDevice,
                          q->stream));
    rc = heap_add(q, n, q->d_reqs, q->d_rc);
    if (rc) return rc;
    std::vector<int32_t> rcs(n);
    HIP_OK(hipMemcpyAsync(rcs.data(), q->d_rc, 4ull * n, hipMemcpyDeviceToHost, q->stream));
    HIP_OK(hipStreamSynchronize(q->stream));
    if (rc_out) std::memcpy(rc_out, rcs.data(), 4ull * n);
    return DMC_OK;
  }
  if (n == 1 && serve_add_ok(q, reqs[0])) return serve_add(q, reqs[0], rc_out);
  if (int rc0 = serve_quiesce(q)) return rc0;
  if (int rc0 = settle_act(q)) return rc0;
  if (int rc0 = sync_idle(q)) return rc0;
  if (!n) return DMC_OK;
  int rc = ensure_batch(q, n);
  if (rc) return rc;
  // U1 with a host client_info_f: the infos the batch's tags read
  rc = fetch_infos(q, n, &reqs[0].slot, sizeof(dmc_request), true);
  if (rc) return rc;
  if (n == 1 && q->single_op && !q->prof_on &&
      (reqs[0].slot >= q->p.max_clients || !q->idle_h[reqs[0].slot])) {
    // the single-op path: one kernel, request and status in host-mapped memory
    q->h_fast->req = reqs[0];
    hipLaunchKernelGGL(k_add_one, dim3(1), dim3(64), 0, q->stream, q->tb,
                       (const dmc_request*)&q->d_fast->req, &q->d_fast->rc, q->tick);
    HIP_OK(hipStreamSynchronize(q->stream));
    q->tick += 1;
    if (rc_out) rc_out[0] = q->h_fast->rc;
    return DMC_OK;
  }
  HIP_OK(hipMemcpyAsync(q->d_reqs, reqs, sizeof(dmc_request) * n,
                        hipMemcpyHostToDevice, q->stream));
  rc = q->n_idle ? add_with_idle(q, reqs, n, q->d_reqs, q->d_rc)
                 : add_segment(q, q->d_reqs, n, q->d_rc, q->tick);
  if (rc) return rc;
  q->tick += n;
  if (rc_out)
    HIP_OK(hipMemcpyAsync(rc_out, q->d_rc, 4ull * n, hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  pflush(q);
  return DMC_OK;
}

int dmc_add_batch_device(dmc_queue* q, uint32_t n, const dmc_request* d_reqs,
                         int32_t* d_rc_out) {
  if (!q || (n && (!d_reqs || !d_rc_out))) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  ++q->gen;
  if (!n) return DMC_OK;
  if (q->heap) return heap_add(q, n, d_reqs, d_rc_out);
  int rc = ensure_batch(q, n);
  if (rc) return rc;
  rc = settle_act(q);
  if (rc) return rc;
  if (maybe_idle(q) && !q->act_split) {
    rc = add_act_batch_dev(q, n, d_reqs, d_rc_out);
  } else if (maybe_idle(q) && (rc = sync_idle(q)) != DMC_OK) {
    return rc;
  } else if (q->n_idle) {
    // the host split (forced): stage the batch on the host
    std::vector<dmc_request> h(n);
    HIP_OK(hipMemcpyAsync(h.data(), d_reqs, sizeof(dmc_request) * n,
                          hipMemcpyDeviceToHost, q->stream));
    HIP_OK(hipStreamSynchronize(q->stream));
    rc = add_with_idle(q, h.data(), n, d_reqs, d_rc_out);
  } else {
    rc = add_segment(q, d_reqs, n, d_rc_out, q->tick);
  }
  if (rc) return rc;
  q->tick += n;
  pflush(q);  // no-op unless profiling (then it waits for the add kernels)
  return DMC_OK;
}

int dmc_pull_batch(dmc_queue* q, double now, uint32_t k, dmc_decision* out,
                   dmc_pull_result* result) {
  if (!q || (k && !out)) return DMC_EINVAL;
  QueueLock g(q, true);
  ++q->gen;
  if (g.rc) return g.rc;
  if (q->heap) {
    if (int rc0 = serve_quiesce(q)) return rc0;
    int rc = ensure_dec(q, k);
    if (rc) return rc;
    dmc_pull_result r{};
    rc = heap_pull(q, now, k, q->d_dec, nullptr, &r);
    if (rc) return rc;
    if (r.n_decisions) {
      HIP_OK(hipMemcpyAsync(out, q->d_dec, sizeof(dmc_decision) * r.n_decisions,
                            hipMemcpyDeviceToHost, q->stream));
      HIP_OK(hipStreamSynchronize(q->stream));
    }
    if (result) *result = r;
    return DMC_OK;
  }
  if (q->serve_on && fast_pull_ok(q, k)) return serve_pull(q, now, k, out, result);
  if (int rc0 = serve_quiesce(q)) return rc0;
  if (fast_pull_ok(q, k)) return fast_pull(q, now, k, out, result);
  int rc = ensure_dec(q, k);
  if (rc) return rc;
  dmc_pull_result r{};
  rc = pull_impl(q, now, k, q->d_dec, &r);
  if (rc) return rc;
  if (r.n_decisions)
    HIP_OK(hipMemcpyAsync(out, q->d_dec, sizeof(dmc_decision) * r.n_decisions,
                          hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  if (result) *result = r;
  return DMC_OK;
}

int dmc_pull_batch_device(dmc_queue* q, double now, uint32_t k,
                          dmc_decision* d_out, dmc_pull_result* d_result) {
  if (!q || (k && !d_out)) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  ++q->gen;
  if (q->heap) return heap_pull(q, now, k, d_out, d_result, nullptr);
  dmc_pull_result r{};
  bool dev_wrote = false;
  int rc = pull_impl(q, now, k, d_out, &r, d_result, &dev_wrote);
  if (rc) return rc;
  if (d_result && !dev_wrote) {  // stream-ordered after the call's rounds
    hipLaunchKernelGGL(k_put_result, dim3(1), dim3(1), 0, q->stream, d_result, r);
    HIP_OK(hipGetLastError());
  }
  return DMC_OK;
}

// add_batch followed by pull_batch(now, k), both device-resident: one graph
// launch for the add kernels and the first pull round when nothing needs the
// host in between (no idle client to activate, a batched bin-ranked round),
// otherwise exactly the two calls.
int dmc_add_pull_batch_device(dmc_queue* q, uint32_t n, const dmc_request* d_reqs,
                              int32_t* d_rc_out, double now, uint32_t k,
                              dmc_decision* d_out, dmc_pull_result* d_result) {
  if (!q || (n && (!d_reqs || !d_rc_out)) || (k && !d_out)) return DMC_EINVAL;
  {
    // (a pipelined call left pending is finished after this call's launch)
    QueueLock g(q, false, false);
    if (g.rc) return g.rc;
    ++q->gen;
    for (;;) {
      if (q->heap) {
        if (int rc = settle_pending(q)) return rc;
        if (int rc = heap_add(q, n, d_reqs, d_rc_out)) return rc;
        return heap_pull(q, now, k, d_out, d_result, nullptr);
      }
      if (int rc0 = settle_act(q)) return rc0;
      // (pipelined calls also fuse with graphs off: the kernels launched
      // eagerly, still queued behind the previous call's)
      const bool fuse = n && k && !maybe_idle(q) && q->n_registered > 0 && k > q->small_k &&
                        !q->force_radix && q->radix_batches == 0 && k <= kBinRankMaxK &&
                        (q->use_graphs || q->pipeline);
      if (!fuse) {
        if (int rc = settle_pending(q)) return rc;
        break;  // the two calls
      }
      int rc = ensure_batch(q, n);
      if (!rc) rc = ensure_brec(q);
      if (rc) return rc;
      AddParams ap{d_reqs, d_rc_out, q->tick, n, 0};
      // (k_chain_scan: the batch's epoch, never 0; when the counter wraps the
      // stamps are cleared first, so that no slot keeps a stamp equal to a
      // later batch's epoch)
      uint32_t epoch = 0;
      if (overlap_ok(q, n)) {
        if (++q->epoch == (DMC_STAMP_SC ? 256u : 0u)) {
          if (DMC_STAMP_SC)
            hipLaunchKernelGGL(k_clear_stamps, dim3((q->tb.n + kBlock - 1) / kBlock),
                               dim3(kBlock), 0, q->stream, q->tb);
          else
            HIP_OK(hipMemsetAsync(q->tb.touch, 0, 4ull * q->p.max_clients, q->stream));
          q->epoch = 1;
        }
        epoch = q->epoch;
      }
      CallParams cp{k,     0,   now, d_out, q->tick + n, d_result, ++q->round_seq, q->fault,
                    epoch, q->pipeline ? q->gate : nullptr};
      // DMC_DEFER_APPLY (pipelined calls launched eagerly): this call's
      // k_rapply is left to the next call's filing launch, where it runs
      // beside that filing (k_apply_link), or to settle_pending; the previous
      // call's deferred apply merges into this launch, or -- on any other
      // path -- is launched first, before this call's work
      const bool defer = DMC_DEFER_APPLY && q->pipeline && overlap_ok(q, n);
      const bool merge = defer && q->pend.on && q->pend.apply;
      if (q->pend.on && q->pend.apply && !merge) {
        q->pend.apply = false;
        launch_apply(q);
      }
      auto enqueue = [&] {
        if (overlap_ok(q, n)) {
          enqueue_add_round_overlap(q, ap, cp, merge, defer);
        } else {
          enqueue_add(q, ap);
          enqueue_round(q, cp, false);
        }
      };
      ++q->ctr.fused_calls;
      uint64_t key = (4ull << 56) | ((uint64_t)n << 3) | (use_sample(q, false) ? 2 : 0);
      int err = DMC_OK;
      GraphRec* gr = graph_for(q, key, enqueue, &err, (const void*)k_rscan);
      if (err) return err;
      if (!gr) {
        enqueue();
        HIP_OK(hipGetLastError());
      } else {
        Table tb = q->tb;
        ActBuf noact{};
        void* a1[] = {&ap, &tb, &q->abuf, &q->apos, &q->aslot, &q->apblk,
                      &noact};
        const bool sampled = use_sample(q, false);
        uint64_t* skr = sampled ? q->skr : nullptr;
        uint64_t* skp = sampled ? q->skp : nullptr;
        uint64_t* kr = sampled ? nullptr : q->keyr;
        uint64_t* kp = sampled ? nullptr : q->keyp;
        void* a2[] = {&tb, &kr, &kp, &q->meta, &q->rparts, &q->rd, &cp,
                      &skr, &skp, &q->k32, &q->hist};
        rc = graph_replay(q, *gr, a1, a2);
        if (rc) return rc;
      }
      q->tick += n;
      if (merge) q->pend.apply = false;  // (launched beside this call's filing)
      if (q->pipeline) {
        // the previous call, finished now that this one is queued behind it
        bool clean = true;
        if ((rc = settle_pending(q, &clean))) {
          q->pipe_err = rc;  // (kept: DMC_ENOTRUN below does not say what it was)
          if (clean) {
            // the previous call's round ended its call (the gate stayed
            // open), so this call's kernels, queued behind it, ran -- but
            // its deferred apply is not launched, nor its round read: the
            // queue's state is unknown, and every later call fails
            q->wedged = true;
            return rc;
          }
          // the previous call failed after shutting the gate: this call's
          // graph, queued behind it, did nothing -- it was not executed
          // (its statuses, decisions and result untouched), which
          // DMC_ENOTRUN tells the caller; the gate is open again
          q->tick -= n;
          --q->ctr.fused_calls;
          return DMC_ENOTRUN;
        }
        if (!clean) {
          // it needed the host: the graph just queued found the gate shut
          // and did nothing -- launched again, behind the previous call's
          // remaining work
          q->tick -= n;
          --q->ctr.fused_calls;
          continue;
        }
        q->pend.on = true;
        q->pend.seq = cp.seq;
        q->pend.k = k;
        q->pend.now = now;
        q->pend.out = d_out;
        q->pend.res = d_result;
        q->pend.apply = defer;
        return DMC_OK;
      }
      dmc_pull_result r{};
      bool dev_wrote = false;
      rc = pull_impl(q, now, k, d_out, &r, d_result, &dev_wrote, true);
      if (rc) return rc;
      if (d_result && !dev_wrote) {
        hipLaunchKernelGGL(k_put_result, dim3(1), dim3(1), 0, q->stream, d_result, r);
        HIP_OK(hipGetLastError());
      }
      return DMC_OK;
    }
  }
  int rc = dmc_add_batch_device(q, n, d_reqs, d_rc_out);
  if (rc) return rc;
  return dmc_pull_batch_device(q, now, k, d_out, d_result);
}


// ================================================================ queue groups
// S server queues of one device driven as one: a group step is, for every
// member, get_req_params for the batch (optional device trackers), n
// add_request_time and k pull_request(now) -- each member exactly what
// dmc_tracker_fill + dmc_add_pull_batch_device + dmc_tracker_tally do on
// it alone -- with one launch per kernel over all members (blockIdx.y =
// member, dmc_round.h's multi-table kernels) captured as one hipGraph.
// Members run on the group's stream while they belong to it.

namespace {

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// the members' locks, in member order (a group's members are locked together
// only here; every other call locks one queue)
struct GroupLock {
  std::vector<std::unique_lock<std::mutex>> ls;
  int rc = DMC_OK;
  explicit GroupLock(dmc_group* g) {
    (void)hipSetDevice(g->device);
    for (dmc_queue* q : g->qs) ls.emplace_back(q->mtx);
    for (dmc_queue* q : g->qs) {
      if (q->wedged) rc = DMC_EDEVICE;
      else if (int e = serve_quiesce(q)) rc = e;
      else if (int e2 = settle_pending(q)) rc = e2;
    }
  }
};

}  // namespace

int dmc_group_create(dmc_queue* const* queues, uint32_t n, dmc_group** out) {
  if (!queues || !n || !out) return DMC_EINVAL;
  const dmc_queue_params& p0 = queues[0]->p;
  for (uint32_t i = 0; i < n; ++i) {
    const dmc_queue* q = queues[i];
    if (!q || q->group || q->heap || q->p.device != p0.device ||
        q->p.max_clients != p0.max_clients ||
        q->p.ring_capacity != p0.ring_capacity)
      return DMC_EINVAL;
    for (uint32_t j = 0; j < i; ++j)
      if (queues[j] == q) return DMC_EINVAL;
  }
  dmc_group* g = new dmc_group();
  g->device = p0.device;
  g->qs.assign(queues, queues + n);
  (void)hipSetDevice(g->device);
  const size_t S = n;
  size_t o = 0;
  auto take = [&](size_t sz) {
    const size_t at = o;
    o = align_up(o + sz * S, 64);
    return at;
  };
  g->o_trk = take(sizeof(TrackArgs));
  g->o_add = take(sizeof(AddArgs));
  g->o_scan = take(sizeof(RScanArgs));
  g->o_hist = take(sizeof(RHistArgs));
  g->o_emit = take(sizeof(REmitArgs));
  g->o_rank = take(sizeof(RRankArgs));
  g->o_apply = take(sizeof(RApplyArgs));
  g->bytes = o;
  g->o_tally = take(sizeof(TallyArgs));
  g->tally_bytes = o - g->o_tally;
  if (hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&g->stream2, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&g->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&g->ev_join, hipEventDisableTiming) != hipSuccess ||
      hipHostMalloc((void**)&g->h_blob, o, 0) != hipSuccess ||
      hipMalloc((void**)&g->d_blob, o) != hipSuccess) {
    dmc_group_destroy(g);
    return DMC_ENOMEM;
  }
  std::memset(g->h_blob, 0, o);
  for (dmc_queue* q : g->qs) {
    QueueLock l(q);
    if (l.rc || hipStreamSynchronize(q->stream) != hipSuccess) {
      dmc_group_destroy(g);
      return DMC_EDEVICE;
    }
    q->own_stream = q->stream;
    q->stream = g->stream;
    q->group = g;
  }
  *out = g;
  return DMC_OK;
}

int dmc_group_destroy(dmc_group* g) {
  if (!g) return DMC_EINVAL;
  (void)hipSetDevice(g->device);
  if (g->stream) (void)hipStreamSynchronize(g->stream);
  for (dmc_queue* q : g->qs) {
    if (!q || q->group != g) continue;
    std::lock_guard<std::mutex> l(q->mtx);
    q->stream = q->own_stream;
    q->own_stream = nullptr;
    q->group = nullptr;
  }
  group_graphs_destroy(g);
  for (auto& r : g->prof_pool) {
    if (r.a) (void)hipEventDestroy(r.a);
    if (r.b) (void)hipEventDestroy(r.b);
  }
  if (g->h_blob) (void)hipHostFree(g->h_blob);
  dfree(g->d_blob);
  if (g->stream) (void)hipStreamDestroy(g->stream);
  if (g->cap_stream) (void)hipStreamDestroy(g->cap_stream);
  if (g->stream2) (void)hipStreamDestroy(g->stream2);
  if (g->cap_stream2) (void)hipStreamDestroy(g->cap_stream2);
  if (g->ev_fork) (void)hipEventDestroy(g->ev_fork);
  if (g->ev_join) (void)hipEventDestroy(g->ev_join);
  if (g->side) {
    (void)hipStreamSynchronize(g->side);
    (void)hipStreamDestroy(g->side);
  }
  if (g->ev_side_in) (void)hipEventDestroy(g->ev_side_in);
  if (g->ev_side_out) (void)hipEventDestroy(g->ev_side_out);
  delete g;
  return DMC_OK;
}

void* dmc_group_stream(dmc_group* g) { return g ? (void*)g->stream : nullptr; }

int dmc_group_tracker_collect_sums(dmc_group* g, uint32_t n_slots,
                                   const uint32_t* const* d_client_of_slot,
                                   const uint32_t* const* d_comp_delta,
                                   const uint32_t* const* d_comp_rho, uint32_t* d_sum_delta,
                                   uint32_t* d_sum_rho) {
  if (!g || !d_comp_delta || !d_comp_rho || !d_sum_delta || !d_sum_rho) return DMC_EINVAL;
  const uint32_t S = (uint32_t)g->qs.size();
  for (uint32_t i = 0; i < S; ++i) {
    if (!d_comp_delta[i] || !d_comp_rho[i]) return DMC_EINVAL;
    if (n_slots > g->qs[i]->p.max_clients) return DMC_EINVAL;
  }
  if (!n_slots) return DMC_OK;
  GroupLock gl(g);
  if (gl.rc) return gl.rc;
  if (!g->side) {
    if (hipStreamCreateWithFlags(&g->side, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&g->ev_side_in, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&g->ev_side_out, hipEventDisableTiming) != hipSuccess)
      return DMC_ENOMEM;
  }
  // (a second collection before a join: the first one's sums are ordered
  // before this one's reads of the group's stream anyway; join both)
  HIP_OK(hipEventRecord(g->ev_side_in, g->stream));
  HIP_OK(hipStreamWaitEvent(g->side, g->ev_side_in, 0));
  for (uint32_t i = 0; i < S; ++i)
    hipLaunchKernelGGL(k_track_sums, dim3(grid_for(n_slots, 2048)), dim3(kBlock), 0, g->side,
                       n_slots, d_client_of_slot ? d_client_of_slot[i] : nullptr,
                       d_comp_delta[i], d_comp_rho[i], d_sum_delta, d_sum_rho);
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(g->ev_side_out, g->side));
  g->side_pending = true;
  return DMC_OK;
}

int dmc_group_tracker_join(dmc_group* g) {
  if (!g) return DMC_EINVAL;
  GroupLock gl(g);
  if (gl.rc) return gl.rc;
  if (g->side_pending) {
    HIP_OK(hipStreamWaitEvent(g->stream, g->ev_side_out, 0));
    g->side_pending = false;
  }
  return DMC_OK;
}

void* dmc_group_side_stream(dmc_group* g) { return g ? (void*)g->side : nullptr; }

int dmc_group_profile_enable(dmc_group* g, int on) {
  if (!g) return DMC_EINVAL;
  GroupLock gl(g);
  if (gl.rc) return gl.rc;
  group_prof_flush(g);
  g->prof_on = on != 0;
  for (int i = 0; i < DMC_PROF_NSTAGES; ++i) {
    g->prof_ms[i] = 0.0;
    g->prof_cnt[i] = 0;
  }
  return DMC_OK;
}

int dmc_group_profile_read(dmc_group* g, uint32_t stage, uint64_t* count, double* total_ms) {
  if (!g || stage >= DMC_PROF_NSTAGES || !count || !total_ms) return DMC_EINVAL;
  GroupLock gl(g);
  if (gl.rc) return gl.rc;
  group_prof_flush(g);
  *count = g->prof_cnt[stage];
  *total_ms = g->prof_ms[stage];
  return DMC_OK;
}

int dmc_group_step_device(dmc_group* g, uint32_t n, dmc_request* const* d_reqs,
                          int32_t* const* d_rc, const double* now, uint32_t k,
                          dmc_decision* const* d_out, dmc_pull_result* const* d_result,
                          const dmc_group_tracker* trk) {
  if (!g || !now || (n && (!d_reqs || !d_rc)) || (k && !d_out)) return DMC_EINVAL;
  const uint32_t S = (uint32_t)g->qs.size();
  for (uint32_t i = 0; i < S; ++i)
    if ((n && (!d_reqs[i] || !d_rc[i])) || (k && !d_out[i])) return DMC_EINVAL;
  bool fuse = n && k;
  {
    GroupLock gl(g);
    if (gl.rc) return gl.rc;
    ++g->steps;
    for (dmc_queue* q : g->qs) {
      ++q->gen;
      if (int rc0 = settle_act(q)) return rc0;
      fuse = fuse && !maybe_idle(q) && q->n_registered > 0 && k > q->small_k && !q->force_radix &&
             q->radix_batches == 0 && k <= kBinRankMaxK && q->use_graphs && !q->prof_on;
    }
    if (fuse) {
      for (dmc_queue* q : g->qs) {
        int rc = ensure_batch(q, n);
        if (!rc) rc = ensure_brec(q);
        if (rc) return rc;
      }
      TrackArgs* ta = reinterpret_cast<TrackArgs*>(g->h_blob + g->o_trk);
      AddArgs* aa = reinterpret_cast<AddArgs*>(g->h_blob + g->o_add);
      RScanArgs* sa = reinterpret_cast<RScanArgs*>(g->h_blob + g->o_scan);
      RHistArgs* ha = reinterpret_cast<RHistArgs*>(g->h_blob + g->o_hist);
      REmitArgs* ea = reinterpret_cast<REmitArgs*>(g->h_blob + g->o_emit);
      RRankArgs* ra = reinterpret_cast<RRankArgs*>(g->h_blob + g->o_rank);
      RApplyArgs* pa = reinterpret_cast<RApplyArgs*>(g->h_blob + g->o_apply);
      bool all_sampled = true;
      uint32_t gN = 0, gEm = 0;
      const uint32_t gAdd = (n + kBlock - 1) / kBlock;
      // DMC_GROUP_OVERLAP: the chain and the scan side by side, the batch's
      // slots stamped with each member's epoch (k_chain_scan's scheme; a
      // wrapped epoch clears its table's stamps first)
      const bool ovl = DMC_GROUP_OVERLAP && gAdd <= kFixPartsMax;
      if (ovl) {
        for (dmc_queue* q : g->qs) {
          if (++q->epoch == 256u) {
            hipLaunchKernelGGL(k_clear_stamps, dim3((q->tb.n + kBlock - 1) / kBlock),
                               dim3(kBlock), 0, g->stream, q->tb);
            HIP_OK(hipGetLastError());
            q->epoch = 1;
          }
        }
      }
      // (the add chain and the scan one after the other: k_chain_scan over
      // all tables measured slower, config 5 1.04 vs 0.93 ms, r04o)
      for (uint32_t i = 0; i < S; ++i) {
        dmc_queue* q = g->qs[i];
        const Table& tb = q->tb;
        const uint32_t N = tb.n;
        gN = (N + kScanBlock * kScanSlots - 1) / (kScanBlock * kScanSlots);
        gEm = (N + kEmitChunkM - 1) / kEmitChunkM;
        const bool sampled = use_sample(q, false);
        all_sampled = all_sampled && sampled;
        ta[i] = trk ? TrackArgs{d_reqs[i], n, q->p.max_clients, trk[i].client_of_slot,
                                trk[i].gdelta, trk[i].grho, trk[i].xd, trk[i].xr, trk[i].known,
                                trk[i].first}
                    : TrackArgs{};
        const uint32_t epoch = ovl ? q->epoch : 0u;
        aa[i] = AddArgs{AddParams{d_reqs[i], d_rc[i], q->tick, n, epoch}, tb, q->abuf, q->apos,
                        q->aslot, q->apblk,
                        trk ? TrackFill{d_reqs[i], trk[i].client_of_slot, trk[i].gdelta,
                                        trk[i].grho, trk[i].xd, trk[i].xr, trk[i].known,
                                        q->p.max_clients}
                            : TrackFill{}};
        const CallParams cp{k, 0, now[i], d_out[i], q->tick + n,
                            d_result ? d_result[i] : nullptr, ++q->round_seq, q->fault, epoch};
        const uint32_t np = ovl ? gN + gAdd : gN;  // (the scan's partials, then the chain's)
        sa[i] = RScanArgs{tb, sampled ? nullptr : q->keyr, sampled ? nullptr : q->keyp, q->meta,
                          q->rparts, q->rd, cp, sampled ? q->skr : nullptr,
                          sampled ? q->skp : nullptr, q->k32, q->hist};
        ha[i] = sampled ? RHistArgs{(N + kSample - 1) / kSample, np, q->skr, q->skp, q->rparts,
                                    q->rd, q->hist, q->sample_mode == 2 ? 2 : 1,
                                    (unsigned long long*)q->bcount, q->bsup}
                        : RHistArgs{N, np, q->keyr, q->keyp, q->rparts, q->rd, q->hist, 0,
                                    (unsigned long long*)q->bcount, q->bsup};
        ea[i] = REmitArgs{tb, q->rd, q->k32, q->meta, q->cand, q->bcand, q->post, q->decof,
                          q->brec, q->bcount, q->bsup, q->hist, q->dense, q->ecap};
        // (the trackers' tallies made where the decisions are written)
        const TallyP tp = (trk && d_result) ? TallyP{trk[i].comp_delta, trk[i].comp_rho}
                                             : TallyP{};
        ra[i] = RRankArgs{q->rd, (const unsigned long long*)q->bcount, q->bsup, q->brec, tb.ring,
                          q->decof, tp};
        pa[i] = RApplyArgs{tb, q->rd, q->cand, q->bcand, q->decof, q->post, q->sched,
                           q->d_hround, tp};
      }
      const uint32_t gHist = all_sampled ? kHistBlocksSampled : kHistBlocksR;
      uint8_t* d = g->d_blob;
      // (profiling: eager launches, each kernel's dispatch recording its
      // stage's events; a stage of two kernels -- select: hist + pick -- gets
      // its start from the first and its end from the second)
      hipEvent_t ev_open = nullptr;
      auto gl = [&](hipStream_t st, int stage, int part, auto kernel, dim3 gr, dim3 bl,
                    auto... arg) {
        if (!g->prof_on || (st != g->stream && st != g->stream2) || stage < 0) {
          hipLaunchKernelGGL(kernel, gr, bl, 0, st, arg...);
          return;
        }
        if (part == 0 || part == 2) {  // (a new record: 0 one kernel, 2 first of two)
          if (g->prof_n == g->prof_pool.size()) {
            dmc_group::PRec r;
            if (hipEventCreateWithFlags(&r.a, hipEventDisableSystemFence) != hipSuccess ||
                hipEventCreateWithFlags(&r.b, hipEventDisableSystemFence) != hipSuccess) {
              g->prof_on = false;
              hipLaunchKernelGGL(kernel, gr, bl, 0, st, arg...);
              return;
            }
            g->prof_pool.push_back(r);
          }
          g->prof_pool[g->prof_n].stage = stage;
        }
        dmc_group::PRec& r = g->prof_pool[g->prof_n];
        if (part == 0) {
          hipExtLaunchKernelGGL(kernel, gr, bl, 0, st, r.a, r.b, 0, arg...);
          ++g->prof_n;
        } else if (part == 2) {
          hipExtLaunchKernelGGL(kernel, gr, bl, 0, st, r.a, nullptr, 0, arg...);
          ev_open = r.b;
        } else {  // part 3: the second of two
          hipExtLaunchKernelGGL(kernel, gr, bl, 0, st, nullptr, ev_open, 0, arg...);
          ++g->prof_n;
        }
      };
      auto enqueue = [&](hipStream_t st) {
        (void)hipMemcpyAsync(d, g->h_blob, g->bytes, hipMemcpyHostToDevice, st);
        // (the trackers' get_req_params run inside k_add_chain_m: TrackFill)
        gl(st, DMC_PROF_ADD_LINK, 0, k_add_link_m, dim3(gAdd, S), dim3(kBlock),
           (const AddArgs*)(d + g->o_add));
        if (ovl) {
          // two branches: the chain on st, the scan on the second stream
          hipStream_t st2 = st == g->stream ? g->stream2 : g->cap_stream2;
          (void)hipEventRecord(g->ev_fork, st);
          (void)hipStreamWaitEvent(st2, g->ev_fork, 0);
          gl(st, DMC_PROF_ADD_CHAIN, 0, k_chain_scan_m, dim3(gAdd, S), dim3(kBlock),
             (const AddArgs*)(d + g->o_add), (const RScanArgs*)(d + g->o_scan), gN);
          const uint32_t gS = DMC_GROUP_SCAN_BLOCKS ? std::min<uint32_t>(gN, DMC_GROUP_SCAN_BLOCKS) : gN;
          gl(st2, DMC_PROF_SCAN, 0, k_rscan_mt, dim3(gS, S), dim3(kScanBlock),
             (const RScanArgs*)(d + g->o_scan), gN);
          (void)hipEventRecord(g->ev_join, st2);
          (void)hipStreamWaitEvent(st, g->ev_join, 0);
        } else {
          gl(st, DMC_PROF_ADD_CHAIN, 0, k_add_chain_m, dim3(gAdd, S), dim3(kBlock),
             (const AddArgs*)(d + g->o_add));
          gl(st, DMC_PROF_SCAN, 0, k_rscan_m, dim3(gN, S), dim3(kScanBlock),
             (const RScanArgs*)(d + g->o_scan));
        }
        gl(st, DMC_PROF_SELECT, kPrePickM ? 2 : 0, k_rhist_m, dim3(gHist, S), dim3(1024),
           (const RHistArgs*)(d + g->o_hist));
        if (kPrePickM)
          gl(st, DMC_PROF_SELECT, 3, k_rpick_m, dim3(1, S), dim3(kEmitThreads),
             (const RHistArgs*)(d + g->o_hist));
        if (kPrePickM && DMC_SPLIT_EMIT_M) {
          gl(st, -1, 0, k_rsel_m, dim3(gEm, S), dim3(kEmitThreads),
             (const REmitArgs*)(d + g->o_emit));
          gl(st, -1, 0, k_rwalk_m, dim3(gEm, S), dim3(kWalkThreads),
             (const REmitArgs*)(d + g->o_emit));
        } else {
          gl(st, DMC_PROF_EMIT, 0, k_remit_m, dim3(gEm, S), dim3(kEmitThreads),
             (const REmitArgs*)(d + g->o_emit));
        }
        gl(st, DMC_PROF_RANK, 0, k_rrank_m, dim3(kRankBlocksR, S), dim3(kRankThreads),
           (const RRankArgs*)(d + g->o_rank));
        gl(st, DMC_PROF_APPLY, 0, k_rapply_m, dim3(kApplyPerEmitM * gEm + 1, S), dim3(kBlockR),
           (const RApplyArgs*)(d + g->o_apply));
      };
      // the step's graph: captured at the second sighting of its shape, then
      // replayed (the arguments travel in the blob, no node updates)
      const uint64_t key = ((uint64_t)n << 8) | (trk ? 1 : 0) | (all_sampled ? 2 : 0) |
                           ((uint64_t)k << 36);
      dmc_group::G* gr = nullptr;
      for (auto& x : g->graphs)
        if (x.exec && x.key == key) gr = &x;
      if (g->prof_on) {
        gr = nullptr;  // (profiled steps launch eagerly)
      } else if (!gr) {
        bool seen = false;
        for (uint64_t s0 : g->seen) seen |= s0 == key;
        if (seen) {
          dmc_group::G& x = g->graphs[g->graph_next++ % 4];
          if (x.exec) HIP_OK(hipStreamSynchronize(g->stream));
          if (x.exec) (void)hipGraphExecDestroy(x.exec);
          if (x.graph) (void)hipGraphDestroy(x.graph);
          x = dmc_group::G{};
          if (!g->cap_stream)
            HIP_OK(hipStreamCreateWithFlags(&g->cap_stream, hipStreamNonBlocking));
          if (!g->cap_stream2)
            HIP_OK(hipStreamCreateWithFlags(&g->cap_stream2, hipStreamNonBlocking));
          HIP_OK(hipStreamBeginCapture(g->cap_stream, hipStreamCaptureModeThreadLocal));
          enqueue(g->cap_stream);
          HIP_OK(hipStreamEndCapture(g->cap_stream, &x.graph));
          HIP_OK(hipGraphInstantiate(&x.exec, x.graph, nullptr, nullptr, 0));
          x.key = key;
          gr = &x;
        } else {
          g->seen[g->seen_pos++ % 4] = key;
        }
      }
      if (gr) {
        HIP_OK(hipGraphLaunch(gr->exec, g->stream));
        ++g->graph_launches;
      } else {
        enqueue(g->stream);
      }
      HIP_OK(hipGetLastError());
      ++g->fused_steps;
      for (dmc_queue* q : g->qs) {
        q->tick += n;
        ++q->ctr.fused_calls;
      }
      // each member's round: its outcome, and any follow-up (a re-run, the
      // terminal pull) on the group stream
      // (the decisions later rounds wrote -- re-runs, further rounds -- are
      // tallied by k_tally_m after them; none in a step whose rounds all
      // ended their calls)
      bool more = false;
      TallyArgs* la = reinterpret_cast<TallyArgs*>(g->h_blob + g->o_tally);
      for (uint32_t i = 0; i < S; ++i) {
        dmc_queue* q = g->qs[i];
        dmc_pull_result r{};
        bool dev_wrote = false;
        dmc_pull_result* dres = d_result ? d_result[i] : nullptr;
        q->fused_ndec = 0;
        int rc = pull_impl(q, now[i], k, d_out[i], &r, dres, &dev_wrote, true);
        if (rc) return rc;
        if (dres && !dev_wrote) {
          hipLaunchKernelGGL(k_put_result, dim3(1), dim3(1), 0, q->stream, dres, r);
          HIP_OK(hipGetLastError());
        }
        if (trk && d_result) {
          la[i] = TallyArgs{d_out[i], d_result[i], k, trk[i].comp_delta, trk[i].comp_rho,
                            q->fused_ndec};
          more = more || r.n_decisions > q->fused_ndec;
        }
      }
      if (trk && d_result && more) {
        HIP_OK(hipMemcpyAsync(g->d_blob + g->o_tally, la, g->tally_bytes, hipMemcpyHostToDevice,
                              g->stream));
        hipLaunchKernelGGL(k_tally_m, dim3(grid_for(k, 1024), S), dim3(kBlock), 0, g->stream,
                           (const TallyArgs*)(g->d_blob + g->o_tally));
        HIP_OK(hipGetLastError());
      }
      return DMC_OK;
    }
  }
  // not fusable (activations pending, small k, ...): each member on its own,
  // the same calls in the same order, on the group stream
  for (uint32_t i = 0; i < S; ++i) {
    dmc_queue* q = g->qs[i];
    if (trk && n) {
      int rc = dmc_tracker_fill(q, d_reqs[i], n, trk[i].client_of_slot, trk[i].gdelta,
                                trk[i].grho, trk[i].xd, trk[i].xr, trk[i].known, trk[i].first);
      if (rc) return rc;
    }
    int rc = dmc_add_pull_batch_device(q, n, d_reqs[i], d_rc ? d_rc[i] : nullptr, now[i], k,
                                       d_out ? d_out[i] : nullptr,
                                       d_result ? d_result[i] : nullptr);
    if (rc) return rc;
    if (trk && k && d_result) {
      rc = dmc_tracker_tally(q, d_out[i], d_result[i], k, trk[i].comp_delta, trk[i].comp_rho);
      if (rc) return rc;
    }
  }
  return DMC_OK;
}

int dmc_remove_by_client(dmc_queue* q, uint32_t slot, int reverse,
                         uint64_t* handles_out, uint32_t cap, uint32_t* n_out) {
  if (!q || slot >= q->p.max_clients) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  ++q->gen;
  if (!q->reg_h[slot]) {
    if (n_out) *n_out = 0;
    return DMC_OK;  // client_map.find fails -> return, :599-601
  }
  std::vector<ReqEntry> ents;
  uint32_t h;
  int rc = read_handles(q, slot, &ents, &h);
  if (rc) return rc;
  uint32_t n = (uint32_t)ents.size();
  for (uint32_t i = 0; i < n && i < cap; ++i)
    if (handles_out) handles_out[i] = ents[reverse ? n - 1 - i : i].handle;
  if (n_out) *n_out = n;
  rc = write_queue(q, slot, {}, false);
  if (!rc && q->heap) rc = heap_list(q, k_heap_adjust, {slot});  // (:621-625)
  return rc;
}

int dmc_client_requests(dmc_queue* q, uint32_t slot, uint64_t* handles_out,
                        uint32_t cap, uint32_t* n_out) {
  if (!q || slot >= q->p.max_clients) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  if (!q->reg_h[slot]) return DMC_ENOTREG;
  std::vector<ReqEntry> ents;
  uint32_t h;
  int rc = read_handles(q, slot, &ents, &h);
  if (rc) return rc;
  for (size_t i = 0; i < ents.size() && i < cap; ++i)
    if (handles_out) handles_out[i] = ents[i].handle;
  if (n_out) *n_out = (uint32_t)ents.size();
  return DMC_OK;
}

int dmc_client_filter(dmc_queue* q, uint32_t slot, uint32_t n,
                      const uint8_t* keep) {
  if (!q || slot >= q->p.max_clients) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  ++q->gen;
  if (!q->reg_h[slot]) return DMC_ENOTREG;
  std::vector<ReqEntry> ents;
  uint32_t h;
  int rc = read_handles(q, slot, &ents, &h);
  if (rc) return rc;
  if (n != ents.size() || (n && !keep)) return DMC_EINVAL;
  std::vector<ReqEntry> kept;
  for (uint32_t i = 0; i < n; ++i)
    if (keep[i]) kept.push_back(ents[i]);
  if (kept.size() == ents.size()) return DMC_OK;
  rc = write_queue(q, slot, kept, n > 0 && keep[0]);
  if (!rc && q->heap) rc = heap_list(q, k_heap_adjust, {slot});  // (:580-584)
  return rc;
}

int dmc_queue_requests(dmc_queue* q, uint32_t* counts_out, uint64_t* handles_out,
                       uint64_t cap, uint64_t* n_out) {
  if (!q || !n_out) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  if (int rc0 = settle_act(q)) return rc0;
  const uint32_t N = q->tb.n;
  DevBuf counts, offs, hs;
  if (counts.alloc(4ull * N) || offs.alloc(4ull * N)) return DMC_ENOMEM;
  std::vector<uint32_t> hc;
  uint64_t total = 0;
  if (int rc = list_offsets(q, N, nullptr, counts.u32(), offs.u32(),
                            &hc, &total))
    return rc;
  if (counts_out) std::memcpy(counts_out, hc.data(), 4ull * N);
  *n_out = total;
  q->maint_gen = q->gen;
  q->maint_total = total;
  if (!handles_out || cap < total || !total) return DMC_OK;
  if (hs.alloc(8ull * total)) return DMC_ENOMEM;
  hipLaunchKernelGGL(k_list_gather, dim3((N + kBlock - 1) / kBlock), dim3(kBlock), 0,
                     q->stream, q->tb, N, (const uint32_t*)nullptr,
                     (const uint32_t*)offs.u32(), hs.u64());
  HIP_OK(hipMemcpyAsync(handles_out, hs.p, 8ull * total, hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  return DMC_OK;
}

int dmc_queue_filter(dmc_queue* q, const uint8_t* keep, uint64_t n, int* any_removed) {
  if (!q || (n && !keep)) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  // the queue must be the one the last dmc_queue_requests read
  if (q->maint_gen != q->gen || n != q->maint_total) return DMC_EINVAL;
  ++q->gen;
  if (any_removed) *any_removed = 0;
  if (!n) return DMC_OK;
  const uint32_t N = q->tb.n;
  DevBuf counts, offs, kp, any;
  if (counts.alloc(4ull * N) || offs.alloc(4ull * N) || kp.alloc(n) || any.alloc(4))
    return DMC_ENOMEM;
  std::vector<uint32_t> hc;
  uint64_t total = 0;
  if (int rc = list_offsets(q, N, nullptr, counts.u32(), offs.u32(),
                            &hc, &total))
    return rc;
  if (total != n) return DMC_EINVAL;
  HIP_OK(hipMemcpyAsync(kp.p, keep, n, hipMemcpyHostToDevice, q->stream));
  if (q->heap) {  // sequential, client order: filter, adjust, next client
    std::vector<uint32_t> mod;
    uint64_t at = 0;
    for (uint32_t s = 0; s < N; ++s) {
      bool m = false;
      for (uint32_t j = 0; j < hc[s]; ++j) m |= !keep[at + j];
      at += hc[s];
      if (m) mod.push_back(s);
    }
    if (any_removed) *any_removed = !mod.empty();
    if (mod.empty()) return DMC_OK;
    DevBuf dm;
    if (dm.alloc(4ull * mod.size())) return DMC_ENOMEM;
    HIP_OK(hipMemcpyAsync(dm.p, mod.data(), 4ull * mod.size(), hipMemcpyHostToDevice, q->stream));
    hipLaunchKernelGGL(k_heap_filter, dim3(1), dim3(64), 0, q->stream, q->tb, q->hd,
                       (uint32_t)mod.size(), (const uint32_t*)dm.u32(),
                       (const uint32_t*)offs.u32(), (const uint8_t*)kp.u8());
    HIP_OK(hipGetLastError());
    HIP_OK(hipStreamSynchronize(q->stream));
    return DMC_OK;
  }
  HIP_OK(hipMemsetAsync(any.p, 0, 4, q->stream));
  hipLaunchKernelGGL(k_list_filter, dim3((N + kBlock - 1) / kBlock), dim3(kBlock), 0,
                     q->stream, q->tb, N, (const uint32_t*)nullptr,
                     (const uint32_t*)offs.u32(), (const uint8_t*)kp.u8(),
                     any.u32());
  uint32_t a = 0;
  HIP_OK(hipMemcpyAsync(&a, any.p, 4, hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  if (any_removed) *any_removed = a != 0;
  return DMC_OK;
}

int dmc_client_erase_batch(dmc_queue* q, uint32_t n, const uint32_t* slots,
                           uint32_t* counts_out, uint64_t* handles_out, uint64_t cap,
                           uint64_t* n_out) {
  if (!q || (n && !slots)) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  if (int rc0 = settle_act(q)) return rc0;
  if (int rc0 = sync_idle(q)) return rc0;
  for (uint32_t i = 0; i < n; ++i) {
    if (slots[i] >= q->p.max_clients) return DMC_EINVAL;
    if (!q->reg_h[slots[i]]) return DMC_ENOTREG;
  }
  {  // distinct slots (a repeat would be erased twice)
    std::vector<uint32_t> v(slots, slots + n);
    std::sort(v.begin(), v.end());
    if (std::adjacent_find(v.begin(), v.end()) != v.end()) return DMC_EINVAL;
  }
  if (n_out) *n_out = 0;
  if (!n) return DMC_OK;
  ++q->gen;
  if (q->heap) {  // delete_from_heaps, in the given order, before the state goes
    if (int rc = heap_list(q, k_heap_remove, std::vector<uint32_t>(slots, slots + n))) return rc;
  }
  DevBuf ds, counts, offs, hs;
  if (ds.alloc(4ull * n) || counts.alloc(4ull * n) || offs.alloc(4ull * n)) return DMC_ENOMEM;
  HIP_OK(hipMemcpyAsync(ds.p, slots, 4ull * n, hipMemcpyHostToDevice, q->stream));
  std::vector<uint32_t> hc;
  uint64_t total = 0;
  if (int rc = list_offsets(q, n, ds.u32(), counts.u32(),
                            offs.u32(), &hc, &total))
    return rc;
  if (counts_out) std::memcpy(counts_out, hc.data(), 4ull * n);
  if (n_out) *n_out = total;
  const uint32_t gb = (n + kBlock - 1) / kBlock;
  if (handles_out && total) {
    if (cap < total) return DMC_EINVAL;
    if (hs.alloc(8ull * total)) return DMC_ENOMEM;
    hipLaunchKernelGGL(k_list_gather, dim3(gb), dim3(kBlock), 0, q->stream, q->tb, n,
                       (const uint32_t*)ds.u32(),
                       (const uint32_t*)offs.u32(), hs.u64());
    HIP_OK(hipMemcpyAsync(handles_out, hs.p, 8ull * total, hipMemcpyDeviceToHost,
                          q->stream));
  }
  hipLaunchKernelGGL(k_list_erase, dim3(gb), dim3(kBlock), 0, q->stream, q->tb, n,
                     (const uint32_t*)ds.u32());
  HIP_OK(hipStreamSynchronize(q->stream));
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t s = slots[i];
    if (q->idle_h[s]) --q->n_idle;
    q->reg_h[s] = 0;
    q->idle_h[s] = 0;
    --q->n_registered;
  }
  return DMC_OK;
}

int dmc_tracker_tally(dmc_queue* q, const dmc_decision* d_dec,
                      const dmc_pull_result* d_result, uint32_t cap,
                      uint32_t* d_comp_delta, uint32_t* d_comp_rho) {
  if (!q) return DMC_EINVAL;
  QueueLock lk(q);
  if (lk.rc) return lk.rc;
  if (!q || !d_result || (cap && (!d_dec || !d_comp_delta || !d_comp_rho)))
    return DMC_EINVAL;
  if (!cap) return DMC_OK;
  hipLaunchKernelGGL(k_tally, dim3(grid_for(cap, 1024)), dim3(kBlock), 0, q->stream,
                     d_dec, d_result, cap, d_comp_delta, d_comp_rho);
  HIP_OK(hipGetLastError());
  return DMC_OK;
}

int dmc_tracker_fill(dmc_queue* q, dmc_request* d_reqs, uint32_t n,
                     const uint32_t* d_client_of_slot, const uint32_t* d_gdelta,
                     const uint32_t* d_grho, uint32_t* d_xd, uint32_t* d_xr,
                     uint8_t* d_known, uint32_t* d_first) {
  if (!q) return DMC_EINVAL;
  QueueLock lk(q);
  if (lk.rc) return lk.rc;
  if (!q || (n && (!d_reqs || !d_gdelta || !d_grho || !d_xd || !d_xr ||
                   !d_known || !d_first)))
    return DMC_EINVAL;
  if (!n) return DMC_OK;
  uint32_t g = (n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(k_track_first, dim3(g), dim3(kBlock), 0, q->stream, d_reqs, n,
                     q->p.max_clients, d_first);
  hipLaunchKernelGGL(k_track_params, dim3(g), dim3(kBlock), 0, q->stream, d_reqs, n,
                     q->p.max_clients, d_client_of_slot, d_gdelta, d_grho, d_xd,
                     d_xr, d_known, d_first);
  HIP_OK(hipGetLastError());
  return DMC_OK;
}


int dmc_tracker_collect_sums(dmc_queue* q, uint32_t n_slots, const uint32_t* d_client_of_slot,
                             const uint32_t* d_comp_delta, const uint32_t* d_comp_rho,
                             uint32_t* d_sum_delta, uint32_t* d_sum_rho) {
  if (!q) return DMC_EINVAL;
  QueueLock lk(q);
  if (lk.rc) return lk.rc;
  if (n_slots > q->p.max_clients) return DMC_EINVAL;
  if (!n_slots) return DMC_OK;
  if (!d_comp_delta || !d_comp_rho || !d_sum_delta || !d_sum_rho) return DMC_EINVAL;
  hipLaunchKernelGGL(k_track_sums, dim3(grid_for(n_slots, 2048)), dim3(kBlock), 0, q->stream,
                     n_slots, d_client_of_slot, d_comp_delta, d_comp_rho, d_sum_delta,
                     d_sum_rho);
  HIP_OK(hipGetLastError());
  return DMC_OK;
}

int dmc_tracker_commit(dmc_queue* q, uint32_t n_slots, uint32_t* d_xd, uint32_t* d_xr,
                       uint32_t* d_comp_delta, uint32_t* d_comp_rho) {
  if (!q) return DMC_EINVAL;
  QueueLock lk(q);
  if (lk.rc) return lk.rc;
  if (n_slots > q->p.max_clients) return DMC_EINVAL;
  if (!n_slots) return DMC_OK;
  if (!d_xd || !d_xr || !d_comp_delta || !d_comp_rho) return DMC_EINVAL;
  hipLaunchKernelGGL(k_track_commit, dim3(grid_for(n_slots, 2048)), dim3(kBlock), 0, q->stream,
                     n_slots, d_xd, d_xr, d_comp_delta, d_comp_rho);
  HIP_OK(hipGetLastError());
  return DMC_OK;
}

int dmc_tracker_collect(dmc_queue* q, uint32_t n_slots,
                        const uint32_t* d_client_of_slot, uint32_t* d_xd,
                        uint32_t* d_xr, uint32_t* d_comp_delta, uint32_t* d_comp_rho,
                        uint32_t* d_sum_delta, uint32_t* d_sum_rho) {
  if (!q) return DMC_EINVAL;
  QueueLock lk(q);
  if (lk.rc) return lk.rc;
  if (!q || n_slots > q->p.max_clients) return DMC_EINVAL;
  if (!n_slots) return DMC_OK;
  if (!d_xd || !d_xr || !d_comp_delta || !d_comp_rho || !d_sum_delta || !d_sum_rho)
    return DMC_EINVAL;
  hipLaunchKernelGGL(k_track_collect, dim3(grid_for(n_slots, 2048)), dim3(kBlock), 0,
                     q->stream, n_slots, d_client_of_slot, d_xd, d_xr, d_comp_delta,
                     d_comp_rho, d_sum_delta, d_sum_rho);
  HIP_OK(hipGetLastError());
  return DMC_OK;
}

int dmc_tracker_advance(dmc_queue* q, uint32_t n_clients, uint32_t* d_gdelta,
                        uint32_t* d_grho, uint32_t* d_sum_delta, uint32_t* d_sum_rho) {
  if (!q) return DMC_EINVAL;
  QueueLock lk(q);
  if (lk.rc) return lk.rc;
  if (!q) return DMC_EINVAL;
  if (!n_clients) return DMC_OK;
  if (!d_gdelta || !d_grho || !d_sum_delta || !d_sum_rho) return DMC_EINVAL;
  hipLaunchKernelGGL(k_track_advance, dim3(grid_for(n_clients, 2048)), dim3(kBlock), 0,
                     q->stream, n_clients, d_gdelta, d_grho, d_sum_delta, d_sum_rho);
  HIP_OK(hipGetLastError());
  return DMC_OK;
}

int dmc_queue_set_option(dmc_queue* q, int option, int64_t value) {
  if (!q) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  switch (option) {
    case DMC_OPT_SMALL_K:
      if (value < 0) return DMC_EINVAL;
      q->small_k = (uint32_t)value;
      return DMC_OK;
    case DMC_OPT_FORCE_RADIX:
      q->force_radix = value != 0;
      return DMC_OK;
    case DMC_OPT_GRAPHS:
      q->use_graphs = value != 0;
      if (!q->use_graphs) return invalidate_graphs(q);
      return DMC_OK;
    case DMC_OPT_ACT_SPLIT:
      q->act_split = value != 0;
      return DMC_OK;
    case DMC_OPT_SINGLE_OP:
      q->single_op = value != 0;
      return DMC_OK;
    case DMC_OPT_BREAK_ROUNDS:
      q->brk_rounds = value != 0;
      return DMC_OK;
    case DMC_OPT_SERVE:
      q->serve_on = value != 0;
      if (q->serve_on != q->serve_reg) serve_register(q, q->serve_on);
      return DMC_OK;
    case DMC_OPT_HEAP_ORDER:
      if (value == 0) return q->heap ? DMC_EINVAL : DMC_OK;
      return heap_enable(q, (uint32_t)value);
    case DMC_OPT_PIPELINE:
      if ((value != 0) == q->pipeline) return DMC_OK;
      if (int rc = invalidate_graphs(q)) return rc;  // (the graphs hold the table's gate)
      q->pipeline = value != 0;
      q->tb.gate = q->pipeline ? q->gate : nullptr;
      return DMC_OK;
    case 9:  // (retired: round 3's DMC_OPT_PREDICT; DMC_ABI_VERSION 5)
      return DMC_EINVAL;
    case DMC_OPT_FAULT:
      if (value < 0) return DMC_EINVAL;
      q->fault = (uint32_t)value;
      return DMC_OK;
    case DMC_OPT_FAIL_ALLOC:
      if (value < 0) return DMC_EINVAL;
      q->fail_allocs = (int)value;
      return DMC_OK;
    case DMC_OPT_SAMPLE:
      if (value < 0 || value > 2) return DMC_EINVAL;
      q->sample_mode = (int)value;
      return invalidate_graphs(q);
      return DMC_OK;
    default:
      return DMC_EINVAL;
  }
}

int dmc_queue_counters(dmc_queue* q, dmc_counters* out, int reset) {
  if (!q || !out) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  // (k_act_hard's count, host-mapped: current once the adds have completed;
  // the device owns the word, a reset moves the host's baseline)
  const uint64_t nhard = q->h_nhard ? *(volatile uint64_t*)q->h_nhard : 0;
  q->ctr.act_seq_batches = nhard - q->nhard_base;
  *out = q->ctr;
  if (reset) {
    q->ctr = dmc_counters{};
    q->nhard_base = nhard;
  }
  return DMC_OK;
}

int dmc_queue_counters_sized(dmc_queue* q, void* out, uint64_t size, int reset) {
  if (!q || !out) return DMC_EINVAL;
  dmc_counters c{};
  if (int rc = dmc_queue_counters(q, &c, reset)) return rc;
  std::memcpy(out, &c, size < sizeof(c) ? (size_t)size : sizeof(c));
  return DMC_OK;
}

int dmc_abi_version(void) { return DMC_ABI_VERSION; }

int dmc_queue_pipelined_error(dmc_queue* q, int clear) {
  if (!q) return DMC_EINVAL;
  std::lock_guard<std::mutex> l(q->mtx);
  const int e = q->pipe_err;
  if (clear) q->pipe_err = 0;
  return e;
}

int dmc_profile_enable(dmc_queue* q, int on) {
  if (!q) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  q->prof_on = on != 0;
  q->prof_n = 0;
  return DMC_OK;
}

int dmc_profile_reset(dmc_queue* q) {
  if (!q) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  for (int i = 0; i < DMC_PROF_NSTAGES; ++i) {
    q->prof_ms[i] = 0.0;
    q->prof_cnt[i] = 0;
  }
  return DMC_OK;
}

int dmc_profile_read(dmc_queue* q, uint32_t stage, uint64_t* count,
                     double* total_ms) {
  if (!q || stage >= DMC_PROF_NSTAGES) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  if (count) *count = q->prof_cnt[stage];
  if (total_ms) *total_ms = q->prof_ms[stage];
  return DMC_OK;
}

const char* dmc_profile_stage_name(uint32_t stage) {
  return stage < DMC_PROF_NSTAGES ? kStageNames[stage] : "";
}

int dmc_stats_get(dmc_queue* q, dmc_stats* out) {
  if (!q || !out) return DMC_EINVAL;
  QueueLock g(q);
  if (g.rc) return g.rc;
  unsigned long long sc[2];
  HIP_OK(hipMemsetAsync(q->reqcount, 0, 8, q->stream));
  hipLaunchKernelGGL(k_count_requests, dim3(grid_for(q->tb.n, 1024)), dim3(kBlock),
                     0, q->stream, q->tb, q->reqcount);
  unsigned long long rq = 0;
  HIP_OK(hipMemcpyAsync(&rq, q->reqcount, 8, hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipMemcpyAsync(sc, q->sched, 16, hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  out->tick = q->tick;
  out->reserv_sched_count = sc[0];
  out->prop_sched_count = sc[1];
  out->limit_break_sched_count = 0;  // never incremented by the reference, :812
  out->clients = q->n_registered;
  out->requests = rq;
  return DMC_OK;
}

}  // extern "C"
