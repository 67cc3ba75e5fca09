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
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <mutex>
#include <vector>

#include "../../include/dmclock_gpu.h"
#include "dmc_device.h"

using namespace dmc;

namespace {

constexpr int kBlock = 256;
constexpr int kHistBins = 2048;
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

// Per-phase selection / bookkeeping block (device resident).
struct Sel {
  uint32_t n_elig;      // eligible fronts
  uint32_t phase;       // 0 = R, 1 = P
  uint64_t kmin, kmax;  // ordered-key range of eligible fronts
  uint64_t T;           // ordered-key threshold (0: nothing, ~0-1: all)
  uint32_t n_cand;      // candidate clients (key <= T)
  uint32_t n_extra;     // entries beyond each candidate's first
  uint32_t n_entries;   // pops (R) / groups (P) to rank
  uint32_t shift;       // 32-bit sort key scaling
  uint32_t n_dec_phase; // decisions taken by this phase
  uint32_t g_last;      // last priority (limit-scan) pull index, kNone if none
  uint32_t terminal;    // 1 if this phase ended the batch early
  uint32_t n_prio_groups; // priority pops applied by phase P
  uint32_t hshift;      // histogram bin of key k: (k - kmin) >> hshift
  uint32_t tbin;        // histogram bin holding T (last bin of the rank table)
  uint32_t bin_ovf;     // a rank bin outgrew kBinCap (skewed keys)
};

// Per-pull-batch control block (device resident): the batched phases read
// their remaining budget from it, so a whole batch runs without host round
// trips.
struct Ctl {
  uint32_t k_total;    // pulls requested
  uint32_t n_dec;      // decisions made so far
  uint32_t overflow;   // an entry buffer was too small: later kernels no-op
  uint32_t terminal;   // eligible work ran out before k_total
  uint32_t nc[2];      // candidates of phase R / P (capacity hints)
  uint32_t nx[2];      // extra entries of phase R / P
  uint32_t next_type;  // DMC_NEXT_* of the stopping pull
  uint32_t pad;
  double when;
  // per-call parameters, published by k_scan<0> (the graph's parameter node)
  double now;
  dmc_decision* out;
  uint64_t tick;
};

struct ScanPart {
  uint32_t cnt, pad;
  uint64_t mn, mx;
};

__device__ inline uint32_t k_left(const Ctl* c) {
  return c->overflow ? 0u : c->k_total - c->n_dec;
}

// Per-call parameters of a pull round: the arguments of its first kernel
// (k_scan<0>, the graph's parameter node), published through Ctl.
struct CallParams {
  uint32_t k_total;
  uint32_t pad;
  double now;
  dmc_decision* out;
  uint64_t tick;
};

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
__global__ void k_register(Table tb, uint32_t n, const uint32_t* slots,
                           const double* rinv, const double* winv,
                           const double* linv, int active, uint64_t tick) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t s = slots[i];
  if (s >= tb.n) return;
  // ClientRec(client, info, tick), dmclock_server.h:381-393
  tb.prev_r[s] = 0.0;
  tb.prev_p[s] = 0.0;
  tb.prev_l[s] = 0.0;
  tb.prev_arr[s] = 0.0;
  tb.r_inv[s] = rinv[i];
  tb.w_inv[s] = winv[i];
  tb.l_inv[s] = linv[i];
  tb.pd[s] = 0.0;
  tb.front_r[s] = 0.0;
  tb.front_p[s] = 0.0;
  tb.front_l[s] = 0.0;
  tb.head[s] = 0;
  tb.count[s] = 0;
  tb.cur_delta[s] = 1;
  tb.cur_rho[s] = 1;
  tb.last_tick[s] = tick;
  tb.flags[s] = F_REG | (active ? 0 : F_IDLE);
}

// ------------------------------------------------------------------ add path
// A batch (a run of add_request_time calls with no activation inside) is
// grouped by client without sorting: k_add_link counts each client's requests
// with one atomic per request and files the first kAddSlots batch positions
// in the client's slot buffer; k_add_chain then lets one thread per client
// replay that client's requests in batch order.  Clients with more than
// kAddSlots requests in the batch (rare: 64K requests over 1M clients is
// Poisson(1/16)) are replayed by a scan of the batch's slot column, in order.
constexpr uint32_t kAddSlots = 16;

struct AddParams {
  const dmc_request* reqs;
  int32_t* rc;
  uint64_t tick_base;
  uint32_t n;
  uint32_t pad;
};

// The first node of an add segment: its arguments are the segment's per-call
// parameters (updated in place on graph replays); block 0 publishes them for
// k_add_chain.
__global__ void k_add_link(AddParams p, Table tb, uint32_t* acnt,
                           uint32_t* abuf, uint32_t* apos, uint32_t* aslot,
                           AddParams* pblk) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) *pblk = p;
  if (i >= p.n) return;
  uint32_t s = p.reqs[i].slot;
  aslot[i] = s;
  if (s >= tb.n) {
    apos[i] = kNone;
    return;
  }
  uint32_t pos = atomicAdd(&acnt[s], 1u);
  apos[i] = pos;
  if (pos < kAddSlots) abuf[(size_t)s * kAddSlots + pos] = i;
}

// do_add_request for one client's requests of the batch, in batch order:
// minus the idle reset (handled before, per activation), initial_tag
// (:878-907), the Reject check (:989-993), the enqueue and cur_rho/cur_delta
// (:995-1009).
struct AddState {
  Tag3 prev;
  double rinv, winv, linv;
  uint32_t head, count, cd, cr;
  uint64_t last_tick;
  uint8_t flags;
  bool front_set;
  Tag3 front;
};

__device__ inline void add_one(const Table& tb, AddState& st, ReqEntry* ring,
                               const AddParams& p, uint32_t pos) {
  const dmc_request rq = p.reqs[pos];
  uint64_t tick = p.tick_base + pos + 1;  // ++tick, :918
  if (rq.rho > rq.delta) {  // ReqParams asserts rho <= delta
    p.rc[pos] = DMC_EBADPARAMS;
    return;
  }
  if (st.count >= tb.q) {  // documented deviation: bounded ring
    p.rc[pos] = DMC_EQUEUEFULL;
    return;
  }
  Tag3 tag;
  if (!tb.delayed || st.count == 0) {
    if (!make_tag(st.prev, st.rinv, st.winv, st.linv, rq.delta, rq.rho, rq.time,
                  rq.cost, tb.antic, &tag)) {
      p.rc[pos] = DMC_EBADTAG;
      return;
    }
    // update_req_tag, :405-412
    assign_unpinned(st.prev.r, tag.r);
    assign_unpinned(st.prev.l, tag.l);
    assign_unpinned(st.prev.p, tag.p);
    st.prev.arrival = tag.arrival;
    st.last_tick = tick;
  } else {
    if (rq.cost == 0) {
      p.rc[pos] = DMC_EBADTAG;
      return;
    }
    tag = Tag3{0.0, 0.0, 0.0, rq.time};  // placeholder, :880
  }
  if (tb.at_limit == DMC_AT_LIMIT_REJECT &&
      tag.l > __dadd_rn(rq.time, tb.reject_thr)) {
    p.rc[pos] = DMC_EAGAIN;
    return;
  }
  ReqEntry e;
  e.r = tag.r;
  e.p = tag.p;
  e.l = tag.l;
  e.arrival = tag.arrival;
  e.handle = rq.handle;
  e.cost = rq.cost;
  e.delta = (tb.delayed && st.count > 0) ? 0u : rq.delta;
  e.rho = (tb.delayed && st.count > 0) ? 0u : rq.rho;
  e.pad = 0;
  e.pad2 = 0;
  ring[(st.head + st.count) & tb.qmask] = e;
  if (st.count == 0) {
    st.front = tag;
    st.front_set = true;
    st.flags &= (uint8_t)~F_READY;  // a new tag is not ready, :155
  }
  ++st.count;
  st.cd = rq.delta;
  st.cr = rq.rho;
  p.rc[pos] = DMC_OK;
}

__global__ void k_add_chain(Table tb, const AddParams* pblk, uint32_t* acnt,
                            const uint32_t* abuf, const uint32_t* apos,
                            const uint32_t* aslot) {
  const AddParams p = *pblk;
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  uint32_t pos0 = apos[i];
  if (pos0 == kNone) {
    p.rc[i] = DMC_ENOTREG;
    return;
  }
  if (pos0 != 0) return;  // the client's first filer replays its requests
  uint32_t s = aslot[i];
  uint32_t m = acnt[s];
  acnt[s] = 0;  // ready for the next batch
  if (!(tb.flags[s] & F_REG)) {
    if (m <= kAddSlots) {
      for (uint32_t j = 0; j < m; ++j) p.rc[abuf[(size_t)s * kAddSlots + j]] = DMC_ENOTREG;
    } else {
      for (uint32_t j = 0; j < p.n; ++j)
        if (aslot[j] == s) p.rc[j] = DMC_ENOTREG;
    }
    return;
  }
  AddState st;
  st.prev = Tag3{tb.prev_r[s], tb.prev_p[s], tb.prev_l[s], tb.prev_arr[s]};
  st.rinv = tb.r_inv[s];
  st.winv = tb.w_inv[s];
  st.linv = tb.l_inv[s];
  st.head = tb.head[s];
  st.count = tb.count[s];
  st.cd = tb.cur_delta[s];
  st.cr = tb.cur_rho[s];
  st.last_tick = tb.last_tick[s];
  st.flags = tb.flags[s];
  st.front_set = false;
  ReqEntry* ring = tb.ring + (size_t)s * tb.q;
  if (m == 1) {
    add_one(tb, st, ring, p, i);
  } else if (m <= kAddSlots) {
    // the client's batch positions in ascending order, by repeated selection
    // over its (L2-resident) slot-buffer row
    const uint32_t* row = abuf + (size_t)s * kAddSlots;
    uint32_t last = 0;
    for (uint32_t j = 0; j < m; ++j) {
      uint32_t next = 0xffffffffu;
      for (uint32_t k = 0; k < m; ++k) {
        uint32_t v = row[k];
        if ((j == 0 || v > last) && v < next) next = v;
      }
      add_one(tb, st, ring, p, next);
      last = next;
    }
  } else {
    for (uint32_t j = 0; j < p.n; ++j)
      if (aslot[j] == s) add_one(tb, st, ring, p, j);
  }
  tb.prev_r[s] = st.prev.r;
  tb.prev_p[s] = st.prev.p;
  tb.prev_l[s] = st.prev.l;
  tb.prev_arr[s] = st.prev.arrival;
  tb.count[s] = st.count;
  tb.cur_delta[s] = st.cd;
  tb.cur_rho[s] = st.cr;
  tb.last_tick[s] = st.last_tick;
  tb.flags[s] = st.flags;
  if (st.front_set) {
    tb.front_r[s] = st.front.r;
    tb.front_p[s] = st.front.p;
    tb.front_l[s] = st.front.l;
  }
}

// idle reset, :937-985: L = min over non-idle clients of
// (has_request ? front.p : prev.p) + prop_delta
__global__ void k_contrib_min(Table tb, uint64_t* parts) {
  uint64_t m = kMaxKey;
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < tb.n;
       s += gridDim.x * blockDim.x) {
    uint8_t f = tb.flags[s];
    if ((f & F_REG) && !(f & F_IDLE)) {
      double p = tb.count[s] ? tb.front_p[s] : tb.prev_p[s];
      uint64_t k = okey(__dadd_rn(p, tb.pd[s]));
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
  if (lowest < trigger) tb.pd[s] = __dsub_rn(lowest, t);
  tb.flags[s] &= (uint8_t)~F_IDLE;
}

// ------------------------------------------------------------------ pull: scans
// Phase R scan: key = front reservation tag, eligible iff r <= now.
// Phase P scan: first commits the limit scan of the first priority pull
// (:1135-1144: every front with limit <= now becomes ready), then
// key = p + prop_delta, eligible iff ready and p < inf (:1146-1151).
// Nothing runs once the batch is complete (no further pull took place).
// Per-block partials (count, min, max) go to `parts`: no same-address
// atomics (thousands of waves hitting one word serialise at the memory side).
template <int PH>
__global__ void k_scan(Table tb, uint64_t* keys, ScanPart* parts, Ctl* ctl,
                       CallParams cp) {
  if (PH == 0) {  // the round's first kernel: publish the call's parameters
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      Ctl c{};
      c.k_total = cp.k_total;
      c.next_type = DMC_NEXT_RETURNING;
      c.now = cp.now;
      c.out = cp.out;
      c.tick = cp.tick;
      *ctl = c;
    }
    if (cp.k_total == 0) return;
  } else if (k_left(ctl) == 0) {
    return;
  }
  const double now = PH == 0 ? cp.now : ctl->now;
  uint32_t cnt = 0;
  uint64_t mn = kMaxKey, mx = 0;
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < tb.n;
       s += gridDim.x * blockDim.x) {
    uint64_t k = kMaxKey;
    uint32_t c = tb.count[s];
    if (c) {
      if (PH == 0) {
        double r = tb.front_r[s];
        if (r <= now) k = okey(r);
      } else {
        uint8_t f = tb.flags[s];
        bool rdy = (f & F_READY) != 0;
        if (!rdy && tb.front_l[s] <= now) {
          rdy = true;
          tb.flags[s] = f | F_READY;
        }
        double p = tb.front_p[s];
        if (rdy && p < kInf) k = okey(__dadd_rn(p, tb.pd[s]));
      }
    }
    keys[s] = k;
    if (k != kMaxKey) {
      ++cnt;
      mn = k < mn ? k : mn;
      mx = k > mx ? k : mx;
    }
  }
  cnt = wave_sum_u32(cnt);
  mn = wave_min_u64(mn);
  mx = wave_max_u64(mx);
  __shared__ ScanPart sh[kBlock / 64];
  int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sh[w] = ScanPart{cnt, 0, mn, mx};
  __syncthreads();
  if (threadIdx.x == 0) {
    ScanPart o = sh[0];
    for (int i = 1; i < (int)(blockDim.x / 64); ++i) {
      o.cnt += sh[i].cnt;
      o.mn = sh[i].mn < o.mn ? sh[i].mn : o.mn;
      o.mx = sh[i].mx > o.mx ? sh[i].mx : o.mx;
    }
    parts[blockIdx.x] = o;
  }
}

// block-wide reduction of the scan partials (every thread gets the result)
__device__ inline ScanPart reduce_parts(const ScanPart* parts, uint32_t nparts) {
  __shared__ ScanPart sh[1024];
  ScanPart o{0, 0, kMaxKey, 0};
  for (uint32_t i = threadIdx.x; i < nparts; i += blockDim.x) {
    ScanPart b = parts[i];
    o.cnt += b.cnt;
    o.mn = b.mn < o.mn ? b.mn : o.mn;
    o.mx = b.mx > o.mx ? b.mx : o.mx;
  }
  sh[threadIdx.x] = o;
  __syncthreads();
  for (int d = blockDim.x / 2; d > 0; d >>= 1) {
    if ((int)threadIdx.x < d) {
      ScanPart& a = sh[threadIdx.x];
      const ScanPart& b = sh[threadIdx.x + d];
      a.cnt += b.cnt;
      a.mn = b.mn < a.mn ? b.mn : a.mn;
      a.mx = b.mx > a.mx ? b.mx : a.mx;
    }
    __syncthreads();
  }
  ScanPart r = sh[0];
  __syncthreads();
  return r;
}

__device__ inline uint32_t hist_shift(uint64_t range) {
  // smallest shift with (range >> shift) < kHistBins
  uint32_t bits = range ? 64 - __clzll((long long)range) : 0;
  uint32_t hb = 11;  // log2(kHistBins)
  return bits > hb ? bits - hb : 0;
}

// Histogram of eligible keys over [kmin, kmax] in kHistBins integer buckets
// of the ordered-key space (monotone in the key), with the max key per
// bucket.  kHistBlocks blocks of 1024 threads: few enough that the global
// flush (one atomic per non-empty bin per block) stays cheap.
constexpr int kHistBlocks = 128;
__global__ void __launch_bounds__(1024)
k_hist(uint32_t n, const uint64_t* keys, const ScanPart* parts,
       uint32_t nparts, const Ctl* ctl, uint32_t* hist, uint64_t* hmax) {
  uint32_t k_rem = k_left(ctl);
  if (k_rem == 0) return;
  ScanPart tot = reduce_parts(parts, nparts);
  if (tot.cnt == 0) return;  // (also feeds the rank bins when cnt <= k_rem)
  __shared__ uint32_t sh[kHistBins];
  __shared__ unsigned long long smx[kHistBins];
  for (int b = threadIdx.x; b < kHistBins; b += blockDim.x) {
    sh[b] = 0;
    smx[b] = 0;
  }
  __syncthreads();
  uint64_t kmin = tot.mn;
  uint32_t sh_ = hist_shift(tot.mx - kmin);
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < n;
       s += gridDim.x * blockDim.x) {
    uint64_t k = keys[s];
    if (k == kMaxKey) continue;
    uint32_t b = (uint32_t)((k - kmin) >> sh_);
    atomicAdd(&sh[b], 1u);
    atomicMax(&smx[b], (unsigned long long)k);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < kHistBins; b += blockDim.x) {
    if (sh[b]) {
      atomicAdd(&hist[b], sh[b]);
      atomicMax((unsigned long long*)&hmax[b], smx[b]);
    }
  }
}

// Threshold T: every key <= T is a candidate and at least k_rem eligible
// fronts are <= T (T is the largest key of the bin holding the k_rem-th
// smallest), or everything when no more than k_rem are eligible.  Also
// (re)initialises the phase's Sel and builds the rank-bin table: the kNB rank
// bins are spread over the histogram bins up to T's bin in proportion to
// their counts (each gets 1 + its share), so that the rank bins stay small
// however the keys are distributed (the rank pass is quadratic per bin).
// kPickThreads threads; each owns kHistBins / kPickThreads bins.
constexpr int kNB = 4096;  // rank bins
constexpr int kPickThreads = 1024;
constexpr int kBinsPerThread = kHistBins / kPickThreads;
__device__ inline uint32_t block_excl_scan_1024(uint32_t v, uint32_t* wsum,
                                                uint32_t* total) {
  int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t incl = v;
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t o = __shfl_up(incl, d);
    if (lane >= d) incl += o;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  uint32_t wbase = 0, tot = 0;
  for (int i = 0; i < kPickThreads / 64; ++i) {
    if (i < w) wbase += wsum[i];
    tot += wsum[i];
  }
  __syncthreads();
  if (total) *total = tot;
  return wbase + incl - v;
}

__global__ void __launch_bounds__(kPickThreads)
k_pick(const ScanPart* parts, uint32_t nparts, Sel* sel, const Ctl* ctl,
       uint32_t* hist, uint64_t* hmax, uint32_t phase, uint32_t* sbase,
       uint32_t* snum) {
  __shared__ uint32_t wsum[kPickThreads / 64];
  __shared__ uint32_t s_tb, s_C;
  uint32_t k_rem = k_left(ctl);
  ScanPart tot = reduce_parts(parts, nparts);
  uint32_t ne = k_rem ? tot.cnt : 0;
  int t = threadIdx.x;
  uint32_t sh1 = hist_shift(tot.mx - tot.mn);
  if (t == 0) {
    Sel z{};
    z.n_elig = ne;
    z.phase = phase;
    z.kmin = tot.mn;
    z.kmax = tot.mx;
    z.g_last = kNone;
    z.T = (k_rem == 0 || ne == 0) ? 0 : kMaxKey - 1;
    z.hshift = sh1;
    z.tbin = ne ? (uint32_t)((tot.mx - tot.mn) >> sh1) : 0;
    *sel = z;
    s_tb = z.tbin;
    s_C = 0;
  }
  uint32_t h[kBinsPerThread];
  uint32_t local = 0;
  for (int j = 0; j < kBinsPerThread; ++j) {
    h[j] = hist[t * kBinsPerThread + j];
    local += h[j];
  }
  uint32_t before = block_excl_scan_1024(local, wsum, nullptr);
  if (k_rem && ne > k_rem && before < k_rem && before + local >= k_rem) {
    uint32_t cum = before;
    for (int j = 0; j < kBinsPerThread; ++j) {
      cum += h[j];
      if (cum >= k_rem) {
        sel->T = hmax[t * kBinsPerThread + j];
        sel->tbin = t * kBinsPerThread + j;
        s_tb = t * kBinsPerThread + j;
        break;
      }
    }
  }
  __syncthreads();
  uint32_t tb = s_tb;
  {
    uint32_t cum = before;
    for (int j = 0; j < kBinsPerThread; ++j) {
      cum += h[j];
      if ((uint32_t)(t * kBinsPerThread + j) == tb) s_C = cum;
    }
  }
  __syncthreads();
  uint32_t C = s_C > 0 ? s_C : 1;
  uint32_t S = kNB - (tb + 1);
  uint32_t ns[kBinsPerThread], lns = 0;
  for (int j = 0; j < kBinsPerThread; ++j) {
    uint32_t b = t * kBinsPerThread + j;
    ns[j] = b <= tb ? 1u + (uint32_t)((uint64_t)h[j] * S / C) : 0u;
    lns += ns[j];
  }
  uint32_t nb = block_excl_scan_1024(lns, wsum, nullptr);
  for (int j = 0; j < kBinsPerThread; ++j) {
    uint32_t b = t * kBinsPerThread + j;
    sbase[b] = nb;
    snum[b] = ns[j];
    nb += ns[j];
    hist[b] = 0;
    hmax[b] = 0;
  }
}

// Rank bin of an entry key (monotone in the key): its histogram bin's share
// of the kNB rank bins, split linearly (k_pick's table).
__device__ inline uint32_t rank_bin(uint64_t k, uint64_t kmin, uint32_t sh1,
                                    uint32_t tb, const uint32_t* sbase,
                                    const uint32_t* snum) {
  uint64_t d = k > kmin ? k - kmin : 0;
  uint64_t hb = d >> sh1;
  uint32_t h = hb > tb ? tb : (uint32_t)hb;
  uint64_t lo = d - ((uint64_t)h << sh1);
  uint32_t ns = snum[h];
  uint64_t sub = sh1 <= 51 ? (lo * ns) >> sh1 : ((lo >> 12) * ns) >> (sh1 - 12);
  if (sub >= ns) sub = ns - 1;
  return sbase[h] + (uint32_t)sub;
}

// ------------------------------------------------------------------ pull: walks
struct CountVisit {
  uint32_t pops = 0, groups = 0;
  __device__ void pop(uint32_t, const Tag3&, uint32_t, uint64_t, bool) { ++pops; }
  __device__ void group(uint64_t, uint32_t) { ++groups; }
};

// Entry id of the j-th entry of candidate i: the first lives at i, the rest
// in the extras region (after cap1) at the candidate's extras base.
__device__ inline uint32_t entry_id(uint32_t i, uint32_t j, uint32_t cap1,
                                    uint32_t xbase) {
  return j == 0 ? i : cap1 + xbase + j - 1;
}

// Rank-bin record of one entry (bin-rank path): the full order key
// (okey, slot, seq), the group's run (P) and the entry id.
constexpr uint32_t kBinCap = 256;  // entries per rank bin (more: bin_ovf)
struct BRec {
  uint64_t okey;
  uint32_t slot;
  uint32_t e;
  uint32_t seq;
  uint32_t run;
};

struct EmitVisit {
  uint64_t* eokey;
  uint32_t* eslot;
  uint32_t* eseq;
  uint32_t* erun;
  uint32_t i, cap1, xbase, cap2, slot;
  int ph;
  // bin-rank path (brec != nullptr): k_pick's rank-bin table
  BRec* brec;
  uint32_t* bcount;
  uint32_t* bsize;
  const uint32_t* sbase;
  const uint32_t* snum;
  uint64_t kmin;
  uint32_t sh1, tbin;
  Sel* sel;
  uint32_t n = 0;
  uint64_t kmax = 0;
  uint32_t q = 0;  // bin-rank path: entry id = candidate * q + n
  __device__ void put(uint64_t key, uint32_t run) {
    if (brec) {
      if (i < cap1) {
        uint32_t e = i * q + n;
        uint32_t b = rank_bin(key, kmin, sh1, tbin, sbase, snum);
        uint32_t pos = atomicAdd(&bcount[b], 1u);
        atomicAdd(&bsize[b], ph == 0 ? 1u : 1u + run);
        if (pos < kBinCap)
          brec[(size_t)b * kBinCap + pos] = BRec{key, slot, e, n, run};
        else
          sel->bin_ovf = 1;
      }
    } else if (n == 0 ? i < cap1 : xbase + n - 1 < cap2) {
      uint32_t e = entry_id(i, n, cap1, xbase);
      {
        eokey[e] = key;
        eslot[e] = slot;
        eseq[e] = n;
        erun[e] = run;
      }
    }
    kmax = key > kmax ? key : kmax;
    ++n;
  }
  __device__ void pop(uint32_t, const Tag3& t, uint32_t, uint64_t, bool) {
    if (ph == 0) put(okey(t.r), 0);
  }
  __device__ void group(uint64_t key, uint32_t run) { put(key, run); }
};

// Candidates = slots whose key <= T, compacted (any order: the final order
// is fixed by the ranking on full keys).  kCandBlocks blocks, one atomic each.
constexpr int kCandBlocks = 256;
__global__ void k_cand(uint32_t n, const uint64_t* keys, Sel* sel,
                       uint32_t* cand) {
  __shared__ uint32_t wsum[kBlock / 64];
  __shared__ uint32_t base;
  uint64_t T = sel->T;
  if (T == 0) return;
  uint32_t per = (n + gridDim.x - 1) / gridDim.x;
  uint32_t lo = blockIdx.x * per, hi = lo + per < n ? lo + per : n;
  // pass 1: count
  uint32_t c = 0;
  for (uint32_t s = lo + threadIdx.x; s < hi; s += blockDim.x) c += keys[s] <= T;
  uint32_t incl = c;
  int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t o = __shfl_up(incl, d);
    if (lane >= d) incl += o;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  uint32_t wb = 0, tot = 0;
  for (int i = 0; i < (int)(blockDim.x / 64); ++i) {
    if (i < w) wb += wsum[i];
    tot += wsum[i];
  }
  if (threadIdx.x == 0) base = tot ? atomicAdd(&sel->n_cand, tot) : 0;
  __syncthreads();
  uint32_t o = base + wb + incl - c;
  for (uint32_t s = lo + threadIdx.x; s < hi; s += blockDim.x)
    if (keys[s] <= T) cand[o++] = s;
}

// One thread per candidate enumerates its entries (R: pops with
// r <= min(now, T); P: groups with key <= T) and emits (key, slot, seq, run).
// Bin-rank path (BIN): each entry goes straight to its rank bin, with entry id
// candidate * q + seq (no allocation needed).  Radix path: a counting walk
// first, extras allocated with one atomic per block, then the entries go to
// the entry arrays; per-block max key to emax[] for the 32-bit key scaling.
template <int PH, bool BIN>
__global__ void __launch_bounds__(kBlock)
k_emit(Table tb, Sel* sel, const Ctl* ctl, const uint32_t* cand, uint32_t cap1,
       uint32_t cap2, uint32_t* cxbase, uint64_t* eokey, uint32_t* eslot,
       uint32_t* eseq, uint32_t* erun, uint64_t* emax, BRec* brec,
       uint32_t* bcount, uint32_t* bsize, const uint32_t* sbase,
       const uint32_t* snum) {
  __shared__ uint32_t wsum[kBlock / 64];
  __shared__ uint32_t base;
  __shared__ unsigned long long bmax;
  uint32_t nc = sel->n_cand;
  if (blockIdx.x * blockDim.x >= nc || ctl->overflow) return;
  const double now = ctl->now;
  uint64_t T = sel->T;
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t s = i < nc ? cand[i] : 0;
  if (BIN) {
    if (i >= nc) return;
    EmitVisit v{nullptr, nullptr, nullptr, nullptr, i, cap1, 0, cap2, s, PH,
                brec, bcount, bsize, sbase, snum, sel->kmin, sel->hshift,
                sel->tbin, sel};
    v.q = tb.q;
    if (PH == 0)
      walk_r(tb, s, now, T, 0xffffffffu, v, nullptr, nullptr, nullptr);
    else
      walk_p(tb, s, now, T, 0xffffffffu, v, nullptr, nullptr, nullptr);
    return;
  }
  uint32_t c = 0;
  if (i < nc) {
    CountVisit v;
    c = PH == 0 ? walk_r(tb, s, now, T, 0xffffffffu, v, nullptr, nullptr, nullptr)
                : walk_p(tb, s, now, T, 0xffffffffu, v, nullptr, nullptr, nullptr).groups;
  }
  uint32_t x = c ? c - 1 : 0;
  uint32_t incl = x;
  int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t o = __shfl_up(incl, d);
    if (lane >= d) incl += o;
  }
  if (lane == 63) wsum[w] = incl;
  if (threadIdx.x == 0) bmax = 0;
  __syncthreads();
  uint32_t wb = 0, tot = 0;
  for (int k = 0; k < (int)(blockDim.x / 64); ++k) {
    if (k < w) wb += wsum[k];
    tot += wsum[k];
  }
  if (threadIdx.x == 0) base = tot ? atomicAdd(&sel->n_extra, tot) : 0;
  __syncthreads();
  uint32_t xb = base + wb + incl - x;
  if (i < nc) {
    cxbase[i] = xb;
    EmitVisit v{eokey, eslot, eseq, erun, i, cap1, xb, cap2, s, PH,
                nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, 0, sel};
    if (PH == 0)
      walk_r(tb, s, now, T, 0xffffffffu, v, nullptr, nullptr, nullptr);
    else
      walk_p(tb, s, now, T, 0xffffffffu, v, nullptr, nullptr, nullptr);
    atomicMax(&bmax, (unsigned long long)v.kmax);
  }
  __syncthreads();
  if (threadIdx.x == 0) emax[blockIdx.x] = bmax;
}

// 32-bit sort keys: (okey - kmin) >> shift with the smallest shift that keeps
// every real key below 0xffffffff; padding entries get 0xffffffff.  Pads are
// region-1 ids in [n_cand, cap1) and region-2 ids past the extras.
__global__ void k_key32(Sel* sel, Ctl* ctl, uint32_t cap1, uint32_t cap2,
                        const uint64_t* emax, uint32_t nemax,
                        const uint64_t* eokey, uint32_t* ek32, uint32_t* eval) {
  __shared__ unsigned long long sh[kBlock];
  uint32_t nc = sel->n_cand, nx = sel->n_extra;
  bool ovf = ctl->overflow || nc > cap1 || nx > cap2;
  uint64_t m = 0;
  uint32_t nb = (nc + kBlock - 1) / kBlock;  // emit blocks that ran
  if (nb < nemax) nemax = nb;
  for (uint32_t b = threadIdx.x; b < nemax; b += blockDim.x)
    m = emax[b] > m ? emax[b] : m;
  sh[threadIdx.x] = m;
  __syncthreads();
  for (int d = blockDim.x / 2; d > 0; d >>= 1) {
    if ((int)threadIdx.x < d && sh[threadIdx.x + d] > sh[threadIdx.x])
      sh[threadIdx.x] = sh[threadIdx.x + d];
    __syncthreads();
  }
  uint64_t kmin = sel->kmin;
  uint64_t range = sh[0] > kmin ? sh[0] - kmin : 0;
  uint32_t shift = 0;
  while ((range >> shift) >= 0xffffffffull) ++shift;
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid == 0) {
    sel->n_entries = ovf ? 0 : nc + nx;
    sel->shift = shift;
    ctl->nc[sel->phase] = nc;
    ctl->nx[sel->phase] = nx;
    if (ovf) ctl->overflow = 1;
  }
  uint32_t E = cap1 + cap2;
  for (uint32_t e = tid; e < E; e += gridDim.x * blockDim.x) {
    bool real = !ovf && (e < nc || (e >= cap1 && e < cap1 + nx));
    uint64_t k = real ? eokey[e] : 0;
    ek32[e] = !real ? 0xffffffffu
                    : (k > kmin ? (uint32_t)((k - kmin) >> shift) : 0u);
    eval[e] = e;
  }
}

// Full order among entries: (okey, slot, seq).
__device__ inline bool ent_less(uint32_t a, uint32_t b, const uint64_t* eokey,
                                const uint32_t* eslot, const uint32_t* eseq) {
  if (eokey[a] != eokey[b]) return eokey[a] < eokey[b];
  if (eslot[a] != eslot[b]) return eslot[a] < eslot[b];
  return eseq[a] < eseq[b];
}

// After the 32-bit radix sort, runs of equal 32-bit keys are ordered by the
// full key (insertion sort by the run's first thread; runs are short).
__global__ void k_fixup(const Sel* sel, const uint32_t* sk32, uint32_t* sval,
                        const uint64_t* eokey, const uint32_t* eslot,
                        const uint32_t* eseq) {
  uint32_t n = sel->n_entries;
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < n;
       p += gridDim.x * blockDim.x) {
    if (p > 0 && sk32[p - 1] == sk32[p]) continue;
    uint32_t q = p + 1;
    while (q < n && sk32[q] == sk32[p]) ++q;
    for (uint32_t a = p + 1; a < q; ++a) {
      uint32_t v = sval[a];
      uint32_t b = a;
      while (b > p && ent_less(v, sval[b - 1], eokey, eslot, eseq)) {
        sval[b] = sval[b - 1];
        --b;
      }
      sval[b] = v;
    }
  }
}

__device__ inline bool tie_at(const uint64_t* eokey, const uint32_t* sval,
                              const uint32_t* eslot, uint32_t n, uint32_t pos) {
  uint32_t e = sval[pos];
  if (pos > 0) {
    uint32_t f = sval[pos - 1];
    if (eokey[f] == eokey[e] && eslot[f] != eslot[e]) return true;
  }
  if (pos + 1 < n) {
    uint32_t f = sval[pos + 1];
    if (eokey[f] == eokey[e] && eslot[f] != eslot[e]) return true;
  }
  return false;
}

// R: the first k_rem sorted pops are dispatched in sorted order.
__global__ void k_decide_r(const Ctl* ctl, const uint64_t* eokey,
                           const uint32_t* sval, const uint32_t* eslot,
                           uint32_t* eoff, uint8_t* etie, uint32_t* applied,
                           Sel* sel) {
  if (ctl->overflow) return;
  uint32_t n = sel->n_entries, k_rem = k_left(ctl), n_dec = ctl->n_dec;
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid == 0) {
    sel->n_dec_phase = n < k_rem ? n : k_rem;
    sel->terminal = 0;
  }
  for (uint32_t pos = tid; pos < n; pos += gridDim.x * blockDim.x) {
    uint32_t e = sval[pos];
    if (pos < k_rem) {
      eoff[e] = n_dec + pos;
      etie[e] = tie_at(eokey, sval, eslot, n, pos) ? 1 : 0;
      atomicAdd(&applied[eslot[e]], 1u);
    } else {
      eoff[e] = kNone;
    }
  }
}

__global__ void k_group_sizes(const Ctl* ctl, const Sel* sel, uint32_t E,
                              const uint32_t* sval, const uint32_t* erun,
                              uint32_t* gsz) {
  uint32_t n = (!ctl->overflow) ? sel->n_entries : 0;
  for (uint32_t pos = blockIdx.x * blockDim.x + threadIdx.x; pos < E;
       pos += gridDim.x * blockDim.x)
    gsz[pos] = pos < n ? 1 + erun[sval[pos]] : 0;
}

// P: groups (priority pop + the reservation run it exposes) in key order;
// decisions are the prefix of their concatenation up to k_rem.
__global__ void k_decide_p(const Ctl* ctl, const uint64_t* eokey,
                           const uint32_t* sval, const uint32_t* eslot,
                           const uint32_t* gsz, const uint32_t* goff,
                           uint32_t* eoff, uint8_t* etie, uint32_t* applied,
                           Sel* sel) {
  if (ctl->overflow) return;
  uint32_t n = sel->n_entries, k_rem = k_left(ctl), n_dec = ctl->n_dec;
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (n == 0) {
    if (tid == 0) {
      sel->n_dec_phase = 0;
      sel->terminal = k_rem > 0 ? 1 : 0;
    }
    return;
  }
  for (uint32_t pos = tid; pos < n; pos += gridDim.x * blockDim.x) {
    uint32_t e = sval[pos];
    uint32_t o = goff[pos];
    if (pos == n - 1) {
      uint32_t tot = o + gsz[pos];
      sel->n_dec_phase = tot < k_rem ? tot : k_rem;
      sel->terminal = tot < k_rem ? 1 : 0;
    }
    if (o < k_rem) {
      eoff[e] = n_dec + o;
      etie[e] = tie_at(eokey, sval, eslot, n, pos) ? 1 : 0;
      uint32_t na = gsz[pos];
      if (na > k_rem - o) na = k_rem - o;
      atomicAdd(&applied[eslot[e]], na);
      if (pos == n - 1 || goff[pos + 1] >= k_rem) {
        // the last applied group: its priority pop is this phase's last
        // limit-scanning pull
        sel->g_last = n_dec + o;
        sel->n_prio_groups = pos + 1;
      }
    } else {
      eoff[e] = kNone;
    }
  }
}

// ---------------------------------------------------------- pull: bin-rank
// Ranking the entries without a general sort: k_emit files each entry in its
// rank bin (k_pick's table: monotone in the key, balanced over the keys'
// histogram); an entry's rank is the number of entries in earlier bins plus
// those of its own bin that precede it in the full order (okey, slot, seq).
// One wave per bin ranks it in LDS; each block first sums the counts and
// group sizes of all earlier bins.  The same pass yields the group-size prefix
// (P) and the tie flag, and decides.  A bin past kBinCap (bin_ovf) aborts the
// batch (ctl->overflow = 2); the host then redoes it through the radix path.
constexpr int kRankBins = kBlock / 64;        // bins per block (one per wave)
constexpr int kRankBlocks = kNB / kRankBins;  // 1024
template <int PH>
__global__ void __launch_bounds__(kBlock)
k_rank(Sel* sel, Ctl* ctl, uint32_t cap1, uint32_t cap2, const uint32_t* bcount,
       const uint32_t* bsize, const BRec* brec, uint32_t* eoff, uint8_t* etie,
       uint32_t* applied) {
  __shared__ BRec sh[kBlock / 64][kBinCap];
  __shared__ uint32_t s_off[kRankBins], s_soff[kRankBins], s_cnt[kRankBins];
  __shared__ uint32_t s_pc[kBlock / 64], s_ps[kBlock / 64];
  __shared__ uint32_t s_tc[kBlock / 64], s_ts[kBlock / 64], s_ne;
  uint32_t nc = sel->n_cand, nx = 0;  // (no extra-entry region on this path)
  bool ovf = ctl->overflow || nc > cap1 || sel->bin_ovf;
  bool last = blockIdx.x == 0;
  uint32_t k_rem = k_left(ctl), n_dec = ctl->n_dec;
  if (ovf) {
    if (last && threadIdx.x == 0) {
      sel->n_entries = 0;
      ctl->nc[PH] = nc;
      ctl->nx[PH] = nx;
      if (!ctl->overflow)
        ctl->overflow = nc <= cap1 ? 2u : 1u;
    }
    return;
  }
  uint32_t b0 = blockIdx.x * kRankBins;
  // entries and group sizes of all bins before b0, and in all bins
  uint32_t pc = 0, ps = 0, tc = 0, ts = 0;
  for (uint32_t b = threadIdx.x; b < (uint32_t)kNB; b += kBlock) {
    uint32_t c = bcount[b], z = bsize[b];
    if (b < b0) {
      pc += c;
      ps += z;
    }
    tc += c;
    ts += z;
  }
  pc = wave_sum_u32(pc);
  ps = wave_sum_u32(ps);
  tc = wave_sum_u32(tc);
  ts = wave_sum_u32(ts);
  int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    s_pc[w] = pc;
    s_ps[w] = ps;
    s_tc[w] = tc;
    s_ts[w] = ts;
  }
  if (threadIdx.x < kRankBins) s_cnt[threadIdx.x] = bcount[b0 + threadIdx.x];
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t PC = 0, PS = 0, TC = 0, TS = 0;
    for (int k = 0; k < kBlock / 64; ++k) {
      PC += s_pc[k];
      PS += s_ps[k];
      TC += s_tc[k];
      TS += s_ts[k];
    }
    s_ne = TC;
    for (int k = 0; k < kRankBins; ++k) {
      s_off[k] = PC;
      s_soff[k] = PS;
      PC += s_cnt[k];
      PS += bsize[b0 + k];
    }
    if (last) {  // totals: the phase's decision count, terminal flag
      sel->n_entries = TC;
      ctl->nc[PH] = nc;
      ctl->nx[PH] = nx;
      sel->n_dec_phase = TS < k_rem ? TS : k_rem;
      sel->terminal = (PH == 1 && TS < k_rem) ? 1 : 0;
    }
  }
  __syncthreads();
  const uint32_t ne = s_ne;
  for (int j = 0; j < kRankBins / (kBlock / 64); ++j) {
    uint32_t lb = w * (kRankBins / (kBlock / 64)) + j;
    uint32_t b = b0 + lb;
    uint32_t cnt = s_cnt[lb];
    const BRec* src = brec + (size_t)b * kBinCap;
    for (uint32_t q = lane; q < cnt; q += 64) sh[w][q] = src[q];
    __syncthreads();
    for (uint32_t q = lane; q < cnt; q += 64) {
      BRec me = sh[w][q];
      uint32_t rank = 0, gl = 0;
      bool tie = false;
      for (uint32_t f = 0; f < cnt; ++f) {
        if (f == q) continue;
        const BRec& o = sh[w][f];
        bool less = o.okey < me.okey ||
                    (o.okey == me.okey &&
                     (o.slot < me.slot || (o.slot == me.slot && o.seq < me.seq)));
        if (less) {
          ++rank;
          gl += PH == 0 ? 1u : 1u + o.run;
        }
        if (o.okey == me.okey && o.slot != me.slot) tie = true;
      }
      uint32_t grank = s_off[lb] + rank;
      uint32_t goff = PH == 0 ? grank : s_soff[lb] + gl;
      uint32_t size = PH == 0 ? 1u : 1u + me.run;
      if (goff < k_rem) {
        eoff[me.e] = n_dec + goff;
        etie[me.e] = tie ? 1 : 0;
        uint32_t na = size < k_rem - goff ? size : k_rem - goff;
        atomicAdd(&applied[me.slot], na);
        if (PH == 1 && (goff + size >= k_rem || grank == ne - 1)) {
          // the last applied group: its priority pop is this phase's last
          // limit-scanning pull
          sel->g_last = n_dec + goff;
          sel->n_prio_groups = grank + 1;
        }
      } else {
        eoff[me.e] = kNone;
      }
    }
    __syncthreads();
  }
}

struct ApplyVisit {
  dmc_decision* out;
  const uint32_t* eoff;
  const uint8_t* etie;
  uint32_t i, cap1, xbase;  // candidate index, region-2 layout
  uint32_t slot;
  int ph;
  uint32_t qbin;  // bin-rank path: entry id = i * qbin + seq (else region layout)
  __device__ uint32_t id(uint32_t j) const {
    return qbin ? i * qbin + j : entry_id(i, j, cap1, xbase);
  }
  uint32_t npop = 0, ngroup = 0, inrun = 0;
  uint32_t last_idx = 0;
  __device__ void pop(uint32_t, const Tag3& t, uint32_t cost, uint64_t h,
                      bool prio) {
    uint32_t idx, tie;
    if (ph == 0) {
      uint32_t e = id(npop);
      idx = eoff[e];
      tie = etie[e];
    } else {
      uint32_t e = id(ngroup);
      if (prio) inrun = 0;
      idx = eoff[e] + inrun;
      tie = prio ? etie[e] : 0;
      ++inrun;
    }
    dmc_decision d;
    d.handle = h;
    d.tag_r = t.r;
    d.tag_p = t.p;
    d.tag_l = t.l;
    d.slot = slot;
    d.cost = cost;
    d.phase = prio ? DMC_PHASE_PRIORITY : DMC_PHASE_RESERVATION;
    d.flags = tie;
    out[idx] = d;
    last_idx = idx;
    ++npop;
  }
  __device__ void group(uint64_t, uint32_t) { ++ngroup; }
};

// One thread per candidate replays its walk for exactly the pops that were
// dispatched, writes their decision records, and stores the client's new
// state: ring head/count, front cache, reduced reservation tags (immediate:
// every queued request, :1088-1095; delayed: the front, :1077-1085), prev tag,
// and the front's ready flag (set iff a later limit scan saw it with
// limit <= now).
template <int PH>
__global__ void k_apply(Table tb, const Sel* sel, Ctl* ctl,
                        const uint32_t* cand, const uint32_t* cxbase,
                        uint32_t cap1, const uint32_t* eoff,
                        const uint8_t* etie, uint32_t* applied,
                        uint32_t* bcount, uint32_t* bsize,
                        unsigned long long* sched, uint32_t qbin) {
  if (blockIdx.x == 0) {
    // the bin-rank counters are consumed: reset them
    for (int b = threadIdx.x; b < kNB; b += blockDim.x) {
      bcount[b] = 0;
      bsize[b] = 0;
    }
    // end of phase: the phase's decisions are counted once here (sched[0]
    // reservation, sched[1] priority: one per applied group), :1469,1479.
    // No other block of this kernel reads the fields written here.
    if (threadIdx.x == 0 && !ctl->overflow && k_left(ctl) != 0) {
      uint32_t d = sel->n_entries ? sel->n_dec_phase : 0;
      uint32_t np = PH == 1 && sel->n_entries ? sel->n_prio_groups : 0;
      ctl->n_dec += d;
      sched[0] += d - np;
      sched[1] += np;
      if (PH == 1 && ctl->n_dec < ctl->k_total) ctl->terminal = 1;
    }
  }
  if (ctl->overflow || sel->n_entries == 0) return;
  const double now = ctl->now;
  const uint64_t tick = ctl->tick;
  dmc_decision* out = ctl->out;
  uint32_t nc = sel->n_cand;
  uint32_t g_last = sel->g_last;
  uint32_t terminal = sel->terminal;
  uint64_t T = sel->T;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nc;
       i += gridDim.x * blockDim.x) {
    uint32_t s = cand[i];
    uint32_t a = applied[s];
    if (!a) continue;
    applied[s] = 0;
    ApplyVisit v{out, eoff, etie, i, cap1, qbin ? 0u : cxbase[i], s, PH, qbin};
    Tag3 prev{tb.prev_r[s], tb.prev_p[s], tb.prev_l[s], tb.prev_arr[s]};
    Tag3 front{};
    uint32_t fcost = 0;
    uint32_t c = tb.count[s], h = tb.head[s];
    uint64_t pmask = 0;
    uint32_t pops;
    if (PH == 0) {
      pops = walk_r(tb, s, now, T, a, v, &prev, &front, &fcost);
    } else {
      WalkP w = walk_p(tb, s, now, T, a, v, &prev, &front, &fcost);
      pops = w.pops;
      pmask = w.pmask;
    }
    ReqEntry* ring = tb.ring + (size_t)s * tb.q;
    uint32_t nc2 = c - pops, nh = (h + pops) & tb.qmask;
    if (!tb.delayed) {
      if (PH == 1 && pmask) {
        double rinv = tb.r_inv[s];
        // remaining requests: all reductions, in order
        for (uint32_t k = pops; k < c; ++k)
          ring[(h + k) & tb.qmask].r = reduced_r(ring, h, tb.qmask, k, pmask, rinv);
        double pr = prev.r;
        for (uint32_t j = 0; j < pops; ++j)
          if ((pmask >> j) & 1ull) {
            const ReqEntry& ej = ring[(h + j) & tb.qmask];
            pr = __dsub_rn(pr, resv_offset(rinv, ej.cost, ej.rho));
          }
        tb.prev_r[s] = pr;
      }
      if (nc2) {
        const ReqEntry& f = ring[nh];
        front = Tag3{f.r, f.p, f.l, f.arrival};
      }
    } else {
      // delayed: the walk recomputed the new front and prev
      if (nc2) {
        ReqEntry& f = ring[nh];
        f.r = front.r;
        f.p = front.p;
        f.l = front.l;
        f.delta = tb.cur_delta[s];
        f.rho = tb.cur_rho[s];
      }
      tb.prev_r[s] = prev.r;
      tb.prev_p[s] = prev.p;
      tb.prev_l[s] = prev.l;
      tb.prev_arr[s] = prev.arrival;
      if (c >= 2) tb.last_tick[s] = tick;
    }
    tb.head[s] = nh;
    tb.count[s] = nc2;
    uint8_t f = tb.flags[s] & (uint8_t)~F_READY;
    if (nc2) {
      tb.front_r[s] = front.r;
      tb.front_p[s] = front.p;
      tb.front_l[s] = front.l;
      bool later_scan = PH == 1 && (terminal || (g_last != kNone && v.last_idx < g_last));
      if (later_scan && front.l <= now) f |= F_READY;
    }
    tb.flags[s] = f;
  }
}

// ------------------------------------------------------------------ future
__device__ inline double min_not_0(double cur, double possible) {  // :1192-1195
  return possible == 0.0 ? cur : (possible < cur ? possible : cur);
}

// ------------------------------------------------------------------ single step
// General do_next_request(now) one pull at a time (used for small k and for
// AtLimit::Allow limit breaks, :1157-1165).  Reductions are per block, then
// one block combines them.
__global__ void k_step_scan(Table tb, double now, StepRed* part,
                            const Ctl* ctl) {
  // as the terminal pull of a batch: only if the batch ran out of work
  if (ctl && (ctl->overflow || !ctl->terminal)) return;
  if (ctl) now = ctl->now;
  ArgMin r{kMaxKey, kNone, 0}, p{kMaxKey, kNone, 0}, pnr{kMaxKey, kNone, 0};
  uint64_t lnr = kMaxKey, lrd = kMaxKey;
  uint32_t nany = 0, nrd = 0, nnr = 0;
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < tb.n;
       s += gridDim.x * blockDim.x) {
    if (!tb.count[s]) continue;
    ++nany;
    ArgMin a{okey(tb.front_r[s]), s, 1};
    r = argmin_combine(r, a);
    double l = tb.front_l[s];
    bool rdy = (tb.flags[s] & F_READY) || l <= now;
    double pv = tb.front_p[s];
    uint64_t kp = okey(__dadd_rn(pv, tb.pd[s]));
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
  r = wave_argmin(r);
  p = wave_argmin(p);
  pnr = wave_argmin(pnr);
  lnr = wave_min_u64(lnr);
  lrd = wave_min_u64(lrd);
  nany = wave_sum_u32(nany);
  nrd = wave_sum_u32(nrd);
  nnr = wave_sum_u32(nnr);
  __shared__ StepRed sh[kBlock / 64];
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
    for (int i = 1; i < (int)(blockDim.x / 64); ++i) {
      o.r = argmin_combine(o.r, sh[i].r);
      o.p = argmin_combine(o.p, sh[i].p);
      o.pnr = argmin_combine(o.pnr, sh[i].pnr);
      o.lmin_nr = sh[i].lmin_nr < o.lmin_nr ? sh[i].lmin_nr : o.lmin_nr;
      o.lmin_rd = sh[i].lmin_rd < o.lmin_rd ? sh[i].lmin_rd : o.lmin_rd;
      o.n_any += sh[i].n_any;
      o.n_ready += sh[i].n_ready;
      o.n_notready += sh[i].n_notready;
    }
    part[blockIdx.x] = o;
  }
}

__device__ inline void stepred_combine(StepRed& o, const StepRed& b) {
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
__global__ void k_step_decide(uint32_t nparts, const StepRed* part, double now,
                              int at_limit, uint32_t nregistered,
                              StepCtl* sc, Ctl* ctl) {
  if (ctl && (ctl->overflow || !ctl->terminal)) return;
  if (ctl) now = ctl->now;
  __shared__ StepRed sh[kBlock];
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
  for (int d = blockDim.x / 2; d > 0; d >>= 1) {
    if ((int)threadIdx.x < d) stepred_combine(sh[threadIdx.x], sh[threadIdx.x + d]);
    __syncthreads();
  }
  if (threadIdx.x) return;
  StepRed o = sh[0];
  StepCtl c{};
  c.type = DMC_NEXT_NONE;
  c.slot = kNone;
  if (nregistered == 0) {  // resv_heap.empty(), :1118-1120
    *sc = c;
    if (ctl) {
      ctl->next_type = c.type;
      ctl->when = c.when;
    }
    return;
  }
  double rtop = o.n_any ? from_okey(o.r.key) : kInf;
  if (o.n_any && rtop <= now) {  // :1124-1128
    c.type = DMC_NEXT_RETURNING;
    c.prio = 0;
    c.slot = o.r.slot;
    c.tie = o.r.cnt > 1;
    *sc = c;
    if (ctl) {
      ctl->next_type = c.type;
      ctl->when = c.when;
    }
    return;
  }
  c.mark = 1;  // the limit scan ran
  if (o.p.slot != kNone) {  // :1146-1151
    c.type = DMC_NEXT_RETURNING;
    c.prio = 1;
    c.slot = o.p.slot;
    c.tie = o.p.cnt > 1;
    *sc = c;
    if (ctl) {
      ctl->next_type = c.type;
      ctl->when = c.when;
    }
    return;
  }
  if (at_limit == DMC_AT_LIMIT_ALLOW && o.n_any) {  // :1157-1165
    // ready-heap top: ready fronts first (all have p == inf here), else the
    // min p+pd over not-ready fronts
    bool top_ready = o.n_ready > 0;
    if (!top_ready && o.pnr.slot != kNone &&
        from_okey(o.pnr.key) < kInf) {
      c.type = DMC_NEXT_RETURNING;
      c.prio = 1;
      c.slot = o.pnr.slot;
      c.tie = o.pnr.cnt > 1;
      *sc = c;
      if (ctl) {
        ctl->next_type = c.type;
        ctl->when = c.when;
      }
      return;
    }
    if (rtop < kInf) {
      c.type = DMC_NEXT_RETURNING;
      c.prio = 0;
      c.slot = o.r.slot;
      c.tie = o.r.cnt > 1;
      *sc = c;
      if (ctl) {
        ctl->next_type = c.type;
        ctl->when = c.when;
      }
      return;
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
  *sc = c;
  if (ctl) {
    ctl->next_type = c.type;
    ctl->when = c.when;
  }
}

__global__ void k_step_mark(Table tb, double now, const StepCtl* sc) {
  if (!sc->mark) return;
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < tb.n;
       s += gridDim.x * blockDim.x) {
    if (tb.count[s] && !(tb.flags[s] & F_READY) && tb.front_l[s] <= now)
      tb.flags[s] |= F_READY;
  }
}

// pop_process_request (+ reduce_reservation_tags for ready-heap pops) of the
// chosen client, :1046-1111.
__global__ void k_step_apply(Table tb, uint64_t tick, const StepCtl* sc,
                             dmc_decision* out, uint32_t out_idx,
                             unsigned long long* sched) {
  if (threadIdx.x || blockIdx.x) return;
  if (sc->type != DMC_NEXT_RETURNING) return;
  uint32_t s = sc->slot;
  bool prio = sc->prio != 0;
  ReqEntry* ring = tb.ring + (size_t)s * tb.q;
  uint32_t h = tb.head[s], c = tb.count[s];
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
  double rinv = tb.r_inv[s];
  if (tb.delayed && nc) {  // update_next_tag, :1021-1036
    ReqEntry& f = ring[nh];
    Tag3 pt{popped.r, popped.p, popped.l, popped.arrival};
    Tag3 nt;
    uint32_t cd = tb.cur_delta[s], cr = tb.cur_rho[s];
    if (make_tag(pt, rinv, tb.w_inv[s], tb.l_inv[s], cd, cr, f.arrival, f.cost,
                 tb.antic, &nt)) {
      f.r = nt.r;
      f.p = nt.p;
      f.l = nt.l;
      f.delta = cd;
      f.rho = cr;
      double pr = tb.prev_r[s], pp = tb.prev_p[s], pl = tb.prev_l[s];
      assign_unpinned(pr, nt.r);
      assign_unpinned(pl, nt.l);
      assign_unpinned(pp, nt.p);
      tb.prev_r[s] = pr;
      tb.prev_p[s] = pp;
      tb.prev_l[s] = pl;
      tb.prev_arr[s] = nt.arrival;
      tb.last_tick[s] = tick;
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
    tb.prev_r[s] = __dsub_rn(tb.prev_r[s], o);
  }
  tb.head[s] = nh;
  tb.count[s] = nc;
  tb.flags[s] &= (uint8_t)~F_READY;
  if (nc) {
    const ReqEntry& f = ring[nh];
    tb.front_r[s] = f.r;
    tb.front_p[s] = f.p;
    tb.front_l[s] = f.l;
  }
  atomicAdd(&sched[prio ? 1 : 0], 1ull);
}

// ------------------------------------------------------------------ stats
__global__ void k_count_requests(Table tb, unsigned long long* out) {
  unsigned long long t = 0;
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < tb.n;
       s += gridDim.x * blockDim.x)
    t += tb.count[s];
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
struct GraphRec {
  uint64_t key = 0;
  uint64_t last_use = 0;
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  hipGraphNode_t param_node = nullptr;
  hipKernelNodeParams kp{};
};

struct dmc_queue {
  dmc_queue_params p{};
  hipStream_t stream = nullptr;
  Table tb{};
  std::mutex mtx;  // C-ABI calls on one handle are serialised (data_mtx, :762)
  // host mirrors
  std::vector<uint8_t> reg_h, idle_h;
  uint32_t n_registered = 0;
  uint32_t n_idle = 0;
  uint64_t tick = 0;
  // device scratch
  uint64_t* keys = nullptr;   // N
  uint32_t* cnt = nullptr;    // N
  uint32_t* off = nullptr;    // N
  uint32_t* applied = nullptr;// N
  uint32_t* hist = nullptr;
  uint64_t* hmax = nullptr;
  uint32_t *sbase = nullptr, *snum = nullptr;  // rank-bin table (k_pick)
  Sel* sel = nullptr;
  StepRed* red = nullptr;     // step partials (grid) + future record
  StepCtl* sctl = nullptr;
  uint64_t* act_min = nullptr;
  unsigned long long* sched = nullptr;  // [0] reservation, [1] priority
  unsigned long long* reqcount = nullptr;
  // entries (grown on demand)
  uint32_t ecap = 0;
  uint64_t* eokey = nullptr;  // full ordered key per entry
  uint32_t *ek32 = nullptr, *sk32 = nullptr;  // 32-bit sort keys
  uint32_t *eval = nullptr, *sval = nullptr, *eslot = nullptr, *erun = nullptr;
  uint32_t *eseq = nullptr;
  uint32_t *eoff = nullptr, *gsz = nullptr, *goff = nullptr;
  uint8_t* etie = nullptr;
  size_t idcap = 0;           // eoff / etie capacity
  Ctl* h_ctl = nullptr;              // pinned: round control readback
  dmc_pull_result* h_res = nullptr;  // pinned: device-API result staging
  // add batch buffers
  uint32_t bcap = 0;
  dmc_request* d_reqs = nullptr;
  int32_t* d_rc = nullptr;
  uint32_t *apos = nullptr, *aslot = nullptr;   // per batch request
  uint32_t *acnt = nullptr, *abuf = nullptr;    // per client (N, N * kAddSlots)
  AddParams* apblk = nullptr;
  // decisions (host API)
  uint32_t dcap = 0;
  dmc_decision* d_dec = nullptr;
  void* temp = nullptr;
  size_t temp_bytes = 0;
  uint32_t step_grid = 0;
  uint32_t small_k = 8;  // pulls with k <= small_k run the single-step path
  Ctl* ctl = nullptr;
  ScanPart* parts = nullptr;  // per-block scan partials
  // entry capacities per phase: [0] first entries (= candidates), [1] extras
  uint32_t cap_hint[2][2] = {{4096, 4096}, {4096, 4096}};
  uint32_t* cand = nullptr;    // N
  bool use_radix = false;      // rank entries with the radix sort (fallback)
  bool force_radix = false;    // DMC_OPT_FORCE_RADIX
  uint32_t radix_batches = 0;  // batches left on the fallback path
  uint32_t *bcount = nullptr, *bsize = nullptr;  // kNB rank-bin counters
  uint32_t* cxbase = nullptr;  // N
  BRec* brec = nullptr;        // kNB * kBinCap rank-bin records
  uint64_t* emax = nullptr;    // N / kBlock + 1
  // captured pull rounds / add segments (see launch_round)
  bool use_graphs = true;
  std::vector<GraphRec> graphs = std::vector<GraphRec>(8);
  std::vector<uint64_t> graph_seen = std::vector<uint64_t>(8, 0);
  uint32_t graph_seen_pos = 0;
  uint64_t graph_clock = 0;
  // stage timers (HIP events on the queue's stream), see dmc_profile_*
  struct ProfRec {
    hipEvent_t a, b;
    int stage;
  };
  bool prof_on = false;
  std::vector<ProfRec> prof_pool;
  size_t prof_n = 0;
  double prof_ms[DMC_PROF_NSTAGES] = {};
  uint64_t prof_cnt[DMC_PROF_NSTAGES] = {};
};

namespace {

const char* kStageNames[DMC_PROF_NSTAGES] = {
    "add_link", "add_chain", "activate",
    "r_scan", "r_select", "r_cand", "r_emit", "r_key32", "r_sort",
    "r_decide", "r_apply",
    "p_scan", "p_select", "p_cand", "p_emit", "p_key32", "p_sort",
    "p_decide", "p_apply",
    "step", "future"};

void pb(dmc_queue* q, int stage) {
  if (!q->prof_on) return;
  if (q->prof_n == q->prof_pool.size()) {
    dmc_queue::ProfRec r;
    if (hipEventCreate(&r.a) != hipSuccess || hipEventCreate(&r.b) != hipSuccess) {
      q->prof_on = false;
      return;
    }
    q->prof_pool.push_back(r);
  }
  q->prof_pool[q->prof_n].stage = stage;
  (void)hipEventRecord(q->prof_pool[q->prof_n].a, q->stream);
}

void pe(dmc_queue* q) {
  if (!q->prof_on) return;
  (void)hipEventRecord(q->prof_pool[q->prof_n].b, q->stream);
  ++q->prof_n;
}

void pflush(dmc_queue* q) {
  if (!q->prof_on || !q->prof_n) return;
  (void)hipEventSynchronize(q->prof_pool[q->prof_n - 1].b);
  for (size_t i = 0; i < q->prof_n; ++i) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, q->prof_pool[i].a, q->prof_pool[i].b) == hipSuccess) {
      q->prof_ms[q->prof_pool[i].stage] += ms;
      q->prof_cnt[q->prof_pool[i].stage] += 1;
    }
  }
  q->prof_n = 0;
}

void dfree(void* p) {
  if (p) (void)hipFree(p);
}

int graph_replay(dmc_queue* q, GraphRec& g, void** args) {
  hipKernelNodeParams kp = g.kp;
  kp.kernelParams = args;
  kp.extra = nullptr;
  HIP_OK(hipGraphExecKernelNodeSetParams(g.exec, g.param_node, &kp));
  HIP_OK(hipGraphLaunch(g.exec, q->stream));
  return DMC_OK;
}

// Capture `enqueue` (which must start with the parameter kernel) as a graph.
template <typename F>
int graph_capture(dmc_queue* q, GraphRec& g, F enqueue) {
  HIP_OK(hipStreamBeginCapture(q->stream, hipStreamCaptureModeThreadLocal));
  enqueue();
  hipGraph_t graph = nullptr;
  HIP_OK(hipStreamEndCapture(q->stream, &graph));
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
  HIP_OK(hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0));
  g.graph = graph;
  g.param_node = root;
  return DMC_OK;
}

void graph_destroy(GraphRec& g) {
  if (g.exec) (void)hipGraphExecDestroy(g.exec);
  if (g.graph) (void)hipGraphDestroy(g.graph);
  g = GraphRec{};
}

// Find (or, on the second sighting, build) the graph for `key`; nullptr if the
// caller should launch eagerly this time.
template <typename F>
GraphRec* graph_for(dmc_queue* q, uint64_t key, F enqueue) {
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
  graph_destroy(*slot);
  if (graph_capture(q, *slot, enqueue) != DMC_OK) {
    graph_destroy(*slot);
    q->use_graphs = false;  // capture unsupported: stay eager
    return nullptr;
  }
  slot->key = key;
  slot->last_use = ++q->graph_clock;
  return slot;
}

// Buffers captured into graphs are about to move: drop every graph.
void invalidate_graphs(dmc_queue* q) {
  for (auto& g : q->graphs) graph_destroy(g);
}

int ensure_temp(dmc_queue* q, size_t need) {
  if (need <= q->temp_bytes) return DMC_OK;
  invalidate_graphs(q);
  if (q->temp) dfree(q->temp);
  q->temp = nullptr;
  size_t sz = need + (need >> 2) + 4096;
  HIP_OK(hipMalloc(&q->temp, sz));
  q->temp_bytes = sz;
  return DMC_OK;
}

// decision offset / tie flag per entry id: region layout (cap1 + cap2) on the
// radix path, candidate * ring capacity + seq on the bin-rank path
int ensure_ids(dmc_queue* q, size_t n) {
  if (n <= q->idcap) return DMC_OK;
  size_t cap = std::max<size_t>(n + (n >> 2), 1u << 16);
  invalidate_graphs(q);
  dfree(q->eoff);
  dfree(q->etie);
  q->eoff = nullptr;
  q->etie = nullptr;
  HIP_OK(hipMalloc(&q->eoff, sizeof(uint32_t) * cap));
  HIP_OK(hipMalloc(&q->etie, cap));
  q->idcap = cap;
  return DMC_OK;
}

int ensure_entries(dmc_queue* q, uint32_t n) {
  if (n <= q->ecap) return DMC_OK;
  uint32_t cap = std::max<uint32_t>(n + (n >> 1), 1u << 16);
  invalidate_graphs(q);
  dfree(q->eokey); dfree(q->ek32); dfree(q->sk32); dfree(q->eval);
  dfree(q->sval); dfree(q->eslot); dfree(q->erun); dfree(q->eseq);
  dfree(q->gsz); dfree(q->goff);
  HIP_OK(hipMalloc(&q->eokey, sizeof(uint64_t) * cap));
  HIP_OK(hipMalloc(&q->ek32, sizeof(uint32_t) * cap));
  HIP_OK(hipMalloc(&q->sk32, sizeof(uint32_t) * cap));
  HIP_OK(hipMalloc(&q->eval, sizeof(uint32_t) * cap));
  HIP_OK(hipMalloc(&q->sval, sizeof(uint32_t) * cap));
  HIP_OK(hipMalloc(&q->eslot, sizeof(uint32_t) * cap));
  HIP_OK(hipMalloc(&q->erun, sizeof(uint32_t) * cap));
  HIP_OK(hipMalloc(&q->eseq, sizeof(uint32_t) * cap));
  HIP_OK(hipMalloc(&q->gsz, sizeof(uint32_t) * cap));
  HIP_OK(hipMalloc(&q->goff, sizeof(uint32_t) * cap));
  q->ecap = cap;
  int rc = ensure_ids(q, cap);
  if (rc) return rc;
  size_t t1 = 0, t2 = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, t1, q->ek32, q->sk32, q->eval,
                                           q->sval, (int)cap, 0, 32, q->stream);
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, t2, q->gsz, q->goff, (int)cap,
                                         q->stream);
  return ensure_temp(q, std::max(t1, t2));
}

int ensure_batch(dmc_queue* q, uint32_t n) {
  if (n <= q->bcap) return DMC_OK;
  uint32_t cap = std::max<uint32_t>(n, 1024);
  invalidate_graphs(q);
  dfree(q->d_reqs); dfree(q->d_rc); dfree(q->apos); dfree(q->aslot);
  HIP_OK(hipMalloc(&q->d_reqs, sizeof(dmc_request) * cap));
  HIP_OK(hipMalloc(&q->d_rc, sizeof(int32_t) * cap));
  HIP_OK(hipMalloc(&q->apos, sizeof(uint32_t) * cap));
  HIP_OK(hipMalloc(&q->aslot, sizeof(uint32_t) * cap));
  q->bcap = cap;
  return DMC_OK;
}

int ensure_dec(dmc_queue* q, uint32_t n) {
  if (n <= q->dcap) return DMC_OK;
  dfree(q->d_dec);
  uint32_t cap = std::max<uint32_t>(n, 1024);
  HIP_OK(hipMalloc(&q->d_dec, sizeof(dmc_decision) * cap));
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
  uint32_t g = (ap.n + kBlock - 1) / kBlock;
  pb(q, DMC_PROF_ADD_LINK);
  hipLaunchKernelGGL(k_add_link, dim3(g), dim3(kBlock), 0, q->stream, ap, q->tb,
                     q->acnt, q->abuf, q->apos, q->aslot, q->apblk);
  pe(q);
  pb(q, DMC_PROF_ADD_CHAIN);
  hipLaunchKernelGGL(k_add_chain, dim3(g), dim3(kBlock), 0, q->stream, q->tb,
                     (const AddParams*)q->apblk, q->acnt, (const uint32_t*)q->abuf,
                     (const uint32_t*)q->apos, (const uint32_t*)q->aslot);
  pe(q);
}

int add_segment(dmc_queue* q, const dmc_request* d_reqs, uint32_t n,
                int32_t* d_rc, uint64_t tick_base) {
  if (!n) return DMC_OK;
  AddParams ap{d_reqs, d_rc, tick_base, n, 0};
  uint64_t key = (2ull << 56) | n;
  GraphRec* g = graph_for(q, key, [&] { enqueue_add(q, ap); });
  if (!g) {
    enqueue_add(q, ap);
    HIP_OK(hipGetLastError());
    return DMC_OK;
  }
  Table tb = q->tb;
  void* args[] = {&ap, &tb, &q->acnt, &q->abuf, &q->apos, &q->aslot, &q->apblk};
  return graph_replay(q, *g, args);
}

int activate(dmc_queue* q, uint32_t slot, double t) {
  pb(q, DMC_PROF_ACTIVATE);
  uint32_t g = grid_for(q->tb.n, 2048);
  hipLaunchKernelGGL(k_contrib_min, dim3(g), dim3(kBlock), 0, q->stream, q->tb,
                     (uint64_t*)q->parts);
  hipLaunchKernelGGL(k_activate, dim3(1), dim3(kBlock), 0, q->stream, q->tb, slot,
                     t, (const uint64_t*)q->parts, g);
  pe(q);
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

// --------------------------------------------------------------- pull phases
// Larger pulls rank through the radix path: the kNB x kBinCap rank bins hold
// about a million entries when balanced.
constexpr uint32_t kBinRankMaxK = 1u << 18;

uint32_t pow2_at_least(uint32_t x) {
  uint32_t p = 4096;
  while (p < x && p < (1u << 31)) p <<= 1;
  return p;
}

// Enqueue one batched phase; no host synchronisation.  `cap` is the entry
// capacity the sort runs over (entries beyond it set ctl->overflow and the
// rest of the batch no-ops; the host retries with a larger capacity).
template <int PH>
int launch_phase(dmc_queue* q, uint32_t cap1, uint32_t cap2, const CallParams& cp) {
  const Table& tb = q->tb;
  uint32_t N = tb.n;
  uint32_t gN = grid_for(N, 2048);
  uint32_t E = cap1 + cap2;
  uint32_t gE = grid_for(E, 1024);
  const int S0 = PH == 0 ? DMC_PROF_R_SCAN : DMC_PROF_P_SCAN;  // stage base
  pb(q, S0 + 0);
  hipLaunchKernelGGL(k_scan<PH>, dim3(gN), dim3(kBlock), 0, q->stream, tb,
                     q->keys, q->parts, q->ctl, cp);
  pe(q);
  pb(q, S0 + 1);
  hipLaunchKernelGGL(k_hist, dim3(kHistBlocks), dim3(1024), 0, q->stream, N,
                     (const uint64_t*)q->keys, (const ScanPart*)q->parts, gN,
                     (const Ctl*)q->ctl, q->hist, q->hmax);
  hipLaunchKernelGGL(k_pick, dim3(1), dim3(kPickThreads), 0, q->stream,
                     (const ScanPart*)q->parts, gN, q->sel, (const Ctl*)q->ctl,
                     q->hist, q->hmax, (uint32_t)PH, q->sbase, q->snum);
  pe(q);
  uint32_t gX = (N + kBlock - 1) / kBlock;  // one thread per candidate
  pb(q, S0 + 2);
  hipLaunchKernelGGL(k_cand, dim3(kCandBlocks), dim3(kBlock), 0, q->stream, N,
                     (const uint64_t*)q->keys, q->sel, q->cand);
  pe(q);
  pb(q, S0 + 3);
  if (q->use_radix)
    hipLaunchKernelGGL((k_emit<PH, false>), dim3(gX), dim3(kBlock), 0, q->stream,
                       tb, q->sel, (const Ctl*)q->ctl, (const uint32_t*)q->cand,
                       cap1, cap2, q->cxbase, q->eokey, q->eslot, q->eseq, q->erun,
                       q->emax, nullptr, nullptr, nullptr, nullptr, nullptr);
  else
    hipLaunchKernelGGL((k_emit<PH, true>), dim3(gX), dim3(kBlock), 0, q->stream,
                       tb, q->sel, (const Ctl*)q->ctl, (const uint32_t*)q->cand,
                       cap1, cap2, q->cxbase, q->eokey, q->eslot, q->eseq, q->erun,
                       q->emax, q->brec, q->bcount, q->bsize,
                       (const uint32_t*)q->sbase, (const uint32_t*)q->snum);
  pe(q);
  if (!q->use_radix) {
    pb(q, S0 + 6);
    hipLaunchKernelGGL(k_rank<PH>, dim3(kRankBlocks), dim3(kBlock), 0, q->stream,
                       q->sel, q->ctl, cap1, cap2, (const uint32_t*)q->bcount,
                       (const uint32_t*)q->bsize, (const BRec*)q->brec, q->eoff,
                       q->etie, q->applied);
    pe(q);
  } else {
    pb(q, S0 + 4);
    hipLaunchKernelGGL(k_key32, dim3(gE), dim3(kBlock), 0, q->stream, q->sel,
                       q->ctl, cap1, cap2, (const uint64_t*)q->emax, gX,
                       (const uint64_t*)q->eokey, q->ek32, q->eval);
    pe(q);
    pb(q, S0 + 5);
    size_t tbytes = q->temp_bytes;
    HIP_OK(hipcub::DeviceRadixSort::SortPairs(q->temp, tbytes, q->ek32, q->sk32,
                                              q->eval, q->sval, (int)E, 0, 32,
                                              q->stream));
    hipLaunchKernelGGL(k_fixup, dim3(gE), dim3(kBlock), 0, q->stream,
                       (const Sel*)q->sel, (const uint32_t*)q->sk32, q->sval,
                       (const uint64_t*)q->eokey, (const uint32_t*)q->eslot,
                       (const uint32_t*)q->eseq);
    pe(q);
    pb(q, S0 + 6);
    if (PH == 0) {
      hipLaunchKernelGGL(k_decide_r, dim3(gE), dim3(kBlock), 0, q->stream,
                         (const Ctl*)q->ctl, (const uint64_t*)q->eokey,
                         (const uint32_t*)q->sval, (const uint32_t*)q->eslot,
                         q->eoff, q->etie, q->applied, q->sel);
    } else {
      hipLaunchKernelGGL(k_group_sizes, dim3(gE), dim3(kBlock), 0, q->stream,
                         (const Ctl*)q->ctl, (const Sel*)q->sel, E,
                         (const uint32_t*)q->sval, (const uint32_t*)q->erun, q->gsz);
      tbytes = q->temp_bytes;
      HIP_OK(hipcub::DeviceScan::ExclusiveSum(q->temp, tbytes, q->gsz, q->goff,
                                              (int)E, q->stream));
      hipLaunchKernelGGL(k_decide_p, dim3(gE), dim3(kBlock), 0, q->stream,
                         (const Ctl*)q->ctl, (const uint64_t*)q->eokey,
                         (const uint32_t*)q->sval, (const uint32_t*)q->eslot,
                         (const uint32_t*)q->gsz, (const uint32_t*)q->goff, q->eoff,
                         q->etie, q->applied, q->sel);
    }
    pe(q);
  }
  pb(q, S0 + 7);
  hipLaunchKernelGGL(k_apply<PH>, dim3(grid_for(N, 1024)), dim3(kBlock), 0,
                     q->stream, tb, (const Sel*)q->sel, q->ctl,
                     (const uint32_t*)q->cand, (const uint32_t*)q->cxbase, cap1,
                     (const uint32_t*)q->eoff, (const uint8_t*)q->etie, q->applied,
                     q->bcount, q->bsize, q->sched, q->use_radix ? 0u : tb.q);
  pe(q);
  return DMC_OK;
}

// Terminal pull of a Wait/Reject batch: one general do_next_request, which
// (nothing being eligible) computes min_not_0 over the reservation- and
// limit-heap tops, :1170-1185.  No-op unless ctl->terminal.
int launch_future(dmc_queue* q, Ctl* ctl) {
  const double now = 0.0;  // read from ctl by the kernels
  pb(q, DMC_PROF_FUTURE);
  hipLaunchKernelGGL(k_step_scan, dim3(q->step_grid), dim3(kBlock), 0, q->stream,
                     q->tb, now, q->red, (const Ctl*)ctl);
  hipLaunchKernelGGL(k_step_decide, dim3(1), dim3(kBlock), 0, q->stream,
                     q->step_grid, (const StepRed*)q->red, now, q->p.at_limit,
                     q->n_registered, q->sctl, ctl);
  pe(q);
  return DMC_OK;
}

// one general pull_request(now); returns the NextReqType in *type
int step_once(dmc_queue* q, double now, dmc_decision* d_out, uint32_t idx,
              int* type, double* when) {
  const Table& tb = q->tb;
  pb(q, DMC_PROF_STEP);
  hipLaunchKernelGGL(k_step_scan, dim3(q->step_grid), dim3(kBlock), 0, q->stream,
                     tb, now, q->red, (const Ctl*)nullptr);
  hipLaunchKernelGGL(k_step_decide, dim3(1), dim3(kBlock), 0, q->stream,
                     q->step_grid, (const StepRed*)q->red, now, q->p.at_limit,
                     q->n_registered, q->sctl, (Ctl*)nullptr);
  hipLaunchKernelGGL(k_step_mark, dim3(grid_for(tb.n, 2048)), dim3(kBlock), 0,
                     q->stream, tb, now, (const StepCtl*)q->sctl);
  hipLaunchKernelGGL(k_step_apply, dim3(1), dim3(64), 0, q->stream, tb, q->tick,
                     (const StepCtl*)q->sctl, d_out, idx, q->sched);
  pe(q);
  StepCtl sc;
  HIP_OK(hipMemcpyAsync(&sc, q->sctl, sizeof(sc), hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  pflush(q);
  *type = sc.type;
  *when = sc.when;
  return DMC_OK;
}

// One pull round: phase R + phase P (+ the terminal pull).  The sequence
// depends on the per-call parameters only through k_scan<0>'s
// arguments, so it is captured once per shape (entry capacities, ranking
// path, terminal pull) into a hipGraph and replayed with k_scan<0>'s
// arguments updated: one graph launch instead of ~25 kernel launches, which
// removes the host's per-launch cost from the critical path.  A shape is
// captured the second time it is seen; profiling runs eagerly (the stage
// timers are events between kernels).
void enqueue_round(dmc_queue* q, const CallParams& cp, const uint32_t* cap1,
                   const uint32_t* cap2, bool future) {
  launch_phase<0>(q, cap1[0], cap2[0], cp);
  launch_phase<1>(q, cap1[1], cap2[1], cp);
  if (future) launch_future(q, q->ctl);
}

int launch_round(dmc_queue* q, double now, uint32_t kk, dmc_decision* out,
                 const uint32_t* cap1, const uint32_t* cap2, bool future) {
  uint64_t key = 1;  // shape: capacities (powers of two), ranking path, future
  for (int ph = 0; ph < 2; ++ph)
    key = key * 64 + (uint64_t)__builtin_ctz(cap1[ph]),
    key = key * 64 + (uint64_t)__builtin_ctz(cap2[ph]);
  key = key * 4 + (q->use_radix ? 2 : 0) + (future ? 1 : 0);
  CallParams cp{kk, 0, now, out, q->tick};
  GraphRec* g = graph_for(q, key, [&] { enqueue_round(q, cp, cap1, cap2, future); });
  if (!g) {
    enqueue_round(q, cp, cap1, cap2, future);
    HIP_OK(hipGetLastError());
    return DMC_OK;
  }
  Table tb = q->tb;
  void* args[] = {&tb, &q->keys, &q->parts, &q->ctl, &cp};
  return graph_replay(q, *g, args);
}

// k successive pull_request(now).  Batched phases run with one host
// synchronisation per round; a round ends the batch unless an entry buffer
// overflowed (retry with more capacity) or, with AtLimit::Allow, the eligible
// work ran out (one general limit-break step, then another round).
int pull_impl(dmc_queue* q, double now, uint32_t k, dmc_decision* d_out,
              dmc_pull_result* res) {
  dmc_pull_result r{};
  r.next_type = DMC_NEXT_RETURNING;
  uint32_t n_dec = 0;
  bool allow = q->p.at_limit == DMC_AT_LIMIT_ALLOW;
  while (n_dec < k) {
    if (q->n_registered == 0) {
      r.next_type = DMC_NEXT_NONE;
      break;
    }
    uint32_t kk = k - n_dec;
    if (kk <= q->small_k) {
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
      continue;
    }
    uint32_t cap1[2], cap2[2];
    for (int ph = 0; ph < 2; ++ph) {
      cap1[ph] = std::max(q->cap_hint[ph][0], pow2_at_least(std::min(kk, 1u << 16)));
      cap2[ph] = q->cap_hint[ph][1];
      int rc = ensure_entries(q, cap1[ph] + cap2[ph]);
      if (rc) return rc;
    }
    q->use_radix = q->force_radix || q->radix_batches > 0 || kk > kBinRankMaxK;
    if (q->radix_batches) --q->radix_batches;
    if (!q->use_radix) {
      int rc = ensure_ids(q, (size_t)std::max(cap1[0], cap1[1]) * q->tb.q);
      if (rc) return rc;
    }
    int rc = launch_round(q, now, kk, d_out + n_dec, cap1, cap2, !allow);
    if (rc) return rc;
    // one host round trip per round, through pinned memory
    HIP_OK(hipMemcpyAsync(q->h_ctl, q->ctl, sizeof(Ctl), hipMemcpyDeviceToHost,
                          q->stream));
    HIP_OK(hipStreamSynchronize(q->stream));
    const Ctl c = *q->h_ctl;
    pflush(q);
    n_dec += c.n_dec;
    for (int ph = 0; ph < 2; ++ph) {
      uint32_t need[2] = {c.nc[ph], c.nx[ph]};
      for (int r = 0; r < 2; ++r) {
        uint32_t want = pow2_at_least(need[r] + (need[r] >> 2) + 1);
        uint32_t& h = q->cap_hint[ph][r];
        h = want > h ? want : std::max(want, h / 2);  // grow at once, shrink slowly
      }
    }
    if (c.overflow == 2) q->radix_batches = 8;  // skewed keys: sort instead
    if (c.overflow) continue;  // state before the overflowing phase is intact
    if (n_dec >= k || !c.terminal) break;
    if (allow) {
      int type;
      double when;
      rc = step_once(q, now, d_out, n_dec, &type, &when);
      if (rc) return rc;
      if (type != DMC_NEXT_RETURNING) {
        r.next_type = type;
        r.when = when;
        break;
      }
      ++n_dec;
      continue;
    }
    r.next_type = c.next_type;
    r.when = c.when;
    break;
  }
  r.n_decisions = n_dec;
  if (res) *res = r;
  return DMC_OK;
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
  rc |= A(&t.prev_r, N); rc |= A(&t.prev_p, N); rc |= A(&t.prev_l, N);
  rc |= A(&t.prev_arr, N); rc |= A(&t.r_inv, N); rc |= A(&t.w_inv, N);
  rc |= A(&t.l_inv, N); rc |= A(&t.pd, N); rc |= A(&t.front_r, N);
  rc |= A(&t.front_p, N); rc |= A(&t.front_l, N); rc |= A(&t.head, N);
  rc |= A(&t.count, N); rc |= A(&t.cur_delta, N); rc |= A(&t.cur_rho, N);
  rc |= A(&t.last_tick, N); rc |= A(&t.flags, N);
  rc |= A(&t.ring, (size_t)N * p.ring_capacity);
  rc |= A(&q->keys, N); rc |= A(&q->cnt, N); rc |= A(&q->off, N);
  rc |= A(&q->applied, N);
  rc |= A(&q->hist, kHistBins); rc |= A(&q->hmax, kHistBins);
  rc |= A(&q->sbase, kHistBins); rc |= A(&q->snum, kHistBins);
  rc |= A(&q->sel, 1);
  q->step_grid = grid_for(N, 1024);
  rc |= A(&q->red, q->step_grid + 1);
  rc |= A(&q->sctl, 1);
  rc |= A(&q->ctl, 1);
  rc |= A(&q->parts, 4096);
  rc |= A(&q->cand, N);
  rc |= A(&q->bcount, kNB);
  rc |= A(&q->bsize, kNB);
  rc |= A(&q->cxbase, N);
  rc |= A(&q->brec, (size_t)kNB * kBinCap);
  rc |= A(&q->emax, N / kBlock + 2);
  rc |= A(&q->act_min, 1);
  rc |= A(&q->acnt, N);
  rc |= A(&q->abuf, (size_t)N * kAddSlots);
  rc |= A(&q->apblk, 1);
  rc |= A(&q->sched, 2);
  rc |= A(&q->reqcount, 1);
  if (hipHostMalloc((void**)&q->h_ctl, sizeof(Ctl), 0) != hipSuccess ||
      hipHostMalloc((void**)&q->h_res, sizeof(dmc_pull_result), 0) != hipSuccess)
    rc |= DMC_ENOMEM;
  if (rc) {
    dmc_queue_destroy(q);
    return DMC_ENOMEM;
  }
  size_t tscan = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tscan, q->cnt, q->off, (int)N, q->stream);
  if (ensure_temp(q, tscan) || ensure_entries(q, std::max<uint32_t>(p.max_batch, 1u << 16)) ||
      ensure_batch(q, std::max<uint32_t>(p.max_batch, 1024)) ||
      ensure_dec(q, std::max<uint32_t>(p.max_batch, 1024))) {
    dmc_queue_destroy(q);
    return DMC_ENOMEM;
  }
  q->reg_h.assign(N, 0);
  q->idle_h.assign(N, 0);
  if (hipStreamSynchronize(q->stream) != hipSuccess) {
    dmc_queue_destroy(q);
    return DMC_EDEVICE;
  }
  *out = q;
  return DMC_OK;
}

int dmc_queue_destroy(dmc_queue* q) {
  if (!q) return DMC_EINVAL;
  if (q->stream) (void)hipStreamSynchronize(q->stream);
  invalidate_graphs(q);
  Table& t = q->tb;
  void* ptrs[] = {t.prev_r, t.prev_p, t.prev_l, t.prev_arr, t.r_inv, t.w_inv,
                  t.l_inv, t.pd, t.front_r, t.front_p, t.front_l, t.head,
                  t.count, t.cur_delta, t.cur_rho, t.last_tick, t.flags, t.ring,
                  q->keys, q->cnt, q->off, q->applied, q->hist, q->hmax, q->sbase, q->snum, q->sel,
                  q->red, q->sctl, q->act_min, q->sched, q->reqcount, q->eokey,
                  q->ek32, q->sk32, q->eval, q->sval, q->eslot, q->erun, q->eseq,
                  q->eoff, q->gsz, q->goff, q->etie, q->d_reqs, q->d_rc, q->apos, q->aslot,
                  q->acnt, q->abuf, q->apblk, q->d_dec, q->temp, q->ctl,
                  q->parts, q->cand, q->cxbase, q->brec, q->emax, q->bcount,
                  q->bsize};
  for (void* p : ptrs)
    dfree(p);
  if (q->h_ctl) (void)hipHostFree(q->h_ctl);
  if (q->h_res) (void)hipHostFree(q->h_res);
  for (auto& r : q->prof_pool) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  if (q->stream) (void)hipStreamDestroy(q->stream);
  delete q;
  return DMC_OK;
}

void* dmc_queue_stream(dmc_queue* q) { return q ? (void*)q->stream : nullptr; }

int dmc_queue_sync(dmc_queue* q) {
  if (!q) return DMC_EINVAL;
  HIP_OK(hipStreamSynchronize(q->stream));
  return DMC_OK;
}

static double inv_of(double x) { return x == 0.0 ? 0.0 : 1.0 / x; }  // :115-117

int dmc_client_register_batch(dmc_queue* q, uint32_t n, const uint32_t* slots,
                              const double* r, const double* w, const double* l,
                              int active) {
  if (!q || (n && (!slots || !r || !w || !l))) return DMC_EINVAL;
  std::lock_guard<std::mutex> g(q->mtx);
  for (uint32_t i = 0; i < n; ++i)
    if (slots[i] >= q->p.max_clients) return DMC_EINVAL;
  if (!n) return DMC_OK;
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
                     q->stream, q->tb, n, d_slots, d_r, d_w, d_l, active, q->tick);
  HIP_OK(hipStreamSynchronize(q->stream));
  dfree(d_slots); dfree(d_r); dfree(d_w); dfree(d_l);
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t s = slots[i];
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
  std::lock_guard<std::mutex> g(q->mtx);
  if (!q->reg_h[slot]) return DMC_ENOTREG;
  double v[3] = {inv_of(r), inv_of(w), inv_of(l)};
  HIP_OK(hipMemcpyAsync(q->tb.r_inv + slot, &v[0], 8, hipMemcpyHostToDevice, q->stream));
  HIP_OK(hipMemcpyAsync(q->tb.w_inv + slot, &v[1], 8, hipMemcpyHostToDevice, q->stream));
  HIP_OK(hipMemcpyAsync(q->tb.l_inv + slot, &v[2], 8, hipMemcpyHostToDevice, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  return DMC_OK;
}

int dmc_client_mark_idle(dmc_queue* q, uint32_t slot) {
  if (!q || slot >= q->p.max_clients) return DMC_EINVAL;
  std::lock_guard<std::mutex> g(q->mtx);
  if (!q->reg_h[slot]) return DMC_ENOTREG;
  uint8_t f;
  HIP_OK(hipMemcpyAsync(&f, q->tb.flags + slot, 1, hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  f |= F_IDLE;
  HIP_OK(hipMemcpyAsync(q->tb.flags + slot, &f, 1, hipMemcpyHostToDevice, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  if (!q->idle_h[slot]) {
    q->idle_h[slot] = 1;
    ++q->n_idle;
  }
  return DMC_OK;
}

static int read_handles(dmc_queue* q, uint32_t slot, std::vector<ReqEntry>* ents,
                        uint32_t* head) {
  uint32_t h, c;
  HIP_OK(hipMemcpyAsync(&h, q->tb.head + slot, 4, hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipMemcpyAsync(&c, q->tb.count + slot, 4, hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
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
// only if the front survived
static int write_queue(dmc_queue* q, uint32_t slot, const std::vector<ReqEntry>& ents,
                       bool front_kept) {
  uint32_t Q = q->p.ring_capacity;
  std::vector<ReqEntry> ring(Q);
  for (size_t i = 0; i < ents.size(); ++i) ring[i] = ents[i];
  HIP_OK(hipMemcpyAsync(q->tb.ring + (size_t)slot * Q, ring.data(), sizeof(ReqEntry) * Q,
                        hipMemcpyHostToDevice, q->stream));
  uint32_t z = 0, c = (uint32_t)ents.size();
  HIP_OK(hipMemcpyAsync(q->tb.head + slot, &z, 4, hipMemcpyHostToDevice, q->stream));
  HIP_OK(hipMemcpyAsync(q->tb.count + slot, &c, 4, hipMemcpyHostToDevice, q->stream));
  if (c) {
    HIP_OK(hipMemcpyAsync(q->tb.front_r + slot, &ring[0].r, 8, hipMemcpyHostToDevice, q->stream));
    HIP_OK(hipMemcpyAsync(q->tb.front_p + slot, &ring[0].p, 8, hipMemcpyHostToDevice, q->stream));
    HIP_OK(hipMemcpyAsync(q->tb.front_l + slot, &ring[0].l, 8, hipMemcpyHostToDevice, q->stream));
  }
  uint8_t f;
  HIP_OK(hipMemcpyAsync(&f, q->tb.flags + slot, 1, hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  if (!front_kept || !c) f &= (uint8_t)~F_READY;
  HIP_OK(hipMemcpyAsync(q->tb.flags + slot, &f, 1, hipMemcpyHostToDevice, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  return DMC_OK;
}

int dmc_client_erase(dmc_queue* q, uint32_t slot, uint64_t* handles_out,
                     uint32_t cap, uint32_t* n_out) {
  if (!q || slot >= q->p.max_clients) return DMC_EINVAL;
  std::lock_guard<std::mutex> g(q->mtx);
  if (!q->reg_h[slot]) return DMC_ENOTREG;
  std::vector<ReqEntry> ents;
  uint32_t h;
  int rc = read_handles(q, slot, &ents, &h);
  if (rc) return rc;
  for (size_t i = 0; i < ents.size() && i < cap; ++i)
    if (handles_out) handles_out[i] = ents[i].handle;
  if (n_out) *n_out = (uint32_t)ents.size();
  uint32_t z = 0;
  uint8_t f = 0;
  HIP_OK(hipMemcpyAsync(q->tb.count + slot, &z, 4, hipMemcpyHostToDevice, q->stream));
  HIP_OK(hipMemcpyAsync(q->tb.flags + slot, &f, 1, hipMemcpyHostToDevice, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  if (q->idle_h[slot]) --q->n_idle;
  q->reg_h[slot] = 0;
  q->idle_h[slot] = 0;
  --q->n_registered;
  return DMC_OK;
}

int dmc_client_get_state(dmc_queue* q, uint32_t slot, dmc_client_state* s) {
  if (!q || !s || slot >= q->p.max_clients) return DMC_EINVAL;
  std::lock_guard<std::mutex> g(q->mtx);
  std::memset(s, 0, sizeof(*s));
  const Table& t = q->tb;
  auto D = [&](double* dst, const double* src) {
    return hipMemcpyAsync(dst, src + slot, 8, hipMemcpyDeviceToHost, q->stream);
  };
  uint32_t head = 0;
  uint8_t f = 0;
  HIP_OK(D(&s->prev_r, t.prev_r)); HIP_OK(D(&s->prev_p, t.prev_p));
  HIP_OK(D(&s->prev_l, t.prev_l)); HIP_OK(D(&s->prev_arrival, t.prev_arr));
  HIP_OK(D(&s->prop_delta, t.pd)); HIP_OK(D(&s->front_r, t.front_r));
  HIP_OK(D(&s->front_p, t.front_p)); HIP_OK(D(&s->front_l, t.front_l));
  HIP_OK(D(&s->r_inv, t.r_inv)); HIP_OK(D(&s->w_inv, t.w_inv));
  HIP_OK(D(&s->l_inv, t.l_inv));
  HIP_OK(hipMemcpyAsync(&s->last_tick, t.last_tick + slot, 8, hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipMemcpyAsync(&s->count, t.count + slot, 4, hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipMemcpyAsync(&head, t.head + slot, 4, hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipMemcpyAsync(&s->cur_delta, t.cur_delta + slot, 4, hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipMemcpyAsync(&s->cur_rho, t.cur_rho + slot, 4, hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipMemcpyAsync(&f, t.flags + slot, 1, hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  if (s->count) {
    ReqEntry e;
    HIP_OK(hipMemcpyAsync(&e, t.ring + (size_t)slot * t.q + head, sizeof(e),
                          hipMemcpyDeviceToHost, q->stream));
    HIP_OK(hipStreamSynchronize(q->stream));
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
  std::lock_guard<std::mutex> g(q->mtx);
  HIP_OK(hipMemcpyAsync(out, q->tb.last_tick, 8ull * n, hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  return DMC_OK;
}

int dmc_add_batch(dmc_queue* q, uint32_t n, const dmc_request* reqs,
                  int32_t* rc_out) {
  if (!q || (n && !reqs)) return DMC_EINVAL;
  std::lock_guard<std::mutex> g(q->mtx);
  if (!n) return DMC_OK;
  int rc = ensure_batch(q, n);
  if (rc) return rc;
  HIP_OK(hipMemcpyAsync(q->d_reqs, reqs, sizeof(dmc_request) * n,
                        hipMemcpyHostToDevice, q->stream));
  rc = q->n_idle ? add_host_split(q, reqs, n, q->d_reqs, q->d_rc)
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
  std::lock_guard<std::mutex> g(q->mtx);
  if (!n) return DMC_OK;
  int rc = ensure_batch(q, n);
  if (rc) return rc;
  if (q->n_idle) {
    // activations need the host-ordered split: stage the batch on the host
    std::vector<dmc_request> h(n);
    HIP_OK(hipMemcpyAsync(h.data(), d_reqs, sizeof(dmc_request) * n,
                          hipMemcpyDeviceToHost, q->stream));
    HIP_OK(hipStreamSynchronize(q->stream));
    rc = add_host_split(q, h.data(), n, d_reqs, d_rc_out);
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
  std::lock_guard<std::mutex> g(q->mtx);
  int rc = ensure_dec(q, k);
  if (rc) return rc;
  dmc_pull_result r{};
  rc = pull_impl(q, now, k, q->d_dec, &r);
  if (rc) return rc;
  if (r.n_decisions)
    HIP_OK(hipMemcpyAsync(out, q->d_dec, sizeof(dmc_decision) * r.n_decisions,
                          hipMemcpyDeviceToHost, q->stream));
  HIP_OK(hipStreamSynchronize(q->stream));
  for (uint32_t i = 0; i < r.n_decisions; ++i)
    (out[i].phase == DMC_PHASE_RESERVATION ? r.n_reservation : r.n_priority)++;
  if (result) *result = r;
  return DMC_OK;
}

int dmc_pull_batch_device(dmc_queue* q, double now, uint32_t k,
                          dmc_decision* d_out, dmc_pull_result* d_result) {
  if (!q || (k && !d_out)) return DMC_EINVAL;
  std::lock_guard<std::mutex> g(q->mtx);
  dmc_pull_result r{};
  int rc = pull_impl(q, now, k, d_out, &r);
  if (rc) return rc;
  if (d_result) {
    // stream-ordered: pull_impl has synchronised, so the pinned staging
    // record is free, and the copy completes before any later work
    *q->h_res = r;
    HIP_OK(hipMemcpyAsync(d_result, q->h_res, sizeof(r), hipMemcpyHostToDevice,
                          q->stream));
  }
  return DMC_OK;
}

int dmc_remove_by_client(dmc_queue* q, uint32_t slot, int reverse,
                         uint64_t* handles_out, uint32_t cap, uint32_t* n_out) {
  if (!q || slot >= q->p.max_clients) return DMC_EINVAL;
  std::lock_guard<std::mutex> g(q->mtx);
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
  return write_queue(q, slot, {}, false);
}

int dmc_client_requests(dmc_queue* q, uint32_t slot, uint64_t* handles_out,
                        uint32_t cap, uint32_t* n_out) {
  if (!q || slot >= q->p.max_clients) return DMC_EINVAL;
  std::lock_guard<std::mutex> g(q->mtx);
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
  std::lock_guard<std::mutex> g(q->mtx);
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
  return write_queue(q, slot, kept, n > 0 && keep[0]);
}

int dmc_queue_set_option(dmc_queue* q, int option, int64_t value) {
  if (!q) return DMC_EINVAL;
  std::lock_guard<std::mutex> g(q->mtx);
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
      if (!q->use_graphs) invalidate_graphs(q);
      return DMC_OK;
    default:
      return DMC_EINVAL;
  }
}

int dmc_profile_enable(dmc_queue* q, int on) {
  if (!q) return DMC_EINVAL;
  std::lock_guard<std::mutex> g(q->mtx);
  q->prof_on = on != 0;
  q->prof_n = 0;
  return DMC_OK;
}

int dmc_profile_reset(dmc_queue* q) {
  if (!q) return DMC_EINVAL;
  std::lock_guard<std::mutex> g(q->mtx);
  for (int i = 0; i < DMC_PROF_NSTAGES; ++i) {
    q->prof_ms[i] = 0.0;
    q->prof_cnt[i] = 0;
  }
  return DMC_OK;
}

int dmc_profile_read(dmc_queue* q, uint32_t stage, uint64_t* count,
                     double* total_ms) {
  if (!q || stage >= DMC_PROF_NSTAGES) return DMC_EINVAL;
  std::lock_guard<std::mutex> g(q->mtx);
  if (count) *count = q->prof_cnt[stage];
  if (total_ms) *total_ms = q->prof_ms[stage];
  return DMC_OK;
}

const char* dmc_profile_stage_name(uint32_t stage) {
  return stage < DMC_PROF_NSTAGES ? kStageNames[stage] : "";
}

int dmc_stats_get(dmc_queue* q, dmc_stats* out) {
  if (!q || !out) return DMC_EINVAL;
  std::lock_guard<std::mutex> g(q->mtx);
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
