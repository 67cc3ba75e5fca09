// SPDX-License-Identifier: LGPL-2.1
//
// dmc_heap.h -- tie-exact dispatch (DMC_OPT_HEAP_ORDER): the reference's
// three indirect heaps kept on the device and driven in the reference's
// order, so that among equal keys the winner is the reference's heap top.
//
// The engine's rounds break ties by lowest slot: the
// reference's winner among equal keys is whichever tied client sits at index
// 0 of its IndIntruHeap, a function of every sift since the queue was built
// (support/src/indirect_intrusive_heap.h:240-564; comparators
// src/dmclock_server.h:722-757).  No client attribute predicts it, so a
// caller that needs the reference's exact dispatch sequence on tie-heavy
// traces (closed loops of identical clients, config 2 without jitter) turns
// this mode on: every add and pull then runs in call order on one workgroup
// of the device, with the heaps as arrays of slots plus each slot's index in
// each heap, and the same per-client state (ScanRec / ClientRec / ring) and
// tag arithmetic as every other path.  It trades the rounds' throughput for
// the heap's sequential semantics; the heaps' top decides, exactly as
// do_next_request does (:1115-1186).
//
// Heap order per operation (what the reference calls, in its order):
//   register      resv.push, limit.push, ready.push            (:925-931)
//   add           the idle reset (:937-985); initial_tag; Reject returns
//                 before any heap call (:989-993); a first request adjusts
//                 the three heaps (:996-1006), every accepted one again
//                 (:1011-1016)
//   pull          the resv top if due (:1124-1128); the limit loop's ready
//                 marks with ready.promote / limit.demote (:1135-1144); the
//                 ready top if ready (:1146-1151); Allow's fallbacks
//                 (:1157-1165); future / none (:1170-1185).  A pop
//                 (:1046-1073): pop the front, update_next_tag, then
//                 resv.demote, limit.adjust, ready.demote; a priority pop
//                 then reduce_reservation_tags and resv.promote (:1098-1111)
//   erase         resv, limit, ready remove (delete_from_heaps, :1259-1275)
//   filter, remove_by_client   adjust x 3 for each modified client (:567-625)
// (included by dmc_engine.hip inside its anonymous namespace, after the
// step path's helpers)
#pragma once

enum : int { kHResv = 0, kHLim = 1, kHReady = 2 };

struct HeapDev {
  uint32_t* hp;   // [3][n] heap arrays (slots)
  uint32_t* hix;  // [3][n] each slot's index in each heap
  uint32_t* cnt;  // [3] heap sizes
  uint32_t n, k;  // capacity, branching (IndIntruHeap's K)
};

// ClientCompare (:722-757): clients with a request precede those without;
// resv by r; limit: not-ready first (ReadyOption::lowers), then l; ready:
// ready first (raises), then p + prop_delta (the cached pk, the same double
// add); strict less.
__device__ inline bool heap_less(const Table& tb, int h, uint32_t a, uint32_t b) {
  const ScanRec ra = tb.sc[a], rb = tb.sc[b];
  if (!ra.count) return false;
  if (!rb.count) return true;
  if (h == kHResv) return ra.r < rb.r;
  const bool rda = (ra.flags & F_READY) != 0, rdb = (rb.flags & F_READY) != 0;
  if (h == kHLim) return rda == rdb ? ra.l < rb.l : rdb;
  return rda == rdb ? ra.pk < rb.pk : rda;
}

// One heap, IndIntruHeap's algorithms (indirect_intrusive_heap.h): sift_up
// moves only on strict less (:462-474); K == 2 sift_down takes the left child
// unless the right one is strictly smaller (:514-548), K > 2 the first
// smallest child (:479-510); sift picks the direction (:550-564); remove
// swaps in the last element and sifts with the count already reduced, the
// removed element still in the array (:433-445).
struct HeapRef {
  const Table& tb;
  int h;
  uint32_t* a;  // the heap array
  uint32_t* x;  // slot -> index
  uint32_t* cnt;
  uint32_t k;
  __device__ HeapRef(const Table& t, const HeapDev& d, int hh)
      : tb(t), h(hh), a(d.hp + (size_t)hh * d.n), x(d.hix + (size_t)hh * d.n),
        cnt(d.cnt + hh), k(d.k) {}
  __device__ bool less(uint32_t i, uint32_t j) const { return heap_less(tb, h, a[i], a[j]); }
  __device__ void swap(uint32_t i, uint32_t j) {
    const uint32_t si = a[i], sj = a[j];
    a[i] = sj;
    a[j] = si;
    x[sj] = i;
    x[si] = j;
  }
  __device__ void sift_up(uint32_t i) {
    while (i > 0) {
      const uint32_t p = (i - 1) / k;
      if (!less(i, p)) break;
      swap(i, p);
      i = p;
    }
  }
  __device__ void sift_down(uint32_t i, uint32_t n) {
    if (i >= n) return;
    if (k == 2) {
      for (;;) {
        const uint32_t li = 2 * i + 1, ri = li + 1;
        if (li >= n) break;
        if (less(li, i)) {
          if (ri < n && less(ri, li)) {
            swap(i, ri);
            i = ri;
          } else {
            swap(i, li);
            i = li;
          }
        } else if (ri < n && less(ri, i)) {
          swap(i, ri);
          i = ri;
        } else {
          break;
        }
      }
      return;
    }
    for (;;) {
      const uint32_t li = k * i + 1;
      if (li >= n) break;
      const uint32_t ri = min(k * i + k, n - 1);
      uint32_t mi = li;
      for (uint32_t c = li + 1; c <= ri; ++c)
        if (less(c, mi)) mi = c;
      if (!less(mi, i)) break;
      swap(i, mi);
      i = mi;
    }
  }
  __device__ void sift(uint32_t i, uint32_t n) {
    if (i == 0) sift_down(i, n);
    else if (less(i, (i - 1) / k)) sift_up(i);
    else sift_down(i, n);
  }
  __device__ void push(uint32_t s) {
    const uint32_t i = *cnt;
    a[i] = s;
    x[s] = i;
    *cnt = i + 1;
    sift_up(i);
  }
  __device__ void remove_slot(uint32_t s) {
    const uint32_t i = x[s], last = *cnt - 1;
    swap(i, last);
    sift(i, last);
    *cnt = last;
  }
  __device__ void promote(uint32_t s) { sift_up(x[s]); }
  __device__ void demote(uint32_t s) { sift_down(x[s], *cnt); }
  __device__ void adjust(uint32_t s) { sift(x[s], *cnt); }
  __device__ uint32_t top() const { return a[0]; }
};

struct Heaps {
  HeapRef resv, lim, ready;
  __device__ Heaps(const Table& t, const HeapDev& d)
      : resv(t, d, kHResv), lim(t, d, kHLim), ready(t, d, kHReady) {}
  __device__ void adjust3(uint32_t s) {
    resv.adjust(s);
    lim.adjust(s);
    ready.adjust(s);
  }
};

// ------------------------------------------------------------------ kernels
// registration (client_map.emplace + three pushes, in the given order)
__global__ void k_heap_push(Table tb, HeapDev hd, const uint32_t* slots, uint32_t n) {
  if (threadIdx.x) return;
  Heaps H(tb, hd);
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t s = slots[i];
    H.resv.push(s);
    H.lim.push(s);
    H.ready.push(s);
  }
}

// erase (delete_from_heaps, before the client's state goes)
__global__ void k_heap_remove(Table tb, HeapDev hd, const uint32_t* slots, uint32_t n) {
  if (threadIdx.x) return;
  Heaps H(tb, hd);
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t s = slots[i];
    H.resv.remove_slot(s);
    H.lim.remove_slot(s);
    H.ready.remove_slot(s);
  }
}

// clients whose queues a filter / remove_by_client modified, ascending
__global__ void k_heap_adjust(Table tb, HeapDev hd, const uint32_t* slots, uint32_t n) {
  if (threadIdx.x) return;
  Heaps H(tb, hd);
  for (uint32_t i = 0; i < n; ++i) H.adjust3(slots[i]);
}

constexpr int kHeapThreads = 256;

// The idle reset's minimum (:957-978) over every registered non-idle client
// but `self`: the block reduces (front p or prev p) + prop_delta as ordered
// keys; every thread returns it.
__device__ inline double heap_idle_lowest(const Table& tb, uint64_t* sh) {
  uint64_t m = kMaxKey;
  for (uint32_t s = threadIdx.x; s < tb.n; s += blockDim.x) {
    const ScanRec r = tb.sc[s];
    if (!(r.flags & F_REG) || (r.flags & F_IDLE)) continue;
    const double v = r.count ? r.pk : __dadd_rn(tb.rec[s].prev_p, tb.rec[s].pd);
    const uint64_t o = okey(v);
    m = o < m ? o : m;
  }
  for (int d = 32; d > 0; d >>= 1) {
    const uint64_t o = shfl_down_u64(m, d);
    m = o < m ? o : m;
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = m;
  __syncthreads();
  uint64_t r = kMaxKey;
  for (uint32_t w = 0; w < blockDim.x / 64; ++w) r = sh[w] < r ? sh[w] : r;
  __syncthreads();
  return r == kMaxKey ? 1.7976931348623157e308 : from_okey(r);
}

// n add_request_time calls in order (do_add_request, :913-1018)
__global__ void __launch_bounds__(kHeapThreads) k_heap_add(Table tb, HeapDev hd, AddParams p) {
  __shared__ uint64_t sh[kHeapThreads / 64];
  __shared__ uint32_t s_idle;
  Heaps H(tb, hd);
  for (uint32_t i = 0; i < p.n; ++i) {
    const uint32_t s = p.reqs[i].slot;
    if (threadIdx.x == 0) s_idle = s < tb.n && (tb.sc[s].flags & (F_REG | F_IDLE)) == (F_REG | F_IDLE);
    __syncthreads();
    const bool idle = s_idle != 0;
    double lowest = 0.0;
    if (idle) lowest = heap_idle_lowest(tb, sh);  // (the client itself is idle: not counted)
    if (threadIdx.x == 0) {
      if (s >= tb.n || !(tb.sc[s].flags & F_REG)) {
        p.rc[i] = DMC_ENOTREG;
      } else {
        if (idle) {  // :981-984 (prop_delta kept when the trigger does not fire)
          const double trigger = 1.7976931348623157e308 / 3.0;
          const double pd = lowest < trigger ? __dsub_rn(lowest, p.reqs[i].time) : tb.rec[s].pd;
          tb.rec[s].pd = pd;
          const ScanRec r = tb.sc[s];
          if (r.count) tb.sc[s].pk = __dadd_rn(tb.ring[(size_t)s * tb.q + (r.head & tb.qmask)].p, pd);
          tb.sc[s].flags = (uint8_t)(r.flags & ~F_IDLE);
        }
        const uint32_t count0 = tb.sc[s].count;
        AddState st;
        add_chain_slot(tb, p, s, 1, i, nullptr, nullptr, ActBuf{}, &st);
        if (p.rc[i] == DMC_OK) {
          if (count0 == 0) H.adjust3(s);  // a first request (:996-1006)
          H.adjust3(s);                   // (:1011-1016)
        }
      }
    }
    __syncthreads();
  }
}

// The pop of the top of heap `hsel` (pop_process_request, :1046-1073, with
// reduce_reservation_tags, :1077-1111, for a priority pop): the decision,
// the front popped and (delayed) the new front's tag (update_next_tag,
// :1021-1036), the heap calls with that state, then the reduction and
// resv.promote.
__device__ inline void heap_pop(const Table& tb, Heaps& H, uint32_t s, bool prio, uint64_t tick,
                                dmc_decision* out, unsigned long long* sched) {
  ReqEntry* ring = tb.ring + (size_t)s * tb.q;
  const ScanRec sr = tb.sc[s];
  const uint32_t h = sr.head, c = sr.count;
  const ReqEntry popped = ring[h];
  dmc_decision d;
  d.handle = popped.handle;
  d.tag_r = popped.r;
  d.tag_p = popped.p;
  d.tag_l = popped.l;
  d.slot = s;
  d.cost = popped.cost;
  d.phase = prio ? DMC_PHASE_PRIORITY : DMC_PHASE_RESERVATION;
  d.flags = 0;  // (the heap top is the reference's winner: no tie to flag)
  *out = d;
  const uint32_t nh = (h + 1) & tb.qmask, nc = c - 1;
  double rinv = tb.rec[s].r_inv;
  if (tb.delayed && nc) {  // update_next_tag
    ReqEntry& f = ring[nh];
    const Tag3 pt{popped.r, popped.p, popped.l, popped.arrival};
    Tag3 nt;
    const uint32_t cd = tb.aux[s].cur_delta, cr = tb.aux[s].cur_rho;
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
    if (make_tag(pt, rinv, winv, linv, cd, cr, f.arrival, f.cost, tb.antic, &nt)) {
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
  ScanRec o{0.0, 0.0, 0.0, (uint8_t)nh, (uint8_t)nc, (uint8_t)(sr.flags & ~F_READY), 0, 0};
  if (nc) {
    const ReqEntry& f = ring[nh];
    o.r = f.r;
    o.pk = __dadd_rn(f.p, tb.rec[s].pd);
    o.l = f.l;
  }
  tb.sc[s] = o;
  H.resv.demote(s);
  H.lim.adjust(s);
  H.ready.demote(s);
  if (prio) {
    const double off = resv_offset(rinv, popped.cost, popped.rho);
    if (tb.delayed) {
      if (nc) ring[nh].r = __dsub_rn(ring[nh].r, off);
    } else {
      for (uint32_t i = 1; i < c; ++i) {
        ReqEntry& e = ring[(h + i) & tb.qmask];
        e.r = __dsub_rn(e.r, off);
      }
    }
    tb.rec[s].prev_r = __dsub_rn(tb.rec[s].prev_r, off);
    if (nc) tb.sc[s].r = ring[nh].r;
    H.resv.promote(s);
  }
  atomicAdd(&sched[prio ? 1 : 0], 1ull);
}

struct HeapPullRes {
  uint32_t n, n_res, n_prio;
  int32_t type;
  double when;
  uint32_t pend_slot, pend_prio;  // mode 1: the decided pop, left to mode 2
};

// k pull_request(now) calls in order (do_next_request, :1115-1186).
// mode 0: all k; mode 1 (U1 with a host client_info_f, delayed: the host
// fetches the popped client's info between selection and pop, :870-875,
// :1021-1036): one pull decided -- the limit loop's marks made -- and its
// pop left in res->pend_*; mode 2: that pop.
__global__ void k_heap_pull(Table tb, HeapDev hd, double now, uint32_t k, int at_limit,
                            uint64_t tick, dmc_decision* out, HeapPullRes* res,
                            dmc_pull_result* d_result, unsigned long long* sched,
                            int mode = 0) {
  if (threadIdx.x) return;
  Heaps H(tb, hd);
  HeapPullRes r{0, 0, 0, DMC_NEXT_RETURNING, 0.0, 0, 0};
  if (mode == 2) {
    const HeapPullRes pr = *res;
    heap_pop(tb, H, pr.pend_slot, pr.pend_prio != 0, tick, out, sched);
    r.n = 1;
    if (pr.pend_prio) r.n_prio = 1;
    else r.n_res = 1;
    *res = r;
    return;
  }
  // each iteration decides one pull (pop_slot / pop_prio) or stops; the pop
  // is made at its end (mode 1: recorded for mode 2 instead)
  while (r.n < k) {
    uint32_t pop_slot = kNone;
    bool pop_prio = false;
    if (*H.resv.cnt == 0) {  // no clients: none (:1118-1120)
      r.type = DMC_NEXT_NONE;
      break;
    }
    const uint32_t rs = H.resv.top();
    const ScanRec rsr = tb.sc[rs];
    if (rsr.count && rsr.r <= now) {
      pop_slot = rs;
    } else {
      for (;;) {  // the limit loop
        const uint32_t ls = H.lim.top();
        const ScanRec lr = tb.sc[ls];
        if (!(lr.count && !(lr.flags & F_READY) && lr.l <= now)) break;
        tb.sc[ls].flags = (uint8_t)(lr.flags | F_READY);
        H.ready.promote(ls);
        H.lim.demote(ls);
      }
      const uint32_t ps = H.ready.top();
      const ScanRec pr = tb.sc[ps];
      if (pr.count && (pr.flags & F_READY) && pr.pk < kInf) {
        pop_slot = ps;
        pop_prio = true;
      } else if (at_limit == DMC_AT_LIMIT_ALLOW && pr.count && pr.pk < kInf) {
        pop_slot = ps;
        pop_prio = true;
      } else if (at_limit == DMC_AT_LIMIT_ALLOW && rsr.count && rsr.r < kInf) {
        pop_slot = rs;
      }
    }
    if (pop_slot == kNone) {
      // future / none (:1170-1185; min_not_0_time excludes exact 0,
      // :1192-1195; kTimeMax = DBL_MAX: an infinite tag is no future)
      constexpr double kTimeMax = 1.7976931348623157e308;
      double next = kTimeMax;
      const uint32_t rt = H.resv.top(), lt = H.lim.top();
      if (tb.sc[rt].count) {
        const double v = tb.sc[rt].r;
        if (v != 0.0) next = v < next ? v : next;
      }
      if (tb.sc[lt].count) {
        const double v = tb.sc[lt].l;
        if (v != 0.0) next = v < next ? v : next;
      }
      if (next < kTimeMax) {
        r.type = DMC_NEXT_FUTURE;
        r.when = next;
      } else {
        r.type = DMC_NEXT_NONE;
      }
      break;
    }
    if (mode == 1) {
      r.pend_slot = pop_slot;
      r.pend_prio = pop_prio ? 1u : 0u;
      break;
    }
    heap_pop(tb, H, pop_slot, pop_prio, tick, out + r.n, sched);
    ++r.n;
    if (pop_prio) ++r.n_prio;
    else ++r.n_res;
  }
  *res = r;
  if (d_result) {
    dmc_pull_result x{};
    x.n_decisions = r.n;
    x.next_type = r.type;
    x.when = r.type == DMC_NEXT_FUTURE ? r.when : 0.0;
    x.n_priority = r.n_prio;
    x.n_reservation = r.n_res;
    *d_result = x;
  }
}

