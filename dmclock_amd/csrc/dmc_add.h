// SPDX-License-Identifier: LGPL-2.1
//
// dmc_add.h -- the add path's per-client replay (do_add_request,
// dmclock_server.h:913-1018, minus the idle reset): shared by k_add_chain
// (one thread per client of a batch) and by k_rscan when an add batch and a
// pull round run as one launch sequence (the scan thread that owns a slot
// replays that slot's requests of the batch before scanning it).
#pragma once

#include "dmc_device.h"

namespace dmc {

// A batch (a run of add_request_time calls with no activation inside) is
// grouped by client without sorting: k_add_link counts each client's requests
// with one atomic per request on the client's ScanRec line (ScanRec::nadd,
// the line k_add_chain reads anyway) and files the batch positions of the
// client's later filers (filing order 1 .. kAddSlots - 1) in its slot buffer;
// k_add_chain then lets the first filer replay that client's requests in
// batch order.  Clients with more than kAddSlots requests in the batch (rare:
// 64K requests over 1M clients is Poisson(1/16)) are replayed by a scan of
// the batch's slot column, in order.
constexpr uint32_t kAddSlots = 16;

struct AddParams {
  const dmc_request* reqs;
  int32_t* rc;
  uint64_t tick_base;
  uint32_t n;
  uint32_t epoch;  // k_chain_scan's batches: k_add_link stamps the batch's slots with it
                   // (Table::touch) so that the scan beside the chain leaves them; else 0
};

// Batched activations (the idle reset of every idle client's first request
// in one batch, resolved on the device; see k_act_resolve).  A non-idle
// client with an empty queue contributes (prev p) + prop_delta until its
// first accepted request, then (front p) + prop_delta; each of its requests
// up to that one may change it (under AtLimit::Reject a rejected request
// still moves prev p, :899-906), and the values never decrease (a tag is
// max(time, prev + increment) >= prev, or the max_tag a weight of 0 gives).
// Per batch position where the contribution changed: the value before the
// change (cold, stored at index n - 1 - position); at the client's last change
// the value after it (cnew).  An activation at position q then sees the
// client's current value as min(suffix minimum of cold over positions > q,
// prefix minimum of cnew over positions < q) -- the value before the first
// later change, or after the last one.  At an activation position the
// post-add proportion basis (actp: front p if the client has a request, else
// prev p).
struct ActBuf {
  uint64_t* cold;
  uint64_t* cnew;
  double* actp;
  uint64_t* pre;     // exclusive prefix minima of cnew
  uint64_t* suf;     // exclusive prefix minima of cold (reversed): suffix minima
  const uint32_t* idx;  // activation positions, ascending
  uint32_t m;
  const uint64_t* parts;  // k_act_base partials
  uint32_t nparts;
  uint64_t* extra;   // contributions of touched empty clients left unchanged
  // device-detected activations (dmc_add_batch_device): k_add_chain flags
  // each activating position, a compaction builds idx and the count *dm
  uint32_t* flag = nullptr;
  const uint32_t* dm = nullptr;
  // AtLimit::Reject: an activated client whose activating request was
  // rejected stays empty, and each later request of the batch may move its
  // proportion basis until one is accepted.  At such a change (position r):
  // hev_q[r] = the client's activation position, hev_p[r] = its new basis;
  // hard[activation position] = 1 and *anyhard = 1 (k_act_hard resolves the
  // batch).  hev_q is kNone elsewhere.
  uint32_t* hev_q = nullptr;
  double* hev_p = nullptr;
  uint32_t* hard = nullptr;
  uint32_t* anyhard = nullptr;
};

// Client trackers fused into the add (a queue group's step, config 5):
// get_req_params (dmclock_client.h:241-251) for every request of the batch,
// written into the request before its tag is calculated -- the first request
// of a (server, client) pair in batch order gets the responses since its
// previous request (or (1, 1) from a server it never asked), later ones
// (0, 0) -- exactly what dmc_tracker_fill's two kernels compute, without
// their separate passes over the batch.
struct TrackFill {
  dmc_request* reqs;  // the batch (delta / rho written back)
  const uint32_t *cmap, *gd, *gr;
  uint32_t *xd, *xr;
  uint8_t* known;
  uint32_t nslots;
};

// (the pair's state, loaded ahead: *c the global client; its counters next)
struct TrackSlot {
  uint32_t xd, xr, c;
  uint8_t known;
};
__device__ inline TrackSlot track_load(const TrackFill& t, uint32_t s) {
  return TrackSlot{t.xd[s], t.xr[s], t.cmap ? t.cmap[s] : s, t.known[s]};
}
// the first request's parameters; the pair's state moves to the counters
__device__ inline void track_first(const TrackFill& t, uint32_t s, const TrackSlot& ts,
                                   uint32_t D, uint32_t R, uint32_t* delta, uint32_t* rho) {
  if (!ts.known) {
    t.known[s] = 1;
    *delta = 1;
    *rho = 1;
  } else {
    *delta = D - ts.xd;
    *rho = R - ts.xr;
  }
  t.xd[s] = D;
  t.xr[s] = R;
}

// do_add_request for one client's requests of the batch, in batch order:
// minus the idle reset (handled before, per activation), initial_tag
// (:878-907), the Reject check (:989-993), the enqueue and cur_rho/cur_delta
// (:995-1009).
struct AddState {
  Tag3 prev;
  double rinv, winv, linv;  // client.info (U1: replaced at each tag calculation)
  BoundInfo bound;          // U1: what client_info_f returns now
  bool fetched;             // U1: a tag calculation fetched the bound info
  uint32_t head, count, cd, cr;
  uint64_t last_tick;
  uint8_t flags;
  bool front_set;
  bool cd_set, tick_set;    // cur_delta / cur_rho, last_tick changed (ClientAux is
                            // written, never read, by the add path)
  Tag3 front;
  // the batch's first two enqueued requests' r, p, l (add_chain_slot, for
  // k_chain_scan's scan of the slot)
  double n0r, n0p, n0l, n1r, n1p, n1l;
  uint32_t nq = 0;          // requests enqueued by the batch so far
};

__device__ inline void add_one(const Table& tb, AddState& st, ReqEntry* ring,
                               const AddParams& p, uint32_t pos,
                               const dmc_request* pre = nullptr) {
  const dmc_request rq = pre ? *pre : p.reqs[pos];
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
    if (tb.binfo) {  // get_cli_info, :870-875
      st.rinv = st.bound.r_inv;
      st.winv = st.bound.w_inv;
      st.linv = st.bound.l_inv;
      st.fetched = true;
    }
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
    st.tick_set = true;
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
  e.dec = kNoDec;
  e.tie = 0;
  e.pad = 0;
  ring[(st.head + st.count) & tb.qmask] = e;
  if (st.nq == 0) {
    st.n0r = tag.r;
    st.n0p = tag.p;
    st.n0l = tag.l;
  } else if (st.nq == 1) {
    st.n1r = tag.r;
    st.n1p = tag.p;
    st.n1l = tag.l;
  }
  ++st.nq;
  if (st.count == 0) {
    st.front = tag;
    st.front_set = true;
    st.flags &= (uint8_t)~F_READY;  // a new tag is not ready, :155
  }
  ++st.count;
  st.cd = rq.delta;
  st.cr = rq.rho;
  st.cd_set = true;
  p.rc[pos] = DMC_OK;
}

// Slot s of the batch is not registered: every request of it gets ENOTREG
// (with fused trackers its requests still get their parameters, as
// dmc_tracker_fill gives them to every request of a table slot).
__device__ inline void add_chain_notreg(const AddParams& p, uint32_t s, uint32_t m,
                                        uint32_t i1, const uint32_t* abuf,
                                        const uint32_t* aslot, const TrackFill* tf = nullptr) {
  if (tf && s < tf->nslots) {
    uint32_t first = i1;
    if (m <= kAddSlots) {
      for (uint32_t j = 1; j < m; ++j) first = min(first, abuf[(size_t)s * kAddSlots + j]);
    } else {
      for (uint32_t j = 0; j < p.n; ++j)
        if (aslot[j] == s) {
          first = j;
          break;
        }
    }
    const TrackSlot ts = track_load(*tf, s);
    uint32_t d0, r0;
    track_first(*tf, s, ts, tf->gd[ts.c], tf->gr[ts.c], &d0, &r0);
    auto put = [&](uint32_t pos) {
      tf->reqs[pos].delta = pos == first ? d0 : 0u;
      tf->reqs[pos].rho = pos == first ? r0 : 0u;
    };
    if (m <= kAddSlots) {
      put(i1);
      for (uint32_t j = 1; j < m; ++j) put(abuf[(size_t)s * kAddSlots + j]);
    } else {
      for (uint32_t j = 0; j < p.n; ++j)
        if (aslot[j] == s) put(j);
    }
  }
  if (m <= kAddSlots) {
    p.rc[i1] = DMC_ENOTREG;
    for (uint32_t j = 1; j < m; ++j) p.rc[abuf[(size_t)s * kAddSlots + j]] = DMC_ENOTREG;
  } else {
    for (uint32_t j = 0; j < p.n; ++j)
      if (aslot[j] == s) p.rc[j] = DMC_ENOTREG;
  }
}

// The replay of slot s's m requests of the batch (m = its batch count, read
// with the client's state from ScanRec::nadd when `counted`, which is then
// reset for the next batch; i1: the first filer's batch position, the other
// positions in abuf, or found by a scan of the slot column when m >
// kAddSlots), in batch order, with the activation bookkeeping of ActBuf when
// act.cold is set.  An unregistered slot (checked here when counted) rejects
// its requests.  Leaves the slot's new state in *out (count, flags, front
// when set).  Every load is issued before the first store (on gfx950 a
// load's wait also waits for the wave's earlier stores); ClientAux is only
// written.
__device__ inline void add_chain_slot(const Table& tb, const AddParams& p, uint32_t s,
                                      uint32_t m, uint32_t i1, const uint32_t* abuf,
                                      const uint32_t* aslot, const ActBuf& act,
                                      AddState* out, bool counted = false,
                                      const TrackFill* tf = nullptr) {
  const uint32_t i = i1;
  // position i1's request, requested with the client's state (the usual
  // case, m == 1, needs nothing else from the batch)
  const dmc_request rq1 = p.reqs[i];
  // fused trackers: the pair's state with the client's, its counters next
  TrackSlot ts{};
  uint32_t tD = 0, tR = 0;
  if (tf) {
    ts = track_load(*tf, s);
    tD = tf->gd[ts.c];
    tR = tf->gr[ts.c];
  }
  // the ScanRec's cursor word: head, count, flags and the batch count
  ScanRec* const cw = tb.sc + s;
  const uint64_t cur = cursor_load(cw);
  if (counted) m = (uint32_t)(cur >> 32);
  AddState st;
  st.prev = Tag3{tb.rec[s].prev_r, tb.rec[s].prev_p, tb.rec[s].prev_l, tb.rec[s].prev_arr};
  st.rinv = tb.rec[s].r_inv;
  st.winv = tb.rec[s].w_inv;
  st.linv = tb.rec[s].l_inv;
  st.fetched = false;
  if (tb.binfo) st.bound = tb.binfo[s];
  const double pd = tb.rec[s].pd;
  st.head = (uint32_t)(cur & 0xffu);
  st.count = (uint32_t)((cur >> 8) & 0xffu);
  st.flags = (uint8_t)(cur >> 16);
  st.cd = st.cr = 0;
  st.last_tick = 0;
  st.cd_set = st.tick_set = false;
  st.front_set = false;
  ReqEntry* ring = tb.ring + (size_t)s * tb.q;
  // batched activations: this client's contribution to the idle reset before
  // and after its requests (see ActBuf)
  // the cursor word as stored back: the batch count cleared for the next batch
  auto store_cursor = [&] {
    cursor_store(cw, (uint64_t)(st.head & 0xffu) | ((uint64_t)(st.count & 0xffu) << 8) |
                         ((uint64_t)st.flags << 16) | (cur & 0xff000000ull));
  };
  if (counted && !(st.flags & F_REG)) {
    store_cursor();  // (unchanged; the batch count cleared)
    add_chain_notreg(p, s, m, i, abuf, aslot, tf);
    return;
  }
  const bool idle0 = (st.flags & F_IDLE) != 0;
  const uint32_t count0 = st.count;
  const double front_p0 = (act.cold && count0) ? ring[st.head & tb.qmask].p : 0.0;
  const double prev_p0 = st.prev.p;
  bool act_done = false, chg_done = false, tf_done = false;
  // (the empty client's proportion basis as of the last step, and the batch
  // position of its last change; an activated client left empty: its
  // activation position, while it stays empty)
  double cur_p = prev_p0;
  uint32_t chg_last = 0xffffffffu, act_q = 0xffffffffu;
  auto step = [&](uint32_t pos) {
    // (heap order: the reference's heap calls for this request, below)
    const uint32_t cnt_before = st.count;
    const bool activating = tb.hev && act.cold && idle0 && !act_done &&
                            p.reqs[pos].rho <= p.reqs[pos].delta;
    if (tf) {  // get_req_params, batch order
      dmc_request rq = pos == i ? rq1 : p.reqs[pos];
      rq.delta = rq.rho = 0;
      if (!tf_done) {
        tf_done = true;
        track_first(*tf, s, ts, tD, tR, &rq.delta, &rq.rho);
      }
      tf->reqs[pos].delta = rq.delta;
      tf->reqs[pos].rho = rq.rho;
      add_one(tb, st, ring, p, pos, &rq);
    } else {
      add_one(tb, st, ring, p, pos, pos == i ? &rq1 : nullptr);
    }
    if (tb.hev) {
      // an accepted request: adjust x 3, twice for a client's first (:996-1016);
      // a refused activation: the idle reset's prop_delta moved the ready
      // key of a client with requests, and no heap call follows (:989-993)
      uint8_t e = 0;
      if (p.rc[pos] == DMC_OK) e = cnt_before == 0 ? 3 : 2;
      else if (activating && st.count > 0) e = 1;
      tb.hev[pos] = e;
    }
    if (!act.cold) return;
    if (idle0) {
      const dmc_request& rq = p.reqs[pos];
      if (!act_done && rq.rho <= rq.delta) {  // the activating request
        act_done = true;
        cur_p = st.count ? (count0 ? front_p0 : st.front.p) : st.prev.p;
        act.actp[pos] = cur_p;
        if (act.flag) act.flag[pos] = 1;
        if (!st.count) act_q = pos;  // rejected (or no tag): still empty
      } else if (act_q != 0xffffffffu) {
        const double np = st.count ? st.front.p : st.prev.p;
        if (dbits(np) != dbits(cur_p)) {
          cur_p = np;
          act.hev_q[pos] = act_q;
          act.hev_p[pos] = np;
          if (!act.hard[act_q]) {
            act.hard[act_q] = 1u;
            *act.anyhard = 1u;
          }
        }
        if (st.count) act_q = 0xffffffffu;
      }
    } else if (count0 == 0 && !chg_done) {
      const double np = st.count ? st.front.p : st.prev.p;
      if (dbits(np) != dbits(cur_p)) {
        act.cold[p.n - 1 - pos] = okey(__dadd_rn(cur_p, pd));  // reversed order
        cur_p = np;
        chg_last = pos;
      }
      chg_done = st.count != 0;
    }
  };
  if (m == 1) {
    step(i);
  } else if (m <= kAddSlots) {
    // the client's batch positions in ascending order, by repeated selection
    // over its (L2-resident) slot-buffer row
    // (filing order 0 is this thread's own position i)
    const uint32_t* row = abuf + (size_t)s * kAddSlots;
    uint32_t last = 0;
    for (uint32_t j = 0; j < m; ++j) {
      uint32_t next = 0xffffffffu;
      for (uint32_t k = 0; k < m; ++k) {
        uint32_t v = k == 0 ? i : row[k];
        if ((j == 0 || v > last) && v < next) next = v;
      }
      step(next);
      last = next;
    }
  } else {
    for (uint32_t j = 0; j < p.n; ++j)
      if (aslot[j] == s) step(j);
  }
  if (act.cold && !idle0 && count0 == 0) {
    if (chg_last != 0xffffffffu)
      act.cnew[chg_last] = okey(__dadd_rn(cur_p, pd));
    else  // unchanged by the batch
      atomicMin((unsigned long long*)act.extra,
                (unsigned long long)okey(__dadd_rn(prev_p0, pd)));
  }
  tb.rec[s].prev_r = st.prev.r;
  tb.rec[s].prev_p = st.prev.p;
  tb.rec[s].prev_l = st.prev.l;
  tb.rec[s].prev_arr = st.prev.arrival;
  if (st.fetched) {
    tb.rec[s].r_inv = st.rinv;
    tb.rec[s].w_inv = st.winv;
    tb.rec[s].l_inv = st.linv;
  }
  store_cursor();
  if (st.cd_set && st.tick_set) {
    tb.aux[s] = ClientAux{st.cd, st.cr, st.last_tick};
  } else if (st.cd_set) {
    tb.aux[s].cur_delta = st.cd;
    tb.aux[s].cur_rho = st.cr;
  } else if (st.tick_set) {
    tb.aux[s].last_tick = st.last_tick;
  }
  if (st.front_set) {
    // the new front's heap keys (pk with the prop_delta it has now; an
    // activation later in the batch rewrites it, k_act_resolve)
    tb.sc[s].r = st.front.r;
    tb.sc[s].pk = __dadd_rn(st.front.p, pd);
    tb.sc[s].l = st.front.l;
  }
  *out = st;
}

}  // namespace dmc
