// SPDX-License-Identifier: LGPL-2.1
//
// dmc_oracle_capi.cc -- TEST INFRASTRUCTURE ONLY.
// C-ABI over the CPU restatement in dmc_oracle.hpp, loaded with ctypes by
// tests/ and by bench.py's cpu_baseline leg.  Mirrors include/dmclock_gpu.h so
// that the same driver can run a trace through both engines.
#include <chrono>
#include <cstring>
#include <deque>
#include <map>
#include <memory>

#include "../include/dmclock_gpu.h"
#include "dmc_oracle.hpp"

using namespace dmc_oracle;

namespace {

// client_info_f model: each client maps to a ClientInfo object; set_info with
// fresh=0 mutates that object in place (the cached pointer sees it, as when a
// reference test assigns to the ClientInfo its lambda returns), fresh=1 points
// the client at a new object (visible after update_client_info or with U1).
struct InfoTable {
  std::deque<ClientInfo> objects;
  std::map<uint32_t, ClientInfo*> current;
  const ClientInfo* get(uint32_t c) const {
    auto it = current.find(c);
    return it == current.end() ? nullptr : it->second;
  }
  void set(uint32_t c, double r, double w, double l, bool fresh) {
    auto it = current.find(c);
    if (it == current.end() || fresh) {
      objects.emplace_back(r, w, l);
      current[c] = &objects.back();
    } else {
      it->second->set(r, w, l);
    }
  }
};

struct OQueue {
  InfoTable infos;
  std::unique_ptr<Queue> q;
  uint64_t ties = 0;
};

void fill_decision(const Queue::PullResult& r, dmc_decision* d) {
  d->handle = r.handle;
  d->tag_r = r.tag.reservation;
  d->tag_p = r.tag.proportion;
  d->tag_l = r.tag.limit;
  d->slot = r.client;
  d->cost = r.cost;
  d->phase = uint32_t(r.phase);
  d->flags = r.tie ? 1u : 0u;
}

}  // namespace

extern "C" {

void* dmo_queue_create(int delayed, int dynamic_info, unsigned branching,
                       int at_limit, double reject_threshold,
                       double anticipation) {
  auto* o = new OQueue;
  InfoTable* tbl = &o->infos;
  o->q.reset(new Queue([tbl](uint32_t c) { return tbl->get(c); },
                       delayed != 0, dynamic_info != 0, branching,
                       AtLimit(at_limit), reject_threshold, anticipation));
  return o;
}

void dmo_queue_destroy(void* h) { delete static_cast<OQueue*>(h); }

void dmo_set_track_ties(void* h, int on) {
  static_cast<OQueue*>(h)->q->track_ties = on != 0;
}

void dmo_info_set(void* h, uint32_t client, double r, double w, double l,
                  int fresh) {
  static_cast<OQueue*>(h)->infos.set(client, r, w, l, fresh != 0);
}

int dmo_register_active(void* h, uint32_t client) {
  return static_cast<OQueue*>(h)->q->register_active(client);
}

int dmo_register_active_batch(void* h, uint32_t n, const uint32_t* clients,
                              const double* r, const double* w,
                              const double* l) {
  auto* o = static_cast<OQueue*>(h);
  for (uint32_t i = 0; i < n; ++i) {
    o->infos.set(clients[i], r[i], w[i], l[i], true);
    int rc = o->q->register_active(clients[i]);
    if (rc) return rc;
  }
  return 0;
}

int dmo_add(void* h, uint64_t handle, uint32_t client, uint32_t delta,
            uint32_t rho, double time, uint32_t cost) {
  return static_cast<OQueue*>(h)->q->add_request(handle, client, delta, rho,
                                                 time, cost);
}

int dmo_add_batch(void* h, uint32_t n, const dmc_request* reqs,
                  int32_t* rc_out) {
  auto* o = static_cast<OQueue*>(h);
  for (uint32_t i = 0; i < n; ++i) {
    const dmc_request& r = reqs[i];
    int rc = o->q->add_request(r.handle, r.slot, r.delta, r.rho, r.time,
                               r.cost);
    if (rc_out) rc_out[i] = rc;
  }
  return 0;
}

// one pull_request(now); returns the NextReqType
int dmo_pull(void* h, double now, dmc_decision* out, double* when) {
  auto* o = static_cast<OQueue*>(h);
  Queue::PullResult r = o->q->pull(now);
  if (r.type == Queue::NextType::returning) {
    if (out) fill_decision(r, out);
    if (r.tie) ++o->ties;
  }
  if (when) *when = r.when;
  return int(r.type);
}

int dmo_pull_batch(void* h, double now, uint32_t k, dmc_decision* out,
                   dmc_pull_result* res) {
  auto* o = static_cast<OQueue*>(h);
  dmc_pull_result pr{};
  pr.next_type = DMC_NEXT_RETURNING;
  for (uint32_t i = 0; i < k; ++i) {
    Queue::PullResult r = o->q->pull(now);
    if (r.type != Queue::NextType::returning) {
      pr.next_type = r.type == Queue::NextType::future ? DMC_NEXT_FUTURE
                                                       : DMC_NEXT_NONE;
      pr.when = r.when;
      break;
    }
    if (r.tie) ++o->ties;
    if (out) fill_decision(r, &out[pr.n_decisions]);
    if (r.phase == Phase::reservation)
      ++pr.n_reservation;
    else
      ++pr.n_priority;
    ++pr.n_decisions;
  }
  if (res) *res = pr;
  return 0;
}

uint64_t dmo_ties(void* h) { return static_cast<OQueue*>(h)->ties; }

// Tie study (tools/tie_rules.py): log every tied decision's tied set.
void dmo_tie_log_enable(void* h, int on) { static_cast<OQueue*>(h)->q->log_ties = on != 0; }

// The log since the last read, flattened into 64-bit words: per tie [heap,
// chosen slot, m] then m members [slot, arrival bits, front_since,
// last_tick]; returns the words needed (reads and clears only if cap
// suffices).
uint64_t dmo_tie_log_read(void* h, uint64_t* out, uint64_t cap) {
  auto& log = static_cast<OQueue*>(h)->q->tie_log;
  uint64_t need = 0;
  for (auto& t : log) need += 3 + 4 * t.members.size();
  if (!out || cap < need) return need;
  uint64_t o = 0;
  for (auto& t : log) {
    out[o++] = uint64_t(t.heap);
    out[o++] = t.chosen;
    out[o++] = t.members.size();
    for (auto& m : t.members) {
      uint64_t a;
      std::memcpy(&a, &m.arrival, 8);
      out[o++] = m.slot;
      out[o++] = a;
      out[o++] = m.front_since;
      out[o++] = m.last_tick;
    }
  }
  log.clear();
  return need;
}

uint64_t dmo_request_count(void* h) {
  return static_cast<OQueue*>(h)->q->request_count();
}
uint64_t dmo_client_count(void* h) {
  return static_cast<OQueue*>(h)->q->client_count();
}
int dmo_empty(void* h) { return static_cast<OQueue*>(h)->q->empty() ? 1 : 0; }
uint64_t dmo_tick(void* h) { return static_cast<OQueue*>(h)->q->tick(); }
void dmo_sched_counts(void* h, uint64_t* resv, uint64_t* prop) {
  auto* q = static_cast<OQueue*>(h)->q.get();
  *resv = q->reserv_sched_count;
  *prop = q->prop_sched_count;
}

uint32_t dmo_remove_by_client(void* h, uint32_t client, int reverse,
                              uint64_t* out, uint32_t cap) {
  uint32_t n = 0;
  static_cast<OQueue*>(h)->q->remove_by_client(
      client, reverse != 0, [&](uint64_t hd) {
        if (n < cap && out) out[n] = hd;
        ++n;
      });
  return n;
}

typedef int (*dmo_filter_fn)(uint64_t handle, void* ctx);
int dmo_remove_by_req_filter(void* h, dmo_filter_fn fn, void* ctx,
                             int backwards) {
  return static_cast<OQueue*>(h)->q->remove_by_req_filter(
             [&](uint64_t hd) { return fn(hd, ctx) != 0; }, backwards != 0)
             ? 1
             : 0;
}

void dmo_update_client_info(void* h, uint32_t client) {
  static_cast<OQueue*>(h)->q->update_client_info(client);
}
void dmo_update_client_infos(void* h) {
  static_cast<OQueue*>(h)->q->update_client_infos();
}
uint64_t dmo_clean(void* h, uint64_t erase_point, uint64_t idle_point,
                   uint64_t erase_max) {
  return static_cast<OQueue*>(h)->q->clean(erase_point, idle_point, erase_max);
}
void dmo_mark_idle(void* h, uint32_t client) {
  static_cast<OQueue*>(h)->q->mark_idle(client);
}
int dmo_erase(void* h, uint32_t client) {
  return static_cast<OQueue*>(h)->q->erase_client(client) ? 1 : 0;
}

int dmo_client_state(void* h, uint32_t client, dmc_client_state* s) {
  auto* q = static_cast<OQueue*>(h)->q.get();
  std::memset(s, 0, sizeof(*s));
  Queue::ClientRec* c = q->find(client);
  if (!c) return DMC_ENOTREG;
  s->prev_r = c->prev.reservation;
  s->prev_p = c->prev.proportion;
  s->prev_l = c->prev.limit;
  s->prev_arrival = c->prev.arrival;
  s->prop_delta = c->prop_delta;
  if (c->has_request()) {
    const Tag& f = c->front();
    s->front_r = f.reservation;
    s->front_p = f.proportion;
    s->front_l = f.limit;
    s->front_arrival = f.arrival;
    s->front_ready = f.ready ? 1 : 0;
  }
  if (c->info) {
    s->r_inv = c->info->reservation_inv;
    s->w_inv = c->info->weight_inv;
    s->l_inv = c->info->limit_inv;
  }
  s->last_tick = c->last_tick;
  s->count = uint32_t(c->requests.size());
  s->cur_delta = c->cur_delta;
  s->cur_rho = c->cur_rho;
  s->idle = c->idle ? 1 : 0;
  s->registered = 1;
  return 0;
}

// all queued tags of one client (r, p, l per request, FIFO order)
uint32_t dmo_client_tags(void* h, uint32_t client, double* out, uint32_t cap) {
  auto* q = static_cast<OQueue*>(h)->q.get();
  Queue::ClientRec* c = q->find(client);
  if (!c) return 0;
  uint32_t n = 0;
  for (auto& r : c->requests) {
    if (n < cap) {
      out[3 * n + 0] = r.tag.reservation;
      out[3 * n + 1] = r.tag.proportion;
      out[3 * n + 2] = r.tag.limit;
    }
    ++n;
  }
  return n;
}

// ---------------------------------------------------------------- int heap
// Exposes IndHeap over ints for the reference's heap KATs
// (support/test/test_indirect_intrusive_heap.cc).  mode 0: ascending
// (ElemCompare :52-57); mode 1: evens first high-to-low then odds high-to-low
// (ElemCompareAlt :61-75).
struct IElem {
  int data;
  size_t idx = 0;
  size_t idx_alt = 0;
};
struct ILess {
  int mode;
  bool operator()(const IElem& a, const IElem& b) const {
    if (mode == 0) return a.data < b.data;
    bool ae = (a.data % 2) == 0, be = (b.data % 2) == 0;
    if (ae) return be ? a.data > b.data : true;
    if (be) return false;
    return a.data > b.data;
  }
};
static size_t& ielem_idx(IElem& e) { return e.idx; }
static size_t& ielem_idx_alt(IElem& e) { return e.idx_alt; }
struct IHeap {
  std::deque<std::shared_ptr<IElem>> elems;  // element ids index this
  std::unique_ptr<IndHeap<std::shared_ptr<IElem>, IElem, ILess>> h;
};

void* dmo_iheap_create(unsigned k, int mode, int alt_index) {
  auto* ih = new IHeap;
  ih->h.reset(new IndHeap<std::shared_ptr<IElem>, IElem, ILess>(
      k, alt_index ? &ielem_idx_alt : &ielem_idx, ILess{mode}));
  return ih;
}
void dmo_iheap_destroy(void* h) { delete static_cast<IHeap*>(h); }
// new element (not yet in any heap); returns its id
int dmo_ielem_new(void* h, int value) {
  auto* ih = static_cast<IHeap*>(h);
  ih->elems.push_back(std::make_shared<IElem>(IElem{value}));
  return int(ih->elems.size() - 1);
}
// push an element created in (possibly another) heap object `src`
void dmo_iheap_push(void* h, void* src, int id) {
  auto* ih = static_cast<IHeap*>(h);
  auto* s = static_cast<IHeap*>(src);
  ih->h->push(s->elems[id]);
}
void dmo_ielem_set(void* src, int id, int value) {
  static_cast<IHeap*>(src)->elems[id]->data = value;
}
int dmo_iheap_top(void* h) { return static_cast<IHeap*>(h)->h->top().data; }
int dmo_iheap_size(void* h) { return int(static_cast<IHeap*>(h)->h->size()); }
void dmo_iheap_pop(void* h) { static_cast<IHeap*>(h)->h->pop(); }
void dmo_iheap_promote(void* h, void* src, int id) {
  static_cast<IHeap*>(h)->h->promote(*static_cast<IHeap*>(src)->elems[id]);
}
void dmo_iheap_demote(void* h, void* src, int id) {
  static_cast<IHeap*>(h)->h->demote(*static_cast<IHeap*>(src)->elems[id]);
}
void dmo_iheap_adjust(void* h, void* src, int id) {
  static_cast<IHeap*>(h)->h->adjust(*static_cast<IHeap*>(src)->elems[id]);
}
// find by value (first in array order, as IndIntruHeap::find(const T&)) and
// remove; returns 1 if found
int dmo_iheap_remove_value(void* h, int value) {
  auto* ih = static_cast<IHeap*>(h);
  auto& raw = ih->h->raw();
  for (size_t i = 0; i < raw.size(); ++i)
    if (raw[i]->data == value) {
      ih->h->remove_at(i);
      return 1;
    }
  return 0;
}
// array order (what the reference's iterator walks)
int dmo_iheap_dump(void* h, int* out, int cap) {
  auto& raw = static_cast<IHeap*>(h)->h->raw();
  int n = int(raw.size());
  for (int i = 0; i < n && i < cap; ++i) out[i] = raw[i]->data;
  return n;
}

// ---------------------------------------------------------------- trackers
struct TrackerBox {
  int kind;
  ServiceTracker<OrigTracker> orig;
  ServiceTracker<BorrowingTracker> borrow;
};
void* dmo_tracker_create(int kind) { return new TrackerBox{kind, {}, {}}; }
void dmo_tracker_destroy(void* h) { delete static_cast<TrackerBox*>(h); }
void dmo_tracker_track_resp(void* h, uint32_t server, int phase,
                            uint64_t cost) {
  auto* t = static_cast<TrackerBox*>(h);
  if (t->kind == 0)
    t->orig.track_resp(server, Phase(phase), cost);
  else
    t->borrow.track_resp(server, Phase(phase), cost);
}
void dmo_tracker_get_req_params(void* h, uint32_t server, uint32_t* d,
                                uint32_t* r) {
  auto* t = static_cast<TrackerBox*>(h);
  if (t->kind == 0)
    t->orig.get_req_params(server, d, r);
  else
    t->borrow.get_req_params(server, d, r);
}

// ---------------------------------------------------------------- timing
// Wall time of a pull+add replay for the CPU baseline (bench.py).
double dmo_now_seconds() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

}  // extern "C"
