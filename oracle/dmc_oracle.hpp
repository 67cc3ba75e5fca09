// SPDX-License-Identifier: LGPL-2.1
//
// dmc_oracle.hpp -- TEST INFRASTRUCTURE ONLY.
//
// A from-scratch CPU restatement of the dmClock server queue of the reference
// (zte-opensource/dmclock, /root/reference/src/dmclock_server.h and
// /root/reference/support/src/indirect_intrusive_heap.h), used as the parity
// checker for the HIP engine in dmclock_amd/csrc.  Only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
//
// Parity pinning: the reference itself is UNBUILDABLE in this image (its
// server header includes <boost/variant.hpp> and its tests need GTest; neither
// is installed, and stand-ins are not allowed).  This restatement is pinned
// instead by every known-answer test the reference's own suites hold for the
// path (test/test_dmclock_server.cc, test/test_dmclock_client.cc,
// support/test/test_indirect_intrusive_heap.cc), restated with explicit times
// in tests/test_oracle_kats.py.
//
// It deliberately mirrors the reference's data structures (std::map of
// shared_ptr client records, per-client std::deque, three indirect binary
// heaps) so that its timing is a faithful single-core CPU baseline and its
// tie-breaking (heap sift history) is the reference's.
//
// Build: g++ -O2 -std=c++17 -ffp-contract=off (never -march=native: FMA
// contraction would change tag bits; reference note dmclock_server.h:256).
#pragma once

#include <cassert>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <deque>
#include <functional>
#include <limits>
#include <map>
#include <memory>
#include <vector>

namespace dmc_oracle {

using Time = double;
using Cost = uint32_t;
using Counter = uint64_t;

constexpr double kMaxTag = std::numeric_limits<double>::infinity();   // :60-62
constexpr double kMinTag = -std::numeric_limits<double>::infinity();  // :63-65
constexpr Time kTimeZero = 0.0;                                       // dmclock_util.h:34
constexpr Time kTimeMax = std::numeric_limits<double>::max();         // dmclock_util.h:35

enum class Phase : uint8_t { reservation = 0, priority = 1 };  // dmclock_recs.h:33
enum class AtLimit : int { Wait = 0, Allow = 1, Reject = 2 };  // dmclock_server.h:74-84

// status codes (the reference aborts via assert where we return a code)
enum : int {
  kOk = 0,
  kErrBadTag = -1001,   // cost==0, or reservation and proportion both +inf (:158,:182)
  kErrBadParams = -1002,// rho > delta (dmclock_recs.h:51)
  kErrNoInfo = -1003,   // client_info_f returned null (:885,:900)
};

// ---------------------------------------------------------------- ClientInfo
// dmclock_server.h:95-118: x_inv = (x == 0) ? 0 : 1/x
struct ClientInfo {
  double reservation = 0, weight = 0, limit = 0;
  double reservation_inv = 0, weight_inv = 0, limit_inv = 0;
  ClientInfo() = default;
  ClientInfo(double r, double w, double l) { set(r, w, l); }
  void set(double r, double w, double l) {
    reservation = r;
    weight = w;
    limit = l;
    reservation_inv = (r == 0.0) ? 0.0 : 1.0 / r;
    weight_inv = (w == 0.0) ? 0.0 : 1.0 / w;
    limit_inv = (l == 0.0) ? 0.0 : 1.0 / l;
  }
};

// ---------------------------------------------------------------- RequestTag
struct Tag {
  double reservation = 0, proportion = 0, limit = 0;
  uint32_t delta = 0, rho = 0;
  Cost cost = 1;
  bool ready = false;
  Time arrival = 0;
};

// dmclock_server.h:246-259.  inc * (uint64(dist) + cost) is a u64 add then a
// single rounding to double, then one multiply and one add (no FMA), then
// std::max(time, x) -- which returns `time` when the two compare equal.
inline double tag_step(Time time, double prev, double inc, uint32_t dist,
                       bool extreme_is_high, Cost cost) {
  if (inc == 0.0) return extreme_is_high ? kMaxTag : kMinTag;
  double step = inc * double(uint64_t(dist) + uint64_t(cost));
  double cand = prev + step;
  return (time < cand) ? cand : time;
}

// dmclock_server.h:145-183.  Returns false where the reference asserts.
inline bool make_tag(const Tag& prev, const ClientInfo& info, uint32_t delta,
                     uint32_t rho, Time time, Cost cost, double antic,
                     Tag* out) {
  Tag t;
  t.delta = delta;
  t.rho = rho;
  t.cost = cost;
  t.ready = false;
  t.arrival = time;
  if (cost == 0) return false;
  Time max_time = time;
  if (time - antic < prev.arrival) max_time -= antic;
  t.reservation = tag_step(max_time, prev.reservation, info.reservation_inv,
                           rho, true, cost);
  t.proportion = tag_step(max_time, prev.proportion, info.weight_inv, delta,
                          true, cost);
  t.limit = tag_step(max_time, prev.limit, info.limit_inv, delta, false, cost);
  if (!(t.reservation < kMaxTag || t.proportion < kMaxTag)) return false;
  *out = t;
  return true;
}

// ---------------------------------------------------------------- IndHeap
// Indirect intrusive K-ary min-heap, indirect_intrusive_heap.h:47-565.
// Each element records its own index through `idx_of`.  Semantics that matter
// for parity: sift_up moves only on strict `less`; K==2 sift_down prefers the
// left child unless the right is strictly smaller; remove() swaps in the last
// element and calls sift (not sift_down).
template <typename P, typename T, typename Less>
class IndHeap {
 public:
  using IndexFn = size_t& (*)(T&);
  IndHeap(unsigned k, IndexFn idx_of, Less less = Less())
      : k_(k), idx_of_(idx_of), less_(less) {
    assert(k_ >= 2);
  }
  bool empty() const { return data_.empty(); }
  size_t size() const { return data_.size(); }
  T& top() { return *data_[0]; }
  const T& top() const { return *data_[0]; }
  P& top_ind() { return data_[0]; }
  T& at(size_t i) { return *data_[i]; }
  const T& at(size_t i) const { return *data_[i]; }
  const std::vector<P>& raw() const { return data_; }

  void push(P item) {  // :240-245
    size_t i = data_.size();
    idx_of_(*item) = i;
    data_.push_back(std::move(item));
    sift_up(i);
  }
  void pop() { remove_at(0); }  // :252-254
  void remove_at(size_t i) {    // :433-445
    size_t last = data_.size() - 1;
    std::swap(data_[i], data_[last]);
    idx_of_(*data_[i]) = i;
    // note: the reference sifts BEFORE popping the moved-out element, so
    // `count` already excludes it while the vector still holds it.
    count_override_ = last;
    sift(i);
    count_override_ = SIZE_MAX;
    data_.pop_back();
  }
  void promote(T& item) { sift_up(idx_of_(item)); }    // :357-359
  void demote(T& item) { sift_down(idx_of_(item)); }   // :361-363
  void adjust(T& item) { sift(idx_of_(item)); }        // :365-367
  bool less(const T& a, const T& b) const { return less_(a, b); }
  unsigned branching() const { return k_; }

 private:
  size_t count() const {
    return count_override_ == SIZE_MAX ? data_.size() : count_override_;
  }
  size_t parent(size_t i) const { return (i - 1) / k_; }
  void swap_idx(size_t a, size_t b) {
    std::swap(data_[a], data_[b]);
    idx_of_(*data_[a]) = a;
    idx_of_(*data_[b]) = b;
  }
  void sift_up(size_t i) {  // :462-474
    while (i > 0) {
      size_t pi = parent(i);
      if (!less_(*data_[i], *data_[pi])) break;
      swap_idx(i, pi);
      i = pi;
    }
  }
  void sift_down(size_t i) {
    size_t n = count();
    if (i >= n) return;
    if (k_ == 2) {  // :514-548
      for (;;) {
        size_t li = 2 * i + 1, ri = li + 1;
        if (li >= n) break;
        if (less_(*data_[li], *data_[i])) {
          if (ri < n && less_(*data_[ri], *data_[li])) {
            swap_idx(i, ri);
            i = ri;
          } else {
            swap_idx(i, li);
            i = li;
          }
        } else if (ri < n && less_(*data_[ri], *data_[i])) {
          swap_idx(i, ri);
          i = ri;
        } else {
          break;
        }
      }
    } else {  // :479-510
      for (;;) {
        size_t li = k_ * i + 1;
        if (li >= n) break;
        size_t ri = std::min<size_t>(k_ * i + k_, n - 1);
        size_t mi = li;
        for (size_t c = li + 1; c <= ri; ++c)
          if (less_(*data_[c], *data_[mi])) mi = c;
        if (less_(*data_[mi], *data_[i])) {
          swap_idx(i, mi);
          i = mi;
        } else {
          break;
        }
      }
    }
  }
  void sift(size_t i) {  // :550-564
    if (i == 0) {
      sift_down(i);
    } else if (less_(*data_[i], *data_[parent(i)])) {
      sift_up(i);
    } else {
      sift_down(i);
    }
  }

  unsigned k_;
  IndexFn idx_of_;
  Less less_;
  std::vector<P> data_;
  size_t count_override_ = SIZE_MAX;
};

// ---------------------------------------------------------------- Queue
// The reference's PriorityQueueBase + PullPriorityQueue (dmclock_server.h
// :283-1501) with C = uint32_t client id and R = uint64_t request handle.
// `info_of(client)` plays client_info_f; it returns a pointer the queue
// caches (static mode) or re-reads on every tag (U1 / dynamic mode).
class Queue {
 public:
  using InfoFn = std::function<const ClientInfo*(uint32_t)>;

  struct Req {
    Tag tag;
    uint32_t client;
    uint64_t handle;
  };

  struct ClientRec {
    uint32_t client;
    Tag prev;  // prev_tag(0,0,0,TimeZero) :385
    std::deque<Req> requests;
    double prop_delta = 0.0;
    size_t resv_idx = 0, lim_idx = 0, ready_idx = 0;
    const ClientInfo* info = nullptr;
    bool idle = true;
    Counter last_tick = 0;
    uint32_t cur_rho = 1, cur_delta = 1;
    // tie study only (tools/tie_rules.py): when the current front became the
    // front (a running count of front changes)
    uint64_t front_since = 0;
    bool has_request() const { return !requests.empty(); }
    const Tag& front() const { return requests.front().tag; }
  };
  using RecRef = std::shared_ptr<ClientRec>;

  // ClientCompare, :722-757
  enum class ReadyOpt { ignore, lowers, raises };
  template <int Field, ReadyOpt RO, bool UsePD>
  struct Cmp {
    static double field(const Tag& t) {
      return Field == 0 ? t.reservation : (Field == 1 ? t.proportion : t.limit);
    }
    bool operator()(const ClientRec& a, const ClientRec& b) const {
      if (a.has_request()) {
        if (b.has_request()) {
          const Tag& ta = a.front();
          const Tag& tb = b.front();
          if (RO == ReadyOpt::ignore || ta.ready == tb.ready) {
            if (UsePD)
              return (field(ta) + a.prop_delta) < (field(tb) + b.prop_delta);
            return field(ta) < field(tb);
          } else if (RO == ReadyOpt::raises) {
            return ta.ready;
          } else {
            return tb.ready;
          }
        }
        return true;
      }
      return false;
    }
  };
  using ResvCmp = Cmp<0, ReadyOpt::ignore, false>;
  using LimCmp = Cmp<2, ReadyOpt::lowers, false>;
  using ReadyCmp = Cmp<1, ReadyOpt::raises, true>;

  static size_t& resv_idx_of(ClientRec& c) { return c.resv_idx; }
  static size_t& lim_idx_of(ClientRec& c) { return c.lim_idx; }
  static size_t& ready_idx_of(ClientRec& c) { return c.ready_idx; }

  enum class NextType { returning = 0, future = 1, none = 2 };

  struct PullResult {
    NextType type = NextType::none;
    uint32_t client = 0;
    uint64_t handle = 0;
    Phase phase = Phase::reservation;
    Cost cost = 0;
    Time when = 0;
    Tag tag;      // the popped tag (before reduction), for tag-level parity
    bool tie = false;  // another client compared equal to the heap top
  };

  // Tie study (test infrastructure, tools/tie_rules.py): with log_ties, every
  // tied decision records the heap it came from, the client dispatched and
  // every client tied with it (slot, front arrival, front_since, last_tick).
  struct TieMember {
    uint32_t slot;
    double arrival;
    uint64_t front_since, last_tick;
  };
  struct TieRec {
    int heap;  // 0 reservation, 1 ready
    uint32_t chosen;
    std::vector<TieMember> members;
  };
  bool log_ties = false;
  std::vector<TieRec> tie_log;

  Queue(InfoFn info_of, bool delayed, bool dynamic_info, unsigned branching,
        AtLimit at_limit, double reject_threshold, double anticipation)
      : info_of_(std::move(info_of)),
        delayed_(delayed),
        dynamic_(dynamic_info),
        at_limit_(at_limit),
        reject_threshold_(reject_threshold),
        antic_(anticipation),
        resv_(branching, &resv_idx_of),
        limit_(branching, &lim_idx_of),
        ready_(branching, &ready_idx_of) {}

  bool track_ties = true;

  // ---- the idle reset's minimum (:937-985), exactly, in O(log N)
  // The reference scans every client for the lowest (front or prev)
  // proportion + prop_delta of the non-idle ones: an O(N) pass per
  // activation, which makes a 1M-client churn trace take hours here.  ActMin
  // keeps the same minimum in a segment tree over client ids (the
  // client_map_ order): a leaf holds a client's value iff it is non-idle and
  // not NaN (the scan's `p < lowest` never takes NaN); a node keeps its left
  // child unless the right one is strictly smaller -- the first client in map
  // order among the minimal ones, which is exactly the value the scan ends
  // with (strict `<` keeps the first of values that compare equal, +0.0 and
  // -0.0 included).  Every mutation of a client's requests, prev tag,
  // prop_delta or idle flag refreshes its leaf (am_touch).  Client ids above
  // kActMinMaxId fall back to the scan.  DMO_ACTMIN_CHECK=1 (tests) runs both
  // and aborts on any difference.
  static constexpr uint32_t kActMinMaxId = 1u << 24;
  struct ActMin {
    uint32_t cap = 0;              // leaves (a power of two)
    std::vector<double> val;       // 2 cap nodes
    std::vector<uint8_t> ok;       // a value is present
    bool disabled = false;         // an id >= kActMinMaxId was seen
    void grow(uint32_t id) {
      uint32_t nc = cap ? cap : 1024;
      while (nc <= id) nc <<= 1;
      std::vector<double> v2(2 * (size_t)nc, 0.0);
      std::vector<uint8_t> o2(2 * (size_t)nc, 0);
      for (uint32_t i = 0; i < cap; ++i) {
        v2[nc + i] = val[cap + i];
        o2[nc + i] = ok[cap + i];
      }
      cap = nc;
      val.swap(v2);
      ok.swap(o2);
      for (uint32_t n = cap; n-- > 1;) pull(n);
    }
    void pull(uint32_t n) {
      const uint32_t a = 2 * n, b = a + 1;
      if (ok[a] && (!ok[b] || !(val[b] < val[a]))) {
        val[n] = val[a];
        ok[n] = 1;
      } else {
        val[n] = val[b];
        ok[n] = ok[b];
      }
    }
    void set(uint32_t id, bool present, double v) {
      if (disabled) return;
      if (id >= kActMinMaxId) {
        disabled = true;
        return;
      }
      if (id >= cap) {
        if (!present) return;
        grow(id);
      }
      uint32_t n = cap + id;
      val[n] = v;
      ok[n] = present ? 1 : 0;
      for (n >>= 1; n >= 1; n >>= 1) pull(n);
    }
    bool min(double* out) const {  // false: no value present
      if (!cap || !ok[1]) return false;
      *out = val[1];
      return true;
    }
  };
  ActMin am_;
  bool am_check_ = getenv("DMO_ACTMIN_CHECK") && atoi(getenv("DMO_ACTMIN_CHECK"));

  void am_touch(const ClientRec& c) {
    const double p = c.has_request() ? c.front().proportion + c.prop_delta
                                     : c.prev.proportion + c.prop_delta;
    am_.set(c.client, !c.idle && p == p, p);
  }
  void am_forget(uint32_t client) { am_.set(client, false, 0.0); }
  // the reference's lowest: DBL_MAX, or the smallest value below it
  double am_lowest() {
    double lowest = std::numeric_limits<double>::max();
    double m;
    const bool tree = !am_.disabled;
    if (tree && am_.min(&m) && m < lowest) lowest = m;
    if (!tree || am_check_) {
      double l2 = std::numeric_limits<double>::max();
      for (auto const& kv : client_map_) {
        const ClientRec& o = *kv.second;
        if (o.idle) continue;
        double p = o.has_request() ? o.front().proportion + o.prop_delta
                                   : o.prev.proportion + o.prop_delta;
        if (p < l2) l2 = p;
      }
      if (tree && std::memcmp(&l2, &lowest, sizeof l2) != 0) {
        std::fprintf(stderr, "dmc_oracle: ActMin %.17g != scan %.17g\n", lowest, l2);
        std::abort();
      }
      lowest = l2;
    }
    return lowest;
  }
  // refreshes a client's leaf when it goes out of scope (every return path
  // of a mutating call)
  struct AmTouch {
    Queue* q;
    const ClientRec* c;
    ~AmTouch() { q->am_touch(*c); }
  };

  // ---- public API mirrors
  size_t client_count() const { return resv_.size(); }  // :551-554
  size_t request_count() const {                         // :557-564
    size_t n = 0;
    for (auto& p : client_map_) n += p.second->requests.size();
    return n;
  }
  bool empty() const {  // :545-548
    return resv_.empty() || !resv_.top().has_request();
  }
  Counter tick() const { return tick_; }
  size_t reserv_sched_count = 0, prop_sched_count = 0;

  ClientRec* find(uint32_t client) {
    auto it = client_map_.find(client);
    return it == client_map_.end() ? nullptr : it->second.get();
  }
  const std::map<uint32_t, RecRef>& clients() const { return client_map_; }

  // Bulk registration (a documented deviation used identically on both
  // sides for 1M-client populations): creates the client record as if it had
  // been created and activated, i.e. idle=false, prop_delta=0, no requests.
  int register_active(uint32_t client) {
    auto ins = client_map_.emplace(client, RecRef{});
    if (!ins.second) return kOk;
    const ClientInfo* info = info_of_(client);
    if (!info) {
      client_map_.erase(ins.first);
      return kErrNoInfo;
    }
    auto rec = std::make_shared<ClientRec>();
    rec->client = client;
    rec->info = info;
    rec->idle = false;
    rec->last_tick = tick_;
    resv_.push(rec);
    limit_.push(rec);
    ready_.push(rec);
    am_touch(*rec);
    ins.first->second = std::move(rec);
    return kOk;
  }

  // do_add_request, :913-1018.  Returns 0, EAGAIN, or a negative error.
  int add_request(uint64_t handle, uint32_t client_id, uint32_t delta,
                  uint32_t rho, Time time, Cost cost) {
    if (rho > delta) return kErrBadParams;
    ++tick_;
    auto ins = client_map_.emplace(client_id, RecRef{});
    if (ins.second) {
      const ClientInfo* info = info_of_(client_id);
      auto rec = std::make_shared<ClientRec>();
      rec->client = client_id;
      rec->info = info;
      rec->idle = true;
      rec->last_tick = tick_;
      resv_.push(rec);
      limit_.push(rec);
      ready_.push(rec);
      ins.first->second = std::move(rec);
    }
    ClientRec& c = *ins.first->second;
    AmTouch am_guard{this, &c};

    if (c.idle) {  // :937-985
      constexpr double trigger = std::numeric_limits<double>::max() / 3.0;
      // (the lowest over the non-idle clients: am_lowest, the scan's value)
      const double lowest = am_lowest();
      if (lowest < trigger) c.prop_delta = lowest - time;
      c.idle = false;
    }

    Tag tag;
    int rc = initial_tag(c, delta, rho, time, cost, &tag);
    if (rc != kOk) return rc;

    if (at_limit_ == AtLimit::Reject && tag.limit > time + reject_threshold_)
      return EAGAIN;  // :989-993 (prev tag already advanced)

    c.requests.push_back(Req{tag, client_id, handle});
    if (c.requests.size() == 1) {
      c.front_since = ++front_seq_;
      resv_.adjust(c);
      limit_.adjust(c);
      ready_.adjust(c);
    }
    c.cur_rho = rho;
    c.cur_delta = delta;
    resv_.adjust(c);
    limit_.adjust(c);
    ready_.adjust(c);
    return kOk;
  }

  // pull_request(now), :1425-1489 over do_next_request, :1115-1186
  PullResult pull(Time now) {
    PullResult res;
    if (resv_.empty()) return res;  // none

    ClientRec& reserv = resv_.top();
    if (reserv.has_request() && reserv.front().reservation <= now) {
      res.tie = track_ties && top_tied(resv_);
      if (res.tie) log_tie(resv_, 0);
      pop_into(resv_, Phase::reservation, &res);
      ++reserv_sched_count;
      return res;
    }

    // limit loop :1135-1144
    ClientRec* lim = &limit_.top();
    while (lim->has_request() && !lim->front().ready &&
           lim->front().limit <= now) {
      lim->requests.front().tag.ready = true;
      ready_.promote(*lim);
      limit_.demote(*lim);
      lim = &limit_.top();
    }

    ClientRec& readys = ready_.top();
    if (readys.has_request() && readys.front().ready &&
        readys.front().proportion < kMaxTag) {
      res.tie = track_ties && top_tied(ready_);
      if (res.tie) log_tie(ready_, 1);
      pop_ready_into(&res);
      return res;
    }

    if (at_limit_ == AtLimit::Allow) {  // :1157-1165
      if (readys.has_request() && readys.front().proportion < kMaxTag) {
        res.tie = track_ties && top_tied(ready_);
        pop_ready_into(&res);
        return res;
      } else if (reserv.has_request() &&
                 reserv.front().reservation < kMaxTag) {
        res.tie = track_ties && top_tied(resv_);
        pop_into(resv_, Phase::reservation, &res);
        ++reserv_sched_count;
        return res;
      }
    }

    Time next_call = kTimeMax;  // :1170-1185
    if (resv_.top().has_request())
      next_call = min_not_0(next_call, resv_.top().front().reservation);
    if (limit_.top().has_request())
      next_call = min_not_0(next_call, limit_.top().front().limit);
    if (next_call < kTimeMax) {
      res.type = NextType::future;
      res.when = next_call;
    }
    return res;
  }

  // ---- maintenance API, :567-648
  template <typename F>
  bool remove_by_req_filter(F&& filter, bool backwards) {
    bool any = false;
    for (auto& kv : client_map_) {
      ClientRec& c = *kv.second;
      bool modified = false;
      if (!backwards) {
        for (auto i = c.requests.begin(); i != c.requests.end();) {
          if (filter(i->handle)) {
            modified = true;
            i = c.requests.erase(i);
          } else {
            ++i;
          }
        }
      } else {
        for (size_t j = c.requests.size(); j-- > 0;) {
          if (filter(c.requests[j].handle)) {
            modified = true;
            c.requests.erase(c.requests.begin() + j);
          }
        }
      }
      if (modified) {
        resv_.adjust(c);
        limit_.adjust(c);
        ready_.adjust(c);
        am_touch(c);
        any = true;
      }
    }
    return any;
  }

  template <typename F>
  void remove_by_client(uint32_t client, bool reverse, F&& accum) {
    auto it = client_map_.find(client);
    if (it == client_map_.end()) return;
    ClientRec& c = *it->second;
    if (reverse) {
      for (auto j = c.requests.rbegin(); j != c.requests.rend(); ++j)
        accum(j->handle);
    } else {
      for (auto& r : c.requests) accum(r.handle);
    }
    c.requests.clear();
    resv_.adjust(c);
    limit_.adjust(c);
    ready_.adjust(c);
    am_touch(c);
  }

  void update_client_info(uint32_t client) {  // :633-640
    auto it = client_map_.find(client);
    if (it != client_map_.end()) it->second->info = info_of_(client);
  }
  void update_client_infos() {  // :643-648
    for (auto& kv : client_map_) kv.second->info = info_of_(kv.first);
  }

  // do_clean core, :1232-1244: with explicit erase/idle points (ticks).
  // Returns the number erased.
  Counter clean(Counter erase_point, Counter idle_point, Counter erase_max) {
    Counter erased = 0;
    if (erase_point > 0 || idle_point > 0) {
      for (auto i = client_map_.begin(); i != client_map_.end();) {
        auto i2 = i++;
        if (erase_point && erased < erase_max &&
            i2->second->last_tick <= erase_point) {
          delete_from_heaps(*i2->second);
          am_forget(i2->first);
          client_map_.erase(i2);
          ++erased;
        } else if (idle_point && i2->second->last_tick <= idle_point) {
          i2->second->idle = true;
          am_touch(*i2->second);
        }
      }
    }
    return erased;
  }
  void mark_idle(uint32_t client) {
    auto it = client_map_.find(client);
    if (it != client_map_.end()) {
      it->second->idle = true;
      am_touch(*it->second);
    }
  }
  bool erase_client(uint32_t client) {
    auto it = client_map_.find(client);
    if (it == client_map_.end()) return false;
    delete_from_heaps(*it->second);
    am_forget(it->first);
    client_map_.erase(it);
    return true;
  }

 private:
  static Time min_not_0(Time cur, Time possible) {  // :1192-1195
    return possible == kTimeZero ? cur : std::min(cur, possible);
  }

  const ClientInfo* cli_info(ClientRec& c) {  // :870-875
    if (dynamic_) c.info = info_of_(c.client);
    return c.info;
  }

  // initial_tag, :878-907
  int initial_tag(ClientRec& c, uint32_t delta, uint32_t rho, Time time,
                  Cost cost, Tag* out) {
    if (delayed_) {
      Tag t;
      t.reservation = 0;
      t.proportion = 0;
      t.limit = 0;
      t.arrival = time;
      t.delta = 0;
      t.rho = 0;
      t.cost = cost;
      if (cost == 0) return kErrBadTag;
      if (!c.has_request()) {
        const ClientInfo* ci = cli_info(c);
        if (!ci) return kErrNoInfo;
        if (!make_tag(c.prev, *ci, delta, rho, time, cost, antic_, &t))
          return kErrBadTag;
        update_prev(c, t);
      }
      *out = t;
      return kOk;
    }
    const ClientInfo* ci = cli_info(c);
    if (!ci) return kErrNoInfo;
    Tag t;
    if (!make_tag(c.prev, *ci, delta, rho, time, cost, antic_, &t))
      return kErrBadTag;
    update_prev(c, t);
    *out = t;
    return kOk;
  }

  // ClientRec::update_req_tag, :399-412
  void update_prev(ClientRec& c, const Tag& t) {
    auto assign = [](double& lhs, double rhs) {
      if (rhs != kMaxTag && rhs != kMinTag) lhs = rhs;
    };
    assign(c.prev.reservation, t.reservation);
    assign(c.prev.limit, t.limit);
    assign(c.prev.proportion, t.proportion);
    c.prev.arrival = t.arrival;
    c.last_tick = tick_;
  }

  // update_next_tag (Delayed), :1021-1036
  void update_next_tag(ClientRec& top, const Tag& popped) {
    if (!delayed_ || !top.has_request()) return;
    Req& nf = top.requests.front();
    const ClientInfo* ci = cli_info(top);
    Tag t;
    if (ci && make_tag(popped, *ci, top.cur_delta, top.cur_rho,
                       nf.tag.arrival, nf.tag.cost, antic_, &t)) {
      nf.tag = t;
      update_prev(top, nf.tag);
    }
  }

  // pop_process_request, :1046-1073
  template <typename H>
  Tag pop_front_of(H& heap, PullResult* res, Phase phase) {
    ClientRec& top = heap.top();
    Req req = top.requests.front();
    top.requests.pop_front();
    if (top.has_request()) top.front_since = ++front_seq_;
    update_next_tag(top, req.tag);
    resv_.demote(top);
    limit_.adjust(top);
    ready_.demote(top);
    am_touch(top);
    res->type = NextType::returning;
    res->client = top.client;
    res->handle = req.handle;
    res->phase = phase;
    res->cost = req.tag.cost;
    res->tag = req.tag;
    return req.tag;
  }

  template <typename H>
  void pop_into(H& heap, Phase phase, PullResult* res) {
    pop_front_of(heap, res, phase);
  }

  void pop_ready_into(PullResult* res) {
    Tag t = pop_front_of(ready_, res, Phase::priority);
    reduce_reservation_tags(res->client, t);
    ++prop_sched_count;
  }

  // reduce_reservation_tags, :1077-1111
  void reduce_reservation_tags(uint32_t client, const Tag& t) {
    auto it = client_map_.find(client);
    assert(it != client_map_.end());
    ClientRec& c = *it->second;
    // uint32 sum (cost + rho) then converted, :1083,:1091
    uint32_t units = uint32_t(t.cost + t.rho);
    double off = c.info->reservation_inv * double(units);
    if (delayed_) {
      if (!c.requests.empty()) c.requests.front().tag.reservation -= off;
    } else {
      for (auto& r : c.requests) r.tag.reservation -= off;
    }
    c.prev.reservation -= off;
    resv_.promote(c);
  }

  void delete_from_heaps(ClientRec& c) {  // :1259-1275
    resv_.remove_at(c.resv_idx);
    limit_.remove_at(c.lim_idx);
    ready_.remove_at(c.ready_idx);
  }

  // True iff some other element compares equal to the heap top.  Elements
  // equal to the root can only be reached through equal ancestors, so a DFS
  // over equal nodes from the root finds them all.
  // the clients with a request comparing equal to the heap top (the top
  // first), logged with the state the study's tie rules read
  template <typename H>
  void log_tie(const H& heap, int heap_id) {
    if (!log_ties) return;
    TieRec rec;
    rec.heap = heap_id;
    const ClientRec& top = heap.at(0);
    rec.chosen = top.client;
    auto add = [&](const ClientRec& e) {
      rec.members.push_back(TieMember{e.client, e.front().arrival, e.front_since,
                                      e.last_tick});
    };
    add(top);
    std::vector<size_t> stack{0};
    const size_t k = heap.branching();
    while (!stack.empty()) {
      size_t i = stack.back();
      stack.pop_back();
      for (size_t c = k * i + 1; c <= k * i + k && c < heap.size(); ++c) {
        const ClientRec& e = heap.at(c);
        if (!heap.less(top, e) && !heap.less(e, top)) {
          if (e.has_request()) add(e);
          stack.push_back(c);
        }
      }
    }
    tie_log.push_back(std::move(rec));
  }

  template <typename H>
  bool top_tied(const H& heap) const {
    const ClientRec& top = heap.at(0);
    std::vector<size_t> stack;
    stack.push_back(0);
    size_t k = heap.branching();
    while (!stack.empty()) {
      size_t i = stack.back();
      stack.pop_back();
      for (size_t c = k * i + 1; c <= k * i + k && c < heap.size(); ++c) {
        const ClientRec& e = heap.at(c);
        if (!heap.less(top, e) && !heap.less(e, top)) {
          if (e.has_request()) return true;
          stack.push_back(c);
        }
      }
    }
    return false;
  }
  InfoFn info_of_;
  bool delayed_;
  bool dynamic_;
  AtLimit at_limit_;
  double reject_threshold_;
  double antic_;
  Counter tick_ = 0;
  uint64_t front_seq_ = 0;  // tie study: front changes so far
  std::map<uint32_t, RecRef> client_map_;
  IndHeap<RecRef, ClientRec, ResvCmp> resv_;
  IndHeap<RecRef, ClientRec, LimCmp> limit_;
  IndHeap<RecRef, ClientRec, ReadyCmp> ready_;
};

// ---------------------------------------------------------------- trackers
// dmclock_client.h:39-84
struct OrigTracker {
  Counter delta_prev_req, rho_prev_req;
  uint32_t my_delta = 0, my_rho = 0;
  OrigTracker(Counter d, Counter r) : delta_prev_req(d), rho_prev_req(r) {}
  void prepare_req(Counter& the_delta, Counter& the_rho, uint32_t* od,
                   uint32_t* orho) {
    Counter dout = the_delta - delta_prev_req - my_delta;
    Counter rout = the_rho - rho_prev_req - my_rho;
    delta_prev_req = the_delta;
    rho_prev_req = the_rho;
    my_delta = 0;
    my_rho = 0;
    *od = uint32_t(dout);
    *orho = uint32_t(rout);
  }
  void resp_update(Phase phase, Counter& the_delta, Counter& the_rho,
                   Cost cost) {
    the_delta += cost;
    my_delta += cost;
    if (phase == Phase::reservation) {
      the_rho += cost;
      my_rho += cost;
    }
  }
};

// dmclock_client.h:90-154
struct BorrowingTracker {
  Counter delta_prev_req, rho_prev_req, delta_borrow = 0, rho_borrow = 0;
  BorrowingTracker(Counter d, Counter r) : delta_prev_req(d), rho_prev_req(r) {}
  static Counter with_borrow(Counter global, Counter previous,
                             Counter& borrow) {
    Counter result = global - previous;
    if (result == 0) {
      ++borrow;
      return 1;
    } else if (result > borrow) {
      result -= borrow;
      borrow = 0;
      return result;
    } else {
      borrow = borrow - result + 1;
      return 1;
    }
  }
  void prepare_req(Counter& the_delta, Counter& the_rho, uint32_t* od,
                   uint32_t* orho) {
    Counter d = with_borrow(the_delta, delta_prev_req, delta_borrow);
    Counter r = with_borrow(the_rho, rho_prev_req, rho_borrow);
    delta_prev_req = the_delta;
    rho_prev_req = the_rho;
    *od = uint32_t(d);
    *orho = uint32_t(r);
  }
  void resp_update(Phase phase, Counter& the_delta, Counter& the_rho,
                   Counter cost) {
    the_delta += cost;
    if (phase == Phase::reservation) the_rho += cost;
  }
};

// ServiceTracker, dmclock_client.h:163-251 (cleaning thread omitted)
template <typename T>
struct ServiceTracker {
  Counter delta_counter = 1, rho_counter = 1;
  std::map<uint32_t, T> server_map;
  void track_resp(uint32_t server, Phase phase, Counter cost) {
    auto it = server_map.find(server);
    if (it == server_map.end())
      it = server_map.emplace(server, T(delta_counter, rho_counter)).first;
    it->second.resp_update(phase, delta_counter, rho_counter, Cost(cost));
  }
  void get_req_params(uint32_t server, uint32_t* d, uint32_t* r) {
    auto it = server_map.find(server);
    if (it == server_map.end()) {
      server_map.emplace(server, T(delta_counter, rho_counter));
      *d = 1;
      *r = 1;
    } else {
      it->second.prepare_req(delta_counter, rho_counter, d, r);
    }
  }
};

}  // namespace dmc_oracle
