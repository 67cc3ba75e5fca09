// SPDX-License-Identifier: LGPL-2.1
//
// dmclock_server.h -- drop-in C++ facade of the reference's server queue
// (crimson::dmclock::PullPriorityQueue / PushPriorityQueue,
// /root/reference/src/dmclock_server.h) on top of the MI355X engine's C-ABI
// (include/dmclock_gpu.h).  Callers keep their code: same namespaces, class
// templates, constructors, add_request / add_request_time / pull_request /
// request_completed, PullReq{type, data variant<Retn, Time>}, and the
// maintenance API (empty, client_count, request_count, remove_by_req_filter,
// remove_by_client, update_client_info(s)).
//
// What happens behind it:
//  * client ids C map to dense device slots (std::map<C, slot>, so iteration
//    order is the reference's client_map order);
//  * requests R stay on the host, keyed by a 64-bit handle; the device sees
//    handles only;
//  * client_info_f is called at the reference's moments: at client creation,
//    on update_client_info(s), and, when U1 is set, by the engine (its
//    dmc_info_fn) right before each tag calculation: per added request and,
//    in delayed mode, for each popped client between selection and pop --
//    O(1) host work per call, no per-pull sweep over the clients;
//  * the idle/erase cleaner runs on a thread every check_time (the reference's
//    RunEvery job, :858-861 / :1206-1255), erasing in client-id order.
//
// Deviations:
//  * in-place mutation of a ClientInfo object the queue cached is seen at the
//    next add of that client or update_client_info(s) (the reference also sees
//    it at pops); under U1 at the client's next tag calculation;
//  * a client's queue is a bounded ring (GpuQueueOptions::ring_capacity);
//    add_request returns DMC_EQUEUEFULL (< 0) when it is full;
//  * the push queue's sched-ahead timer waits on the right clock (the
//    reference converts a CLOCK_REALTIME Time into a steady_clock deadline,
//    :1771-1773, so its timer never fires on time).
#pragma once

#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <type_traits>
#include <unordered_map>
#include <variant>
#include <vector>

#include "../../include/dmclock_gpu.h"
#include "dmclock_recs.h"

namespace crimson {
namespace dmclock {

constexpr double max_tag = std::numeric_limits<double>::infinity();
constexpr double min_tag = -std::numeric_limits<double>::infinity();

constexpr auto standard_idle_age = std::chrono::seconds(300);
constexpr auto standard_erase_age = std::chrono::seconds(600);
constexpr auto standard_check_time = std::chrono::seconds(60);
constexpr auto aggressive_check_time = std::chrono::seconds(5);
constexpr unsigned standard_erase_max = 2000;

enum class AtLimit { Wait, Allow, Reject };  // :74-84
using RejectThreshold = Time;                 // :89
using AtLimitParam = std::variant<AtLimit, RejectThreshold>;  // :93

// :95-132
struct ClientInfo {
  double reservation, weight, limit;
  double reservation_inv, weight_inv, limit_inv;
  ClientInfo(double r, double w, double l) { update(r, w, l); }
  inline void update(double r, double w, double l) {
    reservation = r;
    weight = w;
    limit = l;
    reservation_inv = (0.0 == r) ? 0.0 : 1.0 / r;
    weight_inv = (0.0 == w) ? 0.0 : 1.0 / w;
    limit_inv = (0.0 == l) ? 0.0 : 1.0 / l;
  }
  friend std::ostream& operator<<(std::ostream& out, const ClientInfo& c) {
    return out << "{ ClientInfo:: r:" << c.reservation << " w:" << c.weight
               << " l:" << c.limit << " }";
  }
};

// Engine sizing (the reference has none: its containers are unbounded).
struct GpuQueueOptions {
  uint32_t max_clients = 4096;
  uint32_t ring_capacity = 64;
  uint32_t max_batch = 1u << 16;
  int device = 0;
  // single add_request / pull_request calls answered by the engine's
  // persistent serve kernel (DMC_OPT_SERVE): no kernel launch per call
  // (DMCLOCK_GPU_SERVE=0: the single-op kernels)
  bool serve = true;
  static GpuQueueOptions from_env() {
    GpuQueueOptions o;
    if (const char* s = std::getenv("DMCLOCK_GPU_MAX_CLIENTS")) o.max_clients = std::atoi(s);
    if (const char* s = std::getenv("DMCLOCK_GPU_RING")) o.ring_capacity = std::atoi(s);
    if (const char* s = std::getenv("DMCLOCK_GPU_DEVICE")) o.device = std::atoi(s);
    if (const char* s = std::getenv("DMCLOCK_GPU_SERVE")) o.serve = std::atoi(s) != 0;
    return o;
  }
};

class GpuError : public std::runtime_error {
 public:
  explicit GpuError(const std::string& what, int code)
      : std::runtime_error(what + ": " + dmc_strerror(code)), code(code) {}
  int code;
};

namespace detail {
inline void check(int rc, const char* what) {
  if (rc != DMC_OK) throw GpuError(what, rc);
}
// whether T can key an unordered_map: std::hash<T> enabled (a disabled
// specialization is not default-constructible) and T equality-comparable
template <typename T, typename = void>
struct has_std_hash : std::false_type {};
template <typename T>
struct has_std_hash<T, std::void_t<decltype(std::hash<T>{}(std::declval<const T&>())),
                                   decltype(std::declval<const T&>() == std::declval<const T&>())>>
    : std::true_type {};
}  // namespace detail

// PriorityQueueBase (:283-1276) over the engine.
template <typename C, typename R, bool IsDelayed, bool U1, unsigned B>
class PriorityQueueBase {
 public:
  using RequestRef = std::unique_ptr<R>;
  using ClientInfoFunc = std::function<const ClientInfo*(const C&)>;
  enum class NextReqType { returning, future, none };  // :506

  bool empty() const {  // :545-548
    std::lock_guard<std::mutex> g(data_mtx);
    return requests_.empty();
  }
  size_t client_count() const {  // :551-554
    std::lock_guard<std::mutex> g(data_mtx);
    return slot_of_.size();
  }
  size_t request_count() const {  // :557-564
    std::lock_guard<std::mutex> g(data_mtx);
    return requests_.size();
  }

  // :567-585 -- clients in ascending C order; each client front to back (or
  // back to front); the filter receives the request and returns true to
  // remove it.  One readback of every queued handle (dmc_queue_requests), the
  // filter on the host, one device compaction pass (dmc_queue_filter).
  bool remove_by_req_filter(std::function<bool(RequestRef&&)> filter_accum,
                            bool visit_backwards = false) {
    std::lock_guard<std::mutex> g(data_mtx);
    std::vector<uint32_t> counts(opts_.max_clients);
    uint64_t total = 0;
    detail::check(dmc_queue_requests(q_, counts.data(), nullptr, 0, &total),
                  "dmc_queue_requests");
    if (!total) return false;
    std::vector<uint64_t> hs(total);
    detail::check(dmc_queue_requests(q_, nullptr, hs.data(), total, &total),
                  "dmc_queue_requests");
    std::vector<uint64_t> offs(counts.size() + 1, 0);
    for (size_t s = 0; s < counts.size(); ++s) offs[s + 1] = offs[s] + counts[s];
    std::vector<uint8_t> keep(total, 1);
    bool modified = false;
    for (auto& kv : slot_of_) {
      const uint64_t a = offs[kv.second], n = counts[kv.second];
      for (uint64_t j = 0; j < n; ++j) {
        const uint64_t i = a + (visit_backwards ? n - 1 - j : j);
        auto it = requests_.find(hs[i]);
        if (filter_accum(std::move(it->second))) {
          keep[i] = 0;
          modified = true;
        }
      }
    }
    if (!modified) return false;
    for (uint64_t i = 0; i < total; ++i)
      if (!keep[i]) requests_.erase(hs[i]);
    int any = 0;
    detail::check(dmc_queue_filter(q_, keep.data(), total, &any), "dmc_queue_filter");
    return any != 0;
  }

  static void request_sink(RequestRef&&) {}

  // :594-625
  void remove_by_client(const C& client, bool reverse = false,
                        std::function<void(RequestRef&&)> accum = request_sink) {
    std::lock_guard<std::mutex> g(data_mtx);
    const uint32_t* sp = find_slot(client);
    if (!sp) return;
    std::vector<uint64_t> hs(opts_.ring_capacity);
    uint32_t n = 0;
    detail::check(dmc_remove_by_client(q_, *sp, reverse ? 1 : 0,
                                       hs.data(), (uint32_t)hs.size(), &n),
                  "dmc_remove_by_client");
    for (uint32_t i = 0; i < n; ++i) {
      auto r = requests_.find(hs[i]);
      accum(std::move(r->second));
      requests_.erase(r);
    }
  }

  unsigned get_heap_branching_factor() const { return B; }

  void update_client_info(const C& client_id) {  // :633-640
    std::lock_guard<std::mutex> g(data_mtx);
    const uint32_t* sp = find_slot(client_id);
    if (!sp) return;
    info_of_[*sp] = client_info_f(client_id);
    push_info(*sp);
  }

  void update_client_infos() {  // :643-648
    std::lock_guard<std::mutex> g(data_mtx);
    for (auto& kv : slot_of_) {
      info_of_[kv.second] = client_info_f(kv.first);
      push_info(kv.second);
    }
  }

  // counters, :810-812
  size_t reserv_sched_count() const { return stats().reserv_sched_count; }
  size_t prop_sched_count() const { return stats().prop_sched_count; }

  dmc_queue* engine() { return q_; }

 protected:
  PriorityQueueBase(ClientInfoFunc f, std::chrono::milliseconds idle_age,
                    std::chrono::milliseconds erase_age,
                    std::chrono::milliseconds check_time, AtLimitParam alp,
                    double anticipation, GpuQueueOptions opts)
      : client_info_f(std::move(f)),
        opts_(opts),
        idle_age_(idle_age),
        erase_age_(erase_age),
        check_time_(check_time) {
    if (erase_age < idle_age || check_time >= idle_age)
      throw std::invalid_argument("dmclock: erase_age >= idle_age > check_time");
    if (const AtLimit* a = std::get_if<AtLimit>(&alp)) {
      at_limit_ = *a;
    } else {
      at_limit_ = AtLimit::Reject;
      reject_threshold_ = std::get<RejectThreshold>(alp);
    }
    dmc_queue_params p{};
    p.max_clients = opts_.max_clients;
    p.ring_capacity = opts_.ring_capacity;
    p.max_batch = opts_.max_batch;
    p.delayed = IsDelayed ? 1 : 0;
    p.dynamic_info = U1 ? 1 : 0;
    p.at_limit = (int)at_limit_;
    p.reject_threshold = reject_threshold_;
    p.anticipation_timeout = anticipation;
    p.device = opts_.device;
    detail::check(dmc_queue_create(&p, &q_), "dmc_queue_create");
    if (opts_.serve)
      detail::check(dmc_queue_set_option(q_, DMC_OPT_SERVE, 1), "dmc_queue_set_option");
    if (U1)  // get_cli_info (:870-875): the engine asks right before each tag
      detail::check(dmc_queue_set_info_fn(q_, &PriorityQueueBase::info_fn, this),
                    "dmc_queue_set_info_fn");
    info_of_.assign(opts_.max_clients, nullptr);
    dev_info_.assign(opts_.max_clients, ClientInfo(0, 0, 0));
    cleaner_ = std::thread([this] { clean_loop(); });
  }

  ~PriorityQueueBase() {
    {
      std::lock_guard<std::mutex> l(clean_mtx_);
      finishing_ = true;
    }
    clean_cv_.notify_all();
    if (cleaner_.joinable()) cleaner_.join();
    dmc_queue_destroy(q_);
  }

  dmc_stats stats() const {
    dmc_stats st{};
    detail::check(dmc_stats_get(q_, &st), "dmc_stats_get");
    return st;
  }

  // data_mtx held: map C to a slot; first sight registers the client, as
  // do_add_request's client_map.emplace + client_info_f (:920-932)
  uint32_t slot_for(const C& client) {
    if (const uint32_t* sp = find_slot(client)) return *sp;
    uint32_t s;
    if (!free_slots_.empty()) {
      s = free_slots_.back();
      free_slots_.pop_back();
    } else {
      if (next_slot_ >= opts_.max_clients)
        throw GpuError("dmclock: client table full", DMC_EINVAL);
      s = next_slot_++;
    }
    const ClientInfo* info = client_info_f(client);
    if (!info) throw GpuError("dmclock: client_info_f returned null", DMC_EINVAL);
    detail::check(dmc_client_register(q_, s, info->reservation, info->weight,
                                      info->limit, 0),
                  "dmc_client_register");
    slot_of_.emplace(client, s);
    if constexpr (kHashIndex) slot_idx_.emplace(client, s);
    if (client_of_.size() <= s) client_of_.resize(s + 1);
    client_of_[s] = client;
    info_of_[s] = info;
    dev_info_[s] = *info;
    return s;
  }

  // U1: client_info_f for the engine (dmc_info_fn), called inside engine
  // calls made under data_mtx, as the reference calls it under data_mtx
  static int info_fn(void* ctx, uint32_t slot, double* r, double* w, double* l) {
    auto* self = static_cast<PriorityQueueBase*>(ctx);
    if (slot >= self->client_of_.size()) return 1;
    const ClientInfo* ci = self->client_info_f(self->client_of_[slot]);
    if (!ci) return 1;
    self->info_of_[slot] = ci;
    *r = ci->reservation;
    *w = ci->weight;
    *l = ci->limit;
    return 0;
  }

  // data_mtx held: make the device copy of a slot's ClientInfo current
  void push_info(uint32_t s) {
    const ClientInfo* ci = info_of_[s];
    if (!ci) return;
    const ClientInfo& d = dev_info_[s];
    if (d.reservation == ci->reservation && d.weight == ci->weight &&
        d.limit == ci->limit)
      return;
    detail::check(dmc_client_update_info(q_, s, ci->reservation, ci->weight,
                                         ci->limit),
                  "dmc_client_update_info");
    dev_info_[s] = *ci;
  }

  // data_mtx held: do_add_request (:913-1018) for one request
  int do_add_request(RequestRef&& request, const C& client_id,
                     const ReqParams& req_params, Time time, Cost cost) {
    uint32_t s = slot_for(client_id);
    // U1: the engine fetches the info through info_fn at the tag calculation;
    // otherwise values changed in place through the cached pointer are pushed
    if (!U1) push_info(s);
    uint64_t h = next_handle_++;
    dmc_request rq{s, cost, time, req_params.delta, req_params.rho, h};
    int32_t rc = 0;
    detail::check(dmc_add_batch(q_, 1, &rq, &rc), "dmc_add_batch");
    if (rc == DMC_OK) requests_.emplace(h, std::move(request));
    if (rc == DMC_EBADTAG)
      throw GpuError("dmclock: bad tag (reservation and proportion both 0)", rc);
    return rc;
  }

  // data_mtx held: one pull_request(now) on the engine
  int do_pull(Time now, dmc_decision* d, dmc_pull_result* res) {
    // U1, delayed: the engine calls info_fn for the client it pops
    detail::check(dmc_pull_batch(q_, now, 1, d, res), "dmc_pull_batch");
    return res->n_decisions ? 0 : (int)res->next_type;
  }

  RequestRef take_request(uint64_t h) {
    auto it = requests_.find(h);
    RequestRef r = std::move(it->second);
    requests_.erase(it);
    return r;
  }

  // do_clean, :1206-1255, driven by the cleaner thread
  void do_clean() {
    auto now = std::chrono::steady_clock::now();
    std::lock_guard<std::mutex> g(data_mtx);
    dmc_stats st = stats();
    mark_points_.emplace_back(now, st.tick);
    Counter erase_point = last_erase_point_;
    auto point = mark_points_.front();
    while (point.first <= now - erase_age_) {
      last_erase_point_ = point.second;
      erase_point = last_erase_point_;
      mark_points_.pop_front();
      point = mark_points_.front();
    }
    Counter idle_point = 0;
    for (auto& i : mark_points_) {
      if (i.first <= now - idle_age_) idle_point = i.second;
      else break;
    }
    Counter erased = 0;
    if (erase_point > 0 || idle_point > 0) {
      std::vector<uint64_t> ticks(next_slot_);
      if (next_slot_)
        detail::check(dmc_client_last_ticks(q_, next_slot_, ticks.data()),
                      "dmc_client_last_ticks");
      // one pass over the clients in C order, then one erase batch and one
      // idle-marking batch on the engine
      std::vector<uint32_t> to_erase, to_idle;
      for (auto i = slot_of_.begin(); i != slot_of_.end();) {
        auto i2 = i++;
        uint32_t s = i2->second;
        if (erase_point && erased < erase_max_ && ticks[s] <= erase_point) {
          to_erase.push_back(s);
          free_slots_.push_back(s);
          info_of_[s] = nullptr;
          if constexpr (kHashIndex) slot_idx_.erase(i2->first);
          slot_of_.erase(i2);
          ++erased;
        } else if (idle_point && ticks[s] <= idle_point) {
          to_idle.push_back(s);
        }
      }
      if (!to_erase.empty()) {
        std::vector<uint64_t> hs((size_t)to_erase.size() * opts_.ring_capacity);
        uint64_t n = 0;
        detail::check(dmc_client_erase_batch(q_, (uint32_t)to_erase.size(),
                                             to_erase.data(), nullptr, hs.data(),
                                             hs.size(), &n),
                      "dmc_client_erase_batch");
        for (uint64_t j = 0; j < n; ++j) requests_.erase(hs[j]);
      }
      if (!to_idle.empty())
        detail::check(dmc_client_mark_idle_batch(q_, (uint32_t)to_idle.size(),
                                                 to_idle.data()),
                      "dmc_client_mark_idle_batch");
      next_period_ = erased >= erase_max_
                         ? std::chrono::duration_cast<std::chrono::milliseconds>(
                               aggressive_check_time)
                         : check_time_;
      if (erased < erase_max_) last_erase_point_ = 0;
    }
  }

  void clean_loop() {
    std::unique_lock<std::mutex> l(clean_mtx_);
    next_period_ = check_time_;
    while (!finishing_) {
      if (clean_cv_.wait_for(l, next_period_, [this] { return finishing_; })) break;
      l.unlock();
      try {
        do_clean();
      } catch (...) {
      }
      l.lock();
    }
  }

  ClientInfoFunc client_info_f;
  mutable std::mutex data_mtx;
  dmc_queue* q_ = nullptr;
  GpuQueueOptions opts_;
  AtLimit at_limit_ = AtLimit::Wait;
  RejectThreshold reject_threshold_ = 0;
  std::map<C, uint32_t> slot_of_;
  // a hash index of the same map for the per-call lookups, when C is
  // hashable (a 1M-client std::map lookup is ≈20 dependent cache misses);
  // slot_of_ keeps the reference's client_map order for the cleaner
  static constexpr bool kHashIndex = detail::has_std_hash<C>::value;
  std::conditional_t<kHashIndex, std::unordered_map<C, uint32_t>, std::map<C, uint32_t>*>
      slot_idx_{};
  const uint32_t* find_slot(const C& c) const {
    if constexpr (kHashIndex) {
      auto it = slot_idx_.find(c);
      return it == slot_idx_.end() ? nullptr : &it->second;
    } else {
      auto it = slot_of_.find(c);
      return it == slot_of_.end() ? nullptr : &it->second;
    }
  }
  std::vector<C> client_of_;
  std::vector<const ClientInfo*> info_of_;
  std::vector<ClientInfo> dev_info_;
  std::vector<uint32_t> free_slots_;
  uint32_t next_slot_ = 0;
  std::unordered_map<uint64_t, RequestRef> requests_;
  uint64_t next_handle_ = 1;
  // cleaner
  std::chrono::milliseconds idle_age_, erase_age_, check_time_;
  std::chrono::milliseconds next_period_{0};
  std::deque<std::pair<std::chrono::steady_clock::time_point, Counter>> mark_points_;
  Counter last_erase_point_ = 0;
  Counter erase_max_ = standard_erase_max;
  std::mutex clean_mtx_;
  std::condition_variable clean_cv_;
  bool finishing_ = false;
  std::thread cleaner_;
};

// :1279-1501
template <typename C, typename R, bool IsDelayed = false, bool U1 = false,
          unsigned B = 2>
class PullPriorityQueue : public PriorityQueueBase<C, R, IsDelayed, U1, B> {
  using super = PriorityQueueBase<C, R, IsDelayed, U1, B>;

 public:
  using typename super::NextReqType;
  using typename super::RequestRef;
  using typename super::ClientInfoFunc;

  struct PullReq {  // :1286-1306
    struct Retn {
      C client;
      RequestRef request;
      PhaseType phase;
      Cost cost;
    };
    NextReqType type;
    std::variant<Retn, Time> data;
    bool is_none() const { return type == NextReqType::none; }
    bool is_retn() const { return type == NextReqType::returning; }
    Retn& get_retn() { return std::get<Retn>(data); }
    bool is_future() const { return type == NextReqType::future; }
    Time getTime() const { return std::get<Time>(data); }
  };

  template <typename Rep, typename Per>
  PullPriorityQueue(ClientInfoFunc f, std::chrono::duration<Rep, Per> idle_age,
                    std::chrono::duration<Rep, Per> erase_age,
                    std::chrono::duration<Rep, Per> check_time,
                    AtLimitParam at_limit_param = AtLimit::Wait,
                    double anticipation_timeout = 0.0,
                    GpuQueueOptions opts = GpuQueueOptions::from_env())
      : super(f, std::chrono::duration_cast<std::chrono::milliseconds>(idle_age),
              std::chrono::duration_cast<std::chrono::milliseconds>(erase_age),
              std::chrono::duration_cast<std::chrono::milliseconds>(check_time),
              at_limit_param, anticipation_timeout, opts) {}

  PullPriorityQueue(ClientInfoFunc f, AtLimitParam at_limit_param = AtLimit::Wait,
                    double anticipation_timeout = 0.0,
                    GpuQueueOptions opts = GpuQueueOptions::from_env())
      : PullPriorityQueue(f, standard_idle_age, standard_erase_age,
                          standard_check_time, at_limit_param,
                          anticipation_timeout, opts) {}

  int add_request(R&& request, const C& client_id, const ReqParams& req_params,
                  const Cost cost = 1u) {
    return add_request(RequestRef(new R(std::move(request))), client_id,
                       req_params, get_time(), cost);
  }
  int add_request(R&& request, const C& client_id, const Cost cost = 1u) {
    static const ReqParams null_req_params;
    return add_request(RequestRef(new R(std::move(request))), client_id,
                       null_req_params, get_time(), cost);
  }
  int add_request_time(R&& request, const C& client_id,
                       const ReqParams& req_params, const Time time,
                       const Cost cost = 1u) {
    return add_request(RequestRef(new R(std::move(request))), client_id,
                       req_params, time, cost);
  }
  int add_request(RequestRef&& request, const C& client_id,
                  const ReqParams& req_params, const Cost cost = 1u) {
    return add_request(std::move(request), client_id, req_params, get_time(),
                       cost);
  }
  int add_request(RequestRef&& request, const C& client_id,
                  const Cost cost = 1u) {
    static const ReqParams null_req_params;
    return add_request(std::move(request), client_id, null_req_params,
                       get_time(), cost);
  }
  // :1398-1417 -- on EAGAIN the request is not taken (ownership stays)
  int add_request(RequestRef&& request, const C& client_id,
                  const ReqParams& req_params, const Time time,
                  const Cost cost = 1u) {
    std::lock_guard<std::mutex> g(this->data_mtx);
    // do_add_request moves from `request` only on success, so on EAGAIN the
    // caller keeps ownership (test_dmclock_server.cc:1329-1335)
    return this->do_add_request(std::move(request), client_id, req_params,
                                time, cost);
  }

  inline PullReq pull_request() { return pull_request(get_time()); }

  PullReq pull_request(const Time now) {  // :1425-1489
    PullReq result;
    std::lock_guard<std::mutex> g(this->data_mtx);
    dmc_decision d{};
    dmc_pull_result res{};
    int t = this->do_pull(now, &d, &res);
    if (t == DMC_NEXT_NONE) {
      result.type = NextReqType::none;
      return result;
    }
    if (t == DMC_NEXT_FUTURE) {
      result.type = NextReqType::future;
      result.data = res.when;
      return result;
    }
    result.type = NextReqType::returning;
    result.data = typename PullReq::Retn{
        this->client_of_[d.slot], this->take_request(d.handle),
        d.phase == DMC_PHASE_RESERVATION ? PhaseType::reservation
                                         : PhaseType::priority,
        d.cost};
    return result;
  }

  // Extension: k pull_request(now) in one batched engine call; returns the
  // dispatched requests in order and the stopping result in *stop.
  std::vector<typename PullReq::Retn> pull_requests(Time now, uint32_t k,
                                                    PullReq* stop = nullptr) {
    std::lock_guard<std::mutex> g(this->data_mtx);
    std::vector<dmc_decision> ds(k);
    dmc_pull_result res{};
    detail::check(dmc_pull_batch(this->q_, now, k, ds.data(), &res),
                  "dmc_pull_batch");
    std::vector<typename PullReq::Retn> out;
    out.reserve(res.n_decisions);
    for (uint32_t i = 0; i < res.n_decisions; ++i)
      out.push_back(typename PullReq::Retn{
          this->client_of_[ds[i].slot], this->take_request(ds[i].handle),
          ds[i].phase == DMC_PHASE_RESERVATION ? PhaseType::reservation
                                               : PhaseType::priority,
          ds[i].cost});
    if (stop) {
      stop->type = res.next_type == DMC_NEXT_FUTURE ? NextReqType::future
                   : res.next_type == DMC_NEXT_NONE ? NextReqType::none
                                                    : NextReqType::returning;
      if (stop->type == NextReqType::future) stop->data = res.when;
    }
    return out;
  }
};

// :1505-1797
template <typename C, typename R, bool IsDelayed = false, bool U1 = false,
          unsigned B = 2>
class PushPriorityQueue : public PriorityQueueBase<C, R, IsDelayed, U1, B> {
  using super = PriorityQueueBase<C, R, IsDelayed, U1, B>;

 public:
  using typename super::NextReqType;
  using typename super::RequestRef;
  using typename super::ClientInfoFunc;
  using CanHandleRequestFunc = std::function<bool(void)>;
  using HandleRequestFunc =
      std::function<void(const C&, RequestRef, PhaseType, uint64_t)>;

  template <typename Rep, typename Per>
  PushPriorityQueue(ClientInfoFunc f, CanHandleRequestFunc can_handle_f,
                    HandleRequestFunc handle_f,
                    std::chrono::duration<Rep, Per> idle_age,
                    std::chrono::duration<Rep, Per> erase_age,
                    std::chrono::duration<Rep, Per> check_time,
                    AtLimitParam at_limit_param = AtLimit::Wait,
                    double anticipation_timeout = 0.0,
                    GpuQueueOptions opts = GpuQueueOptions::from_env())
      : super(f, std::chrono::duration_cast<std::chrono::milliseconds>(idle_age),
              std::chrono::duration_cast<std::chrono::milliseconds>(erase_age),
              std::chrono::duration_cast<std::chrono::milliseconds>(check_time),
              at_limit_param, anticipation_timeout, opts),
        can_handle_f_(std::move(can_handle_f)),
        handle_f_(std::move(handle_f)) {
    sched_thd_ = std::thread([this] { run_sched_ahead(); });
  }

  PushPriorityQueue(ClientInfoFunc f, CanHandleRequestFunc can_handle_f,
                    HandleRequestFunc handle_f,
                    AtLimitParam at_limit_param = AtLimit::Wait,
                    double anticipation_timeout = 0.0,
                    GpuQueueOptions opts = GpuQueueOptions::from_env())
      : PushPriorityQueue(f, can_handle_f, handle_f, standard_idle_age,
                          standard_erase_age, standard_check_time,
                          at_limit_param, anticipation_timeout, opts) {}

  ~PushPriorityQueue() {
    {
      std::lock_guard<std::mutex> l(sched_mtx_);
      finishing_ = true;
    }
    sched_cv_.notify_one();
    sched_thd_.join();
  }

  int add_request(R&& request, const C& client_id, const ReqParams& req_params,
                  const Cost cost = 1u) {
    return add_request(RequestRef(new R(std::move(request))), client_id,
                       req_params, get_time(), cost);
  }
  int add_request(RequestRef&& request, const C& client_id,
                  const ReqParams& req_params, const Cost cost = 1u) {
    return add_request(std::move(request), client_id, req_params, get_time(),
                       cost);
  }
  int add_request_time(const R& request, const C& client_id,
                       const ReqParams& req_params, const Time time,
                       const Cost cost = 1u) {
    return add_request(RequestRef(new R(request)), client_id, req_params, time,
                       cost);
  }
  int add_request(RequestRef&& request, const C& client_id,
                  const ReqParams& req_params, const Time time,
                  const Cost cost = 1u) {  // :1627-1648
    std::lock_guard<std::mutex> g(this->data_mtx);
    int rc = this->do_add_request(std::move(request), client_id, req_params,
                                  time, cost);
    if (rc != DMC_OK) return rc;
    schedule_request();
    return rc;
  }

  void request_completed() {  // :1651-1660
    std::lock_guard<std::mutex> g(this->data_mtx);
    schedule_request();
  }

 protected:
  // data_mtx held, :1741-1755; handle_f runs under the lock, as in the
  // reference (:1682-1689)
  void schedule_request() {
    if (!can_handle_f_()) return;
    dmc_decision d{};
    dmc_pull_result res{};
    int t = this->do_pull(get_time(), &d, &res);
    if (t == DMC_NEXT_NONE) return;
    if (t == DMC_NEXT_FUTURE) {
      sched_at(res.when);
      return;
    }
    handle_f_(this->client_of_[d.slot], this->take_request(d.handle),
              d.phase == DMC_PHASE_RESERVATION ? PhaseType::reservation
                                               : PhaseType::priority,
              d.cost);
  }

  void sched_at(Time when) {  // :1789-1796
    std::lock_guard<std::mutex> l(sched_mtx_);
    if (finishing_) return;
    if (sched_when_ == TimeZero || when < sched_when_) {
      sched_when_ = when;
      sched_cv_.notify_one();
    }
  }

  // :1760-1786, with the deadline taken on the clock Time is measured on
  void run_sched_ahead() {
    std::unique_lock<std::mutex> l(sched_mtx_);
    while (!finishing_) {
      if (sched_when_ == TimeZero) {
        sched_cv_.wait(l, [this] { return finishing_ || sched_when_ != TimeZero; });
        continue;
      }
      Time when = sched_when_;
      double wait_s = when - get_time();
      if (wait_s > 0) {
        auto d = std::chrono::duration<double>(std::min(wait_s, 3600.0));
        if (sched_cv_.wait_for(l, d, [this, when] {
              return finishing_ || (sched_when_ != when);
            }))
          continue;  // finishing, or rescheduled earlier
      }
      sched_when_ = TimeZero;
      if (finishing_) return;
      l.unlock();
      {
        std::lock_guard<std::mutex> g(this->data_mtx);
        schedule_request();
      }
      l.lock();
    }
  }

  CanHandleRequestFunc can_handle_f_;
  HandleRequestFunc handle_f_;
  std::mutex sched_mtx_;
  std::condition_variable sched_cv_;
  Time sched_when_ = TimeZero;
  bool finishing_ = false;
  std::thread sched_thd_;
};

}  // namespace dmclock
}  // namespace crimson
