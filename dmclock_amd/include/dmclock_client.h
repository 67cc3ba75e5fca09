// SPDX-License-Identifier: LGPL-2.1
//
// dmclock_client.h -- client-side delta/rho tracking of the reference
// (/root/reference/src/dmclock_client.h:39-287): OrigTracker,
// BorrowingTracker and ServiceTracker<S, T>.  Host-side C++ (it runs where
// requests are issued); the multi-GPU deployment sums the completion
// counters per epoch with an RCCL all-reduce instead (multi-GPU).
#pragma once

#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <mutex>
#include <thread>

#include "dmclock_recs.h"

namespace crimson {
namespace dmclock {

// dmclock_client.h:39-84
class OrigTracker {
  Counter delta_prev_req;
  Counter rho_prev_req;
  uint32_t my_delta;
  uint32_t my_rho;

 public:
  OrigTracker(Counter global_delta, Counter global_rho)
      : delta_prev_req(global_delta), rho_prev_req(global_rho), my_delta(0),
        my_rho(0) {}
  static inline OrigTracker create(Counter d, Counter r) { return OrigTracker(d, r); }
  inline ReqParams prepare_req(Counter& the_delta, Counter& the_rho) {
    Counter dout = the_delta - delta_prev_req - my_delta;
    Counter rout = the_rho - rho_prev_req - my_rho;
    delta_prev_req = the_delta;
    rho_prev_req = the_rho;
    my_delta = 0;
    my_rho = 0;
    return ReqParams(uint32_t(dout), uint32_t(rout));
  }
  inline void resp_update(PhaseType phase, Counter& the_delta, Counter& the_rho,
                          Cost cost) {
    the_delta += cost;
    my_delta += cost;
    if (phase == PhaseType::reservation) {
      the_rho += cost;
      my_rho += cost;
    }
  }
  inline Counter get_last_delta() const { return delta_prev_req; }
};

// dmclock_client.h:90-154
class BorrowingTracker {
  Counter delta_prev_req;
  Counter rho_prev_req;
  Counter delta_borrow;
  Counter rho_borrow;

 public:
  BorrowingTracker(Counter global_delta, Counter global_rho)
      : delta_prev_req(global_delta), rho_prev_req(global_rho),
        delta_borrow(0), rho_borrow(0) {}
  static inline BorrowingTracker create(Counter d, Counter r) {
    return BorrowingTracker(d, r);
  }
  inline Counter calc_with_borrow(const Counter& global, const Counter& previous,
                                  Counter& borrow) {
    Counter result = global - previous;
    if (0 == result) {
      ++borrow;  // borrow a future reply
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
  inline ReqParams prepare_req(Counter& the_delta, Counter& the_rho) {
    Counter d = calc_with_borrow(the_delta, delta_prev_req, delta_borrow);
    Counter r = calc_with_borrow(the_rho, rho_prev_req, rho_borrow);
    delta_prev_req = the_delta;
    rho_prev_req = the_rho;
    return ReqParams(uint32_t(d), uint32_t(r));
  }
  inline void resp_update(PhaseType phase, Counter& the_delta, Counter& the_rho,
                          Counter cost) {
    the_delta += cost;
    if (phase == PhaseType::reservation) the_rho += cost;
  }
  inline Counter get_last_delta() const { return delta_prev_req; }
};

// dmclock_client.h:163-287
template <typename S, typename T = OrigTracker>
class ServiceTracker {
  using TimePoint = std::chrono::steady_clock::time_point;
  using MarkPoint = std::pair<TimePoint, Counter>;

  Counter delta_counter;  // # reqs completed
  Counter rho_counter;    // # reqs completed via reservation
  std::map<S, T> server_map;
  mutable std::mutex data_mtx;
  std::deque<MarkPoint> clean_mark_points;
  std::chrono::milliseconds clean_every, clean_age;
  std::mutex clean_mtx;
  std::condition_variable clean_cv;
  bool finishing = false;
  std::thread cleaner;

 public:
  template <typename Rep, typename Per>
  ServiceTracker(std::chrono::duration<Rep, Per> _clean_every,
                 std::chrono::duration<Rep, Per> _clean_age)
      : delta_counter(1), rho_counter(1),
        clean_every(std::chrono::duration_cast<std::chrono::milliseconds>(_clean_every)),
        clean_age(std::chrono::duration_cast<std::chrono::milliseconds>(_clean_age)) {
    cleaner = std::thread([this] {
      std::unique_lock<std::mutex> l(clean_mtx);
      while (!finishing) {
        if (clean_cv.wait_for(l, clean_every, [this] { return finishing; })) break;
        l.unlock();
        do_clean();
        l.lock();
      }
    });
  }
  ServiceTracker() : ServiceTracker(std::chrono::minutes(5), std::chrono::minutes(10)) {}
  ~ServiceTracker() {
    {
      std::lock_guard<std::mutex> l(clean_mtx);
      finishing = true;
    }
    clean_cv.notify_all();
    cleaner.join();
  }

  void track_resp(const S& server_id, const PhaseType& phase,
                  Counter request_cost = 1u) {  // :221-236
    std::lock_guard<std::mutex> g(data_mtx);
    auto it = server_map.find(server_id);
    if (server_map.end() == it)
      it = server_map.emplace(server_id, T::create(delta_counter, rho_counter)).first;
    it->second.resp_update(phase, delta_counter, rho_counter, request_cost);
  }

  ReqParams get_req_params(const S& server) {  // :241-251
    std::lock_guard<std::mutex> g(data_mtx);
    auto it = server_map.find(server);
    if (server_map.end() == it) {
      server_map.emplace(server, T::create(delta_counter, rho_counter));
      return ReqParams(1, 1);
    }
    return it->second.prepare_req(delta_counter, rho_counter);
  }

  size_t server_count() const {
    std::lock_guard<std::mutex> g(data_mtx);
    return server_map.size();
  }

  // :263-286
  void do_clean() {
    TimePoint now = std::chrono::steady_clock::now();
    std::lock_guard<std::mutex> g(data_mtx);
    clean_mark_points.emplace_back(MarkPoint(now, delta_counter));
    Counter earliest = 0;
    auto point = clean_mark_points.front();
    while (point.first <= now - clean_age) {
      earliest = point.second;
      clean_mark_points.pop_front();
      point = clean_mark_points.front();
    }
    if (earliest > 0) {
      for (auto i = server_map.begin(); i != server_map.end();) {
        auto i2 = i++;
        if (i2->second.get_last_delta() <= earliest) server_map.erase(i2);
      }
    }
  }
};

}  // namespace dmclock
}  // namespace crimson
