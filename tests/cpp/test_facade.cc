// SPDX-License-Identifier: LGPL-2.1
//
// The reference's server/client known-answer tests
// (/root/reference/test/test_dmclock_server.cc, test_dmclock_client.cc),
// re-expressed against the drop-in C++ facade: same crimson::dmclock names,
// same calls, same expected values; the queue underneath is the MI355X
// engine.  A tiny assertion harness stands in for GTest (not installed).
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <functional>
#include <list>
#include <string>
#include <thread>
#include <vector>

#include "dmclock_client.h"
#include "dmclock_server.h"

namespace dmc = crimson::dmclock;
using namespace crimson::dmclock;

static int g_fail = 0, g_checks = 0;
static std::string g_test;
#define EXPECT_TRUE(c)                                                        \
  do {                                                                        \
    ++g_checks;                                                               \
    if (!(c)) {                                                               \
      ++g_fail;                                                               \
      std::fprintf(stderr, "FAIL %s %s:%d: %s\n", g_test.c_str(), __FILE__,   \
                   __LINE__, #c);                                             \
    }                                                                         \
  } while (0)
#define EXPECT_EQ(a, b)                                                       \
  do {                                                                        \
    ++g_checks;                                                               \
    auto va_ = (a);                                                           \
    auto vb_ = (b);                                                           \
    if (!(va_ == vb_)) {                                                      \
      ++g_fail;                                                               \
      std::fprintf(stderr, "FAIL %s %s:%d: %s == %s (%s vs %s)\n",           \
                   g_test.c_str(), __FILE__, __LINE__, #a, #b,                \
                   std::to_string(va_).c_str(), std::to_string(vb_).c_str()); \
    }                                                                         \
  } while (0)

struct Request {};

static std::vector<std::pair<std::string, std::function<void()>>>& registry() {
  static std::vector<std::pair<std::string, std::function<void()>>> r;
  return r;
}
struct Reg {
  Reg(const char* n, std::function<void()> f) { registry().emplace_back(n, f); }
};
#define TEST(name)                         \
  static void name();                      \
  static Reg reg_##name(#name, name);      \
  static void name()

TEST(pull_weight) {  // :822-874
  using Queue = dmc::PullPriorityQueue<int, Request>;
  int client1 = 17, client2 = 98;
  dmc::ClientInfo info1(0.0, 1.0, 0.0), info2(0.0, 2.0, 0.0);
  auto client_info_f = [&](int c) -> const dmc::ClientInfo* {
    return c == client1 ? &info1 : &info2;
  };
  Queue pq(client_info_f, AtLimit::Wait);
  ReqParams req_params(1, 1);
  for (int i = 0; i < 5; ++i) {
    EXPECT_EQ(0, pq.add_request(Request{}, client1, req_params));
    EXPECT_EQ(0, pq.add_request(Request{}, client2, req_params));
  }
  int c1 = 0, c2 = 0;
  for (int i = 0; i < 6; ++i) {
    Queue::PullReq pr = pq.pull_request();
    EXPECT_TRUE(pr.is_retn());
    auto& retn = pr.get_retn();
    (retn.client == client1 ? c1 : c2)++;
    EXPECT_TRUE(retn.phase == PhaseType::priority);
  }
  EXPECT_EQ(2, c1);
  EXPECT_EQ(4, c2);
}

TEST(pull_reservation) {  // :877-929
  using Queue = dmc::PullPriorityQueue<int, Request>;
  int client1 = 52, client2 = 8;
  dmc::ClientInfo info1(2.0, 0.0, 0.0), info2(1.0, 0.0, 0.0);
  auto client_info_f = [&](int c) -> const dmc::ClientInfo* {
    return c == client1 ? &info1 : &info2;
  };
  Queue pq(client_info_f, AtLimit::Wait);
  ReqParams req_params(1, 1);
  auto old_time = dmc::get_time() - 100.0;
  for (int i = 0; i < 5; ++i) {
    EXPECT_EQ(0, pq.add_request_time(Request{}, client1, req_params, old_time));
    EXPECT_EQ(0, pq.add_request_time(Request{}, client2, req_params, old_time));
    old_time += 0.001;
  }
  int c1 = 0, c2 = 0;
  for (int i = 0; i < 6; ++i) {
    Queue::PullReq pr = pq.pull_request();
    EXPECT_TRUE(pr.is_retn());
    (pr.get_retn().client == client1 ? c1 : c2)++;
    EXPECT_TRUE(pr.get_retn().phase == PhaseType::reservation);
  }
  EXPECT_EQ(4, c1);
  EXPECT_EQ(2, c2);
}

TEST(update_client_info) {  // :932-1018
  using Queue = dmc::PullPriorityQueue<int, Request, false>;
  int client1 = 17, client2 = 98;
  dmc::ClientInfo info1(0.0, 100.0, 0.0), info2(0.0, 200.0, 0.0);
  auto client_info_f = [&](int c) -> const dmc::ClientInfo* {
    return c == client1 ? &info1 : &info2;
  };
  Queue pq(client_info_f, AtLimit::Wait);
  ReqParams req_params(1, 1);
  for (int i = 0; i < 5; ++i) {
    EXPECT_EQ(0, pq.add_request(Request{}, client1, req_params));
    EXPECT_EQ(0, pq.add_request(Request{}, client2, req_params));
  }
  int c1 = 0, c2 = 0;
  for (int i = 0; i < 10; ++i) {
    Queue::PullReq pr = pq.pull_request();
    EXPECT_TRUE(pr.is_retn());
    if (i > 5) continue;
    (pr.get_retn().client == client1 ? c1 : c2)++;
  }
  EXPECT_EQ(2, c1);
  EXPECT_EQ(4, c2);
  std::this_thread::sleep_for(std::chrono::milliseconds(100));
  info1 = dmc::ClientInfo(0.0, 200.0, 0.0);
  pq.update_client_info(17);
  for (int i = 0; i < 5; ++i) {
    EXPECT_EQ(0, pq.add_request(Request{}, client1, req_params));
    EXPECT_EQ(0, pq.add_request(Request{}, client2, req_params));
  }
  c1 = c2 = 0;
  for (int i = 0; i < 6; ++i) {
    Queue::PullReq pr = pq.pull_request();
    EXPECT_TRUE(pr.is_retn());
    (pr.get_retn().client == client1 ? c1 : c2)++;
  }
  EXPECT_EQ(3, c1);
  EXPECT_EQ(3, c2);
}

TEST(dynamic_cli_info_f) {  // :1021-1114
  using Queue = dmc::PullPriorityQueue<int, Request, true, true>;
  int client1 = 17, client2 = 98;
  std::vector<dmc::ClientInfo> info1{{0.0, 100.0, 0.0}, {0.0, 150.0, 0.0}};
  std::vector<dmc::ClientInfo> info2{{0.0, 200.0, 0.0}, {0.0, 50.0, 0.0}};
  size_t group = 0;
  auto client_info_f = [&](int c) -> const dmc::ClientInfo* {
    return c == client1 ? &info1[group] : &info2[group];
  };
  Queue pq(client_info_f, AtLimit::Wait);
  ReqParams req_params(1, 1);
  for (int i = 0; i < 5; ++i) {
    EXPECT_EQ(0, pq.add_request(Request{}, client1, req_params));
    EXPECT_EQ(0, pq.add_request(Request{}, client2, req_params));
  }
  int c1 = 0, c2 = 0;
  for (int i = 0; i < 10; ++i) {
    Queue::PullReq pr = pq.pull_request();
    EXPECT_TRUE(pr.is_retn());
    if (i > 5) continue;
    (pr.get_retn().client == client1 ? c1 : c2)++;
  }
  EXPECT_EQ(2, c1);
  EXPECT_EQ(4, c2);
  std::this_thread::sleep_for(std::chrono::milliseconds(100));
  group = 1;
  for (int i = 0; i < 6; ++i) {
    EXPECT_EQ(0, pq.add_request(Request{}, client1, req_params));
    EXPECT_EQ(0, pq.add_request(Request{}, client2, req_params));
  }
  c1 = c2 = 0;
  for (int i = 0; i < 8; ++i) {
    Queue::PullReq pr = pq.pull_request();
    EXPECT_TRUE(pr.is_retn());
    (pr.get_retn().client == client1 ? c1 : c2)++;
  }
  EXPECT_EQ(6, c1);
  EXPECT_EQ(2, c2);
}

TEST(ready_and_under_limit) {  // :1120-1181
  using Queue = dmc::PullPriorityQueue<int, Request>;
  int client1 = 52, client2 = 8;
  dmc::ClientInfo info1(1.0, 0.0, 0.0), info2(1.0, 0.0, 0.0);
  auto client_info_f = [&](int c) -> const dmc::ClientInfo* {
    return c == client1 ? &info1 : &info2;
  };
  Queue pq(client_info_f, AtLimit::Wait);
  ReqParams req_params(0, 0);
  auto start_time = dmc::get_time() - 100.0;
  for (int i = 0; i < 3; ++i) {
    EXPECT_EQ(0, pq.add_request_time(Request{}, client1, req_params, start_time));
    EXPECT_EQ(0, pq.add_request_time(Request{}, client2, req_params, start_time));
  }
  using T = Queue::NextReqType;
  T expect[9] = {T::returning, T::returning, T::future, T::returning,
                 T::returning, T::future,    T::returning, T::returning,
                 T::none};
  for (int i = 0; i < 9; ++i) {
    Queue::PullReq pr = pq.pull_request(start_time + 0.5 + (i / 3));
    EXPECT_TRUE(pr.type == expect[i]);
  }
}

TEST(pull_none) {  // :1184-1205
  using Queue = dmc::PullPriorityQueue<int, Request>;
  dmc::ClientInfo info(1.0, 1.0, 1.0);
  Queue pq([&](int) { return &info; }, AtLimit::Wait);
  EXPECT_TRUE(pq.pull_request(dmc::get_time() + 100).is_none());
}

TEST(pull_future) {  // :1208-1236
  using Queue = dmc::PullPriorityQueue<int, Request>;
  dmc::ClientInfo info(1.0, 0.0, 1.0);
  Queue pq([&](int) { return &info; }, AtLimit::Wait);
  auto now = dmc::get_time();
  EXPECT_EQ(0, pq.add_request_time(Request{}, 52, ReqParams(1, 1), now + 100));
  Queue::PullReq pr = pq.pull_request(now);
  EXPECT_TRUE(pr.is_future());
  EXPECT_TRUE(pr.getTime() == now + 100);
}

TEST(pull_future_limit_break_weight) {  // :1239-1267
  using Queue = dmc::PullPriorityQueue<int, Request>;
  dmc::ClientInfo info(0.0, 1.0, 1.0);
  Queue pq([&](int) { return &info; }, AtLimit::Allow);
  auto now = dmc::get_time();
  EXPECT_EQ(0, pq.add_request_time(Request{}, 52, ReqParams(1, 1), now + 100));
  Queue::PullReq pr = pq.pull_request(now);
  EXPECT_TRUE(pr.is_retn());
  EXPECT_EQ(52, pr.get_retn().client);
}

TEST(pull_future_limit_break_reservation) {  // :1270-1298
  using Queue = dmc::PullPriorityQueue<int, Request>;
  dmc::ClientInfo info(1.0, 0.0, 1.0);
  Queue pq([&](int) { return &info; }, AtLimit::Allow);
  auto now = dmc::get_time();
  EXPECT_EQ(0, pq.add_request_time(Request{}, 52, ReqParams(1, 1), now + 100));
  Queue::PullReq pr = pq.pull_request(now);
  EXPECT_TRUE(pr.is_retn());
  EXPECT_EQ(52, pr.get_retn().client);
}

TEST(pull_reject_at_limit) {  // :1301-1336
  using Queue = dmc::PullPriorityQueue<int, Request, false>;
  using MyReqRef = Queue::RequestRef;
  dmc::ClientInfo info(0.0, 1.0, 1.0);
  Queue pq([&](int) { return &info; }, AtLimit::Reject);
  EXPECT_EQ(0, pq.add_request_time({}, 52, {}, Time{1}));
  EXPECT_EQ(0, pq.add_request_time({}, 52, {}, Time{2}));
  EXPECT_EQ(0, pq.add_request_time({}, 52, {}, Time{3}));
  EXPECT_EQ(EAGAIN, pq.add_request_time({}, 52, {}, Time{3.9}));
  EXPECT_EQ(EAGAIN, pq.add_request_time({}, 52, {}, Time{4}));
  EXPECT_EQ(0, pq.add_request_time({}, 52, {}, Time{6}));
  auto r1 = MyReqRef{new Request};
  EXPECT_EQ(0, pq.add_request(std::move(r1), 53, {}, Time{1}));
  EXPECT_TRUE(nullptr == r1);  // taken on success
  auto r2 = MyReqRef{new Request};
  EXPECT_EQ(EAGAIN, pq.add_request(std::move(r2), 53, {}, Time{1}));
  EXPECT_TRUE(nullptr != r2);  // not taken on failure
}

TEST(pull_reject_threshold) {  // :1339-1360
  using Queue = dmc::PullPriorityQueue<int, Request, false>;
  dmc::ClientInfo info(0.0, 1.0, 1.0);
  Queue pq([&](int) { return &info; }, RejectThreshold{3.0});
  EXPECT_EQ(0, pq.add_request_time({}, 52, {}, Time{1}));
  EXPECT_EQ(0, pq.add_request_time({}, 52, {}, Time{1}));
  EXPECT_EQ(0, pq.add_request_time({}, 52, {}, Time{1}));
  EXPECT_EQ(0, pq.add_request_time({}, 52, {}, Time{1}));
  EXPECT_EQ(EAGAIN, pq.add_request_time({}, 52, {}, Time{1}));
  EXPECT_EQ(0, pq.add_request_time({}, 52, {}, Time{3}));
}

TEST(pull_wait_at_limit) {  // :1363-1471
  using Queue = dmc::PullPriorityQueue<int, Request>;
  int client1 = 52, client2 = 8;
  dmc::ClientInfo info1(1.0, 2.0, 100.0), info2(1.0, 1.0, 2.0);
  auto client_info_f = [&](int c) -> const dmc::ClientInfo* {
    return c == client1 ? &info1 : &info2;
  };
  Queue pq(client_info_f, AtLimit::Wait);
  ReqParams req_params(1, 1);
  auto add_time = dmc::get_time() - 1.0;
  auto old_time = add_time;
  for (int i = 0; i < 50; ++i) {
    EXPECT_EQ(0, pq.add_request_time(Request{}, client1, req_params, add_time));
    EXPECT_EQ(0, pq.add_request_time(Request{}, client2, req_params, add_time));
    add_time += 0.01;
  }
  EXPECT_EQ(2u, pq.client_count());
  EXPECT_EQ(100u, pq.request_count());
  int c1 = 0, c2 = 0;
  for (int i = 0; i < 2; ++i) {
    Queue::PullReq pr = pq.pull_request();
    EXPECT_TRUE(pr.is_retn());
    (pr.get_retn().client == client1 ? c1 : c2)++;
    EXPECT_TRUE(pr.get_retn().phase == PhaseType::reservation);
  }
  EXPECT_EQ(1, c1);
  EXPECT_EQ(1, c2);
  EXPECT_EQ(98u, pq.request_count());
  for (int i = 0; i < 50; ++i) {
    Queue::PullReq pr = pq.pull_request();
    EXPECT_TRUE(pr.is_retn());
    (pr.get_retn().client == client1 ? c1 : c2)++;
    EXPECT_TRUE(pr.get_retn().phase == PhaseType::priority);
  }
  EXPECT_EQ(48u, pq.request_count());
  Queue::PullReq pr = pq.pull_request();
  EXPECT_TRUE(pr.is_future());
  EXPECT_TRUE(pr.getTime() == old_time + 2.0);
  EXPECT_EQ(50, c1);
  EXPECT_EQ(2, c2);
  pr = pq.pull_request(old_time + 2.0);
  EXPECT_TRUE(pr.is_retn());
  EXPECT_EQ(client2, pr.get_retn().client);
  EXPECT_EQ(47u, pq.request_count());
}

TEST(delayed_tag_calc) {  // :273-316
  ClientInfo info(0.0, 1.0, 1.0);
  auto client_info_f = [&](int) -> const ClientInfo* { return &info; };
  Time t{1};
  {
    PullPriorityQueue<int, Request, true> queue(client_info_f);
    queue.add_request_time({}, 17, {0, 0}, t);
    queue.add_request_time({}, 17, {0, 0}, t + 1);
    queue.add_request_time({}, 17, {10, 10}, t + 2);
    EXPECT_TRUE(queue.pull_request(t).is_retn());
    auto pr2 = queue.pull_request(t + 1);
    EXPECT_TRUE(pr2.is_future());
    EXPECT_TRUE(pr2.getTime() == t + 11);
  }
  {
    PullPriorityQueue<int, Request, false> queue(client_info_f);
    queue.add_request_time({}, 17, {0, 0}, t);
    queue.add_request_time({}, 17, {0, 0}, t + 1);
    queue.add_request_time({}, 17, {10, 10}, t + 2);
    EXPECT_TRUE(queue.pull_request(t).is_retn());
    EXPECT_TRUE(queue.pull_request(t + 1).is_retn());
    auto pr3 = queue.pull_request(t + 2);
    EXPECT_TRUE(pr3.is_future());
    EXPECT_TRUE(pr3.getTime() == t + 12);
  }
}

struct MyReq {
  int id;
  MyReq(int i) : id(i) {}
};

TEST(remove_by_req_filter) {  // :373-440
  using Queue = dmc::PullPriorityQueue<int, MyReq>;
  using MyReqRef = Queue::RequestRef;
  dmc::ClientInfo info1(0.0, 1.0, 0.0);
  Queue pq([&](int) { return &info1; }, AtLimit::Allow);
  EXPECT_EQ(0u, pq.client_count());
  EXPECT_EQ(0u, pq.request_count());
  ReqParams rp(1, 1);
  int ids1[] = {1, 11}, ids2[] = {2, 0, 13, 2, 13, 98};
  for (int i : ids1) EXPECT_EQ(0, pq.add_request(MyReq(i), 17, rp));
  for (int i : ids2) EXPECT_EQ(0, pq.add_request(MyReq(i), 98, rp));
  EXPECT_EQ(0, pq.add_request(MyReq(44), 17, rp));
  EXPECT_EQ(2u, pq.client_count());
  EXPECT_EQ(9u, pq.request_count());
  pq.remove_by_req_filter([](MyReqRef&& r) -> bool { return 1 == r->id % 2; });
  EXPECT_EQ(5u, pq.request_count());
  std::list<MyReq> capture;
  pq.remove_by_req_filter(
      [&capture](MyReqRef&& r) -> bool {
        if (0 == r->id % 2) {
          capture.push_front(*r);
          return true;
        }
        return false;
      },
      true);
  EXPECT_EQ(0u, pq.request_count());
  EXPECT_EQ(5u, capture.size());
  int total = 0;
  for (auto i : capture) total += i.id;
  EXPECT_EQ(146, total);
}

TEST(remove_by_req_filter_ordering) {  // :443-605
  using Queue = dmc::PullPriorityQueue<int, MyReq>;
  using MyReqRef = Queue::RequestRef;
  dmc::ClientInfo info1(0.0, 1.0, 0.0);
  for (int backwards = 0; backwards < 2; ++backwards) {
    Queue pq([&](int) { return &info1; }, AtLimit::Allow);
    for (int i = 1; i <= 6; ++i) EXPECT_EQ(0, pq.add_request(MyReq(i), 17, ReqParams(1, 1)));
    std::vector<MyReq> cap;
    pq.remove_by_req_filter(
        [&](MyReqRef&& r) -> bool {
          if (1 == r->id % 2) {
            if (backwards) cap.insert(cap.begin(), *r);
            else cap.push_back(*r);
            return true;
          }
          return false;
        },
        backwards);
    EXPECT_EQ(3u, pq.request_count());
    EXPECT_EQ(3u, cap.size());
    EXPECT_TRUE(cap[0].id == 1 && cap[1].id == 3 && cap[2].id == 5);
    std::vector<MyReq> cap2;
    pq.remove_by_req_filter(
        [&](MyReqRef&& r) -> bool {
          if (0 == r->id % 2) {
            if (backwards) cap2.push_back(*r);
            else cap2.insert(cap2.begin(), *r);
            return true;
          }
          return false;
        },
        backwards);
    EXPECT_EQ(0u, pq.request_count());
    EXPECT_TRUE(cap2.size() == 3 && cap2[0].id == 6 && cap2[1].id == 4 &&
                cap2[2].id == 2);
  }
}

TEST(remove_by_client) {  // :608-681
  using Queue = dmc::PullPriorityQueue<int, MyReq>;
  using MyReqRef = Queue::RequestRef;
  dmc::ClientInfo info1(0.0, 1.0, 0.0);
  Queue pq([&](int) { return &info1; }, AtLimit::Allow);
  ReqParams rp(1, 1);
  int ids1[] = {1, 11}, ids2[] = {2, 0, 13, 2, 13, 98};
  for (int i : ids1) EXPECT_EQ(0, pq.add_request(MyReq(i), 17, rp));
  for (int i : ids2) EXPECT_EQ(0, pq.add_request(MyReq(i), 98, rp));
  EXPECT_EQ(0, pq.add_request(MyReq(44), 17, rp));
  EXPECT_EQ(9u, pq.request_count());
  std::list<MyReq> removed;
  pq.remove_by_client(17, true, [&removed](MyReqRef&& r) { removed.push_front(*r); });
  EXPECT_EQ(3u, removed.size());
  EXPECT_EQ(1, removed.front().id);
  removed.pop_front();
  EXPECT_EQ(11, removed.front().id);
  removed.pop_front();
  EXPECT_EQ(44, removed.front().id);
  EXPECT_EQ(6u, pq.request_count());
  Queue::PullReq pr = pq.pull_request();
  EXPECT_TRUE(pr.is_retn());
  EXPECT_EQ(2, pr.get_retn().request->id);
  pr = pq.pull_request();
  EXPECT_TRUE(pr.is_retn());
  EXPECT_EQ(0, pr.get_retn().request->id);
  pq.remove_by_client(98);
  EXPECT_EQ(0u, pq.request_count());
}

TEST(add_req_ref) {  // :684-751 and :754-819
  using Queue = dmc::PullPriorityQueue<int, MyReq>;
  using MyReqRef = Queue::RequestRef;
  dmc::ClientInfo info(0.0, 1.0, 0.0);
  for (int nullp = 0; nullp < 2; ++nullp) {
    Queue pq([&](int) { return &info; }, AtLimit::Allow);
    int order[][2] = {{22, 1}, {44, 2}, {22, 3}, {44, 4}, {44, 5}};
    for (auto& o : order) {
      MyReqRef r(new MyReq(o[1]));
      if (nullp) EXPECT_EQ(0, pq.add_request(std::move(r), o[0]));
      else EXPECT_EQ(0, pq.add_request(std::move(r), o[0], ReqParams(1, 1)));
    }
    EXPECT_EQ(2u, pq.client_count());
    EXPECT_EQ(5u, pq.request_count());
    int first_mod = nullp ? 1 : 0;  // first removal: evens (ref) / odds (null)
    pq.remove_by_req_filter([&](MyReqRef&& r) -> bool { return first_mod == r->id % 2; });
    EXPECT_EQ(nullp ? 2u : 3u, pq.request_count());
    std::list<MyReq> capture;
    pq.remove_by_req_filter(
        [&](MyReqRef&& r) -> bool {
          if (first_mod != r->id % 2) {
            capture.push_front(*r);
            return true;
          }
          return false;
        },
        true);
    EXPECT_EQ(0u, pq.request_count());
    int total = 0;
    for (auto i : capture) total += i.id;
    EXPECT_EQ(nullp ? 6 : 9, total);
  }
}

TEST(client_idle_erase) {  // :100-185 with a 10x faster clock
  using Queue = dmc::PushPriorityQueue<int, Request>;
  dmc::ClientInfo ci(100.0, 1.0, 0.0);
  auto server_ready_f = []() -> bool { return true; };
  auto submit_req_f = [](const int&, std::unique_ptr<Request>, dmc::PhaseType,
                         uint64_t) {};
  Queue pq([&](int) { return &ci; }, server_ready_f, submit_req_f,
           std::chrono::milliseconds(300), std::chrono::milliseconds(500),
           std::chrono::milliseconds(200), AtLimit::Wait);
  EXPECT_EQ(0u, pq.client_count());
  Request req;
  EXPECT_EQ(0, pq.add_request_time(req, 17, ReqParams(1, 1), dmc::get_time()));
  std::this_thread::sleep_for(std::chrono::milliseconds(100));
  EXPECT_EQ(1u, pq.client_count());
  std::this_thread::sleep_for(std::chrono::milliseconds(800));
  EXPECT_EQ(0u, pq.client_count());
}

TEST(add_req_pushprio_queue) {  // :188-270: handle_f sees every request
  struct R2 {
    int id;
    R2(int i) : id(i) {}
  };
  using Queue = dmc::PushPriorityQueue<int, R2>;
  dmc::ClientInfo ci(0.0, 1.0, 0.0);
  std::vector<int> handled;
  Queue pq([&](int) { return &ci; }, []() { return true; },
           [&](const int&, std::unique_ptr<R2> r, dmc::PhaseType, uint64_t) {
             handled.push_back(r->id);
           },
           AtLimit::Wait);
  EXPECT_EQ(0, pq.add_request(Queue::RequestRef(new R2(11)), 17, ReqParams(1, 1)));
  EXPECT_EQ(0, pq.add_request(R2(22), 34, ReqParams(1, 1)));
  EXPECT_EQ(2u, pq.client_count());
  EXPECT_EQ(2u, handled.size());
}

TEST(push_sched_ahead_fires) {
  // A limit-throttled request must be dispatched by the sched-ahead timer
  // (the reference's timer never fires on time, dmclock_server.h:1771-1773).
  // limit 5/s: the 2nd and 3rd requests become eligible 0.4 s and 0.8 s
  // after the 1st; without completions only the timer can dispatch them.
  using Queue = dmc::PushPriorityQueue<int, Request>;
  dmc::ClientInfo ci(0.0, 1.0, 5.0);
  std::atomic<int> handled{0};
  Queue pq([&](int) { return &ci; }, []() { return true; },
           [&](const int&, std::unique_ptr<Request>, dmc::PhaseType, uint64_t) {
             ++handled;
           },
           AtLimit::Wait);
  for (int i = 0; i < 3; ++i)
    EXPECT_EQ(0, pq.add_request(Request{}, 17, ReqParams(1, 1)));
  EXPECT_EQ(1, handled.load());  // the first goes out at once
  std::this_thread::sleep_for(std::chrono::milliseconds(600));
  EXPECT_EQ(2, handled.load());  // the timer dispatched the second
  pq.request_completed();        // schedules the third for t0 + 0.8 s
  std::this_thread::sleep_for(std::chrono::milliseconds(600));
  EXPECT_EQ(3, handled.load());
}

TEST(tracker_orig) {  // test_dmclock_client.cc:231-304
  dmc::ServiceTracker<int, OrigTracker> st(std::chrono::seconds(2),
                                           std::chrono::seconds(3));
  int s1 = 101, s2 = 7;
  auto eq = [](ReqParams p, uint32_t d, uint32_t r) { return p.delta == d && p.rho == r; };
  EXPECT_TRUE(eq(st.get_req_params(s1), 1, 1));
  EXPECT_TRUE(eq(st.get_req_params(s1), 0, 0));
  st.track_resp(s1, PhaseType::priority, 1u);
  EXPECT_TRUE(eq(st.get_req_params(s1), 0, 0));
  st.track_resp(s2, PhaseType::priority, 1u);
  EXPECT_TRUE(eq(st.get_req_params(s1), 1, 0));
  EXPECT_TRUE(eq(st.get_req_params(s1), 0, 0));
  st.track_resp(s2, PhaseType::reservation, 1u);
  EXPECT_TRUE(eq(st.get_req_params(s1), 1, 1));
  st.track_resp(s2, PhaseType::reservation, 1u);
  st.track_resp(s1, PhaseType::priority, 1u);
  st.track_resp(s2, PhaseType::priority, 1u);
  st.track_resp(s2, PhaseType::reservation, 1u);
  st.track_resp(s1, PhaseType::reservation, 1u);
  st.track_resp(s1, PhaseType::priority, 1u);
  st.track_resp(s2, PhaseType::priority, 1u);
  EXPECT_TRUE(eq(st.get_req_params(s1), 4, 2));
  EXPECT_TRUE(eq(st.get_req_params(s2), 3, 1));
  EXPECT_TRUE(eq(st.get_req_params(s1), 0, 0));
  EXPECT_TRUE(eq(st.get_req_params(s2), 0, 0));
}

TEST(tracker_borrowing) {  // test_dmclock_client.cc:108-225
  dmc::ServiceTracker<int, BorrowingTracker> st(std::chrono::seconds(2),
                                                std::chrono::seconds(3));
  int s1 = 101, s2 = 7;
  auto eq = [](ReqParams p, uint32_t d, uint32_t r) { return p.delta == d && p.rho == r; };
  EXPECT_TRUE(eq(st.get_req_params(s1), 1, 1));
  EXPECT_TRUE(eq(st.get_req_params(s1), 1, 1));
  st.track_resp(s1, PhaseType::priority, 1u);
  EXPECT_TRUE(eq(st.get_req_params(s1), 1, 1));
  st.track_resp(s2, PhaseType::priority, 1u);
  EXPECT_TRUE(eq(st.get_req_params(s1), 1, 1));
  EXPECT_TRUE(eq(st.get_req_params(s1), 1, 1));
  st.track_resp(s2, PhaseType::reservation, 1u);
  EXPECT_TRUE(eq(st.get_req_params(s1), 1, 1));
  st.track_resp(s2, PhaseType::reservation, 1u);
  st.track_resp(s1, PhaseType::priority, 1u);
  st.track_resp(s2, PhaseType::priority, 1u);
  st.track_resp(s2, PhaseType::reservation, 1u);
  st.track_resp(s1, PhaseType::reservation, 1u);
  st.track_resp(s1, PhaseType::priority, 1u);
  st.track_resp(s2, PhaseType::priority, 1u);
  EXPECT_TRUE(eq(st.get_req_params(s1), 5, 1));
  EXPECT_TRUE(eq(st.get_req_params(s2), 9, 4));
  EXPECT_TRUE(eq(st.get_req_params(s1), 1, 1));
  EXPECT_TRUE(eq(st.get_req_params(s2), 1, 1));
}

int main(int argc, char** argv) {
  bool host_only = argc > 1 && std::string(argv[1]) == "--host-only";
  int ran = 0;
  for (auto& t : registry()) {
    if (host_only && t.first.rfind("tracker", 0) != 0) continue;
    g_test = t.first;
    int before = g_fail;
    try {
      t.second();
    } catch (const std::exception& e) {
      ++g_fail;
      std::fprintf(stderr, "FAIL %s: exception %s\n", t.first.c_str(), e.what());
    }
    std::printf("%s %s\n", g_fail == before ? "PASS" : "FAIL", t.first.c_str());
    ++ran;
  }
  std::printf("%d tests, %d checks, %d failures\n", ran, g_checks, g_fail);
  return g_fail ? 1 : 0;
}
