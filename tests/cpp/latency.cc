// SPDX-License-Identifier: LGPL-2.1
//
// Single-call latency of the drop-in API: what a caller
// that does not batch gets.  Three legs run the same operation sequence --
// N clients each given one request (the reference registers a client at its
// first add, idle), then M rounds of one add_request_time of a random client
// followed by one pull_request(now):
//   facade  crimson::dmclock::PullPriorityQueue (dmclock_amd/include) on the
//           engine, one C-ABI call per operation, as drop-in callers use it;
//   engine  the C-ABI directly (dmc_add_batch n=1, dmc_pull_batch k=1);
//   oracle  the CPU restatement of the reference's queue (oracle/, test
//           infrastructure: the reference's heaps, one thread).
// The engine and oracle legs register the clients active in bulk (the
// facade registers each at its first add, idle, as the reference does).
// Prints one JSON line with p50 / p99 / mean per call in microseconds.
//
// --serve: the facade and engine legs with DMC_OPT_SERVE (the persistent
// serve kernel answers each single call; no launch per call).
//
// --queues Q: the engine leg on Q queues of N clients each, the rounds
// dealt round-robin over them from this one thread (more serving queues than
// the process's hardware queues: each call first stops the other queues'
// idle serve kernels).
//
// usage: latency N M [--no-oracle] [--no-facade] [--serve] [--queues Q]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "dmclock_gpu.h"
#include "dmclock_server.h"

extern "C" {  // oracle/dmc_oracle_capi.cc
void* dmo_queue_create(int delayed, int dynamic_info, unsigned branching, int at_limit,
                       double reject_threshold, double anticipation);
void dmo_queue_destroy(void* h);
void dmo_info_set(void* h, uint32_t client, double r, double w, double l, int fresh);
int dmo_register_active_batch(void* h, uint32_t n, const uint32_t* clients, const double* r,
                              const double* w, const double* l);
int dmo_add(void* h, uint64_t handle, uint32_t client, uint32_t delta, uint32_t rho,
            double time, uint32_t cost);
int dmo_pull(void* h, double now, dmc_decision* out, double* when);
}

namespace dmc = crimson::dmclock;
using Clock = std::chrono::steady_clock;

struct Stat {
  std::vector<double> us;
  void add(Clock::time_point a, Clock::time_point b) {
    us.push_back(std::chrono::duration<double, std::micro>(b - a).count());
  }
  std::string json() {
    if (us.empty()) return "null";
    std::vector<double> v = us;
    std::sort(v.begin(), v.end());
    double s = 0;
    for (double x : v) s += x;
    char buf[160];
    std::snprintf(buf, sizeof buf, "{\"p50\": %.2f, \"p99\": %.2f, \"mean\": %.2f, \"n\": %zu}",
                  v[v.size() / 2], v[(v.size() * 99) / 100], s / v.size(), v.size());
    return buf;
  }
};

struct Info {
  double r, w, l;
};

static std::vector<Info> make_infos(uint32_t n) {
  std::mt19937_64 g(7);
  std::uniform_real_distribution<double> u(0.0, 1.0);
  std::vector<Info> v(n);
  for (auto& x : v) {
    x.r = u(g) < 0.5 ? 1.0 + 9.0 * u(g) : 0.0;
    x.w = 0.5 + u(g);
    x.l = 0.0;
  }
  return v;
}

struct Op {
  uint32_t client;
  double t;
};

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: latency N M [--no-oracle] [--no-facade] [--serve]\n");
    return 2;
  }
  const uint32_t N = (uint32_t)std::atol(argv[1]);
  const uint32_t M = (uint32_t)std::atol(argv[2]);
  bool oracle = true, facade = true, serve = false;
  uint32_t nq = 1;
  for (int i = 3; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--queues") && i + 1 < argc) nq = (uint32_t)std::atol(argv[++i]);
    if (!std::strcmp(argv[i], "--serve")) serve = true;
    if (!std::strcmp(argv[i], "--no-oracle")) oracle = false;
    if (!std::strcmp(argv[i], "--no-facade")) facade = false;
  }
  const std::vector<Info> infos = make_infos(N);
  // the operation sequence: N first adds, then M (add, pull) rounds; the
  // arrival rate is 2 requests/s per client
  std::mt19937_64 g(11);
  const double dt = 1.0 / (2.0 * N);
  double t = 1.0;
  std::vector<Op> pre(N), ops(M);
  for (uint32_t c = 0; c < N; ++c) pre[c] = Op{c, t += dt};
  for (auto& o : ops) o = Op{(uint32_t)(g() % N), t += dt};

  Stat f_add, f_pull, e_add, e_pull, o_add, o_pull;
  double f_pre_s = 0, o_pre_s = 0;

  if (facade) {
    struct Req {
      uint64_t id;
    };
    std::vector<dmc::ClientInfo> ci;
    ci.reserve(N);
    for (auto& x : infos) ci.emplace_back(x.r, x.w, x.l);
    dmc::GpuQueueOptions opts;
    opts.max_clients = N;
    opts.ring_capacity = 64;
    opts.serve = serve;
    dmc::PullPriorityQueue<uint32_t, Req> pq(
        [&](const uint32_t& c) -> const dmc::ClientInfo* { return &ci[c]; },
        dmc::AtLimit::Wait, 0.0, opts);
    auto a = Clock::now();
    for (auto& o : pre) pq.add_request_time(Req{o.client}, o.client, dmc::ReqParams(1, 1), o.t, 1u);
    f_pre_s = std::chrono::duration<double>(Clock::now() - a).count();
    for (auto& o : ops) {
      auto t0 = Clock::now();
      pq.add_request_time(Req{o.client}, o.client, dmc::ReqParams(1, 1), o.t, 1u);
      auto t1 = Clock::now();
      auto pr = pq.pull_request(o.t);
      auto t2 = Clock::now();
      (void)pr;
      f_add.add(t0, t1);
      f_pull.add(t1, t2);
    }
  }

  {  // the engine's C-ABI, one call per operation
    dmc_queue_params p{};
    p.max_clients = N;
    p.ring_capacity = 64;
    p.max_batch = 1u << 16;
    p.at_limit = DMC_AT_LIMIT_WAIT;
    std::vector<dmc_queue*> qs(nq, nullptr);
    for (auto& q : qs)
      if (dmc_queue_create(&p, &q)) {
        std::fprintf(stderr, "dmc_queue_create failed\n");
        return 1;
      }
    std::vector<uint32_t> sl(N);
    std::vector<double> r(N), w(N), l(N);
    for (uint32_t c = 0; c < N; ++c) {
      sl[c] = c;
      r[c] = infos[c].r;
      w[c] = infos[c].w;
      l[c] = infos[c].l;
    }
    std::vector<dmc_request> rq(N);
    for (uint32_t c = 0; c < N; ++c) rq[c] = dmc_request{c, 1, pre[c].t, 1, 1, c};
    for (auto q : qs) {
      dmc_client_register_batch(q, N, sl.data(), r.data(), w.data(), l.data(), 1);
      if (serve) dmc_queue_set_option(q, DMC_OPT_SERVE, 1);
      for (uint32_t a = 0; a < N; a += 1u << 16) {
        uint32_t n = std::min<uint32_t>(1u << 16, N - a);
        dmc_add_batch(q, n, rq.data() + a, nullptr);
      }
    }
    uint64_t h = N;
    dmc_decision d;
    dmc_pull_result res;
    uint32_t i = 0;
    for (auto& o : ops) {
      dmc_queue* q = qs[i++ % nq];
      dmc_request one{o.client, 1, o.t, 1, 1, h++};
      int32_t rc = 0;
      auto t0 = Clock::now();
      dmc_add_batch(q, 1, &one, &rc);
      auto t1 = Clock::now();
      dmc_pull_batch(q, o.t, 1, &d, &res);
      auto t2 = Clock::now();
      e_add.add(t0, t1);
      e_pull.add(t1, t2);
    }
    for (auto q : qs) {
      dmc_counters c{};
      dmc_queue_counters(q, &c, 0);
      if (nq > 1) std::fprintf(stderr, "queue: serve calls %llu launches %llu yields %llu\n",
                               (unsigned long long)c.serve_calls,
                               (unsigned long long)c.serve_launches,
                               (unsigned long long)c.serve_yields);
      dmc_queue_destroy(q);
    }
  }

  if (oracle) {
    void* q = dmo_queue_create(0, 0, 2, DMC_AT_LIMIT_WAIT, 0.0, 0.0);
    // bulk registration of active clients, as the engine leg (a first add of
    // an idle client costs the reference an O(N) scan for the idle reset,
    // :937-985, which would dominate the pre-population at large N)
    std::vector<uint32_t> sl(N);
    std::vector<double> r(N), w(N), l(N);
    for (uint32_t c = 0; c < N; ++c) {
      sl[c] = c;
      r[c] = infos[c].r;
      w[c] = infos[c].w;
      l[c] = infos[c].l;
    }
    dmo_register_active_batch(q, N, sl.data(), r.data(), w.data(), l.data());
    auto a = Clock::now();
    for (uint32_t c = 0; c < N; ++c) dmo_add(q, c, c, 1, 1, pre[c].t, 1);
    o_pre_s = std::chrono::duration<double>(Clock::now() - a).count();
    uint64_t h = N;
    dmc_decision d;
    double when;
    for (auto& o : ops) {
      auto t0 = Clock::now();
      dmo_add(q, h++, o.client, 1, 1, o.t, 1);
      auto t1 = Clock::now();
      dmo_pull(q, o.t, &d, &when);
      auto t2 = Clock::now();
      o_add.add(t0, t1);
      o_pull.add(t1, t2);
    }
    dmo_queue_destroy(q);
  }

  std::printf("{\"serve\": %s, \"queues\": %u, \"clients\": %u, \"rounds\": %u, \"facade_prepop_s\": %.3f, "
              "\"oracle_prepop_s\": %.3f, \"facade_add_us\": %s, \"facade_pull_us\": %s, "
              "\"engine_add_us\": %s, \"engine_pull_us\": %s, \"oracle_add_us\": %s, "
              "\"oracle_pull_us\": %s}\n",
              serve ? "true" : "false", nq, N, M, f_pre_s, o_pre_s, f_add.json().c_str(), f_pull.json().c_str(),
              e_add.json().c_str(), e_pull.json().c_str(), o_add.json().c_str(),
              o_pull.json().c_str());
  return 0;
}
