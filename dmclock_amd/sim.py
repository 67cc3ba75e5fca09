"""Deterministic virtual-time equivalent of the reference simulator `dmc_sim`
(/root/reference/sim/src: test_dmclock_main.cc, sim_client.h, sim_server.h,
simulate.h, config.cc) driving any queue with this package's Python queue API
(register / add / pull; the HIP engine in production, the oracle in tests).

The reference simulator is wall-clock and thread-driven (sleeps, condition
variables, a PRNG seeded from system_clock: SURVEY.md finding 6) and its push
queue's sched-ahead timer never fires on time (finding 5), so a "replayed
trace" has to come from a driver like this one: the same model, events in
virtual time, one seeded PRNG, ties between simultaneous events broken by
insertion order.

Model (reference lines cited inline):
* INI config with the keys of config.cc:123-184 and the defaults of
  config.h:36-122 (`load_conf`).
* Client c of group g: after client_wait seconds issues client_total_ops
  requests, one every round(1e6 / iops_goal) us (sim_client.h:60-68), never
  more than client_outstanding_ops outstanding (:233-236: when blocked it
  issues as soon as a response arrives); each request goes to
  server_select(o) (simulate.h:408-438, alternating or random range) with
  ReqParams from its ServiceTracker<ServerId, OrigTracker> (:241-251) and
  cost client_req_cost; responses feed track_resp (:300-304).
* Server: PushPriorityQueue semantics on a pull queue: after every add, every
  completion and every sched-ahead timer one schedule_request
  (dmclock_server.h:1741-1755): if a thread can take work
  (inner queue size <= threads, sim_server.h:171-174) one
  pull_request(now); a returned request joins the inner queue, a future
  arms the timer (sched_at, :1787-1794; here it fires at `when`), none does
  nothing.  A thread serves a request for round(threads * 1e6 / iops) us
  times its cost (sim_server.h:130-133, 222).  AtLimit::Allow iff
  server_soft_limit (test_dmclock_main.cc:191-194).
* Deviations (documented in DESIGN.md): clients are registered up front on
  every server (bulk registration, so no activation aligns proportion keys:
  SURVEY.md section 7), each client's start is offset by a small seeded
  jitter (identical clients issuing at identical instants tie in every tag),
  and times start at t0 = 1000 s: a client's first tags then come from its
  (jittered) arrival rather than from the zero prev tag plus an integer
  (w = 1 makes every later proportion tag that value plus an integer), so
  different clients' tags never coincide.
"""
import configparser
import heapq
from collections import deque
from dataclasses import dataclass, field

import numpy as np

from .tracker import ServiceTracker


@dataclass
class ClientGroup:  # config.h:36-71
    client_count: int = 100
    client_wait: int = 0
    client_total_ops: int = 1000
    client_server_select_range: int = 10
    client_iops_goal: int = 50
    client_outstanding_ops: int = 100
    client_reservation: float = 20.0
    client_limit: float = 60.0
    client_weight: float = 1.0
    client_req_cost: int = 1


@dataclass
class ServerGroup:  # config.h:89-100
    server_count: int = 100
    server_iops: int = 40
    server_threads: int = 1


@dataclass
class SimConfig:  # config.h:113-131
    server_groups: int = 1
    client_groups: int = 1
    server_random_selection: bool = False
    server_soft_limit: bool = True
    anticipation_timeout: float = 0.0
    cli_group: list = field(default_factory=list)
    srv_group: list = field(default_factory=list)


def _bool(v):  # config.cc stobool: "true"/"false" or a number
    v = v.strip().lower()
    return v == "true" or (v not in ("false",) and v.isdigit() and int(v) != 0)


def load_conf(path=None, text=None):
    """parse_config_file (config.cc:123-184)."""
    cp = configparser.ConfigParser(inline_comment_prefixes=(";", "#"))
    if text is not None:
        cp.read_string(text)
    else:
        with open(path) as f:
            cp.read_file(f)
    g = SimConfig()
    if cp.has_section("global"):
        s = cp["global"]
        g.server_groups = int(s.get("server_groups", g.server_groups))
        g.client_groups = int(s.get("client_groups", g.client_groups))
        if "server_random_selection" in s:
            g.server_random_selection = _bool(s["server_random_selection"])
        if "server_soft_limit" in s:
            g.server_soft_limit = _bool(s["server_soft_limit"])
        g.anticipation_timeout = float(s.get("anticipation_timeout",
                                             g.anticipation_timeout))
    for i in range(g.server_groups):
        st = ServerGroup()
        sec = f"server.{i}"
        if cp.has_section(sec):
            for k in ("server_count", "server_iops", "server_threads"):
                if k in cp[sec]:
                    setattr(st, k, int(cp[sec][k]))
        g.srv_group.append(st)
    for i in range(g.client_groups):
        ct = ClientGroup()
        sec = f"client.{i}"
        if cp.has_section(sec):
            for k, typ in (("client_count", int), ("client_wait", int),
                           ("client_total_ops", int),
                           ("client_server_select_range", int),
                           ("client_iops_goal", int),
                           ("client_outstanding_ops", int),
                           ("client_reservation", float), ("client_limit", float),
                           ("client_weight", float), ("client_req_cost", int)):
                if k in cp[sec]:
                    setattr(ct, k, typ(cp[sec][k]))
        g.cli_group.append(ct)
    return g


@dataclass
class _Client:
    group: int
    tracker: ServiceTracker
    ops_left: int
    max_out: int
    gap: float
    cost: int
    outstanding: int = 0
    blocked: bool = False
    o: int = 0  # next op index (server_select's seed)


@dataclass
class _Server:
    q: object
    threads: int
    op_time: float
    inner: deque = field(default_factory=deque)
    busy: int = 0
    timer: float = None


class Simulation:
    """One run of the model over `conf`; make_queue(at_limit, anticipation)
    builds each server's queue."""

    def __init__(self, conf, make_queue, seed=42, t0=1000.0, jitter=1e-3,
                 ops_per_client=None):
        self.conf = conf
        self.rng = np.random.default_rng(seed)
        self.t0 = t0
        self.events = []
        self.seq = 0
        self.handle = 0
        at_limit = 1 if conf.server_soft_limit else 0
        # clients (test_dmclock_main.cc:63-112, 177-183)
        self.clients = []
        self.cinfo = []
        for gi, g in enumerate(conf.cli_group):
            for _ in range(g.client_count):
                ops = g.client_total_ops if ops_per_client is None else ops_per_client
                us = int(0.5 + 1.0 / g.client_iops_goal * 1000000)
                self.clients.append(_Client(gi, ServiceTracker("orig"), ops,
                                            g.client_outstanding_ops, us * 1e-6,
                                            g.client_req_cost))
                self.cinfo.append((g.client_reservation, g.client_weight,
                                   g.client_limit))
        n = len(self.clients)
        r = np.array([c[0] for c in self.cinfo])
        w = np.array([c[1] for c in self.cinfo])
        l = np.array([c[2] for c in self.cinfo])
        # servers (sim_server.h:120-133)
        self.servers = []
        for sg in conf.srv_group:
            for _ in range(sg.server_count):
                q = make_queue(at_limit, conf.anticipation_timeout)
                q.register(np.arange(n, dtype=np.uint32), r, w, l, True)
                op_us = int(0.5 + sg.server_threads * 1000000.0 / sg.server_iops)
                self.servers.append(_Server(q, sg.server_threads, op_us * 1e-6))
        self.log_dec = [[] for _ in self.servers]   # per server: decisions
        self.log_req = []                            # (t, client, server, d, r)
        self.log_stop = [[] for _ in self.servers]   # (t, type, when)
        for ci, c in enumerate(self.clients):
            g = conf.cli_group[c.group]
            start = t0 + g.client_wait + float(self.rng.uniform(0.0, jitter))
            self._push(start, 0, ci)

    # ---- events: (time, seq, kind, arg); kinds 0 issue, 1 done, 2 timer, 3 resp
    def _push(self, t, kind, arg):
        heapq.heappush(self.events, (t, self.seq, kind, arg))
        self.seq += 1

    def _select(self, ci, o):
        """make_server_select_{alt,ran}_range (simulate.h:408-438)."""
        g = self.conf.cli_group[self.clients[ci].group]
        ns, nc = len(self.servers), len(self.clients)
        factor = ns / nc
        per = g.client_server_select_range
        off = (int(self.rng.integers(0, 1 << 62)) if self.conf.server_random_selection
               else o) % per
        return (int(0.5 + ci * factor) + off) % ns

    def _issue(self, t, ci):
        c = self.clients[ci]
        s = self._select(ci, c.o)
        d, r = c.tracker.get_req_params(s)
        self.log_req.append((t, ci, s, d, r))
        self.handle += 1
        srv = self.servers[s]
        rc = srv.q.add(ci, t, delta=d, rho=r, cost=c.cost, handle=self.handle)
        c.o += 1
        c.ops_left -= 1
        c.outstanding += 1
        if rc == 0:
            self._schedule(t, s)
        else:  # rejected: treat as an immediate empty response
            c.outstanding -= 1
        if c.ops_left > 0:
            self._push(t + c.gap, 0, ci)

    def _schedule(self, t, s):
        """schedule_request (dmclock_server.h:1741-1755)."""
        srv = self.servers[s]
        if len(srv.inner) > srv.threads:  # has_avail_thread (sim_server.h:171-174)
            return
        typ, rec, when = srv.q.pull(t)
        if typ == 0:
            self.log_dec[s].append((t, rec))
            srv.inner.append((int(rec["slot"]), int(rec["phase"]), int(rec["cost"])))
            self._start(t, s)
        else:
            self.log_stop[s].append((t, typ, when))
            if typ == 1 and when > t and (srv.timer is None or when < srv.timer):
                srv.timer = when  # sched_at (:1787-1794)
                self._push(when, 2, s)

    def _start(self, t, s):
        srv = self.servers[s]
        while srv.busy < srv.threads and srv.inner:
            ci, ph, cost = srv.inner.popleft()
            srv.busy += 1
            self._push(t + srv.op_time * cost, 1, (s, ci, ph, cost))

    def run(self, max_events=None):
        n = 0
        while self.events:
            t, _, kind, arg = heapq.heappop(self.events)
            n += 1
            if max_events is not None and n > max_events:
                raise RuntimeError("simulation did not finish")
            if kind == 0:
                c = self.clients[arg]
                if c.outstanding >= c.max_out:
                    c.blocked = True
                else:
                    self._issue(t, arg)
            elif kind == 1:  # a server thread finished (sim_server.h:209-235)
                s, ci, ph, cost = arg
                srv = self.servers[s]
                srv.busy -= 1
                self._schedule(t, s)  # request_completed (:1651-1660)
                self._start(t, s)
                self._push(t, 3, (ci, s, ph, cost))
            elif kind == 2:
                srv = self.servers[arg]
                if srv.timer == t:
                    srv.timer = None
                    self._schedule(t, arg)
            else:  # the client's response thread (sim_client.h:286-318)
                ci, s, ph, cost = arg
                c = self.clients[ci]
                c.tracker.track_resp(s, ph, cost)
                c.outstanding -= 1
                if c.blocked and c.ops_left > 0:
                    c.blocked = False
                    self._issue(t, ci)
        self.end_time = t if n else self.t0
        return self

    def stats(self):
        """per-client reservation / priority op counts (test_dmclock_main.cc
        client_data) and per-server decision counts"""
        nc = len(self.clients)
        res = np.zeros(nc, np.int64)
        prio = np.zeros(nc, np.int64)
        per_server = []
        for lg in self.log_dec:
            r = p = 0
            for _, rec in lg:
                if int(rec["phase"]) == 0:
                    res[int(rec["slot"])] += 1
                    r += 1
                else:
                    prio[int(rec["slot"])] += 1
                    p += 1
            per_server.append((r, p))
        return {"reservation_ops": res, "priority_ops": prio,
                "server_ops": per_server, "end_time": self.end_time,
                "requests": len(self.log_req)}


def main(argv=None):
    """`python -m dmclock_amd.sim -c sim/dmc_sim_100th.conf`: the dmc_sim
    equivalent on the HIP engine (one queue per server on one GPU)."""
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("-c", "--conf", required=True)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--ops", type=int, default=None,
                    help="ops per client (default: the conf's client_total_ops)")
    a = ap.parse_args(argv)
    from .gpu import GpuQueue
    conf = load_conf(a.conf)
    ncl = sum(g.client_count for g in conf.cli_group)

    def mk(at_limit, antic):
        return GpuQueue(max_clients=ncl, ring_capacity=64, max_batch=1024,
                        at_limit=at_limit, anticipation=antic)

    sim = Simulation(conf, mk, seed=a.seed, ops_per_client=a.ops).run()
    st = sim.stats()
    print(f"clients {ncl} servers {len(sim.servers)} requests {st['requests']} "
          f"virtual end time {st['end_time'] - sim.t0:.3f} s")
    print(f"reservation ops {int(st['reservation_ops'].sum())} "
          f"priority ops {int(st['priority_ops'].sum())}")
    for ci in list(range(min(3, ncl))) + list(range(max(3, ncl - 3), ncl)):
        print(f"client {ci}: res {int(st['reservation_ops'][ci])} "
              f"prop {int(st['priority_ops'][ci])}")


if __name__ == "__main__":
    main()
