"""Deterministic synthetic dmClock traces (BASELINE.json configs 3-4 and the
parity-test traces).

A trace is a client table plus a list of operations, replayed identically on
the HIP engine and on the CPU restatement:
    ("add", reqs)            REQUEST_DTYPE array, in arrival order
    ("pull", now, k)         up to k pull_request(now)
    ("idle", slots)          do_clean's idle marking for these clients
    ("info", slot, r, w, l)  client_info_f changes + update_client_info
    ("bind", slots, r, w, l) client_info_f returns fresh ClientInfo objects for
                             these clients (seen under U1 at the next tag
                             calculation, dmclock_server.h:870-875)

Time base t0 = 1.0 s (epoch-scale times create rounding
ties between tags).  Client ids are slots.
"""
from dataclasses import dataclass, field

import numpy as np

from ._abi import REQUEST_DTYPE


@dataclass
class ClientTable:
    slots: np.ndarray
    r: np.ndarray
    w: np.ndarray
    l: np.ndarray
    active: bool = True


@dataclass
class Trace:
    clients: ClientTable
    ops: list = field(default_factory=list)
    params: dict = field(default_factory=dict)


def client_table(rng, n, frac_r=0.5, r_range=(1.0, 10.0), w_range=(0.5, 1.5),
                 frac_l=0.3, l_range=(5.0, 25.0), active=True):
    """Config 3 mix: r ~ U[1,10] for frac_r of clients (else 0);
    w ~ U[0.5,1.5]; l ~ U[5,25] for frac_l (else 0)."""
    slots = np.arange(n, dtype=np.uint32)
    r = np.where(rng.random(n) < frac_r, rng.uniform(*r_range, n), 0.0)
    w = rng.uniform(*w_range, n)
    l = np.where(rng.random(n) < frac_l, rng.uniform(*l_range, n), 0.0)
    return ClientTable(slots, r, w, l, active)


def arrivals(rng, n_clients, n, t_start, rate, costs=(1, 2, 3),
             delta_rho="ones", handle_base=0, clients=None):
    """n requests of a Poisson process of aggregate `rate` over uniformly
    chosen clients (or the given client subset)."""
    gaps = rng.exponential(1.0 / rate, n)
    times = t_start + np.cumsum(gaps)
    out = np.zeros(n, dtype=REQUEST_DTYPE)
    if clients is None:
        out["slot"] = rng.integers(0, n_clients, n, dtype=np.uint32)
    else:
        out["slot"] = rng.choice(clients, n)
    out["time"] = times
    out["cost"] = rng.choice(np.asarray(costs, dtype=np.uint32), n)
    if delta_rho == "ones":
        out["delta"] = 1
        out["rho"] = 1
    else:
        d = rng.integers(0, 4, n, dtype=np.uint32)
        out["delta"] = d
        out["rho"] = (rng.random(n) * (d + 1)).astype(np.uint32)
    out["handle"] = np.arange(handle_base, handle_base + n, dtype=np.uint64)
    return out


def steady_trace(seed, n_clients, n_steps, adds_per_step, pulls_per_step,
                 rate=None, depth=4, t0=1.0, delta_rho="ones", costs=(1, 2, 3),
                 table_kw=None, k_choices=None):
    """Config-3-style trace: bulk-registered active clients, a pre-population
    of `depth` requests per client, then steps of `adds_per_step` arrivals
    followed by pulls at the step's end time."""
    rng = np.random.default_rng(seed)
    tab = client_table(rng, n_clients, **(table_kw or {}))
    rate = rate or 2.0 * n_clients
    tr = Trace(tab, params=dict(seed=seed, n_clients=n_clients, rate=rate))
    handle = 0
    t = t0
    pre = depth * n_clients
    if pre:
        reqs = arrivals(rng, n_clients, pre, t, rate, costs, delta_rho, handle)
        handle += pre
        t = float(reqs["time"][-1])
        tr.ops.append(("add", reqs))
    for _ in range(n_steps):
        reqs = arrivals(rng, n_clients, adds_per_step, t, rate, costs,
                        delta_rho, handle)
        handle += adds_per_step
        t = float(reqs["time"][-1])
        tr.ops.append(("add", reqs))
        k = pulls_per_step if k_choices is None else int(rng.choice(k_choices))
        tr.ops.append(("pull", t, k))
    return tr


def churn_trace(seed, n_clients, n_steps, adds_per_step, pulls_per_step,
                idle_frac=0.1, rate=None, t0=1.0, delta_rho="random",
                k_choices=None):
    """Config-4-style trace: like steady_trace but each step marks a random
    fraction of clients idle first; their next request re-activates them
    through the idle reset (prop_delta = L - t, dmclock_server.h:937-985)."""
    rng = np.random.default_rng(seed)
    tr = steady_trace(seed, n_clients, 0, 0, 0, rate=rate, depth=2, t0=t0,
                      delta_rho=delta_rho)
    rate = tr.params["rate"]
    handle = 2 * n_clients
    t = float(tr.ops[-1][1]["time"][-1])
    for _ in range(n_steps):
        idle = rng.choice(n_clients, max(1, int(idle_frac * n_clients)),
                          replace=False).astype(np.uint32)
        tr.ops.append(("idle", np.sort(idle)))
        reqs = arrivals(rng, n_clients, adds_per_step, t, rate, (1, 2, 3),
                        delta_rho, handle)
        handle += adds_per_step
        t = float(reqs["time"][-1])
        tr.ops.append(("add", reqs))
        k = pulls_per_step if k_choices is None else int(rng.choice(k_choices))
        tr.ops.append(("pull", t, k))
    return tr


def config3_trace(seed, n_clients, n_steps, batch, depth=4, settle=None, t0=1.0):
    """bench.py's workload (BASELINE config 3) at any client count:
    bulk-registered clients in the config-3 mix, `depth` requests per client
    from a Poisson process of 2 req/s per client, a settle pull of depth/2 per
    client at the pre-population's end, then steps of `batch` adds + `batch`
    pulls at the step's last arrival."""
    rng = np.random.default_rng(seed)
    tab = client_table(rng, n_clients)
    rate = 2.0 * n_clients
    tr = Trace(tab, params=dict(seed=seed, config=3))
    pre = arrivals(rng, n_clients, depth * n_clients, t0, rate)
    t = float(pre["time"][-1])
    tr.ops.append(("add", pre))
    tr.ops.append(("pull", t, depth * n_clients // 2 if settle is None else settle))
    h = len(pre)
    for _ in range(n_steps):
        reqs = arrivals(rng, n_clients, batch, t, rate, handle_base=h)
        h += batch
        t = float(reqs["time"][-1])
        tr.ops.append(("add", reqs))
        tr.ops.append(("pull", t, batch))
    return tr


def config4_trace(seed, n_clients, n_steps, batch, depth=4, idle_frac=0.10,
                  throttled=0.10):
    """bench.py --config 4 (BASELINE config 4) at any client count: config 3
    plus `throttled` of the tenants limited below their arrival rate (l ~
    U[0.5, 1.5] against 2 req/s, AtLimit::Wait throttles them) and, before
    every step, do_clean's idle marking of `idle_frac` of all clients drawn
    from those without an arrival in the two previous steps (their next
    request re-activates them through the idle reset, :937-985)."""
    rng = np.random.default_rng(seed)
    tab = client_table(rng, n_clients)
    thr = rng.random(n_clients) < throttled
    tab.l = np.where(thr, rng.uniform(0.5, 1.5, n_clients), tab.l)
    rate = 2.0 * n_clients
    tr = Trace(tab, params=dict(seed=seed, config=4))
    pre = arrivals(rng, n_clients, depth * n_clients, 1.0, rate)
    t = float(pre["time"][-1])
    tr.ops.append(("add", pre))
    tr.ops.append(("pull", t, depth * n_clients // 2))
    h = len(pre)
    last = np.full(n_clients, -1, np.int64)
    for i in range(n_steps):
        quiet = np.flatnonzero(last < i - 2)
        m = min(len(quiet), int(idle_frac * n_clients))
        sel = np.sort(rng.choice(quiet, m, replace=False)).astype(np.uint32)
        tr.ops.append(("idle", sel))
        reqs = arrivals(rng, n_clients, batch, t, rate, handle_base=h)
        h += batch
        t = float(reqs["time"][-1])
        last[reqs["slot"]] = i
        tr.ops.append(("add", reqs))
        tr.ops.append(("pull", t, batch))
    return tr


def reject_churn_trace(seed, n_clients, n_steps, batch, idle_frac=0.3, throttled=0.4,
                       t0=1.0, delta_rho="random"):
    """AtLimit::Reject with activations: config 4's churn with `throttled` of
    the tenants limited far below their arrival rate (l ~ U[0.2, 1] against
    2 req/s, so their limit tags run ahead of the clock) and idle marking
    drawn from all clients: activating requests of throttled clients are
    rejected -- the idle reset still applies and prev moves
    (dmclock_server.h:937-993) -- and clients emptied by the pulls see
    rejected requests move their proportion basis before one is accepted.
    batch >= n_clients gives clients several requests per batch (a rejected
    activation followed by more requests: the host split); smaller batches
    mostly one."""
    rng = np.random.default_rng(seed)
    tab = client_table(rng, n_clients)
    thr = rng.random(n_clients) < throttled
    tab.l = np.where(thr, rng.uniform(0.2, 1.0, n_clients), tab.l)
    rate = 2.0 * n_clients
    tr = Trace(tab, params=dict(seed=seed, reject=True))
    pre = arrivals(rng, n_clients, 2 * n_clients, t0, rate, delta_rho=delta_rho)
    t = float(pre["time"][-1])
    tr.ops.append(("add", pre))
    tr.ops.append(("pull", t, n_clients))
    h = len(pre)
    for _ in range(n_steps):
        sel = rng.choice(n_clients, int(idle_frac * n_clients), replace=False)
        tr.ops.append(("idle", np.sort(sel).astype(np.uint32)))
        reqs = arrivals(rng, n_clients, batch, t, rate, delta_rho=delta_rho, handle_base=h)
        h += batch
        t = float(reqs["time"][-1])
        tr.ops.append(("add", reqs))
        tr.ops.append(("pull", t, batch))
    return tr


def dynamic_trace(seed, n_clients, n_steps, adds_per_step, change_frac=0.2,
                  k_choices=(1, 3, 16, 64, 256), depth=3):
    """U1 (dynamic client info) trace: steady_trace with random delta/rho and,
    before every pull, fresh ClientInfo for a random `change_frac` of the
    clients (ClientInfo re-read at every tag, reductions with the cached one)."""
    rng = np.random.default_rng(seed + 1000)
    base = steady_trace(seed, n_clients, n_steps, adds_per_step, 0, depth=depth,
                        delta_rho="random", k_choices=k_choices)
    tr = Trace(base.clients, params=dict(base.params, dynamic=True))
    for op in base.ops:
        if op[0] == "pull":
            m = max(1, int(change_frac * n_clients))
            sl = np.sort(rng.choice(n_clients, m, replace=False)).astype(np.uint32)
            t = client_table(rng, m)
            tr.ops.append(("bind", sl, t.r, t.w, t.l))
        tr.ops.append(op)
    return tr


def replay(q, trace, check=None):
    """Replay a trace on a queue exposing register/add_batch/pull_batch/
    mark_idle/set_info/update_client_info.  Yields per-op outputs."""
    c = trace.clients
    q.register(c.slots, c.r, c.w, c.l, c.active)
    outs = []
    for op in trace.ops:
        if op[0] == "add":
            outs.append(("add", q.add_batch(op[1])))
        elif op[0] == "pull":
            d, res = q.pull_batch(op[1], op[2])
            outs.append(("pull", d, (res.n_decisions, res.next_type,
                                     res.when if res.next_type == 1 else 0.0)))
        elif op[0] == "idle":
            if hasattr(q, "mark_idle_batch"):
                q.mark_idle_batch(op[1])
            else:
                for s in op[1].tolist():
                    q.mark_idle(s)
            outs.append(("idle", None))
        elif op[0] == "info":
            _, s, r, w, l = op
            q.set_info(s, r, w, l)
            q.update_client_info(s)
            outs.append(("info", None))
        elif op[0] == "bind":
            _, sl, r, w, l = op
            for i, s in enumerate(sl.tolist()):
                q.set_info(s, r[i], w[i], l[i], fresh=True)
            if getattr(q, "explicit_bind", False):
                q.bind_info(sl, r, w, l)  # dirty pushes instead of a callback
            outs.append(("bind", None))
        if check is not None:
            check(op, outs[-1])
    return outs
