"""Tie-exact dispatch (DMC_OPT_HEAP_ORDER, csrc/dmc_heap.h; SURVEY.md 8(a)
row A11): the reference's three indirect heaps on the device, driven in the
reference's order, so that among equal keys the reference's heap top wins
(support/src/indirect_intrusive_heap.h:240-564, src/dmclock_server.h:722-797,
1046-1186).  Checked against the oracle, which restates the same heaps, on
traces built to tie -- where the default engine (lowest slot wins) provably
diverges -- with every decision (client, phase, cost, handle, tag bits),
status and client state bit-exact (needs an MI355X)."""
import numpy as np
import pytest

import kats
import pyoracle
from dmclock_amd import sim, workloads
from dmclock_amd._abi import AT_LIMIT_ALLOW, AT_LIMIT_REJECT, AT_LIMIT_WAIT
from parity import run_parity

pytestmark = pytest.mark.gpu


def mk_heap(branching=2):
    def mk(**kw):
        from dmclock_amd.gpu import GpuQueue
        kw.setdefault("max_clients", 256)
        kw.setdefault("ring_capacity", 64)
        kw.setdefault("branching", branching)
        return GpuQueue(heap_order=True, **kw)
    return mk


@pytest.mark.parametrize("kat", kats.SERVER_KATS, ids=lambda f: f.__name__)
def test_server_kats_heap_order(kat):
    """the reference's server KATs (test_dmclock_server.cc) in heap order"""
    kat(mk_heap())


CONF_100TH = __import__("os").path.join(
    __import__("os").path.dirname(__import__("os").path.abspath(__file__)), "golden",
    "dmc_sim_100th.conf")


def _digest(s):
    dec = [[(t, int(r["slot"]), int(r["phase"]), int(r["cost"]), int(r["handle"]),
             float(r["tag_r"]), float(r["tag_p"]), float(r["tag_l"]))
            for t, r in lg] for lg in s.log_dec]
    return dec, list(s.log_req), [list(x) for x in s.log_stop]


@pytest.mark.timeout(600)
def test_config2_without_jitter_tie_exact():
    """BASELINE config 2 (dmc_sim_100th.conf) with the start jitter off:
    identical clients issue at identical instants, ~0.8 % of the decisions
    are ties, and with lowest-slot ties the per-server sequences drift apart
    (DESIGN.md section 4).  In heap order every server's whole dispatch
    sequence, every request's delta/rho and every future equal the
    oracle's (the reference's heaps) -- all 100,000 decisions."""
    from dmclock_amd.gpu import GpuQueue
    conf = sim.load_conf(CONF_100TH)
    ncl = sum(g.client_count for g in conf.cli_group)

    def ora(at_limit, antic):
        return pyoracle.OracleQueue(at_limit=at_limit, anticipation=antic)

    def gpu(at_limit, antic):
        return GpuQueue(max_clients=ncl, ring_capacity=64, max_batch=1024,
                        at_limit=at_limit, anticipation=antic, heap_order=True)

    o = sim.Simulation(conf, ora, seed=7, jitter=0.0).run(max_events=10_000_000)
    ties = sum(s.q.ties for s in o.servers)
    assert ties > 100, ties  # the trace does tie
    g = sim.Simulation(conf, gpu, seed=7, jitter=0.0).run(max_events=10_000_000)
    do, ro, so = _digest(o)
    dg, rg, sg = _digest(g)
    assert rg == ro
    for s in range(len(do)):
        assert dg[s] == do[s], f"server {s}"
    assert sg == so
    assert sum(len(x) for x in dg) == 100_000
    print(f"config 2 without jitter: {ties} tied decisions, every one the reference's")


MODES = [dict(at_limit=AT_LIMIT_WAIT), dict(at_limit=AT_LIMIT_WAIT, delayed=True),
         dict(at_limit=AT_LIMIT_ALLOW), dict(at_limit=AT_LIMIT_REJECT, reject_threshold=0.5),
         dict(at_limit=AT_LIMIT_WAIT, branching=3), dict(at_limit=AT_LIMIT_WAIT, branching=4)]


@pytest.mark.parametrize("mode", MODES, ids=lambda m: "-".join(f"{k}={v}" for k, v in m.items()))
def test_epoch_time_ties_tie_exact(mode):
    """open loop at the reference's clock scale (t0 = 1.7e9 s, what
    get_time() returns: rounding collisions make equal tags), idle marking
    between steps (activations whose prop_delta aligns keys exactly,
    :957-985), random delta/rho, pulls of k in 1..128: every decision,
    status and client state equal to the oracle's (the reference's heaps)"""
    rng = np.random.default_rng(5)
    tr = workloads.churn_trace(5, 700, 160, 150, 0, idle_frac=0.05, t0=1.7e9,
                               k_choices=[1, 3, 17, 64, 128])
    if mode.get("at_limit") == AT_LIMIT_REJECT:
        tr.clients.l = np.where(rng.random(700) < 0.5, rng.uniform(0.3, 1.5, 700), 0.0)
    n, qg, qo = run_parity(tr, mk_heap(mode.get("branching", 2)), queue_kw=mode,
                           state_sample=700, require_tie_free=False)
    assert n > 1000, n
    assert qo.ties > 0, "the trace should tie"
    qg.close()


@pytest.mark.timeout(900)
def test_heap_order_1m_clients_epoch_time():
    """A11 at scale: BASELINE config 3 at 1,048,576
    clients on the reference's clock scale (t0 = 1.7e9 s), in heap order:
    4,194,304 pre-populated requests, a 2,097,152-pull settle, then two
    steps of 65,536 adds + 65,536 pulls.  Every add status, every decision
    (client, phase, cost, handle, tag bits), every result and 4,096 sampled
    client states equal to the oracle's -- which replays the reference's
    heaps and counts the tied decisions: there are ties, and each went to
    the reference's heap top."""
    tr = workloads.config3_trace(42, 1 << 20, 2, 1 << 16, depth=4, t0=1.7e9)
    n, qg, qo = run_parity(tr, mk_heap(), state_sample=4096, require_tie_free=False,
                           gpu_kw=dict(max_batch=1 << 20))
    assert n > 2_000_000, n
    assert qo.ties > 0, qo.ties
    print(f"1M clients in heap order: {n} decisions, {qo.ties} tied, all the reference's")
    qg.close()


def _tie_trace(seed, n, steps, reject=False):
    """churn (idle marking between steps: activations, whose prop_delta
    aligns keys exactly, :957-985) with few distinct client rates and
    arrival times on a 1 ms grid, random delta/rho and pulls of k in 1..128:
    equal tags everywhere"""
    rng = np.random.default_rng(seed)
    tr = workloads.churn_trace(seed, n, steps, 150, 0, idle_frac=0.05,
                               k_choices=[1, 3, 17, 64, 128])
    c = tr.clients
    c.r = rng.choice([0.0, 4.0, 8.0], n)
    c.w = rng.choice([0.5, 1.0, 2.0], n)
    c.l = (rng.choice([0.0, 0.5, 1.0], n) if reject else
           rng.choice([0.0, 0.0, 16.0], n))
    ops = []
    for op in tr.ops:
        if op[0] == "add":
            r = op[1].copy()
            r["time"] = np.round(r["time"], 3)
            ops.append(("add", r))
        elif op[0] == "pull":
            ops.append(("pull", round(op[1], 3), op[2]))
        else:
            ops.append(op)
    tr.ops = ops
    return tr


@pytest.mark.parametrize("mode", MODES, ids=lambda m: "-".join(f"{k}={v}" for k, v in m.items()))
def test_tied_trace_tie_exact(mode):
    """a tie-heavy trace (_tie_trace): every decision, status and client
    state equal to the oracle's (the reference's heaps)"""
    tr = _tie_trace(5, 700, 60, reject=mode.get("at_limit") == AT_LIMIT_REJECT)
    n, qg, qo = run_parity(tr, mk_heap(mode.get("branching", 2)), queue_kw=mode,
                           state_sample=700, require_tie_free=False)
    assert n > 1000, n
    assert qo.ties > 50, qo.ties
    qg.close()


@pytest.mark.parametrize("ops", ["erase", "remove_by_client", "filter", "all"])
def test_maintenance_in_heap_order(ops):
    """erase (delete_from_heaps), remove_by_client and remove_by_req_filter
    (adjust x 3 per modified client) between tied pulls: the heaps stay the
    reference's"""
    from parity import compare_decisions
    rng = np.random.default_rng(8)
    tr = workloads.steady_trace(8, 300, 0, 0, 0, depth=4)
    c = tr.clients
    c.r = rng.choice([0.0, 4.0], 300)
    c.w = rng.choice([1.0, 2.0], 300)
    c.l = np.zeros(300)
    tr.ops[0][1]["time"] = np.round(tr.ops[0][1]["time"], 2)
    qo = pyoracle.OracleQueue()
    qg = mk_heap()(max_clients=300)
    for q in (qo, qg):
        q.register(c.slots, c.r, c.w, c.l, True)
        q.add_batch(tr.ops[0][1])
    t = float(tr.ops[0][1]["time"][-1])
    h = int(tr.ops[0][1]["handle"].max()) + 1
    gone = set()
    for step in range(12):
        kind = ["erase", "remove_by_client", "filter"][step % 3]
        if ops not in ("all", kind):
            kind = None
        if kind == "erase":
            gone |= {3 * step + 1, 3 * step + 2}
        for q in (qo, qg):
            if kind == "erase":
                for cl in (3 * step + 1, 3 * step + 2):
                    assert q.erase(cl)
            if kind == "remove_by_client":
                q.remove_by_client(5 * step, reverse=bool(step & 2))
            if kind == "filter":
                q.remove_by_req_filter(lambda hd: hd % 7 == step % 7, backwards=bool(step & 4))
        reqs = workloads.arrivals(rng, 300, 200, t, 600.0, handle_base=h)
        reqs["time"] = np.round(reqs["time"], 2)
        reqs = reqs[~np.isin(reqs["slot"], sorted(gone))]  # (no re-creation of erased clients)
        h += 200
        t = float(reqs["time"][-1]) if len(reqs) else t
        ro, rg = qo.add_batch(reqs), qg.add_batch(reqs)
        assert np.array_equal(ro, rg), step
        do, reso = qo.pull_batch(t, 150)
        dg, resg = qg.pull_batch(t, 150)
        compare_decisions(dg, do, f"step {step}")
        assert (reso.n_decisions, reso.next_type) == (resg.n_decisions, resg.next_type)
    assert qo.ties > 0
    qg.close()
