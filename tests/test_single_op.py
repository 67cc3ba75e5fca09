"""The single-op path (DMC_OPT_SINGLE_OP): host-API adds of one request of a
non-idle client (one kernel, k_add_one) and pulls of k <= 8 (two kernels per
pull_request, k_fast_decide / k_fast_apply, results in host-mapped memory)
-- the facade's per-call path -- against the oracle, the serve path
(DMC_OPT_SERVE: the same calls answered by the persistent k_serve from
per-group summaries) and the general step path (option off) on the same
traces.  Modes as the reference's
do_next_request branches (dmclock_server.h:1115-1200): AtLimit::Wait,
AtLimit::Allow (limit breaks), delayed tags, non-monotone `now`."""
import numpy as np
import pytest

from dmclock_amd import workloads
from dmclock_amd._abi import (AT_LIMIT_ALLOW, AT_LIMIT_REJECT, AT_LIMIT_WAIT, OPT_SERVE,
                              OPT_SINGLE_OP)
from parity import run_parity

pytestmark = pytest.mark.gpu

MODES = [dict(at_limit=AT_LIMIT_WAIT), dict(at_limit=AT_LIMIT_WAIT, delayed=True),
         dict(at_limit=AT_LIMIT_ALLOW)]


def _mk(single_op):
    def mk(**kw):
        from dmclock_amd.gpu import GpuQueue
        q = GpuQueue(ring_capacity=64, **kw)
        q.set_option(OPT_SINGLE_OP, int(bool(single_op)))
        q.set_option(OPT_SERVE, int(single_op == "serve"))
        return q
    return mk


def _single_add_trace(seed, n, steps, delta_rho="random", table_kw=None):
    """adds one request per op (the facade's add_request) between pulls of
    k in 1..8 at sometimes decreasing `now`"""
    base = workloads.steady_trace(seed, n, steps, 24, 0, depth=2, delta_rho=delta_rho,
                                  k_choices=[1, 2, 3, 5, 8], table_kw=table_kw)
    return _singles(base, seed)


def _singles(base, seed):
    """the trace's small add batches as single adds, its pulls at sometimes
    decreasing `now`; other ops (idle marking) kept"""
    rng = np.random.default_rng(seed)
    tr = workloads.Trace(base.clients, params=base.params)
    for op in base.ops:
        if op[0] == "add" and len(op[1]) <= 64:
            for i in range(len(op[1])):
                tr.ops.append(("add", op[1][i:i + 1].copy()))
        elif op[0] == "pull":
            now = op[1] - (0.3 if rng.random() < 0.2 else 0.0)  # non-monotone
            tr.ops.append(("pull", now, op[2]))
        else:
            tr.ops.append(op)
    return tr


@pytest.mark.parametrize("single_op", ["serve", True, False])
@pytest.mark.parametrize("mode", range(len(MODES)))
def test_single_op_parity(mode, single_op):
    tr = _single_add_trace(3 + mode, 512, 80)
    n, qg, qo = run_parity(tr, _mk(single_op), queue_kw=MODES[mode], state_sample=512)
    assert n > 250, n
    c = qg.counters()
    assert c["rounds"] == 0 and c["single_steps"] >= n, c
    if single_op == "serve":
        assert c["serve_calls"] > 500 and c["serve_launches"] >= 1, c
    qg.close()


@pytest.mark.parametrize("mode", range(len(MODES)))
def test_serve_many_groups(mode):
    """k_serve over 300,000 slots: 293 group summaries (the last one partial),
    the limit scan's marks re-summarising only the stale groups; a run of
    single adds and pulls between the trace's batch adds (each batch call
    stops k_serve; the next single call rebuilds the summaries and
    relaunches it)"""
    tr = _single_add_trace(11 + mode, 300_000, 40)
    n, qg, qo = run_parity(tr, _mk("serve"), queue_kw=MODES[mode], state_sample=4096)
    assert n > 100, n
    c = qg.counters()
    assert c["serve_calls"] > 300 and c["serve_launches"] >= 1, c
    qg.close()


def test_serve_concurrent_queues():
    """six queues on the serve path driven from six host threads at once:
    more k_serve kernels than the process's hardware queues (4), so some
    wait behind others; each one's lifetime lets them through.  Every add
    status and decision of every queue against the oracle."""
    import threading

    import pyoracle
    from parity import compare_decisions
    traces = [_single_add_trace(21 + i, 2000, 30) for i in range(6)]
    want = []
    for tr in traces:
        qo = pyoracle.OracleQueue(**MODES[0])
        want.append(workloads.replay(qo, tr))
        assert qo.ties == 0
    qs = [_mk("serve")(max_clients=2000, **MODES[0]) for _ in traces]
    got, errs = [None] * len(qs), []

    def drive(i):
        try:
            got[i] = workloads.replay(qs[i], traces[i])
        except Exception as e:  # noqa: BLE001 (reported below)
            errs.append(e)

    th = [threading.Thread(target=drive, args=(i,)) for i in range(len(qs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for i, (g, w) in enumerate(zip(got, want)):
        assert len(g) == len(w)
        for j, (a, b) in enumerate(zip(g, w)):
            assert a[0] == b[0]
            if a[0] == "add":
                assert np.array_equal(a[1], b[1]), (i, j)
            elif a[0] == "pull":
                compare_decisions(a[1], b[1], f"queue {i} op {j}")
                assert a[2] == b[2], (i, j, a[2], b[2])
        c = qs[i].counters()
        assert c["serve_calls"] > 500, c
        qs[i].close()


@pytest.mark.timeout(300)
def test_serve_1m_clients():
    """the serve path at the latency benchmark's size: 1,048,576 clients
    (1,024 group summaries of 1,024 slots), 2M pre-populated requests, then
    single adds and pulls with sometimes decreasing `now`; every decision,
    status and sampled state against the oracle"""
    tr = _single_add_trace(31, 1 << 20, 60)
    n, qg, qo = run_parity(tr, _mk("serve"), queue_kw=MODES[0], state_sample=4096)
    assert n > 100, n
    c = qg.counters()
    assert c["serve_calls"] > 1000, c
    qg.close()


def test_serve_reject_parity():
    """AtLimit::Reject on the serve path: tenants limited below
    their arrival rate, so single adds are rejected with EAGAIN (the
    request's prev tag still advances, :899-906, and the group summary is
    unchanged); every status, decision and sampled state against the
    oracle, with the serve kernel answering every single call"""
    kw = dict(at_limit=AT_LIMIT_REJECT)
    tr = _single_add_trace(41, 512, 80, table_kw=dict(frac_l=0.6, l_range=(0.3, 1.5)))
    n, qg, qo = run_parity(tr, _mk("serve"), queue_kw=kw, state_sample=512)
    assert n > 150, n
    c = qg.counters()
    assert c["serve_calls"] > 500 and c["rounds"] == 0, c
    rejected = sum(int((o[1] != 0).sum()) for o in workloads.replay(
        __import__("pyoracle").OracleQueue(**kw), tr) if o[0] == "add")
    assert rejected > 50, rejected
    qg.close()


@pytest.mark.parametrize("mode", [0, 2])
def test_serve_idle_transitions_parity(mode):
    """Switching between the serve path and its fallbacks inside one trace
    (ADVICE r3): clients marked idle between steps, then single adds that
    mix idle clients (the general add path with its activation: k_serve
    stopped, the summaries rebuilt at the next serve call) and non-idle ones
    (served), and single pulls; every decision, status and state against the
    oracle"""
    base = workloads.churn_trace(51 + mode, 600, 40, 20, 0, idle_frac=0.05,
                                 k_choices=[1, 2, 3, 5, 8])
    tr = _singles(base, 51 + mode)
    n, qg, qo = run_parity(tr, _mk("serve"), queue_kw=MODES[mode], state_sample=600)
    assert n > 100, n
    c = qg.counters()
    assert c["serve_calls"] > 300 and c["serve_launches"] >= 10, c
    qg.close()


def test_serve_queues_one_thread_yield():
    """More serving queues than the process's hardware queues, driven
    round-robin from ONE thread: a queue's call first stops the
    other queues' idle k_serve, so no call waits behind another queue's
    kernel (its idle timeout).  Every decision against the oracle, the
    yields counted, and the per-call time bounded far below the idle
    timeout's 0.2 ms plus lifetime."""
    import time

    import pyoracle
    from parity import compare_decisions
    nq = 6
    traces = [_single_add_trace(61 + i, 1000, 20) for i in range(nq)]
    want = []
    for tr in traces:
        qo = pyoracle.OracleQueue(**MODES[0])
        want.append(workloads.replay(qo, tr))
    qs = [_mk("serve")(max_clients=1000, **MODES[0]) for _ in traces]
    c0 = [tr.clients for tr in traces]
    for q, c in zip(qs, c0):
        q.register(c.slots, c.r, c.w, c.l, c.active)
    got = [[] for _ in qs]
    ops = [tr.ops for tr in traces]
    lat = []
    for j in range(max(len(o) for o in ops)):
        for i, q in enumerate(qs):
            if j >= len(ops[i]):
                continue
            op = ops[i][j]
            t0 = time.perf_counter()
            if op[0] == "add":
                got[i].append(("add", q.add_batch(op[1])))
            else:
                d, res = q.pull_batch(op[1], op[2])
                got[i].append(("pull", d, (res.n_decisions, res.next_type,
                                           res.when if res.next_type == 1 else 0.0)))
            if j > 4:
                lat.append(time.perf_counter() - t0)
    for i in range(nq):
        for j, (a, b) in enumerate(zip(got[i], want[i])):
            assert a[0] == b[0]
            if a[0] == "add":
                assert np.array_equal(a[1], b[1]), (i, j)
            else:
                compare_decisions(a[1], b[1], f"queue {i} op {j}")
                assert a[2] == b[2], (i, j, a[2], b[2])
    yields = sum(q.counters()["serve_yields"] for q in qs)
    assert yields > 100, yields
    lat.sort()
    p50, p99 = lat[len(lat) // 2], lat[len(lat) * 99 // 100]
    print(f"one thread, {nq} serving queues: p50 {p50 * 1e6:.1f} us, p99 {p99 * 1e6:.1f} us")
    assert p50 < 150e-6, (p50, p99)
    for q in qs:
        q.close()
