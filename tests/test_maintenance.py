"""Whole-queue maintenance on the device against the
oracle: remove_by_req_filter (dmclock_server.h:567-585, ClientRec
:440-480) as one handle readback (dmc_queue_requests), a host filter and one
device compaction pass (dmc_queue_filter); do_clean's erase (:1244-1255) of
many clients as one pass (dmc_client_erase_batch).

After each maintenance call the trace continues (adds and pulls) and every
decision, add status and sampled client state is compared bit for bit: a
removed delayed-mode front leaves the next request's stored tag as the front
(the reference's deque erase), the front's ready flag survives only with the
front, and the heap keys follow the new front.
"""
import time

import numpy as np
import pytest

import pyoracle
from dmclock_amd import workloads
from parity import compare_decisions, compare_states

pytestmark = pytest.mark.gpu


def _mk(n, **kw):
    from dmclock_amd.gpu import GpuQueue
    return GpuQueue(max_clients=n, ring_capacity=64, **kw)


def _pred(seed, mod):
    # a deterministic handle predicate (the same on both engines)
    return lambda h: ((h * 2654435761 + seed) >> 7) % mod == 0


def _replay_ops(qg, qo, ops):
    for i, op in enumerate(ops):
        if op[0] == "add":
            a, b = qg.add_batch(op[1]), qo.add_batch(op[1])
            assert np.array_equal(a, b), i
        elif op[0] == "pull":
            dg, rg = qg.pull_batch(op[1], op[2])
            do, ro = qo.pull_batch(op[1], op[2])
            compare_decisions(dg, do, f"op {i}")
            assert (rg.n_decisions, rg.next_type) == (ro.n_decisions, ro.next_type), i


@pytest.mark.parametrize("backwards", [False, True])
@pytest.mark.parametrize("delayed", [False, True])
def test_queue_filter_parity(delayed, backwards):
    """a 4096-client trace, a filter pass removing ~1/3 of the queued
    requests (fronts included), then more steps: bit-exact throughout"""
    tr = workloads.steady_trace(11, 4096, 6, 2048, 0, depth=4, delta_rho="random",
                                k_choices=[64, 512, 2048])
    kw = dict(delayed=delayed)
    qo = pyoracle.OracleQueue(**kw)
    qg = _mk(4096, **kw)
    c = tr.clients
    qo.register(c.slots, c.r, c.w, c.l, c.active)
    qg.register(c.slots, c.r, c.w, c.l, c.active)
    half = len(tr.ops) // 2
    _replay_ops(qg, qo, tr.ops[:half])
    n0 = qo.request_count()
    seen_g, seen_o = [], []
    base = _pred(3, 3)
    if delayed:
        # a removed delayed-mode front exposes its successor's placeholder tag
        # (0, 0, 0): every such client would tie at 0 (the reference's heap
        # order then decides, A11).  Fronts stay here; the single-client test
        # below removes one.
        counts, hs = qg.queue_requests()
        offs = np.concatenate([[0], np.cumsum(counts, dtype=np.int64)]).astype(np.int64)
        fronts = set(int(hs[offs[s]]) for s in range(4096) if counts[s])
        fg = fo = (lambda h: h not in fronts and base(h))
    else:
        fg = fo = base
    rg = qg.remove_by_req_filter(lambda h: seen_g.append(h) or fg(h), backwards)
    ro = qo.remove_by_req_filter(lambda h: seen_o.append(h) or fo(h), backwards)
    assert rg == ro is True
    assert seen_g == seen_o  # the visit order: clients ascending, FIFO or LIFO
    assert qg.request_count() == qo.request_count() < n0
    compare_states(qg, qo, range(4096), "after filter")
    _replay_ops(qg, qo, tr.ops[half:])
    compare_states(qg, qo, range(4096), "final")
    assert tuple(qg.sched_counts()) == tuple(qo.sched_counts())
    # a pass that removes nothing reports so and changes nothing
    assert qg.remove_by_req_filter(lambda h: False) is False
    qg.close()


@pytest.mark.parametrize("backwards", [False, True])
def test_filter_removes_delayed_front(backwards):
    """ClientRec::remove_by_req_filter on a delayed-mode front (:440-480):
    the successor keeps its stored placeholder tag as the front tag, exactly
    as the reference's deque erase leaves it; one client, so no tie."""
    qo = pyoracle.OracleQueue(delayed=True)
    qg = _mk(4, delayed=True)
    adds = [(1.0, 1, 1, 1, 10), (1.1, 2, 1, 2, 11), (1.2, 1, 0, 1, 12),
            (1.3, 1, 1, 3, 13), (1.4, 2, 2, 1, 14)]  # time, delta, rho, cost, handle
    for q in (qo, qg):
        q.set_info(1, 1.0, 1.0, 0.0)
        for t, d, r, c, h in adds:
            assert q.add(1, t, d, r, c, h) == 0
    pred = lambda h: h in (10, 12)
    assert qg.remove_by_req_filter(pred, backwards) == qo.remove_by_req_filter(pred, backwards)
    compare_states(qg, qo, [1], "after filter")
    for now in (5.0, 5.0, 5.0, 9.0, 9.0):
        tg, dg, wg = qg.pull(now)
        to, do, wo = qo.pull(now)
        assert tg == to and wg == wo, (now, tg, to)
        if dg is not None:
            for f in ("handle", "cost", "phase"):
                assert dg[f] == do[f], (f, dg, do)
            for f in ("tag_r", "tag_p", "tag_l"):
                assert np.float64(dg[f]).view(np.uint64) == np.float64(do[f]).view(np.uint64)
    compare_states(qg, qo, [1], "final")
    qg.close()


def test_erase_batch_parity():
    """dmc_client_erase_batch vs the oracle's per-client erase: handles,
    request counts and the following pulls"""
    tr = workloads.steady_trace(5, 2048, 3, 1024, 0, depth=3, k_choices=[256])
    qo = pyoracle.OracleQueue()
    qg = _mk(2048)
    c = tr.clients
    qo.register(c.slots, c.r, c.w, c.l, c.active)
    qg.register(c.slots, c.r, c.w, c.l, c.active)
    _replay_ops(qg, qo, tr.ops[:3])
    victims = sorted(np.random.default_rng(2).choice(2048, 300, replace=False).tolist())
    want = []
    for v in victims:
        want.extend(int(h) for h in qo.remove_by_client(v))
        assert qo.erase(v)
    got = qg.erase_batch(victims)
    assert got.tolist() == want
    assert qg.request_count() == qo.request_count()
    assert qg.client_count() == qo.client_count()
    _replay_ops(qg, qo, [op for op in tr.ops[3:] if op[0] == "pull"])
    qg.close()


def test_filter_pass_1m_clients_milliseconds():
    """A 1M-client filter pass (2M queued requests) through the C-ABI: one
    readback, a vectorised host predicate, one compaction -- milliseconds,
    not 2M synchronous calls.  Size-independent checks: the removed handles
    are exactly the predicate's, the survivors keep their per-client order,
    and no removed handle is dispatched afterwards."""
    import ctypes
    tr = workloads.config3_trace(42, 1 << 20, 0, 0, depth=2, settle=0)
    q = _mk(1 << 20, max_batch=1 << 21)
    c = tr.clients
    q.register(c.slots, c.r, c.w, c.l, c.active)
    q.add_batch(tr.ops[0][1])
    n_before = q.request_count()
    t0 = time.perf_counter()
    counts, hs = q.queue_requests()
    keep = ((hs * 2654435761 >> 7) % 5 != 0).astype(np.uint8)
    anyr = ctypes.c_int(0)
    rc = q.L.dmc_queue_filter(q.h, keep.ctypes.data_as(ctypes.c_void_p), len(keep),
                              ctypes.byref(anyr))
    dt = time.perf_counter() - t0
    assert rc == 0 and anyr.value == 1
    assert len(hs) == n_before == 2 * (1 << 20)
    counts2, hs2 = q.queue_requests()
    assert np.array_equal(hs2, hs[keep.astype(bool)])
    assert counts2.sum() == keep.sum()
    d, _ = q.pull_batch(1e9, 1 << 16)
    assert not np.isin(d["handle"], hs[~keep.astype(bool)]).any()
    print(f"1M-client filter pass: {len(hs)} handles, {dt * 1e3:.1f} ms")
    assert dt < 2.0, dt
    q.close()
