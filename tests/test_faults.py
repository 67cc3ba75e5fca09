"""Device failures surface as status codes, never as corrupted state
(the boundary's contract, include/dmclock_gpu.h).

DMC_OPT_FAIL_ALLOC (a test hook) makes a queue's next device allocations
fail as an exhausted device would.  Each call that needs one -- a radix
round's dense-entry growth, an add batch's buffers, an activation batch's
buffers, the host-API decision buffer -- must return DMC_ENOMEM before it
launches anything, and the same call retried must then give exactly what the
oracle gives for the whole trace (reference: dmclock_server.h:1115-1186,
:913-1018).
"""
import numpy as np
import pytest

import pyoracle
from dmclock_amd import workloads
from dmclock_amd._abi import OPT_FAIL_ALLOC, OPT_FORCE_RADIX
from parity import compare_decisions, compare_states

pytestmark = pytest.mark.gpu


def _expect_enomem(fn):
    from dmclock_amd.gpu import DmcError
    with pytest.raises(DmcError) as e:
        fn()
    assert "(-2)" in str(e.value), str(e.value)


def test_failed_growth_returns_enomem_and_retry_is_exact():
    from dmclock_amd.gpu import GpuQueue
    n = 8192
    tr = workloads.config3_trace(5, n, 3, 4096, depth=16)
    qo = pyoracle.OracleQueue()
    outs_o = workloads.replay(qo, tr)
    assert qo.ties == 0
    k = tr.ops[1][2]
    qg = GpuQueue(max_clients=n, ring_capacity=64, max_batch=k)
    c = tr.clients
    qg.register(c.slots, c.r, c.w, c.l, c.active)
    pre = tr.ops[0][1]
    # the pre-population (twice max_batch) needs the add buffers grown
    qg.set_option(OPT_FAIL_ALLOC, 1)
    _expect_enomem(lambda: qg.add_batch(pre))
    assert qg.request_count() == 0  # nothing was added
    rc = qg.add_batch(pre)
    assert np.array_equal(rc, outs_o[0][1])
    # the settle pull on the radix path: its first round overflows the
    # dense buffer (65,536 entries), whose growth fails -- twice
    qg.set_option(OPT_FORCE_RADIX, 1)
    now = tr.ops[1][1]
    qg.set_option(OPT_FAIL_ALLOC, 2)
    _expect_enomem(lambda: qg.pull_batch(now, k))
    _expect_enomem(lambda: qg.pull_batch(now, k))
    assert qg.request_count() == len(pre)  # nothing was dispatched
    d, res = qg.pull_batch(now, k)
    compare_decisions(d, outs_o[1][1], "settle")
    assert (res.n_decisions, res.next_type) == outs_o[1][2][:2]
    ctr = qg.counters()
    assert ctr["radix_rounds"] >= 1 and ctr["dense_overflows"] >= 1, ctr
    qg.set_option(OPT_FORCE_RADIX, 0)
    for i, op in enumerate(tr.ops[2:], start=2):
        if op[0] == "add":
            assert np.array_equal(qg.add_batch(op[1]), outs_o[i][1]), i
        else:
            d, res = qg.pull_batch(op[1], op[2])
            compare_decisions(d, outs_o[i][1], f"op {i}")
    compare_states(qg, qo, np.arange(0, n, 7), "final")
    assert qg.request_count() == qo.request_count()
    qg.close()


def test_failed_activation_buffers_return_enomem():
    """an add batch with idle clients needs the activation buffers: their
    allocation fails, nothing is added, the retry is exact"""
    from dmclock_amd.gpu import GpuQueue
    tr = workloads.churn_trace(21, 2000, 3, 500, 400)
    qo = pyoracle.OracleQueue()
    outs_o = workloads.replay(qo, tr)
    qg = GpuQueue(max_clients=2000, ring_capacity=64, max_batch=4096)
    c = tr.clients
    qg.register(c.slots, c.r, c.w, c.l, c.active)
    failed = False
    for i, op in enumerate(tr.ops):
        if op[0] == "add":
            if not failed and i > 1:
                qg.set_option(OPT_FAIL_ALLOC, 1)
                try:
                    qg.add_batch(op[1])
                    qg.set_option(OPT_FAIL_ALLOC, 0)  # (nothing needed allocating)
                    raise AssertionError("expected the activation buffers to fail")
                except Exception as e:  # noqa: BLE001
                    assert "(-2)" in str(e), str(e)
                failed = True
                assert qg.request_count() == qo_count_before(outs_o, i, tr)
            assert np.array_equal(qg.add_batch(op[1]), outs_o[i][1]), i
        elif op[0] == "pull":
            d, res = qg.pull_batch(op[1], op[2])
            compare_decisions(d, outs_o[i][1], f"op {i}")
        elif op[0] == "idle":
            qg.mark_idle_batch(op[1])
    assert failed
    compare_states(qg, qo, np.arange(2000), "final")
    qg.close()


def qo_count_before(outs_o, i, tr):
    """requests queued in the oracle's replay just before op i"""
    q = pyoracle.OracleQueue()
    c = tr.clients
    q.register(c.slots, c.r, c.w, c.l, c.active)
    for op in tr.ops[:i]:
        if op[0] == "add":
            q.add_batch(op[1])
        elif op[0] == "pull":
            q.pull_batch(op[1], op[2])
        elif op[0] == "idle":
            for s in op[1].tolist():
                q.mark_idle(s)
    n = q.request_count()
    q.close()
    return n
