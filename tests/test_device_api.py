"""The device-resident API (dmc_add_batch_device / dmc_pull_batch_device, the
path bench.py times) against the host API on the same trace: identical
decisions and add statuses, and the device result record
(n_decisions, next_type, when, n_reservation, n_priority) equal to the host
call's, with the phase counts equal to the decisions' phases.  The result is
written on the device by the round's last kernel when one round ends the
call, and by the host's view otherwise (overflow retries, AtLimit::Allow
steps, small-k steps): every path is exercised.
"""
import numpy as np
import pytest

from dmclock_amd import workloads
from dmclock_amd._abi import (AT_LIMIT_ALLOW, AT_LIMIT_WAIT, DECISION_DTYPE,
                              OPT_FORCE_RADIX, OPT_GRAPHS, OPT_SMALL_K, PullResult)

pytestmark = pytest.mark.gpu


def _mk(variant, **kw):
    from dmclock_amd.gpu import GpuQueue
    q = GpuQueue(max_clients=kw.pop("n"), ring_capacity=64, **kw)
    if variant == "radix":
        q.set_option(OPT_FORCE_RADIX, 1)
    elif variant == "steps":
        q.set_option(OPT_SMALL_K, 1 << 30)
    elif variant == "eager":
        q.set_option(OPT_GRAPHS, 0)
    return q


def _res(d_res):
    return PullResult.from_buffer_copy(d_res.cpu().numpy().tobytes())


def _check_pull(qh, now, k, d_out, d_res):
    dh, rh = qh.pull_batch(now, k)
    rd = _res(d_res)
    dd = d_out.cpu().numpy().view(DECISION_DTYPE)[:rd.n_decisions]
    assert (rd.n_decisions, rd.next_type) == (rh.n_decisions, rh.next_type)
    if rh.next_type == 1:
        assert rd.when == rh.when
    assert np.array_equal(dd, dh)
    n_res = int((dh["phase"] == 0).sum())
    assert (rd.n_reservation, rd.n_priority) == (n_res, len(dh) - n_res)
    assert (rh.n_reservation, rh.n_priority) == (n_res, len(dh) - n_res)
    return rd.next_type


@pytest.mark.parametrize("api", ["separate", "fused"])
@pytest.mark.parametrize("variant", ["default", "radix", "steps", "eager"])
@pytest.mark.parametrize("at_limit", [AT_LIMIT_WAIT, AT_LIMIT_ALLOW],
                         ids=["wait", "allow"])
def test_device_api_matches_host_api(variant, at_limit, api):
    import torch
    n = 400
    tr = workloads.steady_trace(7, n, 10, 300, 0, depth=2, delta_rho="random",
                                k_choices=(1, 5, 40, 300, 900, 5000))
    qh = _mk(variant, n=n, at_limit=at_limit)
    qd = _mk(variant, n=n, at_limit=at_limit)
    c = tr.clients
    for q in (qh, qd):
        q.register(c.slots, c.r, c.w, c.l, c.active)
    dev = torch.device("cuda", 0)
    kinds = set()
    ops = list(tr.ops)
    i = 0
    while i < len(ops):
        op = ops[i]
        if op[0] == "add":
            reqs = op[1]
            rc_h = qh.add_batch(reqs)
            d_reqs = torch.from_numpy(reqs.view(np.uint8).copy()).to(dev)
            d_rc = torch.full((len(reqs),), -7, dtype=torch.int32, device=dev)
            if api == "fused" and i + 1 < len(ops) and ops[i + 1][0] == "pull":
                _, now, k = ops[i + 1]
                d_out = torch.zeros(max(k, 1) * DECISION_DTYPE.itemsize,
                                    dtype=torch.uint8, device=dev)
                d_res = torch.full((24,), 0xAB, dtype=torch.uint8, device=dev)
                qd.add_pull_batch_device(d_reqs.data_ptr(), len(reqs), d_rc.data_ptr(),
                                         now, k, d_out.data_ptr(), d_res.data_ptr())
                qd.sync()
                assert np.array_equal(d_rc.cpu().numpy(), rc_h)
                kinds.add(_check_pull(qh, now, k, d_out, d_res))
                i += 2
                continue
            qd.add_batch_device(d_reqs.data_ptr(), len(reqs), d_rc.data_ptr())
            qd.sync()
            assert np.array_equal(d_rc.cpu().numpy(), rc_h)
            i += 1
            continue
        _, now, k = op
        d_out = torch.zeros(max(k, 1) * DECISION_DTYPE.itemsize, dtype=torch.uint8,
                            device=dev)
        d_res = torch.full((24,), 0xAB, dtype=torch.uint8, device=dev)
        qd.pull_batch_device(now, k, d_out.data_ptr(), d_res.data_ptr())
        qd.sync()
        kinds.add(_check_pull(qh, now, k, d_out, d_res))
        i += 1
    assert 0 in kinds  # some pulls returned k decisions


@pytest.mark.parametrize("api", ["separate", "fused"])
@pytest.mark.parametrize("at_limit", [AT_LIMIT_WAIT, AT_LIMIT_ALLOW],
                         ids=["wait", "allow"])
def test_device_api_activations(at_limit, api):
    """Idle churn through the device API: k_add_chain flags the activating
    requests on the device (the requests never reach the host) and the
    host's idle mirror catches up lazily; the host API finds them on the
    host.  Identical add statuses, decisions, result records and final
    client state, over batches that mark a third of the clients idle (batch
    marking on one queue, one client at a time on the other)."""
    import torch
    from parity import compare_states
    n = 400
    tr = workloads.churn_trace(5, n, 10, 600, 0, idle_frac=0.35,
                               k_choices=[1, 9, 64, 300, 2000])
    qh = _mk("default", n=n, at_limit=at_limit)
    qd = _mk("default", n=n, at_limit=at_limit)
    c = tr.clients
    for q in (qh, qd):
        q.register(c.slots, c.r, c.w, c.l, c.active)
    dev = torch.device("cuda", 0)
    ops = list(tr.ops)
    i = 0
    while i < len(ops):
        op = ops[i]
        if op[0] == "idle":
            for s in op[1].tolist():
                qh.mark_idle(s)
            qd.mark_idle_batch(op[1])
            i += 1
            continue
        if op[0] == "add":
            reqs = op[1]
            rc_h = qh.add_batch(reqs)
            d_reqs = torch.from_numpy(reqs.view(np.uint8).copy()).to(dev)
            d_rc = torch.full((len(reqs),), -7, dtype=torch.int32, device=dev)
            if api == "fused" and i + 1 < len(ops) and ops[i + 1][0] == "pull":
                _, now, k = ops[i + 1]
                d_out = torch.zeros(max(k, 1) * DECISION_DTYPE.itemsize,
                                    dtype=torch.uint8, device=dev)
                d_res = torch.full((24,), 0xAB, dtype=torch.uint8, device=dev)
                qd.add_pull_batch_device(d_reqs.data_ptr(), len(reqs), d_rc.data_ptr(),
                                         now, k, d_out.data_ptr(), d_res.data_ptr())
                qd.sync()
                assert np.array_equal(d_rc.cpu().numpy(), rc_h)
                _check_pull(qh, now, k, d_out, d_res)
                i += 2
                continue
            qd.add_batch_device(d_reqs.data_ptr(), len(reqs), d_rc.data_ptr())
            qd.sync()
            assert np.array_equal(d_rc.cpu().numpy(), rc_h)
            i += 1
            continue
        _, now, k = op
        d_out = torch.zeros(max(k, 1) * DECISION_DTYPE.itemsize, dtype=torch.uint8,
                            device=dev)
        d_res = torch.full((24,), 0xAB, dtype=torch.uint8, device=dev)
        qd.pull_batch_device(now, k, d_out.data_ptr(), d_res.data_ptr())
        qd.sync()
        _check_pull(qh, now, k, d_out, d_res)
        i += 1
    compare_states(qd, qh, np.arange(n), "final")
    assert qd.stats().clients == qh.stats().clients
