"""U1 (dynamic ClientInfo, dmclock_server.h:870-875) on the device.

The reference re-reads client_info_f at every tag calculation -- initial_tag
(:878-907) and, in delayed mode, update_next_tag (:1021-1036) -- and stores
the result as the client's cached info, which reduce_reservation_tags uses
(:1077-1111).  The engine models client_info_f as a bound ClientInfo per slot
(dmc_client_bind_info_batch, or the host dmc_info_fn the engine calls before
each tag calculation of a host-API call).

Traces: workloads.dynamic_trace -- fresh ClientInfo objects for 20 % of the
clients before every pull, random delta/rho, pulls of k in {1, 3, 16, 64,
256} (single steps and batched rounds).  Every decision, tag, add status and
every client's state including the cached inverses bit-exact against the
oracle, which holds the reference's ClientInfo pointers (oracle/dmc_oracle.hpp).
"""
import numpy as np
import pytest

import pyoracle
from dmclock_amd import workloads
from parity import run_parity


def _pulls(q, tr):
    return [o for o in workloads.replay(q, tr) if o[0] == "pull"]


@pytest.mark.parametrize("delayed", [False, True])
def test_u1_changes_decisions_oracle(delayed):
    """The traces are U1-sensitive: the oracle's decisions with and without
    dynamic_info differ (else the GPU tests below would prove nothing)."""
    tr = workloads.dynamic_trace(1, 300, 12, 200)
    a = _pulls(pyoracle.OracleQueue(delayed=delayed, dynamic_info=True), tr)
    b = _pulls(pyoracle.OracleQueue(delayed=delayed, dynamic_info=False), tr)
    differ = sum(1 for x, y in zip(a, b)
                 if len(x[1]) != len(y[1]) or (x[1]["slot"] != y[1]["slot"]).any()
                 or (x[1]["tag_r"] != y[1]["tag_r"]).any())
    assert differ >= 3, differ


def _mk(**kw):
    from dmclock_amd.gpu import GpuQueue
    kw.setdefault("ring_capacity", 64)
    return GpuQueue(**kw)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 4])
@pytest.mark.parametrize("mode", ["callback", "bind"])
@pytest.mark.parametrize("delayed", [False, True])
def test_u1_parity(delayed, mode, seed):
    """callback: the engine calls client_info_f (dmc_info_fn) per add and, in
    delayed mode, per dispatched client between selection and pop (pulls run
    one at a time).  bind: the caller pushes the changed clients'
    ClientInfo (dmc_client_bind_info_batch) and pulls run as batched rounds,
    whose walks read the bound info at every delayed tag."""
    tr = workloads.dynamic_trace(seed, 300, 12, 200)
    n, qg, qo = run_parity(tr, _mk, queue_kw=dict(delayed=delayed, dynamic_info=True),
                           state_sample=300, gpu_kw=dict(info_callback=mode == "callback"),
                           info=True)
    assert n > 300, n
    c = qg.counters()
    if mode == "bind":
        assert c["rounds"] > 0, c
    elif delayed:
        assert c["rounds"] == 0 and c["single_steps"] >= n, c
    qg.close()


@pytest.mark.gpu
def test_u1_bind_unchanged_is_free():
    """Binding values equal to the bound ones does no device work and changes
    nothing; binding new values before any tag leaves the cached info alone
    until a tag calculation reads them."""
    q = _mk(max_clients=8, dynamic_info=True, info_callback=False)
    q.register(np.arange(4, dtype=np.uint32), np.full(4, 2.0), np.ones(4),
               np.zeros(4), True)
    q.bind_info(np.arange(4, dtype=np.uint32), np.full(4, 2.0), np.ones(4), np.zeros(4))
    s = q.client_state(1)
    assert s.r_inv == 0.5 and s.w_inv == 1.0
    q.bind_info(np.array([1], np.uint32), [4.0], [2.0], [0.0])
    s = q.client_state(1)
    assert s.r_inv == 0.5 and s.w_inv == 1.0  # cached: not yet read
    from dmclock_amd._abi import make_requests
    assert q.add_batch(make_requests([1], [1.0], [1], [1], [1], [7]))[0] == 0
    s = q.client_state(1)
    assert s.r_inv == 0.25 and s.w_inv == 0.5  # initial_tag read the bound info
    q.close()
