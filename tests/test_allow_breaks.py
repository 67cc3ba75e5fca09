"""AtLimit::Allow's limit breaks as batched rounds.

Once a batch of pulls at one `now` has taken every eligible request, each
further pull_request(now) under AtLimit::Allow pops the ready-heap top
regardless of its limit (dmclock_server.h:1157-1165): the not-ready front
with the smallest p + prop_delta.  Its reduce_reservation_tags can expose the
client's next requests to the next pulls (r <= now: a reservation pop; l <=
now: readied by the next limit scan and popped as the only ready front).  So
the limit breaks are a merge of per-client groups by key -- another round
(walk_p's brk groups) instead of one general step per pull.

Checked bit-exact against the oracle (the reference's heaps): every decision,
result record and sampled client state, with the engine counters showing the
pulls ran as limit-break rounds; and with weight-0 clients (p = inf, which
break the merge's assumptions) the engine falls back to general pulls.
"""
import numpy as np
import pytest

import pyoracle
from dmclock_amd import workloads
from dmclock_amd._abi import AT_LIMIT_ALLOW, OPT_BREAK_ROUNDS
from parity import run_parity

pytestmark = pytest.mark.gpu


def limited_trace(seed, n, steps, batch, k, zero_w=0):
    """every client limited below its arrival rate (l ~ U[0.3, 1.2] against
    about 2 requests/s), 20 % with a reservation, pulls of k at each step's
    end: most of a pull batch is limit breaks"""
    tr = workloads.steady_trace(seed, n, steps, batch, k, depth=3,
                                table_kw=dict(frac_r=0.2, frac_l=1.0,
                                              l_range=(0.3, 1.2)))
    if zero_w:
        rng = np.random.default_rng(seed + 7)
        z = rng.choice(n, zero_w, replace=False)
        tr.clients.w[z] = 0.0
        # (r or w must be > 0) a reservation below the arrival rate keeps
        # requests queued behind the clock: fronts with p = inf when the
        # limit breaks start
        tr.clients.r[z] = 0.5
    return tr


def _mk(brk):
    def mk(**kw):
        from dmclock_amd.gpu import GpuQueue
        q = GpuQueue(ring_capacity=64, max_batch=1 << 16, **kw)
        q.set_option(OPT_BREAK_ROUNDS, int(brk))
        return q
    return mk


@pytest.mark.parametrize("n,batch,k,seed", [(1 << 16, 8192, 16384, 3),
                                            (4096, 1024, 3000, 5)])
def test_limit_breaks_as_rounds_parity(n, batch, k, seed):
    tr = limited_trace(seed, n, 4, batch, k)
    nd, qg, qo = run_parity(tr, _mk(True), queue_kw=dict(at_limit=AT_LIMIT_ALLOW),
                            state_sample=2048)
    c = qg.counters()
    print("counters", c)
    assert c["brk_rounds"] >= 2, c
    assert c["brk_fallbacks"] == 0, c
    # (general steps only where a round was cut inside a break group's run)
    assert c["single_steps"] < 4 * 8, c
    res, prio = qo.sched_counts()
    assert prio > 10_000 or n < 10_000, (res, prio)
    qg.close()


def test_weight_zero_clients_fall_back_to_general_pulls():
    tr = limited_trace(9, 4096, 3, 1024, 2500, zero_w=1)  # (two would tie at p = inf)
    nd, qg, qo = run_parity(tr, _mk(True), queue_kw=dict(at_limit=AT_LIMIT_ALLOW),
                            state_sample=4096)
    c = qg.counters()
    assert c["brk_fallbacks"] >= 1, c
    qg.close()


def test_break_rounds_equal_single_steps():
    """the same trace with limit breaks as single steps (the round-2 path):
    identical decisions and state (a property of the engine)"""
    from parity import compare_decisions, compare_states
    tr = limited_trace(11, 8192, 3, 2048, 4000)
    qa = _mk(True)(max_clients=8192, at_limit=AT_LIMIT_ALLOW)
    qb = _mk(False)(max_clients=8192, at_limit=AT_LIMIT_ALLOW)
    oa, ob = workloads.replay(qa, tr), workloads.replay(qb, tr)
    for i, (a, b) in enumerate(zip(oa, ob)):
        if a[0] == "pull":
            compare_decisions(a[1], b[1], f"op {i}")
            assert a[2] == b[2], i
    compare_states(qa, qb, np.arange(8192), "final")
    assert qa.counters()["brk_rounds"] >= 2
    assert qb.counters()["brk_rounds"] == 0
    assert qb.counters()["single_steps"] > qa.counters()["single_steps"] + 1000
