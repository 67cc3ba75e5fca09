"""Parity of the device-buffer API -- the exact calls bench.py times -- against
the oracle, at the benchmark's own sizes (needs an MI355X).

bench.py times dmc_add_pull_batch_device: the add kernels and the first pull
round captured as one hipGraph and replayed with the step's parameters.
These tests drive that same call with HBM-resident requests, decisions and
result records and compare, bit for bit, every add status, every decision
(client, phase, cost, handle, tag bits), every result record and sampled
client state with the oracle replaying the same trace through the
reference's sequential semantics (oracle/dmc_oracle.hpp).

  * config 3 at full size (1,048,576 clients): the fused graph path, its
    replays checked through the engine counters;
  * config 4 at 65,536 clients: idle marking of 10 % of the clients before
    every step (activations through the idle reset, resolved on the device)
    and 10 % of the tenants limited below their arrival rate under
    AtLimit::Wait; seeds verified tie-free by the oracle.
"""
import numpy as np
import pytest

import pyoracle
from dmclock_amd import workloads
from dmclock_amd._abi import DECISION_DTYPE, PullResult
from parity import compare_decisions, compare_states

pytestmark = pytest.mark.gpu


def replay_device(q, trace, fuse=True, host_ops=False):
    """workloads.replay through the device API: an add followed by a pull is
    one dmc_add_pull_batch_device call (fuse) -- bench.py's step -- other ops
    dmc_add_batch_device / dmc_pull_batch_device; inputs are copied to HBM
    before each call and outputs read back after it."""
    import torch
    dev = torch.device("cuda", 0)
    c = trace.clients
    q.register(c.slots, c.r, c.w, c.l, c.active)
    ops = trace.ops
    maxk = max([op[2] for op in ops if op[0] == "pull"] + [1])
    maxn = max([len(op[1]) for op in ops if op[0] == "add"] + [1])
    d_out = torch.zeros(maxk * DECISION_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    d_rc = torch.zeros(maxn, dtype=torch.int32, device=dev)
    d_res = torch.zeros(24, dtype=torch.uint8, device=dev)

    def pull_out():
        res = PullResult.from_buffer_copy(d_res.cpu().numpy().tobytes())
        dec = d_out[:res.n_decisions * DECISION_DTYPE.itemsize].cpu().numpy() \
            .view(DECISION_DTYPE).copy()
        return ("pull", dec, (res.n_decisions, res.next_type,
                              res.when if res.next_type == 1 else 0.0))

    outs = []
    i = 0
    while i < len(ops):
        op = ops[i]
        if host_ops and op[0] == "add":  # host API after device-side idle marking
            outs.append(("add", q.add_batch(op[1])))
        elif host_ops and op[0] == "pull":
            d, res = q.pull_batch(op[1], op[2])
            outs.append(("pull", d, (res.n_decisions, res.next_type,
                                     res.when if res.next_type == 1 else 0.0)))
        elif op[0] == "add":
            reqs = torch.from_numpy(op[1].view(np.uint8).copy()).to(dev)
            n = len(op[1])
            torch.cuda.synchronize()  # the copy ran on torch's stream
            if fuse and i + 1 < len(ops) and ops[i + 1][0] == "pull":
                now, k = ops[i + 1][1], ops[i + 1][2]
                q.add_pull_batch_device(reqs.data_ptr(), n, d_rc.data_ptr(), now, k,
                                        d_out.data_ptr(), d_res.data_ptr())
                q.sync()
                outs.append(("add", d_rc[:n].cpu().numpy().copy()))
                outs.append(pull_out())
                i += 2
                continue
            q.add_batch_device(reqs.data_ptr(), n, d_rc.data_ptr())
            q.sync()
            outs.append(("add", d_rc[:n].cpu().numpy().copy()))
        elif op[0] == "pull":
            q.pull_batch_device(op[1], op[2], d_out.data_ptr(), d_res.data_ptr())
            q.sync()
            outs.append(pull_out())
        elif op[0] == "idle":
            # bench.py's config-4 marking: the list resident in HBM
            d_idle = torch.from_numpy(np.ascontiguousarray(op[1], dtype=np.uint32)
                                      .view(np.int32)).to(dev)
            torch.cuda.synchronize()
            q.mark_idle_batch_device(d_idle.data_ptr(), len(op[1]))
            q.sync()
            outs.append(("idle", None))
        else:
            raise ValueError(op[0])
        i += 1
    return outs


def device_parity(trace, queue_kw=None, state_sample=4096, fuse=True, host_ops=False):
    from dmclock_amd.gpu import GpuQueue
    queue_kw = queue_kw or {}
    qo = pyoracle.OracleQueue(**queue_kw)
    outs_o = workloads.replay(qo, trace)
    assert qo.ties == 0, f"trace has {qo.ties} tied decisions; pick another seed"
    n = int(trace.clients.slots.max()) + 1
    maxb = max(len(op[1]) for op in trace.ops if op[0] == "add")
    qg = GpuQueue(max_clients=n, ring_capacity=64, max_batch=maxb, **queue_kw)
    outs_g = replay_device(qg, trace, fuse=fuse, host_ops=host_ops)
    n_dec = 0
    for i, (a, b) in enumerate(zip(outs_g, outs_o)):
        assert a[0] == b[0], i
        if a[0] == "add":
            assert np.array_equal(a[1], b[1]), (i, np.nonzero(a[1] != b[1]))
        elif a[0] == "pull":
            compare_decisions(a[1], b[1], f"op {i}")
            assert a[2] == b[2], (i, a[2], b[2])
            n_dec += len(a[1])
    rng = np.random.default_rng(1)
    slots = trace.clients.slots
    compare_states(qg, qo, rng.choice(slots, min(state_sample, len(slots)),
                                      replace=False), "final")
    assert qg.request_count() == qo.request_count()
    assert tuple(qg.sched_counts()) == tuple(qo.sched_counts())
    return n_dec, qg, qo


def test_fused_bench_call_parity_1m_clients():
    """BASELINE config 3 at full size through bench.py's call: 1,048,576
    clients, 2M pre-populated requests, a 1M-pull settle round, then four
    steps of 64K adds + 64K pulls, each one dmc_add_pull_batch_device; from
    the second step on the add kernels and the round replay one captured
    graph.  Every decision, add status and result record bit-exact."""
    tr = workloads.config3_trace(42, 1 << 20, 4, 1 << 16, depth=2)
    n, qg, qo = device_parity(tr)
    assert n > 1_200_000
    c = qg.counters()
    assert c["fused_calls"] == 4, c
    assert c["graph_replays"] >= 3, c
    qg.close()


@pytest.mark.parametrize("seed", [1, 2])
@pytest.mark.parametrize("api", ["device", "host", "mixed"])
def test_config4_churn_throttled_parity_64k(seed, api):
    """BASELINE config 4 at 65,536 clients: before each of four steps of 4096
    adds + 4096 pulls, 10 % of the clients (those without an arrival in the
    two previous steps) are marked idle; 10 % of the tenants are limited
    below their arrival rate (AtLimit::Wait).  Seeds 1 and 2 are tie-free
    under the oracle.  Every API bit-exact, hundreds of activations per step."""
    from parity import run_parity
    tr = workloads.config4_trace(seed, 1 << 16, 4, 1 << 12)
    idle = np.zeros(1 << 16, bool)
    acts = 0
    for op in tr.ops:
        if op[0] == "idle":
            idle[op[1]] = True
        elif op[0] == "add":
            u = np.unique(op[1]["slot"])
            acts += int(idle[u].sum())
            idle[u] = False
    assert acts > 500, acts
    if api in ("device", "mixed"):
        # mixed: HBM idle lists, then host-API adds / pulls (the engine
        # re-reads its idle view from the device)
        n, qg, qo = device_parity(tr, host_ops=api == "mixed")
    else:
        from test_gpu_parity import mk_gpu
        n, qg, qo = run_parity(tr, mk_gpu, state_sample=4096)
    res, prio = qo.sched_counts()
    assert n > 100_000 and res > 1000 and prio > 1000, (n, res, prio)
