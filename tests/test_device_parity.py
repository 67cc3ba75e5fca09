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


def device_parity(trace, queue_kw=None, state_sample=4096, fuse=True, host_ops=False,
                  options=()):
    from dmclock_amd.gpu import GpuQueue
    queue_kw = queue_kw or {}
    qo = pyoracle.OracleQueue(**queue_kw)
    outs_o = workloads.replay(qo, trace)
    assert qo.ties == 0, f"trace has {qo.ties} tied decisions; pick another seed"
    n = int(trace.clients.slots.max()) + 1
    maxb = max(len(op[1]) for op in trace.ops if op[0] == "add")
    qg = GpuQueue(max_clients=n, ring_capacity=64, max_batch=maxb, **queue_kw)
    for opt, val in options:
        qg.set_option(opt, val)
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


def test_unset_phase_selection_fails_loudly():
    """A round whose pick leaves a phase's selection unset (the failure a
    k_remit block-size mismatch once caused: a 512-thread build dispatched
    469,585 of 1,310,720 decisions with status OK) must fail its outcome
    check in k_rrank: the call returns DMC_EDEVICE, nothing is dispatched,
    and bad_rounds counts it.  DMC_OPT_FAULT=1 injects exactly that (phase
    1's PhaseSel left unwritten) in both the eager and the graph path; with
    the hook off, the same queue dispatches again."""
    import torch
    from dmclock_amd._abi import OPT_FAULT
    from dmclock_amd.gpu import DmcError, GpuQueue
    tr = workloads.config3_trace(7, 1 << 16, 3, 1 << 12, depth=2)
    c = tr.clients
    q = GpuQueue(max_clients=1 << 16, ring_capacity=64, max_batch=1 << 16)
    q.register(c.slots, c.r, c.w, c.l, c.active)
    q.add_batch(tr.ops[0][1])
    q.set_option(OPT_FAULT, 1)
    now = tr.ops[1][1]
    for _ in range(3):  # eager, then the captured graph (second sighting on)
        with pytest.raises(DmcError, match=r"\(-3\)"):
            q.pull_batch(now, 4096)
    cnt = q.counters()
    assert cnt["bad_rounds"] == 3, cnt
    assert cnt["decisions"] == 0, cnt
    q.set_option(OPT_FAULT, 0)
    d, res = q.pull_batch(now, 4096)
    assert res.n_decisions == 4096 and len(d) == 4096
    torch.cuda.synchronize()
    q.close()


def test_pipelined_failure_next_call_not_run():
    """DMC_OPT_PIPELINE + DMC_OPT_FAULT: call N's round fails its
    outcome check and shuts the gate, so call N+1's graph, queued behind it,
    does nothing.  Call N+1 must say so -- DMC_ENOTRUN, its statuses and
    decisions untouched, the tick not advanced -- and the queue must go on:
    call N+2 equals the oracle that saw call N's adds (applied before its
    failed round, which dispatched nothing) and call N+2, not call N+1."""
    import torch
    from dmclock_amd._abi import DMC_ENOTRUN, OPT_FAULT, OPT_GRAPHS, OPT_PIPELINE
    from dmclock_amd.gpu import DmcError, GpuQueue
    tr = workloads.config3_trace(11, 1 << 16, 3, 1 << 12, depth=2)
    c = tr.clients
    steps = [(tr.ops[i][1], tr.ops[i + 1][1], tr.ops[i + 1][2])
             for i in range(2, len(tr.ops), 2)]
    qg = GpuQueue(max_clients=1 << 16, ring_capacity=64, max_batch=1 << 16)
    qo = pyoracle.OracleQueue()
    for q in (qg, qo):
        q.register(c.slots, c.r, c.w, c.l, c.active)
        q.add_batch(tr.ops[0][1])
        q.pull_batch(tr.ops[1][1], tr.ops[1][2])
    qg.set_option(OPT_PIPELINE, 1)
    qg.set_option(OPT_GRAPHS, 0)
    dev = torch.device("cuda", 0)
    k = 1 << 12
    d_reqs = [torch.from_numpy(r.view(np.uint8)).to(dev) for r, _, _ in steps]
    d_rc = [torch.full((k,), 77, dtype=torch.int32, device=dev) for _ in steps]
    d_out = [torch.zeros(k * DECISION_DTYPE.itemsize, dtype=torch.uint8, device=dev)
             for _ in steps]
    d_res = torch.zeros((len(steps), 24), dtype=torch.uint8, device=dev)

    def call(i):
        reqs, now, kk = steps[i]
        qg.add_pull_batch_device(d_reqs[i].data_ptr(), len(reqs), d_rc[i].data_ptr(), now,
                                 kk, d_out[i].data_ptr(), d_res[i].data_ptr())

    qg.set_option(OPT_FAULT, 1)
    call(0)  # pipelined: its failure is reported by the next call
    with pytest.raises(DmcError, match=rf"\({DMC_ENOTRUN}\)"):
        call(1)
    # (the error DMC_ENOTRUN stands for -- call 0's failed round
    # -- stays readable)
    from dmclock_amd._abi import DMC_EDEVICE
    assert qg.pipelined_error() == DMC_EDEVICE
    assert qg.pipelined_error() == 0  # (read and cleared)
    qg.set_option(OPT_FAULT, 0)
    call(2)
    qg.sync()
    torch.cuda.synchronize()
    assert (d_rc[1].cpu().numpy() == 77).all()  # call 1 never ran
    assert qg.counters()["bad_rounds"] >= 1
    with pytest.raises(DmcError):  # option 9: the retired DMC_OPT_PREDICT
        qg.set_option(9, 1)
    import ctypes
    buf = ctypes.create_string_buffer(16)  # a caller with an older, smaller struct
    assert qg.L.dmc_queue_counters_sized(qg.h, buf, 16, 0) == 0
    assert int.from_bytes(buf.raw[:8], "little") == qg.counters()["rounds"]
    qo.add_batch(steps[0][0])
    rc_o = qo.add_batch(steps[2][0])
    do, ro = qo.pull_batch(steps[2][1], steps[2][2])
    assert qo.ties == 0
    assert np.array_equal(d_rc[2].cpu().numpy(), rc_o)
    pr = PullResult.from_buffer_copy(d_res[2].cpu().numpy().tobytes())
    assert (pr.n_decisions, pr.next_type) == (ro.n_decisions, ro.next_type)
    dg = d_out[2][:pr.n_decisions * DECISION_DTYPE.itemsize].cpu().numpy().view(DECISION_DTYPE)
    compare_decisions(dg, do, "call 2")
    rng = np.random.default_rng(3)
    compare_states(qg, qo, rng.choice(c.slots, 1024, replace=False), "after")
    qg.close()
    qo.close()


def _bench_setup(q, tr):
    """bench.py's prepare(): bulk registration, the pre-population in 1M
    chunks and the settle pulls in 1M chunks, through the host API"""
    c = tr.clients
    q.register(c.slots, c.r, c.w, c.l, c.active)
    pre = tr.ops[0][1]
    rcs = [q.add_batch(pre[i:i + (1 << 20)]) for i in range(0, len(pre), 1 << 20)]
    now, k = tr.ops[1][1], tr.ops[1][2]
    outs, done = [], 0
    while done < k:
        kk = min(k - done, 1 << 20)
        d, res = q.pull_batch(now, kk)
        outs.append((d, (res.n_decisions, res.next_type)))
        done += kk
    return rcs, outs


@pytest.mark.timeout(480)
@pytest.mark.parametrize("mode", ["bench", "graphs"])
def test_bench_exact_trace_parity(mode):
    """bench.py's own workload, call for call,
    `bench`: as bench.py runs it (DMC_OPT_PIPELINE, kernels launched
    eagerly, no synchronisation between the calls, one status buffer per
    step); `graphs`: unpipelined calls replaying the captured graph:
    config3_trace(42, 2^20, 33 steps, 64K, depth 4) is make_workload's trace
    at the default arguments (seed 42, 4,194,304 pre-populated requests, a
    2,097,152-pull settle in two host calls, then warmup 3 + timed 20 +
    profiled 10 steps, each one dmc_add_pull_batch_device of 64K adds + 64K
    pulls replaying the captured graph).  The oracle replays the same calls
    concurrently (ctypes releases the GIL).  Every add status, decision and
    result record bit-exact, 4096 sampled client states, and the engine
    counters: no radix round, no bin overflow, no sample re-run."""
    import threading
    import torch
    from dmclock_amd.gpu import GpuQueue
    tr = workloads.config3_trace(42, 1 << 20, 33, 1 << 16, depth=4)
    steps = [(tr.ops[i][1], tr.ops[i + 1][1], tr.ops[i + 1][2])
             for i in range(2, len(tr.ops), 2)]
    want = {}

    def oracle():
        qo = pyoracle.OracleQueue()
        want["setup"] = _bench_setup(qo, tr)
        out = []
        for reqs, now, k in steps:
            rc = qo.add_batch(reqs)
            d, res = qo.pull_batch(now, k)
            out.append((rc, d, (res.n_decisions, res.next_type)))
        want["steps"] = out
        want["q"] = qo

    th = threading.Thread(target=oracle)
    th.start()
    dev = torch.device("cuda", 0)
    qg = GpuQueue(max_clients=1 << 20, ring_capacity=64, max_batch=1 << 20)
    got_setup = _bench_setup(qg, tr)
    if mode == "bench":
        from dmclock_amd._abi import OPT_GRAPHS, OPT_PIPELINE
        qg.set_option(OPT_PIPELINE, 1)
        qg.set_option(OPT_GRAPHS, 0)
    d_reqs = [torch.from_numpy(r.view(np.uint8)).to(dev) for r, _, _ in steps]
    k = 1 << 16
    d_rcs = [torch.zeros(k, dtype=torch.int32, device=dev) for _ in steps]
    d_out = [torch.zeros(k * DECISION_DTYPE.itemsize, dtype=torch.uint8, device=dev)
             for _ in steps]
    d_res = torch.zeros((len(steps), 24), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    qg.counters(reset=True)
    rcs = []
    for i, (reqs, now, kk) in enumerate(steps):
        qg.add_pull_batch_device(d_reqs[i].data_ptr(), len(reqs), d_rcs[i].data_ptr(), now,
                                 kk, d_out[i].data_ptr(), d_res[i].data_ptr())
        if mode != "bench":
            qg.sync()
    qg.sync()
    rcs = d_rcs
    ctr = qg.counters()
    torch.cuda.synchronize()
    th.join()
    assert "q" in want, "oracle thread failed"
    qo = want["q"]
    assert qo.ties == 0, f"trace has {qo.ties} tied decisions"
    for a, b in zip(got_setup[0], want["setup"][0]):
        assert np.array_equal(a, b)
    for i, ((dg, rg), (do, ro)) in enumerate(zip(got_setup[1], want["setup"][1])):
        compare_decisions(dg, do, f"settle call {i}")
        assert rg == ro, (i, rg, ro)
    n = 0
    for i, (rc_o, do, ro) in enumerate(want["steps"]):
        assert np.array_equal(rcs[i].cpu().numpy(), rc_o), i
        pr = PullResult.from_buffer_copy(d_res[i].cpu().numpy().tobytes())
        assert (pr.n_decisions, pr.next_type) == ro, (i, pr.n_decisions, ro)
        dg = d_out[i][:pr.n_decisions * DECISION_DTYPE.itemsize].cpu().numpy() \
            .view(DECISION_DTYPE)
        compare_decisions(dg, do, f"step {i}")
        n += len(do)
    assert n > 30 * 60000, n
    assert ctr["fused_calls"] == len(steps), ctr
    assert ctr["radix_rounds"] == 0 and ctr["bin_overflows"] == 0, ctr
    assert ctr["sample_retries"] == 0, ctr
    rng = np.random.default_rng(1)
    compare_states(qg, qo, rng.choice(tr.clients.slots, 4096, replace=False), "final")
    assert qg.request_count() == qo.request_count()
    assert tuple(qg.sched_counts()) == tuple(qo.sched_counts())
    qo.close()
    qg.close()


def test_fused_device_vs_host_api_200_steps():
    """A 200-step horizon at bench.py's shape (the key spread keeps growing,
    DESIGN.md section 6): the fused device call against the host-buffer API
    on a second queue, every step's decisions and results bit-exact (a
    property of the engine: both APIs run the same rounds; the oracle's
    horizon is test_bench_exact_trace_parity's 33 steps)."""
    import torch
    from dmclock_amd.gpu import GpuQueue
    n_steps = 200
    tr = workloads.config3_trace(7, 1 << 20, n_steps, 1 << 16, depth=4)
    steps = [(tr.ops[i][1], tr.ops[i + 1][1], tr.ops[i + 1][2])
             for i in range(2, len(tr.ops), 2)]
    dev = torch.device("cuda", 0)
    qa = GpuQueue(max_clients=1 << 20, ring_capacity=64, max_batch=1 << 20)
    qb = GpuQueue(max_clients=1 << 20, ring_capacity=64, max_batch=1 << 20)
    for q in (qa, qb):
        _bench_setup(q, tr)
    qa.counters(reset=True)
    k = 1 << 16
    d_rc = torch.zeros(k, dtype=torch.int32, device=dev)
    d_out = torch.zeros(k * DECISION_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    d_res = torch.zeros(24, dtype=torch.uint8, device=dev)
    n = 0
    for i, (reqs, now, kk) in enumerate(steps):
        d_reqs = torch.from_numpy(reqs.view(np.uint8)).to(dev)
        torch.cuda.synchronize()
        qa.add_pull_batch_device(d_reqs.data_ptr(), len(reqs), d_rc.data_ptr(), now, kk,
                                 d_out.data_ptr(), d_res.data_ptr())
        qa.sync()
        rb = qb.add_batch(reqs)
        db, resb = qb.pull_batch(now, kk)
        assert np.array_equal(d_rc.cpu().numpy(), rb), i
        pr = PullResult.from_buffer_copy(d_res.cpu().numpy().tobytes())
        assert (pr.n_decisions, pr.next_type) == (resb.n_decisions, resb.next_type), i
        da = d_out[:pr.n_decisions * DECISION_DTYPE.itemsize].cpu().numpy() \
            .view(DECISION_DTYPE)
        compare_decisions(da, db, f"step {i}")
        n += len(db)
    assert n > n_steps * 60000, n
    rng = np.random.default_rng(2)
    sl = rng.choice(tr.clients.slots, 2048, replace=False)
    compare_states(qa, qb, sl, "final")
    # (over 200 steps the key spread grows: an overflowed rank bin re-runs
    # the round smaller, bin_splits; none needs the radix path)
    c = qa.counters()
    assert c["radix_rounds"] == 0, c
    assert c["bin_overflows"] == c["bin_splits"] <= 4, c
    qa.close()
    qb.close()


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


@pytest.mark.timeout(900)
def test_config4_1m_device_activations_vs_oracle():
    """BASELINE config 4 at its full size, 1,048,576 clients, against the
    oracle.  The oracle's idle reset
    (dmclock_server.h:937-985) keeps the reference's minimum over the
    non-idle clients exactly in a segment tree instead of the reference's
    O(N) scan per activation (oracle/dmc_oracle.hpp ActMin, pinned bit for
    bit against the scan by tests/test_oracle_actmin.py): the 1M replay takes
    about a minute instead of hours.
    Activations make ties: an activated client's proportion key is
    p + (L - t) with p = t for a client that was idle, i.e. the current
    lowest key L up to rounding, so config-4 traces at this size tie a few
    dozen decisions (no tie-free seed over the steps that hold activations:
    idle marking starts at step 2).  The engine therefore runs in tie-exact
    order (DMC_OPT_HEAP_ORDER), through the device API bench.py --config 4
    uses -- HBM idle lists, fused add + pull calls, the batch's activations
    found and resolved on the device by the same kernels as the default
    mode (k_add_chain's detection, the speculated min-plus scan of DESIGN
    section 3.1) -- so that every decision can be compared, ties included.
    Four steps of 65,536 adds + 65,536 pulls, 10 % of the clients marked idle
    before each: every add status, decision (slot, phase, cost, handle, tag
    bits) and result record, and 4096 sampled client states (prop_delta
    included) bit-exact; the ties present went to the reference's heap top."""
    from dmclock_amd.gpu import GpuQueue
    tr = workloads.config4_trace(3, 1 << 20, 4, 1 << 16)
    acts = 0
    idle = np.zeros(1 << 20, bool)
    for op in tr.ops:
        if op[0] == "idle":
            idle[op[1]] = True
        elif op[0] == "add":
            u = np.unique(op[1]["slot"])
            acts += int(idle[u].sum())
            idle[u] = False
    assert acts > 10_000, acts
    qo = pyoracle.OracleQueue()
    outs_o = workloads.replay(qo, tr)
    maxb = max(len(op[1]) for op in tr.ops if op[0] == "add")
    qg = GpuQueue(max_clients=1 << 20, ring_capacity=64, max_batch=maxb, heap_order=True)
    outs_g = replay_device(qg, tr, fuse=True)
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
    compare_states(qg, qo, rng.choice(tr.clients.slots, 4096, replace=False), "final")
    assert qg.request_count() == qo.request_count()
    assert tuple(qg.sched_counts()) == tuple(qo.sched_counts())
    assert n_dec > 4 * 60_000, n_dec
    assert qo.ties > 0, qo.ties
    c = qg.counters()
    assert c["act_batches"] >= 2, c
    print(f"config 4 at 1M clients: {acts} activations, {n_dec} decisions, "
          f"{qo.ties} tied, all the reference's")
    qg.close()
    qo.close()


def test_reject_activations_device_api():
    """AtLimit::Reject through the device API: activations detected by
    k_add_chain on the device, rejected activations whose client's basis
    moves again in the batch resolved in order (k_act_hard), the host's idle
    mirror never consulted.  Every add status, decision, result record and
    sampled client state bit-exact against the oracle (tie-free seed)."""
    from dmclock_amd._abi import AT_LIMIT_REJECT
    tr = workloads.reject_churn_trace(4, 2000, 6, 4000, idle_frac=0.1)
    n, qg, qo = device_parity(tr, queue_kw=dict(at_limit=AT_LIMIT_REJECT,
                                                reject_threshold=0.5))
    c = qg.counters()
    assert c["act_batches"] == 6 and c["act_seq_batches"] >= 1, c
    qg.close()


def replay_pipelined(q, trace):
    """The trace's add + pull pairs as dmc_add_pull_batch_device calls with
    DMC_OPT_PIPELINE on, issued back to back with no synchronisation between
    them (each call its own status, decision and result buffers, as a caller
    overlapping its calls would hold them); other ops through the device
    API.  One dmc_queue_sync at the end, then every output read back."""
    import torch
    from dmclock_amd._abi import OPT_PIPELINE
    dev = torch.device("cuda", 0)
    c = trace.clients
    q.register(c.slots, c.r, c.w, c.l, c.active)
    q.set_option(OPT_PIPELINE, 1)
    ops = trace.ops
    pending = []  # (kind, buffers)
    keep = []
    i = 0
    while i < len(ops):
        op = ops[i]
        if op[0] == "add":
            reqs = torch.from_numpy(op[1].view(np.uint8).copy()).to(dev)
            n = len(op[1])
            d_rc = torch.zeros(n, dtype=torch.int32, device=dev)
            torch.cuda.synchronize()  # (the copies ran on torch's stream)
            keep.append(reqs)
            if i + 1 < len(ops) and ops[i + 1][0] == "pull":
                now, k = ops[i + 1][1], ops[i + 1][2]
                d_out = torch.zeros(k * DECISION_DTYPE.itemsize, dtype=torch.uint8, device=dev)
                d_res = torch.zeros(24, dtype=torch.uint8, device=dev)
                q.add_pull_batch_device(reqs.data_ptr(), n, d_rc.data_ptr(), now, k,
                                        d_out.data_ptr(), d_res.data_ptr())
                pending.append(("add", d_rc))
                pending.append(("pull", (d_out, d_res)))
                i += 2
                continue
            q.add_batch_device(reqs.data_ptr(), n, d_rc.data_ptr())
            pending.append(("add", d_rc))
        elif op[0] == "pull":
            k = op[2]
            d_out = torch.zeros(k * DECISION_DTYPE.itemsize, dtype=torch.uint8, device=dev)
            d_res = torch.zeros(24, dtype=torch.uint8, device=dev)
            q.pull_batch_device(op[1], k, d_out.data_ptr(), d_res.data_ptr())
            pending.append(("pull", (d_out, d_res)))
        else:
            raise ValueError(op[0])
        i += 1
    q.sync()
    outs = []
    for kind, buf in pending:
        if kind == "add":
            outs.append(("add", buf.cpu().numpy().copy()))
        else:
            d_out, d_res = buf
            res = PullResult.from_buffer_copy(d_res.cpu().numpy().tobytes())
            dec = d_out[:res.n_decisions * DECISION_DTYPE.itemsize].cpu().numpy() \
                .view(DECISION_DTYPE).copy()
            outs.append(("pull", dec, (res.n_decisions, res.next_type,
                                       res.when if res.next_type == 1 else 0.0)))
    return outs


@pytest.mark.parametrize("variant", ["default", "sample_retry", "terminal", "eager",
                                     "eager_retry", "eager_delayed", "eager_exact"])
def test_pipelined_calls_parity(variant):
    """DMC_OPT_PIPELINE (bench.py's default): config-3 steps at 65,536
    clients issued as back-to-back pipelined calls.  `sample_retry` runs the
    sampled thresholds with no margin, so that every round fails validation
    and needs the host (a re-run): each such round shuts the device-side gate,
    the next call's already-queued graph does nothing and is launched again
    -- the path a caller never sees.  `terminal` puts a step that pulls more
    than is queued in the middle (a terminal round: the host's terminal pull,
    then the next call's graph launched again).  `eager` / `eager_retry`:
    the same with graphs off (each call's kernels launched eagerly, still
    queued behind the previous call's -- and the add chain beside the
    scan, k_chain_scan); `eager_delayed`: DelayedTagCalc; `eager_exact`:
    the exact threshold histogram (every slot's keys written).
    Every add status, decision and result record bit-exact against the
    oracle."""
    from dmclock_amd._abi import OPT_SAMPLE
    from dmclock_amd.gpu import GpuQueue
    tr = workloads.config3_trace(42, 1 << 16, 6, 1 << 12, depth=2)
    if variant == "terminal":
        # a step in the middle pulls more than is queued (a terminal round)
        t = float(tr.ops[7][1])
        reqs = workloads.arrivals(np.random.default_rng(5), 1 << 16, 1 << 12, t, 2.0 * (1 << 16),
                                  handle_base=10 ** 7)
        tr.ops[8:8] = [("add", reqs), ("pull", float(reqs["time"][-1]), 1 << 18)]
    kw = dict(delayed=True) if variant == "eager_delayed" else {}
    qo = pyoracle.OracleQueue(**kw)
    outs_o = workloads.replay(qo, tr)
    assert qo.ties == 0
    qg = GpuQueue(max_clients=1 << 16, ring_capacity=64, max_batch=1 << 18, **kw)
    if variant in ("sample_retry", "eager_retry"):
        qg.set_option(OPT_SAMPLE, 2)
    if variant == "eager_exact":
        qg.set_option(OPT_SAMPLE, 0)
    if variant.startswith("eager"):
        from dmclock_amd._abi import OPT_GRAPHS
        qg.set_option(OPT_GRAPHS, 0)
    outs_g = replay_pipelined(qg, tr)
    assert len(outs_g) == len(outs_o)
    for i, (a, b) in enumerate(zip(outs_g, outs_o)):
        assert a[0] == b[0], i
        if a[0] == "add":
            assert np.array_equal(a[1], b[1]), (i, np.nonzero(a[1] != b[1]))
        else:
            compare_decisions(a[1], b[1], f"op {i}")
            assert a[2] == b[2], (i, a[2], b[2])
    compare_states(qg, qo, np.random.default_rng(3).choice(1 << 16, 2048, replace=False),
                   "final")
    c = qg.counters()
    print(variant, c)
    assert c["fused_calls"] >= 6, c
    if variant in ("sample_retry", "eager_retry"):
        assert c["sample_retries"] >= 6, c
    qg.close()


def test_pipelined_deferred_apply_interleaved():
    """DMC_DEFER_APPLY: a pipelined call's apply is launched by the next
    call's filing launch (k_apply_link) -- or, before any other work, by
    whatever comes next.  Pipelined calls (kernels launched eagerly) with a
    lone add batch, a small pull (the single-op path, no fusing) and a lone
    batched pull between them, and the queue's statistics read in the
    middle: every status, decision and result record bit-exact against the
    oracle, and the sampled states at the end."""
    from dmclock_amd._abi import OPT_GRAPHS
    from dmclock_amd.gpu import GpuQueue
    tr = workloads.config3_trace(7, 1 << 16, 6, 1 << 12, depth=2)
    t = float(tr.ops[3][1])
    extra = workloads.arrivals(np.random.default_rng(9), 1 << 16, 1 << 11, t, 2.0 * (1 << 16),
                               handle_base=10 ** 7)
    te = float(extra["time"][-1])
    tr.ops[4:4] = [("add", extra), ("pull", te, 4), ("pull", te, 1 << 12)]
    qo = pyoracle.OracleQueue()
    outs_o = workloads.replay(qo, tr)
    assert qo.ties == 0
    qg = GpuQueue(max_clients=1 << 16, ring_capacity=64, max_batch=1 << 16)
    qg.set_option(OPT_GRAPHS, 0)
    outs_g = replay_pipelined(qg, tr)
    assert len(outs_g) == len(outs_o)
    for i, (a, b) in enumerate(zip(outs_g, outs_o)):
        assert a[0] == b[0], i
        if a[0] == "add":
            assert np.array_equal(a[1], b[1]), (i, np.nonzero(a[1] != b[1]))
        else:
            compare_decisions(a[1], b[1], f"op {i}")
            assert a[2] == b[2], (i, a[2], b[2])
    compare_states(qg, qo, np.random.default_rng(4).choice(1 << 16, 2048, replace=False),
                   "final")
    assert qg.counters()["fused_calls"] >= 6
    qg.close()


def test_pipelined_bench_call_parity_1m_clients():
    """bench.py's timed call as it runs by default (DMC_OPT_PIPELINE, kernels
    launched eagerly) at full size: 1,048,576 clients, four pipelined steps of 64K adds + 64K
    pulls after the pre-population and settle; every output bit-exact."""
    from dmclock_amd.gpu import GpuQueue
    tr = workloads.config3_trace(42, 1 << 20, 4, 1 << 16, depth=2)
    qo = pyoracle.OracleQueue()
    outs_o = workloads.replay(qo, tr)
    assert qo.ties == 0
    qg = GpuQueue(max_clients=1 << 20, ring_capacity=64, max_batch=1 << 20)
    from dmclock_amd._abi import OPT_GRAPHS
    qg.set_option(OPT_GRAPHS, 0)  # (bench.py's launch mode)
    outs_g = replay_pipelined(qg, tr)
    for i, (a, b) in enumerate(zip(outs_g, outs_o)):
        if a[0] == "add":
            assert np.array_equal(a[1], b[1]), i
        else:
            compare_decisions(a[1], b[1], f"op {i}")
            assert a[2] == b[2], (i, a[2], b[2])
    assert qg.counters()["fused_calls"] >= 4
    qg.close()
