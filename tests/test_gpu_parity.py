"""Parity of the HIP engine against the oracle (needs an MI355X).

Bar: bit-exact.  Every decision (client, phase, cost, request handle and the
dispatched tag's bits), every add status, every stopping pull's type and
future time, the scheduling counters, and sampled per-client state (prev tag,
prop_delta, front tag, ready/idle flags) must equal the oracle's.  Traces are
checked tie-free by the oracle first (among equal keys
the reference's winner is its heap history; the engine breaks ties by lowest
slot and flags them).
"""
import numpy as np
import pytest

import kats
from dmclock_amd import workloads
from dmclock_amd._abi import AT_LIMIT_ALLOW, AT_LIMIT_REJECT, AT_LIMIT_WAIT
from parity import run_parity

pytestmark = pytest.mark.gpu


def mk_gpu(**kw):
    from dmclock_amd.gpu import GpuQueue
    kw.setdefault("max_clients", 256)
    kw.setdefault("ring_capacity", 64)
    return GpuQueue(**kw)


def mk_variant(variant):
    """engine paths: default (bin-rank batches, single steps for k <= 8),
    radix-sorted batches, and single steps for every pull"""
    from dmclock_amd._abi import OPT_FORCE_RADIX, OPT_GRAPHS, OPT_SAMPLE, OPT_SMALL_K

    def mk(**kw):
        q = mk_gpu(**kw)
        if variant == "exact":
            q.set_option(OPT_SAMPLE, 0)
        elif variant == "sample_retry":
            q.set_option(OPT_SAMPLE, 2)
        elif variant == "radix":
            q.set_option(OPT_FORCE_RADIX, 1)
        elif variant == "steps":
            q.set_option(OPT_SMALL_K, 1 << 30)
        elif variant == "batched":
            q.set_option(OPT_SMALL_K, 0)
        elif variant == "eager":
            q.set_option(OPT_GRAPHS, 0)
        return q
    return mk


@pytest.mark.parametrize("kat", kats.SERVER_KATS, ids=lambda f: f.__name__)
def test_server_kat_gpu(kat):
    kat(mk_gpu)


MODES = [
    dict(at_limit=AT_LIMIT_WAIT),
    dict(at_limit=AT_LIMIT_WAIT, delayed=True),
    dict(at_limit=AT_LIMIT_ALLOW),
    dict(at_limit=AT_LIMIT_REJECT, reject_threshold=0.5),
]


@pytest.mark.parametrize("mode", MODES, ids=lambda m: "-".join(
    f"{k}={v}" for k, v in m.items()))
@pytest.mark.parametrize("seed", [1, 2])
def test_steady_trace_parity(mode, seed):
    tr = workloads.steady_trace(seed, 300, 12, 200, 150, depth=3,
                                delta_rho="random",
                                k_choices=[1, 2, 7, 40, 150, 600, 5000])
    n, _, _ = run_parity(tr, mk_gpu, mode)
    assert n > 500


@pytest.mark.parametrize("variant", ["radix", "steps", "batched", "eager"])
@pytest.mark.parametrize("mode", MODES, ids=lambda m: "-".join(
    f"{k}={v}" for k, v in m.items()))
def test_engine_paths_parity(mode, variant):
    """The three ways the engine answers pulls give the same decisions."""
    tr = workloads.steady_trace(3, 200, 8, 150, 120, depth=2,
                                delta_rho="random",
                                k_choices=[1, 3, 9, 64, 120, 2000])
    run_parity(tr, mk_variant(variant), mode)


@pytest.mark.parametrize("mode", MODES[:2], ids=["imm", "delayed"])
def test_churn_trace_parity(mode):
    tr = workloads.churn_trace(7, 300, 10, 250, 200, idle_frac=0.15,
                               k_choices=[1, 9, 64, 200, 1000])
    run_parity(tr, mk_gpu, mode, require_tie_free=False)


def test_mixed_reservation_priority_mix():
    """A trace tuned so that both phases and the R-runs after priority pops
    (reduce_reservation_tags re-exposing reservations) occur."""
    tr = workloads.steady_trace(11, 500, 15, 400, 380, depth=2,
                                table_kw=dict(frac_r=0.4, r_range=(0.2, 2.0),
                                              frac_l=0.4, l_range=(0.5, 4.0)),
                                k_choices=[380, 2000])
    n, qg, qo = run_parity(tr, mk_gpu, dict(at_limit=AT_LIMIT_WAIT))
    res, prio = qo.sched_counts()
    assert res > 100 and prio > 100


def test_non_monotone_now_ready_flags():
    """pull_request(now) with now going backwards: fronts marked ready at a
    later `now` stay ready (the flag lives on the tag, :1139)."""
    tr = workloads.steady_trace(5, 200, 6, 150, 0, depth=2,
                                table_kw=dict(frac_l=0.8, l_range=(0.3, 2.0)))
    ops = [op for op in tr.ops if op[0] == "add"]
    t_end = float(ops[-1][1]["time"][-1])
    for i, t in enumerate([t_end, t_end - 1.0, t_end + 0.5, t_end - 2.0,
                           t_end + 1.0, t_end + 3.0]):
        ops.append(("pull", t, [3, 50, 1, 200, 17, 10000][i]))
    tr.ops = ops
    run_parity(tr, mk_gpu, dict(at_limit=AT_LIMIT_WAIT))


def test_edge_empty_and_none():
    """pull on an empty queue -> none; registered clients with no requests ->
    none; limit-0 clients (limit tag -inf) with reservation r > now -> a
    future at -inf (min_not_0_time excludes only 0.0, :1192-1195)."""
    import pyoracle
    from parity import compare_decisions
    q = mk_gpu()
    assert q.pull(1.0)[0] == 2
    for qq in (q, pyoracle.OracleQueue()):
        qq.register(np.array([0, 1], np.uint32), [1.0, 1.0], [0.0, 0.0],
                    [0.0, 0.0], True)
        assert qq.pull(1.0)[0] == 2
    reqs = workloads.arrivals(np.random.default_rng(0), 2, 6, 5.0, 10.0)
    outs = []
    for qq in (q, pyoracle.OracleQueue()):
        if not isinstance(qq, type(q)):
            qq.register(np.array([0, 1], np.uint32), [1.0, 1.0], [0.0, 0.0],
                        [0.0, 0.0], True)
        qq.add_batch(reqs)
        outs.append([qq.pull_batch(now, k) for now, k in
                     ((5.0, 10), (5.5, 1), (6.0, 3), (9.0, 100))])
    for (dg, rg), (do, ro) in zip(*outs):
        compare_decisions(dg, do, "edge")
        assert (rg.n_decisions, rg.next_type) == (ro.n_decisions, ro.next_type)
        if rg.next_type == 1:
            assert np.float64(rg.when).view(np.uint64) == \
                np.float64(ro.when).view(np.uint64)


def bench_shaped_trace(seed, n_clients, n_steps, batch, depth=4):
    """bench.py's workload (BASELINE config 3) at a reduced client count:
    bulk-registered clients, `depth` requests per client, a settle pull of
    depth/2 per client at the pre-population's end, then steps of `batch`
    adds + `batch` pulls.  Its priority keys are heavily skewed (a dense
    cluster just above the reservation backlog), which is what the rank-bin
    table of k_pick exists for."""
    rng = np.random.default_rng(seed)
    tab = workloads.client_table(rng, n_clients)
    rate = 2.0 * n_clients
    tr = workloads.Trace(tab, params=dict(seed=seed))
    pre = workloads.arrivals(rng, n_clients, depth * n_clients, 1.0, rate)
    t = float(pre["time"][-1])
    tr.ops.append(("add", pre))
    tr.ops.append(("pull", t, depth * n_clients // 2))
    h = len(pre)
    for _ in range(n_steps):
        reqs = workloads.arrivals(rng, n_clients, batch, t, rate,
                                  handle_base=h)
        h += batch
        t = float(reqs["time"][-1])
        tr.ops.append(("add", reqs))
        tr.ops.append(("pull", t, batch))
    return tr


@pytest.mark.parametrize("variant", ["default", "exact", "sample_retry", "radix", "eager"])
def test_bench_shaped_parity(variant):
    """The benchmark's own key distributions, 64K clients, bit-exact: with
    the thresholds from a 1/8 sample of the first keys (default), from the
    exact histogram, and from a sample without its margin (validation fails
    and the rounds are re-run exactly: the counters show the retries)."""
    tr = bench_shaped_trace(42, 1 << 16, 4, 1 << 12)
    n, qg, qo = run_parity(tr, mk_variant(variant),
                           dict(at_limit=AT_LIMIT_WAIT), state_sample=256)
    assert n > 100000
    c = qg.counters()
    print(variant, c)
    if variant == "sample_retry":
        assert c["sample_retries"] >= 1, c
    elif variant in ("default", "exact"):
        assert c["sample_retries"] == 0, c


def test_full_size_parity_1m_clients():
    """BASELINE config 3 at its full size: 1,048,576 bulk-registered clients,
    2M pre-populated requests, a 1M-pull settle round, then two steps of
    64K adds + 64K pulls — every decision (≈1.18M) and every add status
    bit-exact against the oracle, the trace tie-free (oracle ≈13 s)."""
    tr = bench_shaped_trace(42, 1 << 20, 2, 1 << 16, depth=2)
    n, qg, qo = run_parity(tr, mk_variant("default"),
                           dict(at_limit=AT_LIMIT_WAIT), state_sample=4096)
    assert n > 1_000_000


def test_full_size_parity_1m_clients_delayed():
    """The same at full size with DelayedTagCalc (the Ceph configuration:
    tags computed at pop time, update_next_tag :1021-1036, front-only
    reductions): 1,048,576 clients, every decision and add status
    bit-exact, the trace tie-free."""
    tr = bench_shaped_trace(42, 1 << 20, 2, 1 << 16, depth=2)
    n, qg, qo = run_parity(tr, mk_variant("default"),
                           dict(at_limit=AT_LIMIT_WAIT, delayed=True), state_sample=4096)
    assert n > 1_000_000


def test_dynamic_info_rounds_64k():
    """U1 through batched rounds at 65,536 clients: 20 % of the clients get a
    fresh ClientInfo before every pull (published with
    dmc_client_bind_info_batch), delayed tags, pulls of 4096 -- every
    decision and every client's cached inverses bit-exact."""
    from dmclock_amd import workloads as wl
    tr = wl.dynamic_trace(7, 1 << 16, 4, 1 << 12, k_choices=(1 << 12,), depth=2)
    n, qg, qo = run_parity(tr, mk_gpu, dict(delayed=True, dynamic_info=True),
                           state_sample=4096, gpu_kw=dict(info_callback=False), info=True)
    assert n > 10_000, n
    assert qg.counters()["rounds"] >= 4


# ------------------------------------------------ batched activations
MODES_ACT = [dict(at_limit=AT_LIMIT_WAIT), dict(at_limit=AT_LIMIT_WAIT, delayed=True),
             dict(at_limit=AT_LIMIT_ALLOW)]


def mk_act(split):
    from dmclock_amd._abi import OPT_ACT_SPLIT

    def mk(**kw):
        q = mk_gpu(**kw)
        q.set_option(OPT_ACT_SPLIT, int(split))
        return q
    return mk


CHURN_ORACLE_SEEDS = (3, 19)


@pytest.mark.parametrize("mode", MODES_ACT, ids=["imm", "delayed", "allow"])
@pytest.mark.parametrize("seed", [3, 11, 19])
def test_churn_activations_parity(mode, seed):
    """Many activations per batch (a third of the clients idle before every
    step): the device-resolved idle resets equal the sequential ones (the
    host split, one activation at a time) in every decision and every
    client's state; and for seeds 3 and 19, verified tie-free, both equal
    the oracle (activations align proportion keys, p + L - t, so ties occur
    -- seed 11 has one -- and then the heap's history picks, SURVEY.md
    section 7)."""
    from parity import compare_decisions, compare_states
    tr = workloads.churn_trace(seed, 400, 8, 600, 300, idle_frac=0.35,
                               k_choices=[1, 9, 64, 300, 2000])
    qa = mk_act(0)(max_clients=400, **mode)
    qb = mk_act(1)(max_clients=400, **mode)
    oa, ob = workloads.replay(qa, tr), workloads.replay(qb, tr)
    for i, (a, b) in enumerate(zip(oa, ob)):
        if a[0] == "add":
            assert np.array_equal(a[1], b[1]), i
        elif a[0] == "pull":
            compare_decisions(a[1], b[1], f"op {i}")
            assert a[2] == b[2], i
    compare_states(qa, qb, np.arange(400), "final")
    import pyoracle
    qo = pyoracle.OracleQueue(**mode)
    workloads.replay(qo, tr)
    if seed in CHURN_ORACLE_SEEDS:
        # verified tie-free (checked on the CPU): the oracle leg runs
        assert qo.ties == 0, (seed, qo.ties)
        run_parity(tr, mk_act(0), mode, state_sample=400)
    else:
        # seed 11 has one tied decision under the oracle (the heap's history
        # picks among equal keys); it stays a device-vs-host-split check
        assert qo.ties > 0, seed


REJECT = dict(at_limit=AT_LIMIT_REJECT, reject_threshold=0.5)


def device_vs_split(tr, n, mode):
    """The trace on the device-resolved activations and on the host split (one
    activation at a time): every add status, decision, result and final
    client state equal.  Returns both queues and the device run's outputs."""
    from parity import compare_decisions, compare_states
    qa = mk_act(0)(max_clients=n, **mode)
    qb = mk_act(1)(max_clients=n, **mode)
    oa, ob = workloads.replay(qa, tr), workloads.replay(qb, tr)
    for i, (a, b) in enumerate(zip(oa, ob)):
        if a[0] == "add":
            assert np.array_equal(a[1], b[1]), (i, np.nonzero(a[1] != b[1]))
        elif a[0] == "pull":
            compare_decisions(a[1], b[1], f"op {i}")
            assert a[2] == b[2], i
    compare_states(qa, qb, np.arange(n), "final")
    return qa, qb, oa


@pytest.mark.parametrize("n,batch,seed,oracle", [
    (2000, 250, 1, True), (2000, 250, 2, False), (2000, 4000, 1, True),
    (2000, 4000, 4, True), (2000, 4000, 2, False)])
def test_reject_activations_parity(n, batch, seed, oracle):
    """AtLimit::Reject batches with activations resolved on the device (no
    host split): 40 % of the tenants limited far below their arrival rate,
    10 % of the clients marked idle before every step, so activating requests
    are rejected (the idle reset still applies, :937-993) and emptied clients
    see rejected requests move their proportion basis.  Every add status,
    decision and client state equals the host split's; the engine's counters
    show every activation batch resolved on the device, and exactly the
    batches the oracle's request-by-request replay finds "hard" (a rejected
    activation whose basis moves again in the batch) resolved in order by
    k_act_hard; on the tie-free seeds everything equals the oracle."""
    from parity import activation_batches
    tr = workloads.reject_churn_trace(seed, n, 6, batch, idle_frac=0.1)
    qa, qb, oa = device_vs_split(tr, n, REJECT)
    rejected = sum(int((o[1] == 11).sum()) for o in oa if o[0] == "add")
    assert rejected > 1000, rejected
    n_act, n_hard = activation_batches(tr, REJECT)
    c = qa.counters()
    print(f"n={n} batch={batch} seed={seed} rejected={rejected} predicted "
          f"{n_act}/{n_hard} counters {c['act_batches']}/{c['act_seq_batches']}")
    assert (c["act_batches"], c["act_seq_batches"]) == (n_act, n_hard), c
    assert qb.counters()["act_batches"] == 0
    if oracle:
        run_parity(tr, mk_act(0), REJECT, state_sample=n)


def test_reject_activations_64k():
    """The same at 65,536 clients with 8,192-request batches: device
    resolution equal to the host split in every output and client state,
    the in-order resolution (k_act_hard) taken (oracle leg: the CPU
    restatement's idle resets are O(N) each, 2 minutes here)."""
    n = 1 << 16
    tr = workloads.reject_churn_trace(1, n, 6, 8192, idle_frac=0.1)
    qa, qb, oa = device_vs_split(tr, n, REJECT)
    c = qa.counters()
    assert c["act_batches"] == 6 and c["act_seq_batches"] >= 1, c


def test_activation_undercut_by_earlier_activation():
    """An activated client's contribution undercuts the minimum a later
    activation sees once the former minimum client gets its first request
    (k_act_resolve's sequential fallback)."""
    from dmclock_amd._abi import make_requests
    n = 30
    slots = np.arange(n, dtype=np.uint32)
    r = np.zeros(n)
    w = np.linspace(0.6, 1.4, n)
    l = np.zeros(n)
    tr = workloads.Trace(workloads.ClientTable(slots, r, w, l, True))
    # clients 1..9 queued (contributions ~ their tags); client 0 empty with
    # prev p = 0: the initial minimum
    tr.ops.append(("add", make_requests(np.arange(1, 10), 1.0 + 0.01 * np.arange(9),
                                        handles=np.arange(9))))
    tr.ops.append(("idle", np.arange(10, 30, dtype=np.uint32)))
    order = [10, 0, 11, 12, 0, 13, 14, 15, 16, 17, 18, 19, 20]
    times = 2.0 + 0.1 * np.arange(len(order))
    tr.ops.append(("add", make_requests(order, times, handles=100 + np.arange(len(order)))))
    tr.ops.append(("pull", 5.0, 40))
    tr.ops.append(("add", make_requests(np.arange(20, 30), 6.0 + 0.03 * np.arange(10),
                                        handles=200 + np.arange(10))))
    tr.ops.append(("pull", 20.0, 100))
    # activations align keys (ties): device vs one-at-a-time host split
    from parity import compare_decisions, compare_states
    qa = mk_act(0)(max_clients=n, at_limit=AT_LIMIT_WAIT)
    qb = mk_act(1)(max_clients=n, at_limit=AT_LIMIT_WAIT)
    oa, ob = workloads.replay(qa, tr), workloads.replay(qb, tr)
    for i, (a, b) in enumerate(zip(oa, ob)):
        if a[0] == "pull":
            compare_decisions(a[1], b[1], f"op {i}")
            assert a[2] == b[2], i
        elif a[0] == "add":
            assert np.array_equal(a[1], b[1]), i
    compare_states(qa, qb, slots, "final")


@pytest.mark.parametrize("queued_frac", [1.0, 0.5, 0.05])
def test_activation_records_across_chunks(queued_frac):
    """Thousands of activations in one batch, across several 1024-entry
    chunks of k_act_resolve, where every activated client with a queued
    front behind the clock lowers the running minimum (each one a new
    minimum for the wave-stepped recurrence; queued_frac = 1 makes every
    activation one).  Device resolution equals the host split, one
    activation at a time, in every decision and every client's state."""
    from dmclock_amd._abi import make_requests
    from parity import compare_decisions, compare_states
    rng = np.random.default_rng(7)
    n = 5000
    slots = np.arange(n, dtype=np.uint32)
    r = np.where(rng.random(n) < 0.3, rng.uniform(1, 5, n), 0.0)
    w = rng.uniform(0.5, 1.5, n)
    l = np.zeros(n)
    tr = workloads.Trace(workloads.ClientTable(slots, r, w, l, True))
    # a base of non-idle clients with queued requests, and idle clients of
    # which queued_frac hold an old front far behind the later clock
    base = slots[:200]
    queued = slots[200:][rng.random(n - 200) < queued_frac]
    first = np.concatenate([base, queued])
    tr.ops.append(("add", make_requests(first, 1.0 + 1e-4 * rng.random(len(first)),
                                        handles=np.arange(len(first)))))
    tr.ops.append(("idle", slots[200:]))
    order = rng.permutation(slots[200:])
    tr.ops.append(("add", make_requests(order, 50.0 + 1e-5 * np.arange(len(order)),
                                        handles=10000 + np.arange(len(order)))))
    tr.ops.append(("pull", 60.0, 3000))
    tr.ops.append(("idle", slots[1000:4000]))
    order = rng.permutation(slots[1000:4000])
    tr.ops.append(("add", make_requests(order, 61.0 + 1e-5 * np.arange(len(order)),
                                        handles=20000 + np.arange(len(order)))))
    tr.ops.append(("pull", 70.0, 20000))
    qa = mk_act(0)(max_clients=n, at_limit=AT_LIMIT_WAIT)
    qb = mk_act(1)(max_clients=n, at_limit=AT_LIMIT_WAIT)
    oa, ob = workloads.replay(qa, tr), workloads.replay(qb, tr)
    for i, (a, b) in enumerate(zip(oa, ob)):
        if a[0] == "pull":
            compare_decisions(a[1], b[1], f"op {i}")
            assert a[2] == b[2], i
        elif a[0] == "add":
            assert np.array_equal(a[1], b[1]), i
    compare_states(qa, qb, slots, "final")


@pytest.mark.parametrize("seed", [1, 3, 5])
def test_key_range_straddles_zero(seed):
    """Forty idle clients with queued fronts are activated 100 s later: the
    idle reset gives them prop_delta ~ -600 s, so the proportion keys of the
    next pulls straddle zero and the histogram coordinates switch from
    bit-pattern offsets to the value-linear map (KeyMap, dmc_round.h) with
    binary-searched thresholds.  Tie-free; bit-exact against the oracle
    through the bin-ranked path (k = 50 / 700 / 2500)."""
    from dmclock_amd._abi import make_requests
    rng = np.random.default_rng(seed)
    tr = workloads.steady_trace(seed, 3000, 3, 1500, 0, depth=3)
    t = max(float(o[1]["time"][-1]) for o in tr.ops if o[0] == "add")
    idle = rng.choice(3000, 40, replace=False).astype(np.uint32)
    tr.ops.append(("idle", np.sort(idle)))
    tr.ops.append(("add", make_requests(idle, t + 100 + 0.37 * np.arange(40),
                                        handles=10**6 + np.arange(40))))
    t2 = t + 100 + 0.37 * 40
    for i in range(4):
        tr.ops.append(("pull", t2 + 0.5 * i, int(rng.choice([50, 700, 2500]))))
    run_parity(tr, mk_gpu, state_sample=3000)


@pytest.mark.parametrize("n", [200, 300, 500, 700, 1400])
def test_tied_rank_bins(n):
    """Massively tied keys put a round's entries into two rank bins (the tied
    first keys, and every later entry in the last bin): n = 200's first call
    ranks a 400-record bin in passes (above one k_rrank block of 256); bins
    past kBinCapR = 512 abort the round, which is re-run as a smaller round
    (k >= 4096, scaled by the largest bin) or on the radix path (then the
    next call tries the bins again); n = 1400 also emits more
    entries than the radix path's initial dense buffer holds (65,536; the
    retry is sized from the overflowed round's total, no dense overflow).  The bin-ranked,
    radix-sorted and single-step engines must give the same decisions bit
    for bit (ties broken by lowest slot), and the engine counters show which
    path each round took."""
    from dmclock_amd._abi import REQUEST_DTYPE
    ctrs = {}

    def run(variant):
        q = mk_variant(variant)(max_clients=max(1024, n))
        slots = np.arange(n, dtype=np.uint32)
        q.register_active(slots, np.zeros(n), np.ones(n), np.zeros(n))
        out = []
        depth = 3 if n <= 700 else 48
        for call in range(3):
            reqs = np.zeros(depth * n, REQUEST_DTYPE)
            reqs["slot"] = np.tile(slots, depth)
            reqs["cost"] = 1
            reqs["time"] = 1.0 + call
            reqs["delta"] = 1
            reqs["rho"] = 1
            reqs["handle"] = np.arange(depth * n) + call * depth * n
            rc = q.add_batch(reqs)
            assert (rc == 0).all()
            k = 2 * n + 7 if n <= 700 else 40 * n
            d, res = q.pull_batch(10.0 + call, k)
            assert res.n_decisions == k
            out.append(d[:res.n_decisions].copy())
        ctrs[variant] = q.counters()
        q.close()
        return np.concatenate(out)

    base = run("default")
    c = ctrs["default"]
    print(f"n={n} counters {c}")
    # the first keys tie in one bin and every later entry lands in the last
    # rank bin of the threshold's histogram bin: as the queues deepen over
    # the three calls that bin outgrows its 512 records and the round is
    # re-run on the radix path, its dense buffer sized from the overflowed
    # round (no dense overflow)
    assert c["bin_overflows"] >= 1, c
    assert c["radix_rounds"] + c["bin_splits"] >= c["bin_overflows"], c
    assert c["radix_rounds"] >= 1, c  # (tied keys: a smaller round ties as well)
    assert c["dense_overflows"] == 0, c
    if n == 200:
        # the first call's last bin holds 400 records: ranked in passes of
        # one record per thread (above one k_rrank block of 256)
        assert c["max_bin"] > 256, c
    assert (base["flags"] != 0).mean() > 0.5  # tied and flagged
    assert base.tobytes() == run("radix").tobytes()
    if n > 700:
        return  # the single-step variant would take 40 x n general steps
    # single steps flag a tie among the fronts of one pull, not a round's
    # entries: every other field must match
    steps = run("steps")
    for f in ("handle", "tag_r", "tag_p", "tag_l", "slot", "cost", "phase"):
        assert base[f].tobytes() == steps[f].tobytes(), f
