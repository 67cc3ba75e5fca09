"""The deterministic dmc_sim equivalent (dmclock_amd/sim.py): BASELINE
configs 1 and 2.

CPU: the INI reader on the reference's own config files (tests/golden/), the
product ServiceTracker against the oracle's tracker restatement, determinism
and completion of the virtual-time driver on oracle queues (config 1 hangs in
the reference: its sched-ahead timer never fires on time).
GPU: the driver on HIP queues equals the driver on oracle queues -- every
request's delta/rho, every server's dispatch sequence (client, phase, cost,
handle, tag bits) and every stopping pull -- on tie-free runs: the whole
dmc_sim_100th.conf run (BASELINE config 2: 100 servers, 100 clients, 100,000
requests; the oracle gives 79,158 reservation / 20,842 priority decisions,
the reference's wall-clock run 79,373 / 20,627) and config 1.
"""
import os

import numpy as np
import pytest

import pyoracle
from dmclock_amd import sim
from dmclock_amd.tracker import ServiceTracker

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
CONF_100TH = os.path.join(GOLDEN, "dmc_sim_100th.conf")
CONF_EXAMPLE = os.path.join(GOLDEN, "dmc_sim_example.conf")


def test_load_conf_reference_files():
    c = sim.load_conf(CONF_100TH)
    assert (c.server_groups, c.client_groups) == (1, 2)
    assert c.server_random_selection and c.server_soft_limit
    assert [g.client_count for g in c.cli_group] == [99, 1]
    assert [g.client_wait for g in c.cli_group] == [0, 10]
    g = c.cli_group[0]
    assert (g.client_total_ops, g.client_server_select_range, g.client_iops_goal,
            g.client_outstanding_ops) == (1000, 10, 50, 100)
    assert (g.client_reservation, g.client_limit, g.client_weight) == (20.0, 60.0, 1.0)
    s = c.srv_group[0]
    assert (s.server_count, s.server_iops, s.server_threads) == (100, 40, 1)
    e = sim.load_conf(CONF_EXAMPLE)
    assert not e.server_random_selection and not e.server_soft_limit
    assert [g.client_limit for g in e.cli_group] == [0.0, 40.0, 50.0, 50.0]
    assert [g.client_req_cost for g in e.cli_group] == [1, 1, 1, 3]  # config.h default 1
    assert e.srv_group[0].server_iops == 160


@pytest.mark.parametrize("kind", ["orig", "borrow"])
def test_service_tracker_matches_oracle(kind):
    rng = np.random.default_rng(4)
    a = ServiceTracker(kind)
    b = pyoracle.Tracker(kind)
    for _ in range(3000):
        s = int(rng.integers(0, 6))
        if rng.random() < 0.5:
            assert a.get_req_params(s) == b.get_req_params(s)
        else:
            ph, cost = int(rng.integers(0, 2)), int(rng.integers(1, 4))
            a.track_resp(s, ph, cost)
            b.track_resp(s, ph, cost)


def _oracle_mk(at_limit, antic):
    return pyoracle.OracleQueue(at_limit=at_limit, anticipation=antic)


def _run(conf, mk, ops, seed=7):
    return sim.Simulation(conf, mk, seed=seed, ops_per_client=ops).run(
        max_events=10_000_000)


def _digest(s):
    dec = [[(t, int(r["slot"]), int(r["phase"]), int(r["cost"]), int(r["handle"]),
             float(r["tag_r"]), float(r["tag_p"]), float(r["tag_l"]))
            for t, r in lg] for lg in s.log_dec]
    return dec, list(s.log_req), [list(x) for x in s.log_stop]


def test_sim_deterministic_and_complete_on_oracle():
    conf = sim.load_conf(CONF_100TH)
    a = _run(conf, _oracle_mk, 15)
    b = _run(conf, _oracle_mk, 15)
    assert _digest(a) == _digest(b)
    st = a.stats()
    assert st["requests"] == 100 * 15
    assert int(st["reservation_ops"].sum() + st["priority_ops"].sum()) == 100 * 15
    assert sum(s.q.ties for s in a.servers) == 0
    # every request was answered: trackers saw one response per request
    assert all(c.outstanding == 0 for c in a.clients)


def test_sim_example_conf_completes_with_limits():
    """BASELINE config 1 (the reference binary hangs on it, SURVEY finding 5):
    completes, and the limited clients stay within their limits."""
    conf = sim.load_conf(CONF_EXAMPLE)
    s = _run(conf, _oracle_mk, None)  # the conf's 2,000 ops per client
    st = s.stats()
    assert st["requests"] == 4 * 2000
    assert int(st["reservation_ops"].sum() + st["priority_ops"].sum()) == 8000
    assert sum(x.q.ties for x in s.servers) == 0
    # client 1: limit 40 ops/s under AtLimit::Wait
    times = [t for t, r in s.log_dec[0] if int(r["slot"]) == 1]
    span = times[-1] - times[0]
    assert (len(times) - 1) / span <= 40.0 * 1.001


@pytest.mark.gpu
@pytest.mark.parametrize("conf_path,ops", [(CONF_100TH, None), (CONF_EXAMPLE, None)],
                         ids=["config2_100th_full", "config1_example"])
def test_sim_replay_parity_gpu(conf_path, ops):
    from dmclock_amd.gpu import GpuQueue
    conf = sim.load_conf(conf_path)
    ncl = sum(g.client_count for g in conf.cli_group)

    def gpu_mk(at_limit, antic):
        return GpuQueue(max_clients=ncl, ring_capacity=64, max_batch=1024,
                        at_limit=at_limit, anticipation=antic)

    o = _run(conf, _oracle_mk, ops)
    assert sum(s.q.ties for s in o.servers) == 0
    g = _run(conf, gpu_mk, ops)
    do, ro, so = _digest(o)
    dg, rg, sg = _digest(g)
    assert rg == ro  # every request: time, client, server, delta, rho
    for s in range(len(do)):
        assert dg[s] == do[s], f"server {s}"
    assert sg == so
    if conf_path == CONF_100TH:  # the whole config-2 run: 100 servers x 100 clients x 1000 ops
        st = g.stats()
        assert st["requests"] == 100_000
        print("config2 replay: reservation", int(st["reservation_ops"].sum()),
              "priority", int(st["priority_ops"].sum()),
              "virtual seconds", round(st["end_time"] - g.t0, 3))
