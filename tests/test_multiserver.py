"""Multi-server dmClock with epoch-delivered client trackers (BASELINE config
5).

CPU: the epoch restatement (oracle/epoch_tracker.py) equals the sequential
ServiceTracker<S, OrigTracker> restatement (oracle pyoracle.Tracker) driven
with the same calls; the per-rank sums combined with a world-size-2 gloo
all-reduce equal the single-process sums.
GPU: the device trackers equal the restatement bit for bit, and S server
queues driven by them make the same decisions as S oracle queues driven by
the restatement.
"""
import os
import sys

import numpy as np
import pytest

import pyoracle
from epoch_tracker import EpochTrackers
from dmclock_amd import workloads
from dmclock_amd._abi import DECISION_DTYPE, REQUEST_DTYPE


def epoch_batches(rng, n_servers, n_clients, n_epochs, per_server, t0=1.0,
                  rate=None):
    """Per epoch, per server: a batch of requests (Poisson arrivals over all
    clients), delta/rho left for the trackers."""
    rate = rate or 2.0 * n_clients
    t = t0
    h = 0
    out = []
    for _ in range(n_epochs):
        ep = []
        for _s in range(n_servers):
            r = workloads.arrivals(rng, n_clients, per_server, t, rate, handle_base=h)
            h += per_server
            ep.append(r)
        t = max(float(b["time"][-1]) for b in ep)
        out.append((t, ep))
    return out


def client_maps(rng, n_servers, n_slots, n_clients):
    """each server table: n_slots distinct global clients in random order"""
    return np.stack([rng.permutation(n_clients)[:n_slots] for _ in range(n_servers)])


@pytest.mark.parametrize("mapped", [False, True])
def test_epoch_restatement_matches_sequential_tracker(mapped):
    rng = np.random.default_rng(3)
    S, N = 3, 40
    G = 70 if mapped else N
    cmap = client_maps(rng, S, N, G) if mapped else np.tile(np.arange(N), (S, 1))
    et = EpochTrackers(S, N, G, cmap if mapped else None)
    seq = [pyoracle.Tracker("orig") for _ in range(G)]
    for epoch in range(6):
        batches = []
        for s in range(S):
            reqs = np.zeros(rng.integers(5, 60), dtype=REQUEST_DTYPE)
            reqs["slot"] = rng.integers(0, N, len(reqs))
            et.fill(s, reqs)
            for i in range(len(reqs)):
                d, r = seq[cmap[s, reqs["slot"][i]]].get_req_params(s)
                assert (d, r) == (reqs["delta"][i], reqs["rho"][i]), (epoch, s, i)
            batches.append(reqs)
        for s in range(S):
            n = len(batches[s])
            dec = np.zeros(n, dtype=DECISION_DTYPE)
            dec["slot"] = batches[s]["slot"]
            dec["cost"] = rng.integers(1, 4, n)
            dec["phase"] = rng.integers(0, 2, n)
            et.tally(s, dec)
            for x in dec:
                seq[cmap[s, x["slot"]]].track_resp(s, int(x["phase"]), int(x["cost"]))
        et.deliver()


def test_lagged_restatement_matches_sequential_tracker():
    """The overlapped exchange (lag=True): epoch e's responses reach the
    clients at boundary e + 1, i.e. the sequential ServiceTracker receives
    its track_resp calls one epoch late -- otherwise the same arithmetic
    (dmclock_client.h:221-251); finish() flushes the last epoch."""
    rng = np.random.default_rng(4)
    S, N, G = 3, 40, 70
    cmap = client_maps(rng, S, N, G)
    et = EpochTrackers(S, N, G, cmap, lag=True)
    seq = [pyoracle.Tracker("orig") for _ in range(G)]
    held = []  # the responses of the epoch whose delivery is pending
    asked = [[] for _ in range(S)]
    for epoch in range(7):
        for s in range(S):
            reqs = np.zeros(rng.integers(5, 60), dtype=REQUEST_DTYPE)
            reqs["slot"] = rng.integers(0, N, len(reqs))
            asked[s] = sorted(set(asked[s]) | set(reqs["slot"].tolist()))
            et.fill(s, reqs)
            for i in range(len(reqs)):
                d, r = seq[cmap[s, reqs["slot"][i]]].get_req_params(s)
                assert (d, r) == (reqs["delta"][i], reqs["rho"][i]), (epoch, s, i)
        cur = []
        for s in range(S):
            # (responses answer requests: the slots this server was asked by)
            n = int(rng.integers(5, 40))
            dec = np.zeros(n, dtype=DECISION_DTYPE)
            dec["slot"] = rng.choice(asked[s], n)
            dec["cost"] = rng.integers(1, 4, n)
            dec["phase"] = rng.integers(0, 2, n)
            et.tally(s, dec)
            cur += [(s, x) for x in dec]
        et.deliver()
        for s, x in held:  # the previous epoch's responses arrive now
            seq[cmap[s, x["slot"]]].track_resp(s, int(x["phase"]), int(x["cost"]))
        held = cur
    et.finish()
    for s, x in held:
        seq[cmap[s, x["slot"]]].track_resp(s, int(x["phase"]), int(x["cost"]))
    for s in range(S):  # one more request each: every counter delivered
        for slot in range(N):
            reqs = np.zeros(1, dtype=REQUEST_DTYPE)
            reqs["slot"] = slot
            et.fill(s, reqs)
            d, r = seq[cmap[s, slot]].get_req_params(s)
            assert (d, r) == (reqs["delta"][0], reqs["rho"][0]), (s, slot)


def _gloo_worker(rank, world, port, q, lag=False):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(11)
        S_total, N = 4, 64
        S = S_total // world
        et = EpochTrackers(S, N, lag=lag)
        for epoch in range(4):
            for s in range(S):
                gs = rank * S + s
                r2 = np.random.default_rng(100 * epoch + gs)
                dec = np.zeros(50, dtype=DECISION_DTYPE)
                dec["slot"] = r2.integers(0, N, 50)
                dec["cost"] = r2.integers(1, 4, 50)
                dec["phase"] = r2.integers(0, 2, 50)
                et.tally(s, dec)
            sd, sr = et.local_sums()
            both = torch.from_numpy(np.stack([sd, sr]).view(np.int32).copy())
            dist.all_reduce(both, op=dist.ReduceOp.SUM)
            allr = both.numpy().view(np.uint32)
            et.deliver(allr[0], allr[1])
        et.finish()
        q.put((rank, et.gd.copy(), et.gr.copy(), et.xd.copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("lag", [False, True])
def test_epoch_allreduce_gloo_world2(lag):
    """Per-rank sums + all-reduce == one process holding every server (both
    delivery schedules)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port + int(lag), q, lag))
             for r in range(2)]
    for p in procs:
        p.start()
    res = dict()
    for _ in procs:
        rank, gd, gr, xd = q.get(timeout=120)
        res[rank] = (gd, gr, xd)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single process, all 4 servers
    S_total, N = 4, 64
    et = EpochTrackers(S_total, N, lag=lag)
    for epoch in range(4):
        for gs in range(S_total):
            r2 = np.random.default_rng(100 * epoch + gs)
            dec = np.zeros(50, dtype=DECISION_DTYPE)
            dec["slot"] = r2.integers(0, N, 50)
            dec["cost"] = r2.integers(1, 4, 50)
            dec["phase"] = r2.integers(0, 2, 50)
            et.tally(gs, dec)
        et.deliver()
    et.finish()
    for rank in (0, 1):
        gd, gr, xd = res[rank]
        assert np.array_equal(gd, et.gd) and np.array_equal(gr, et.gr)
        assert np.array_equal(xd, et.xd[rank * 2:(rank + 1) * 2])


@pytest.mark.gpu
def test_device_trackers_and_multiserver_parity():
    """S GPU server queues + device trackers vs S oracle queues + the
    restatement: bit-exact delta/rho, decisions and tracker state."""
    import torch
    from dmclock_amd.multiserver import DeviceTrackers, make_queues
    from parity import compare_decisions
    S, N, G = 4, 300, 500
    rng = np.random.default_rng(5)
    cmap = client_maps(rng, S, N, G)
    tab = workloads.client_table(rng, N)
    qg = make_queues(S, N, device=0, ring_capacity=64)
    qo = [pyoracle.OracleQueue() for _ in range(S)]
    for q in qg + qo:
        q.register(tab.slots, tab.r, tab.w, tab.l, True)
    dev = torch.device("cuda", 0)
    dt = DeviceTrackers(qg, N, dev, n_clients=G, client_of_slot=cmap)
    et = EpochTrackers(S, N, G, cmap)
    n_dec = 0
    for t, ep in epoch_batches(rng, S, N, n_epochs=6, per_server=250):
        for s in range(S):
            reqs = ep[s].copy()
            d_reqs = torch.from_numpy(reqs.view(np.uint8)).to(dev)
            dt.fill(s, d_reqs.data_ptr(), len(reqs))
            qg[s].sync()
            got = d_reqs.cpu().numpy().view(REQUEST_DTYPE)
            et.fill(s, reqs)
            assert np.array_equal(got["delta"], reqs["delta"])
            assert np.array_equal(got["rho"], reqs["rho"])
            rc_g = qg[s].add_batch(got)
            rc_o = qo[s].add_batch(reqs)
            assert np.array_equal(rc_g, rc_o)
        for s in range(S):
            k = 200
            d_out = torch.zeros(k * DECISION_DTYPE.itemsize, dtype=torch.uint8, device=dev)
            d_res = torch.zeros(24, dtype=torch.uint8, device=dev)
            qg[s].pull_batch_device(t, k, d_out.data_ptr(), d_res.data_ptr())
            dt.tally(s, d_out.data_ptr(), d_res.data_ptr(), k)
            qg[s].sync()
            from dmclock_amd._abi import PullResult
            res = PullResult.from_buffer_copy(d_res.cpu().numpy().tobytes())
            dg = d_out.cpu().numpy().view(DECISION_DTYPE)[:res.n_decisions]
            do, ro = qo[s].pull_batch(t, k)
            compare_decisions(dg, do, f"server {s}")
            et.tally(s, do)
            n_dec += len(do)
        dt.deliver()
        et.deliver()
        st = dt.state()
        for f in ("gd", "gr", "xd", "xr", "known"):
            assert np.array_equal(st[f], getattr(et, f)), f
    assert n_dec > 1000


# ---------------------------------------------------- world size 2 on the GPU
W2 = dict(S_total=4, N=300, G=500, epochs=5, per_server=250, k=200, seed=9)


def _w2_workload():
    """the same global workload in every process: maps, table, batches"""
    rng = np.random.default_rng(W2["seed"])
    cmap = client_maps(rng, W2["S_total"], W2["N"], W2["G"])
    tab = workloads.client_table(rng, W2["N"])
    eps = epoch_batches(rng, W2["S_total"], W2["N"], W2["epochs"], W2["per_server"])
    return cmap, tab, eps


def _device_trackers_worker(rank, world, port, out_q, backend="gloo", lagged=False,
                            grouped=False):
    """One rank: servers [rank * S, (rank + 1) * S) as GPU queues on cuda:0
    with DeviceTrackers, the per-epoch delivery all-reducing over `backend`
    (the product's DeviceTrackers.deliver: host-staged under gloo, on the
    device buffers under nccl = RCCL)."""
    import torch
    import torch.distributed as dist
    from dmclock_amd._abi import PullResult
    from dmclock_amd.multiserver import DeviceTrackers, make_queues
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        cmap, tab, eps = _w2_workload()
        S = W2["S_total"] // world
        mine = list(range(rank * S, (rank + 1) * S))
        qg = make_queues(S, W2["N"], device=0, ring_capacity=64)
        for q in qg:
            q.register(tab.slots, tab.r, tab.w, tab.l, True)
        dt = DeviceTrackers(qg, W2["N"], dev, n_clients=W2["G"],
                            client_of_slot=cmap[mine], lagged=lagged)
        gg = None
        if grouped:  # (the members on a group's stream, the sums on its side stream)
            from dmclock_amd.multiserver import GpuGroup
            gg = GpuGroup(qg)
            dt.attach_group(gg)
        decs = []
        k = W2["k"]
        for t, ep in eps:
            for j, s in enumerate(mine):
                reqs = ep[s].copy()
                d_reqs = torch.from_numpy(reqs.view(np.uint8)).to(dev)
                torch.cuda.synchronize()
                dt.fill(j, d_reqs.data_ptr(), len(reqs))
                qg[j].sync()
                got = d_reqs.cpu().numpy().view(REQUEST_DTYPE).copy()
                rc = qg[j].add_batch(got)
                assert (rc == 0).all()
                decs.append(("req", s, got["delta"].copy(), got["rho"].copy()))
            for j, s in enumerate(mine):
                d_out = torch.zeros(k * DECISION_DTYPE.itemsize, dtype=torch.uint8,
                                    device=dev)
                d_res = torch.zeros(24, dtype=torch.uint8, device=dev)
                torch.cuda.synchronize()
                qg[j].pull_batch_device(t, k, d_out.data_ptr(), d_res.data_ptr())
                dt.tally(j, d_out.data_ptr(), d_res.data_ptr(), k)
                qg[j].sync()
                res = PullResult.from_buffer_copy(d_res.cpu().numpy().tobytes())
                dg = d_out.cpu().numpy().view(DECISION_DTYPE)[:res.n_decisions].copy()
                decs.append(("dec", s, dg))
            dt.deliver()
        dt.finish()
        st = dt.state()
        out_q.put((rank, st, decs, dt.allreduce_ms))
        if gg is not None:
            gg.close()
        for q in qg:
            q.close()
    finally:
        dist.destroy_process_group()


def _oracle_reference(world, lag=False):
    """all four servers on the oracle with the epoch restatement"""
    cmap, tab, eps = _w2_workload()
    S_total, N, G, k = W2["S_total"], W2["N"], W2["G"], W2["k"]
    qo = [pyoracle.OracleQueue() for _ in range(S_total)]
    for q in qo:
        q.register(tab.slots, tab.r, tab.w, tab.l, True)
    et = EpochTrackers(S_total, N, G, cmap, lag=lag)
    want = {}
    for e, (t, ep) in enumerate(eps):
        for s in range(S_total):
            reqs = ep[s].copy()
            et.fill(s, reqs)
            want[("req", e, s)] = (reqs["delta"].copy(), reqs["rho"].copy())
            assert (qo[s].add_batch(reqs) == 0).all()
        for s in range(S_total):
            do, _ = qo[s].pull_batch(t, k)
            et.tally(s, do)
            want[("dec", e, s)] = do
        et.deliver()
    et.finish()
    return eps, et, want


@pytest.mark.gpu
@pytest.mark.parametrize("lagged,grouped", [(False, False), (True, False), (True, True)])
def test_device_trackers_world1_rccl(lagged, grouped):
    """The RCCL branch of DeviceTrackers.deliver: one rank on GPU 0 in an
    `nccl` (RCCL) process group holding all four servers -- every epoch's
    all-reduce runs through RCCL on the device buffers (the identity at
    world size 1; the 8-GPU runs reduce over xGMI) -- against the oracle
    queues with the epoch restatement: every request's delta/rho, every
    decision and the final tracker state bit-exact.  grouped: the queues in a
    GpuGroup with the trackers attached -- each epoch's sums on the group's
    side stream, the RCCL all-reduce waiting for it on the device."""
    import torch.multiprocessing as mp
    from parity import compare_decisions
    ctx = mp.get_context("spawn")
    out_q = ctx.Queue()
    port = 31500 + os.getpid() % 1000
    p = ctx.Process(target=_device_trackers_worker,
                    args=(0, 1, port + int(lagged) + 2 * int(grouped), out_q, "nccl", lagged,
                          grouped))
    p.start()
    try:
        rank, st, decs, ar_ms = out_q.get(timeout=240)
    finally:
        p.join(timeout=60)
    assert p.exitcode == 0
    if lagged:  # the overlapped all-reduce ran (and was timed) every epoch
        assert len(ar_ms) == W2["epochs"], ar_ms
    eps, et, want = _oracle_reference(1, lag=lagged)
    n_dec = 0
    it = iter(decs)
    S = W2["S_total"]
    for e in range(len(eps)):
        for _ in range(S):
            kind, s, d, r = next(it)
            wd, wr = want[("req", e, s)]
            assert np.array_equal(d, wd) and np.array_equal(r, wr), (e, s)
        for _ in range(S):
            kind, s, dg = next(it)
            compare_decisions(dg, want[("dec", e, s)], f"epoch {e} server {s}")
            n_dec += len(dg)
    for f in ("gd", "gr", "xd", "xr", "known"):
        assert np.array_equal(st[f], getattr(et, f)), f
    assert n_dec > 1000


@pytest.mark.gpu
@pytest.mark.parametrize("lagged,grouped", [(False, False), (True, False), (True, True)])
def test_device_trackers_world2_gloo(lagged, grouped):
    """Two ranks sharing GPU 0, two server queues each, device trackers with
    the per-epoch all-reduce of DeviceTrackers.deliver over gloo: every
    request's delta/rho, every decision and the final tracker state equal one
    process running all four oracle queues with the epoch restatement
    (grouped: each rank's queues in a GpuGroup, the sums on its side
    stream, joined before the host-staged all-reduce)."""
    import torch.multiprocessing as mp
    from parity import compare_decisions
    ctx = mp.get_context("spawn")
    out_q = ctx.Queue()
    port = 30500 + os.getpid() % 1000
    procs = [ctx.Process(target=_device_trackers_worker,
                         args=(r, 2, port + int(lagged) + 2 * int(grouped), out_q, "gloo",
                               lagged, grouped))
             for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in procs:
            rank, st, decs, _ = out_q.get(timeout=240)
            res[rank] = (st, decs)
    finally:
        for p in procs:
            p.join(timeout=60)
    for p in procs:
        assert p.exitcode == 0
    # one process: all four servers on the oracle, epoch restatement
    cmap, tab, eps = _w2_workload()
    S_total, N, G, k = W2["S_total"], W2["N"], W2["G"], W2["k"]
    qo = [pyoracle.OracleQueue() for _ in range(S_total)]
    for q in qo:
        q.register(tab.slots, tab.r, tab.w, tab.l, True)
    et = EpochTrackers(S_total, N, G, cmap, lag=lagged)
    want = {}
    for e, (t, ep) in enumerate(eps):
        for s in range(S_total):
            reqs = ep[s].copy()
            et.fill(s, reqs)
            want[("req", e, s)] = (reqs["delta"].copy(), reqs["rho"].copy())
            assert (qo[s].add_batch(reqs) == 0).all()
        for s in range(S_total):
            do, _ = qo[s].pull_batch(t, k)
            et.tally(s, do)
            want[("dec", e, s)] = do
        et.deliver()
    et.finish()
    n_dec = 0
    for rank, (st, decs) in res.items():
        S = S_total // 2
        it = iter(decs)
        for e in range(len(eps)):
            for _ in range(S):
                kind, s, d, r = next(it)
                wd, wr = want[("req", e, s)]
                assert np.array_equal(d, wd) and np.array_equal(r, wr), (rank, e, s)
            for _ in range(S):
                kind, s, dg = next(it)
                compare_decisions(dg, want[("dec", e, s)], f"rank {rank} epoch {e} server {s}")
                n_dec += len(dg)
        assert np.array_equal(st["gd"], et.gd) and np.array_equal(st["gr"], et.gr)
        sl = slice(rank * S, (rank + 1) * S)
        for f in ("xd", "xr", "known"):
            assert np.array_equal(st[f], getattr(et, f)[sl]), (rank, f)
    assert n_dec > 1000
