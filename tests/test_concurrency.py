"""Concurrent server queues on one GPU: BASELINE config 5's per-GPU shape
("next" item 1).

Several server queues, each driven from its own host thread on its own HIP
stream with no synchronisation between its calls, in a process started with
GPU_MAX_HW_QUEUES=8 so that every queue's stream has a hardware queue of its
own (true cross-queue concurrency: the configuration whose settle pulls
faulted in round 2).  Per server, as bench_multiserver.py drives it:
pre-population through the device trackers (dmc_tracker_fill, then
dmc_add_batch_device), one settle call of k = 2^20 pulls (four rounds of
2^18), then epochs of fused add + pull steps with every decision tallied and
the epoch delivery (collect, all-reduce, advance) -- gloo between two ranks
in the world-2 variant.  Every request's delta/rho, every decision (client,
phase, cost, handle, tag bits), every result record and the final tracker
state are compared with oracle queues driven by the epoch restatement
(oracle/epoch_tracker.py; reference: sim/src/simulate.h:118-136,
src/dmclock_client.h:59-79, src/dmclock_server.h:1115-1186).
"""
import os
import tempfile
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import pyoracle
from epoch_tracker import EpochTrackers
from dmclock_amd import workloads
from dmclock_amd._abi import DECISION_DTYPE, REQUEST_DTYPE

pytestmark = pytest.mark.gpu

SHAPE = dict(S_total=4, N=1 << 18, G=1 << 19, depth=6, settle=1 << 20, epochs=3,
             steps=2, batch=1 << 14, seed=21, chunk=1 << 19)


def workload(sh):
    """client table, server maps and, per server, the pre-population chunks
    and the step batches (delta/rho left for the trackers)"""
    rng = np.random.default_rng(sh["seed"])
    S, N, G = sh["S_total"], sh["N"], sh["G"]
    tab = workloads.client_table(rng, N)
    cmap = np.stack([rng.permutation(G)[:N] for _ in range(S)]).astype(np.int32)
    srv = []
    for s in range(S):
        r2 = np.random.default_rng([sh["seed"], s])
        pre = workloads.arrivals(r2, N, sh["depth"] * N, 1.0, 2.0 * N)
        t = float(pre["time"][-1])
        chunks = [pre[i:i + sh["chunk"]].copy() for i in range(0, len(pre), sh["chunk"])]
        steps = []
        h = len(pre)
        for _ in range(sh["epochs"] * sh["steps"]):
            b = workloads.arrivals(r2, N, sh["batch"], t, 2.0 * N, handle_base=h)
            h += sh["batch"]
            t = float(b["time"][-1])
            steps.append(b)
        srv.append((chunks, t_pre_of(chunks), steps))
    return tab, cmap, srv


def t_pre_of(chunks):
    return float(chunks[-1]["time"][-1])


def _rank(rank, world, port, sh, outdir, out_q):
    """One process: servers [rank * S, (rank + 1) * S), one host thread per
    queue, device trackers, gloo delivery when world > 1."""
    import torch
    from dmclock_amd.multiserver import DeviceTrackers, make_queues
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        tab, cmap, srv = workload(sh)
        S = sh["S_total"] // world
        mine = list(range(rank * S, (rank + 1) * S))
        N, k = sh["N"], sh["batch"]
        qs = make_queues(S, N, device=0, ring_capacity=64, max_batch=sh["chunk"])
        trk = DeviceTrackers(qs, N, dev, n_clients=sh["G"], client_of_slot=cmap[mine])
        group = None
        if sh.get("group"):
            from dmclock_amd.multiserver import GpuGroup
            group = GpuGroup(qs)  # (members run on the group's stream from here)
        # every device buffer lives to the end: no call waits for another
        d_pre = [[torch.from_numpy(c.view(np.uint8)).to(dev) for c in srv[s][0]]
                 for s in mine]
        d_steps = [[torch.from_numpy(b.view(np.uint8)).to(dev) for b in srv[s][2]]
                   for s in mine]
        d_rc = [torch.zeros(sh["chunk"], dtype=torch.int32, device=dev) for _ in mine]
        d_set = [torch.zeros(sh["settle"] * DECISION_DTYPE.itemsize, dtype=torch.uint8,
                             device=dev) for _ in mine]
        n_steps = sh["epochs"] * sh["steps"]
        d_out = [[torch.zeros(k * DECISION_DTYPE.itemsize, dtype=torch.uint8, device=dev)
                  for _ in range(n_steps)] for _ in mine]
        d_res = torch.zeros((S, n_steps + 1, 24), dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        rc_bad = [0] * S

        def prepare(j):
            q = qs[j]
            q.register_active(tab.slots, tab.r, tab.w, tab.l)
            for c, d in zip(srv[mine[j]][0], d_pre[j]):
                trk.fill(j, d.data_ptr(), len(c))
                q.add_batch_device(d.data_ptr(), len(c), d_rc[j].data_ptr())
                q.sync()  # (the status readback below runs on torch's stream)
                rc_bad[j] += int((d_rc[j][:len(c)] != 0).sum())
            t_pre = srv[mine[j]][1]
            q.pull_batch_device(t_pre, sh["settle"], d_set[j].data_ptr(),
                                d_res[j, n_steps].data_ptr())
            trk.tally(j, d_set[j].data_ptr(), d_res[j, n_steps].data_ptr(), sh["settle"])
            q.sync()

        def run_group(i0, i1):
            gtrk = trk.group_trackers()
            for i in range(i0, i1):
                bs = [srv[mine[j]][2][i] for j in range(S)]
                group.step(len(bs[0]), [d_steps[j][i].data_ptr() for j in range(S)],
                           [d_rc[j].data_ptr() for j in range(S)],
                           [float(b["time"][-1]) for b in bs], k,
                           [d_out[j][i].data_ptr() for j in range(S)],
                           [d_res[j, i].data_ptr() for j in range(S)], gtrk)
            qs[0].sync()

        def run(j, i0, i1):
            q = qs[j]
            for i in range(i0, i1):
                b = srv[mine[j]][2][i]
                trk.fill(j, d_steps[j][i].data_ptr(), len(b))
                q.add_pull_batch_device(d_steps[j][i].data_ptr(), len(b), d_rc[j].data_ptr(),
                                        float(b["time"][-1]), k, d_out[j][i].data_ptr(),
                                        d_res[j, i].data_ptr())
                trk.tally(j, d_out[j][i].data_ptr(), d_res[j, i].data_ptr(), k)
            q.sync()

        with ThreadPoolExecutor(S) as pool:
            list(pool.map(prepare, range(S)))
            trk.deliver()
            # (the deep settle rounds may overflow rank bins and re-run on
            # the radix path; the steps' counters start here)
            settle_ctr = [q.counters(reset=True) for q in qs]
            for e in range(sh["epochs"]):
                i0 = e * sh["steps"]
                if group is not None:
                    run_group(i0, i0 + sh["steps"])
                else:
                    list(pool.map(lambda j: run(j, i0, i0 + sh["steps"]), range(S)))
                trk.deliver()
        torch.cuda.synchronize()
        assert sum(rc_bad) == 0, rc_bad
        st = trk.state()
        res = d_res.cpu().numpy()
        for j, s in enumerate(mine):
            out = {"settle": d_set[j].cpu().numpy(), "res": res[j]}
            # (requests: only the delta / rho the trackers filled in)
            for ci, d in enumerate(d_pre[j]):
                out[f"pre{ci}"] = _dr(d.cpu().numpy().view(REQUEST_DTYPE))
            for i in range(n_steps):
                out[f"req{i}"] = _dr(d_steps[j][i].cpu().numpy().view(REQUEST_DTYPE))
                out[f"dec{i}"] = d_out[j][i].cpu().numpy()
            for f in ("xd", "xr", "known"):
                out[f] = st[f][j]
            out["gd"], out["gr"] = st["gd"], st["gr"]
            c = qs[j].counters()
            out["counters"] = np.array([c["radix_rounds"], c["rounds"],
                                        settle_ctr[j]["rounds"],
                                        settle_ctr[j]["radix_rounds"], c["fused_calls"]])
            np.savez(os.path.join(outdir, f"srv{s}.npz"), **out)
        if group is not None:
            group.close()
        for q in qs:
            q.close()
        out_q.put((rank, "ok"))
    except BaseException as e:  # reported to the parent
        out_q.put((rank, repr(e)))
        raise
    finally:
        if dist:
            dist.destroy_process_group()


def _dr(reqs):
    """a batch's delta and rho columns"""
    return np.stack([reqs["delta"], reqs["rho"]])


def oracle_run(sh):
    """all servers on oracle queues + the epoch restatement, the same call
    sequence per server (threads: ctypes releases the GIL in the oracle)"""
    tab, cmap, srv = workload(sh)
    S, N, k = sh["S_total"], sh["N"], sh["batch"]
    et = EpochTrackers(S, N, sh["G"], cmap)
    qo = [pyoracle.OracleQueue() for _ in range(S)]
    want = [dict() for _ in range(S)]

    def prepare(s):
        qo[s].register(tab.slots, tab.r, tab.w, tab.l, True)
        for ci, c in enumerate(srv[s][0]):
            c = c.copy()
            et.fill(s, c)
            want[s][f"pre{ci}"] = _dr(c)
            assert (qo[s].add_batch(c) == 0).all()
        d, res = qo[s].pull_batch(srv[s][1], sh["settle"])
        want[s]["settle"] = (d, res)
        et.tally(s, d)

    def run(s, i0, i1):
        for i in range(i0, i1):
            b = srv[s][2][i].copy()
            et.fill(s, b)
            want[s][f"req{i}"] = _dr(b)
            assert (qo[s].add_batch(b) == 0).all()
            d, res = qo[s].pull_batch(float(b["time"][-1]), k)
            want[s][f"dec{i}"] = (d, res)
            et.tally(s, d)

    with ThreadPoolExecutor(S) as pool:
        list(pool.map(prepare, range(S)))
        et.deliver()
        for e in range(sh["epochs"]):
            i0 = e * sh["steps"]
            list(pool.map(lambda s: run(s, i0, i0 + sh["steps"]), range(S)))
            et.deliver()
    ties = sum(q.ties for q in qo)
    for q in qo:
        q.close()
    return want, et, ties


def _check(sh, outdir, want, et):
    from dmclock_amd._abi import PullResult
    from parity import compare_decisions
    n_steps = sh["epochs"] * sh["steps"]
    n_dec = 0
    for s in range(sh["S_total"]):
        g = np.load(os.path.join(outdir, f"srv{s}.npz"))
        w = want[s]
        for key in [kk for kk in w if kk.startswith("pre")] + \
                [f"req{i}" for i in range(n_steps)]:
            assert np.array_equal(g[key][0], w[key][0]), (s, key, "delta")
            assert np.array_equal(g[key][1], w[key][1]), (s, key, "rho")
        res = g["res"]
        for key, row, buf in [("settle", n_steps, g["settle"])] + \
                [(f"dec{i}", i, g[f"dec{i}"]) for i in range(n_steps)]:
            pr = PullResult.from_buffer_copy(res[row].tobytes())
            d, r = w[key]
            assert (pr.n_decisions, pr.next_type) == (r.n_decisions, r.next_type), (s, key)
            dg = buf.view(DECISION_DTYPE)[:pr.n_decisions]
            compare_decisions(dg, d, f"server {s} {key}")
            n_dec += len(d)
        sl = s
        for f in ("xd", "xr"):
            assert np.array_equal(g[f], getattr(et, f)[sl]), (s, f)
        assert np.array_equal(g["known"].astype(bool), et.known[sl]), s
        assert np.array_equal(g["gd"], et.gd) and np.array_equal(g["gr"], et.gr), s
        # steps: bin-ranked rounds only; the settle: at least four rounds
        # (k = 2^20 in rounds of at most 2^18 pulls)
        assert g["counters"][0] == 0, ("radix rounds", s, g["counters"])
        assert g["counters"][2] >= sh["settle"] >> 18, ("settle rounds", s, g["counters"])
        assert g["counters"][4] == n_steps, ("fused steps", s, g["counters"])
    return n_dec


def _spawn(world, sh, outdir):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    out_q = ctx.Queue()
    port = 31500 + os.getpid() % 1000
    old = os.environ.get("GPU_MAX_HW_QUEUES")
    os.environ["GPU_MAX_HW_QUEUES"] = "8"  # inherited by the children only
    try:
        procs = [ctx.Process(target=_rank, args=(r, world, port, sh, outdir, out_q))
                 for r in range(world)]
        for p in procs:
            p.start()
    finally:
        if old is None:
            del os.environ["GPU_MAX_HW_QUEUES"]
        else:
            os.environ["GPU_MAX_HW_QUEUES"] = old
    msgs = {}
    try:
        for _ in procs:
            rank, msg = out_q.get(timeout=sh.get("wait", 240))
            msgs[rank] = msg
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(m == "ok" for m in msgs.values()), msgs
    for p in procs:
        assert p.exitcode == 0


@pytest.mark.timeout(480)
@pytest.mark.parametrize("world", [1, 2])
def test_concurrent_queues_trackers_parity(world):
    """world 1: four queues in one process, four host threads; world 2: two
    processes of two queues each, the epoch all-reduce over gloo.  Every
    delta/rho, decision, result and tracker word bit-exact; the k = 2^20
    settle ran as rounds of at most 2^18 pulls (deep queues can overflow a
    rank bin there: those rounds re-run on the radix path, concurrently on
    the four streams), the steps as bin-ranked rounds."""
    sh = dict(SHAPE)
    with tempfile.TemporaryDirectory() as outdir:
        _spawn(world, sh, outdir)
        want, et, ties = oracle_run(sh)
        assert ties == 0, f"{ties} tied decisions: pick another seed"
        n = _check(sh, outdir, want, et)
    assert n > sh["S_total"] * sh["settle"]


@pytest.mark.timeout(900)
def test_group_bench_shape_vs_oracle():
    """BASELINE config 5's per-GPU shape at its full size against the oracle
    (VERDICT r5, next item 3): eight server tables of 2,097,152 client slots
    in one queue group (bench.py --config 5), depth 4 (8M queued requests per
    table), a 2M-pull settle per table, then two steps of 64K adds + 64K
    pulls per table with the device trackers' fill and tally inside the
    group step and an epoch delivery after each.  The tables hold different
    subsets of 4,194,304 global clients (each server's 2M drawn at random:
    clients shared across servers, G < S * N), so delta/rho carry other
    servers' responses (dmclock_client.h:59-79).  Every request's delta/rho,
    every decision (tag bits included), result record and tracker word of
    all eight tables bit-exact against eight oracle queues (run on eight host
    threads) and the epoch restatement (simulate.h:118-136)."""
    sh = dict(SHAPE, S_total=8, N=1 << 21, G=1 << 22, depth=4, settle=1 << 21, epochs=2,
              steps=1, batch=1 << 16, seed=21, chunk=1 << 20, group=True, wait=600)
    with tempfile.TemporaryDirectory() as outdir:
        _spawn(1, sh, outdir)
        want, et, ties = oracle_run(sh)
        assert ties == 0, f"{ties} tied decisions: pick another seed"
        n = _check(sh, outdir, want, et)
    assert n > sh["S_total"] * (sh["settle"] + 2 * sh["batch"]) * 0.99


@pytest.mark.timeout(480)
def test_group_queues_trackers_parity_8():
    """The multi-table path: eight server queues in
    one queue group (dmc_group_step_device: one launch per kernel over the
    eight tables, blockIdx.y = table, one graph per step, device trackers'
    fill and tally inside the step), after the same per-queue preparation and
    settle; every delta/rho, decision, result and tracker word bit-exact
    against eight oracle queues and the epoch restatement."""
    sh = dict(SHAPE, S_total=8, N=1 << 17, G=1 << 19, settle=1 << 19, group=True)
    with tempfile.TemporaryDirectory() as outdir:
        _spawn(1, sh, outdir)
        want, et, ties = oracle_run(sh)
        assert ties == 0, f"{ties} tied decisions: pick another seed"
        n = _check(sh, outdir, want, et)
    assert n > sh["S_total"] * sh["settle"]
