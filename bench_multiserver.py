"""bench.py --config 5: multi-server dmClock (BASELINE.json config 5).

Workload: every GPU (rank) hosts --servers server queues (default 8), each
with a table of --clients client slots (default 2M) in the config-3 mix
(r ~ U[1,10] for 50 %, w ~ U[0.5,1.5], l ~ U[5,25] for 30 %, cost in
{1,2,3}).  Global clients: servers x slots per rank, in blocks -- block s is
held by server s of every rank, each server table in its own random slot
order (client_of_slot) -- so with 8 ranks x 8 servers = 64 servers every one
of the 16M clients uses 8 servers (select range R = 8, SURVEY.md section
8(d) config 5), one on each GPU.

The clients' ServiceTracker<S, OrigTracker> state lives on the device
(dmclock_amd/multiserver.py, csrc/dmc_tracker.h): each request's delta/rho
is filled by get_req_params on the device right before its add; every
decision is tallied per slot; every --epoch-steps steps the per-client
response sums are collected, all-reduced over the ranks (RCCL over xGMI,
int32 sum of 2 x 16M counters) and delivered.  A "step" is, on every server
of every rank: fill delta/rho for the next 64K arrivals, add them, pull 64K
decisions at the batch's last arrival, tally -- by default one queue-group
step (dmc_group_step_device: one launch per kernel over the rank's S server
tables, one graph), with --separate-queues one host thread and HIP stream
per queue, each server its own fill + fused call + tally.  The epoch delivery
(collect + all-reduce + advance) is inside the timed region.

value = (adds + decisions) of all servers of all ranks / max-over-ranks time.
"""
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def server_workload(args, rank, s, n_steps):
    """client table (the block's clients in this server's slot order),
    pre-population and per-step batches of server s on `rank`"""
    from dmclock_amd import workloads
    N = args.clients
    # client info belongs to the client: same on every server holding it
    tab = workloads.client_table(np.random.default_rng([args.seed, s]), N)
    rng = np.random.default_rng([args.seed, 1000 + rank, s])
    perm = rng.permutation(N)
    tab.r, tab.w, tab.l = tab.r[perm], tab.w[perm], tab.l[perm]
    cmap = (s * N + perm).astype(np.int32)
    rate = 2.0 * N
    pre = workloads.arrivals(rng, N, args.depth * N, 1.0, rate)
    t = float(pre["time"][-1])
    steps = []
    h = len(pre)
    for _ in range(n_steps):
        reqs = workloads.arrivals(rng, N, args.batch, t, rate, handle_base=h)
        h += args.batch
        t = float(reqs["time"][-1])
        steps.append(reqs)
    return tab, cmap, pre, steps


def cpu_baseline_multi(args, wl, n_steps):
    """The oracle (CPU restatement of the reference queue, one thread per
    server queue, C = min(servers, 16) threads: the box's CPU share per GPU)
    on a bounded sample of the same workload: each thread builds server s's
    queue (same table, pre-population and settle pulls; delta = rho = 1 as
    the requests carry them, the device trackers' fill is not restated) and
    is then timed over --cpu-steps steps of 64K adds + 64K pulls.  ctypes
    releases the GIL inside the oracle's calls, so the queues run in
    parallel."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from bench import prepare
    S = len(wl)
    C = min(S, 16)
    k = args.pulls or args.batch
    steps = min(args.cpu_steps, n_steps)

    def one(s):
        tab, _, pre, bat = wl[s]
        q = pyoracle.OracleQueue(track_ties=False)
        prepare(q, args, tab, pre)
        t0 = time.perf_counter()
        ops = 0
        for reqs in bat[:steps]:
            q.add_batch(reqs)
            d, res = q.pull_batch(float(reqs["time"][-1]), k)
            ops += len(reqs) + res.n_decisions
        t1 = time.perf_counter()
        q.close()
        return ops, t0, t1

    with ThreadPoolExecutor(C) as ex:
        out = list(ex.map(one, range(S)))
    ops = sum(o[0] for o in out)
    span = max(o[2] for o in out) - min(o[1] for o in out)
    busy = sum(o[2] - o[1] for o in out)
    return {"value": ops / span, "unit": "ops/s", "cores": C, "kind": "port",
            "sample": (f"oracle (CPU restatement, std::map + 3 binary heaps), "
                       f"{S} server queues of {args.clients} clients on {C} host "
                       f"threads, each after the same pre-population and settle, "
                       f"{steps} steps of {args.batch} adds + {k} pulls per queue; "
                       f"{span:.1f} s wall ({busy:.1f} thread-s)")}


def main(args):
    import torch
    from dmclock_amd._abi import DECISION_DTYPE, PullResult
    from dmclock_amd.multiserver import DeviceTrackers, GpuGroup, make_queues
    from bench import METRIC

    from bench import rank_env
    rank, world, local, backend = rank_env()
    dist = None
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(backend)
    dev = torch.device("cuda", local)

    S, N, E = args.servers, args.clients, args.epoch_steps
    k = args.pulls or args.batch
    n_steps = args.warmup + args.steps
    n_prof = 0 if args.no_profile else args.prof_steps
    t_gen = time.perf_counter()
    with ThreadPoolExecutor(min(S, 8)) as ex:
        wl = list(ex.map(lambda s: server_workload(args, rank, s, n_steps + n_prof),
                         range(S)))
    t_gen = time.perf_counter() - t_gen

    queues = make_queues(S, N, device=local, ring_capacity=args.ring,
                         max_batch=max(args.batch, k, 1 << 20))
    cmap = np.stack([w[1] for w in wl])
    trk = DeviceTrackers(queues, N, dev, n_clients=S * N, client_of_slot=cmap,
                         lagged=not args.sequential_epochs)

    chunk = 1 << 20
    d_rc = [torch.zeros(chunk, dtype=torch.int32, device=dev) for _ in range(S)]
    d_out = [torch.zeros(max(k, chunk) * DECISION_DTYPE.itemsize, dtype=torch.uint8,
                         device=dev) for _ in range(S)]
    d_res = torch.zeros((S, n_steps + n_prof + 64, 24), dtype=torch.uint8, device=dev)
    # every step's add statuses in a slice of their own (all asserted)
    d_rcs = torch.full((S, n_steps + n_prof, args.batch), -1, dtype=torch.int32, device=dev)
    d_steps = [[torch.from_numpy(r.view(np.uint8)).to(dev) for r in w[3]] for w in wl]
    nows = [[float(r["time"][-1]) for r in w[3]] for w in wl]

    def prepare(s):
        """registration, pre-population through the trackers, settle pulls"""
        q = queues[s]
        tab, _, pre, _ = wl[s]
        q.register_active(tab.slots, tab.r, tab.w, tab.l)
        for i in range(0, len(pre), chunk):
            part = torch.from_numpy(pre[i:i + chunk].view(np.uint8)).to(dev)
            n = len(pre[i:i + chunk])
            trk.fill(s, part.data_ptr(), n)
            q.add_batch_device(part.data_ptr(), n, d_rc[s].data_ptr())
            q.sync()
            assert int((d_rc[s][:n] != 0).sum()) == 0
        settle = args.settle if args.settle is not None else args.depth * N // 2
        t_pre = float(pre["time"][-1])
        done, j = 0, n_steps + n_prof
        while done < settle:
            kk = min(settle - done, chunk)
            q.pull_batch_device(t_pre, kk, d_out[s].data_ptr(), d_res[s, j].data_ptr())
            trk.tally(s, d_out[s].data_ptr(), d_res[s, j].data_ptr(), kk)
            q.sync()
            done += kk
            j += 1
        return settle

    def run(s, i0, i1):
        q = queues[s]
        for i in range(i0, i1):
            d = d_steps[s][i]
            trk.fill(s, d.data_ptr(), args.batch)
            # the add batch and the pull batch in one graph launch
            q.add_pull_batch_device(d.data_ptr(), args.batch, d_rcs[s, i].data_ptr(),
                                    nows[s][i], k, d_out[s].data_ptr(),
                                    d_res[s, i].data_ptr())
            trk.tally(s, d_out[s].data_ptr(), d_res[s, i].data_ptr(), k)
        q.sync()

    pool = ThreadPoolExecutor(S)
    group = None if args.separate_queues else GpuGroup(queues)
    if group is not None and trk.lagged:
        trk.attach_group(group)  # (the epoch's sums beside the next steps)
    g_args = [([d_steps[s][i].data_ptr() for s in range(S)], [nows[s][i] for s in range(S)],
               [d_res[s, i].data_ptr() for s in range(S)],
               [d_rcs[s, i].data_ptr() for s in range(S)])
              for i in range(n_steps + n_prof)]
    g_out = [d_out[s].data_ptr() for s in range(S)]

    def segment(i0, i1):
        if group is None:
            list(pool.map(lambda s: run(s, i0, i1), range(S)))
            return
        for i in range(i0, i1):
            reqs, nw, res, rcs = g_args[i]
            group.step(args.batch, reqs, rcs, nw, k, g_out, res, trk.group_trackers())

    t_prep = time.perf_counter()
    settle = list(pool.map(prepare, range(S)))[0]
    trk.deliver()
    t_prep = time.perf_counter() - t_prep

    def steps_with_epochs(i0, i1, epochs):
        i = i0
        while i < i1:
            j = min(i1, (i // E + 1) * E)
            segment(i, j)
            i = j
            if i % E == 0:
                t = time.perf_counter()
                trk.deliver()
                epochs.append(time.perf_counter() - t)

    warm_epochs = []
    steps_with_epochs(0, args.warmup, warm_epochs)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    epochs = []
    t0 = time.perf_counter()
    steps_with_epochs(args.warmup, n_steps, epochs)
    trk.finish()  # (the last epoch's overlapped delivery)
    for q in queues:
        q.sync()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    pool.shutdown()
    grp_ctr = None
    if group is not None:
        grp_ctr = {"fused_calls": sum(q.counters()["fused_calls"] for q in queues),
                   "graph_replays": sum(q.counters()["graph_replays"] for q in queues)}

    # roofline: the kernels the timed steps ran.  Queue group: the group's
    # next n_prof steps with its stage timers on (the same multi-table
    # kernels, launched eagerly, each timed by its own dispatch), the
    # algorithmic bytes of all S tables per launch (_stage_bytes is linear in
    # the counts: the members' counters summed).  Separate queues: server 0's
    # next n_prof steps alone, stage-timed like config 3.
    from bench import roofline
    roof = None
    if n_prof and group is not None:
        for q in queues:
            q.counters(reset=True)
        group.profile(True)
        torch.cuda.synchronize()
        epochs_prof = []
        steps_with_epochs(n_steps, n_steps + n_prof, epochs_prof)
        for q in queues:
            q.sync()
        torch.cuda.synchronize()
        prof = group.profile_read()
        group.profile(False)
        ctr = {}
        for q in queues:
            for key, v in q.counters().items():
                if isinstance(v, (int, float)):
                    ctr[key] = ctr.get(key, 0) + v
        roof = roofline(args, prof, n_prof, ctr, k, n_clients=S * N,
                        n_adds=S * args.batch)
        if roof is not None:
            roof["kernel"] = {"emit": "k_remit_m", "scan": "k_rscan_m",
                              "add_chain": "k_add_chain_m", "add_link": "k_add_link_m",
                              "select": "k_rhist_m + k_rpick_m", "rank": "k_rrank_m",
                              "apply": "k_rapply_m"}.get(roof["kernel"], roof["kernel"])
            roof["note"] = (f"queue group: the multi-table kernels of {n_prof} group "
                            f"steps after the timed region (eager launches, each "
                            f"timed by its own dispatch), {S} tables per launch")
    elif n_prof:
        q0 = queues[0]
        q0.profile(True)
        q0.profile_reset()
        q0.counters(reset=True)
        torch.cuda.synchronize()
        run(0, n_steps, n_steps + n_prof)
        torch.cuda.synchronize()
        q0.profile(False)
        roof = roofline(args, q0.profile_read(), n_prof, q0.counters(), k,
                        n_clients=N)
        if roof is not None:
            roof["note"] = ("separate queues: server 0 alone after the timed "
                            "region, its dominant stage per launch")

    res = d_res[:, args.warmup:n_steps].cpu().numpy()
    n_dec = sum(PullResult.from_buffer_copy(row.tobytes()).n_decisions
                for srv in res for row in srv)
    n_adds = S * args.steps * args.batch
    # every step that ran (warmup, timed, the roofline pass), every server
    # (separate queues: the roofline pass ran server 0 alone)
    rc = d_rcs[:, :n_steps].cpu().numpy()
    assert (rc == 0).all(), np.unique(rc, return_counts=True)
    if n_prof:
        rcp = (d_rcs[:, n_steps:n_steps + n_prof] if group is not None
               else d_rcs[:1, n_steps:n_steps + n_prof]).cpu().numpy()
        assert (rcp == 0).all(), np.unique(rcp, return_counts=True)
    local_ops = n_dec + n_adds
    ep_ms = 1e3 * float(np.mean(epochs)) if epochs else None
    if dist:
        rdev = dev if backend == "nccl" else torch.device("cpu")
        t = torch.tensor([dt], dtype=torch.float64, device=rdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        o = torch.tensor([local_ops, n_dec, n_adds], dtype=torch.float64, device=rdev)
        dist.all_reduce(o, op=dist.ReduceOp.SUM)
        local_ops, n_dec, n_adds = (float(x) for x in o.tolist())
    st = trk.state() if rank == 0 else None
    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    # all-reduce bytes per epoch: 2 x int32 per global client
    ar_bytes = 2 * 4 * S * N
    # a ring all-reduce moves 2 (n - 1) / n of the buffer over each GPU's
    # busiest link; xGMI: ~153 GB/s per link (MI355X_MICROARCH.md)
    ring_ms = 2.0 * (world - 1) / world * ar_bytes / 153e9 * 1e3
    ar_ms = trk.allreduce_ms[-len(epochs):] if epochs and trk.allreduce_ms else []
    out = {
        "metric": METRIC,
        "value": round(local_ops / dt, 1),
        "unit": "ops/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": f"config5: multi-server dmClock, {S} server queues "
                               f"per GPU x {N} client slots, {S * N} global "
                               f"clients per server block set, delta/rho from "
                               f"device trackers, all-reduce every {E} steps",
                   "servers_per_gpu": S, "servers_total": S * world,
                   "slots_per_server": N, "global_clients": S * N,
                   "servers_per_client": world,
                   "adds_per_step_per_server": args.batch,
                   "pulls_per_step_per_server": k, "epoch_steps": E,
                   "ring_capacity": args.ring, "settle_pulls": settle,
                   "parallelism": (f"{world} rank(s) x {S} queues, one host "
                                   f"thread + HIP stream per queue" if group is None else
                                   f"{world} rank(s) x one queue group of {S} tables "
                                   f"(one launch per kernel over all tables)")},
        "decisions_per_s": round(n_dec / dt, 1),
        "tag_updates_per_s": round(n_adds / dt, 1),
        "epochs_timed": len(epochs),
        "epoch_delivery_ms": None if ep_ms is None else round(ep_ms, 3),
        "allreduce_bytes_per_epoch": ar_bytes,
        "allreduce_ms_per_epoch": round(float(np.mean(ar_ms)), 4) if ar_ms else None,
        "allreduce_ring_bound_ms": round(ring_ms, 4),
        "epoch_exchange": ("sequential" if args.sequential_epochs else
                           "overlapped: an epoch's sums all-reduced during the next "
                           "epoch's steps, delivered at its end"),
        "tracker_known_frac": round(float(st["known"].mean()), 4),
        "setup_s": {"generate": round(t_gen, 1), "prepopulate": round(t_prep, 1)},
        "roofline": roof,
        "group_counters": grp_ctr,
        "cpu_baseline": (None if args.no_cpu_baseline or world > 1 else
                         cpu_baseline_multi(args, wl, n_steps)),
    }
    print(json.dumps(out))
    if dist:
        dist.destroy_process_group()
