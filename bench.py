#!/usr/bin/env python3
"""Benchmark: BASELINE.json config 3 on the HIP engine.

Workload ("step"): one dmClock server queue with 1M bulk-registered clients
(r ~ U[1,10] for 50 %, w ~ U[0.5,1.5], l ~ U[5,25] for 30 %, cost in {1,2,3},
delta = rho = 1), pre-populated with ~4 queued requests per client from a
Poisson process of 2M req/s; each step adds the next 64K arrivals
(tag updates) and then makes up to 64K pull_request(now) decisions at the
step's last arrival time.  Inputs of every step are resident in HBM before
the timed region; each step runs dmc_add_pull_batch_device (= dmc_add_batch_device
+ dmc_pull_batch_device, fused into one graph launch; --separate-calls for two).

metric = BASELINE.json metric: dispatch decisions/s + tag updates/s, whole job.
With --gpus N each rank runs its own server queue (dmClock servers are
independent: SURVEY.md section 8(e)), so scaling is weak and there is no
collective on the data path.

Extra fields: roofline (dominant stage, HIP-event timed inside the timed
region on the engine's stream), cpu_baseline (the CPU restatement timed on
this host, rank 0, bounded sample).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "dispatch decisions/sec + tag updates/sec at 1M clients; % of HBM peak"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec

# Algorithmic bytes of each stage: (per client slot of the table, per added
# request, per decision) -- DESIGN.md section 6.  A pull round streams the
# client-table columns it needs once per kernel and touches the candidates'
# rings and state; the add path touches one client record per request.
STAGE_BYTES = {
    # k_rscan: count 4 + front_r 8 + flags 1 + front_p 8 + front_l 8 +
    #   prop_delta 8 read, keyr 8 + keyp 8 + R-prefix length 1 written
    "scan": (54, 0, 0),
    # k_rhist: keyr + keyp read (its last block: 2 x 2048-bin thresholds)
    "select": (16, 0, 0),
    # k_rcand: keyr + keyp + flags read per slot; per candidate (about one
    #   per decision) its slot written to the candidate list
    "cand": (17, 0, 4),
    # k_remit: per candidate its slot 4 and keyr + keyp 16 read; per
    #   dispatched entry its ring entry 64 read and rank record 24 written
    "emit": (0, 0, 108),
    # k_rrank: rank record 24 read, decision offset + tie 8 written into the
    #   ring entry
    "rank": (0, 0, 32),
    # k_rapply: applied 4 + flags 1 per slot; per decision its ring entry 64
    #   read, decision record 48 written, client state ~120 read/written
    "apply": (5, 0, 232),
    # k_add_link: request slot 32 (line) read, apos/aslot 8 written, slot
    #   counter 4 + slot buffer 4
    "add_link": (0, 48, 0),
    # k_add_chain (one request per client): apos/aslot 8 + acnt 8 + abuf 4
    #   + request 32 + rc 4 + ring entry 64 + client state read 81
    #   (prev tag 32, inverses 24, head/count/cur_delta/cur_rho 16,
    #   last_tick 8, flags 1) and written 77 (prev 32, count/cur_* 12,
    #   last_tick 8, flags 1, front tag 24)
    "add_chain": (0, 278, 0),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--clients", type=int, default=1 << 20)
    ap.add_argument("--batch", type=int, default=1 << 16)
    ap.add_argument("--pulls", type=int, default=None,
                    help="decisions per step (default: = --batch)")
    ap.add_argument("--depth", type=int, default=4)
    ap.add_argument("--settle", type=int, default=None,
                    help="pulls at the pre-population's end time before the "
                         "steps (default: depth/2 per client), which drain "
                         "the reservation backlog so that steps run in "
                         "steady state with both phases")
    ap.add_argument("--ring", type=int, default=64)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--cpu-steps", type=int, default=30)
    ap.add_argument("--cpu-budget", type=float, default=20.0,
                    help="config 4: seconds of oracle work in the CPU sample")
    ap.add_argument("--separate-calls", action="store_true",
                    help="dmc_add_batch_device + dmc_pull_batch_device per step "
                         "instead of dmc_add_pull_batch_device")
    ap.add_argument("--host-api", action="store_true",
                    help="host-buffer API per step (dmc_add_batch + dmc_pull_batch: "
                         "requests in and decisions out over PCIe every call, "
                         "what the C++ facade uses); a PCIe-inclusive rate, "
                         "never the headline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true",
                    help="skip the second, stage-timed pass")
    ap.add_argument("--prof-steps", type=int, default=10,
                    help="steps of the stage-timed pass (eager launches with "
                         "HIP events between kernels; run after the timed "
                         "region, on the following batches)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles",
                                                      "traffic_r01.json"))
    ap.add_argument("--config", type=int, default=3, choices=(3, 4, 5),
                    help="3: one server queue (default); 4: config 3 with "
                         "idle/active churn (do_clean idle marking before "
                         "every step, activations with the prop_delta reset) "
                         "and 10%% limit-throttled tenants; 5: multi-server "
                         "dmClock, --servers queues per GPU with device client "
                         "trackers and a per-epoch all-reduce")
    ap.add_argument("--idle-frac", type=float, default=0.10,
                    help="config 4: fraction of the clients marked idle before "
                         "each step, drawn from those without an arrival in "
                         "the previous two steps")
    ap.add_argument("--servers", type=int, default=8,
                    help="config 5: server queues per GPU")
    ap.add_argument("--epoch-steps", type=int, default=16,
                    help="config 5: steps per delta/rho epoch (16 x 64K = 1M "
                         "decisions per server)")
    args = ap.parse_args()
    if args.config == 5 and "--clients" not in sys.argv:
        args.clients = 1 << 21  # 2M client slots per server table
    return args


def make_workload(args, seed):
    from dmclock_amd import workloads
    rng = np.random.default_rng(seed)
    n = args.clients
    tab = workloads.client_table(rng, n)
    if args.config == 4:
        # 10 % of the tenants limited below their arrival rate (2 req/s each)
        thr = rng.random(n) < 0.10
        tab.l = np.where(thr, rng.uniform(0.5, 1.5, n), tab.l)
    rate = 2.0 * n
    pre = workloads.arrivals(rng, n, args.depth * n, 1.0, rate)
    t = float(pre["time"][-1])
    steps = []
    handle = len(pre)
    for _ in range(args.warmup + args.steps + args.prof_steps):
        reqs = workloads.arrivals(rng, n, args.batch, t, rate,
                                  handle_base=handle)
        handle += args.batch
        t = float(reqs["time"][-1])
        steps.append(reqs)
    idle = None
    if args.config == 4:
        # do_clean's idle pass before each step (:1230-1250): clients without
        # an arrival in the two previous batches, a random idle_frac of all
        idle = []
        last = np.full(n, -1, np.int64)
        is_idle = np.zeros(n, bool)
        args.activations = []
        for i, reqs in enumerate(steps):
            quiet = np.flatnonzero(last < i - 2)
            m = min(len(quiet), int(args.idle_frac * n))
            sel = np.sort(rng.choice(quiet, m, replace=False)).astype(np.uint32)
            idle.append(sel)
            is_idle[sel] = True
            u = np.unique(reqs["slot"])
            args.activations.append(int(is_idle[u].sum()))  # first arrivals of idle clients
            is_idle[u] = False
            last[reqs["slot"]] = i
    return tab, pre, steps, idle


def prepare(q, args, tab, pre):
    """Same setup on either engine: bulk registration, pre-population,
    settle pulls."""
    q.register_active(tab.slots, tab.r, tab.w, tab.l)
    chunk = 1 << 20
    for i in range(0, len(pre), chunk):
        rc = q.add_batch(pre[i:i + chunk])
        assert (rc == 0).all(), np.unique(rc)
    settle = args.settle if args.settle is not None else \
        args.depth * args.clients // 2
    t_pre = float(pre["time"][-1])
    done = 0
    while done < settle:
        k = min(settle - done, 1 << 20)
        d, res = q.pull_batch(t_pre, k)
        done += k
        if res.n_decisions < k:
            break
    return settle


def cpu_baseline(args, tab, pre, steps, idle=None):
    """The oracle (CPU restatement of the reference queue, one core) on a
    bounded sample of the same workload: same 1M clients and pre-population,
    timed over --cpu-steps steps."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    q = pyoracle.OracleQueue(track_ties=False)
    prepare(q, args, tab, pre)
    k = args.pulls or args.batch
    ops = 0
    if idle is not None:
        return cpu_baseline_churn(args, q, steps, idle)
    t0 = time.perf_counter()
    for i, reqs in enumerate(steps[:args.cpu_steps]):
        q.add_batch(reqs)
        d, res = q.pull_batch(float(reqs["time"][-1]), k)
        ops += len(reqs) + res.n_decisions
    dt = time.perf_counter() - t0
    return {"value": ops / dt, "unit": "ops/s", "cores": 1, "kind": "port",
            "sample": (f"oracle (CPU restatement, std::map + 3 binary heaps) on "
                       f"the same {args.clients}-client queue after the same "
                       f"pre-population and settle, {args.cpu_steps} steps of "
                       f"{args.batch} adds + {k} pulls, {dt:.2f} s")}


def cpu_baseline_churn(args, q, steps, idle):
    """Config 4 on the oracle: every activation scans all clients (O(N),
    SURVEY finding 4), so the sample is the first step's idle marking and
    then its adds in chunks of 256, each followed by as many pulls, until
    --cpu-budget seconds have passed."""
    budget = args.cpu_budget
    ops = acts = 0
    i0 = next((i for i, s in enumerate(idle) if len(s)), 0)
    t0 = time.perf_counter()
    for c in idle[i0].tolist():
        q.mark_idle(c)
    reqs = steps[i0]
    idle_set = np.zeros(args.clients, bool)
    idle_set[idle[i0]] = True
    n_add = 0
    last = t0
    for j in range(0, len(reqs), 256):
        sub = reqs[j:j + 256]
        u = np.unique(sub["slot"])
        acts += int(idle_set[u].sum())
        idle_set[u] = False
        q.add_batch(sub)
        d, res = q.pull_batch(float(sub["time"][-1]), len(sub))
        ops += len(sub) + res.n_decisions
        n_add += len(sub)
        now = time.perf_counter()
        if now - last > 20:
            print(f"cpu baseline: {n_add} adds, {now - t0:.0f} s", file=sys.stderr,
                  flush=True)
            last = now
        if now - t0 > budget:
            break
    dt = time.perf_counter() - t0
    return {"value": ops / dt, "unit": "ops/s", "cores": 1, "kind": "port",
            "sample": (f"oracle (CPU restatement, std::map + 3 binary heaps) on "
                       f"the same {args.clients}-client queue after the same "
                       f"pre-population and settle: a step's idle "
                       f"marking ({len(idle[i0])} clients), then its first "
                       f"{n_add} adds ({acts} activations, each an O(N) scan) "
                       f"in chunks of 256, each followed by as many pulls, "
                       f"{dt:.2f} s")}


def main():
    args = parse()
    if args.config == 5:
        import bench_multiserver
        return bench_multiserver.main(args)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    from dmclock_amd.gpu import GpuQueue
    from dmclock_amd._abi import DECISION_DTYPE, PullResult

    tab, pre, steps, idle = make_workload(args, args.seed + rank)
    k = args.pulls or args.batch
    q = GpuQueue(max_clients=args.clients, ring_capacity=args.ring,
                 max_batch=max(args.batch, k, 1 << 20), device=local)
    settle = prepare(q, args, tab, pre)

    dev = torch.device("cuda", local)
    d_reqs = [torch.from_numpy(r.view(np.uint8)).to(dev) for r in steps]
    d_rc = torch.zeros(args.batch, dtype=torch.int32, device=dev)
    d_out = torch.zeros(k * DECISION_DTYPE.itemsize, dtype=torch.uint8,
                        device=dev)
    res_sz = 24
    d_res = torch.zeros((len(steps), res_sz), dtype=torch.uint8, device=dev)
    nows = [float(r["time"][-1]) for r in steps]
    torch.cuda.synchronize()

    host_t = {"mark_idle": 0.0, "add_pull": 0.0}
    timing = os.environ.get("BENCH_HOST_TIMING") is not None

    def step(i):
        if idle is not None:
            t_a = time.perf_counter()
            q.mark_idle_batch(idle[i])
            if timing:
                host_t["mark_idle"] += time.perf_counter() - t_a
        t_b = time.perf_counter()
        _step_calls(i)
        if timing:
            host_t["add_pull"] += time.perf_counter() - t_b

    host_res = {}

    def _step_calls(i):
        if args.host_api:
            rc = q.add_batch(steps[i])
            assert (rc == 0).all()
            _, host_res[i] = q.pull_batch(nows[i], k)
        elif args.separate_calls:
            q.add_batch_device(d_reqs[i].data_ptr(), args.batch, d_rc.data_ptr())
            q.pull_batch_device(nows[i], k, d_out.data_ptr(), d_res[i].data_ptr())
        else:  # the same two operations, one graph launch
            q.add_pull_batch_device(d_reqs[i].data_ptr(), args.batch, d_rc.data_ptr(),
                                    nows[i], k, d_out.data_ptr(), d_res[i].data_ptr())

    for i in range(args.warmup):
        step(i)
    st_t0 = q.stats()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.warmup, args.warmup + args.steps):
        step(i)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    st_t1 = q.stats()
    res = d_res[args.warmup:args.warmup + args.steps].cpu().numpy()
    if timing:
        print("host time per step (ms): " + ", ".join(
            f"{k} {v / args.steps * 1e3:.3f}" for k, v in host_t.items())
            + f", wall {dt / args.steps * 1e3:.3f}", file=sys.stderr)

    # stage-timed pass: the next prof_steps batches, launched eagerly behind
    # a GPU-side gate with HIP events on the engine's stream around each stage
    prof = {}
    prof_steps = 0
    if not args.no_profile and args.prof_steps > 0:
        q.profile(True)
        q.profile_reset()
        torch.cuda.synchronize()
        for i in range(args.warmup + args.steps,
                       args.warmup + args.steps + args.prof_steps):
            step(i)
        torch.cuda.synchronize()
        q.profile(False)
        prof = q.profile_read()
        prof_steps = args.prof_steps

    n_dec = 0
    n_res = 0
    for j, row in enumerate(res):
        pr = (host_res[args.warmup + j] if args.host_api
              else PullResult.from_buffer_copy(row.tobytes()))
        n_dec += pr.n_decisions
    rc_last = d_rc.cpu().numpy()
    assert args.host_api or (rc_last == 0).all(), np.unique(rc_last, return_counts=True)
    st = st_t1
    n_adds = args.steps * args.batch
    local_ops = n_dec + n_adds

    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        o = torch.tensor([local_ops, n_dec, n_adds], dtype=torch.float64,
                         device=dev)
        dist.all_reduce(o, op=dist.ReduceOp.SUM)
        local_ops, n_dec, n_adds = (float(x) for x in o.tolist())

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    # roofline: the dominant stage (largest time per step) of the stage-timed
    # pass, its algorithmic bytes per launch over its mean launch duration
    roof = None
    cand = [(ms, name) for name, (c, ms) in prof.items()
            if name in STAGE_BYTES and c > 0]
    if cand:
        ms, name = max(cand)
        c = prof[name][0]
        per_client, per_req, per_dec = STAGE_BYTES[name]
        launches_per_step = c / max(prof_steps, 1)
        per_launch = (per_client * args.clients
                      + (per_req * args.batch + per_dec * k)
                      / launches_per_step)
        avg_s = ms / c / 1e3
        achieved = per_launch / avg_s / 1e9
        # HBM bytes per launch of the same stage from the PMC passes of
        # scripts/gpu_pmc.sh (tools/pmc_traffic.py: 2 x FETCH_SIZE +
        # WRITE_SIZE, the guide's gfx950 correction), committed under
        # profiles/; null if that file is absent
        traffic = None
        if os.path.exists(args.traffic):
            try:
                t = json.load(open(args.traffic)).get(name)
                traffic = t["hbm_bytes"] if t else None
            except Exception:
                traffic = None
        roof = {"bound": "hbm", "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic, "kernel": name,
                "bytes_per_launch": int(per_launch),
                "avg_launch_us": round(avg_s * 1e6, 2)}

    cpu = None
    if not args.no_cpu_baseline and world == 1:
        cpu = cpu_baseline(args, tab, pre, steps[args.warmup:],
                           None if idle is None else idle[args.warmup:])

    ms_step = dt / args.steps * 1e3
    out = {
        "metric": METRIC,
        "value": round(local_ops / dt, 1),
        "unit": "ops/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": ("config3: single server queue, synthetic 1M "
                                "clients mixed r/w/l, 64K adds + 64K pulls "
                                "per step") if args.config == 3 else
                               ("config4: config 3 + do_clean idle marking of "
                                f"{args.idle_frac:.0%} of the clients before each "
                                "step (activations with the prop_delta reset) "
                                "+ 10% limit-throttled tenants"),
                   "clients": args.clients, "adds_per_step": args.batch,
                   "pulls_per_step": k, "prepopulated": len(pre),
                   "settle_pulls": settle,
                   "ring_capacity": args.ring,
                   "api": ("host buffers (dmc_add_batch + dmc_pull_batch, PCIe "
                           "inclusive)" if args.host_api else
                           "device buffers (dmc_add_pull_batch_device)"),
                   "parallelism": f"{world} independent server queue(s)"},
        "decisions_per_s": round(n_dec / dt, 1),
        "activations_per_step": (None if args.config != 4 else
                                 round(float(np.mean(args.activations[args.warmup:
                                       args.warmup + args.steps])), 1)),
        "tag_updates_per_s": round(n_adds / dt, 1),
        "reservation_decisions": int(st.reserv_sched_count - st_t0.reserv_sched_count),
        "priority_decisions": int(st.prop_sched_count - st_t0.prop_sched_count),
        "queued_after": int(st.requests),
        "roofline": roof,
        "cpu_baseline": cpu,
        "stages_ms_per_step": {n: round(ms / max(prof_steps, 1), 4)
                               for n, (c, ms) in prof.items() if c},
        "stages_note": "stage times from a second pass of prof_steps steps "
                       "launched eagerly behind a GPU-side gate (all of a "
                       "call's kernels queued before the first starts) with "
                       "HIP events around each stage; the timed region "
                       "replays captured hipGraphs",
        "prof_steps": prof_steps,
    }
    print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
