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

# Algorithmic bytes of each stage per step, from the step's counts: N client
# slots, R added requests, D decisions, C candidate clients, E rank records
# emitted, A activations.  The pull-round stages stream
# the client-table columns they need once per kernel and touch the
# candidates' state and rings; the add path touches one client record per
# request.  Bytes a kernel needs, not the lines it moves (the PMC traffic,
# roofline.traffic, is the lines).
def _stage_bytes(N, R, D, C, E, A, sampled=True):
    return {
        # k_rscan: ScanRec 32 read; the quantized first keys 8 + meta 4
        #   written; the 1/8 key sample 2 (unsampled rounds: + the 64-bit
        #   keys 16)
        "scan": (46 if sampled else 62) * N,
        # k_rhist: the sampled first keys (2 x 8 B per 8 slots), or every
        #   slot's keyr + keyp (exact)
        "select": (2 if sampled else 16) * N,
        # k_remit: quantized keys 8 + meta 4 streamed per slot; per candidate
        #   its ClientRec fields 40 (inverses, prop_delta, prev r), two ring
        #   entries 128 and position 2's r 8 read, its CandRec 8, PostRec 64
        #   and decision offset 4 written; per record the bin atomic 8 and the
        #   64-byte record
        "emit": 12 * N + 252 * C + 72 * E,
        # k_rrank: the records 64 read; per decision the 48-byte record and
        #   the candidate's decision offset 4 written
        "rank": 64 * E + 52 * D,
        # k_rapply: per candidate CandRec 8, decision offset 4, PostRec 128
        #   read; ScanRec 32, prev r 8 and the queued requests' reduced r
        #   (about 2 x 8) written
        "apply": 196 * C,
        # k_add_link: request slot 4 read, apos/aslot 8 written, the
        #   client's counter 4 (atomic) and slot-buffer entry 4
        "add_link": 20 * R,
        # k_add_chain (one request per client): link records 16 + request 32
        #   + status 4 + ring entry 64 written + client state read 73
        #   (prev tag 32, inverses 24, head/count/cur_delta/cur_rho 16, flags
        #   1) and written 85 (prev 32, count/cur_* 12, last_tick 8, flags 1,
        #   front tag 24, counter reset 4, ...)
        "add_chain": 278 * R,
        # activations (config 4): k_act_base streams flags 1, count 4, front
        #   p 8, prop_delta 8, prev p 8 and the batch counter 4 per slot; per
        #   request the cold/new contributions and their two min-scans (4 x 8
        #   written + read); per activation its inputs and result (~56)
        "activate": 33 * N + 64 * R + 56 * A,
        # k_chain_scan (a fused call's add chain beside the round's scan, one
        #   launch): the two stages' bytes
        "chain_scan": (46 if sampled else 62) * N + 278 * R,
        # k_apply_link (pipelined calls: the previous call's deferred apply
        #   beside this call's filing, one launch): the two stages' bytes
        "apply_link": 196 * C + 20 * R,
    }


def roofline(args, prof, prof_steps, ctr, k, n_clients=None, n_adds=None,
             activations=None):
    """The dominant stage (largest time per step) of the stage-timed pass:
    its algorithmic bytes per launch (_stage_bytes over that pass's counts)
    over its mean launch duration, against the HBM peak."""
    cand = [(ms, name) for name, (c, ms) in prof.items() if c > 0]
    if not cand or not prof_steps or ctr is None:
        return None
    N = n_clients or args.clients
    R = n_adds if n_adds is not None else args.batch
    per_step = lambda key: ctr[key] / prof_steps
    D, C, E = per_step("decisions"), per_step("candidates"), per_step("entries")
    A = activations or 0.0
    # sampled thresholds: tables of >= 65,536 slots (kSampleMinN) unless a
    # round's sample failed validation (counted)
    sampled = N >= (1 << 16) and not ctr.get("sample_retries", 0)
    model = _stage_bytes(N, R, D, C, E, A, sampled)
    cand = [(ms, name) for ms, name in cand if name in model]
    if not cand:
        return None
    # every stage's own roofline (algorithmic bytes per launch / mean launch)
    per = {}
    for ms_s, nm in cand:
        c = prof[nm][0]
        # (a stage launched several times per step shares the step's bytes;
        # one launched less than once per step -- the pipelined pass's first
        # filing alone, its last apply alone -- still does one call's work)
        bl = model[nm] / max(c / prof_steps, 1.0)
        a_s = ms_s / c / 1e3
        per[nm] = {"bytes_per_launch": int(bl), "avg_launch_us": round(a_s * 1e6, 2),
                   "launches_per_step": round(c / prof_steps, 2),
                   "achieved": round(bl / a_s / 1e9, 1),
                   "frac": round(bl / a_s / 1e9 / HBM_PEAK_GBS, 4)}
    ms, name = max(cand)
    r = per[name]
    return {"bound": "hbm", "achieved": r["achieved"],
            "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": r["frac"],
            "traffic": None, "kernel": name,
            "bytes_per_launch": r["bytes_per_launch"],
            "avg_launch_us": r["avg_launch_us"],
            "counts_per_step": {"clients": N, "adds": R, "decisions": round(D, 1),
                                "candidates": round(C, 1), "records": round(E, 1),
                                "activations": A},
            "stages": per}


def latest_traffic():
    """the newest round's PMC traffic file, profiles/traffic_rNN.json"""
    import glob
    import re
    best = None
    for f in glob.glob(os.path.join(ROOT, "profiles", "traffic_r*.json")):
        m = re.fullmatch(r"traffic_r(\d+)\.json", os.path.basename(f))
        if m and (best is None or int(m.group(1)) > best[0]):
            best = (int(m.group(1)), f)
    return best[1] if best else None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100,
                    help="timed steps (the queue's key spread grows over a run: "
                         "a longer window is the steadier, lower number)")
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
    ap.add_argument("--cpu-steps", type=int, default=30,
                    help="steps of the CPU baseline's sample, timed as three "
                         "consecutive repeats (the median is the value)")
    ap.add_argument("--cpu-budget", type=float, default=20.0,
                    help="config 4: seconds of oracle work in the CPU sample")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="each dmc_add_pull_batch_device call waits for its round "
                         "(default: DMC_OPT_PIPELINE, a call queues its graph behind the "
                         "previous one and returns; the timed region ends with "
                         "dmc_queue_sync, which finishes the last call)")
    ap.add_argument("--no-graphs", action="store_true",
                    help="DMC_OPT_GRAPHS 0: every kernel launched eagerly (the default "
                         "for pipelined calls)")
    ap.add_argument("--graphs", action="store_true",
                    help="pipelined calls replay captured hipGraphs (default: launched "
                         "eagerly -- a replayed graph starts 8.5 us after the previous "
                         "one ends, eager kernels back to back, r04j)")
    ap.add_argument("--separate-calls", action="store_true",
                    help="dmc_add_batch_device + dmc_pull_batch_device per step "
                         "instead of dmc_add_pull_batch_device")
    ap.add_argument("--host-api", action="store_true",
                    help="host-buffer API per step (dmc_add_batch + dmc_pull_batch: "
                         "requests in and decisions out over PCIe every call, "
                         "what the C++ facade uses); a PCIe-inclusive rate, "
                         "never the headline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--t0", type=float, default=None,
                    help="time base of the arrivals in seconds (default 1.0; "
                         "--heap-order: 1.7e9, get_time()'s epoch scale, where "
                         "rounding makes equal tags)")
    ap.add_argument("--heap-order", type=int, nargs="?", const=2, default=0,
                    help="tie-exact dispatch (DMC_OPT_HEAP_ORDER = K, default 2): "
                         "the reference's three K-ary heaps on the device, every "
                         "add and pull in call order on one wave; the timed step "
                         "is the same call.  No stage pass")
    ap.add_argument("--no-profile", action="store_true",
                    help="skip the second, stage-timed pass")
    ap.add_argument("--prof-steps", type=int, default=10,
                    help="steps of the stage-timed pass (eager launches with "
                         "HIP events between kernels; run after the timed "
                         "region, on the following batches)")
    ap.add_argument("--traffic", default=None,
                    help="PMC traffic file (tools/pmc_traffic.py) for roofline.traffic "
                         "(default: the newest profiles/traffic_rNN.json)")
    ap.add_argument("--config", type=int, default=3, choices=(3, 4, 5),
                    help="3: one server queue (default); 4: config 3 with "
                         "idle/active churn (do_clean idle marking before "
                         "every step, activations with the prop_delta reset) "
                         "and 10%% limit-throttled tenants; 5: multi-server "
                         "dmClock, --servers queues per GPU with device client "
                         "trackers and a per-epoch all-reduce")
    ap.add_argument("--host-idle", action="store_true",
                    help="config 4: mark idle from host lists (dmc_client_mark_idle_batch) "
                         "instead of HBM-resident lists")
    ap.add_argument("--idle-frac", type=float, default=0.10,
                    help="config 4: fraction of the clients marked idle before "
                         "each step, drawn from those without an arrival in "
                         "the previous two steps")
    ap.add_argument("--servers", type=int, default=8,
                    help="config 5: server queues per GPU")
    ap.add_argument("--sequential-epochs", action="store_true",
                    help="config 5: deliver each epoch's responses at its end "
                         "(collect, all-reduce, advance in sequence) instead of "
                         "overlapping the all-reduce with the next epoch")
    ap.add_argument("--separate-queues", action="store_true",
                    help="config 5: drive each server queue from its own host "
                         "thread and stream instead of one queue-group step")
    ap.add_argument("--epoch-steps", type=int, default=16,
                    help="config 5: steps per delta/rho epoch (16 x 64K = 1M "
                         "decisions per server)")
    args = ap.parse_args()
    if args.config == 5 and "--clients" not in sys.argv:
        args.clients = 1 << 21  # 2M client slots per server table
    if args.t0 is None:
        args.t0 = 1.7e9 if args.heap_order else 1.0
    if args.heap_order:
        args.no_profile = True
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
    pre = workloads.arrivals(rng, n, args.depth * n, args.t0, rate)
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
    t0 = time.perf_counter()
    for i in range(0, len(pre), chunk):
        rc = q.add_batch(pre[i:i + chunk])
        assert (rc == 0).all(), np.unique(rc)
        if args.heap_order:  # (minutes in heap order: progress for the log)
            print(f"prepare: {i + chunk} adds, {time.perf_counter() - t0:.1f} s",
                  file=sys.stderr, flush=True)
    settle = args.settle if args.settle is not None else \
        args.depth * args.clients // 2
    t_pre = float(pre["time"][-1])
    done = 0
    while done < settle:
        k = min(settle - done, 1 << 20)
        d, res = q.pull_batch(t_pre, k)
        done += k
        if args.heap_order:
            print(f"prepare: {done} settle pulls, {time.perf_counter() - t0:.1f} s",
                  file=sys.stderr, flush=True)
        if res.n_decisions < k:
            break
    return settle


def cpu_model():
    """the host CPU's model name (the baseline's cores differ box to box)"""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or None


def cpu_baseline(args, tab, pre, steps, idle=None):
    """The oracle (CPU restatement of the reference queue, one core) on a
    bounded sample of the same workload: same 1M clients and pre-population,
    --cpu-steps steps timed as three consecutive repeats; the value is their
    median (one core's rate moves with the box's other load)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    q = pyoracle.OracleQueue(track_ties=bool(args.heap_order))
    prepare(q, args, tab, pre)
    ties0 = q.ties if args.heap_order else 0
    k = args.pulls or args.batch
    if idle is not None:
        out = cpu_baseline_churn(args, q, steps, idle)
        out["cpu_model"] = cpu_model()
        return out
    reps = 3
    per = max(1, args.cpu_steps // reps)
    rates, ops_all, dt_all = [], 0, 0.0
    for r in range(reps):
        ops = 0
        t0 = time.perf_counter()
        for reqs in steps[r * per:(r + 1) * per]:
            q.add_batch(reqs)
            d, res = q.pull_batch(float(reqs["time"][-1]), k)
            ops += len(reqs) + res.n_decisions
        dt = time.perf_counter() - t0
        rates.append(ops / dt)
        ops_all += ops
        dt_all += dt
    out = {"value": float(np.median(rates)), "unit": "ops/s", "cores": 1, "kind": "port",
           "cpu_model": cpu_model(),
           "repeats": [round(x, 1) for x in rates],
           "sample": (f"oracle (CPU restatement, std::map + 3 binary heaps) on "
                      f"the same {args.clients}-client queue after the same "
                      f"pre-population and settle, {reps} consecutive repeats of "
                      f"{per} steps of {args.batch} adds + {k} pulls "
                      f"({dt_all:.2f} s in all); value = their median")}
    if args.heap_order:  # (tie tracking is on: its cost is in the sample)
        out["tied_decisions"] = {"setup": int(ties0), "sample": int(q.ties - ties0)}
    return out


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


def rank_env():
    """(rank, world, local device, backend) from the torchrun environment.
    BENCH_SHARE_DEVICE=1 rehearses a multi-rank run on a one-GPU box: every
    rank on device 0, gloo for the barrier and the reductions (RCCL needs a
    device per rank)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = "nccl"
    if os.environ.get("BENCH_SHARE_DEVICE") == "1":
        local, backend = 0, "gloo"
    return rank, world, local, backend


def spawn_ranks(n):
    """bench.py --gpus N run directly (no torchrun environment): launch the N
    ranks as child processes through torch.distributed.run, one per GPU,
    before this process touches a GPU, and exit with their status."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1",
           f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus and "WORLD_SIZE" in os.environ:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}; "
              f"running {world_env} ranks", file=sys.stderr)
    if args.config == 5:
        import bench_multiserver
        return bench_multiserver.main(args)
    rank, world, local, backend = rank_env()
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(backend)
    from dmclock_amd.gpu import GpuQueue
    from dmclock_amd._abi import DECISION_DTYPE, PullResult

    tab, pre, steps, idle = make_workload(args, args.seed + rank)
    k = args.pulls or args.batch
    q = GpuQueue(max_clients=args.clients, ring_capacity=args.ring,
                 max_batch=max(args.batch, k, 1 << 20), device=local,
                 heap_order=bool(args.heap_order), branching=args.heap_order or 2)
    settle = prepare(q, args, tab, pre)
    pipelined = not (args.no_pipeline or args.host_api or args.separate_calls or
                     args.heap_order)
    if args.no_graphs or (pipelined and not args.graphs):
        from dmclock_amd._abi import OPT_GRAPHS
        q.set_option(OPT_GRAPHS, 0)
    if pipelined:
        from dmclock_amd._abi import OPT_PIPELINE
        q.set_option(OPT_PIPELINE, 1)

    dev = torch.device("cuda", local)
    d_reqs = [torch.from_numpy(r.view(np.uint8)).to(dev) for r in steps]
    # config 4: the idle lists resident in HBM like the requests (device-side
    # marking, dmc_client_mark_idle_batch_device); --host-idle: host lists
    d_idle = None
    if idle is not None and not args.host_api and not args.host_idle:
        d_idle = [torch.from_numpy(np.ascontiguousarray(x, dtype=np.uint32).view(np.int32))
                  .to(dev) for x in idle]
    # every step's add statuses in a slice of their own (all asserted after
    # the run, not only the last step's)
    d_rc = torch.full((len(steps), args.batch), -1, dtype=torch.int32, device=dev)
    d_out = torch.zeros(k * DECISION_DTYPE.itemsize, dtype=torch.uint8,
                        device=dev)
    res_sz = 24
    d_res = torch.zeros((len(steps), res_sz), dtype=torch.uint8, device=dev)
    nows = [float(r["time"][-1]) for r in steps]
    # device addresses resolved before the timed loop (a torch view per step
    # costs microseconds of Python the engine call does not need)
    p_reqs = [t.data_ptr() for t in d_reqs]
    p_res = [d_res[i].data_ptr() for i in range(len(steps))]
    p_rc = [d_rc[i].data_ptr() for i in range(len(steps))]
    p_out = d_out.data_ptr()
    torch.cuda.synchronize()

    host_t = {"mark_idle": 0.0, "add_pull": 0.0}
    timing = os.environ.get("BENCH_HOST_TIMING") is not None

    def step(i):
        if idle is not None:
            t_a = time.perf_counter()
            if d_idle is not None:
                q.mark_idle_batch_device(d_idle[i].data_ptr(), len(idle[i]))
            else:
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
            q.add_batch_device(p_reqs[i], args.batch, p_rc[i])
            q.pull_batch_device(nows[i], k, p_out, p_res[i])
        else:  # the same two operations, one graph launch
            q.add_pull_batch_device(p_reqs[i], args.batch, p_rc[i], nows[i], k, p_out, p_res[i])

    for i in range(args.warmup):
        step(i)
    q.sync()
    st_t0 = q.stats()
    q.counters(reset=True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.warmup, args.warmup + args.steps):
        step(i)
        if args.heap_order:
            print(f"step {i}", file=sys.stderr, flush=True)
    q.sync()  # (the last call's round read: with pipelining it is finished here)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    st_t1 = q.stats()
    ctr_timed = q.counters()
    res = d_res[args.warmup:args.warmup + args.steps].cpu().numpy()
    if timing:
        print("host time per step (ms): " + ", ".join(
            f"{k} {v / args.steps * 1e3:.3f}" for k, v in host_t.items())
            + f", wall {dt / args.steps * 1e3:.3f}", file=sys.stderr)

    # stage-timed pass: the next prof_steps batches, launched eagerly behind
    # a GPU-side gate with HIP events on the engine's stream around each stage
    prof = {}
    prof_steps = 0
    prof_ctr = None
    if not args.no_profile and args.prof_steps > 0:
        q.profile(True)
        q.profile_reset()
        q.counters(reset=True)
        torch.cuda.synchronize()
        for i in range(args.warmup + args.steps,
                       args.warmup + args.steps + args.prof_steps):
            step(i)
        torch.cuda.synchronize()
        q.profile(False)
        prof = q.profile_read()
        prof_ctr = q.counters()
        prof_steps = args.prof_steps

    n_dec = 0
    n_res = 0
    for j, row in enumerate(res):
        pr = (host_res[args.warmup + j] if args.host_api
              else PullResult.from_buffer_copy(row.tobytes()))
        n_dec += pr.n_decisions
    if not args.host_api:
        # every step that ran (warmup, timed, stage pass): each add accepted
        ran = args.warmup + args.steps + prof_steps
        rc_all = d_rc[:ran].cpu().numpy()
        assert (rc_all == 0).all(), np.unique(rc_all, return_counts=True)
    st = st_t1
    n_adds = args.steps * args.batch
    local_ops = n_dec + n_adds

    if dist:
        rdev = dev if backend == "nccl" else torch.device("cpu")
        t = torch.tensor([dt], dtype=torch.float64, device=rdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        o = torch.tensor([local_ops, n_dec, n_adds], dtype=torch.float64,
                         device=rdev)
        dist.all_reduce(o, op=dist.ReduceOp.SUM)
        local_ops, n_dec, n_adds = (float(x) for x in o.tolist())

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    acts = None
    if args.config == 4 and prof_steps:
        i0 = args.warmup + args.steps
        acts = float(np.mean(args.activations[i0:i0 + prof_steps]))
    roof = roofline(args, prof, prof_steps, prof_ctr, k, activations=acts)
    if roof is not None:
        # HBM bytes per launch of the same stage from the PMC passes of
        # scripts/gpu_pmc.sh (tools/pmc_traffic.py), committed under
        # profiles/; null if that file is absent or lacks the stage.  The
        # committed passes run config 3's bench: another config's line
        # carries traffic only from a file given for it (--traffic)
        traffic = None
        tfile = args.traffic or (latest_traffic() if args.config == 3 else None)
        if tfile and os.path.exists(tfile):
            try:
                t = json.load(open(tfile)).get(roof["kernel"])
                traffic = t["hbm_bytes"] if t else None
            except Exception:
                traffic = None
        roof["traffic"] = traffic
        roof["traffic_file"] = os.path.relpath(tfile, ROOT) if tfile else None

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
        "config": {"workload": (f"config3: single server queue, synthetic "
                                f"{args.clients} clients mixed r/w/l, {args.batch} "
                                f"adds + {k} pulls per step"
                                + (f", tie-exact heap order (DMC_OPT_HEAP_ORDER={args.heap_order})"
                                   if args.heap_order else "")
                                + (f", arrivals from t0 = {args.t0:g} s" if args.t0 != 1.0
                                   else "")) if args.config == 3 else
                               (f"config4: config 3 ({args.clients} clients, "
                                f"{args.batch} adds + {k} pulls per step) + "
                                f"do_clean idle marking of {args.idle_frac:.0%} of "
                                "the clients before each step (activations with the "
                                "prop_delta reset) + 10% limit-throttled tenants"),
                   "clients": args.clients, "adds_per_step": args.batch,
                   "heap_order": args.heap_order, "t0": args.t0,
                   "pulls_per_step": k, "prepopulated": len(pre),
                   "settle_pulls": settle,
                   "ring_capacity": args.ring,
                   "api": ("host buffers (dmc_add_batch + dmc_pull_batch, PCIe "
                           "inclusive)" if args.host_api else
                           "device buffers (dmc_add_pull_batch_device"
                           + (", pipelined: DMC_OPT_PIPELINE" if pipelined else "")
                           + (", kernels launched eagerly)" if (args.no_graphs or
                              (pipelined and not args.graphs)) else ", hipGraphs)")),
                   "parallelism": f"{world} independent server queue(s)"
                                  + ("" if backend == "nccl" else
                                     " (rehearsal: ranks share device 0, gloo)")},
        "decisions_per_s": round(n_dec / dt, 1),
        "activations_per_step": (None if args.config != 4 else
                                 round(float(np.mean(args.activations[args.warmup:
                                       args.warmup + args.steps])), 1)),
        "tag_updates_per_s": round(n_adds / dt, 1),
        "reservation_decisions": int(st.reserv_sched_count - st_t0.reserv_sched_count),
        "priority_decisions": int(st.prop_sched_count - st_t0.prop_sched_count),
        "queued_after": int(st.requests),
        "roofline": roof,
        "roofline_note": (None if not args.heap_order else
                          "heap order: one wave's chain of dependent sift round trips "
                          "(latency-bound, a few hundred bytes per operation): no HBM "
                          "roofline applies"),
        "cpu_baseline": cpu,
        "stages_ms_per_step": {n: round(ms / max(prof_steps, 1), 4)
                               for n, (c, ms) in prof.items() if c},
        "stages_note": "stage times from a second pass of prof_steps steps "
                       "after the timed region, the same calls with the same "
                       "kernels (fused, pipelined, launched eagerly: "
                       "apply_link -- the previous call's deferred apply beside "
                       "this call's add_link, one launch -- chain_scan, select, "
                       "emit, rank; the pass's last apply alone) behind a "
                       "GPU-side gate: one-kernel stages timed by HIP events "
                       "the kernel's own dispatch records "
                       "(hipExtLaunchKernel: execution time, as rocprofv3 "
                       "reports it), multi-kernel stages by event pairs; "
                       + ("the timed region replays captured hipGraphs"
                          if (not pipelined or args.graphs) and not args.no_graphs
                          else "the timed region launches the same kernels "
                               "eagerly, pipelined behind the previous call"),
        "prof_steps": prof_steps,
        "engine_counters": ctr_timed,
    }
    print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
