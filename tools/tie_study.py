#!/usr/bin/env python3
"""Measured cost of the tie contract (DESIGN.md
section 4), on the GPU box.

Among clients whose keys are equal the reference dispatches the heap top,
a function of the heap's sift history (indirect_intrusive_heap.h:462-564);
the engine dispatches the lowest slot and flags the decision.  Decisions
with a unique minimum are bit-exact.  This tool runs traces that DO tie,
on the engine and on the oracle (the reference's heaps restated), and
reports:

  * tied decisions: the oracle's decisions whose heap top compared equal to
    another eligible client (flags bit 0), as a fraction of all decisions;
  * where the two dispatch sequences first differ, relative to the first
    tied decision (before it they must be identical);
  * how many decisions differ afterwards (position by position, by client
    and phase), and whether the per-pull dispatched sets and the per-client
    service totals re-converge.

Traces:
  A. BASELINE config 2 (dmc_sim_100th.conf, closed loop) with the start
     jitter off: identical clients issue at identical instants, so their
     tags tie (SURVEY's tie source 1).
  B. an open-loop config-3-shaped trace at epoch-scale time t0 = 1.7e9 s,
     where rounding collisions tie tags (SURVEY's probe: 34 of 73k).

Usage: python tools/tie_study.py [--out profiles/r02_tie_study.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import pyoracle  # noqa: E402  (test infrastructure: the checker)
from dmclock_amd import sim, workloads  # noqa: E402


def seq_compare(dg, do):
    """position-by-position comparison of two decision arrays by (slot,
    phase, cost); returns (first differing index or None, differing count)"""
    n = min(len(dg), len(do))
    a = np.stack([dg["slot"][:n], dg["phase"][:n], dg["cost"][:n]], 1)
    b = np.stack([do["slot"][:n], do["phase"][:n], do["cost"][:n]], 1)
    bad = np.flatnonzero((a != b).any(1))
    extra = abs(len(dg) - len(do))
    first = int(bad[0]) if bad.size else (n if extra else None)
    return first, int(bad.size) + extra


def study_open_loop(n_clients, steps, batch, t0, seed):
    from dmclock_amd.gpu import GpuQueue
    rng = np.random.default_rng(seed)
    tr = workloads.config3_trace(seed, n_clients, steps, batch, depth=2, t0=t0)
    qo = pyoracle.OracleQueue()
    qg = GpuQueue(max_clients=n_clients, ring_capacity=64, max_batch=1 << 20)
    oo = workloads.replay(qo, tr)
    og = workloads.replay(qg, tr)
    total = ties = 0
    first_tie = first_diff = None
    differ = set_differ = 0
    k0 = 0
    per_pull = []
    for a, b in zip(og, oo):
        if a[0] != "pull":
            continue
        dg, do = a[1], b[1]
        tflag = np.flatnonzero(do["flags"] & 1)
        if first_tie is None and tflag.size:
            first_tie = k0 + int(tflag[0])
        f, nd = seq_compare(dg, do)
        if first_diff is None and f is not None:
            first_diff = k0 + f
        sg = set(zip(dg["slot"].tolist(), dg["handle"].tolist()))
        so = set(zip(do["slot"].tolist(), do["handle"].tolist()))
        per_pull.append({"decisions": len(do), "tied": int(tflag.size),
                         "differ_positions": nd,
                         "differ_set": len(sg ^ so) // 2})
        total += len(do)
        ties += int(tflag.size)
        differ += nd
        set_differ += len(sg ^ so) // 2
        k0 += len(do)
    mism = 0
    sample = rng.choice(n_clients, min(4096, n_clients), replace=False)
    for s in sample:
        a, b = qg.client_state(int(s)), qo.client_state(int(s))
        if any(np.float64(getattr(a, f)).view(np.uint64) !=
               np.float64(getattr(b, f)).view(np.uint64)
               for f in ("prev_r", "prev_p", "prev_l", "front_r", "front_p")) or \
                a.count != b.count:
            mism += 1
    qg.close()
    return {"trace": f"open loop, config-3 mix, {n_clients} clients, t0 = {t0:g} s, "
                     f"depth 2, settle round + {steps} steps of {batch} adds + "
                     f"{batch} pulls, seed {seed}",
            "decisions": total, "tied_decisions": ties,
            "tied_frac": ties / max(total, 1),
            "first_tied_decision": first_tie, "first_differing_decision": first_diff,
            "differ_positions": differ, "differ_positions_frac": differ / max(total, 1),
            "differ_dispatched_set": set_differ,
            "client_state_mismatch_of_4096_sampled": mism,
            "per_pull": per_pull}


def study_sim(conf_path, jitter, t0, seed):
    from dmclock_amd.gpu import GpuQueue
    conf = sim.load_conf(conf_path)
    ncl = sum(g.client_count for g in conf.cli_group)

    def gpu_mk(at_limit, antic):
        return GpuQueue(max_clients=ncl, ring_capacity=64, max_batch=1024,
                        at_limit=at_limit, anticipation=antic)

    def ora_mk(at_limit, antic):
        return pyoracle.OracleQueue(at_limit=at_limit, anticipation=antic)

    o = sim.Simulation(conf, ora_mk, seed=seed, t0=t0, jitter=jitter).run()
    g = sim.Simulation(conf, gpu_mk, seed=seed, t0=t0, jitter=jitter).run()
    total = sum(len(x) for x in o.log_dec)
    ties = 0
    firsts = []
    differ = 0
    # in virtual time, over all servers: the first tied decision and the
    # first decision where the two dispatch sequences differ (a closed loop
    # couples the servers through the clients, so a difference on one server
    # can stem from a tie on another: only a global first difference at or
    # after the global first tie rules out a non-tie divergence)
    t_tie = t_diff = None
    for s in range(len(o.log_dec)):
        do = [r for _, r in o.log_dec[s]]
        dg = [r for _, r in g.log_dec[s]]
        to = [t for t, _ in o.log_dec[s]]
        tg = [t for t, _ in g.log_dec[s]]
        tf = [i for i, r in enumerate(do) if int(r["flags"]) & 1]
        ties += len(tf)
        n = min(len(do), len(dg))
        d = [i for i in range(n) if (int(do[i]["slot"]), int(do[i]["phase"]),
                                     to[i]) != (int(dg[i]["slot"]), int(dg[i]["phase"]),
                                                tg[i])]
        if len(do) != len(dg) and not d:
            d = [n]
        differ += len([i for i in d if i < n]) + abs(len(do) - len(dg))
        if tf:
            t = to[tf[0]]
            t_tie = t if t_tie is None else min(t_tie, t)
        if d:
            i = d[0]
            t = min(to[i] if i < len(to) else np.inf, tg[i] if i < len(tg) else np.inf)
            t_diff = t if t_diff is None else min(t_diff, t)
        if tf or d:
            firsts.append((s, tf[0] if tf else None, d[0] if d else None))
    before_tie_ok = all(fd is None or (ft is not None and fd >= ft)
                        for _, ft, fd in firsts)
    global_ok = t_diff is None or (t_tie is not None and t_diff >= t_tie)
    so, sg = o.stats(), g.stats()
    l1_res = int(np.abs(so["reservation_ops"] - sg["reservation_ops"]).sum())
    l1_prio = int(np.abs(so["priority_ops"] - sg["priority_ops"]).sum())
    return {"trace": f"{os.path.basename(conf_path)} closed loop (dmc_sim restated), "
                     f"start jitter {jitter:g} s, t0 = {t0:g} s, seed {seed}",
            "decisions": total, "tied_decisions": ties,
            "tied_frac": ties / max(total, 1),
            "servers_with_a_tie_or_difference": len(firsts),
            "sequences_identical_until_first_tie": before_tie_ok,
            "first_tie_virtual_time": t_tie,
            "first_difference_virtual_time": t_diff,
            "no_difference_before_the_first_tie_anywhere": global_ok,
            "differ_positions": differ, "differ_positions_frac": differ / max(total, 1),
            "reservation_ops_oracle": int(so["reservation_ops"].sum()),
            "reservation_ops_engine": int(sg["reservation_ops"].sum()),
            "priority_ops_oracle": int(so["priority_ops"].sum()),
            "priority_ops_engine": int(sg["priority_ops"].sum()),
            "per_client_service_l1": {"reservation": l1_res, "priority": l1_prio},
            "per_client_service_l1_frac": (l1_res + l1_prio) / max(total, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "tie_study.json"))
    ap.add_argument("--clients", type=int, default=1 << 16)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--batch", type=int, default=1 << 12)
    ap.add_argument("--ops", type=int, default=None,
                    help="config 2: ops per client (default: the conf's 1000)")
    a = ap.parse_args()
    out = {}
    t = time.time()
    out["open_loop_t0_1.7e9"] = study_open_loop(a.clients, a.steps, a.batch, 1.7e9, 42)
    print("open loop", round(time.time() - t, 1), "s", flush=True)
    conf = os.path.join(ROOT, "tests", "golden", "dmc_sim_100th.conf")
    t = time.time()
    out["config2_no_jitter"] = study_sim(conf, 0.0, 1000.0, 7)
    print("config 2", round(time.time() - t, 1), "s", flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    for k, v in out.items():
        print(k, {x: y for x, y in v.items() if x != "per_pull"})


if __name__ == "__main__":
    main()
