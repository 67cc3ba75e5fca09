#!/usr/bin/env python3
"""Which tie-break rule reproduces the reference's heap top (A11; VERDICT r2
"next" item 6)?  CPU only: the oracle (the reference's indirect heaps
restated, indirect_intrusive_heap.h:462-564) logs, for every decision whose
heap top compared equal to another eligible client, the tied set; each rule
below is scored by how often it picks the client the heap dispatched.

Rules (each falls back to the lowest slot):
  lowest_slot      the engine's rule in rounds 1-2
  fifo_arrival     the earliest front-request arrival
  front_since      the client whose front became the front first (a front
                   that has waited longest; an element that reached its heap
                   position earlier is not passed by an equal one: sift_up
                   swaps on strictly-less only)
  last_tick        the client with the oldest last tag assignment

Traces: BASELINE config 2 (dmc_sim_100th.conf, closed loop, start jitter
off: identical clients issue at identical instants) and an open-loop
config-3 mix at epoch-scale t0 = 1.7e9 s (rounding collisions).

Usage: python tools/tie_rules.py [--out profiles/r03_tie_rules.json]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import pyoracle  # noqa: E402  (test infrastructure: the checker)
from dmclock_amd import sim, workloads  # noqa: E402

RULES = {
    "lowest_slot": lambda m: (m[0],),
    "fifo_arrival": lambda m: (m[1], m[0]),
    "front_since": lambda m: (m[2], m[0]),
    "last_tick": lambda m: (m[3], m[0]),
    "fifo_then_front_since": lambda m: (m[1], m[2], m[0]),
}


def score(log):
    out = {"ties": len(log), "by_heap": {0: 0, 1: 0}}
    for name in RULES:
        out[name] = 0
    sizes = []
    for heap, chosen, mem in log:
        out["by_heap"][heap] += 1
        sizes.append(len(mem))
        for name, key in RULES.items():
            pick = min(mem, key=key)[0]
            out[name] += pick == chosen
    out["by_heap"] = {"reservation": out["by_heap"][0], "ready": out["by_heap"][1]}
    out["mean_tied_set"] = float(np.mean(sizes)) if sizes else 0.0
    for name in RULES:
        out[name + "_frac"] = out[name] / max(len(log), 1)
    return out


def config2(conf_path, seed, ops=None):
    conf = sim.load_conf(conf_path)
    if ops:
        for g in conf.cli_group:
            g.client_total_ops = ops
    qs = []

    def mk(at_limit, antic):
        q = pyoracle.OracleQueue(at_limit=at_limit, anticipation=antic)
        q.tie_log(True)
        qs.append(q)
        return q

    sim.Simulation(conf, mk, seed=seed, t0=1000.0, jitter=0.0).run()
    log = []
    for q in qs:
        log += q.read_tie_log()
    return log


def open_loop(n_clients, steps, batch, t0, seed):
    tr = workloads.config3_trace(seed, n_clients, steps, batch, depth=2, t0=t0)
    q = pyoracle.OracleQueue()
    q.tie_log(True)
    workloads.replay(q, tr)
    return q.read_tie_log()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "tie_rules.json"))
    ap.add_argument("--clients", type=int, default=1 << 16)
    a = ap.parse_args()
    res = {}
    conf = os.path.join(ROOT, "tests", "golden", "dmc_sim_100th.conf")
    for seed in (7, 8):
        res[f"config2_no_jitter_seed{seed}"] = score(config2(conf, seed))
    res["open_loop_t0_1.7e9"] = score(open_loop(a.clients, 4, 1 << 12, 1.7e9, 42))
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    for k, v in res.items():
        print(k, {x: (round(y, 4) if isinstance(y, float) else y) for x, y in v.items()
                  if x.endswith("_frac") or x in ("ties", "by_heap", "mean_tied_set")})


if __name__ == "__main__":
    main()
