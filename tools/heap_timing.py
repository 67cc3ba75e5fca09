"""Tie-exact mode (DMC_OPT_HEAP_ORDER) at scale: BASELINE config 3's shape
(config3_trace) on the reference's clock scale, GPU heap order against the
oracle -- the time of each phase on both and every decision compared.

usage: python tools/heap_timing.py N_CLIENTS [STEPS] [--t0 1.7e9] [--batch 65536]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("n", type=int)
    ap.add_argument("steps", type=int, nargs="?", default=2)
    ap.add_argument("--t0", type=float, default=1.7e9)
    ap.add_argument("--batch", type=int, default=1 << 16)
    ap.add_argument("--depth", type=int, default=4)
    ap.add_argument("--no-oracle", action="store_true")
    a = ap.parse_args()
    import pyoracle
    from dmclock_amd import workloads
    from dmclock_amd.gpu import GpuQueue
    from parity import compare_decisions
    tr = workloads.config3_trace(42, a.n, a.steps, a.batch, depth=a.depth, t0=a.t0)
    c = tr.clients
    qs = [("gpu", GpuQueue(max_clients=a.n, ring_capacity=64, max_batch=1 << 20,
                           heap_order=True))]
    if not a.no_oracle:
        qs.append(("oracle", pyoracle.OracleQueue()))
    outs = {}
    for name, q in qs:
        t = time.perf_counter()
        q.register(c.slots, c.r, c.w, c.l, c.active)
        times = {"register": time.perf_counter() - t}
        out = []
        for op in tr.ops:
            t = time.perf_counter()
            if op[0] == "add":
                reqs = op[1]
                rc = np.concatenate([q.add_batch(reqs[i:i + (1 << 20)])
                                     for i in range(0, len(reqs), 1 << 20)])
                out.append(("add", rc))
                key = "add"
            else:
                d, res = q.pull_batch(op[1], op[2])
                out.append(("pull", d, (res.n_decisions, res.next_type)))
                key = "pull"
            dt = time.perf_counter() - t
            n_ops = len(op[1]) if op[0] == "add" else len(out[-1][1])
            times.setdefault(key, []).append((n_ops, dt))
            print(f"{name} {key} {n_ops} ops {dt:.3f} s = {dt / max(n_ops, 1) * 1e6:.2f} us/op",
                  flush=True)
        outs[name] = (out, q)
    if "oracle" in outs:
        og, qg = outs["gpu"]
        oo, qo = outs["oracle"]
        n = 0
        for i, (x, y) in enumerate(zip(og, oo)):
            if x[0] == "add":
                assert np.array_equal(x[1], y[1]), i
            else:
                compare_decisions(x[1], y[1], f"op {i}")
                assert x[2] == y[2], (i, x[2], y[2])
                n += len(x[1])
        from parity import compare_states
        rng = np.random.default_rng(0)
        compare_states(qg, qo, rng.choice(c.slots, min(4096, a.n), replace=False), "final")
        print(f"parity: {n} decisions bit-exact, oracle ties {qo.ties}", flush=True)


if __name__ == "__main__":
    main()
