"""Per-round engine diagnostics (DMC_DEBUG=1 prints one line per round on
stderr) for one server of tests/test_concurrency.py's workload, or for
bench.py's config-3 workload (--bench): rank-bin maxima, thresholds,
candidate kinds; --config4: bench.py --config 4's workload.  GPU box only."""
import os
import sys

os.environ["DMC_DEBUG"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))  # (test_concurrency imports it; unused here)
import numpy as np  # noqa: E402


def main():
    import torch
    from dmclock_amd import workloads
    from dmclock_amd.gpu import GpuQueue
    if "--bench" in sys.argv:
        tr = workloads.config3_trace(42, 1 << 20, 6, 1 << 16, depth=4)
        q = GpuQueue(max_clients=1 << 20, ring_capacity=64, max_batch=1 << 20)
        c = tr.clients
        q.register(c.slots, c.r, c.w, c.l, c.active)
        pre = tr.ops[0][1]
        for i in range(0, len(pre), 1 << 20):
            q.add_batch(pre[i:i + (1 << 20)])
        print("=== settle", file=sys.stderr, flush=True)
        now, k = tr.ops[1][1], tr.ops[1][2]
        q.pull_batch(now, k)
        for i in range(2, len(tr.ops), 2):
            print(f"=== step {i // 2 - 1}", file=sys.stderr, flush=True)
            q.add_batch(tr.ops[i][1])
            q.pull_batch(tr.ops[i + 1][1], tr.ops[i + 1][2])
        print(q.counters(), file=sys.stderr)
        return
    if "--config4" in sys.argv:
        tr = workloads.config4_trace(42, 1 << 20, 6, 1 << 16, depth=4)
        q = GpuQueue(max_clients=1 << 20, ring_capacity=64, max_batch=1 << 20)
        c = tr.clients
        q.register(c.slots, c.r, c.w, c.l, c.active)
        for i, op in enumerate(tr.ops):
            if op[0] == "add":
                for j in range(0, len(op[1]), 1 << 20):
                    q.add_batch(op[1][j:j + (1 << 20)])
            elif op[0] == "pull":
                print(f"=== op {i}", file=sys.stderr, flush=True)
                q.pull_batch(op[1], op[2])
            elif op[0] == "idle":
                q.mark_idle_batch(op[1])
        print(q.counters(), file=sys.stderr)
        return
    from test_concurrency import SHAPE, workload
    sh = dict(SHAPE)
    tab, cmap, srv = workload(sh)
    chunks, t_pre, steps = srv[0]
    q = GpuQueue(max_clients=sh["N"], ring_capacity=64, max_batch=sh["chunk"])
    q.register(tab.slots, tab.r, tab.w, tab.l, True)
    for c in chunks:
        q.add_batch(c)
    print("=== settle", file=sys.stderr, flush=True)
    q.pull_batch(t_pre, sh["settle"])
    for i, b in enumerate(steps):
        print(f"=== step {i}", file=sys.stderr, flush=True)
        q.add_batch(b)
        q.pull_batch(float(b["time"][-1]), sh["batch"])
    print(q.counters(), file=sys.stderr)


if __name__ == "__main__":
    main()
