"""k_rrank's per-bin clocks on bench.py's config-3 workload (DMC_DEBUG=1,
DMC_DEBUG_BINS): for every round, the kernel's span over its blocks and the
slowest bins -- their record counts, start offsets and durations -- to find
what sets the rank kernel's length in its slow rounds.  GPU box only.

usage: python tools/rank_bins.py [STEPS] > out.txt
"""
import os
import sys
import tempfile

import numpy as np

os.environ["DMC_DEBUG"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
NBR = 4096


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    fn = os.path.join(tempfile.gettempdir(), f"rank_bins_{os.getpid()}.bin")
    os.environ["DMC_DEBUG_BINS"] = fn
    from dmclock_amd import workloads
    from dmclock_amd.gpu import GpuQueue
    tr = workloads.config3_trace(42, 1 << 20, steps, 1 << 16, depth=4)
    q = GpuQueue(max_clients=1 << 20, ring_capacity=64, max_batch=1 << 20)
    c = tr.clients
    q.register(c.slots, c.r, c.w, c.l, c.active)
    pre = tr.ops[0][1]
    for i in range(0, len(pre), 1 << 20):
        q.add_batch(pre[i:i + (1 << 20)])
    os.environ.pop("DMC_DEBUG_BINS")
    now, k = tr.ops[1][1], tr.ops[1][2]
    q.pull_batch(now, k)
    if os.path.exists(fn):
        os.remove(fn)
    os.environ["DMC_DEBUG_BINS"] = fn
    for i in range(2, len(tr.ops), 2):
        q.add_batch(tr.ops[i][1])
        q.pull_batch(tr.ops[i + 1][1], tr.ops[i + 1][2])
    rec = 4 * NBR + 8 * 2 * NBR + 8 * 2 * 262144 + 4
    raw = open(fn, "rb").read()
    os.remove(fn)
    n = len(raw) // rec
    print(f"{n} rounds")
    for r in range(n):
        b = raw[r * rec:(r + 1) * rec]
        hb = np.frombuffer(b[:4 * NBR], np.uint32)
        wt = np.frombuffer(b[4 * NBR:4 * NBR + 16 * NBR], np.uint64).reshape(NBR, 2)
        live = (wt[:, 1] > 0) & (hb > 0)
        st, en = wt[live, 0].astype(np.int64), wt[live, 1].astype(np.int64)
        t0 = st.min()
        dur = (en - st) / 100.0
        span = (en.max() - t0) / 100.0
        idx = np.flatnonzero(live)
        top = np.argsort(-dur)[:4]
        last = np.argsort(-(en - t0))[:3]
        print(f"round {r}: span {span:.2f} us, bins {live.sum()}, max count {hb.max()}, "
              f"p99 count {np.percentile(hb[hb > 0], 99):.0f}; slowest: " +
              ", ".join(f"bin {idx[j]} n={hb[idx[j]]} {dur[j]:.2f}us@{(st[j] - t0) / 100:.2f}"
                        for j in top) +
              "; last to end: " +
              ", ".join(f"bin {idx[j]} n={hb[idx[j]]} end {(en[j] - t0) / 100:.2f}" for j in last))


if __name__ == "__main__":
    main()
