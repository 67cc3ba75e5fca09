"""Per-candidate apply stage timings from a DMC_DEBUG_BINS dump (engine
debug mode): each round appends 4096 rank-bin counts (u32), 2 x 4096
rank-block clocks (u64), 524288 u64 of apply clocks -- 8 per candidate for
the first 65,536: start, staged, walked, reduced, end (wall_clock64,
100 MHz) -- and the candidate count (u32)."""
import sys

import numpy as np

path = sys.argv[1]
raw = open(path, "rb").read()
rec = 4096 * 4 + 8192 * 8 + 524288 * 8 + 4
n = len(raw) // rec
for r in range(n):
    b = raw[r * rec:(r + 1) * rec]
    o = 4096 * 4 + 8192 * 8
    at = np.frombuffer(b[o:o + 524288 * 8], dtype=np.uint64).astype(np.int64).reshape(-1, 8)
    o += 524288 * 8
    nc = int(np.frombuffer(b[o:o + 4], dtype=np.uint32)[0])
    m = min(nc, 65536)
    a = at[:m]
    ok = (a[:, 0] > 0) & (a[:, 4] >= a[:, 0])
    if not ok.any():
        continue
    a = a[ok]
    t0 = a[:, 0].min()
    q = lambda x: f"{np.percentile(x, 50) / 100:.2f}/{np.percentile(x, 90) / 100:.2f}"
    stg = a[:, 1] - a[:, 0]
    walk = np.where(a[:, 2] > 0, a[:, 2] - a[:, 1], 0)
    red = np.where(a[:, 3] > 0, a[:, 3] - a[:, 2], 0)
    tail = np.where(a[:, 3] > 0, a[:, 4] - a[:, 3], a[:, 4] - a[:, 2])
    print(f"round {r}: cand {nc} start spread {(a[:, 0].max() - t0) / 100:.2f} span "
          f"{(a[:, 4].max() - t0) / 100:.2f} | p50/p90 us: stage {q(stg)} walk {q(walk)} "
          f"reduce {q(red)} stores {q(tail)} total {q(a[:, 4] - a[:, 0])}")
