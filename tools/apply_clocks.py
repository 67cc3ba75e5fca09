"""k_rapply's slow candidates' clocks over bench.py rounds (DMC_DEBUG=1,
DMC_DEBUG_BINS dumps, the pull rounds of `bench.py --config 4`): per round,
the slow path's candidates (several records, cut groups: apply_one) with
their start offsets and durations -- staging of the client record and ring,
the walks' replay, the queue's reductions, the final stores -- to find what
sets the apply kernel's length.  GPU box only.

usage: python tools/apply_clocks.py DUMP [ROUNDS] > out.txt
       (DUMP written by: DMC_DEBUG=1 DMC_DEBUG_BINS=DUMP python bench.py ...)
"""
import sys

import numpy as np

NBR = 4096


def main():
    fn = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    rec = 4 * NBR + 8 * 2 * NBR + 8 * 2 * 262144 + 4
    raw = open(fn, "rb").read()
    n = len(raw) // rec
    print(f"{n} rounds in the dump, the last {last}:")
    for r in range(max(0, n - last), n):
        b = raw[r * rec:(r + 1) * rec]
        off = 4 * NBR + 16 * NBR
        at = np.frombuffer(b[off:off + 16 * 262144], np.uint64).reshape(65536, 8)
        live = at[:, 0] > 0
        if not live.any():
            print(f"round {r}: no slow candidates")
            continue
        a = at[live].astype(np.int64)
        t0 = a[:, 0].min()
        st, stage, walk, red, end = ((a[:, 0] - t0) / 100.0, (a[:, 1] - a[:, 0]) / 100.0,
                                     (a[:, 2] - a[:, 1]) / 100.0, (a[:, 3] - a[:, 2]) / 100.0,
                                     (a[:, 4] - a[:, 3]) / 100.0)
        tot = (a[:, 4] - a[:, 0]) / 100.0
        fin = (a[:, 4] - t0) / 100.0
        q = lambda x: f"p50 {np.percentile(x, 50):.2f} p90 {np.percentile(x, 90):.2f} max {x.max():.2f}"
        print(f"round {r}: slow {live.sum()}, span to the last end {fin.max():.2f} us; "
              f"start {q(st)} | stage {q(stage)} | walks {q(walk)} | reductions {q(red)} | "
              f"stores {q(end)} | total {q(tot)}")
        for i in np.argsort(-fin)[:4]:
            print(f"   late: start {st[i]:.2f} stage {stage[i]:.2f} walks {walk[i]:.2f} "
                  f"reductions {red[i]:.2f} stores {end[i]:.2f} end {fin[i]:.2f}")


if __name__ == "__main__":
    main()
